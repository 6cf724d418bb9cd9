# round-2: one-wave BN finalize kernels -- parity (cad + dp), A/B cfg2 + cfg4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cad_gpu.py tests/test_dp.py > gpurun_out/r2ao_test.log 2>&1 || exit 1
bash tools/ab_so.sh r2ao2 3 || exit 1
bash tools/ab_so.sh r2ao4 2 --config 4 || exit 1
