# in-kernel BN forward finalize (knob bn_fin_fused): parity, then A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cad_gpu.py tests/test_kernels_gpu.py tests/test_dp.py > gpurun_out/fin_test.log 2>&1 || exit 1
bash tools/ab_knob.sh fin2 3 bn_fin_fused 0 1 || exit 1
bash tools/ab_knob.sh fin4 2 bn_fin_fused 0 1 --config 4 || exit 1
