# round-2: bf16 activation storage (config 4) -- parity tests, config-4 and config-2 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cad_gpu.py > gpurun_out/r2ak_test.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bf16 or stem" > gpurun_out/r2ak_ktest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --steps 20 --breakdown-out gpurun_out/r2ak_bd4.json > gpurun_out/r2ak_b4.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --steps 30 > gpurun_out/r2ak_b4b.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 > gpurun_out/r2ak_b2.log 2>&1 || exit 1
