# round-2: x3 resident weights -- kernel + cad GPU tests, bench breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_cad_gpu.py tests/test_dp.py tests/test_a2_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2g_gt.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2g_bd.json > gpurun_out/r2g_bench.log 2>&1
