# round-2: fused BN backward -- cad/kernel/dp GPU tests, then bench with breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cad_gpu.py tests/test_dp.py tests/test_kernels_gpu.py tests/test_mc_gpu.py -x -v -s -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2d_gt.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --breakdown-out gpurun_out/r2d_bd.json > gpurun_out/r2d_bench.log 2>&1
