# round-2: side-stream head/detector chains -- GPU tests, step trace, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cad_gpu.py tests/test_dp.py tests/test_kernels_gpu.py tests/test_a2_gpu.py tests/test_mc_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2h_gt.log 2>&1 && \

timeout -k 10 300 python bench.py --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2h_bd.json > gpurun_out/r2h_bench.log 2>&1
