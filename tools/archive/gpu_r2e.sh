# round-2: reverted BN flow (analytic conv-bias grad) -- cad GPU tests + bench breakdown; list PMC counters
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_cad_gpu.py tests/test_dp.py tests/test_mc_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2e_gt.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2e_bd.json > gpurun_out/r2e_bench.log 2>&1
