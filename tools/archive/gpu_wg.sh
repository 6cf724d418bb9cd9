# kernel tests for the conv families, then the bench with a breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/wg.log 2>&1 && \
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --breakdown-out gpurun_out/bd.json > gpurun_out/bench.log 2>&1
