set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_cad_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread -k "bf16 or config4" > gpurun_out/bf.log 2>&1 && \
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gt.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
