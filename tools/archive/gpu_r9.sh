set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_kernels_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gt12.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --breakdown-out gpurun_out/bd12.json > gpurun_out/bench12.log 2>&1
