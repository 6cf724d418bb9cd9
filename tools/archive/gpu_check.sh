set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/gt.log 2>&1 && \
timeout -k 10 200 python tools/tune_conv.py --patch > gpurun_out/patch.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --breakdown-out gpurun_out/bd.json > gpurun_out/bench.log 2>&1
