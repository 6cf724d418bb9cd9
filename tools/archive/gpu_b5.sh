set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bbox.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/bb.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench2.log 2>&1 && \
timeout -k 10 300 python bench.py --config 5 > gpurun_out/bench5.log 2>&1
