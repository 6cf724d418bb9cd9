set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_data.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/data.log 2>&1
