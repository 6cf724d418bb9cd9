# round-2: full GPU suite (pinned-gradient and config-3 DP tests included)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -s > gpurun_out/r2b_gt.log 2>&1
