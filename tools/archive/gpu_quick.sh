# GPU tests + a bench line with the per-phase breakdown (no tuning sweep)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 && \
timeout -k 10 300 python bench.py --breakdown-out gpurun_out/bd.json > gpurun_out/bench.log 2>&1
