set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/tune_wg.py > gpurun_out/wg_tune.log 2>&1 && \
timeout -k 10 200 python tools/tune_x3.py > gpurun_out/x3_tune.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --breakdown-out gpurun_out/bd.json > gpurun_out/bench.log 2>&1
