set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench2.log 2>&1 && \
timeout -k 10 300 python bench.py --config 4 > gpurun_out/bench4.log 2>&1 && \
timeout -k 10 300 python bench.py --config 4 --dtype fp32 --no-cpu-baseline > gpurun_out/bench4f.log 2>&1
