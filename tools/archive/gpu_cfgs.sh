# The non-default BASELINE configs on the current build (1 GPU), each with its CPU leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config 4 > gpurun_out/bench_cfg4.log 2>&1 && \
timeout -k 10 300 python bench.py --config 1 > gpurun_out/bench_cfg1.log 2>&1 && \
timeout -k 10 300 python bench.py --config 5 > gpurun_out/bench_cfg5.log 2>&1 && \
timeout -k 10 300 python bench.py --config cad1 > gpurun_out/bench_cad1.log 2>&1
