# round-2: the other BASELINE configs after the wgrad / stem changes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2o_bd4.json > gpurun_out/r2o_cfg4.log 2>&1 && \
timeout -k 10 300 python bench.py --config 4 --dtype fp32 --no-cpu-baseline --h2d-steps 0 > gpurun_out/r2o_cfg4f.log 2>&1 && \
timeout -k 10 300 python bench.py --config 1 --no-cpu-baseline > gpurun_out/r2o_cfg1.log 2>&1 && \
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/r2o_cfg5.log 2>&1
