# per-label breakdown (HIP events per kernel label) of the cfg2 and cfg4 benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 20 --breakdown-out gpurun_out/bd_cfg2.json > gpurun_out/bd_cfg2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 20 --config 4 --breakdown-out gpurun_out/bd_cfg4.json > gpurun_out/bd_cfg4.log 2>&1 || exit 1
