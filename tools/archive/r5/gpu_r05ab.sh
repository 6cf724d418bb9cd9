# config 2: kernel + HIP runtime API trace of a few steps (host submission timing around the forward / backward
# boundary of the cad step)
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $ROOT/gpurun_out/r05ab_cfg2_api -o run -- python3 $ROOT/bench.py --no-cpu-baseline --h2d-steps 0 --steps 6 --warmup 3 > $ROOT/gpurun_out/r05ab_cfg2_api.log 2>&1
