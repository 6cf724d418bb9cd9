# kernel trace (no counters) of a short bench: bash tools/gpu_r4_trace1.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/$TAG -o run -- python3 $ROOT/bench.py --no-cpu-baseline --h2d-steps 0 --steps 8 --warmup 3 "$@" > $ROOT/gpurun_out/$TAG.log 2>&1
