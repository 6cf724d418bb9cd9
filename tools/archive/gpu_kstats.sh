# one rocprofv3 kernel-stats pass over a short bench run (per-kernel average durations)
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/kst -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 20 > $ROOT/gpurun_out/kst_bench.log 2>&1
