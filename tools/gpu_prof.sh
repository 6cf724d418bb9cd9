set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 20 > $ROOT/gpurun_out/prof_bench.log 2>&1
