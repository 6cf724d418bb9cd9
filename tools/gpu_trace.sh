# one rocprofv3 kernel-trace pass over a short bench run (timeline of a step); extra args go to bench.py
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
TAG=${TAG:-tr}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/$TAG -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 --h2d-steps 0 --prof-every 1000 "$@" > $ROOT/gpurun_out/${TAG}_bench.log 2>&1
