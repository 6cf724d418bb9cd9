# host-side HIP API trace beside the kernel trace of a short config-2 bench (no counters)
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $ROOT/gpurun_out/r4ht -o run -- python3 $ROOT/bench.py --config 2 --no-cpu-baseline --h2d-steps 0 --steps 6 --warmup 3 > $ROOT/gpurun_out/r4ht.log 2>&1
