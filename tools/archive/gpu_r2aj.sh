# round-2: config-4 (bf16, T=32, 256x256) attribution -- phase breakdown + rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --steps 20 --breakdown-out gpurun_out/r2aj_bd.json > gpurun_out/r2aj_b.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2aj_prof -o r2aj -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r2aj_prof.log 2>&1 || exit 1
