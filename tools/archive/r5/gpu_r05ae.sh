# config 2: weight-gradient slab reduce lanes (knob wgrad_reduce_per_lane 16 / 8 / 4), alternated on one box, then a
# kernel trace of each setting
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in 16 8 4; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune wgrad_reduce_per_lane=$v > gpurun_out/r05ae_cfg2_${v}_$rep.json 2>/dev/null || exit 1
  done
done
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in 16 8 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r05ae_trace_$v -o run -- python3 $ROOT/bench.py --no-cpu-baseline --h2d-steps 0 --steps 10 --tune wgrad_reduce_per_lane=$v > $ROOT/gpurun_out/r05ae_trace_$v.log 2>&1 || exit 1
done
