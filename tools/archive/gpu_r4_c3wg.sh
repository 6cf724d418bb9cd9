# direct Conv3d weight-gradient grid (knob conv3d_wgrad_blocks) at config 1
set -o pipefail
mkdir -p gpurun_out
for r in a b; do
  for v in 256 512 1024; do
    timeout -k 10 200 python bench.py --config 1 --no-cpu-baseline --tune conv3d_wgrad_blocks=$v > gpurun_out/c3wg_cfg1_$v$r.json 2>/dev/null || exit 1
  done
done
