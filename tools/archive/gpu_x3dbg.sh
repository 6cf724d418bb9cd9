# split-conv attribution: per-layer breakdown with parts of the conv kernels switched off (knob conv_split_dbg;
# results wrong, timing only)
set -o pipefail
mkdir -p gpurun_out
for d in 0 1 2 4 8 6 14; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 20 --tune conv_split_dbg=$d --breakdown-out gpurun_out/x3dbg_$d.json > gpurun_out/x3dbg_$d.log 2>&1 || exit 1
done
