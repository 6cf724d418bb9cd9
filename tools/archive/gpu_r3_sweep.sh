# grid-size knob sweep at config 2 after the round-3 stream rebalancing: each setting twice, a default run between
# every two settings (drift control); JSON lines under gpurun_out/r03sw_*.log
set -o pipefail
mkdir -p gpurun_out
i=0
for rep in 1 2; do
  for kv in base conv_wgrad_patch_blocks=320 conv_wgrad_patch_blocks=576 base conv_dgrad_blocks=384 conv_dgrad_blocks=768 base conv_wgrad_s2_blocks=256 conv_wgrad_s2_blocks=512 base conv_wgrad_s1_nt_blocks=256 conv_wgrad_s1_nt_blocks=512; do
    i=$((i+1))
    if [ "$kv" = base ]; then T=""; else T="--tune $kv"; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 $T > gpurun_out/r03sw_${i}_${kv}.log 2>&1 || exit 1
  done
done
