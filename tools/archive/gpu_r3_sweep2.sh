# second knob sweep (kernel-choice knobs) at config 2 after the round-3 stream rebalancing: each setting twice, a default run between
# every two settings (drift control); JSON lines under gpurun_out/r03sx_*.log
set -o pipefail
mkdir -p gpurun_out
i=0
for rep in 1 2; do
  for kv in base conv_wgrad_s1_nt=4 cad_last_wgrad_main=0 base cad_l0_slab=0 conv_split_nt=1 base mlp_tail_wide=1 conv_split_wres=0; do
    i=$((i+1))
    if [ "$kv" = base ]; then T=""; else T="--tune $kv"; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 $T > gpurun_out/r03sx_${i}_${kv}.log 2>&1 || exit 1
  done
done
