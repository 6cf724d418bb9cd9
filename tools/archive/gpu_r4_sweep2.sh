# grid sweeps around the round-4 defaults (configs 2 and 4, two reps each)
set -o pipefail
mkdir -p gpurun_out
run() {  # config tag knob=value
  timeout -k 10 200 python bench.py --config $1 --no-cpu-baseline --h2d-steps 0 --steps 30 ${3:+--tune $3} > gpurun_out/r4s2_c$1_$2.json 2>/dev/null
}
for rep in 1 2; do
  run 2 base_$rep "" || exit 1
  run 2 wg320_$rep conv_wgrad_tr_blocks=320 || exit 1
  run 2 wg448_$rep conv_wgrad_tr_blocks=448 || exit 1
  run 2 dg384_$rep conv_dgrad_blocks=384 || exit 1
  run 2 dg640_$rep conv_dgrad_blocks=640 || exit 1
  run 4 base_$rep "" || exit 1
  run 4 wg320_$rep conv_bfw_blocks=320 || exit 1
  run 4 wg448_$rep conv_bfw_blocks=448 || exit 1
  run 4 bc384_$rep conv_bfc_blocks=384 || exit 1
  run 4 bc640_$rep conv_bfc_blocks=640 || exit 1
done
