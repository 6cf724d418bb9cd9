# final-build profiles (configs 2 and 4) and the stride-2 input-gradient channel-block A/B (knob conv_dgrad_s2_nt)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_dgrad_s2_nt=$v > gpurun_out/nt_cfg2_v${v}_r$r.json 2>/dev/null || exit 1
  done
done
bash tools/gpu_r4_prof.sh 2 r4s && bash tools/gpu_r4_prof.sh 4 r4s
