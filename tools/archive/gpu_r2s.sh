# round-2: phase offset between the two co-resident x3 conv blocks of a CU (knob conv_split_stagger)
set -o pipefail
mkdir -p gpurun_out
for sg in 0 1 2 4 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 10 --warmup 3 --tune conv_split_stagger=$sg --breakdown-out gpurun_out/r2s_bd_$sg.json > gpurun_out/r2s_$sg.log 2>&1 || exit 1
done
