# round-2: x3 conv cost attribution (knob conv_split_dbg: 1 no weight restaging, 2 no split, 4 no MFMA, 8 no patch
# loads; results wrong with any bit)
set -o pipefail
mkdir -p gpurun_out
for d in 0 1 2 4 8 11 15; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 5 --warmup 2 --tune conv_split_dbg=$d --breakdown-out gpurun_out/r2t_bd_$d.json > gpurun_out/r2t_$d.log 2>&1 || exit 1
done
