# round-2: stem kernel cost attribution (knob stem_dbg: 1 no MFMA, 2 no loads, 4 no atomics, 8 no stores)
set -o pipefail
mkdir -p gpurun_out
for d in 0 1 2 4 8 15; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 5 --warmup 2 --tune stem_dbg=$d --breakdown-out gpurun_out/r2q_bd_$d.json > gpurun_out/r2q_$d.log 2>&1 || exit 1
done
