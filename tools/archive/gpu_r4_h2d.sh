# input-inclusive leg vs the early stem: bench config 2 with the H2D leg, knob cad_stem_early 0 / 1
set -o pipefail
mkdir -p gpurun_out
for v in 0 1; do
  timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --steps 20 --tune cad_stem_early=$v > gpurun_out/r4h2d_e$v.json 2>/dev/null || exit 1
done
