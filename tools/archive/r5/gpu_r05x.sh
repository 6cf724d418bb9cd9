# cad1: split-K threshold of the implicit-GEMM convs (knob conv4_split_tiles), alternated on one box; classes batched
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 512 128 32 0; do
    timeout -k 10 200 python bench.py --config cad1 --no-cpu-baseline --tune conv4_split_tiles=$v > gpurun_out/r05x_cad1_${v}_$rep.json 2>/dev/null || exit 1
  done
done
