# cad1: batched parity-class launch threshold sweep (knob conv4_cls_batch_min), alternated on one box
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 512 128 0; do
    timeout -k 10 200 python bench.py --config cad1 --no-cpu-baseline --tune conv4_cls_batch_min=$v > gpurun_out/r05w_cad1_${v}_$rep.json 2>/dev/null || exit 1
  done
done
