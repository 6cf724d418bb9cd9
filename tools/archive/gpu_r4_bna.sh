# BN backward apply: rows in flight per thread (bn_apply_u) and grid cap (bn_apply_blocks) at config 2
set -o pipefail
mkdir -p gpurun_out
for kv in "4 2048 a" "2 2048 a" "8 2048 a" "4 1024 a" "4 4096 a" "4 2048 b" "8 4096 a"; do
  set -- $kv
  timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune bn_apply_u=$1 --tune bn_apply_blocks=$2 --breakdown-out gpurun_out/bna_u$1_b$2_$3.bd.json > gpurun_out/bna_u$1_b$2_$3.json 2>/dev/null || exit 1
done
