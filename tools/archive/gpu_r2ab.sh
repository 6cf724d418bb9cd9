# round-2: input-gradient grid size under stream concurrency
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 "$@"; }
for rep in 1 2; do
for v in 512 384 768 256; do
  run --tune conv_dgrad_blocks=$v > gpurun_out/r2ab_${v}_$rep.log 2>&1 || exit 1
done
done
