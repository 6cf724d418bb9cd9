# round-2: grid-size sweep of the stride-2 split-bf16 weight gradient (kernel + split-K reduce per layer)
set -o pipefail
mkdir -p gpurun_out
for nb in 256 384 512 1024; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --tune conv_wgrad_s2_blocks=$nb --breakdown-out gpurun_out/r2j_bd_$nb.json > gpurun_out/r2j_bench_$nb.log 2>&1 || exit 1
done
