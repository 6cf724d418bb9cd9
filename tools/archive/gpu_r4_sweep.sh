# grid-size sweeps of the weight-gradient kernels (config 2: conv_wgrad_tr_blocks, config 4: conv_bfw_blocks)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in 320 384 448; do
  timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_wgrad_tr_blocks=$v > gpurun_out/r4sw_c2_${v}_$rep.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_bfw_blocks=$v > gpurun_out/r4sw_c4_${v}_$rep.json 2>/dev/null || exit 1
done
done
