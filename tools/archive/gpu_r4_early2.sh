# early-stem variants on config 2: knob cad_stem_early 0 (off), 1 (own stream), 2 (side stream), 3 (wgrad stream),
# and 1 with GPU_MAX_HW_QUEUES=8
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2 3; do
  timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune cad_stem_early=$v > gpurun_out/r4e2_v$v.json 2>/dev/null || exit 1
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune cad_stem_early=1 > gpurun_out/r4e2_v1q8.json 2>/dev/null || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune cad_stem_early=0 > gpurun_out/r4e2_v0q8.json 2>/dev/null || exit 1
