# round-2: 8-wave / 256-pixel-tile split conv kernels for stride-1 layers -- tests + A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_cad_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2ac_t.log 2>&1 && \
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --breakdown-out gpurun_out/r2ac_bd1_$rep.json > gpurun_out/r2ac_1_$rep.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_split_big=0 --breakdown-out gpurun_out/r2ac_bd0_$rep.json > gpurun_out/r2ac_0_$rep.log 2>&1 || exit 1
done
