# round 5: first look at the LDS-DMA weight gradient: unit tests, a knob A/B check of one step, a bench A/B
set -o pipefail
TAG=${1:-r05b}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_kt.log 2>&1 && \
timeout -k 10 200 python -u tools/r5/knob_check.py conv_wgrad_dma 0 1 > gpurun_out/${TAG}_check.log 2>&1 && \
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_wgrad_dma=0 --breakdown-out gpurun_out/${TAG}_bdA_$rep.json > gpurun_out/${TAG}_A_$rep.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_wgrad_dma=1 --breakdown-out gpurun_out/${TAG}_bdB_$rep.json > gpurun_out/${TAG}_B_$rep.log 2>&1 || exit 1
done
