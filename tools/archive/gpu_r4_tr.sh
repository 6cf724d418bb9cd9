# transposed-read weight-gradient kernel: unit tests, cfg2 GPU parity, then A/B of conv_wgrad_tr on config 2.
set -o pipefail
TAG=${1:-r4tr}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_unit.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py -m gpu -k "dir_affine or config4 or full_size" -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_cad.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_wgrad_tr=1 > gpurun_out/${TAG}_c2_A_$rep.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_wgrad_tr=2 > gpurun_out/${TAG}_c2_B_$rep.json 2>/dev/null || exit 1
done
