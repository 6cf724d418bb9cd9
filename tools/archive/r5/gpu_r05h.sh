# round 5: cad1 autoencoder on implicit-GEMM 4x4 convs (no im2col): cad1 parity tests, then a cad1 bench A/B against
# the im2col path (knob ae_direct=0), a kernel-stats pass, and the kernel unit tests after the stride-2 revert
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_ae_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r05h_ae.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config cad1 --no-cpu-baseline --steps 30 > gpurun_out/r05h_cad1_direct_$rep.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --config cad1 --no-cpu-baseline --steps 30 --tune ae_direct=0 > gpurun_out/r05h_cad1_im2col_$rep.log 2>&1 || exit 1
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/gpurun_out/r05h_cad1 -o run -- python3 $ROOT/bench.py --config cad1 --no-cpu-baseline --steps 10 \
  --warmup 3 > $ROOT/gpurun_out/r05h_cad1_prof.log 2>&1) || exit 1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05h_kt.log 2>&1 || exit 1
