# round 5: class-batched GEMMs (a2 3-D input gradient: 8 classes, cad1 4x4 classes: 4 per launch), stepped patch
# loaders, branch-free a2 conv1 weight gradient, unrolled grouped-BN loops: GPU tests, a2 / cad1 / cfg2 benches, stats
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_a2_gpu.py tests/test_ae_gpu.py tests/test_cad_gpu.py tests/test_mc_gpu.py tests/test_bbox.py -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r05m_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config a2 --steps 30 --cpu-seconds 8 > gpurun_out/r05m_a2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config cad1 --steps 30 --cpu-seconds 8 > gpurun_out/r05m_cad1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 40 > gpurun_out/r05m_cfg2.log 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/gpurun_out/r05m_a2 -o run -- python3 $ROOT/bench.py --config a2 --no-cpu-baseline --steps 10 \
  --warmup 3 > $ROOT/gpurun_out/r05m_a2_prof.log 2>&1) && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/gpurun_out/r05m_cad1 -o run -- python3 $ROOT/bench.py --config cad1 --no-cpu-baseline --steps 10 \
  --warmup 3 > $ROOT/gpurun_out/r05m_cad1_prof.log 2>&1)
