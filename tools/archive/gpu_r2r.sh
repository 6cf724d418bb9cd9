# round-2: x3 conv prefetch no longer drained before the MFMAs (unconditional loads + explicit vmcnt after stash)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2r_kt.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2r_cad.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2r_bd.json > gpurun_out/r2r_bench.log 2>&1
