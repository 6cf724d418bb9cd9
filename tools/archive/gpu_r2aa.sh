# round-2: new weight-gradient grid defaults -- tests, config 2 and 4 benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_kernels_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2aa_t.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 > gpurun_out/r2aa_b2.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 > gpurun_out/r2aa_b2b.log 2>&1 && \
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 > gpurun_out/r2aa_b4.log 2>&1
