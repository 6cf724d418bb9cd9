# round-2: deeper weight-load pipeline in the detector MLP tail
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2y_cad.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2y_bd.json > gpurun_out/r2y_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 > gpurun_out/r2y_bench2.log 2>&1
