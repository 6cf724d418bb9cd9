# round-2: backbone weight gradients on their own stream (double-buffered dY)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_dp.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2u_cad.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2u_bd.json > gpurun_out/r2u_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 > gpurun_out/r2u_bench2.log 2>&1
