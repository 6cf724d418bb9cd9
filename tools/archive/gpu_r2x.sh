# round-2: split-bf16 stride-2 input gradient (parity classes sharing one dY patch)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2x_kt.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2x_cad.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2x_bd.json > gpurun_out/r2x_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --tune conv_dgrad_s2_x3=0 --breakdown-out gpurun_out/r2x_bd0.json > gpurun_out/r2x_bench0.log 2>&1 && \
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2x_bd4.json > gpurun_out/r2x_cfg4.log 2>&1
