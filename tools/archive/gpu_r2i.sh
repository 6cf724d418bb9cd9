# round-2: stride-2 split-bf16 weight gradient -- kernel tests, pinned CAD gradients, per-layer breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k "wgrad or bf16_mode" --timeout 200 --timeout-method thread > gpurun_out/r2i_kt.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2i_cad.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2i_bd.json > gpurun_out/r2i_bench.log 2>&1
