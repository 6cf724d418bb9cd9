# round-2: multi-co-tile weight gradients default on (stride 1 <= 16 wide, stride 2), vectorized split-K reduce
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k "wgrad or bf16_mode" --timeout 200 --timeout-method thread > gpurun_out/r2l_kt.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2l_cad.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2l_bd.json > gpurun_out/r2l_bench.log 2>&1
