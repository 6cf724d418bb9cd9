# round-2: stem epilogue on permlane32 swaps -- stem tests, breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cad_gpu.py -x -v -m gpu -k "stem or reference" --timeout 200 --timeout-method thread > gpurun_out/r2n_cad.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2n_bd.json > gpurun_out/r2n_bench.log 2>&1
