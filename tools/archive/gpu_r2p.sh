# round-2: bf16-operand stem for config 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cad_gpu.py -x -v -m gpu -k "config4 or stem" --timeout 200 --timeout-method thread > gpurun_out/r2p_cad.log 2>&1 && \
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2p_bd4.json > gpurun_out/r2p_cfg4.log 2>&1
