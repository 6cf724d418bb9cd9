set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_minicausal.py tests/test_cad_gpu.py tests/test_a2_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gt7.log 2>&1 && \
timeout -k 10 300 python -u tools/tune_wg_s2.py > gpurun_out/wg_s2.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --breakdown-out gpurun_out/bd7.json > gpurun_out/bench7.log 2>&1
