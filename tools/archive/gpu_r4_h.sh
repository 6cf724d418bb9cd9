set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -k "config4" -x -v -s --timeout 250 --timeout-method thread > gpurun_out/r04h_tests.log 2>&1 ; \
TAG=r04tr2 bash tools/gpu_trace.sh --config 2 && TAG=r04tr4 bash tools/gpu_trace.sh --config 4 && \
timeout -k 10 300 python bench.py > gpurun_out/r04h_bench_cfg2.json 2> gpurun_out/r04h_bench_cfg2.err
