# hardened parity tests + one kernel-trace timeline per config 2 and 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -k "module_api or full_size or config4 or config5_packed or mixed_t" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1 && \
TAG=r04tr2 bash tools/gpu_trace.sh --config 2 && TAG=r04tr4 bash tools/gpu_trace.sh --config 4 && \
timeout -k 10 300 python bench.py > gpurun_out/r04g_bench_cfg2.json 2> gpurun_out/r04g_bench_cfg2.err
