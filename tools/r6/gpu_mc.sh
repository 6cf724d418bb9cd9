# minicausal GPU tests + config-1 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_mc_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/mc_tests.log 2>&1 || exit 1
for i in 1 2; do timeout -k 10 200 python bench.py --config 1 --no-cpu-baseline > gpurun_out/mc_bench_$i.log 2>&1 || exit 1; done
