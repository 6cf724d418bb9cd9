# round 5: DP / data-path GPU tests and a config-2 bench on one box
set -o pipefail
TAG=${1:-r05a}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dp.py tests/test_data.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_dp.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_cfg2.json 2> gpurun_out/${TAG}_bench_cfg2.err
