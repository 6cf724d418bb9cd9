# round-2 check: full GPU suite, smoke, default bench (with CPU baseline) + breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2_gt.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r2_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --breakdown-out gpurun_out/r2_bd.json > gpurun_out/r2_bench_bd.log 2>&1
