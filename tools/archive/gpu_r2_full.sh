# round-2 full validation: every GPU test, smoke(), the default bench (with CPU baseline and the H2D leg)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_full_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2_full_smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r2_full_bench.log 2>&1
