# last check of the final build: every GPU test, smoke(), config-2 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04h_gputest.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04h_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r04h_bench_cfg2.json 2> gpurun_out/r04h_bench_cfg2.err && \
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/r04h_bench_cfg4.json 2> gpurun_out/r04h_bench_cfg4.err
