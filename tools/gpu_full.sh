# Full validation on one MI355X box: every GPU test, smoke(), then bench.py at configs 2, 4, 5, 1, cad1 and a2
# (JSON lines under gpurun_out/); stops at the first failure.
# usage: gpurun --timeout 1200 -- 'bash tools/gpu_full.sh TAG'
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest_full.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_cfg2_full.json 2> gpurun_out/${TAG}_bench_cfg2.err && \
timeout -k 10 300 python bench.py --config 4 > gpurun_out/${TAG}_bench_cfg4.json 2> gpurun_out/${TAG}_bench_cfg4.err && \
timeout -k 10 300 python bench.py --config 5 > gpurun_out/${TAG}_bench_cfg5.json 2> gpurun_out/${TAG}_bench_cfg5.err && \
timeout -k 10 300 python bench.py --config 1 > gpurun_out/${TAG}_bench_cfg1.json 2> gpurun_out/${TAG}_bench_cfg1.err && \
timeout -k 10 300 python bench.py --config cad1 > gpurun_out/${TAG}_bench_cad1.json 2> gpurun_out/${TAG}_bench_cad1.err && \
timeout -k 10 300 python bench.py --config a2 > gpurun_out/${TAG}_bench_a2.json 2> gpurun_out/${TAG}_bench_a2.err
