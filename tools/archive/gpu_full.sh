# Round-end rehearsal: GPU parity tests, smoke, default bench, cad1 bench, rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --config cad1 > gpurun_out/bench_cad1.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 20 > $ROOT/gpurun_out/prof_bench.log 2>&1
