# round-2: GRU recurrences without per-step store waits -- head cycle breakdown, cad parity tests, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 2 --warmup 1 --tune head_dbg=1 > gpurun_out/r2ag_dbg.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cad_gpu.py > gpurun_out/r2ag_test.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 > gpurun_out/r2ag_b$rep.log 2>&1 || exit 1
done
