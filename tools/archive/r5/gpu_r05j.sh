# round 5: a2 head / loss as multi-block stage launches: a2 parity, a2 bench + kernel stats, cad1 bench
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_a2_gpu.py tests/test_ae_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05j_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config a2 --steps 30 --cpu-seconds 8 > gpurun_out/r05j_a2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config cad1 --steps 30 --cpu-seconds 8 > gpurun_out/r05j_cad1.log 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/gpurun_out/r05j_a2 -o run -- python3 $ROOT/bench.py --config a2 --no-cpu-baseline --steps 10 \
  --warmup 3 > $ROOT/gpurun_out/r05j_a2_prof.log 2>&1) || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/gpurun_out/r05j_cad1 -o run -- python3 $ROOT/bench.py --config cad1 --no-cpu-baseline --steps 10 \
  --warmup 3 > $ROOT/gpurun_out/r05j_cad1_prof.log 2>&1) || exit 1
