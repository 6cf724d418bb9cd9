# round 3 (w): BN backward reduce (wave-shuffle block tail, 4 rows in flight) and apply: cad / kernel / mc GPU tests,
# rocprofv3 kernel stats, A/B vs the last commit (cfg 2, cfg 4)
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_kernels_gpu.py tests/test_mc_gpu.py -x -q --timeout 250 --timeout-method thread -m gpu > gpurun_out/r3w_tests.log 2>&1 && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r3w_prof -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 3 --h2d-steps 0 > $ROOT/gpurun_out/r3w_prof_bench.log 2>&1) && \
bash tools/ab_so.sh bnr 3 && bash tools/ab_so.sh bnr4 2 --config 4
