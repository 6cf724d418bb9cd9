# round 3 (u): kernel-mode chain marks, kernel GPU tests (weight-gradient reduce), rocprofv3 kernel stats of the
# default bench, A/B vs the last commit's build
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_cad_gpu.py -x -q --timeout 250 --timeout-method thread -m gpu > gpurun_out/r3u_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py --kernel > gpurun_out/r3u_kmarks.txt 2>&1 && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r3u_prof -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 3 --h2d-steps 0 > $ROOT/gpurun_out/r3u_prof_bench.log 2>&1) && \
bash tools/ab_so.sh wrd 3
