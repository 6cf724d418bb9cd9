# minicausal GPU tests + config-1 bench + knob A/B (maxpool3d_bwd_win 0 / 1) + kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_mc_gpu.py tests/test_grad64.py -k "mc" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/mc_tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --config 1 --no-cpu-baseline --tune maxpool3d_bwd_win=0 > gpurun_out/mc_A_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --config 1 --no-cpu-baseline > gpurun_out/mc_B_$i.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/mcprof2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 1 --no-cpu-baseline --steps 10 > gpurun_out/mcprof2.log 2>&1 || exit 1
