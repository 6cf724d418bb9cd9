# column-major BN-backward partials: parity (cad incl. stem grads, DP/SyncBN, minicausal), bench, trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cad_gpu.py tests/test_dp.py tests/test_mc_gpu.py > gpurun_out/bf_test.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 > gpurun_out/bf_b2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --config 4 > gpurun_out/bf_b4.log 2>&1 || exit 1
TAG=trbf bash tools/gpu_trace.sh || exit 1
