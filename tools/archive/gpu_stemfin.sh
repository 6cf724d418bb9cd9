# column-major stem partials + no redundant final join: parity (cad, DP/SyncBN, kernels), bench, cfg4 trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cad_gpu.py tests/test_dp.py tests/test_kernels_gpu.py > gpurun_out/sf_test.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 > gpurun_out/sf_b2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --config 4 > gpurun_out/sf_b4.log 2>&1 || exit 1
TAG=trsf4 bash tools/gpu_trace.sh --config 4 || exit 1
