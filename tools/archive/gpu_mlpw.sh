# 1024-thread detector tail (knob mlp_tail_wide): parity, A/B cfg2 / cfg4, a kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cad_gpu.py tests/test_kernels_gpu.py > gpurun_out/mw_test.log 2>&1 || exit 1
bash tools/ab_knob.sh mw2 3 mlp_tail_wide 0 1 || exit 1
bash tools/ab_knob.sh mw4 2 mlp_tail_wide 0 1 --config 4 || exit 1
TAG=trmw bash tools/gpu_trace.sh || exit 1
