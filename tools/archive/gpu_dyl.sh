# per-layer dY buffers (no dY-reuse waits on the compute stream; knob cad_dy_per_layer): parity, A/B, trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cad_gpu.py tests/test_dp.py > gpurun_out/dyl_test.log 2>&1 || exit 1
bash tools/ab_knob.sh dyl2 3 cad_dy_per_layer 0 1 || exit 1
bash tools/ab_knob.sh dyl4 2 cad_dy_per_layer 0 1 --config 4 || exit 1
TAG=trdyl bash tools/gpu_trace.sh || exit 1
