# wave-specialised kernel for the wide stride-1 input gradients only (conv_split_ws=3): parity, A/B cfg2 / cfg4
set -o pipefail
mkdir -p gpurun_out
VAD_TUNE=conv_split_ws=3 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_cad_gpu.py > gpurun_out/ws3_test.log 2>&1 || exit 1
bash tools/ab_knob.sh ws32 3 conv_split_ws 0 3 || exit 1
bash tools/ab_knob.sh ws34 2 conv_split_ws 0 3 --config 4 || exit 1
