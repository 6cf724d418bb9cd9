# wave-specialised stride-1 conv kernel: kernel + cad parity with the knob on, then A/B cfg2 / cfg4 and a breakdown
set -o pipefail
mkdir -p gpurun_out
VAD_TUNE=conv_split_ws=2 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_cad_gpu.py > gpurun_out/ws_test.log 2>&1 || exit 1
bash tools/ab_knob.sh ws2 2 conv_split_ws 0 2 || exit 1
bash tools/ab_knob.sh ws4 2 conv_split_ws 0 2 --config 4 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 20 --tune conv_split_ws=2 --breakdown-out gpurun_out/ws2_bd.json > gpurun_out/ws2_bd.log 2>&1 || exit 1
