# layer-0 weight gradient on the caller's stream (knob cad_last_wgrad_main): parity, A/B cfg2 / cfg4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cad_gpu.py tests/test_dp.py > gpurun_out/lw_test.log 2>&1 || exit 1
bash tools/ab_knob.sh lw2 3 cad_last_wgrad_main 0 1 || exit 1
bash tools/ab_knob.sh lw4 3 cad_last_wgrad_main 0 1 --config 4 || exit 1
