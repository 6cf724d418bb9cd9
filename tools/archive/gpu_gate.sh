# detector gate: cad parity (incl. forced-detection goldens) + DP tests, then A/B cfg2 / cfg4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cad_gpu.py tests/test_dp.py > gpurun_out/gate_test.log 2>&1 || exit 1
bash tools/ab_knob.sh gate2 3 cad_det_gate 0 1 || exit 1
bash tools/ab_knob.sh gate4 2 cad_det_gate 0 1 --config 4 || exit 1
