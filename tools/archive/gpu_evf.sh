# plan sync events without the system-scope fence (knob cad_event_sysfence): parity, A/B cfg2 / cfg4, trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cad_gpu.py tests/test_dp.py > gpurun_out/evf_test.log 2>&1 || exit 1
bash tools/ab_knob.sh evf2 3 cad_event_sysfence 1 0 || exit 1
bash tools/ab_knob.sh evf4 2 cad_event_sysfence 1 0 --config 4 || exit 1
TAG=trevf bash tools/gpu_trace.sh || exit 1
