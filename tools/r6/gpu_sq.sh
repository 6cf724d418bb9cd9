# early squared-norm pass: cad / dp GPU tests, then A/B of knob cad_sq_early (1 on, 0 off) at configs 2 and 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cad_gpu.py tests/test_dp.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sq_tests.log 2>&1 || exit 1
bash tools/ab_knob.sh sqab 3 cad_sq_early 0 1 || exit 1
bash tools/ab_knob.sh sqab4 2 cad_sq_early 0 1 --config 4 || exit 1
