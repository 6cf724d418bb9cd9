# round 3 (c): conv + cad GPU tests on the stride-2 8-wave forward, then an A/B of knob conv_split_s2big
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_kernels_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1 && \
bash tools/ab_knob.sh s2big 3 conv_split_s2big 0 1
