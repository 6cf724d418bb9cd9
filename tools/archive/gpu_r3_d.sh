# round 3 (d): every GPU test, then an A/B of knob conv_split_s2big (stride-2 8-wave forward)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1 && \
bash tools/ab_knob.sh s2big 3 conv_split_s2big 0 1
