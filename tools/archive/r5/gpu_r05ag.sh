# a2 conv3d_1 weight gradient on 4-channel quads x 2 pairs per thread (B) vs 1 channel x 6 pairs (A): a2 GPU tests on
# B, then a2 lines alternated on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_a2_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r05ag_tests.log 2>&1 || exit 1
bash tools/ab_so.sh r05ag_a2 3 --config a2
rc=$?
cp ab/libvadhip_B.so causal-learning-based-video-anomaly-detection_paper_code_raw_amd/libvadhip.so
exit $rc
