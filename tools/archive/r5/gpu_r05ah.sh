# cad1 1-channel weight gradient on 4-channel quads x 2 taps per thread (B) vs 1 channel x 2 taps (A): cad1 GPU tests
# on B, then cad1 lines alternated on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ae_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r05ah_tests.log 2>&1 || exit 1
bash tools/ab_so.sh r05ah_cad1 3 --config cad1
rc=$?
cp ab/libvadhip_B.so causal-learning-based-video-anomaly-detection_paper_code_raw_amd/libvadhip.so
exit $rc
