# cad step optimizer (sqsum / AdamW) with batched branch-free chunk loads (B) vs HEAD (A): cad GPU tests on B, then
# config-2 lines alternated on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_cad_gpu.py tests/test_dp.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05aa_tests.log 2>&1 || exit 1
bash tools/ab_so.sh r05aa_cfg2 3
rc=$?
cp ab/libvadhip_B.so causal-learning-based-video-anomaly-detection_paper_code_raw_amd/libvadhip.so
exit $rc
