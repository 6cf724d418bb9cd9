# a2: the plan's output / loss-grad copies in one launch each (B) vs one copy per tensor (A): a2 GPU tests on B, then
# a2 lines alternated on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_a2_gpu.py tests/test_mc_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r05ac_tests.log 2>&1 || exit 1
bash tools/ab_so.sh r05ac_a2 3 --config a2
rc=$?
cp ab/libvadhip_B.so causal-learning-based-video-anomaly-detection_paper_code_raw_amd/libvadhip.so
exit $rc
