# branch-free K-contiguous dense loaders (B) vs HEAD (A): GEMM-path GPU tests on B, then cad1 / a2 lines alternated
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ae_gpu.py tests/test_a2_gpu.py tests/test_mc_gpu.py tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r05z_tests.log 2>&1 || exit 1
bash tools/ab_so.sh r05z_cad1 3 --config cad1 && bash tools/ab_so.sh r05z_a2 2 --config a2
rc=$?
cp ab/libvadhip_B.so causal-learning-based-video-anomaly-detection_paper_code_raw_amd/libvadhip.so
exit $rc
