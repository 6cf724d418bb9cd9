# A/B one box: gemm_kernel with one K slice in flight (A) vs two (B), cad1 and a2 bench lines alternated
set -o pipefail
bash tools/ab_so.sh r05v_cad1 3 --config cad1 && bash tools/ab_so.sh r05v_a2 3 --config a2
rc=$?
cp ab/libvadhip_B.so causal-learning-based-video-anomaly-detection_paper_code_raw_amd/libvadhip.so
exit $rc
