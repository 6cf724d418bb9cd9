# round 3 (j): affine direct-classifier backward -- cad / kernel / DP GPU tests, then A/B of the knob (cfg 2, cfg 4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_cad_gpu.py tests/test_kernels_gpu.py tests/test_dp.py -x -q --timeout 250 --timeout-method thread -m gpu > gpurun_out/r3j_tests.log 2>&1 && \
bash tools/ab_knob.sh affine 3 cad_dir_affine 0 1 && bash tools/ab_knob.sh affine4 2 cad_dir_affine 0 1 --config 4
