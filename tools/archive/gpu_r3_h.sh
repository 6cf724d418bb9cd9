# round 3 (h): conv kernel + cad GPU tests on the conflict-free weight-gradient staging, then A/B vs HEAD (cfg 2, cfg 4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_cad_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r3h_tests.log 2>&1 && \
bash tools/ab_so.sh wgremap 3 && bash tools/ab_so.sh wgremap4 3 --config 4
