# round 3 (i): cad GPU tests with the row-parallel avgpool backward, A/B vs the previous build (cfg 2, cfg 4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_kernels_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r3i_tests.log 2>&1 && \
bash tools/ab_so.sh apbwd 3 && bash tools/ab_so.sh apbwd4 2 --config 4
