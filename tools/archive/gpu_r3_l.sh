# round 3 (l): unpredicated loads in the skinny / tail / dir_mid kernels, fused avgpool + temporal mean:
# cad + kernel GPU tests, chain marks, A/B vs the previous build (cfg 2, cfg 4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_kernels_gpu.py -x -q --timeout 250 --timeout-method thread -m gpu > gpurun_out/r3l_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py > gpurun_out/r3l_marks.txt 2>&1 && \
bash tools/ab_so.sh ldq 3 && bash tools/ab_so.sh ldq4 2 --config 4
