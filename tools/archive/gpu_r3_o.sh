# round 3 (o): detector layer-0 split-K reduce fused into the layer 1-4 kernel: cad GPU tests, phase cycles
# (head_dbg=1), chain marks, A/B vs the last commit's build (cfg 2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_kernels_gpu.py -x -q --timeout 250 --timeout-method thread -m gpu > gpurun_out/r3o_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py head_dbg=1 > gpurun_out/r3o_marks.txt 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py > gpurun_out/r3o_marks_nodbg.txt 2>&1 && \
bash tools/ab_so.sh skr 3
