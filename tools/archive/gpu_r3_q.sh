# round 3 (q): dir_mid (group reduce-scatter layers, layer-1 input gradient folded in), mlp_tail 1024-thread
# default with bounded K-slices, skinny dgrad single load batch: cad GPU tests, phase cycles, chain marks, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_kernels_gpu.py -x -q --timeout 250 --timeout-method thread -m gpu > gpurun_out/r3t_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py head_dbg=1 > gpurun_out/r3t_marks.txt 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py > gpurun_out/r3t_marks_nodbg.txt 2>&1 && \
bash tools/ab_so.sh dmt 3 && bash tools/ab_so.sh dmt4 2 --config 4
