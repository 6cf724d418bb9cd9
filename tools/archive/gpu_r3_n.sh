# round 3 (n): dir_mid with inline lane selects + one-batch weight loads, detector/head chain on the caller's stream:
# cad + kernel GPU tests, dir_mid cycles, chain marks, A/B vs the last commit's build (cfg 2, cfg 4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_kernels_gpu.py -x -q --timeout 250 --timeout-method thread -m gpu > gpurun_out/r3n_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py head_dbg=1 > gpurun_out/r3n_marks.txt 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py > gpurun_out/r3n_marks_nodbg.txt 2>&1 && \
bash tools/ab_so.sh chn 3 && bash tools/ab_so.sh chn4 2 --config 4
