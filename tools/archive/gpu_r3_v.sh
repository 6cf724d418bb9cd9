# round 3 (v): detector layer 0 on the split-bf16 dense kernel: cad GPU tests, kernel-mode chain marks for
# det_x3 = 0 / 16 / 32, knob A/B (0 vs 16, 16 vs 32)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cad_gpu.py -x -q --timeout 250 --timeout-method thread -m gpu > gpurun_out/r3v_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py --kernel det_x3=0 > gpurun_out/r3v_kmarks_0.txt 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py --kernel det_x3=16 > gpurun_out/r3v_kmarks_16.txt 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py --kernel det_x3=32 > gpurun_out/r3v_kmarks_32.txt 2>&1 && \
bash tools/ab_knob.sh detx 2 det_x3 0 16 && bash tools/ab_knob.sh detx32 2 det_x3 16 32
