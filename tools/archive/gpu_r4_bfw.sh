# staging geometry / branch-free BN selects (bf16 weight gradient, bf16 forward, pipelined fp32 forward): kernel and
# cad tests on build B, A/B of the two builds on configs 2 and 4, then the weight-gradient grid sweeps
set -o pipefail
mkdir -p gpurun_out
PKG=causal-learning-based-video-anomaly-detection_paper_code_raw_amd
cp ab/libvadhip_B.so $PKG/libvadhip.so || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4bfw_unit.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py -m gpu -x -q -k "config4 or full_size or reference" --timeout 200 --timeout-method thread > gpurun_out/r4bfw_cad.log 2>&1 || exit 1
bash tools/ab_so.sh r4bfw4 2 --config 4 || exit 1
bash tools/ab_so.sh r4bfw2 2 --config 2 || exit 1
cp ab/libvadhip_B.so $PKG/libvadhip.so || exit 1
bash tools/gpu_r4_sweep.sh
