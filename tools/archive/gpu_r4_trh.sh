# half-image transposed-read weight gradient: kernel tests + cad subset on build B, A/B on config 2, then sweep2
set -o pipefail
mkdir -p gpurun_out
PKG=causal-learning-based-video-anomaly-detection_paper_code_raw_amd
cp ab/libvadhip_B.so $PKG/libvadhip.so || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k wgrad --timeout 120 --timeout-method thread > gpurun_out/r4trh_unit.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py -m gpu -x -q -k "full_size or reference" --timeout 200 --timeout-method thread > gpurun_out/r4trh_cad.log 2>&1 || exit 1
bash tools/ab_so.sh r4trh 3 --config 2 || exit 1
cp ab/libvadhip_B.so $PKG/libvadhip.so || exit 1
bash tools/gpu_r4_sweep2.sh
