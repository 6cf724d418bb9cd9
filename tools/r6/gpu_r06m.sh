set -o pipefail
mkdir -p gpurun_out
PKG=causal-learning-based-video-anomaly-detection_paper_code_raw_amd
timeout -k 10 600 python -u -m pytest tests/test_a2_gpu.py tests/test_ae_gpu.py tests/test_grad64.py tests/test_mc_gpu.py tests/test_cad_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06m_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config a2 --no-cpu-baseline > gpurun_out/r06m_a2_D.json 2> gpurun_out/r06m_a2_D.err || exit 1
VARIANTS="A B C D" bash tools/r6/gpu_standalone_ab.sh r06m --layers 2,4,6 --ops dgrad || exit 1
cp ab/libvadhip_D.so $PKG/libvadhip.so
