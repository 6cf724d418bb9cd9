set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k wgrad > gpurun_out/kt.log 2>&1 && \
timeout -k 10 200 python tools/tune_conv.py --patch > gpurun_out/patch.log 2>&1
