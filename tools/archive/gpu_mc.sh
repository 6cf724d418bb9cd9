set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_mc_gpu.py -x -q -m gpu > gpurun_out/mc.log 2>&1
