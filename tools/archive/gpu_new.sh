set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_mc_gpu.py tests/test_a2_gpu.py tests/test_bbox.py -q -m gpu > gpurun_out/new.log 2>&1
