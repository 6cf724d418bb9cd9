# round 3 (g): bbox / mc / a2 GPU tests with the block-per-bin adaptive average pool, then the config-5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bbox.py tests/test_mc_gpu.py tests/test_a2_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3g_tests.log 2>&1 && \
timeout -k 10 200 python bench.py --config 5 --steps 20 > gpurun_out/r3g_cfg5.log 2>&1
