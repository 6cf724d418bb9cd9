# round 3 (e): cad + kernel GPU tests on the cleaned build, the default bench with its per-kernel breakdown, host timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_kernels_gpu.py tests/test_dp.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r3e_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --breakdown-out gpurun_out/r3e_breakdown.json > gpurun_out/r3e_bench.log 2>&1 && \
timeout -k 10 120 python tools/exp/host_time.py > gpurun_out/r3e_host.log 2>&1
