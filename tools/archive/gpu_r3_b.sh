# round 3 (b): config-4 per-rank bf16 errors, the DP tests incl. RCCL world-1, bench config 2, the CPU-threads probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cad_gpu.py -x -v -s --timeout 250 --timeout-method thread -k "config4_shape_per_rank or second_backward" > gpurun_out/r3b_cfg4.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_dp.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r3b_dp.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r3b_bench.log 2>&1 && \
timeout -k 10 200 python tools/cpu_threads_probe.py > gpurun_out/r3b_cpuprobe.log 2>&1
