# slab-sum reduces: cad1 / a2 / cad / mc GPU tests, then cad1, a2 and config-2 benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ae_gpu.py tests/test_a2_gpu.py tests/test_grad64.py tests/test_kernels_gpu.py tests/test_cad_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/red_tests.log 2>&1 || exit 1
for c in cad1 a2 2; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/red_bench_$c.log 2>&1 || exit 1; done
