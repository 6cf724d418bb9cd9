# a2: fused train step queued whole before its one host read of the losses (device NaN gate), a2 GPU tests, then
# a2 bench lines (same library)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_a2_gpu.py tests/test_mc_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r05ad_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --config a2 --no-cpu-baseline > gpurun_out/r05ad_a2_$i.json 2>/dev/null || exit 1
done
