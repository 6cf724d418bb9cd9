# stride-2 bf16 input gradient on 2-frame tiles: kernel tests, config-4 plan tests, A/B of knob conv_bfc_s2_ni2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bf16_native" -m gpu > gpurun_out/s2ni_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cad_gpu.py -k "bf16" -m gpu >> gpurun_out/s2ni_tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_bfc_s2_ni2=$v > gpurun_out/s2ni_cfg4_v${v}_r$r.json 2>/dev/null || exit 1
  done
done
