# pre-split stride-2 Wd planes: cad GPU tests (incl. the bit-equality test), config-2 A/B of knob conv_dgrad_s2_w3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cad_gpu.py tests/test_kernels_gpu.py -m gpu > gpurun_out/w3_tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_dgrad_s2_w3=$v > gpurun_out/w3_cfg2_v${v}_r$r.json 2>/dev/null || exit 1
  done
done
