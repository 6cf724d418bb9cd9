# layer-0 BN backward apply fused into its weight gradient: bit-equality test, cad GPU tests, config-2 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cad_gpu.py -m gpu > gpurun_out/bnf_tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_wgrad_bn_fused=$v > gpurun_out/bnf_cfg2_v${v}_r$r.json 2>/dev/null || exit 1
  done
done
