# cad1: small-layer BN reduce + finalize fused (knob ae_bn_fuse), tests then alternated bench lines on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ae_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r05y_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python bench.py --config cad1 --no-cpu-baseline --tune ae_bn_fuse=$v > gpurun_out/r05y_cad1_${v}_$rep.json 2>/dev/null || exit 1
  done
done
