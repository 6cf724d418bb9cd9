# direct Conv3d for the minicausal plan: mc / a2 GPU tests, config-1 bench A/B of knob conv3d_direct, cad1 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mc_gpu.py tests/test_ae_gpu.py tests/test_a2_gpu.py tests/test_bbox.py -m gpu > gpurun_out/mcd_tests.log 2>&1 || exit 1
for v in 0 1; do
  timeout -k 10 200 python bench.py --config 1 --no-cpu-baseline --tune conv3d_direct=$v > gpurun_out/mcd_cfg1_v$v.json 2>/dev/null || exit 1
done
timeout -k 10 200 python bench.py --config cad1 --no-cpu-baseline > gpurun_out/mcd_cad1.json 2>/dev/null || exit 1
