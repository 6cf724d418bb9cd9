set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4geo_unit.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py -m gpu -x -q -k "full_size or config4 or reference" --timeout 200 --timeout-method thread > gpurun_out/r4geo_cad.log 2>&1 || exit 1
bash tools/ab_so.sh r4geo 3 --config 2
