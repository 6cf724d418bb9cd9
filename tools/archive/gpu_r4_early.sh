# early stem: GPU tests, then A/B of knob cad_stem_early on configs 2 and 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dp.py -m gpu -k "early or world1" -x -v --timeout 300 --timeout-method thread > gpurun_out/r4early_dp.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py -m gpu -x -q -k "full_size or config4 or reference or stem" --timeout 200 --timeout-method thread > gpurun_out/r4early_cad.log 2>&1 || exit 1
bash tools/gpu_r4_ab.sh r4early cad_stem_early 0 1
