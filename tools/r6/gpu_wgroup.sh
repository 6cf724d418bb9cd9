# weight-gradient group combine: kernel tests, cad parity, knob A/B (0 = off, 8 = on) at configs 2 and 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad or bf16_native" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/wg_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py -k "backward_matches_oracle_full_size or hip_step_matches or staged or config4" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/wg_cad.log 2>&1 || exit 1
bash tools/ab_knob.sh wgab 3 conv_wgrad_group 0 8 || exit 1
bash tools/ab_knob.sh wgab4 2 conv_wgrad_group 0 8 --config 4 || exit 1
