# BN-apply parity test, then the a2 profile set (kernel stats + PMC traffic / MFMA / stall passes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "bn_bwd_apply" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/apply_tests.log 2>&1 || exit 1
bash tools/gpu_prof.sh a2 r06a || exit 1
