# round 3 (f): bbox GPU tests on the implicit-GEMM encoder, then an A/B of knob bbox_im2col on config 5
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bbox.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3f_tests.log 2>&1 && \
timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline --steps 20 --tune bbox_im2col=1 > gpurun_out/r3f_cfg5_A.log 2>&1 && \
timeout -k 10 200 python bench.py --config 5 --steps 20 > gpurun_out/r3f_cfg5_B.log 2>&1
