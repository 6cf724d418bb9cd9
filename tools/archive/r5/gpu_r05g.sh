# round 5: config-4 bf16 parity with the direct classifier's ReLUs pinned, the a2 train-step bench line, a cad1 kernel
# trace (per-dispatch, for the direct-conv work), then per-kernel stats of the prefetch builds A / B (tools/r5/gpu_r05f.sh)
set -o pipefail
PKG=causal-learning-based-video-anomaly-detection_paper_code_raw_amd
mkdir -p gpurun_out
ROOT=$(pwd)
cp ab/libvadhip_C.so $PKG/libvadhip.so || exit 1
timeout -k 10 300 python -u -m pytest "tests/test_cad_gpu.py::test_config4_shape_per_rank[bf16]" -m gpu -x -q -s --timeout 280 --timeout-method thread > gpurun_out/r05g_bf16.log 2>&1
echo "bf16 test rc=$?"
timeout -k 10 300 python bench.py --config a2 --steps 30 --cpu-seconds 8 > gpurun_out/r05g_a2.log 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/gpurun_out/r05g_cad1 -o run -- python3 $ROOT/bench.py --config cad1 --no-cpu-baseline --steps 10 \
  --warmup 3 > $ROOT/gpurun_out/r05g_cad1.log 2>&1) || exit 1
bash tools/r5/gpu_r05f.sh; rc=$?
cp ab/libvadhip_C.so $PKG/libvadhip.so
exit $rc
