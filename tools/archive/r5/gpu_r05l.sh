# round 5: a2 conv3d_2 / conv3d_3 on implicit GEMMs + conv3d_1 on LDS halo tiles; a2 grad-norm parts: a2 / cad1 tests,
# a2 bench + kernel stats, then a config-2 A/B of the side-stream priority (knob cad_stream_prio)
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_a2_gpu.py tests/test_ae_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05l_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config a2 --steps 30 --cpu-seconds 8 > gpurun_out/r05l_a2.log 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/gpurun_out/r05l_a2 -o run -- python3 $ROOT/bench.py --config a2 --no-cpu-baseline --steps 10 \
  --warmup 3 > $ROOT/gpurun_out/r05l_a2_prof.log 2>&1) || exit 1
for rep in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 40 --tune cad_stream_prio=$v > gpurun_out/r05l_prio${v}_$rep.log 2>&1 || exit 1
  done
done
