# round-5 final-build profiles: configs 2 and 4 (kernel-trace stats + FETCH_SIZE / WRITE_SIZE / MFMA-busy / stall
# passes, tools/gpu_prof.sh), then cad1 and a2 kernel stats
set -o pipefail
ROOT=$(pwd)
bash tools/gpu_prof.sh 2 r05f && bash tools/gpu_prof.sh 4 r05f || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/gpurun_out/r05f_cad1_trace -o run -- python3 $ROOT/bench.py --config cad1 --no-cpu-baseline --steps 10 \
  --warmup 3 > $ROOT/gpurun_out/r05f_cad1_trace.log 2>&1) && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/gpurun_out/r05f_a2_trace -o run -- python3 $ROOT/bench.py --config a2 --no-cpu-baseline --steps 10 \
  --warmup 3 > $ROOT/gpurun_out/r05f_a2_trace.log 2>&1)
