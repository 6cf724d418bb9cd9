# final round-5 build: full validation (tools/gpu_full.sh) then rocprofv3 kernel stats of the cad1 and a2 lines
set -o pipefail
bash tools/gpu_full.sh r05c || exit 1
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r05c_cad1_trace -o run -- python3 $ROOT/bench.py --config cad1 --no-cpu-baseline --steps 20 > $ROOT/gpurun_out/r05c_cad1_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r05c_a2_trace -o run -- python3 $ROOT/bench.py --config a2 --no-cpu-baseline --steps 20 > $ROOT/gpurun_out/r05c_a2_trace.log 2>&1
