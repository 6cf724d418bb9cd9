# a2 / cad1 on the e03d665 build: repeated bench lines (box spread) and rocprofv3 kernel stats of each
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
for i in 1 2; do
  timeout -k 10 200 python bench.py --config a2 --no-cpu-baseline > gpurun_out/r05o_a2_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --config cad1 --no-cpu-baseline > gpurun_out/r05o_cad1_$i.json 2>/dev/null || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r05o_a2_trace -o run -- python3 $ROOT/bench.py --config a2 --no-cpu-baseline --steps 20 > $ROOT/gpurun_out/r05o_a2_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r05o_cad1_trace -o run -- python3 $ROOT/bench.py --config cad1 --no-cpu-baseline --steps 20 > $ROOT/gpurun_out/r05o_cad1_trace.log 2>&1
