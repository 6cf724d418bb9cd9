# cad1 weight gradients on a side stream (A/B), a2 column-sum / conv1-reduce fixes: tests then bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ae_gpu.py tests/test_a2_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r05q_tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --config cad1 --no-cpu-baseline > gpurun_out/r05q_cad1_side_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --config cad1 --no-cpu-baseline --tune ae_wgrad_stream=0 > gpurun_out/r05q_cad1_main_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --config a2 --no-cpu-baseline > gpurun_out/r05q_a2_$i.json 2>/dev/null || exit 1
done
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r05q_cad1_trace -o run -- python3 $ROOT/bench.py --config cad1 --no-cpu-baseline --steps 20 > $ROOT/gpurun_out/r05q_cad1_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r05q_a2_trace -o run -- python3 $ROOT/bench.py --config a2 --no-cpu-baseline --steps 20 > $ROOT/gpurun_out/r05q_a2_trace.log 2>&1
