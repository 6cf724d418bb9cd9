# a2 / cad1 GPU tests, then the a2 bench and its kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_a2_gpu.py tests/test_ae_gpu.py tests/test_grad64.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/a2k_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config a2 --no-cpu-baseline > gpurun_out/a2k_bench.log 2>&1 || exit 1
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/a2k_trace -o run -- python3 $ROOT/bench.py --config a2 --no-cpu-baseline --steps 20 > $ROOT/gpurun_out/a2k_trace.log 2>&1 || exit 1
