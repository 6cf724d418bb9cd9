# round-2: bench configs 1/2/5 (new fields), data + mc GPU tests, MFMA-utilisation PMC pass
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_data.py tests/test_mc_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2c_gt.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r2c_bench2.log 2>&1 && \
timeout -k 10 300 python bench.py --config 1 --steps 10 --warmup 2 > gpurun_out/r2c_bench1.log 2>&1 && \
timeout -k 10 300 python bench.py --config 5 > gpurun_out/r2c_bench5.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmc_mfma -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 2 --h2d-steps 0 > $ROOT/gpurun_out/pmc_mfma.log 2>&1
