# round-2 profiles: rocprofv3 kernel stats of the default bench, then FETCH_SIZE, WRITE_SIZE and the MFMA-busy
# counters in separate --pmc passes (tools/family_stats.py, pmc_traffic.py, pmc_mfma.py summarise them)
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof -o run -- python3 $ROOT/bench.py --no-cpu-baseline --h2d-steps 0 --steps 20 > $ROOT/gpurun_out/prof_bench.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmc_fetch -o run -- python3 $ROOT/bench.py --no-cpu-baseline --h2d-steps 0 --steps 3 --warmup 2 > $ROOT/gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmc_write -o run -- python3 $ROOT/bench.py --no-cpu-baseline --h2d-steps 0 --steps 3 --warmup 2 > $ROOT/gpurun_out/pmc_write.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmc_mfma -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 2 --h2d-steps 0 > $ROOT/gpurun_out/pmc_mfma.log 2>&1
