# Two separate --pmc passes (FETCH_SIZE, WRITE_SIZE) over a short bench, for tools/pmc_traffic.py
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmc_fetch -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 2 > $ROOT/gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmc_write -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 2 > $ROOT/gpurun_out/pmc_write.log 2>&1
