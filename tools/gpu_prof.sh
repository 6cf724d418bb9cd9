# profiles of one BASELINE config: rocprofv3 kernel-trace --stats of the bench, FETCH_SIZE, WRITE_SIZE, the
# MFMA-busy counters and the two stall passes, each in its own --pmc run (counter limits per pass: MI355X_MICROARCH.md).
# Usage: bash tools/gpu_prof.sh CONFIG TAG [extra bench args]   (outputs under gpurun_out/TAG_cfgCONFIG_*)
set -o pipefail
CFG=$1; TAG=$2; shift 2
mkdir -p gpurun_out
ROOT=$(pwd)
O=$ROOT/gpurun_out/${TAG}_cfg$CFG
B="$ROOT/bench.py --config $CFG --no-cpu-baseline --h2d-steps 0 $*"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_trace -o run -- python3 $B --steps 20 > ${O}_trace.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d ${O}_fetch -o run -- python3 $B --steps 3 --warmup 2 > ${O}_fetch.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d ${O}_write -o run -- python3 $B --steps 3 --warmup 2 > ${O}_write.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d ${O}_mfma -o run -- python3 $B --steps 3 --warmup 2 > ${O}_mfma.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d ${O}_stallA -o run -- python3 $B --steps 3 --warmup 2 > ${O}_stallA.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d ${O}_stallB -o run -- python3 $B --steps 3 --warmup 2 > ${O}_stallB.log 2>&1
