# round-2: stall breakdown of the conv kernels (two PMC passes over a short bench)
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmc_stallA -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 2 --h2d-steps 0 > $ROOT/gpurun_out/pmc_stallA.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmc_stallB -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 2 --h2d-steps 0 > $ROOT/gpurun_out/pmc_stallB.log 2>&1
