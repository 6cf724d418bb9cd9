# PMC passes (stall / instruction mix / LDS conflicts) of tools/r6/conv_standalone.py for ab/libvadhip_A.so and
# ab/libvadhip_B.so on one box.  usage: gpurun -- 'bash tools/r6/gpu_pmc_ab.sh TAG [conv_standalone args...]'
set -o pipefail
TAG=$1; shift
ROOT=$(pwd)
PKG=causal-learning-based-video-anomaly-detection_paper_code_raw_amd
mkdir -p gpurun_out
for v in A B; do
  cp ab/libvadhip_$v.so $PKG/libvadhip.so || exit 1
  O=$ROOT/gpurun_out/${TAG}_$v
  ( cd /tmp && export TMPDIR=/tmp && \
    timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d ${O}_pB -o run -- python3 $ROOT/tools/r6/conv_standalone.py --reps 5 "$@" > ${O}_pB.log 2>&1 && \
    timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d ${O}_pA -o run -- python3 $ROOT/tools/r6/conv_standalone.py --reps 5 "$@" > ${O}_pA.log 2>&1 ) || exit 1
done
