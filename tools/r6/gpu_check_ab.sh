# tests for the changed kernels, then a one-box A/B of ab/libvadhip_A.so vs ab/libvadhip_B.so (B left in place)
# usage: gpurun -- 'bash tools/r6/gpu_check_ab.sh TAG REPS "pytest targets" [bench args...]'
set -o pipefail
TAG=$1; REPS=$2; TESTS=$3; shift 3
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
bash tools/ab_so.sh $TAG $REPS "$@"
