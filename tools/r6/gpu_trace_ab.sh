# kernel traces of one bench config under two values of a knob (A, B): rocprofv3 --kernel-trace --stats each
# usage: bash tools/r6/gpu_trace_ab.sh TAG KNOB VA VB [bench args]
set -o pipefail
TAG=$1; KNOB=$2; VA=$3; VB=$4; shift 4
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in A B; do
  val=$VA; [ $v = B ] && val=$VB
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/${TAG}_$v -o run -- python3 $ROOT/bench.py --no-cpu-baseline --h2d-steps 0 --steps 20 --tune $KNOB=$val "$@" > $ROOT/gpurun_out/${TAG}_$v.log 2>&1 || exit 1
done
