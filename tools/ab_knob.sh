# A/B of one library knob on one box: A = KNOB=VA, B = KNOB=VB, alternated per run
# usage: bash tools/ab_knob.sh TAG REPS KNOB VA VB [extra bench args...]
set -o pipefail
TAG=$1; REPS=$2; KNOB=$3; VA=$4; VB=$5; shift 5
mkdir -p gpurun_out
for rep in $(seq 1 $REPS); do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune $KNOB=$VA "$@" > gpurun_out/${TAG}_A_$rep.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune $KNOB=$VB "$@" > gpurun_out/${TAG}_B_$rep.log 2>&1 || exit 1
done
