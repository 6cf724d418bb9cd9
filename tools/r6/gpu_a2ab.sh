# a2 knob A/B: bash tools/r6/gpu_a2ab.sh TAG KNOB VA VB REPS
set -o pipefail
mkdir -p gpurun_out
TAG=$1; KNOB=$2; VA=$3; VB=$4; REPS=$5
for rep in $(seq 1 $REPS); do
  timeout -k 10 200 python bench.py --config a2 --no-cpu-baseline --tune $KNOB=$VA > gpurun_out/${TAG}_A_$rep.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --config a2 --no-cpu-baseline --tune $KNOB=$VB > gpurun_out/${TAG}_B_$rep.log 2>&1 || exit 1
done
