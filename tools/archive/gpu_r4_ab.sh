# A/B of one library knob on one box for configs 2 and 4, after the cad GPU tests.
# usage: gpurun -- 'bash tools/gpu_r4_ab.sh TAG KNOB VA VB [pytest -k expr]'
set -o pipefail
TAG=$1; KNOB=$2; VA=$3; VB=$4; K=${5:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -k "$K" -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
fi
for cfg in 2 4; do
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --h2d-steps 0 --steps 30 --tune $KNOB=$VA > gpurun_out/${TAG}_c${cfg}_A_$rep.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --h2d-steps 0 --steps 30 --tune $KNOB=$VB > gpurun_out/${TAG}_c${cfg}_B_$rep.json 2>/dev/null || exit 1
done
done
