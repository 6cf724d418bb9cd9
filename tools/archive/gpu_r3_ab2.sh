# Full GPU tests, then a knob A/B at configs 2 and 4 plus a per-label breakdown with the B setting
# usage: gpurun -- 'bash tools/gpu_r3_ab2.sh TAG KNOB VA VB [REPS]'
set -o pipefail
TAG=$1; KNOB=$2; VA=$3; VB=$4; REPS=${5:-3}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 && \
bash tools/ab_knob.sh ${TAG} $REPS $KNOB $VA $VB && \
bash tools/ab_knob.sh ${TAG}c4 2 $KNOB $VA $VB --config 4 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --prof-every 1 --tune $KNOB=$VB --breakdown-out gpurun_out/${TAG}_bd_cfg2.json > gpurun_out/${TAG}_bd_cfg2.log 2>&1
