# One A/B call on a box: conv kernel parity tests, knob A/B at config 2, per-label breakdown with the B setting
# usage: gpurun -- 'bash tools/gpu_r3_ab.sh TAG KNOB VA VB [REPS]'
set -o pipefail
TAG=$1; KNOB=$2; VA=$3; VB=$4; REPS=${5:-3}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "conv3x3 or split_accuracy or bf16_mode" > gpurun_out/${TAG}_ktest.log 2>&1 && \
bash tools/ab_knob.sh ${TAG} $REPS $KNOB $VA $VB && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --prof-every 1 --tune $KNOB=$VB --breakdown-out gpurun_out/${TAG}_bd_cfg2.json > gpurun_out/${TAG}_bd_cfg2.log 2>&1
