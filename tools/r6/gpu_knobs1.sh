# A/B of the detector-gate and prep-stream knobs (config 2), then a kernel + HIP API trace of the default bench
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_knob.sh kgate 2 cad_det_gate 1 0 || exit 1
bash tools/ab_knob.sh kprep 2 cad_prep_stream 1 0 || exit 1
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $ROOT/gpurun_out/hiptr -o run -- python3 $ROOT/bench.py --no-cpu-baseline --h2d-steps 0 --steps 10 --warmup 3 > $ROOT/gpurun_out/hiptr.log 2>&1 || exit 1
