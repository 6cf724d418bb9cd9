# grid of the last (stand-alone) weight gradient: A/B 448 (the shared-GPU grid) vs 512 / 1024, cfg2 and cfg4
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_knob.sh al2a 2 conv_wgrad_alone_blocks 448 512 || exit 1
bash tools/ab_knob.sh al2b 2 conv_wgrad_alone_blocks 448 1024 || exit 1
bash tools/ab_knob.sh al4a 2 conv_wgrad_alone_blocks 448 512 --config 4 || exit 1
