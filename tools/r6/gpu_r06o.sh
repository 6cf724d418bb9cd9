set -o pipefail
mkdir -p gpurun_out
PKG=causal-learning-based-video-anomaly-detection_paper_code_raw_amd
VARIANTS="A B D" bash tools/r6/gpu_standalone_ab.sh r06o --layers 2,4,6 --ops dgrad || exit 1
bash tools/ab_so.sh r06o 3 || exit 1
cp ab/libvadhip_D.so $PKG/libvadhip.so
