# stand-alone conv timings of ab/libvadhip_A.so and ab/libvadhip_B.so on one box (B left in place)
# usage: gpurun -- 'bash tools/r6/gpu_standalone_ab.sh TAG [conv_standalone args...]'
set -o pipefail
TAG=$1; shift
PKG=causal-learning-based-video-anomaly-detection_paper_code_raw_amd
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${VARIANTS:-A B}; do
    cp ab/libvadhip_$v.so $PKG/libvadhip.so || exit 1
    timeout -k 10 120 python tools/r6/conv_standalone.py --tag $v "$@" >> gpurun_out/${TAG}_standalone.jsonl 2>> gpurun_out/${TAG}_standalone.err || exit 1
  done
done
