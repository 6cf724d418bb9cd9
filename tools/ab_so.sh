# A/B of two builds of libvadhip.so on one box: ab/libvadhip_A.so vs ab/libvadhip_B.so, alternated per run
# usage: bash tools/ab_so.sh TAG [REPS] [extra bench args...]
set -o pipefail
TAG=$1; REPS=${2:-3}; shift 2
PKG=causal-learning-based-video-anomaly-detection_paper_code_raw_amd
mkdir -p gpurun_out
for rep in $(seq 1 $REPS); do
  for v in A B; do
    cp ab/libvadhip_$v.so $PKG/libvadhip.so || exit 1
    timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 "$@" > gpurun_out/${TAG}_${v}_$rep.log 2>&1 || exit 1
  done
done
