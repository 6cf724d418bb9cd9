# round 5: per-kernel durations of the fragment-prefetch builds (ab/libvadhip_A.so = before, _B = after), config 2
# and config 4, from rocprofv3 kernel-trace stats (the step-level A/B hides which kernels won and which lost)
set -o pipefail
PKG=causal-learning-based-video-anomaly-detection_paper_code_raw_amd
mkdir -p gpurun_out
ROOT=$(pwd)
for v in A B; do
  cp $ROOT/ab/libvadhip_$v.so $ROOT/$PKG/libvadhip.so || exit 1
  for c in 2 4; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $ROOT/gpurun_out/r05f_${v}_c$c -o run -- python3 $ROOT/bench.py --config $c --no-cpu-baseline --h2d-steps 0 \
      --steps 20 > $ROOT/gpurun_out/r05f_${v}_c$c.log 2>&1) || exit 1
  done
done
cp $ROOT/ab/libvadhip_B.so $ROOT/$PKG/libvadhip.so || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/gpurun_out/r05f_Bnp_c2 -o run -- python3 $ROOT/bench.py --no-cpu-baseline --h2d-steps 0 --steps 20 \
  --tune conv_wgrad_tr_pft=0 > $ROOT/gpurun_out/r05f_Bnp_c2.log 2>&1) || exit 1
