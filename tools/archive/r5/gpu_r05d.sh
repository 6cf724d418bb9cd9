# round 5: fragment prefetch in the split kernels (wgrad tap prefetch, forward / stride-2 dgrad step prefetch): unit
# tests on the new build, then an A/B of the two builds (ab/libvadhip_A.so = before, _B = after) on one box
set -o pipefail
T=r05d
PKG=causal-learning-based-video-anomaly-detection_paper_code_raw_amd
mkdir -p gpurun_out
cp ab/libvadhip_B.so $PKG/libvadhip.so || exit 1
true
for rep in 1 2 3; do
  for v in A B; do
    cp ab/libvadhip_$v.so $PKG/libvadhip.so || exit 1
    timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 40 --breakdown-out gpurun_out/${T}_bd${v}_$rep.json > gpurun_out/${T}_${v}_$rep.log 2>&1 || exit 1
  done
done
cp ab/libvadhip_B.so $PKG/libvadhip.so || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 40 --tune conv_wgrad_tr_pft=0 > gpurun_out/${T}_Bnopft.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_cad_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/${T}_cad.log 2>&1 || exit 1
