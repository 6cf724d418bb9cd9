# round-2: upper bound of fusing the BN backward reduce away (skip it; results wrong) -- timing only
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 > gpurun_out/r2ad_0_$rep.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune dbg_skip_bnred=1 > gpurun_out/r2ad_1_$rep.log 2>&1 || exit 1
done
