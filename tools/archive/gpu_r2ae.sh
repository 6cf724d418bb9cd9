# round-2: upper bound of the causal head's share of the critical path (head kernels skipped; results wrong)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 > gpurun_out/r2ae_0_$rep.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune dbg_skip_bnred=2 > gpurun_out/r2ae_2_$rep.log 2>&1 || exit 1
done
