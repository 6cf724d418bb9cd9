# round-2: stride-1 multi-co-tile weight gradient sweep (frames <= 16 wide: L5, L7)
set -o pipefail
mkdir -p gpurun_out
for nt in 0 2 4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --tune conv_wgrad_s1_nt=$nt --breakdown-out gpurun_out/r2k_bd_$nt.json > gpurun_out/r2k_bench_$nt.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --tune conv_wgrad_s1_nt=2 --tune conv_wgrad_s1_nt_blocks=1024 --breakdown-out gpurun_out/r2k_bd_2b.json > gpurun_out/r2k_bench_2b.log 2>&1
