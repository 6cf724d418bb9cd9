# round-2: weight-gradient grid sizes now that the weight gradients share the GPU with the input gradients
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 "$@"; }
for rep in 1 2; do
run > gpurun_out/r2z_base_$rep.log 2>&1 || exit 1
run --tune conv_wgrad_patch_blocks=256 --tune conv_wgrad_s2_blocks=256 --tune conv_wgrad_s1_nt_blocks=256 > gpurun_out/r2z_256_$rep.log 2>&1 || exit 1
run --tune conv_wgrad_patch_blocks=384 --tune conv_wgrad_s2_blocks=384 --tune conv_wgrad_s1_nt_blocks=384 > gpurun_out/r2z_384_$rep.log 2>&1 || exit 1
run --tune conv_wgrad_patch_blocks=1024 --tune conv_wgrad_s2_blocks=1024 --tune conv_wgrad_s1_nt_blocks=1024 > gpurun_out/r2z_1024_$rep.log 2>&1 || exit 1
done
