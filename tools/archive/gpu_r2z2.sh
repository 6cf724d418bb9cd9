# round-2: weight-gradient grid sizes under stream concurrency, finer sweep
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 "$@"; }
for rep in 1 2; do
for v in "384 384 384" "320 320 320" "448 448 448" "384 512 384" "384 384 512" "512 384 384" "384 256 384"; do
  set -- $v
  run --tune conv_wgrad_patch_blocks=$1 --tune conv_wgrad_s2_blocks=$2 --tune conv_wgrad_s1_nt_blocks=$3 > gpurun_out/r2z2_$1_$2_$3_$rep.log 2>&1 || exit 1
done
done
