# round 5: cad1 / a2 GEMM tile sweep on the final kernels (knobs conv_fwd_tile / conv_dgrad_tile / conv_wgrad_tile,
# ae_wgrad_blocks); tile ids: 0 128x32, 1 256x32, 2 64x64, 3 128x64, 4 64x128, 5 128x128
set -o pipefail
mkdir -p gpurun_out
run() {  # config tag tune...
  local c=$1 tag=$2; shift 2
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 30 "$@" > gpurun_out/r05n_${c}_$tag.log 2>&1 || exit 1
}
run cad1 base
run cad1 d1 --tune conv_dgrad_tile=1
run cad1 d3 --tune conv_dgrad_tile=3
run cad1 f3 --tune conv_fwd_tile=3
run cad1 w4 --tune conv_wgrad_tile=4
run cad1 w7 --tune conv_wgrad_tile=7
run cad1 b512 --tune ae_wgrad_blocks=512
run cad1 b2k --tune ae_wgrad_blocks=2048
run cad1 base2
run a2 base
run a2 d1 --tune conv_dgrad_tile=1
run a2 d2 --tune conv_dgrad_tile=2
run a2 f0 --tune conv_fwd_tile=0
run a2 f3 --tune conv_fwd_tile=3
run a2 base2
