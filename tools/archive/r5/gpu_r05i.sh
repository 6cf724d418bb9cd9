# round 5: cad1 on the implicit-GEMM convs after the BN-finalize / bias-reduce rewrite: parity, then a tile / split
# sweep of its GEMMs (knobs conv_fwd_tile, conv_dgrad_tile, conv_wgrad_tile, ae_wgrad_blocks), and an a2 kernel-stats pass
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_ae_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05i_ae.log 2>&1 || exit 1
run() {  # tag, tune args...
  local tag=$1; shift
  timeout -k 10 120 python bench.py --config cad1 --no-cpu-baseline --steps 30 "$@" > gpurun_out/r05i_$tag.log 2>&1 || exit 1
}
run base
run f3 --tune conv_fwd_tile=3
run f5 --tune conv_fwd_tile=5
run f4 --tune conv_fwd_tile=4
run d3 --tune conv_dgrad_tile=3
run d5 --tune conv_dgrad_tile=5
run d0 --tune conv_dgrad_tile=0
run w4 --tune conv_wgrad_tile=4
run w5 --tune conv_wgrad_tile=5
run b1k --tune ae_wgrad_blocks=1024
run b4k --tune ae_wgrad_blocks=4096
run base2
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $ROOT/gpurun_out/r05i_a2 -o run -- python3 $ROOT/bench.py --config a2 --no-cpu-baseline --steps 10 \
  --warmup 3 > $ROOT/gpurun_out/r05i_a2_prof.log 2>&1) || exit 1
