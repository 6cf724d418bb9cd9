# round-2: A/B of the side-stream weight prep and the weight-gradient stream, same box, alternating runs
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in "1 1" "0 1" "1 0" "0 0"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune cad_prep_stream=$1 --tune cad_wgrad_stream=$2 > gpurun_out/r2v_${1}${2}_$rep.log 2>&1 || exit 1
done
done
