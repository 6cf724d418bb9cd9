# round 3 (p): mlp_tail_fwd phase cycles over rows-per-block / block width
set -o pipefail
mkdir -p gpurun_out
for cfg in "mlp_tail_rb=4" "mlp_tail_rb=4 mlp_tail_wide=1" "mlp_tail_rb=2" "mlp_tail_rb=2 mlp_tail_wide=1" "mlp_tail_rb=8"; do
  tag=$(echo $cfg | tr ' =' '__')
  timeout -k 10 200 python -u tools/exp/chain_marks.py head_dbg=1 $cfg > gpurun_out/r3p_$tag.txt 2>&1 || exit 1
done
