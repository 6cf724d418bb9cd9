# round 3 (k): per-op marks of the post-backbone chain (config 2), default and mlp_tail_wide=1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/exp/chain_marks.py > gpurun_out/r3k_marks.txt 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py mlp_tail_wide=1 > gpurun_out/r3k_marks_wide.txt 2>&1
