# round-2: detector input gradient ahead of its weight grads (critical path into the backbone backward) -- A/B cfg2, cfg4
set -o pipefail
bash tools/ab_so.sh r2al2 3 || exit 1
bash tools/ab_so.sh r2al4 2 --config 4 || exit 1
