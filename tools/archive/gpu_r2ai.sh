# round-2: head MLP phases (quad-split dots, fused independent layers) -- parity, cycle breakdown, A/B vs HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cad_gpu.py > gpurun_out/r2ai_test.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 2 --warmup 1 --tune head_dbg=1 > gpurun_out/r2ai_dbg.log 2>&1 || exit 1
bash tools/ab_so.sh r2ai 3
