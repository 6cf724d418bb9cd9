# round-2: fused stem without LDS atomics (vertical fold in registers, direct pooled stores) -- parity, A/B cfg2 + cfg4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cad_gpu.py -k "stem or config4 or full_size" > gpurun_out/r2am_test.log 2>&1 || exit 1
bash tools/ab_so.sh r2am2 3 || exit 1
bash tools/ab_so.sh r2am4 2 --config 4 || exit 1
