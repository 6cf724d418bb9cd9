# round 3: the cad GPU tests (new train-mode module API, config-4 per-rank, second-backward tests)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_cad_gpu.py -x -v -s --timeout 400 --timeout-method thread --durations=10 > gpurun_out/r3_cad_tests.log 2>&1
