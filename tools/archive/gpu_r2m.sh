# round-2: one-pass frozen stem (conv1 + BN sums + raw max/min pooling; bn1+ReLU on load in layer1.0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cad_gpu.py tests/test_dp.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2m_cad.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --breakdown-out gpurun_out/r2m_bd.json > gpurun_out/r2m_bench.log 2>&1
