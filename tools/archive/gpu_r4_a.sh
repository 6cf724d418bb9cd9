# Round 4: native bf16 conv kernels -- unit parity, config-4 model parity, then an A/B of config 4 (native vs the
# split kernels' bf16 mode) with per-kernel breakdowns.  usage: gpurun -- 'bash tools/gpu_r4_a.sh TAG'
set -o pipefail
TAG=${1:-r04a}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "bf16" -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_kern.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_cad_gpu.py -k "config4" -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_cfg4test.log 2>&1 && \
timeout -k 10 200 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --steps 30 --breakdown-out gpurun_out/${TAG}_bd_new.json > gpurun_out/${TAG}_cfg4_new.json 2> gpurun_out/${TAG}_cfg4_new.err && \
timeout -k 10 200 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_bfc=0 --breakdown-out gpurun_out/${TAG}_bd_old.json > gpurun_out/${TAG}_cfg4_old.json 2> gpurun_out/${TAG}_cfg4_old.err && \
timeout -k 10 200 python bench.py --config 4 --no-cpu-baseline --h2d-steps 0 --steps 30 > gpurun_out/${TAG}_cfg4_new2.json 2> gpurun_out/${TAG}_cfg4_new2.err
