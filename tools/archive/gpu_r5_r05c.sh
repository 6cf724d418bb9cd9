# round 5, first GPU call: DP / data tests, DMA-kernel unit tests, knob checks, bench A/Bs (config 2), bf16 config-4 test
set -o pipefail
T=r05c
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "wgrad or dgrad_s2" --timeout 120 --timeout-method thread > gpurun_out/${T}_kt.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/r5/knob_check.py conv_wgrad_dma 0 1 > gpurun_out/${T}_check_wdma.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --breakdown-out gpurun_out/${T}_bd0.json > gpurun_out/${T}_b0.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_wgrad_dma=1 --breakdown-out gpurun_out/${T}_bd1.json > gpurun_out/${T}_b1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_wgrad_dma=1 --tune conv_dgrad_s2_dma=1 --breakdown-out gpurun_out/${T}_bd2.json > gpurun_out/${T}_b2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_wgrad_dma=1 --tune cad_dy_planes=0 --tune cad_x_planes=0 --breakdown-out gpurun_out/${T}_bd3.json > gpurun_out/${T}_b3.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --breakdown-out gpurun_out/${T}_bd4.json > gpurun_out/${T}_b4.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune conv_wgrad_dma=1 --tune conv_dgrad_s2_dma=1 --breakdown-out gpurun_out/${T}_bd5.json > gpurun_out/${T}_b5.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_dp.py tests/test_data.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_dp.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_cad_gpu.py -m gpu -x -v -s -k "config4_shape_per_rank" --timeout 280 --timeout-method thread > gpurun_out/${T}_cfg4.log 2>&1 || exit 1
