# stage-2 backward (DP: backbone not held behind the causal-head backward): parity + DP tests, 2-rank gloo rehearsal
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cad_gpu.py tests/test_dp.py > gpurun_out/st2_test.log 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > gpurun_out/st2_dp2.log 2>&1 || exit 1
