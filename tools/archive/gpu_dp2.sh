# Rehearse bench.py's N>1 path on a one-GPU box: 2 ranks sharing cuda:0 over gloo (the driver's 8-GPU run uses RCCL)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > gpurun_out/dp2.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 3 --warmup 1 --config 5 --dist-backend gloo > gpurun_out/dp2_cfg5.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 3 --warmup 1 --config cad1 --dist-backend gloo > gpurun_out/dp2_cad1.log 2>&1
