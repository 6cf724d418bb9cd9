"""Data-parallel train step (CadTrainer): world-size-2 runs vs the single-process DDP emulation.

CPU: gloo, 2 processes, oracle-backed engine (tests the DP protocol: broadcasts, one grad+flag all-reduce, 1/world
scaling, RNG keyed by global clip index).  GPU: gloo, 2 processes sharing cuda:0, the real HIP engine."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.dp_util import OracleEngine, emulate_dp_steps, make_batches

SHAPE = dict(B=2, T=4, H=64, W=64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, use_gpu, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vad_amd.cad import CausalAnomalyDetector
        from vad_amd.train import CadTrainer
        torch.manual_seed(0)
        m = CausalAnomalyDetector()
        batches = make_batches(world, **SHAPE)
        x, y = batches[rank]
        if use_gpu:
            m = m.cuda()
            tr = CadTrainer(m, lr=3e-4, seed=0)
            x, y = x.cuda(), y.cuda()
        else:
            tr = CadTrainer(m, lr=3e-4, seed=0, engine=OracleEngine(m))
        for _ in range(2):
            tr.step(x, y)
        if rank == 0:
            torch.save({"params": tr.eng.params.cpu(), "bufs": tr.eng.bufs.cpu()}, out_path)
    finally:
        dist.destroy_process_group()


def _run(use_gpu, tmp_path):
    out = str(tmp_path / "rank0.pt")
    mp.spawn(_worker, args=(2, _free_port(), use_gpu, out), nprocs=2, join=True)
    return torch.load(out, weights_only=True)


def test_dp_protocol_cpu_gloo(tmp_path):
    got = _run(False, tmp_path)
    from vad_amd.cad import CausalAnomalyDetector
    torch.manual_seed(0)
    m = CausalAnomalyDetector()
    eng = OracleEngine(m)
    emulate_dp_steps(eng, make_batches(2, **SHAPE), 2, 2)
    np.testing.assert_allclose(got["params"].numpy(), eng.params.numpy(), rtol=0, atol=1e-6)
    np.testing.assert_allclose(got["bufs"].numpy(), eng.bufs.numpy(), rtol=0, atol=1e-6)


@pytest.mark.gpu
def test_dp_hip_engine_gloo_two_ranks(tmp_path):
    got = _run(True, tmp_path)
    from vad_amd.cad import CausalAnomalyDetector
    torch.manual_seed(0)
    m = CausalAnomalyDetector().cuda()
    eng = m.engine()
    batches = [(x.cuda(), y.cuda()) for x, y in make_batches(2, **SHAPE)]
    emulate_dp_steps(eng, batches, 2, 2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got["params"].numpy(), eng.params.cpu().numpy())
    np.testing.assert_array_equal(got["bufs"].numpy(), eng.bufs.cpu().numpy())
