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


def _worker(rank, world, port, use_gpu, out_path, frozen=False, skip_det=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import contextlib
        import io
        from vad_amd.cad import CausalAnomalyDetector
        from vad_amd.train import CadTrainer, apply_memory_efficient_training
        torch.manual_seed(0)
        m = CausalAnomalyDetector()
        if frozen:
            with contextlib.redirect_stdout(io.StringIO()):
                apply_memory_efficient_training(m)
        batches = make_batches(world, **SHAPE)
        x, y = batches[rank]
        if use_gpu:
            m = m.cuda()
            tr = CadTrainer(m, lr=3e-4, seed=0)
            x, y = x.cuda(), y.cuda()
        else:
            tr = CadTrainer(m, lr=3e-4, seed=0, engine=OracleEngine(m), skip_zero_detector=skip_det)
        for _ in range(2):
            tr.step(x, y)
        if rank == 0:
            torch.save({"params": tr.eng.params.cpu(), "bufs": tr.eng.bufs.cpu(), "grads": tr.eng.grads.cpu(),
                        "allreduce_floats": tr.allreduce_floats, "det_range": list(tr.det_range),
                        "det_flag_sum": getattr(tr, "det_flag_sum", -1.0)}, out_path)
    finally:
        dist.destroy_process_group()


def _sync_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vad_amd.cad import CausalAnomalyDetector
        from vad_amd.train import CadTrainer
        torch.manual_seed(0)
        m = CausalAnomalyDetector()
        x, y = make_batches(world, **SHAPE)[rank]
        tr = CadTrainer(m, lr=3e-4, seed=0, engine=OracleEngine(m), sync_bn=True)
        losses = tr.step(x, y)
        torch.save({"losses": losses, "grads": tr.eng.grads.clone(), "bufs": tr.eng.bufs.clone()},
                   f"{out_path}.{rank}")
    finally:
        dist.destroy_process_group()


def test_dp_syncbn_protocol_cpu_gloo(tmp_path):
    """CadTrainer(sync_bn=True) over 2 gloo ranks (oracle engine with its differentiable SyncBatchNorm) equals the
    single-process step on the 2x-larger batch: mean of the ranks' losses, grads summed over ranks = 2 x the global
    batch's grads, running stats identical on both ranks and equal to the global batch's."""
    out = str(tmp_path / "sync")
    mp.spawn(_sync_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]
    from vad_amd.cad import CausalAnomalyDetector
    from oracle import cad_oracle as co
    torch.manual_seed(0)
    m = CausalAnomalyDetector()
    eng = OracleEngine(m)
    bt = make_batches(2, **SHAPE)
    x = torch.cat([b[0] for b in bt])
    y = torch.cat([b[1] for b in bt])
    lv = eng.forward(x, True, 0, 0, 0, y)["losses"]
    eng.backward(True)
    np.testing.assert_allclose(((got[0]["losses"] + got[1]["losses"]) / 2).numpy(), lv.numpy(), rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(got[0]["grads"][:eng.param_floats].numpy(), 2 * eng.grads[:eng.param_floats].numpy(),
                               rtol=1e-4, atol=2e-6)
    for r in range(2):
        np.testing.assert_allclose(got[r]["bufs"].numpy(), eng.bufs.numpy(), rtol=1e-5, atol=1e-6)


def _run(use_gpu, tmp_path, frozen=False, skip_det=False):
    out = str(tmp_path / "rank0.pt")
    mp.spawn(_worker, args=(2, _free_port(), use_gpu, out, frozen, skip_det), nprocs=2, join=True)
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("skip_det", [False, True], ids=["sum-detector", "skip-zero-detector"])
def test_dp_protocol_cpu_gloo(skip_det, tmp_path):
    """skip-zero-detector: CadTrainer(skip_zero_detector=True) leaves the detector's grads out of the head bucket
    when no rank's detector has a grad (the reference's init: every frame takes the fallback box) -- the same params
    and 13.3 MB less on the wire per step."""
    got = _run(False, tmp_path, skip_det=skip_det)
    if skip_det:  # one more float on the wire (the flag); the detector's grads only when some rank has them
        lo, hi = got["det_range"]
        n = got["grads"].numel() + 1 - ((hi - lo) if got["det_flag_sum"] == 0.0 else 0)
        assert got["det_flag_sum"] >= 0.0 and got["allreduce_floats"] == n, (got["allreduce_floats"], n)
    from vad_amd.cad import CausalAnomalyDetector
    torch.manual_seed(0)
    m = CausalAnomalyDetector()
    eng = OracleEngine(m)
    emulate_dp_steps(eng, make_batches(2, **SHAPE), 2, 2)
    np.testing.assert_allclose(got["params"].numpy(), eng.params.numpy(), rtol=0, atol=1e-6)
    np.testing.assert_allclose(got["bufs"].numpy(), eng.bufs.numpy(), rtol=0, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("frozen", [False, True], ids=["stem-trains", "stem-frozen"])
def test_dp_hip_engine_gloo_two_ranks(frozen, tmp_path):
    """Two gloo ranks on cuda:0 with the bucketed, overlapped all-reduce: params, BN buffers and the summed grads of
    the last step equal the single-process emulation (each rank's backward, then ONE sum of the whole grad buffer)
    bit for bit.  stem-frozen is the trainer default (apply_memory_efficient_training): layer 0's weight gradient
    runs on the caller's stream while layers 1-3's may still run on the weight-gradient stream, and the layers 0-3
    bucket must wait for both."""
    import contextlib
    import io
    got = _run(True, tmp_path, frozen)
    from vad_amd.cad import CausalAnomalyDetector
    from vad_amd.train import apply_memory_efficient_training
    torch.manual_seed(0)
    m = CausalAnomalyDetector()
    if frozen:
        with contextlib.redirect_stdout(io.StringIO()):
            apply_memory_efficient_training(m)
    m = m.cuda()
    eng = m.engine()
    batches = [(x.cuda(), y.cuda()) for x, y in make_batches(2, **SHAPE)]
    emulate_dp_steps(eng, batches, 2, 2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got["params"].numpy(), eng.params.cpu().numpy())
    np.testing.assert_array_equal(got["bufs"].numpy(), eng.bufs.cpu().numpy())
    np.testing.assert_array_equal(got["grads"].numpy(), eng.grads.cpu().numpy())


# ---------------------------------------------------------------- the collective path on RCCL (nccl) at world 1
def _world1_worker(rank, backend, port, sync_bn, forced, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        out = _world1_run(sync_bn, forced, force_dist=True)
        torch.save(out, out_path)
    finally:
        dist.destroy_process_group()


def _world1_run(sync_bn, forced, force_dist, early=False, steps=2):
    from tests.golden.cases import FORCED_A, force_detector
    from vad_amd.cad import CausalAnomalyDetector
    from vad_amd.train import CadTrainer
    torch.manual_seed(0)
    m = CausalAnomalyDetector()
    if forced:
        force_detector(m.state_dict(), FORCED_A)
    m = m.cuda()
    tr = CadTrainer(m, lr=3e-4, seed=0, sync_bn=sync_bn, force_dist=force_dist)
    assert tr.dist == force_dist and tr.sync_bn == (sync_bn and force_dist)
    x, y = make_batches(1, **SHAPE)[0]
    x, y = x.cuda(), y.cuda()
    torch.cuda.synchronize()  # (early: the clips are complete before every step)
    floats, losses = [], []
    for _ in range(steps):
        losses.append(tr.step(x, y, inputs_ready=True if early else None).clone())
        floats.append(tr.allreduce_floats)
        tr.allreduce_floats = 0
    torch.cuda.synchronize()
    return {"params": tr.eng.params.cpu(), "bufs": tr.eng.bufs.cpu(), "grads": tr.eng.grads.cpu(),
            "floats": torch.tensor(floats), "det_range": torch.tensor(tr.det_range),
            "losses": torch.stack(losses).cpu()}


def _early_worker(rank, port, early, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        torch.save(_world1_run(False, False, force_dist=True, early=early, steps=3), out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_early_stem_equals_serial_steps(tmp_path):
    """CadTrainer.step(inputs_ready=True): each step's frozen stem runs on the plan's stem stream beside the previous
    step's queued tail (vad_cad_input_ready; pool and bn1's state alternate between two sets).  Three steps equal
    three serial steps bit for bit -- params, BN buffers (bn1's running statistics are updated on the stem stream),
    grads, losses -- both single-process and with the data-parallel protocol forced on over RCCL at world 1 (the
    BN-buffer broadcast right after each forward, which the next early stem waits for)."""
    plain = _world1_run(False, False, force_dist=False, early=False, steps=3)
    early = _world1_run(False, False, force_dist=False, early=True, steps=3)
    for k in ("params", "bufs", "grads", "losses"):
        assert torch.equal(early[k], plain[k]), k
    res = {}
    for e in (False, True):
        out = str(tmp_path / f"early{int(e)}.pt")
        mp.spawn(_early_worker, args=(_free_port(), e, out), nprocs=1, join=True)
        res[e] = torch.load(out, weights_only=True)
    for k in ("params", "bufs", "grads", "losses"):
        assert torch.equal(res[True][k], res[False][k]), k
        assert torch.equal(res[True][k], plain[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("sync_bn,forced", [(False, False), (False, True), (True, False)],
                         ids=["ddp-fallback", "ddp-forced", "syncbn-fallback"])
def test_collective_path_rccl_world1(sync_bn, forced, tmp_path):
    """CadTrainer's data-parallel protocol forced on at world size 1 (force_dist): the stage-2/stage-1 overlapped
    backward with its all-reduce buckets, the BN-buffer broadcasts and, with sync_bn, the SyncBatchNorm callback (dist.all_reduce from inside the
    library's ctypes callback).  On RCCL (backend nccl) the result equals the gloo run bit for bit, and in DDP mode
    also the plain single-process step (a world-1 all-reduce is the identity).  Every bucket is issued every step
    (the detector bucket too: no host read of the has-grad flag)."""
    res = {}
    for backend in ("nccl", "gloo"):
        out = str(tmp_path / f"{backend}.pt")
        mp.spawn(_world1_worker, args=(backend, _free_port(), sync_bn, forced, out), nprocs=1, join=True)
        res[backend] = torch.load(out, weights_only=True)
    for k in ("params", "bufs", "grads", "floats"):
        assert torch.equal(res["nccl"][k], res["gloo"][k]), k
    total = res["nccl"]["grads"].numel()
    assert res["nccl"]["floats"].tolist() == [total, total]  # every bucket every step (no host-side skip)
    if not sync_bn:
        plain = _world1_run(False, forced, force_dist=False)
        for k in ("params", "bufs", "grads"):
            assert torch.equal(res["nccl"][k], plain[k]), k


# ---------------------------------------------------------------- BASELINE config 3 per-rank shape, vs the oracle
CFG3 = dict(B=8, T=16, H=227, W=227)


def _cfg3_worker(rank, world, port, sync_bn, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import io
        import contextlib
        from vad_amd.cad import CausalAnomalyDetector
        from vad_amd.train import CadTrainer, apply_memory_efficient_training
        from tests.golden_util import hip_relu_masks
        torch.manual_seed(0)
        m = CausalAnomalyDetector()
        with contextlib.redirect_stdout(io.StringIO()):
            apply_memory_efficient_training(m)
        m = m.cuda()
        x, y = make_batches(world, **CFG3)[rank]
        tr = CadTrainer(m, lr=3e-4, seed=0, sync_bn=sync_bn)
        o = tr.step(x.cuda(), y.cuda(), want_outputs=True)
        torch.cuda.synchronize()
        masks = hip_relu_masks(tr.eng, CFG3["B"] * CFG3["T"])
        torch.save({"final": o["final"].cpu(), "probs": o["probs"].cpu(), "losses": o["losses"].cpu(),
                    "grads": tr.eng.grads.cpu(), "bufs": tr.eng.bufs.cpu(), "params": tr.eng.params.cpu(),
                    "masks": [mk.clone() for mk in masks]}, f"{out_path}.{rank}")
    finally:
        dist.destroy_process_group()


def _cfg3_run(sync_bn, tmp_path):
    out = str(tmp_path / "cfg3")
    mp.spawn(_cfg3_worker, args=(2, _free_port(), sync_bn, out), nprocs=2, join=True)
    return [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]


@pytest.mark.gpu
@pytest.mark.parametrize("sync_bn", [False, True], ids=["ddp", "syncbn"])
def test_dp_config3_shape_vs_oracle(sync_bn, tmp_path):
    """Two ranks on cuda:0 (gloo), 8 clips x T=16 x 227x227 per rank: BASELINE config 3's per-rank workload.
    ddp: per-rank BatchNorm statistics (DDP default) vs the oracle run on each rank's micro-batch, grads summed.
    syncbn: SyncBatchNorm mode vs the oracle's single-process step on the 16-clip global batch (the reference's
    semantics at batch 64: BN over all B*T frames, cad:116,131,136).  Scores and losses within 1e-4; the summed
    gradients within relative L2 1e-4 of the mask-pinned float64 oracle (ReLU decisions of the ranks' forwards);
    running stats within 1e-4."""
    from tests.golden_util import check_running_stats, pinned_oracle_grads, rel_l2
    from tests.test_oracle_golden import is_pre_bn_bias
    from oracle import cad_oracle as co
    from vad_amd.cad import CausalAnomalyDetector
    got = _cfg3_run(sync_bn, tmp_path)
    batches = make_batches(2, **CFG3)
    torch.manual_seed(0)
    sd = {k: v.clone() for k, v in CausalAnomalyDetector().state_dict().items()}
    B, T = CFG3["B"], CFG3["T"]
    if sync_bn:
        x = torch.cat([b[0] for b in batches])
        y = torch.cat([b[1] for b in batches])
        masks = [torch.cat([got[0]["masks"][l], got[1]["masks"][l]]) for l in range(8)]
        grads, losses, res = pinned_oracle_grads(sd, x, y, co.CadDraws.make(0, 0, 0, 2 * B, T), masks)
        scores = res["out"]["anomaly_scores"].detach()
        np.testing.assert_allclose(torch.cat([g["final"] for g in got]).numpy(), scores.numpy(), rtol=1e-4, atol=1e-5)
        mean_losses = (got[0]["losses"].double() + got[1]["losses"].double()) / 2
        for i, k in enumerate(("classification", "anomaly", "causal", "kl", "total")):
            assert float(mean_losses[i]) == pytest.approx(float(losses[k]), rel=1e-4, abs=1e-6), k
        ref_g = grads
        scale = 2.0  # sum over ranks of per-rank means = 2 x the gradient of the global mean
        for r in range(2):  # every rank holds the group's running stats
            check_running_stats(got[r]["bufs"], res["bufs"])
    else:
        ref_g, scale = {}, 1.0
        for r in range(2):
            x, y = batches[r]
            grads, losses, res = pinned_oracle_grads(sd, x, y, co.CadDraws.make(0, 0, r * B, B, T), got[r]["masks"])
            np.testing.assert_allclose(got[r]["final"].numpy(), res["out"]["anomaly_scores"].detach().numpy(),
                                       rtol=1e-4, atol=1e-5)
            for i, k in enumerate(("classification", "anomaly", "causal", "kl", "total")):
                assert float(got[r]["losses"][i]) == pytest.approx(float(losses[k]), rel=1e-4, abs=1e-6), k
            for n, gv in grads.items():
                if gv is not None:
                    ref_g[n] = ref_g.get(n, 0) + gv
            if r == 0:  # running stats follow rank 0 (DDP broadcast_buffers)
                check_running_stats(got[0]["bufs"], res["bufs"])
    # the summed grads (what the all-reduce left on the ranks; identical on both)
    from vad_amd import _native as nat
    L = nat.lib()
    names = [L.vad_cad_slot_name(i).decode() for i in range(L.vad_cad_num_slots())]
    offs = [L.vad_cad_slot_offset(i) for i in range(len(names))]
    nels = [L.vad_cad_slot_numel(i) for i in range(len(names))]
    assert torch.equal(got[0]["grads"], got[1]["grads"])
    gr = got[0]["grads"].numpy()
    for n, o, k in zip(names, offs, nels):
        ref = ref_g.get(n)
        if ref is None or is_pre_bn_bias(n):
            continue
        e = rel_l2(gr[o:o + k], scale * ref.numpy())
        assert e <= 1e-4, f"{n}: relative L2 {e:.3g}"
