"""bbox clip scorer (config 5): the CPU oracle against the reference's own predict_anomaly_for_clip fixtures, and
(GPU) the HIP plan against both, including mixed-T packing."""
import numpy as np
import pytest
import torch

from oracle import bbox_oracle as bo
from tests.golden.cases import BBOX_CASES
from tests.golden_util import load


def make_bbox_model(case):
    from vad_amd.bbox import CausalAnomalyDetector
    torch.manual_seed(case["seed"])
    return CausalAnomalyDetector().eval()


@pytest.mark.parametrize("case", BBOX_CASES, ids=[c["name"] for c in BBOX_CASES])
def test_bbox_init_and_oracle_match_reference(case):
    g = load(f"bbox_{case['name']}.npz")
    m = make_bbox_model(case)
    for n, t in m.state_dict().items():
        assert np.float64(t.double().sum()) == g[f"init_sum/{n}"], n
        assert np.float64((t.double() ** 2).sum()) == g[f"init_sq/{n}"], n
    p = {k: v.detach().clone() for k, v in m.state_dict().items()}
    x = bo.synth_clips(case["seed"], case["step"], 0, case["B"], case["T"], case["H"], case["W"])
    with torch.no_grad():
        s, adj, f = bo.bbox_forward(p, x)
    np.testing.assert_allclose(s.numpy(), g["out/scores"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(adj.numpy(), g["out/adj"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(f.numpy(), g["out/features"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(s.numpy(), g["batch/scores"], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("case", BBOX_CASES, ids=[c["name"] for c in BBOX_CASES])
def test_bbox_hip_matches_reference(case):
    g = load(f"bbox_{case['name']}.npz")
    from vad_amd.bbox import AnomalyVisualizer
    vis = AnomalyVisualizer(None, device="cuda")
    vis.model = make_bbox_model(case).cuda()
    x = bo.synth_clips(case["seed"], case["step"], 0, case["B"], case["T"], case["H"], case["W"])
    for b in range(case["B"]):
        s, adj, f = vis.predict_anomaly_for_clip(x[b].numpy())
        assert s == pytest.approx(float(g["out/scores"][b]), rel=1e-4, abs=1e-6)
        np.testing.assert_allclose(adj, g["out/adj"][b], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(f, g["out/features"][b], rtol=1e-4, atol=1e-5)
    with torch.no_grad():
        s, adj, f = vis.model(x.cuda())
    np.testing.assert_allclose(s.cpu().numpy(), g["batch/scores"], rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_bbox_mixed_t_packing_matches_oracle():
    """Clips of T in {8,16,32} scored in one call (one packed batch per T) equal per-clip oracle results."""
    from vad_amd.bbox import AnomalyVisualizer
    case = dict(seed=33)
    vis = AnomalyVisualizer(None, device="cuda")
    vis.model = make_bbox_model(case).cuda()
    p = {k: v.detach().cpu().clone() for k, v in make_bbox_model(case).state_dict().items()}
    clips = []
    for i, T in enumerate([8, 32, 16, 8, 16, 32, 8]):
        clips.append(bo.synth_clips(33, 0, i, 1, T, 64, 64)[0].numpy())
    res = vis.predict_clips(clips)
    for c, (s, adj, f) in zip(clips, res):
        with torch.no_grad():
            rs, radj, rf = bo.bbox_forward(p, torch.from_numpy(c)[None])
        assert s == pytest.approx(float(rs), rel=1e-4, abs=1e-6)
        np.testing.assert_allclose(adj, radj[0].numpy(), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(f, rf[0].numpy(), rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_bbox_config5_packed_64_clips_matches_oracle():
    """BASELINE config 5's per-rank workload: 64 clips with T drawn from {8, 16, 32} (seeded, mixed order), scored in
    one call (one packed batch per T bucket) -- every clip's score, graph and features equal the oracle's (run per T
    bucket on CPU, float32) within 1e-4."""
    from vad_amd.bbox import AnomalyVisualizer
    case = dict(seed=55)
    vis = AnomalyVisualizer(None, device="cuda")
    vis.model = make_bbox_model(case).cuda()
    p = {k: v.detach().cpu().clone() for k, v in make_bbox_model(case).state_dict().items()}
    g = np.random.default_rng(55)
    Ts = [int(t) for t in g.choice([8, 16, 32], size=64)]
    assert len(set(Ts)) == 3
    clips = [bo.synth_clips(55, 0, i, 1, T, 64, 64)[0].numpy() for i, T in enumerate(Ts)]
    res = vis.predict_clips(clips)
    assert len(res) == 64
    for T in (8, 16, 32):
        idx = [i for i, t in enumerate(Ts) if t == T]
        with torch.no_grad():
            rs, radj, rf = bo.bbox_forward(p, torch.from_numpy(np.stack([clips[i] for i in idx])))
        for k, i in enumerate(idx):
            s, adj, f = res[i]
            assert s == pytest.approx(float(rs.reshape(-1)[k]), rel=1e-4, abs=1e-6), (i, T)
            np.testing.assert_allclose(adj, radj[k].numpy(), rtol=1e-4, atol=1e-6)
            np.testing.assert_allclose(f, rf[k].numpy(), rtol=1e-4, atol=1e-5)


def _bbox_dp_worker(rank, world, port, out_path):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vad_amd.bbox import AnomalyVisualizer
        vis = AnomalyVisualizer(None, device="cuda")
        vis.model = make_bbox_model(dict(seed=44)).cuda()
        clips = [bo.synth_clips(44, 0, i, 1, T, 64, 64)[0].numpy() for i, T in enumerate([8, 32, 16, 8, 16, 32, 8])]
        res = vis.predict_clips(clips)
        if rank == 0:
            torch.save({"s": torch.tensor([r[0] for r in res]), "f": torch.tensor(np.stack([r[2] for r in res]))},
                       out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_bbox_data_parallel_two_ranks(tmp_path):
    """Config 5 sharding: two gloo ranks (sharing cuda:0) each score their share of every T bucket; the gathered
    results equal single-process scoring (clips are independent; only the split-K reduction order of the 3-D conv
    GEMMs depends on the batch size, so features agree to fp32 rounding)."""
    import socket
    import torch.multiprocessing as mp
    from vad_amd.bbox import AnomalyVisualizer
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "r0.pt")
    mp.spawn(_bbox_dp_worker, args=(2, port, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    vis = AnomalyVisualizer(None, device="cuda")
    vis.model = make_bbox_model(dict(seed=44)).cuda()
    clips = [bo.synth_clips(44, 0, i, 1, T, 64, 64)[0].numpy() for i, T in enumerate([8, 32, 16, 8, 16, 32, 8])]
    ref = vis.predict_clips(clips)
    np.testing.assert_allclose(got["s"].numpy(), np.array([r[0] for r in ref], dtype=np.float32), rtol=1e-6,
                               atol=1e-7)
    np.testing.assert_allclose(got["f"].numpy(), np.stack([r[2] for r in ref]), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("B,T,H,W", [(3, 7, 33, 50), (2, 2, 16, 18), (1, 32, 64, 64), (5, 9, 20, 70)])
def test_bbox_encoder_ragged_shapes(B, T, H, W):
    """The fused conv1 + ReLU + MaxPool3d kernel and the depth-tap split-bf16 Conv3d (implicit GEMM, no im2col) on
    ragged shapes -- odd T (MaxPool3d floor), pooled planes that are not whole 8 x 8 / 8 x 32 tiles -- against the
    oracle: features (1e-4 of their scale), scores and graphs within 1e-4; and equal (1e-5) to the im2col path."""
    from vad_amd import _native as nat
    m = make_bbox_model(dict(seed=40)).cuda()
    p = {k: v.detach().cpu().clone() for k, v in make_bbox_model(dict(seed=40)).state_dict().items()}
    x = bo.synth_clips(41, 0, 0, B, T, H, W)
    with torch.no_grad():
        rs, radj, rf = bo.bbox_forward(p, x)
        outs = []
        for im2col in (0, 1):
            nat.check(nat.lib().vad_set_tuning(b"bbox_im2col", im2col))
            try:
                outs.append([t.cpu() for t in m(x.cuda())])
            finally:
                nat.check(nat.lib().vad_set_tuning(b"bbox_im2col", 0))
    for s, adj, f in outs:
        scale = float(rf.abs().max())
        np.testing.assert_allclose(f.numpy(), rf.numpy(), rtol=1e-4, atol=1e-4 * scale)
        np.testing.assert_allclose(s.reshape(-1).numpy(), rs.reshape(-1).numpy(), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(adj.numpy(), radj.numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(outs[0][2].numpy(), outs[1][2].numpy(), rtol=1e-5, atol=1e-5 * float(rf.abs().max()))
