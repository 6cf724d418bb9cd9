"""a2 (avenue_training_script2.py) on the GPU: the HIP plan (vad_a2_*) against the reference fixtures (incl. the
shipped checkpoint) and the CPU oracle."""
import numpy as np
import pytest
import torch

from oracle import a2_oracle as ao
from tests.golden.cases import A2_CASES
from tests.golden_util import load
from tests.test_a2_oracle import make_a2_model

pytestmark = pytest.mark.gpu


def _vad(case):
    from vad_amd.a2 import ImprovedMiniCausalVAD
    vad = ImprovedMiniCausalVAD(device="cuda")
    vad.model = make_a2_model(case).to("cuda")
    vad.seed, vad.global_step, vad.clip0 = case["seed"], case["step"], 0
    return vad


@pytest.mark.parametrize("case", A2_CASES, ids=[c["name"] for c in A2_CASES])
def test_a2_step_matches_reference(case):
    g = load(f"a2_{case['name']}.npz")
    vad = _vad(case)
    B, T, H, W = case["B"], case["T"], case["H"], case["W"]
    x = ao.synth_clips(case["seed"], case["step"], 0, B, T, H, W)
    avg, comps = vad.train_epoch_improved([(x, ao.synth_labels(0, B))])
    e = vad.model._engine
    p = e.cur
    torch.cuda.synchronize()
    np.testing.assert_allclose(p.scores.cpu().numpy(), g["out/scores"].reshape(-1), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(p.adj.cpu().numpy(), g["out/adj"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(p.feats.cpu().numpy(), g["out/features"], rtol=1e-4, atol=1e-5)
    assert avg == pytest.approx(float(g["loss/total"]), rel=1e-4)
    for k, v in comps.items():
        assert v == pytest.approx(float(g[f"loss/{k}"]), rel=1e-4, abs=1e-6), k
    assert float(e.losses[8]) == pytest.approx(float(g["grad_total_norm"]), rel=1e-3)
    sd = dict(vad.model.named_parameters())
    for name, off, n in e.slots:
        gf = e.grads[off:off + n].cpu().numpy()
        ref = float(g[f"grad_norm/{name}"])
        assert float(np.linalg.norm(gf.astype(np.float64))) == pytest.approx(ref, rel=2e-3, abs=1e-12), name
        np.testing.assert_allclose(gf[g[f"idx/{name}"]], g[f"grad/{name}"], rtol=2e-3,
                                   atol=2e-4 * ref / np.sqrt(n) + 1e-12, err_msg=name)
        np.testing.assert_allclose(sd[name].detach().cpu().numpy().reshape(-1)[g[f"idx/{name}"]], g[f"post/{name}"],
                                   rtol=1e-6, atol=2.5e-5, err_msg=name)
    x2 = ao.synth_clips(case["seed"], case["step"] + 1, B, B, T, H, W)
    preds, graphs, metrics = vad.evaluate_improved([(x2, ao.synth_labels(B, B))])
    np.testing.assert_allclose(preds, g["eval/preds"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(graphs, g["eval/graphs"], rtol=1e-4, atol=1e-6)
    for k, v in metrics.items():
        if k == "unique_graphs":
            assert v == int(g[f"eval/{k}"])
        elif k in ("avg_edges", "avg_sparsity"):
            assert v == pytest.approx(float(g[f"eval/{k}"]), abs=1e-9), k  # counts of adj > 0.1
        else:
            assert v == pytest.approx(float(g[f"eval/{k}"]), rel=1e-4, abs=1e-6), k


def test_a2_autograd_loss_path_matches_oracle():
    """model(x) -> compute_improved_loss -> loss.backward() through torch autograd (the reference's own call
    sequence, a2:224-235) against the oracle's autograd."""
    case = dict(B=5, T=6, H=40, W=48, seed=23, step=0, ckpt=True)
    vad = _vad(case)
    x = ao.synth_clips(23, 0, 0, 5, 6, 40, 48)
    vad.model.train()
    s, adj, f = vad.model(x.cuda(), seed=23, step=0, clip0=0)
    loss, comps = vad.compute_improved_loss(s, adj, torch.zeros(5, device="cuda"), f)
    loss.backward()
    m = make_a2_model(case)
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    draws = ao.A2Draws.make(23, 0, 0, 5)
    rs, radj, rf = ao.a2_forward(leaves, x, draws, True)
    rtot, rcomps, _ = ao.a2_loss(rs, radj, draws.u_pseudo)
    rtot.backward()
    assert float(loss) == pytest.approx(float(rtot), rel=1e-4)
    for k in rcomps:
        assert comps[k] == pytest.approx(rcomps[k], rel=1e-4, abs=1e-6), k
    for n, p in vad.model.named_parameters():
        gr, gref = p.grad.cpu().numpy(), leaves[n].grad.numpy()
        scale = float(np.abs(gref).max()) + 1e-12
        np.testing.assert_allclose(gr, gref, rtol=2e-3, atol=2e-4 * scale, err_msg=n)


def test_a2_direct_and_im2col_paths_agree():
    """conv3d_1 direct on LDS halo tiles + conv3d_2 / _3 as implicit GEMMs (knob a2_direct = 1, the default) against
    the im2col + GEMM path (a2_direct = 0, latched at plan creation): the train step's loss and every gradient tensor
    agree to float rounding."""
    from vad_amd import _native as nat
    case = dict(B=6, T=8, H=48, W=40, seed=26, step=1, ckpt=False)
    x = ao.synth_clips(26, 1, 0, 6, 8, 48, 40)
    res = []
    for d in (1, 0):
        nat.check(nat.lib().vad_set_tuning(b"a2_direct", d))
        try:
            vad = _vad(case)
            avg, _ = vad.train_epoch_improved([(x, ao.synth_labels(0, 6))])
            e = vad.model._engine
            res.append((avg, {n: e.grads[off:off + k].cpu().double() for n, off, k in e.slots}))
        finally:
            nat.check(nat.lib().vad_set_tuning(b"a2_direct", 1))
    assert res[0][0] == pytest.approx(res[1][0], rel=1e-6)
    for n, g0 in res[0][1].items():
        g1 = res[1][1][n]
        assert float((g0 - g1).norm()) <= 1e-5 * float(g1.norm()) + 1e-12, n


def test_a2_head_per_clip_launch_agrees():
    """The head forward / backward as one block per clip (knob a2_head_clip = 1, the default) against one launch per
    Linear layer (0): the same per-output arithmetic in the same order for every head layer; only fc (Linear(4096,
    16), inside the per-clip kernel on the default path, a split-K GEMM on the other) sums its 4096 products in
    another order -- so the step agrees to fp32 rounding (rel 1e-5), not bit for bit.  (compute_improved_loss stays
    four launches: as phases of one block its B x B clip pairs ran as serial rounds of global loads, a2 0.53 -> 0.70
    ms/step, profiles/r06_bench_a2_loss_block.json.)"""
    from vad_amd import _native as nat
    case = dict(B=6, T=8, H=48, W=40, seed=27, step=2, ckpt=True)
    x = ao.synth_clips(27, 2, 0, 6, 8, 48, 40)
    res = []
    for v in (1, 0):
        nat.check(nat.lib().vad_set_tuning(b"a2_head_clip", v))
        try:
            vad = _vad(case)
            avg, comps = vad.train_epoch_improved([(x, ao.synth_labels(0, 6))])
            e = vad.model._engine
            res.append((avg, comps, e.cur.scores.cpu().clone(), e.grads.cpu().clone()))
        finally:
            nat.check(nat.lib().vad_set_tuning(b"a2_head_clip", 1))
    assert res[0][0] == pytest.approx(res[1][0], rel=1e-5)
    for k, v in res[0][1].items():
        assert v == pytest.approx(res[1][1][k], rel=1e-5, abs=1e-7), k
    torch.testing.assert_close(res[0][2], res[1][2], rtol=1e-5, atol=1e-7)
    g0, g1 = res[0][3].double(), res[1][3].double()
    assert float((g0 - g1).norm() / g1.norm()) < 1e-5


def test_a2_nan_loss_skips_the_step():
    """train_step queues the backward and the optimizer step before reading the loss; on a NaN loss the device gate
    (status word losses[9]) leaves parameters, AdamW moments and step counts untouched like the reference's skip
    (a2:230-232), and the next step is bit-identical to the same step of a run that never saw the NaN batch."""
    case = A2_CASES[0]
    B, T, H, W = case["B"], case["T"], case["H"], case["W"]
    x = ao.synth_clips(case["seed"], case["step"], 0, B, T, H, W)
    y = ao.synth_labels(0, B)
    xn = x.clone()
    xn[0, 0, 0, 0, 0] = float("nan")
    a, b = _vad(case), _vad(case)
    p0 = torch.cat([p.detach().reshape(-1).clone() for p in a.model.parameters()])
    loss, _, stepped = a.train_step(xn, y)
    torch.cuda.synchronize()
    assert not stepped and np.isnan(loss)
    e = a.model._engine
    assert torch.equal(torch.cat([p.detach().reshape(-1) for p in a.model.parameters()]), p0)
    assert float(e.exp_avg.abs().max()) == 0.0 and int(e.steps.max()) == 0
    # the same clean step on both (b never saw the NaN batch; a's skipped step kept its keys' step counter)
    b.global_step, b.clip0 = a.global_step, a.clip0
    la, _, sa = a.train_step(x, y)
    lb, _, sb = b.train_step(x, y)
    torch.cuda.synchronize()
    assert sa and sb and la == lb
    assert torch.equal(torch.cat([p.detach().reshape(-1) for p in a.model.parameters()]),
                       torch.cat([p.detach().reshape(-1) for p in b.model.parameters()]))
