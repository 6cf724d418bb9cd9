"""minicausal (config 1) on the GPU: the HIP plan (vad_mc_*) against the reference fixtures and the CPU oracle."""
import numpy as np
import pytest
import torch

from oracle import mc_oracle as mo
from tests.golden.cases import MC_CASES
from tests.golden_util import load
from tests.test_mc_oracle import make_mc_model, split_state

pytestmark = pytest.mark.gpu
PRE_BN_BIASES = ("features.0.bias", "features.4.bias", "features.8.bias")


def _trainer(case, model):
    from vad_amd.mc import StableTrainer
    B, T, H, W = case["B"], case["T"], case["H"], case["W"]
    x = mo.synth_clips(case["seed"], case["step"], 0, B, T, H, W)
    y = mo.synth_labels(0, B)
    tr = StableTrainer(model, [(x, y)], [], "cuda", lr=1e-3)
    tr.seed, tr.global_step, tr.clip0 = case["seed"], case["step"], 0
    return tr


@pytest.mark.parametrize("direct", [1, 0], ids=["direct", "im2col"])
@pytest.mark.parametrize("case", MC_CASES, ids=[c["name"] for c in MC_CASES])
def test_mc_step_matches_reference(case, direct):
    """direct: the convs on conv3d_direct.hip (the default); im2col: knob conv3d_direct=0 (im2col + GEMM)"""
    from vad_amd import _native as nat
    nat.check(nat.lib().vad_set_tuning(b"conv3d_direct", direct))
    try:
        _mc_step_case(case)
    finally:
        nat.check(nat.lib().vad_set_tuning(b"conv3d_direct", 1))


def _mc_step_case(case):
    g = load(f"mc_{case['name']}.npz")
    model = make_mc_model(case)
    init = {n: p.detach().clone().numpy().reshape(-1) for n, p in model.named_parameters()}
    tr = _trainer(case, model)
    avg_loss, acc = tr.train_epoch()
    e = model._engine
    torch.cuda.synchronize()
    np.testing.assert_allclose(e.scores.cpu().numpy(), g["out/scores"], rtol=1e-4, atol=1e-6)
    assert avg_loss == pytest.approx(float(g["train/avg_loss"]), rel=1e-4)
    assert acc == pytest.approx(float(g["train/acc"]), abs=1e-12)
    losses = e.losses.cpu().numpy()
    assert losses[0] == pytest.approx(float(g["loss/bce"]), rel=1e-4)
    assert losses[1] == pytest.approx(float(g["grad_norm"]), rel=2e-3)
    assert int(losses[2]) == int(g["clipped"])
    assert int(losses[3]) == 2
    sd = model.state_dict()
    for name, off, n in e.slots:
        gf = e.grads[off:off + n].cpu().numpy()
        ref = float(g[f"grad_norm/{name}"])
        if name in PRE_BN_BIASES:
            # the conv bias feeding a train-mode BatchNorm has an exactly-zero true gradient (BN removes the
            # mean); both sides hold rounding noise, required only to stay at noise level
            wn = float(g[f"grad_norm/{name[:-4]}weight"])
            assert float(np.abs(gf).max()) <= 1e-5 * wn + 1e-9, name
            continue
        rel = 1e-2 if name.startswith("features.") else 2e-3
        assert float(np.linalg.norm(gf.astype(np.float64))) == pytest.approx(ref, rel=rel, abs=1e-12), name
        # conv weight grads are sums over up to 5e5 voxels with heavy cancellation (BN-backward dY): the GPU's and
        # the reference CPU's summation orders agree to ~1e-3 of the vector norm, not per tiny element
        # (the 0.01-std classifier init makes the feature-stack grads ~1e-7 against O(1) summed terms: 2e-2 there)
        sampled, want = gf[g[f"idx/{name}"]].astype(np.float64), g[f"grad/{name}"].astype(np.float64)
        tol = 2e-2 if name.startswith("features.") else 5e-3
        assert np.linalg.norm(sampled - want) <= tol * np.linalg.norm(want) + 1e-12, name
        # Adam's first update is lr * g' / (|g'| + eps) with g' = clip_coef * g + wd * p (coupled L2): for |g'| well
        # above eps (1e-8) it is +-lr whatever the rounding; for |g'| within ~100 eps (incl. g and wd * p cancelling)
        # a rounding-level grad difference moves it by up to lr (1e-3)
        got = sd[name].detach().cpu().numpy().reshape(-1)[g[f"idx/{name}"]]
        coef = min(1.0, 1.0 / (float(g["grad_norm"]) + 1e-6)) if int(g["clipped"]) else 1.0
        g_eff = coef * g[f"grad/{name}"] + 1e-5 * init[name][g[f"idx/{name}"]]
        near_eps = np.abs(g_eff) < 1e-6
        np.testing.assert_allclose(got[~near_eps], g[f"post/{name}"][~near_eps], rtol=1e-6, atol=5e-5, err_msg=name)
        np.testing.assert_allclose(got[near_eps], g[f"post/{name}"][near_eps], rtol=0, atol=1.01e-3, err_msg=name)
    for name, t in sd.items():
        if "running" in name:
            np.testing.assert_allclose(t.cpu().numpy().reshape(-1), g[f"post/{name}"], rtol=1e-4, atol=1e-6,
                                       err_msg=name)
        if "num_batches" in name:
            assert int(t) == int(g[f"post/{name}"][0] if np.ndim(g[f"post/{name}"]) else g[f"post/{name}"])
    # evaluate() on the second batch
    B, T, H, W = case["B"], case["T"], case["H"], case["W"]
    x2 = mo.synth_clips(case["seed"], case["step"] + 1, B, B, T, H, W)
    y2 = mo.synth_labels(B, B)
    tr.test_loader = [(x2, y2)]
    el, eauc, eacc = tr.evaluate()
    with torch.no_grad():
        s2 = model(x2.cuda()).cpu().numpy().reshape(-1)
    np.testing.assert_allclose(s2, g["eval/scores"], rtol=1e-4, atol=1e-6)
    assert el == pytest.approx(float(g["eval/loss"]), rel=1e-4)
    assert eauc == pytest.approx(float(g["eval/auc"]), abs=1e-9)
    assert eacc == pytest.approx(float(g["eval/acc"]), abs=1e-12)


def test_mc_module_autograd_matches_oracle():
    """model(x) under torch autograd (train mode): the HIP backward of an arbitrary upstream grad."""
    case = dict(B=3, T=8, H=32, W=40, seed=21, step=5, scale=1.0)
    model = make_mc_model(case).cuda().train()
    params, bufs = split_state(make_mc_model(case))
    x = mo.synth_clips(21, 5, 7, 3, 8, 32, 40)
    out = model(x.cuda(), seed=21, step=5, clip0=7)
    w = torch.tensor([0.3, -1.2, 2.0])
    (out.view(-1) * w.cuda()).sum().backward()
    leaves = {n: t.clone().requires_grad_(True) for n, t in params.items()}
    ref = mo.mc_forward(leaves, bufs, x, mo.McDraws.make(21, 5, 7, 3), True)
    (ref.view(-1) * w).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-4, atol=1e-6)
    for n, p in model.named_parameters():
        gr, gref = p.grad.cpu().numpy(), leaves[n].grad.numpy()
        if n in PRE_BN_BIASES:
            continue  # exactly-zero true gradient (train-mode BN), rounding noise on both sides
        scale = float(np.abs(gref).max()) + 1e-12
        np.testing.assert_allclose(gr, gref, rtol=2e-3, atol=2e-4 * scale, err_msg=n)


def test_mc_nonfinite_input_skips_step():
    """NaN outputs -> the batch is skipped (mc:281-283): no update, not counted."""
    case = dict(B=2, T=8, H=16, W=16, seed=3, step=0, scale=1.0)
    model = make_mc_model(case)
    from vad_amd.mc import StableTrainer
    x = mo.synth_clips(3, 0, 0, 2, 8, 16, 16)
    x[0, 0, 3, 4, 5] = float("nan")
    tr = StableTrainer(model, [(x, mo.synth_labels(0, 2))], [], "cuda")
    before = {n: p.detach().clone() for n, p in model.named_parameters()}
    avg, acc = tr.train_epoch()
    assert avg == 0.0 and acc == 0
    assert int(model._engine.losses[3]) == 0
    for n, p in model.named_parameters():
        assert torch.equal(p.detach(), before[n].to(p.device)), n


@pytest.mark.parametrize("case", MC_CASES, ids=[c["name"] for c in MC_CASES])
def test_mc_maxpool_window_backward_is_bit_identical(case):
    """MaxPool3d backward with one thread per window (knob maxpool3d_bwd_win = 1, the default: the first max found once,
    the window's gradients written together) against one thread per input element (0): the same torch first-max rule,
    so the post-step params are bit-identical.  (Extents the windows do not divide are cleared first on the window
    path; the reference's shapes divide evenly.)"""
    from vad_amd import _native as nat
    out = []
    for v in (1, 0):
        nat.check(nat.lib().vad_set_tuning(b"maxpool3d_bwd_win", v))
        try:
            model = make_mc_model(case)
            tr = _trainer(case, model)
            tr.train_epoch()
            out.append(torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()]))
        finally:
            nat.check(nat.lib().vad_set_tuning(b"maxpool3d_bwd_win", 1))
    assert torch.equal(out[0], out[1])
