"""HIP train step of CausalAnomalyDetector against the reference's golden vectors and the CPU oracle.

Tolerances: scores/losses 1e-4 (north star).  Gradients: the ReLU after every train-mode BatchNorm makes the
gradient discontinuous at BN outputs == 0; an element whose BN output is within one rounding of 0 can take the
other branch in any re-implementation (observed: one element in 131k at 128x128, a handful at 227x227, one in
230k at 96x80 with the split-bf16 conv kernels -- tools/dbg_split.py shows every other gradient agreeing with the
f32 kernels to 1e-9), which moves one output channel of the conv weight grad below it by a few % of its RMS.
Small cases are checked element-wise at fp32-noise level with at most 5% of the sampled elements (one output
channel's worth) allowed to deviate, plus the L2 check; large cases by relative L2 error.
Post-step parameters: AdamW's first step is ~lr*sign(g), so an element whose tiny gradient changes sign moves
by up to 2*lr; they are checked against a fraction of lr with the same outlier allowance."""
import numpy as np
import pytest
import torch

from oracle import cad_oracle as co
from tests.golden_util import cad_cases, load, make_cad_model
from tests.test_oracle_golden import is_pre_bn_bias

pytestmark = pytest.mark.gpu
CASES = cad_cases()


def _hip_step(case, step_opt=True):
    from vad_amd.train import apply_memory_efficient_training
    import io, contextlib
    m = make_cad_model(case)
    with contextlib.redirect_stdout(io.StringIO()):
        apply_memory_efficient_training(m)
    m = m.cuda()
    eng = m.engine()
    B, T, H, W = case["B"], case["T"], case["H"], case["W"]
    x = co.synth_clips(case["seed"], case["step"], 0, B, T, H, W).cuda()
    y = co.synth_labels(0, B).cuda()
    o = eng.forward(x, True, case["seed"], case["step"], 0, y)
    eng.backward(True)
    torch.cuda.synchronize()
    grads = eng.grads.clone()
    tn = torch.zeros(1, device="cuda")
    if step_opt:
        eng.optimizer_step(3e-4, total_norm=tn)
    torch.cuda.synchronize()
    return m, eng, o, grads, tn


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_hip_step_matches_reference(case):
    g = load(f"cad_{case['name']}.npz")
    m, eng, o, grads, tn = _hip_step(case)
    tol = dict(rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(o["final"].cpu().numpy(), g["out/anomaly_scores"], **tol)
    np.testing.assert_allclose(o["probs"].cpu().numpy(), g["out/direct_predictions"], **tol)
    np.testing.assert_allclose(o["causal"].cpu().numpy(), g["out/causal_anomaly_scores"], **tol)
    np.testing.assert_allclose(o["kl"].cpu().numpy(), g["out/kl"], **tol)
    np.testing.assert_array_equal(o["nmax"].cpu().numpy(), g["out/nmax"])
    np.testing.assert_array_equal(o["counts"].cpu().numpy(), g["out/det_count"])
    np.testing.assert_allclose(o["z"].cpu().numpy(), g["out/z"], **tol)
    np.testing.assert_allclose(o["adj"].cpu().numpy(), g["out/adj"], **tol)
    np.testing.assert_allclose(o["boxes"].cpu().numpy(), g["out/det_boxes"], rtol=1e-4, atol=1e-3)
    losses = o["losses"].cpu().numpy()
    for i, k in enumerate(("classification", "anomaly", "causal", "kl", "total")):
        assert losses[i] == pytest.approx(float(g[f"loss/{k}"]), rel=1e-4, abs=1e-6), k
    assert float(tn.item()) == pytest.approx(float(g["grad_total_norm"]), rel=1e-3)
    gr = grads.cpu().numpy()
    flags = gr[eng.param_floats:eng.param_floats + 2]
    for i, n in enumerate(eng.slot_names):
        grp = eng.slot_group[i]
        has = int(g[f"has_grad/{n}"]) if f"has_grad/{n}" in g else 0
        live = grp == 1 or (grp == 2 and flags[0] > 0) or (grp == 3 and flags[1] > 0)
        assert int(live) == has, n
        if not has:
            continue
        off, nel = eng.slot_offset[i], eng.slot_numel[i]
        gf = gr[off:off + nel]
        ref_norm = float(g[f"grad_norm/{n}"])
        if is_pre_bn_bias(n):  # rounding noise only (true grad is 0)
            assert np.abs(gf).max() < 1e-6, n
            continue
        large = case["H"] * case["W"] > 100 * 100
        assert float(np.linalg.norm(gf.astype(np.float64))) == pytest.approx(ref_norm, rel=3e-2 if large else 2e-3,
                                                                           abs=1e-9), n
        if not large:  # large cases: a flipped ReLU element shifts whole output channels; the norm check above
            got, want = gf[g[f"idx/{n}"]], g[f"grad/{n}"]
            bad = ~np.isclose(got, want, rtol=3e-3, atol=1e-7 + 2e-4 * ref_norm / np.sqrt(nel))
            # a flipped BN->ReLU element moves one output channel of the conv below it (1/Co of the samples)
            assert bad.mean() <= 0.05, (n, int(bad.sum()), float(np.abs(got - want).max()))
    sd = m.state_dict()
    for n, t in sd.items():
        if "num_batches" in n:
            assert int(t.item()) == 1, n
            continue
        tf = t.detach().cpu().numpy().reshape(-1)
        atol = 3.01e-4 if is_pre_bn_bias(n) else 1.5e-5
        large = case["H"] * case["W"] > 100 * 100
        check_close(tf[g[f"idx/{n}"]], g[f"post/{n}"], rtol=1e-5, atol=atol, outlier_frac=0.1 if large else 0.0,
                    outlier_atol=6.01e-4, name=n)


def check_close(a, b, rtol, atol, outlier_frac=0.0, outlier_atol=None, name=""):
    """allclose, but up to `outlier_frac` of the elements may deviate (bounded by outlier_atol when given)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    bad = np.abs(a - b) > atol + rtol * np.abs(b)
    if outlier_frac == 0.0:
        np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=name)
        return
    assert bad.mean() <= outlier_frac, f"{name}: {bad.sum()} of {bad.size} elements deviate"
    if outlier_atol is not None:
        assert np.abs(a - b).max() <= outlier_atol, f"{name}: max deviation {np.abs(a - b).max():.3g}"


def test_module_api_forward_backward():
    """model(videos) through torch autograd: output structure and grads of a user-defined loss vs the oracle."""
    case = dict(name="api", B=2, T=4, H=64, W=64, seed=11, step=0, forced=None)
    m = make_cad_model(case).cuda()
    m.eval()
    x = co.synth_clips(11, 0, 0, 2, 4, 64, 64)
    out = m(x.cuda())
    assert set(out) == {"anomaly_scores", "causal_factors", "adjacency_matrices", "kl_losses", "detections",
                        "direct_predictions", "causal_anomaly_scores"}
    assert len(out["detections"]) == 2 and len(out["detections"][0]) == 4
    loss = out["anomaly_scores"].sum() + 0.5 * out["direct_predictions"][:, 0].sum() + sum(out["kl_losses"])
    loss.backward()
    # oracle, eval mode
    mc = make_cad_model(case)
    sd = {k: v.clone() for k, v in mc.state_dict().items()}
    params = {k: v.requires_grad_(True) for k, v in sd.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: v for k, v in sd.items() if "running" in k}
    draws = co.CadDraws.make(0, 0, 0, 2, 4)
    ref = co.cad_forward(params, bufs, x, draws, training=False)
    np.testing.assert_allclose(out["anomaly_scores"].detach().cpu().numpy(), ref["anomaly_scores"].detach().numpy(),
                               rtol=1e-4, atol=1e-5)
    lref = ref["anomaly_scores"].sum() + 0.5 * ref["direct_predictions"][:, 0].sum() + sum(ref["kl_losses"])
    lref.backward()
    for n, p in m.named_parameters():
        pr = params[n]
        if n.startswith(("backbone.conv1", "backbone.bn1")):
            assert p.grad is None, n  # the stem is frozen in this build (cad:596-598)
            continue
        if pr.grad is None or float(pr.grad.abs().max()) == 0.0:
            assert p.grad is None or float(p.grad.abs().max()) < 1e-9, n
            continue
        ref_norm = float(pr.grad.norm())
        np.testing.assert_allclose(p.grad.cpu().numpy(), pr.grad.numpy(), rtol=3e-3,
                                   atol=1e-7 + 2e-4 * ref_norm / np.sqrt(pr.numel()), err_msg=n)


@pytest.mark.parametrize("B,T,H,W", [(8, 16, 227, 227)])
def test_hip_forward_matches_oracle_full_size(B, T, H, W):
    """Config-2 shape (B=8, T=16, 227x227): forward scores and losses vs the CPU oracle."""
    case = dict(name="cfg2", B=B, T=T, H=H, W=W, seed=5, step=2, forced=None)
    m = make_cad_model(case).cuda()
    eng = m.engine()
    x = co.synth_clips(5, 2, 0, B, T, H, W)
    y = co.synth_labels(0, B)
    o = eng.forward(x.cuda(), True, 5, 2, 0, y.cuda())
    mc = make_cad_model(case)
    sd = {k: v.clone() for k, v in mc.state_dict().items()}
    params = {k: v for k, v in sd.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: v for k, v in sd.items() if "running" in k}
    with torch.no_grad():
        ref = co.cad_forward(params, bufs, x, co.CadDraws.make(5, 2, 0, B, T), training=True)
        rl = co.cad_losses(ref, y)
    np.testing.assert_allclose(o["final"].cpu().numpy(), ref["anomaly_scores"].numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(o["probs"].cpu().numpy(), ref["direct_predictions"].numpy(), rtol=1e-4, atol=1e-5)
    assert float(o["losses"][4]) == pytest.approx(float(rl["total"]), rel=1e-4)
    for k in bufs:
        np.testing.assert_allclose(dict(m.named_buffers())[k].cpu().numpy(), bufs[k].numpy(), rtol=1e-4, atol=1e-4,
                                   err_msg=k)


def test_hip_backward_matches_oracle_full_size():
    """Config-2 shape (B=8, T=16, 227x227): every gradient tensor vs the CPU oracle (relative L2)."""
    B, T, H, W = 8, 16, 227, 227
    case = dict(name="cfg2", B=B, T=T, H=H, W=W, seed=6, step=0, forced=None)
    m = make_cad_model(case).cuda()
    eng = m.engine()
    x = co.synth_clips(6, 0, 0, B, T, H, W)
    y = co.synth_labels(0, B)
    eng.forward(x.cuda(), True, 6, 0, 0, y.cuda())
    eng.backward(True)
    gr = eng.grads.cpu().numpy()
    mc = make_cad_model(case)
    sd = {k: v.clone() for k, v in mc.state_dict().items()}
    params = {k: v for k, v in sd.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: v for k, v in sd.items() if "running" in k}
    res = co.cad_train_step(params, bufs, {}, x, y, co.CadDraws.make(6, 0, 0, B, T))
    for i, n in enumerate(eng.slot_names):
        ref = res["grads"].get(n)
        if ref is None or is_pre_bn_bias(n):
            continue
        r = ref.numpy().reshape(-1).astype(np.float64)
        mine = gr[eng.slot_offset[i]:eng.slot_offset[i] + eng.slot_numel[i]].astype(np.float64)
        rel = np.linalg.norm(mine - r) / max(np.linalg.norm(r), 1e-30)
        assert rel < 3e-2, f"{n}: relative L2 error {rel:.3g}"


@pytest.mark.parametrize("B,T,H,W", [(2, 32, 256, 256)])
def test_config4_shape_fp32_and_bf16(B, T, H, W):
    """BASELINE config 4 shape (T=32, 256x256; 2 clips per rank here to bound the oracle's CPU time).
    fp32 mode: scores / loss within the north-star 1e-4 of the CPU oracle.  bf16 mode (conv_bf16: the 3x3 convs
    on bf16 operands, fp32 accumulation, everything else fp32): the outputs move by bf16 rounding of the conv
    operands only -- scores and probabilities (bounded in [0, 1]) within 2e-2 absolute, the total loss within 2e-2
    relative, the global gradient norm within 5 % (tolerance stated for bf16 compute: unit roundoff 2^-8)."""
    case = dict(name="cfg4", B=B, T=T, H=H, W=W, seed=9, step=1, forced=None)
    x = co.synth_clips(9, 1, 0, B, T, H, W)
    y = co.synth_labels(0, B)
    mc = make_cad_model(case)
    sd = {k: v.clone() for k, v in mc.state_dict().items()}
    params = {k: v for k, v in sd.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: v for k, v in sd.items() if "running" in k}
    res = co.cad_train_step(params, bufs, {}, x, y, co.CadDraws.make(9, 1, 0, B, T))
    ref_norm = float(res["total_norm"])
    for dt in (torch.float32, torch.bfloat16):
        m = make_cad_model(case).cuda().set_compute_dtype(dt)
        eng = m.engine()
        o = eng.forward(x.cuda(), True, 9, 1, 0, y.cuda())
        eng.backward(True)
        torch.cuda.synchronize()
        g = eng.grads[:eng.param_floats].double()
        fp32 = dt == torch.float32
        atol = 1e-5 if fp32 else 2e-2
        np.testing.assert_allclose(o["final"].cpu().numpy(), res["out"]["anomaly_scores"].detach().numpy(),
                                   rtol=1e-4 if fp32 else 0, atol=atol)
        np.testing.assert_allclose(o["probs"].cpu().numpy(), res["out"]["direct_predictions"].detach().numpy(),
                                   rtol=1e-4 if fp32 else 0, atol=atol)
        assert float(o["losses"][4]) == pytest.approx(float(res["losses"]["total"]), rel=1e-4 if fp32 else 2e-2)
        # (frozen-stem / no-grad slots are zero in both)
        assert float(g.norm()) == pytest.approx(ref_norm, rel=5e-3 if fp32 else 5e-2)


def test_staged_backward_equals_whole_backward():
    """vad_cad_backward_stage 0 then 1 (the DP overlap path) writes the same grads, bit for bit, as one backward;
    after stage 0 every non-backbone grad is already final."""
    case = CASES[1]
    m, eng, o, grads, tn = _hip_step(case, step_opt=False)
    B, T, H, W = case["B"], case["T"], case["H"], case["W"]
    x = co.synth_clips(case["seed"], case["step"], 0, B, T, H, W).cuda()
    y = co.synth_labels(0, B).cuda()
    eng.forward(x, True, case["seed"], case["step"], 0, y)
    eng.backward(True, stage=0)
    torch.cuda.synchronize()
    nb = eng.backbone_floats
    assert 0 < nb < eng.param_floats
    assert torch.equal(eng.grads[nb:eng.param_floats + 2], grads[nb:eng.param_floats + 2])
    eng.backward(True, stage=1)
    torch.cuda.synchronize()
    assert torch.equal(eng.grads[:eng.param_floats + 2], grads[:eng.param_floats + 2])
