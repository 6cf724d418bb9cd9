"""cad1 memory autoencoder on the GPU: the HIP plan (vad_ae_*) against the reference fixtures and the CPU oracle."""
import numpy as np
import pytest
import torch

from oracle import ae_oracle as ae
from tests.golden.cases import AE_CASES
from tests.golden_util import ae_case_data, load
from tests.test_ae_oracle import PRE_BN_BIASES, make_ae_model

pytestmark = pytest.mark.gpu


def _first_normal(case):
    train, _, _ = ae_case_data(case)
    for v, y in train:
        if bool((y == 0).any()):
            return v[y == 0]
    raise AssertionError("case without normal clips")


@pytest.mark.parametrize("case", AE_CASES, ids=[c["name"] for c in AE_CASES])
def test_ae_forward_matches_reference(case):
    """The module forward in train mode (the first train_model batch) against the reference's outputs."""
    g = load(f"ae_{case['name']}.npz")
    model = make_ae_model(case).cuda().train()
    with torch.no_grad():
        out = model(_first_normal(case).cuda())
    np.testing.assert_allclose(out["sequence_feature"].cpu().numpy(), g["out/seq"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["frame_features"].cpu().numpy(), g["out/ff"], rtol=1e-4, atol=1e-5)
    r = out["reconstructed"].cpu().numpy().reshape(-1)
    np.testing.assert_allclose(r[g["out/recon_idx"]], g["out/recon_val"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["anomaly_score"].cpu().numpy(), g["out/score"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("case", AE_CASES, ids=[c["name"] for c in AE_CASES])
def test_ae_train_steps_match_reference(case):
    """The fused train_model iterations: losses, first-step grads, post-epoch BN stats / counters / ring / params."""
    g = load(f"ae_{case['name']}.npz")
    from vad_amd.ae import AeTrainer
    model = make_ae_model(case).cuda()
    init = {n: p.detach().cpu().numpy().reshape(-1).copy() for n, p in model.named_parameters()}
    tr = AeTrainer(model, lr=case["lr"])
    e = model.engine()
    train, _, _ = ae_case_data(case)
    losses, norms, first = [], [], None
    for v, y in train:
        if not bool((y == 0).any()):
            continue
        l = tr.step(v[y == 0].cuda()).cpu().numpy()
        assert int(l[3]) == 2
        losses.append(float(l[0]))
        norms.append(float(l[1]))
        if first is None:
            first = e.grads.cpu().numpy().copy()
    np.testing.assert_allclose(losses, g["train/step_loss"], rtol=1e-4)
    np.testing.assert_allclose(norms, g["train/norms"], rtol=2e-3)
    for name, off, n in e.slots:
        gf = first[off:off + n]
        if name in PRE_BN_BIASES:
            wn = float(g[f"grad_norm/{name[:-4]}weight"])
            assert float(np.abs(gf).max()) <= 1e-4 * wn + 1e-9, name  # exactly-zero true grad: noise level
            continue
        assert float(np.linalg.norm(gf.astype(np.float64))) == pytest.approx(float(g[f"grad_norm/{name}"]),
                                                                             rel=2e-3), name
        want = g[f"grad/{name}"].astype(np.float64)
        assert np.linalg.norm(gf[g[f"idx/{name}"]] - want) <= 1e-2 * np.linalg.norm(want) + 1e-12, name
    lr = case["lr"]
    steps = len(losses)
    sd = model.state_dict()
    for name, t in sd.items():
        if "running" in name:
            # running means carry the pre-BN biases (lr-level Adam noise, see below)
            np.testing.assert_allclose(t.cpu().numpy().reshape(-1), g[f"post/{name}"], rtol=1e-4,
                                       atol=1e-6 + 2 * lr * steps, err_msg=name)
        elif "num_batches" in name:
            assert int(t) == int(np.asarray(g[f"post/{name}"]).reshape(-1)[0]), name
    np.testing.assert_allclose(sd["normal_memory"].cpu().numpy()[g["memory/rows"]], g["memory/val"], rtol=1e-4,
                               atol=1e-5)
    assert int(sd["memory_ptr"][0]) == int(g["memory/ptr"])
    for name, p in model.named_parameters():
        idx = g[f"idx/{name}"]
        got = p.detach().cpu().numpy().reshape(-1)[idx]
        if name in PRE_BN_BIASES:
            np.testing.assert_allclose(got, g[f"post/{name}"], rtol=0, atol=2 * lr * steps + 1e-7, err_msg=name)
            continue
        # Adam's update is lr * m / (sqrt(v) + eps): elements whose effective grad sits within ~100 eps of zero
        # move by a rounding-dependent fraction of lr
        g_eff = g[f"grad/{name}"] * min(1.0, 0.1 / (float(g["train/norms"][0]) + 1e-6)) + 1e-6 * init[name][idx]
        near = np.abs(g_eff) < 1e-6
        np.testing.assert_allclose(got[~near], g[f"post/{name}"][~near], rtol=1e-5, atol=1e-6 + 1e-2 * lr,
                                   err_msg=name)
        np.testing.assert_allclose(got[near], g[f"post/{name}"][near], rtol=0, atol=2 * lr * steps + 1e-7,
                                   err_msg=name)


@pytest.mark.parametrize("case", AE_CASES, ids=[c["name"] for c in AE_CASES])
def test_ae_train_model_and_scores_match_reference(case, tmp_path):
    """The drop-in train_model (one epoch + validation) and calculate_anomaly_scores."""
    g = load(f"ae_{case['name']}.npz")
    from vad_amd.ae import calculate_anomaly_scores, train_model
    model = make_ae_model(case)
    train, val, test = ae_case_data(case)
    model, tl, vl = train_model(model, train, val, num_epochs=1, lr=case["lr"], save_path=str(tmp_path / "b.pth"))
    np.testing.assert_allclose(tl, g["train/losses"], rtol=1e-4)
    np.testing.assert_allclose(vl, g["val/losses"], rtol=1e-4)
    s, lab, err, ms = calculate_anomaly_scores(model, test)
    np.testing.assert_allclose(err, g["test/recon"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(ms, g["test/memory"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(s, g["test/scores"], rtol=1e-4, atol=1e-5)
    assert (lab == g["test/labels"]).all()


def test_ae_module_autograd_matches_oracle():
    """model(x) under torch autograd (train mode) with upstream grads on every output, against the oracle."""
    case = dict(B=3, T=4, seed=44, lr=1e-5, labels=[[0, 0, 0]], val_labels=[0], test_labels=[0], mem=(40, 40))
    model = make_ae_model(case).cuda().train()
    params, bufs, mem = ae.split_state(make_ae_model(case).state_dict())
    x = ae.synth_clips(44, 3, 0, 3, 4)
    out = model(x.cuda())
    gen = torch.Generator().manual_seed(1)
    w_rec = torch.randn(out["reconstructed"].shape, generator=gen)
    w_seq = torch.randn(out["sequence_feature"].shape, generator=gen)
    w_ff = torch.randn(out["frame_features"].shape, generator=gen)
    ((out["reconstructed"] * w_rec.cuda()).sum() + (out["sequence_feature"] * w_seq.cuda()).sum()
     + (out["frame_features"] * w_ff.cuda()).sum()).backward()
    leaves = {n: t.clone().requires_grad_(True) for n, t in params.items()}
    ref = ae.ae_forward(leaves, bufs, x, True, mem["memory"], mem["ptr"])
    ((ref["reconstructed"] * w_rec).sum() + (ref["sequence_feature"] * w_seq).sum()
     + (ref["frame_features"] * w_ff).sum()).backward()
    np.testing.assert_allclose(out["anomaly_score"].detach().cpu().numpy(), ref["anomaly_score"].detach().numpy(), rtol=1e-4,
                               atol=1e-5)
    np.testing.assert_allclose(out["sequence_feature"].detach().cpu().numpy(), ref["sequence_feature"].detach().numpy(),
                               rtol=1e-4, atol=1e-5)
    for n, p in model.named_parameters():
        if n in PRE_BN_BIASES:
            continue
        gr, gref = p.grad.cpu().numpy(), leaves[n].grad.numpy()
        scale = float(np.abs(gref).max()) + 1e-12
        np.testing.assert_allclose(gr, gref, rtol=2e-3, atol=2e-4 * scale, err_msg=n)


def test_ae_nonfinite_input_skips_the_batch():
    """A NaN clip is skipped before the forward (cad1:385-387): no update of params, BN state, counters or ring."""
    from vad_amd.ae import AeTrainer
    case = dict(B=2, T=4, seed=45, lr=1e-3, labels=[[0, 0]], val_labels=[0], test_labels=[0], mem=(20, 20))
    model = make_ae_model(case).cuda()
    tr = AeTrainer(model, lr=1e-3)
    x = ae.synth_clips(45, 0, 0, 2, 4)
    x[1, 2, 0, 5, 7] = float("nan")
    before = {k: v.detach().clone() for k, v in model.state_dict().items()}
    l = tr.step(x.cuda()).cpu().numpy()
    assert int(l[3]) == 0
    for k, v in model.state_dict().items():
        assert torch.equal(v, before[k]), k


def test_ae_eval_and_standalone_memory_ops_match_oracle():
    """Eval-mode forward, encode_sequence / decode_sequence, update_memory and compute_anomaly_score."""
    case = dict(B=4, T=5, seed=46, lr=1e-5, labels=[[0] * 4], val_labels=[0], test_labels=[0], mem=(30, 30))
    model = make_ae_model(case).cuda().eval()
    params, bufs, mem = ae.split_state(make_ae_model(case).state_dict())
    x = ae.synth_clips(46, 1, 0, 4, 5)
    with torch.no_grad():
        out = model(x.cuda())
        ref = ae.ae_forward(params, bufs, x, False, mem["memory"], mem["ptr"])
        for k in ("reconstructed", "sequence_feature", "frame_features", "anomaly_score"):
            np.testing.assert_allclose(out[k].cpu().numpy(), ref[k].numpy(), rtol=1e-4, atol=1e-5, err_msg=k)
        seq, ff = model.encode_sequence(x.cuda())
        np.testing.assert_allclose(seq.cpu().numpy(), ref["sequence_feature"].numpy(), rtol=1e-4, atol=1e-5)
        rec = model.decode_sequence(seq, 5)
        np.testing.assert_allclose(rec.cpu().numpy(), ref["reconstructed"].numpy(), rtol=1e-4, atol=1e-5)
        feats = torch.randn(7, 64)
        model.update_memory(feats.cuda())
        ptr = ae.update_memory(mem["memory"], mem["ptr"], feats)
        assert int(model.memory_ptr[0]) == ptr
        np.testing.assert_allclose(model.normal_memory.cpu().numpy(), mem["memory"].numpy(), rtol=0, atol=0)
        s = torch.randn(5, 64)
        np.testing.assert_allclose(model.compute_anomaly_score(s.cuda()).cpu().numpy(),
                                   ae.memory_score(s, mem["memory"], ptr).numpy(), rtol=1e-5, atol=1e-6)


def test_ae_wgrad_stream_is_bit_identical():
    """The backward's weight gradients on the plan's side stream (knob ae_wgrad_stream, the default) against the same
    kernels all on the caller's stream: grads after the first step and params after the second step bit-equal."""
    from vad_amd import _native as nat
    from vad_amd.ae import AeTrainer
    case = dict(B=4, T=8, seed=47, lr=1e-4, labels=[[0] * 4], val_labels=[0], test_labels=[0], mem=(30, 30))
    x = ae.synth_clips(47, 0, 0, 4, 8).cuda()
    res = []
    for side in (0, 1):
        nat.check(nat.lib().vad_set_tuning(b"ae_wgrad_stream", side))
        try:
            model = make_ae_model(case).cuda()
            tr = AeTrainer(model, lr=case["lr"])
            l1 = tr.step(x).cpu().numpy()
            g1 = model.engine().grads.cpu().clone()
            tr.step(x)
            torch.cuda.synchronize()
            res.append((l1, g1, {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}))
        finally:
            nat.check(nat.lib().vad_set_tuning(b"ae_wgrad_stream", 1))
    assert int(res[0][0][3]) == 2 and int(res[1][0][3]) == 2
    assert np.array_equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
    for k in res[0][2]:
        assert torch.equal(res[0][2][k], res[1][2][k]), k


def test_ae_class_launch_paths_agree():
    """The transposed convs' parity classes in one batched launch (default, knob conv4_cls_batch_min = 0) against the
    per-class split-K launches (conv4_cls_batch_min = 512 restores them for the small layers): the train step's
    losses and grads agree to float rounding (different summation order of the split-K slabs)."""
    from vad_amd import _native as nat
    from vad_amd.ae import AeTrainer
    case = dict(B=4, T=8, seed=48, lr=1e-4, labels=[[0] * 4], val_labels=[0], test_labels=[0], mem=(30, 30))
    x = ae.synth_clips(48, 0, 0, 4, 8).cuda()
    res = []
    for v in (0, 512):
        nat.check(nat.lib().vad_set_tuning(b"conv4_cls_batch_min", v))
        try:
            model = make_ae_model(case).cuda()
            tr = AeTrainer(model, lr=case["lr"])
            l1 = tr.step(x).cpu().numpy()
            res.append((l1, model.engine().grads.cpu().clone()))
        finally:
            nat.check(nat.lib().vad_set_tuning(b"conv4_cls_batch_min", 0))
    assert int(res[0][0][3]) == 2 and int(res[1][0][3]) == 2
    np.testing.assert_allclose(res[0][0][:2], res[1][0][:2], rtol=1e-5)
    g0, g1 = res[0][1].double(), res[1][1].double()
    assert float((g0 - g1).norm()) <= 1e-5 * float(g1.norm()) + 1e-12


@pytest.mark.parametrize("direct", [1, 0], ids=["direct", "im2col"])
def test_ae_direct_and_im2col_paths_match_float64(direct):
    """The direct kernels (implicit-GEMM 4x4 convs, VALU 1-channel ends; knob ae_direct = 1, the default) and the
    round-4 im2col / col2im + dense GEMM path (ae_direct = 0, latched at plan creation) each against the float64 step
    pinned to that path's own LeakyReLU decisions: every gradient tensor within relative L2 1e-4.  (The two paths are
    not compared with each other: a unit within rounding of zero may take different branches in the two and move
    encoder.0's gradient by ~1e-3 -- tests/test_grad64.py's docstring.)"""
    from vad_amd import _native as nat
    from tests.test_grad64 import ae_step_vs_float64
    case = dict(name="paths", B=4, T=8, seed=49, lr=1e-4, labels=[[0] * 4], val_labels=[0], test_labels=[0],
                mem=(30, 30))
    nat.check(nat.lib().vad_set_tuning(b"ae_direct", direct))
    try:
        ae_step_vs_float64(case)
    finally:
        nat.check(nat.lib().vad_set_tuning(b"ae_direct", 1))
