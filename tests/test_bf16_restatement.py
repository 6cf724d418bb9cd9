"""The bf16-mode restatement of the backbone (oracle.cad_oracle.backbone_forward_bf16, the yardstick of the config-4
bf16 parity test) differs from the exact oracle only by its rounding points: with bf16 rounding replaced by the
identity it reproduces the exact float64 train step (scores, loss, every gradient), the frozen stem's raw signed
pooling + bn1 included; with rounding it stays within bf16 distance of it."""
import numpy as np
import torch

from oracle import cad_oracle as co
from tests.golden_util import make_cad_model, rel_l2

CASE = dict(name="bf16r", B=2, T=3, H=48, W=40, seed=4, step=1, forced=None)


def _step(monkeypatch, bf16, identity=False):
    if identity:
        monkeypatch.setattr(co, "bf16r", lambda t: t)
    m = make_cad_model(CASE)
    sd = m.state_dict()
    # one negative bn1 gamma: that channel pools the minimum of the raw conv output
    sd["backbone.bn1.weight"][3] = -0.7
    params = {k: v.detach().double().clone() for k, v in sd.items() if "running" not in k and "num_batches" not in k}
    for k in list(params):
        if k.startswith(co.FROZEN_PREFIXES):
            params[k].requires_grad_(False)
    bufs = {k: v.detach().double().clone() for k, v in sd.items() if "running" in k}
    B, T, H, W = CASE["B"], CASE["T"], CASE["H"], CASE["W"]
    x = co.synth_clips(4, 1, 0, B, T, H, W).double()
    y = co.synth_labels(0, B)
    res = co.cad_train_step(params, bufs, {}, x, y, co.CadDraws.make(4, 1, 0, B, T), bf16=bf16)
    return res, bufs


def test_restatement_without_rounding_is_the_exact_step(monkeypatch):
    exact, bufs_e = _step(monkeypatch, False)
    ident, bufs_i = _step(monkeypatch, True, identity=True)
    np.testing.assert_allclose(ident["out"]["anomaly_scores"].detach().numpy(),
                               exact["out"]["anomaly_scores"].detach().numpy(), rtol=1e-12, atol=1e-13)
    assert abs(float(ident["losses"]["total"]) - float(exact["losses"]["total"])) < 1e-12
    for n, g in exact["grads"].items():
        if g is None:
            assert ident["grads"][n] is None, n
            continue
        if n.startswith("backbone.layer") and n.endswith(".bias") and n.split(".")[2] in ("0", "3"):
            continue  # pre-BN conv biases: true gradient 0, both are rounding noise
        assert rel_l2(ident["grads"][n].detach().numpy(), g.detach().numpy()) < 1e-9, n
    for k in bufs_e:
        np.testing.assert_allclose(bufs_i[k].numpy(), bufs_e[k].numpy(), rtol=1e-12, atol=1e-14, err_msg=k)


def test_restatement_with_rounding_stays_near_the_exact_step(monkeypatch):
    exact, _ = _step(monkeypatch, False)
    emu, _ = _step(monkeypatch, True)
    d = float((emu["out"]["anomaly_scores"] - exact["out"]["anomaly_scores"]).detach().abs().max())
    assert 0 < d < 1e-2
    assert abs(float(emu["losses"]["total"]) / float(exact["losses"]["total"]) - 1) < 1e-2


def test_head_masks_of_its_own_decisions_change_nothing():
    """direct_forward(masks=...) pinned to the oracle's own direct-classifier ReLU decisions is the unpinned step."""
    sd = make_cad_model(CASE).state_dict()
    B, T, H, W = CASE["B"], CASE["T"], CASE["H"], CASE["W"]
    x = co.synth_clips(4, 1, 0, B, T, H, W).double()
    y = co.synth_labels(0, B)

    def run(**kw):
        params = {k: v.detach().double().clone() for k, v in sd.items()
                  if "running" not in k and "num_batches" not in k}
        for k in list(params):
            if k.startswith(co.FROZEN_PREFIXES):
                params[k].requires_grad_(False)
        bufs = {k: v.detach().double().clone() for k, v in sd.items() if "running" in k}
        rec = {}
        res = co.cad_train_step(params, bufs, {}, x, y, co.CadDraws.make(4, 1, 0, B, T), record=rec, **kw)
        return res, rec

    free, rec = run()
    pinned, _ = run(head_masks=[rec[f"dir_z{i}"] > 0 for i in range(4)])
    for n, g in free["grads"].items():
        if g is None:
            assert pinned["grads"][n] is None, n
            continue
        np.testing.assert_allclose(pinned["grads"][n].detach().numpy(), g.detach().numpy(), rtol=1e-12, atol=1e-15,
                                   err_msg=n)
