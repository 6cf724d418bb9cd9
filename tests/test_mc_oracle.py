"""minicausal (config 1): the CPU oracle (oracle/mc_oracle.py) and the drop-in module's initialisation against
golden vectors produced by the reference itself (tests/golden/make_golden.py, MC_CASES)."""
import numpy as np
import pytest
import torch

from oracle import mc_oracle as mo
from tests.golden.cases import MC_CASES
from tests.golden_util import load


def make_mc_model(case):
    from vad_amd.mc import SimpleVideoAnomalyDetector
    torch.manual_seed(case["seed"])
    m = SimpleVideoAnomalyDetector(input_channels=1, temporal_frames=case["T"], spatial_size=case["H"])
    if case["scale"] != 1.0:
        with torch.no_grad():
            m.classifier[6].weight.mul_(case["scale"])
    return m


def split_state(m):
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    params = {k: v for k, v in sd.items() if "running" not in k and "num_batches" not in k}
    bufs = {k: v for k, v in sd.items() if "running" in k}
    return params, bufs


@pytest.mark.parametrize("case", MC_CASES, ids=[c["name"] for c in MC_CASES])
def test_mc_init_matches_reference(case):
    g = load(f"mc_{case['name']}.npz")
    from vad_amd.mc import SimpleVideoAnomalyDetector
    torch.manual_seed(case["seed"])
    m = SimpleVideoAnomalyDetector(input_channels=1, temporal_frames=case["T"], spatial_size=case["H"])
    for n, t in m.state_dict().items():
        assert np.float64(t.double().sum()) == g[f"init_sum/{n}"], n
        assert np.float64((t.double() ** 2).sum()) == g[f"init_sq/{n}"], n


@pytest.mark.parametrize("case", MC_CASES, ids=[c["name"] for c in MC_CASES])
def test_mc_oracle_matches_reference_step(case):
    g = load(f"mc_{case['name']}.npz")
    params, bufs = split_state(make_mc_model(case))
    B, T, H, W = case["B"], case["T"], case["H"], case["W"]
    x = mo.synth_clips(case["seed"], case["step"], 0, B, T, H, W)
    y = mo.synth_labels(0, B)
    res = mo.mc_train_step(params, bufs, {}, x, y, mo.McDraws.make(case["seed"], case["step"], 0, B))
    assert not res["skipped"]
    np.testing.assert_allclose(res["outputs"].numpy(), g["out/scores"], rtol=1e-5, atol=1e-6)
    assert res["loss"] == pytest.approx(float(g["loss/bce"]), rel=1e-5)
    assert res["grad_norm"] == pytest.approx(float(g["grad_norm"]), rel=1e-4)
    assert int(res["clipped"]) == int(g["clipped"])
    for n, gr in res["grads"].items():
        gf = gr.numpy().reshape(-1)
        ref = float(g[f"grad_norm/{n}"])
        assert float(np.linalg.norm(gf.astype(np.float64))) == pytest.approx(ref, rel=1e-3, abs=1e-12), n
        np.testing.assert_allclose(gf[g[f"idx/{n}"]], g[f"grad/{n}"], rtol=1e-3, atol=1e-6 * ref + 1e-12, err_msg=n)
    # Adam divides by sqrt(v) + eps: a grad rounding error of r moves the first update by up to r * lr (lr 1e-3)
    for n, t in params.items():
        np.testing.assert_allclose(t.numpy().reshape(-1)[g[f"idx/{n}"]], g[f"post/{n}"], rtol=1e-6, atol=5e-5,
                                   err_msg=n)
    for n, t in bufs.items():
        np.testing.assert_allclose(t.numpy().reshape(-1), g[f"post/{n}"], rtol=1e-5, atol=1e-6, err_msg=n)
    # evaluate() on the second batch with the post-step weights and running stats
    x2 = mo.synth_clips(case["seed"], case["step"] + 1, B, B, T, H, W)
    y2 = mo.synth_labels(B, B)
    ev = mo.mc_evaluate(params, bufs, [(x2, y2)])
    np.testing.assert_allclose(ev["outputs"], g["eval/scores"], rtol=1e-5, atol=1e-6)
    assert ev["loss"] == pytest.approx(float(g["eval/loss"]), rel=1e-5)
    assert ev["auc"] == pytest.approx(float(g["eval/auc"]), abs=1e-12)
    assert ev["acc"] == pytest.approx(float(g["eval/acc"]), abs=1e-12)
