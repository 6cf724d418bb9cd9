"""a2 (avenue_training_script2.py): the CPU oracle (oracle/a2_oracle.py) and the drop-in module's initialisation
against golden vectors produced by the reference itself (tests/golden/make_golden.py, A2_CASES), starting from the
reference's shipped checkpoint where the case says so."""
import numpy as np
import pytest
import torch

from oracle import a2_oracle as ao
from tests.golden.cases import A2_CASES
from tests.golden_util import A2_CKPT, load


def make_a2_model(case):
    from vad_amd.a2 import CausalAnomalyDetector
    torch.manual_seed(case["seed"])
    m = CausalAnomalyDetector()
    if case["ckpt"]:
        ck = load(A2_CKPT)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in ck.items()}, strict=True)
    return m


@pytest.mark.parametrize("case", A2_CASES, ids=[c["name"] for c in A2_CASES])
def test_a2_init_matches_reference(case):
    g = load(f"a2_{case['name']}.npz")
    from vad_amd.a2 import CausalAnomalyDetector
    torch.manual_seed(case["seed"])
    m = CausalAnomalyDetector()
    for n, t in m.state_dict().items():
        assert np.float64(t.double().sum()) == g[f"init_sum/{n}"], n
        assert np.float64((t.double() ** 2).sum()) == g[f"init_sq/{n}"], n


def test_a2_checkpoint_fixture_loads_strict():
    m = make_a2_model(dict(seed=0, ckpt=True))
    assert sum(p.numel() for p in m.parameters()) == 188849


@pytest.mark.parametrize("case", A2_CASES, ids=[c["name"] for c in A2_CASES])
def test_a2_oracle_matches_reference_step(case):
    g = load(f"a2_{case['name']}.npz")
    m = make_a2_model(case)
    params = {k: v.detach().clone() for k, v in m.state_dict().items()}
    B, T, H, W = case["B"], case["T"], case["H"], case["W"]
    x = ao.synth_clips(case["seed"], case["step"], 0, B, T, H, W)
    res = ao.a2_train_step(params, {}, x, ao.A2Draws.make(case["seed"], case["step"], 0, B))
    assert not res["skipped"]
    np.testing.assert_allclose(res["scores"].numpy(), g["out/scores"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(res["adj"].numpy(), g["out/adj"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(res["features"].numpy(), g["out/features"], rtol=1e-5, atol=1e-6)
    assert res["loss"] == pytest.approx(float(g["loss/total"]), rel=1e-5)
    for k, v in res["components"].items():
        assert v == pytest.approx(float(g[f"loss/{k}"]), rel=1e-5, abs=1e-7), k
    assert res["total_norm"] == pytest.approx(float(g["grad_total_norm"]), rel=1e-4)
    for n, gr in res["grads"].items():
        gf = gr.numpy().reshape(-1)
        ref = float(g[f"grad_norm/{n}"])
        assert float(np.linalg.norm(gf.astype(np.float64))) == pytest.approx(ref, rel=1e-3, abs=1e-12), n
        np.testing.assert_allclose(gf[g[f"idx/{n}"]], g[f"grad/{n}"], rtol=1e-3, atol=1e-5 * ref + 1e-12, err_msg=n)
        # AdamW moves each weight by <= lr (5e-4) per step
        np.testing.assert_allclose(params[n].numpy().reshape(-1)[g[f"idx/{n}"]], g[f"post/{n}"], rtol=1e-6,
                                   atol=2.5e-5, err_msg=n)
    x2 = ao.synth_clips(case["seed"], case["step"] + 1, B, B, T, H, W)
    preds, graphs, metrics = ao.a2_evaluate(params, [(x2, ao.synth_labels(B, B))])
    np.testing.assert_allclose(preds, g["eval/preds"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(graphs, g["eval/graphs"], rtol=1e-5, atol=1e-6)
    for k, v in metrics.items():
        assert v == pytest.approx(float(g[f"eval/{k}"]), rel=1e-4, abs=1e-6), k
