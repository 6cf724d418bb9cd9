"""cad1 memory autoencoder: the CPU oracle (oracle/ae_oracle.py) and the drop-in module's initialisation against
golden vectors produced by the reference itself (tests/golden/make_golden.py, AE_CASES)."""
import numpy as np
import pytest
import torch

from oracle import ae_oracle as ae
from tests.golden.cases import AE_CASES
from tests.golden_util import ae_case_data, ae_memory_init, load

# conv / conv-transpose biases feeding a train-mode BatchNorm: exactly-zero true gradient (BN removes the mean)
PRE_BN_BIASES = ("encoder.0.bias", "encoder.3.bias", "encoder.6.bias", "encoder.9.bias", "decoder.3.bias",
                 "decoder.6.bias", "decoder.9.bias")


def make_ae_model(case):
    """The drop-in module under the case seed (identical init to the reference) with the case's ring state."""
    from vad_amd.ae import VideoAutoEncoder
    torch.manual_seed(case["seed"])
    m = VideoAutoEncoder(input_channels=1, latent_dim=64)
    mem, ptr = ae_memory_init(case)
    with torch.no_grad():
        m.normal_memory.copy_(mem)
        m.memory_ptr.fill_(ptr)
    return m


@pytest.mark.parametrize("case", AE_CASES, ids=[c["name"] for c in AE_CASES])
def test_ae_init_matches_reference(case):
    g = load(f"ae_{case['name']}.npz")
    from vad_amd.ae import VideoAutoEncoder
    torch.manual_seed(case["seed"])
    m = VideoAutoEncoder(input_channels=1, latent_dim=64)
    for n, t in m.state_dict().items():
        assert np.float64(t.double().sum()) == g[f"init_sum/{n}"], n
        assert np.float64((t.double() ** 2).sum()) == g[f"init_sq/{n}"], n


def run_oracle(case):
    """train_model (one epoch) + its validation + calculate_anomaly_scores replayed on the oracle."""
    params, bufs, mem = ae.split_state(make_ae_model(case).state_dict())
    train, val, test = ae_case_data(case)
    state, steps = {}, []
    for v, y in train:
        steps.append(ae.ae_train_step(params, bufs, mem, state, v, y, lr=case["lr"]))
    vals = [ae.ae_eval_batch(params, bufs, mem, v) for v, _ in val]
    tests = [ae.ae_eval_batch(params, bufs, mem, v) for v, _ in test]
    return params, bufs, mem, steps, vals, tests


@pytest.mark.parametrize("case", AE_CASES, ids=[c["name"] for c in AE_CASES])
def test_ae_oracle_matches_reference(case):
    g = load(f"ae_{case['name']}.npz")
    params, bufs, mem, steps, vals, tests = run_oracle(case)
    ran = [s for s in steps if s["status"] == "stepped"]
    assert len(ran) == len(g["train/step_loss"])
    np.testing.assert_allclose([s["loss"] for s in ran], g["train/step_loss"], rtol=1e-5)
    np.testing.assert_allclose([s["grad_norm"] for s in ran], g["train/norms"], rtol=1e-4)
    o = ran[0]["outputs"]
    np.testing.assert_allclose(o["sequence_feature"].numpy(), g["out/seq"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(o["frame_features"].numpy(), g["out/ff"], rtol=1e-5, atol=1e-6)
    r = o["reconstructed"].numpy().reshape(-1)
    np.testing.assert_allclose(r[g["out/recon_idx"]], g["out/recon_val"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(o["anomaly_score"].numpy(), g["out/score"], rtol=1e-5, atol=1e-6)
    for name, gr in ran[0]["grads"].items():
        gf = gr.numpy().reshape(-1)
        if name in PRE_BN_BIASES:
            wn = float(g[f"grad_norm/{name[:-4]}weight"])
            assert float(np.abs(gf).max()) <= 1e-5 * wn + 1e-9, name  # rounding noise on both sides
            continue
        assert float(np.linalg.norm(gf.astype(np.float64))) == pytest.approx(float(g[f"grad_norm/{name}"]),
                                                                             rel=1e-4), name
        want = g[f"grad/{name}"].astype(np.float64)
        assert np.linalg.norm(gf[g[f"idx/{name}"]] - want) <= 1e-3 * np.linalg.norm(want) + 1e-12, name
    lr = case["lr"]
    for name, t in params.items():
        got = t.numpy().reshape(-1)[g[f"idx/{name}"]]
        # Adam moves an element by <= ~lr per step; a rounding-level grad difference can flip a near-zero one
        tol = 2 * lr * len(ran) + 1e-7 if name in PRE_BN_BIASES else 1e-6 + 1e-3 * lr
        np.testing.assert_allclose(got, g[f"post/{name}"], rtol=1e-5, atol=tol, err_msg=name)
    for name, t in bufs.items():
        # running means carry the pre-BN biases, which may differ by the lr-level Adam noise above
        np.testing.assert_allclose(t.numpy().reshape(-1), g[f"post/{name}"], rtol=1e-5,
                                   atol=1e-7 + 2 * lr * len(ran), err_msg=name)
    np.testing.assert_allclose(mem["memory"].numpy()[g["memory/rows"]], g["memory/val"], rtol=1e-5, atol=1e-6)
    assert mem["ptr"] == int(g["memory/ptr"])
    np.testing.assert_allclose([v["loss"] for v in vals], g["val/batch_loss"], rtol=1e-5)
    err = np.concatenate([t["recon_error"].numpy() for t in tests])
    ms = np.concatenate([t["outputs"]["anomaly_score"].numpy() for t in tests])
    np.testing.assert_allclose(err, g["test/recon"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(ms, g["test/memory"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(np.concatenate([t["combined"].numpy() for t in tests]), g["test/scores"], rtol=1e-5,
                               atol=1e-6)


def test_ae_memory_ring_wraps_like_the_reference():
    """update_memory (cad1:201-219): contiguous write, exact fill to the end (pointer back to 0), wrap-around."""
    mem = torch.zeros(500, 64)
    f = torch.arange(3 * 64, dtype=torch.float32).reshape(3, 64)
    assert ae.update_memory(mem, 10, f) == 13 and torch.equal(mem[10:13], f)
    assert ae.update_memory(mem, 497, f) == 0 and torch.equal(mem[497:], f)
    mem.zero_()
    assert ae.update_memory(mem, 498, f) == 1
    assert torch.equal(mem[498:], f[:2]) and torch.equal(mem[:1], f[2:])
    s = torch.randn(4, 64)
    assert torch.equal(ae.memory_score(s, mem, 9), torch.zeros(4))  # < 10 rows filled: zero scores
