"""avenue_training_script1.py's MiniCausalVAD surface (a1:104-210) and the a2 checkpoint format (a2:438-455):
save/load round trips on CPU, resume-equals-continue on the GPU (bit-exact), AdamW state interchange with torch."""
import numpy as np
import pytest
import torch

from oracle import a2_oracle as ao
from tests.golden.cases import A2_CASES
from tests.golden_util import load
from tests.test_a2_oracle import A2_CKPT


def test_minicausal_import_path_and_surface():
    from vad_amd.minicausal_vad import MiniCausalVAD
    vad = MiniCausalVAD(device="cpu")
    assert vad.optimizer.param_groups[0]["lr"] == 0.001
    for m in ("train_epoch", "evaluate", "save_model", "load_model"):
        assert callable(getattr(vad, m))
    assert sum(p.numel() for p in vad.model.parameters()) == 188849


def test_save_load_roundtrip_cpu(tmp_path):
    from vad_amd.minicausal_vad import MiniCausalVAD
    torch.manual_seed(0)
    a = MiniCausalVAD(device="cpu")
    a.scheduler.best, a.scheduler.bad = 0.25, 3
    a.optimizer.param_groups[0]["lr"] = 2e-4
    a.global_step = 7
    a.save_model(tmp_path / "m.pth")
    torch.manual_seed(1)
    b = MiniCausalVAD(device="cpu")
    b.load_model(tmp_path / "m.pth")
    for (k, v), (k2, v2) in zip(a.model.state_dict().items(), b.model.state_dict().items()):
        assert k == k2 and torch.equal(v, v2), k
    assert b.optimizer.param_groups[0]["lr"] == 2e-4
    assert (b.scheduler.best, b.scheduler.bad, b.global_step) == (0.25, 3, 7)


def test_load_shipped_checkpoint_weights(tmp_path):
    """A bare a2 state_dict (the shipped best_improved_model.pth weights, kept as an npz fixture) loads strictly."""
    from vad_amd.minicausal_vad import MiniCausalVAD
    ck = {k: torch.from_numpy(v) for k, v in load(A2_CKPT).items()}
    torch.save({"model_state_dict": ck, "epoch": 3}, tmp_path / "best.pth")
    vad = MiniCausalVAD(device="cpu")
    vad.load_model(tmp_path / "best.pth")
    for k, v in vad.model.state_dict().items():
        assert torch.equal(v, ck[k]), k


@pytest.mark.gpu
def test_resume_equals_continue_gpu(tmp_path):
    """Two train steps straight through == one step, save_model, load_model into a fresh instance, one more step
    (params and AdamW moments bit-exact); the saved optimizer state loads into torch.optim.AdamW."""
    from vad_amd.minicausal_vad import MiniCausalVAD
    from tests.test_a2_oracle import make_a2_model
    case = A2_CASES[0]
    B, T, H, W = case["B"], case["T"], case["H"], case["W"]
    xs = [ao.synth_clips(case["seed"], s, s * B, B, T, H, W) for s in range(2)]
    ys = [ao.synth_labels(s * B, B) for s in range(2)]

    def fresh():
        v = MiniCausalVAD(device="cuda")
        v.model = make_a2_model(case).to("cuda")
        v.seed = case["seed"]
        return v

    a = fresh()
    a.train_epoch([(xs[0], ys[0])])
    a.save_model(tmp_path / "ck.pth")
    a.train_epoch([(xs[1], ys[1])])

    b = fresh()
    b.load_model(tmp_path / "ck.pth")
    b.clip0 = B
    b.train_epoch([(xs[1], ys[1])])
    torch.cuda.synchronize()
    ea, eb = a.model._engine, b.model._engine
    assert torch.equal(ea.params, eb.params)
    assert torch.equal(ea.exp_avg, eb.exp_avg) and torch.equal(ea.exp_avg_sq, eb.exp_avg_sq)
    assert torch.equal(ea.steps, eb.steps)

    sd = torch.load(tmp_path / "ck.pth", weights_only=True)["optimizer_state_dict"]
    m = make_a2_model(case)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    opt.load_state_dict(sd)
    st = opt.state_dict()["state"]
    assert len(st) == len(list(m.parameters()))
    assert all(float(s["step"]) == 1.0 for s in st.values())
    preds, labels, graphs = b.evaluate([(xs[0], ys[0])])
    assert preds.shape == (B,) and labels.shape == (B,) and graphs.shape == (B, 16, 16)
    assert np.all(np.isfinite(preds))


def test_single_clip_batch_raises_like_reference():
    """B=1: the reference's BCE on a 0-d squeezed score vs (1,) pseudo-targets raises ValueError (a2:146)."""
    from vad_amd.a2 import ImprovedMiniCausalVAD
    vad = ImprovedMiniCausalVAD(device="cpu")
    with pytest.raises(ValueError, match="target size"):
        vad.train_step(torch.zeros(1, 3, 8, 64, 64), torch.zeros(1))
    with pytest.raises(ValueError, match="target size"):
        vad.compute_improved_loss(torch.zeros(1, 1), torch.zeros(1, 16, 16), torch.zeros(1), torch.zeros(1, 16))
