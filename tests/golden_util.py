"""Helpers shared by the parity tests: golden fixture loading and reference-identical model construction."""
import glob
import os

import numpy as np
import torch

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# the reference's shipped a2 checkpoint (best_improved_model.pth, model_state_dict) exported as a safe .npz
A2_CKPT = "a2_best_improved_model.npz"


def load(name):
    return dict(np.load(os.path.join(GOLDEN_DIR, name), allow_pickle=False))


def cad_cases():
    from tests.golden.cases import CAD_CASES
    return CAD_CASES


def make_cad_model(case):
    """Our drop-in module under the case seed (identical init to the reference), with the forced-detector edit."""
    from vad_amd.cad import CausalAnomalyDetector
    from tests.golden.cases import force_detector
    torch.manual_seed(case["seed"])
    m = CausalAnomalyDetector(num_factors=6, reid_dim=64)
    if case["forced"]:
        force_detector(m.state_dict(), case["forced"])
    return m


def ae_memory_init(case):
    """(normal_memory (500, 64), memory_ptr) of a cad1 AE case before training."""
    mem = torch.zeros(500, 64)
    if case["mem"] is None:
        return mem, 0
    rows, ptr = case["mem"]
    mem[:rows] = torch.from_numpy(np.random.default_rng(case["seed"]).standard_normal((rows, 64)).astype(np.float32))
    return mem, ptr


def ae_case_data(case):
    """(train, val, test) lists of (clips (B, T, 1, 64, 64), int64 labels) of a cad1 AE case."""
    from oracle import ae_oracle as ae
    B, T, seed = case["B"], case["T"], case["seed"]
    lab = lambda v: torch.tensor(v, dtype=torch.int64)  # noqa: E731
    train = [(ae.synth_clips(seed, k, k * B, B, T), lab(y)) for k, y in enumerate(case["labels"])]
    val = [(ae.synth_clips(seed, 100, 0, len(case["val_labels"]), T), lab(case["val_labels"]))]
    test = [(ae.synth_clips(seed, 200, 0, len(case["test_labels"]), T), lab(case["test_labels"]))]
    return train, val, test


def golden_names():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


# ---------------------------------------------------------------- mask-pinned oracle gradients (GPU tests)
def read_debug(plan, name, idx=0, n=None, dtype=np.float32):
    """Copy a plan's debug buffer (vad_cad_debug_buffer) to the host."""
    import ctypes
    from vad_amd import _native as nat
    p, k = ctypes.c_void_p(), ctypes.c_int64()
    nat.check(nat.lib().vad_cad_debug_buffer(plan.h, name.encode(), idx, ctypes.byref(p), ctypes.byref(k)))
    n = k.value if n is None else n
    out = np.empty(n, dtype)
    nat.check(nat.lib().vad_debug_d2h(out.ctypes.data, p.value, out.nbytes))
    return out


def hip_relu_masks(eng, NF):
    """The ReLU decisions the HIP forward took after the eight 3x3-conv BatchNorms: relu(fma(y, scale, shift)) is
    taken iff the exact value y*scale + shift > 0.  y*scale is exact in float64 (24-bit x 24-bit mantissas) and the
    float64 add keeps the sign, so the comparison reproduces the device's fp32 fma decision bit for bit.
    Returns 8 bool tensors (NF, C, OH, OW) for oracle.cad_oracle.backbone_forward(relu_masks=...)."""
    pl = eng._last[0]
    masks = []
    for l in range(8):
        st = read_debug(pl, "stats", l + 1)
        C = st.size // 7  # BN stats layout [7C] (csrc/common.h BN_STATS_PER_C)
        y = read_debug(pl, "y", l).astype(np.float64).reshape(NF, -1, C)
        z = y * st[2 * C:3 * C].astype(np.float64) + st[3 * C:4 * C].astype(np.float64)
        masks.append(torch.from_numpy(z > 0).permute(0, 2, 1))  # (NF, C, OH*OW); pinned_oracle_grads reshapes
    return masks


def pinned_oracle_grads(state_dict, x, labels, draws, masks, sync_group=None):
    """float64 oracle forward/backward of one train step with the ReLU decisions of another forward (masks from
    hip_relu_masks): the exact gradient of that forward's piecewise-linear branch, free of kink flips.  Returns
    (grads {name: float64 tensor or None}, losses {name: float64}, the oracle's result dict incl. "bufs")."""
    from oracle import cad_oracle as co
    params = {k: v.detach().double().clone() for k, v in state_dict.items()
              if "running" not in k and "num_batches" not in k}
    bufs = {k: v.detach().double().clone() for k, v in state_dict.items() if "running" in k}
    xd = x.double()
    shapes = []
    NF = xd.shape[0] * xd.shape[1]
    h, w = (xd.shape[3] - 1) // 2 + 1, (xd.shape[4] - 1) // 2 + 1
    h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    for _, _, s in co.BACKBONE_CONVS:
        h, w = (h - 1) // s + 1, (w - 1) // s + 1
        shapes.append((h, w))
    rm = [m.reshape(NF, m.shape[1], hh, ww) for m, (hh, ww) in zip(masks, shapes)]
    res = co.cad_train_step(params, bufs, {}, xd, labels, draws, relu_masks=rm, sync_group=sync_group)
    res["bufs"] = bufs  # running stats after the step's forward
    return res["grads"], res["losses"], res


def rel_l2(a, b):
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def check_running_stats(flat_bufs, ref_bufs, rtol=1e-4, atol=1e-5):
    """The engine's flat BN running-stat buffer (library layout) vs {state_dict name: tensor}."""
    from vad_amd import _native as nat
    L = nat.lib()
    fb = flat_bufs.detach().cpu().numpy()
    for i in range(L.vad_cad_num_bufs()):
        n, o, k = L.vad_cad_buf_name(i).decode(), L.vad_cad_buf_offset(i), L.vad_cad_buf_numel(i)
        np.testing.assert_allclose(fb[o:o + k], ref_bufs[n].detach().double().numpy().reshape(-1), rtol=rtol,
                                   atol=atol, err_msg=n)
