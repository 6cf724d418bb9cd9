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
def read_ae_debug(plan, name, idx=0):
    """Copy a cad1 plan's debug buffer (vad_ae_debug_buffer) to the host (float32)."""
    import ctypes
    from vad_amd import _native as nat
    p, k = ctypes.c_void_p(), ctypes.c_int64()
    nat.check(nat.lib().vad_ae_debug_buffer(plan.h, name.encode(), idx, ctypes.byref(p), ctypes.byref(k)))
    out = np.empty(k.value, np.float32)
    nat.check(nat.lib().vad_debug_d2h(out.ctypes.data, p.value, out.nbytes))
    return out


def ae_leaky_pins(plan, B, T):
    """The LeakyReLU decisions of the device's last cad1 forward, in the oracle's layout (ae_oracle.ae_forward pins):
    the sign of y * scale + shift computed exactly in float64 from the device's raw conv outputs and BN state (the
    device's fp32 fma decision), and of the decoder Linear's output."""
    from oracle import ae_oracle as ae
    enc_hw = (32, 16, 8, 4)
    enc = [[None] * 4 for _ in range(T)]
    for l in range(4):
        C, hw = (32, 64, 128, 128)[l], enc_hw[l]
        y = read_ae_debug(plan, "ey", l).astype(np.float64).reshape(T, B, hw, hw, C)
        st = read_ae_debug(plan, "est", l).astype(np.float64).reshape(T, 8, C)
        z = y * st[:, None, None, None, 2, :] + st[:, None, None, None, 3, :]
        m = torch.from_numpy(np.ascontiguousarray((z > 0).transpose(0, 1, 4, 2, 3)))
        for t in range(T):
            enc[t][l] = m[t]
    dec = [torch.from_numpy(read_ae_debug(plan, "u").reshape(B, 2048) > 0)]
    for j in range(3):
        C, hw = (128, 64, 32)[j], (8, 16, 32)[j]
        y = read_ae_debug(plan, "dy", j).astype(np.float64).reshape(B, hw, hw, C)
        st = read_ae_debug(plan, "dst", j).astype(np.float64).reshape(8, C)
        dec.append(torch.from_numpy(np.ascontiguousarray((y * st[2] + st[3] > 0).transpose(0, 3, 1, 2))))
    assert len(ae.ENC_CONVS) == 4
    return {"enc": enc, "dec": dec}
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


def read_act(plan, name, idx=0):
    """A backbone activation buffer as float64, whatever its storage (fp32, or bf16 when the plan ran act_bf16)."""
    if int(read_debug_len(plan, "act_bf16")) == 1 and name in ("y", "pool"):
        u = read_debug(plan, name, idx, dtype=np.uint16)
        return (u.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    return read_debug(plan, name, idx).astype(np.float64)


def read_debug_len(plan, name, idx=0):
    import ctypes
    from vad_amd import _native as nat
    p, k = ctypes.c_void_p(), ctypes.c_int64()
    nat.check(nat.lib().vad_cad_debug_buffer(plan.h, name.encode(), idx, ctypes.byref(p), ctypes.byref(k)))
    return k.value


def hip_relu_masks(eng, NF):
    """The ReLU decisions the HIP forward took after the eight 3x3-conv BatchNorms: relu(fma(y, scale, shift)) is
    taken iff the exact value y*scale + shift > 0.  y*scale is exact in float64 (24-bit x 24-bit mantissas) and the
    float64 add keeps the sign, so the comparison reproduces the device's fp32 fma decision bit for bit (bf16-stored
    activations are widened exactly first).
    Returns 8 bool tensors (NF, C, OH, OW) for oracle.cad_oracle.backbone_forward(relu_masks=...)."""
    pl = eng._last[0]
    masks = []
    for l in range(8):
        st = read_debug(pl, "stats", l + 1)
        C = st.size // 7  # BN stats layout [7C] (csrc/common.h BN_STATS_PER_C)
        y = read_act(pl, "y", l).reshape(NF, -1, C)
        z = y * st[2 * C:3 * C].astype(np.float64) + st[3 * C:4 * C].astype(np.float64)
        masks.append(torch.from_numpy(z > 0).permute(0, 2, 1))  # (NF, C, OH*OW); pinned_oracle_grads reshapes
    return masks


def hip_stem_pins(eng, NF, H, W):
    """The training stem's decisions in the HIP forward (option stem_grad: conv1's output y1 stored): bn1's ReLU
    mask (exact sign of y1*scale + shift, as hip_relu_masks) and the MaxPool2d(3, 2, 1) window maxima under torch's
    first-max rule (strict >, row-major window scan) over z = relu(fma(y1, scale, shift)) rounded to fp32 as the
    device computes it (backbone.hip maxpool_bwd_kernel).  Returns (mask (NF, 32, H1, W1) bool, idx (NF, 32, HP, WP)
    int64 flat indices into each H1 x W1 plane) for backbone_forward(stem_pins=...)."""
    pl = eng._last[0]
    H1, W1 = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    HP, WP = (H1 - 1) // 2 + 1, (W1 - 1) // 2 + 1
    st = read_debug(pl, "stats", 0).astype(np.float64)
    y1 = read_debug(pl, "y1").astype(np.float64).reshape(NF, H1, W1, 32)
    zz = y1 * st[64:96] + st[96:128]
    mask = zz > 0
    idx = first_max_pool_idx(np.maximum(zz.astype(np.float32), np.float32(0)))
    return (torch.from_numpy(mask).permute(0, 3, 1, 2).contiguous(),
            torch.from_numpy(idx).permute(0, 3, 1, 2).contiguous())


def first_max_pool_idx(z):
    """MaxPool2d(3, 2, 1) window maxima of an NHWC array as flat indices into each H x W plane, torch's rule: scan
    the window row-major, take a value when it is strictly greater than the best so far (padding never wins).
    Returns (N, OH, OW, C) int64."""
    N, H, W, C = z.shape
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    zp = np.full((N, H + 2, W + 2, C), -np.inf, z.dtype)
    zp[:, 1:-1, 1:-1] = z
    best = np.full((N, OH, OW, C), -np.inf, z.dtype)
    idx = np.zeros((N, OH, OW, C), np.int64)
    oy = np.arange(OH)[:, None] * 2
    ox = np.arange(OW)[None, :] * 2
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            v = zp[:, oy + 1 + dy, ox + 1 + dx]
            better = v > best
            best = np.where(better, v, best)
            idx = np.where(better, ((oy + dy) * W + (ox + dx))[None, :, :, None], idx)
    return idx


def reshape_masks(masks, x):
    """hip_relu_masks output (NF, C, OH*OW) -> the (NF, C, OH, OW) tensors backbone_forward takes."""
    from oracle import cad_oracle as co
    shapes = []
    NF = x.shape[0] * x.shape[1]
    h, w = (x.shape[3] - 1) // 2 + 1, (x.shape[4] - 1) // 2 + 1
    h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    for _, _, s in co.BACKBONE_CONVS:
        h, w = (h - 1) // s + 1, (w - 1) // s + 1
        shapes.append((h, w))
    return [m.reshape(NF, m.shape[1], hh, ww) for m, (hh, ww) in zip(masks, shapes)]


def pinned_oracle_grads(state_dict, x, labels, draws, masks, sync_group=None, bf16=False, dtype=torch.float64,
                        head_masks=None):
    """float64 oracle forward/backward of one train step with the ReLU decisions of another forward (masks from
    hip_relu_masks): the exact gradient of that forward's piecewise-linear branch, free of kink flips.  Returns
    (grads {name: float64 tensor or None}, losses {name: float64}, the oracle's result dict incl. "bufs" and
    "record" -- the float64 BatchNorm outputs "z{l}" in front of each pinned ReLU, for check_mask_flips).
    bf16: the backbone as the device computes it in bf16 mode (cad_oracle.backbone_forward_bf16; "reversed": its convs
    sum the input channels in reverse order).  dtype: the oracle's arithmetic (float64; float32 gives further,
    independent restatements at fp32 accumulation).  head_masks: the direct classifier's ReLU decisions too
    (cad_oracle.direct_forward's masks; its pre-activations land in record["dir_z{i}"])."""
    from oracle import cad_oracle as co
    params = {k: v.detach().to(dtype).clone() for k, v in state_dict.items()
              if "running" not in k and "num_batches" not in k}
    bufs = {k: v.detach().to(dtype).clone() for k, v in state_dict.items() if "running" in k}
    xd = x.to(dtype)
    rm = reshape_masks(masks, xd)
    record = {}
    kw = dict(bf16=bf16) if bf16 else {}
    if head_masks is not None:
        kw["head_masks"] = head_masks
    res = co.cad_train_step(params, bufs, {}, xd, labels, draws, relu_masks=rm, sync_group=sync_group,
                            record=record, **kw)
    res["bufs"] = bufs  # running stats after the step's forward
    res["record"] = record
    return res["grads"], res["losses"], res


def check_mask_flips(masks, record, x, ulps=64, unit=2.0 ** -24, accum=True):
    """The mask-pinned method takes the device's ReLU decisions; this bounds them: a decision may differ from the sign
    of the float64 oracle's own BatchNorm output z (the pinned oracle forward, record["z{l}"], i.e. the same branch
    taken in the layers below) only where |z| <= ulps units of the accumulation magnitude of that layer's conv,
    unit * sqrt(K) * RMS_c(z) per channel (K = 9 Ci: a K-term fp32 sum carries ~sqrt(K) roundings of the terms'
    scale; accum=False: unit * RMS_c(z), for bf16 storage whose one rounding of y dominates).  Returns per layer
    (flips, largest |z| at a flip / its bound); raises if a flip lies outside the bound."""
    from oracle import cad_oracle as co
    rm = reshape_masks(masks, x.double())
    out = []
    cin = [32, 32, 32, 64, 64, 128, 128, 256]
    for l, m in enumerate(rm):
        z = record[f"z{l}"]
        rms = z.pow(2).mean(dim=(0, 2, 3)).sqrt()[None, :, None, None]
        bound = ulps * unit * ((9 * cin[l]) ** 0.5 if accum else 1.0) * rms
        flips = (z > 0) != m.to(torch.bool)
        n = int(flips.sum())
        worst = float((z.abs() / bound)[flips].max()) if n else 0.0
        bad = flips & (z.abs() > bound)
        assert not bool(bad.any()), (f"layer {l}: {int(bad.sum())} of {n} ReLU decisions differ from the float64 "
                                     f"forward beyond {ulps} ulp of the accumulation scale (worst |z|/bound {worst:.3g})")
        out.append((n, worst))
    return out


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
