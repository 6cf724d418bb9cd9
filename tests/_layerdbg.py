import sys, ctypes, numpy as np, torch
sys.path.insert(0, '/root/repo')
from oracle import cad_oracle as co
from tests.golden_util import make_cad_model
from vad_amd import _native as nat

def read(pl, name, idx=0, n=None):
    p = ctypes.c_void_p(); k = ctypes.c_int64()
    nat.check(nat.lib().vad_cad_debug_buffer(pl.h, name.encode(), idx, ctypes.byref(p), ctypes.byref(k)))
    n = k.value if n is None else n
    out = np.empty(n, np.float32)
    nat.check(nat.lib().vad_debug_d2h(out.ctypes.data, p.value, n * 4))
    return out

B, T, H, W = [int(v) for v in sys.argv[1:5]]
case = dict(B=B, T=T, H=H, W=W, seed=3, step=0, forced=None)
m = make_cad_model(case).cuda(); eng = m.engine()
x = co.synth_clips(3, 0, 0, B, T, H, W); y = co.synth_labels(0, B)
mc = make_cad_model(case)
sd = {k: v.clone() for k, v in mc.state_dict().items()}
params = {k: v.requires_grad_(not k.startswith(co.FROZEN_PREFIXES)) for k, v in sd.items() if "running" not in k and "num_batches" not in k}
bufs = {k: v for k, v in sd.items() if "running" in k}
rec = {}
out = co.cad_forward(params, bufs, x, co.CadDraws.make(3, 0, 0, B, T), True, rec)
co.cad_losses(out, y)["total"].backward()
def nhwc(t): return t.detach().permute(0, 2, 3, 1).contiguous().numpy().reshape(-1)
def rel(a, b): return float(np.abs(a - b).max() / (np.sqrt((b.astype(np.float64) ** 2).mean()) + 1e-30))
eng.forward(x.cuda(), True, 3, 0, 0, y.cuda()); torch.cuda.synchronize()
pl = eng._last[0]
print("pool", rel(read(pl, "pool"), nhwc(rec["pool"])))
for l in range(8):
    print("fwd y", l, rel(read(pl, "y", l), nhwc(rec[f"y{l}"])))
for stop in range(7, -1, -1):
    nat.check(nat.lib().vad_cad_set_debug(pl.h, b"stop_layer", stop))
    eng.forward(x.cuda(), True, 3, 0, 0, y.cuda()); eng.backward(True); torch.cuda.synchronize()
    yg = nhwc(rec[f"y{stop}"].grad)
    dY = read(pl, "dY", 0, yg.size)
    msg = f"bwd layer {stop}: dY {rel(dY, yg):.2e}"
    if stop > 0:
        ag = nhwc(rec[f"a{stop-1}"].grad)
        msg += f"  dA(prev) {rel(read(pl, 'dA', 0, ag.size), ag):.2e}"
    print(msg, flush=True)

# BN-backward coefficients of one layer vs numpy
L = int(sys.argv[5]) if len(sys.argv) > 5 else 3
nat.check(nat.lib().vad_cad_set_debug(pl.h, b"stop_layer", L))
eng.forward(x.cuda(), True, 3, 0, 0, y.cuda()); eng.backward(True); torch.cuda.synchronize()
yl = rec[f"y{L}"].detach().permute(0, 2, 3, 1).reshape(-1, rec[f"y{L}"].shape[1]).double().numpy()
dA = rec[f"a{L}"].grad.permute(0, 2, 3, 1).reshape(yl.shape).double().numpy()
C = yl.shape[1]
bnn = co.BACKBONE_CONVS[L][1]
gam = params[bnn + ".weight"].detach().double().numpy(); bet = params[bnn + ".bias"].detach().double().numpy()
mean = yl.mean(0); var = yl.var(0); inv = 1 / np.sqrt(var + 1e-5)
xh = (yl - mean) * inv; z = xh * gam + bet; dZ = dA * (z > 0)
ref = np.concatenate([mean, inv, gam * inv, bet - mean * gam * inv, gam * inv, dZ.mean(0), (dZ * xh).mean(0)])
st = read(pl, "stats", L + 1)
names = ["mean", "invstd", "scale", "shift", "k", "mdz", "mdzx"]
for i, n in enumerate(names):
    a, b = st[i * C:(i + 1) * C], ref[i * C:(i + 1) * C]
    print(f"layer {L} {n:7s} max rel err {np.abs(a - b).max() / (np.abs(b).max() + 1e-30):.2e}  first {a[:3]} vs {b[:3]}")
dYg = read(pl, "dY", 0, yl.size).reshape(yl.shape).astype(np.float64)
ref_dY = gam * inv * (dZ - dZ.mean(0) - xh * (dZ * xh).mean(0))
err = np.abs(dYg - ref_dY) / (np.sqrt((ref_dY ** 2).mean()) + 1e-30)
bad = np.argwhere(err > 1e-3)
print("dY bad elements:", len(bad), "of", err.size, "rows", np.unique(bad[:, 0])[:20], "... nrows", len(np.unique(bad[:, 0])), "chans", np.unique(bad[:, 1])[:20])
print("row ranges bad:", bad[:, 0].min() if len(bad) else None, bad[:, 0].max() if len(bad) else None)
