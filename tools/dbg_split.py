"""Compare the CAD train-step gradients of the split-bf16 and f32 conv kernels against the golden vectors of one
case: per slot, the sampled-element violations and, for conv weights, which output channels they sit in."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from tests.golden_util import cad_cases, load  # noqa: E402
from tests.test_cad_gpu import _hip_step  # noqa: E402
import vad_amd._native as nat  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "forced_b3t5_96x80"
case = [c for c in cad_cases() if c["name"] == name][0]
g = load(f"cad_{name}.npz")
res = {}
for split in (0, 1):
    nat.lib().vad_set_tuning(b"conv_split", split)
    m, eng, o, grads, tn = _hip_step(case, step_opt=False)
    res[split] = grads.cpu().numpy()
    print("split", split, "final scores max diff", float(np.abs(o["final"].cpu().numpy() - g["out/anomaly_scores"]).max()))
nat.lib().vad_set_tuning(b"conv_split", 1)
for i, n in enumerate(eng.slot_names):
    k = f"grad/{n}"
    if k not in g:
        continue
    off, nel = eng.slot_offset[i], eng.slot_numel[i]
    idx = g[f"idx/{n}"]
    ref = g[k]
    rn = float(g[f"grad_norm/{n}"])
    for split in (0, 1):
        gf = res[split][off:off + nel]
        err = np.abs(gf[idx] - ref)
        bad = err > 3e-3 * np.abs(ref) + 1e-7 + 2e-4 * rn / np.sqrt(nel)
        if bad.any():
            msg = f"{n} split={split}: {int(bad.sum())}/{len(idx)} bad, max err {err.max():.3e}, rms ref {rn/np.sqrt(nel):.3e}"
            if n.endswith("weight") and nel % 9 == 0:
                per_co = nel // (9 * 1)
                # conv weight [Co][Ci][3][3]: which output channels
                shape_co = None
                for co in (32, 64, 128, 256):
                    if nel % (co * 9) == 0 and nel // (co * 9) in (32, 64, 128, 256):
                        shape_co = co
                        ci = nel // (co * 9)
                        break
                if shape_co:
                    cos = sorted(set((idx[bad] // (ci * 9)).tolist()))
                    msg += f" output channels {cos}"
            print(msg)
    d = res[1][off:off + nel] - res[0][off:off + nel]
    print(f"  {n}: |split - f32| max {np.abs(d).max():.3e}  (rms grad {np.linalg.norm(res[0][off:off+nel])/np.sqrt(nel):.3e})")
