"""Debug helper: per-element view of a minicausal golden case (grad / post-step param) on the GPU."""
import sys
import numpy as np
sys.path.insert(0, ".")
from tests.golden.cases import MC_CASES  # noqa: E402
from tests.golden_util import load  # noqa: E402
from tests.test_mc_gpu import _trainer  # noqa: E402
from tests.test_mc_oracle import make_mc_model  # noqa: E402

for case in MC_CASES:
    g = load(f"mc_{case['name']}.npz")
    model = make_mc_model(case)
    init = {n: p.detach().clone().numpy().reshape(-1) for n, p in model.named_parameters()}
    tr = _trainer(case, model)
    tr.train_epoch()
    e = model._engine
    sd = model.state_dict()
    for name, off, n in e.slots:
        idx = g[f"idx/{name}"]
        got = sd[name].detach().cpu().numpy().reshape(-1)[idx]
        bad = np.abs(got - g[f"post/{name}"]) > 5e-5
        if bad.any():
            gf = e.grads[off:off + n].cpu().numpy()[idx]
            for k in np.nonzero(bad)[0]:
                print(case["name"], name, int(idx[k]), "init", init[name][idx[k]], "grad gpu", gf[k], "grad ref",
                      g[f"grad/{name}"][k], "post gpu", got[k], "post ref", g[f"post/{name}"][k])
