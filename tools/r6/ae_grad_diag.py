"""cad1 bench-shape (B=32, T=16) first-step grads vs the float64 oracle under library knob settings (diagnostic)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import ae_oracle as ae  # noqa: E402
from tests.golden_util import ae_case_data, ae_memory_init  # noqa: E402
from tests.test_ae_oracle import make_ae_model  # noqa: E402
from tests.test_grad64 import AE_BENCH, _d64, _rel  # noqa: E402
from vad_amd import _native as nat  # noqa: E402
from vad_amd.ae import AeTrainer  # noqa: E402

case = dict(AE_BENCH)
if len(sys.argv) > 1:
    case["B"], case["T"] = int(sys.argv[1]), int(sys.argv[2])
    case["labels"] = [[0] * case["B"]]
model0 = make_ae_model(case)
params, bufs, _ = ae.split_state(model0.state_dict())
mem, ptr = ae_memory_init(case)
train, _, _ = ae_case_data(case)
v = train[0][0]
leaves = {n: t.requires_grad_(True) for n, t in _d64(params).items()}
out = ae.ae_forward(leaves, _d64(bufs), v.double(), True, mem.double(), ptr)
ae.safe_mse(out["reconstructed"], v.double()).backward()
ref = {n: t.grad.numpy().reshape(-1) for n, t in leaves.items()}
order = ["decoder.12.weight", "decoder.10.weight", "decoder.10.bias", "decoder.9.weight", "decoder.7.weight",
         "decoder.6.weight", "decoder.4.weight", "decoder.3.weight", "decoder.0.weight", "temporal_encoder.weight_ih_l0",
         "encoder.13.weight", "encoder.10.weight", "encoder.9.weight", "encoder.0.weight"]
for knobs in ([], [("ae_wgrad_stream", 0)], [("ae_direct", 0)], [("conv4_cls_batch_min", 512)],
              [("conv4_split_tiles", 0)]):
    for k, val in knobs:
        nat.check(nat.lib().vad_set_tuning(k.encode(), val))
    m = make_ae_model(case).cuda()
    tr = AeTrainer(m, lr=1e-5)
    tr.step(v.cuda())
    e = m.engine()
    g = e.grads.cpu().numpy().astype(np.float64)
    dev = {name: g[off:off + n] for name, off, n in e.slots}
    print(knobs, " ".join(f"{n.replace('.weight', '')}={_rel(dev[n], ref[n]):.1e}" for n in order), flush=True)
    for k, val in knobs:
        nat.check(nat.lib().vad_set_tuning(k.encode(), {"ae_wgrad_stream": 1, "ae_direct": 1,
                                                         "conv4_cls_batch_min": 0, "conv4_split_tiles": 512}[k]))
