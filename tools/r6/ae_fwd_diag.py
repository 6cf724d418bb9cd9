"""cad1 bench-shape train-mode forward (B=32, T=16) vs the float64 oracle: batched vs per-class parity-class GEMMs."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import ae_oracle as ae  # noqa: E402
from tests.golden_util import ae_case_data, ae_memory_init  # noqa: E402
from tests.test_ae_oracle import make_ae_model  # noqa: E402
from tests.test_grad64 import AE_BENCH, _d64, _rel  # noqa: E402
from vad_amd import _native as nat  # noqa: E402

case = dict(AE_BENCH)
m0 = make_ae_model(case)
params, bufs, _ = ae.split_state(m0.state_dict())
mem, ptr = ae_memory_init(case)
v = ae_case_data(case)[0][0][0]
rec = {}
ref = ae.ae_forward(_d64(params), _d64(bufs), v.double(), True, mem.double(), ptr, record=rec) if "record" in \
    ae.ae_forward.__code__.co_varnames else ae.ae_forward(_d64(params), _d64(bufs), v.double(), True, mem.double(), ptr)
for val in (0, 512):
    nat.check(nat.lib().vad_set_tuning(b"conv4_cls_batch_min", val))
    m = make_ae_model(case).cuda().train()
    with torch.no_grad():
        out = m(v.cuda())
    print(val, {k: f"{_rel(out[k].cpu().double().numpy(), ref[k].detach().numpy()):.2e}"
                for k in ("frame_features", "sequence_feature", "reconstructed")}, flush=True)
nat.check(nat.lib().vad_set_tuning(b"conv4_cls_batch_min", 0))
