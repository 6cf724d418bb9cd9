"""Time the stride-1 weight-gradient kernels (split-bf16 vs f32 LDS-patch, incl. the slab reduce) on the backbone
layers of config 2, with the measurement-only conv_split_dbg bits (2 no split, 4 no MFMA, 8 no global loads).
Usage (GPU box): python tools/tune_wg.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.tune_conv import layers, timeit  # noqa: E402
from vad_amd import _native as nat  # noqa: E402

L = nat.lib()
d = torch.device("cuda")
st = nat.stream_of(d)
part = torch.empty(1 << 24, device=d)
for li, (NF, ci, co, ih, iw, s) in enumerate(layers(8, 16, 227, 227)):
    if s != 1:
        continue
    flops = 2.0 * NF * ih * iw * co * ci * 9
    x = torch.randn(NF, ih, iw, ci, device=d)
    dy = torch.randn(NF, ih, iw, co, device=d)
    dW = torch.empty(co, ci, 3, 3, device=d)
    row = {"layer": li, "gflop": round(flops / 1e9, 2)}
    for name, split, dbg in [("f32", 0, 0), ("x3", 1, 0), ("x3_nosplit", 1, 2), ("x3_nomfma", 1, 4),
                             ("x3_noload", 1, 8), ("x3_only_mfma", 1, 10)]:
        L.vad_set_tuning(b"conv_wgrad_split", split)
        L.vad_set_tuning(b"conv_split_dbg", dbg)
        fn = lambda: nat.check(L.vad_conv3x3_wgrad(x.data_ptr(), dy.data_ptr(), NF, ci, ih, iw, co, 1, dW.data_ptr(),
                                                   part.data_ptr(), part.numel(), st))
        row[name + "_us"] = round(timeit(fn) * 1e3, 1)
    L.vad_set_tuning(b"conv_wgrad_split", 1)
    L.vad_set_tuning(b"conv_split_dbg", 0)
    print(json.dumps(row), flush=True)
