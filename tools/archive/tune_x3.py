"""Time the split-bf16 conv kernels (forward / stride-1 input gradient) on the eight backbone layers of config 2
against the f32 patch kernels, with measurement-only knobs that remove parts of the work (conv_split_dbg bits:
1 no weight restaging, 2 no patch split, 4 no MFMA, 8 no patch loads).  Usage (GPU box): python tools/tune_x3.py"""
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
variants = [("f32", 0, 0, 0), ("x3", 1, 0, 0), ("x3_nt1", 1, 1, 0), ("x3_nt2", 1, 2, 0)] + \
           [(f"x3_dbg{b}", 1, 0, b) for b in (1, 2, 4, 8, 3, 11, 15)]
out = []
for li, (NF, ci, co, ih, iw, s) in enumerate(layers(8, 16, 227, 227)):
    oh, ow = (ih - 1) // s + 1, (iw - 1) // s + 1
    flops = 2.0 * NF * oh * ow * co * ci * 9
    x = torch.randn(NF, ih, iw, ci, device=d)
    wt = torch.randn(co, ci, 3, 3, device=d) * 0.05
    bias = torch.randn(co, device=d)
    y = torch.empty(NF, oh, ow, co, device=d)
    dy = torch.randn(NF, oh, ow, co, device=d)
    dx = torch.empty(NF, ih, iw, ci, device=d)
    wf = torch.empty(9 * ci * co, device=d)
    wd = torch.empty(9 * ci * co, device=d)
    parts = torch.empty((NF * oh * ow // 32 + 8) * 2 * co, device=d)
    row = {"layer": li, "shape": [NF, ci, co, ih, iw, s], "gflop": flops / 1e9}
    for name, split, nt, dbg in variants:
        L.vad_set_tuning(b"conv_split", split)
        L.vad_set_tuning(b"conv_split_nt", nt)
        L.vad_set_tuning(b"conv_split_dbg", dbg)
        fwd = lambda: nat.check(L.vad_conv3x3_forward(x.data_ptr(), NF, ci, ih, iw, wt.data_ptr(), bias.data_ptr(),
                                                      co, s, y.data_ptr(), wf.data_ptr(), wd.data_ptr(),
                                                      parts.data_ptr(), st))
        dg = lambda: nat.check(L.vad_conv3x3_dgrad(dy.data_ptr(), NF, ci, ih, iw, wt.data_ptr(), co, s, dx.data_ptr(),
                                                   wf.data_ptr(), wd.data_ptr(), st))
        row[f"fwd_{name}_us"] = round(timeit(fwd) * 1e3, 1)
        if s == 1:
            row[f"dgrad_{name}_us"] = round(timeit(dg) * 1e3, 1)
    L.vad_set_tuning(b"conv_split", 1)
    L.vad_set_tuning(b"conv_split_nt", 0)
    L.vad_set_tuning(b"conv_split_dbg", 0)
    out.append(row)
    print(json.dumps(row), flush=True)
