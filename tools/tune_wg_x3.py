"""Stride-1 weight gradients at config 2: split-bf16 kernel (incl. the 8x8-frame layer L7, knob
conv_wgrad_split=2) vs the f32 patch kernel, over the split-K grid target (conv_wgrad_patch_blocks).
Usage (GPU box): python tools/tune_wg_x3.py"""
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
part = torch.empty(1 << 25, device=d)
for li, (NF, ci, co, ih, iw, s) in enumerate(layers(8, 16, 227, 227)):
    if s != 1:
        continue
    flops = 2.0 * NF * ih * iw * co * ci * 9
    x = torch.randn(NF, ih, iw, ci, device=d)
    dy = torch.randn(NF, ih, iw, co, device=d)
    dW = torch.empty(co, ci, 3, 3, device=d)
    fn = lambda: nat.check(L.vad_conv3x3_wgrad(x.data_ptr(), dy.data_ptr(), NF, ci, ih, iw, co, 1, dW.data_ptr(),
                                               part.data_ptr(), part.numel(), st))
    res = {}
    ref = None
    for split in (0, 2):
        for blocks in (256, 512, 768, 1024, 2048):
            L.vad_set_tuning(b"conv_wgrad_split", split)
            L.vad_set_tuning(b"conv_wgrad_patch_blocks", blocks)
            t = timeit(fn) * 1e3
            if ref is None:
                ref = dW.clone()
            err = float((dW - ref).abs().max() / ref.abs().max())
            res[f"{'x3' if split else 'f32'}_b{blocks}"] = (round(t, 1), round(flops / t / 1e6, 1), f"{err:.1e}")
    L.vad_set_tuning(b"conv_wgrad_split", 1)
    L.vad_set_tuning(b"conv_wgrad_patch_blocks", 512)
    print(json.dumps({"layer": li, "gflop": round(flops / 1e9, 2), "res": res}), flush=True)
