"""Sweep the implicit-GEMM weight-gradient launch (tile id x split-K grid x min K-slices) against the LDS-patch
kernel for the layers whose weight gradient runs in f32 (stride-2 L2/L4/L6 and L7) at config 2.
Usage (GPU box): python tools/tune_wg_s2.py"""
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
defaults = {"conv_wgrad_tile": -1, "conv_wgrad_blocks": 1024, "conv_wgrad_min_ktiles": 16, "conv_wgrad_patch": 1,
            "conv_wgrad_split": 1}


def setk(**kw):
    for k, v in {**defaults, **kw}.items():
        L.vad_set_tuning(k.encode(), int(v))


for li, (NF, ci, co, ih, iw, s) in enumerate(layers(8, 16, 227, 227)):
    if li not in (2, 4, 6, 7):
        continue
    oh, ow = (ih - 1) // s + 1, (iw - 1) // s + 1
    flops = 2.0 * NF * oh * ow * co * ci * 9
    x = torch.randn(NF, ih, iw, ci, device=d)
    dy = torch.randn(NF, oh, ow, co, device=d)
    dW = torch.empty(co, ci, 3, 3, device=d)
    fn = lambda: nat.check(L.vad_conv3x3_wgrad(x.data_ptr(), dy.data_ptr(), NF, ci, ih, iw, co, s, dW.data_ptr(),
                                               part.data_ptr(), part.numel(), st))
    res = {}
    setk()
    res["default"] = timeit(fn) * 1e3
    ref = dW.clone()
    setk(conv_wgrad_patch=2)
    res["patch"] = timeit(fn) * 1e3
    setk(conv_wgrad_patch=0, conv_wgrad_split=0)
    res["nopatch_nosplit"] = timeit(fn) * 1e3
    for tile in (0, 2, 3, 4, 5, 6, 7, 9):
        for blocks in (256, 512, 1024, 2048):
            for mk in (4, 8, 16, 32):
                setk(conv_wgrad_patch=0, conv_wgrad_tile=tile, conv_wgrad_blocks=blocks, conv_wgrad_min_ktiles=mk)
                try:
                    t = timeit(fn) * 1e3
                except RuntimeError as e:
                    continue
                err = float((dW - ref).abs().max() / ref.abs().max())
                if err > 1e-4:
                    continue
                res[f"t{tile}_b{blocks}_k{mk}"] = t
    setk()
    best = sorted(res.items(), key=lambda kv: kv[1])[:6]
    print(json.dumps({"layer": li, "stride": s, "gflop": round(flops / 1e9, 2), "default_us": round(res["default"], 1),
                      "patch_us": round(res["patch"], 1), "nopatch_us": round(res["nopatch_nosplit"], 1),
                      "best": [(k, round(v, 1), round(flops / v / 1e6, 1)) for k, v in best]}), flush=True)
