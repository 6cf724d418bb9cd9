"""Stand-alone weight-gradient timing per backbone layer (kernel + split-K reduce through vad_conv3x3_wgrad) for
knob conv_wgrad_tr (1: conv_x3w.hip, 0: conv_x3.hip) and grid targets, config-2 shapes unless --B/--T/--H/--W.  Prints one JSON line per (layer,
variant).  Usage: python tools/wgrad_bench.py [--versions 1,0] [--blocks 0,256,512]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import conv_shapes  # noqa: E402
from vad_amd import _native as nat  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=8)
ap.add_argument("--T", type=int, default=16)
ap.add_argument("--H", type=int, default=227)
ap.add_argument("--W", type=int, default=227)
ap.add_argument("--versions", default="1")
ap.add_argument("--blocks", default="0")
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
d = torch.device("cuda")
st = nat.stream_of(d)
part = torch.empty(1 << 25, device=d)
strides = [1, 1, 2, 1, 2, 1, 2, 1]
for l, (NF, ci, co, oh, ow) in enumerate(conv_shapes(a.B, a.T, a.H, a.W)):
    s = strides[l]
    ih, iw = (oh * 2 + 1, ow * 2 + 1) if s == 2 else (oh, ow)
    if l == 2:  # (the stride-2 layers' inputs are the previous layer's maps)
        ih, iw = conv_shapes(a.B, a.T, a.H, a.W)[1][3:5]
    elif s == 2:
        ih, iw = conv_shapes(a.B, a.T, a.H, a.W)[l - 1][3:5]
    x = torch.randn(NF, ih, iw, ci, device=d)
    dy = torch.randn(NF, oh, ow, co, device=d)
    dW = torch.empty(co, ci, 3, 3, device=d)
    flops = 2.0 * NF * oh * ow * co * ci * 9
    for v in [int(t) for t in a.versions.split(",")]:
        for nb in [int(t) for t in a.blocks.split(",")]:
            nat.check(nat.lib().vad_set_tuning(b"conv_wgrad_tr", v))
            nat.check(nat.lib().vad_set_tuning(b"conv_wgrad_tr_blocks", nb))
            call = lambda: nat.check(nat.lib().vad_conv3x3_wgrad(x.data_ptr(), dy.data_ptr(), NF, ci, ih, iw, co, s,  # noqa
                                                                 dW.data_ptr(), part.data_ptr(), part.numel(), st))
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                call()
            e1.record()
            torch.cuda.synchronize()
            us = 1e3 * e0.elapsed_time(e1) / a.iters
            print(json.dumps({"layer": l, "shape": [NF, ci, co, ih, iw, s], "version": v, "blocks": nb,
                              "us": round(us, 2), "tflops": round(flops / us / 1e6, 1)}), flush=True)
nat.check(nat.lib().vad_set_tuning(b"conv_wgrad_tr", 1))
nat.check(nat.lib().vad_set_tuning(b"conv_wgrad_tr_blocks", 0))
