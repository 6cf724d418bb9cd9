"""Stand-alone per-layer timing of the backbone convs at config-2 shapes through the ops API (forward, input gradient,
weight gradient incl. its split-K reduce): nothing else runs beside them.  Usage (GPU box):
python tools/r6/conv_standalone.py [--layers 2,4,6] [--ops fwd,dgrad] [--reps 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.tune_conv import layers, timeit  # noqa: E402
from vad_amd import _native as nat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="0,1,2,3,4,5,6,7")
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    L = nat.lib()
    d = torch.device("cuda")
    st = nat.stream_of(d)
    want = [int(x) for x in a.layers.split(",")]
    for li, (NF, ci, co, ih, iw, s) in enumerate(layers(8, 16, 227, 227)):
        if li not in want:
            continue
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
        part = torch.empty(1 << 25, device=d)
        dW = torch.empty(co, ci, 3, 3, device=d)
        nat.check(L.vad_conv3x3_forward(x.data_ptr(), NF, ci, ih, iw, wt.data_ptr(), bias.data_ptr(), co, s,
                                        y.data_ptr(), wf.data_ptr(), wd.data_ptr(), parts.data_ptr(), st))
        nat.check(L.vad_conv3x3_dgrad(dy.data_ptr(), NF, ci, ih, iw, wt.data_ptr(), co, s, dx.data_ptr(),
                                      wf.data_ptr(), wd.data_ptr(), st))
        fns = {
            "fwd": lambda: nat.check(L.vad_conv3x3_forward(x.data_ptr(), NF, ci, ih, iw, None, bias.data_ptr(), co, s,
                                                           y.data_ptr(), wf.data_ptr(), wd.data_ptr(),
                                                           parts.data_ptr(), st)),
            "dgrad": lambda: nat.check(L.vad_conv3x3_dgrad(dy.data_ptr(), NF, ci, ih, iw, None, co, s, dx.data_ptr(),
                                                           wf.data_ptr(), wd.data_ptr(), st)),
            "wgrad": lambda: nat.check(L.vad_conv3x3_wgrad(x.data_ptr(), dy.data_ptr(), NF, ci, ih, iw, co, s,
                                                           dW.data_ptr(), part.data_ptr(), part.numel(), st)),
        }
        for op in a.ops.split(","):
            if op == "dgrad" and li == 0:
                continue
            ms = timeit(fns[op], a.reps)
            print(json.dumps(dict(tag=a.tag, layer=li, op=op, us=round(ms * 1e3, 2),
                                  tflops=round(flops / ms / 1e9, 2))), flush=True)


if __name__ == "__main__":
    main()
