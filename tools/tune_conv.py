"""Sweep the conv GEMM tile shapes / split-K knobs on the eight ResNetBackbone layers (config-2 shapes).
Usage (GPU box): python tools/tune_conv.py [--B 8 --T 16 --H 227 --W 227] > sweep.json"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vad_amd import _native as nat  # noqa: E402

TILES = {0: "128x32", 1: "256x32", 2: "64x64", 3: "128x64", 4: "64x128", 5: "128x128", 6: "256x64",
         7: "32x128", 8: "32x256", 9: "64x256"}


def layers(B, T, H, W):
    NF = B * T
    h, w = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    out = []
    for ci, co, s in [(32, 32, 1), (32, 32, 1), (32, 64, 2), (64, 64, 1), (64, 128, 2), (128, 128, 1),
                      (128, 256, 2), (256, 256, 1)]:
        out.append((NF, ci, co, h, w, s))
        h, w = (h - 1) // s + 1, (w - 1) // s + 1
    return out


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--H", type=int, default=227)
    ap.add_argument("--W", type=int, default=227)
    ap.add_argument("--patch", action="store_true", help="only compare the LDS-patch kernels with the GEMM path")
    a = ap.parse_args()
    L = nat.lib()
    d = torch.device("cuda")
    st = nat.stream_of(d)
    res = []
    for li, (NF, ci, co, ih, iw, s) in enumerate(layers(a.B, a.T, a.H, a.W)):
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
        if a.patch:
            for op in ("fwd", "dgrad", "wgrad"):
                for on in ((0, 1, 2) if op == "wgrad" else (0, 1)):
                    L.vad_set_tuning(b"conv_patch", min(on, 1))
                    L.vad_set_tuning(b"conv_wgrad_patch", on)
                    if op == "wgrad":
                        fn = lambda: nat.check(L.vad_conv3x3_wgrad(
                            x.data_ptr(), dy.data_ptr(), NF, ci, ih, iw, co, s, dW.data_ptr(), part.data_ptr(),
                            part.numel(), st))
                    elif op == "fwd":
                        fn = lambda: nat.check(L.vad_conv3x3_forward(
                            x.data_ptr(), NF, ci, ih, iw, None, bias.data_ptr(), co, s, y.data_ptr(), wf.data_ptr(),
                            wd.data_ptr(), parts.data_ptr(), st))
                    else:  # the dgrad weight layout depends on the path: re-prepare
                        fn = lambda: nat.check(L.vad_conv3x3_dgrad(
                            dy.data_ptr(), NF, ci, ih, iw, wt.data_ptr(), co, s, dx.data_ptr(), wf.data_ptr(),
                            wd.data_ptr(), st))
                    ms = timeit(fn)
                    r = dict(layer=li, op=op, patch=on, ms=round(ms, 4), tflops=round(flops / ms / 1e9, 2))
                    print(json.dumps(r), flush=True)
            L.vad_set_tuning(b"conv_patch", 1)
            L.vad_set_tuning(b"conv_wgrad_patch", 1)
            continue
        for op in ("fwd", "dgrad", "wgrad"):
            ids = [0, 1, 2, 3, 4, 5, 6, 9] if op != "wgrad" else [2, 3, 4, 5, 7, 8, 9]
            knobs = [(1024, 16)] if op != "wgrad" else [(512, 16), (1024, 16), (2048, 8), (1024, 32)]
            for tid in ids:
                for blocks, mink in knobs:
                    L.vad_set_tuning(f"conv_{op}_tile".encode(), tid)
                    L.vad_set_tuning(b"conv_wgrad_blocks", blocks)
                    L.vad_set_tuning(b"conv_wgrad_min_ktiles", mink)
                    if op == "fwd":
                        fn = lambda: nat.check(L.vad_conv3x3_forward(
                            x.data_ptr(), NF, ci, ih, iw, None, bias.data_ptr(), co, s, y.data_ptr(), wf.data_ptr(),
                            wd.data_ptr(), parts.data_ptr(), st))
                    elif op == "dgrad":
                        fn = lambda: nat.check(L.vad_conv3x3_dgrad(
                            dy.data_ptr(), NF, ci, ih, iw, None, co, s, dx.data_ptr(), wf.data_ptr(), wd.data_ptr(),
                            st))
                    else:
                        fn = lambda: nat.check(L.vad_conv3x3_wgrad(
                            x.data_ptr(), dy.data_ptr(), NF, ci, ih, iw, co, s, dW.data_ptr(), part.data_ptr(),
                            part.numel(), st))
                    ms = timeit(fn)
                    r = dict(layer=li, op=op, tile=TILES[tid], tile_id=tid, blocks=blocks, min_ktiles=mink,
                             ms=round(ms, 4), tflops=round(flops / ms / 1e9, 2))
                    res.append(r)
                    print(json.dumps(r), flush=True)
            L.vad_set_tuning(f"conv_{op}_tile".encode(), -1)
    best = {}
    for r in res:
        k = (r["layer"], r["op"])
        if k not in best or r["ms"] < best[k]["ms"]:
            best[k] = r
    print("BEST", json.dumps([best[k] for k in sorted(best)]))


if __name__ == "__main__":
    main()
