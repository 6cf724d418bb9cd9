"""Round-5 check: one config-2-shape train step with a library knob at A and at B (same init, same clips); reports
the max |diff| of losses / scores and the relative L2 difference of every grad slot between the two runs.
usage: python tools/r5/knob_check.py KNOB A B [--B 8 --T 16 --H 227 --W 227]"""
import argparse
import contextlib
import io
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(knob, v, B, T, H, W):
    from vad_amd import _native as nat
    from vad_amd.cad import CausalAnomalyDetector
    from vad_amd.train import CadTrainer, apply_memory_efficient_training
    nat.check(nat.lib().vad_set_tuning(knob.encode(), int(v)))
    torch.manual_seed(0)
    m = CausalAnomalyDetector()
    with contextlib.redirect_stdout(io.StringIO()):
        apply_memory_efficient_training(m)
    m = m.cuda()
    tr = CadTrainer(m, lr=3e-4, seed=5)
    x = torch.empty(B, T, 1, H, W, device="cuda")
    nat.check(nat.lib().vad_synth_frames(7, 0, 0, B * T, H * W, 0, x.data_ptr(), nat.stream_of(x.device)))
    y = torch.tensor([b % 2 for b in range(B)], device="cuda")
    o = tr.step(x, y, want_outputs=True)
    torch.cuda.synchronize()
    return {"losses": o["losses"].cpu(), "final": o["final"].cpu(), "grads": tr.eng.grads.cpu(),
            "names": tr.eng.slot_names, "offs": tr.eng.slot_offset, "nels": tr.eng.slot_numel}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("knob")
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--H", type=int, default=227)
    ap.add_argument("--W", type=int, default=227)
    a = ap.parse_args()
    ra = run(a.knob, a.a, a.B, a.T, a.H, a.W)
    rb = run(a.knob, a.b, a.B, a.T, a.H, a.W)
    print("losses", ra["losses"].tolist(), rb["losses"].tolist())
    print("max |final diff|", float((ra["final"] - rb["final"]).abs().max()))
    worst = 0.0
    for n, o, k in zip(ra["names"], ra["offs"], ra["nels"]):
        ga, gb = ra["grads"][o:o + k].double(), rb["grads"][o:o + k].double()
        den = float(ga.norm())
        e = float((ga - gb).norm()) / den if den > 0 else float((ga - gb).norm())
        if n.startswith("backbone.") and "conv" in n and n.endswith("weight"):
            print(f"{n}: rel L2 {e:.3g}")
        worst = max(worst, e if den > 1e-6 else 0.0)
    print("worst rel L2 (non-negligible slots)", worst)


if __name__ == "__main__":
    main()
