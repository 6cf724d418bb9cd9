"""Per-op HIP-event marks (breakdown mode: hipEventRecord around every labelled op, on its stream) of the post-backbone
chain of one config-2 train step: from the end of the last forward conv to the start of avgpool_bwd.
usage: python tools/exp/chain_marks.py [KNOB=V ...]"""
import os, sys, io, contextlib
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vad_amd import _native as nat
from vad_amd.cad import CausalAnomalyDetector
from vad_amd.train import CadTrainer, apply_memory_efficient_training
for kv in [a for a in sys.argv[1:] if "=" in a]:
    k, v = kv.split("=")
    nat.check(nat.lib().vad_set_tuning(k.encode(), int(v)))
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = CausalAnomalyDetector()
with contextlib.redirect_stdout(io.StringIO()):
    apply_memory_efficient_training(m)
m = m.to(dev)
tr = CadTrainer(m, lr=3e-4, seed=1234)
B, T, H, W = 8, 16, 227, 227
x = torch.empty(B, T, 1, H, W, device=dev)
nat.check(nat.lib().vad_synth_frames(7, 0, 0, B * T, H * W, 0, x.data_ptr(), nat.stream_of(dev)))
y = torch.tensor([b % 2 for b in range(B)], device=dev)
eng = tr.eng
for _ in range(5):
    tr.step(x, y)
torch.cuda.synchronize()
# kernel mode (--kernel): only the chain's kernels, timed by their own dispatch events (no marker packets between
# them, so the gaps are the real launch / queue hand-off latencies); default: every labelled op (event records)
KMODE = "--kernel" in sys.argv
PREFIX = "conv_fwd/L7|avgpool|det_fwd|head_rows|head_seq|tail|dir_fwd|dir_pre"
for rep in range(3):
    eng.profile(True, PREFIX if KMODE else "")
    tr.step(x, y)
    torch.cuda.synchronize()
    marks = eng.profile_marks()
    eng.profile(False)
    i0 = [i for i, m_ in enumerate(marks) if m_[0] == "conv_fwd/L7"][0]
    t0 = marks[i0][2]
    print(f"--- rep {rep} (us after the end of conv_fwd/L7) {' '.join(sys.argv[1:])}")
    for lab, a, b in marks[i0 + 1:]:
        print(f"{lab:22s} {1e3 * (a - t0):8.1f} {1e3 * (b - t0):8.1f}  ({1e3 * (b - a):6.1f})")
        if lab == "avgpool_bwd":
            break
