"""Host-side enqueue time of one train step (config 2): forward / backward / optimizer calls without synchronising,
against the GPU step time -- is the host on the critical path?"""
import os, sys, time, io, contextlib
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vad_amd import _native as nat
from vad_amd.cad import CausalAnomalyDetector
from vad_amd.train import CadTrainer, apply_memory_efficient_training
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
tf, tb, to = [], [], []
t00 = time.perf_counter()
for _ in range(30):
    a = time.perf_counter()
    eng.forward(x, True, 1, 0, 0, y, want_outputs=False)
    b = time.perf_counter()
    eng.backward(True)
    c = time.perf_counter()
    eng.optimizer_step(3e-4)
    d = time.perf_counter()
    tf.append(b - a); tb.append(c - b); to.append(d - c)
torch.cuda.synchronize()
el = time.perf_counter() - t00
med = lambda v: sorted(v)[len(v) // 2] * 1e6
print(f"host us per call: forward {med(tf):.0f}  backward {med(tb):.0f}  optimizer {med(to):.0f}; "
      f"wall per step {el / 30 * 1e6:.0f} us")
