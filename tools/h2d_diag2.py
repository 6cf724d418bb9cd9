"""Input-inclusive leg at config 2: feeding strategies, each tried with copy streams on four consecutive HW queues
(streams are spread over GPU_MAX_HW_QUEUES = 4 queues round robin, so four consecutively created streams cover
them all).  Measurement only (prints one JSON line)."""
import contextlib
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: F401  (installs the vad_amd alias)
import torch
from vad_amd import _native as nat
from vad_amd.cad import CausalAnomalyDetector
from vad_amd.data import ClipStager
from vad_amd.train import CadTrainer, apply_memory_efficient_training

B, T, H, W = 8, 16, 227, 227
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
torch.manual_seed(0)
model = CausalAnomalyDetector()
with contextlib.redirect_stdout(io.StringIO()):
    apply_memory_efficient_training(model)
model = model.to(dev)
tr = CadTrainer(model, lr=3e-4, seed=1234)
pool = []
for i in range(2):
    x = torch.empty(B, T, 1, H, W, device=dev)
    nat.check(nat.lib().vad_synth_frames(7, i, 0, B * T, H * W, 0, x.data_ptr(), nat.stream_of(dev)))
    pool.append(x)
labels = torch.tensor([b % 2 for b in range(B)], dtype=torch.int64, device=dev)
u8 = [torch.randint(0, 256, (B, T, 1, H, W), dtype=torch.uint8).pin_memory() for _ in range(2)]
torch.cuda.synchronize()
res = {}


def timed(name, fn, n=20, warm=3):
    for i in range(warm):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    torch.cuda.synchronize()
    res[name] = round(1e3 * (time.perf_counter() - t0) / n, 4)


timed("pool_ready", lambda i: tr.step(pool[i % 2], labels, inputs_ready=True))


def zero_copy(i):
    """u8 -> fp32 conversion reading the pinned host batch directly (no copy stream)"""
    out = torch.empty(u8[0].shape, dtype=torch.float32, device=dev)
    nat.check(nat.lib().vad_u8_to_clip(u8[i % 2].data_ptr(), u8[0].numel(), 0, out.data_ptr(), nat.stream_of(dev)))
    tr.step(out, labels)


timed("zero_copy", zero_copy)
for q in range(4):
    # three pool streams per q (one here, one per ClipStager): the stream used, 3q mod 4, visits all four HW queues
    sq = torch.cuda.Stream(dev)
    for direct in (True, False):
        st = ClipStager(dev, mode=0, direct=direct)
        st.stream = sq
        hs = [st.issue(u8[0])]

        def waited(i):
            x = st.finish(hs[0])
            hs[0] = st.issue(u8[(i + 1) % 2])
            tr.step(x, labels)

        def unwaited(i):
            x, ready = st.finish(hs[0], wait=False), hs[0].ready
            hs[0] = st.issue(u8[(i + 1) % 2])
            tr.step(x, labels, inputs_ready=ready)

        tag = "direct" if direct else "copy"
        timed(f"q{q}_{tag}_waited", waited)
        timed(f"q{q}_{tag}_unwaited", unwaited)
        st.finish(hs[0])
        torch.cuda.synchronize()
timed("zero_copy_end", zero_copy)
print(json.dumps(res))
