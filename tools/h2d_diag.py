"""Diagnose the input-inclusive (H2D) leg of bench.py at config 2: step time of several input-feeding variants in one
process, each after its own warm-up.  Measurement only (prints one JSON line)."""
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
for kv in sys.argv[1:]:
    k, v = kv.split("=")
    nat.check(nat.lib().vad_set_tuning(k.encode(), int(v)))
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
torch.cuda.synchronize()
res = {}


def timed(name, fn, n=20, warm=3):
    for i in range(warm):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    te = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    res[name] = {"ms": round(1e3 * (t1 - t0) / n, 4), "host_ms": round(1e3 * (te - t0) / n, 4)}


timed("pool_ready", lambda i: tr.step(pool[i % 2], labels, inputs_ready=True))
timed("pool_plain", lambda i: tr.step(pool[i % 2], labels))


def fresh(i):
    x = torch.empty_like(pool[i % 2])
    x.copy_(pool[i % 2])
    tr.step(x, labels)


timed("fresh_dev_copy", fresh)
u8 = [torch.randint(0, 256, (B, T, 1, H, W), dtype=torch.uint8).pin_memory() for _ in range(2)]
u8d = [u.to(dev) for u in u8]
torch.cuda.synchronize()


def conv_only(i):
    out = torch.empty(u8d[0].shape, dtype=torch.float32, device=dev)
    nat.check(nat.lib().vad_u8_to_clip(u8d[i % 2].data_ptr(), u8d[0].numel(), 0, out.data_ptr(), nat.stream_of(dev)))
    tr.step(out, labels)


timed("u8_convert_no_copy", conv_only)
st = ClipStager(dev, mode=0)
h = [st.issue(u8[0])]


def h2d(i):
    x = st.finish(h[0])
    h[0] = st.issue(u8[(i + 1) % 2])
    tr.step(x, labels)


timed("h2d", h2d)
timed("h2d_long", h2d, n=40)


def copy_same_stream(i):
    d = u8d[i % 2]
    d.copy_(u8[i % 2], non_blocking=True)
    out = torch.empty(d.shape, dtype=torch.float32, device=dev)
    nat.check(nat.lib().vad_u8_to_clip(d.data_ptr(), d.numel(), 0, out.data_ptr(), nat.stream_of(dev)))
    tr.step(out, labels)


timed("h2d_same_stream", copy_same_stream)
cs = torch.cuda.Stream(dev)
ev_c = [torch.cuda.Event(), torch.cuda.Event()]
ev_r = [torch.cuda.Event(), torch.cuda.Event()]


def variant(i, wait_copy, wait_read, pin_check=False):
    """batch i+1's copy on the side stream (optionally after slot's read event); batch i converted on the current
    stream (optionally after its copy event)"""
    k, n = i % 2, (i + 1) % 2
    if pin_check:
        assert u8[n].is_pinned()
    cur = torch.cuda.current_stream(dev)
    if wait_copy:
        cur.wait_event(ev_c[k])
    out = torch.empty(u8d[0].shape, dtype=torch.float32, device=dev)
    nat.check(nat.lib().vad_u8_to_clip(u8d[k].data_ptr(), u8d[0].numel(), 0, out.data_ptr(), nat.stream_of(dev)))
    ev_r[k].record(cur)
    if wait_read:
        cs.wait_event(ev_r[n])
    with torch.cuda.stream(cs):
        u8d[n].copy_(u8[n], non_blocking=True)
        ev_c[n].record(cs)
    tr.step(out, labels)


for wc in (0, 1):
    for wr in (0, 1):
        timed(f"side_copy_waitcopy{wc}_waitread{wr}", lambda i: variant(i, wc, wr))
timed("side_copy_waits_is_pinned", lambda i: variant(i, 1, 1, True))
for j in range(5):  # consecutive copy streams land on consecutive HW queues (round robin)
    st = ClipStager(dev, mode=0)
    h = [st.issue(u8[0])]
    timed(f"h2d_stager{j}", h2d)
    st.finish(h[0])
    torch.cuda.synchronize()
for prio in (-1, 0):
    st = ClipStager(dev, mode=0)
    st.copy_stream = torch.cuda.Stream(dev, priority=prio)
    h = [st.issue(u8[0])]
    timed(f"h2d_stager_prio{prio}", h2d)
    st.finish(h[0])
    torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(100):
    u8[0].is_pinned()
res["is_pinned_us"] = round(1e6 * (time.perf_counter() - t0) / 100, 2)


def copy_only_side(i):
    with torch.cuda.stream(cs):
        u8d[i % 2].copy_(u8[i % 2], non_blocking=True)
    tr.step(pool[i % 2], labels, inputs_ready=True)


timed("pool_ready_plus_side_h2d", copy_only_side)
with torch.no_grad():
    tr.eng.forward(pool[0], False, 0, 0, 0, None)
torch.cuda.synchronize()
timed("h2d_after_eval", h2d)
timed("pool_ready_after_eval", lambda i: tr.step(pool[i % 2], labels, inputs_ready=True))
st.finish(h[0])
torch.cuda.synchronize()
# the bare copy: pinned u8 batch -> device, back to back (GB/s), on the side stream and on the current one
nb = u8[0].numel()
for name, s in (("copy_side", cs), ("copy_current", torch.cuda.current_stream(dev))):
    with torch.cuda.stream(s):
        for i in range(3):
            u8d[i % 2].copy_(u8[i % 2], non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(20):
            u8d[i % 2].copy_(u8[i % 2], non_blocking=True)
        te = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    res[name] = {"ms": round(1e3 * (t1 - t0) / 20, 4), "host_ms": round(1e3 * (te - t0) / 20, 4),
                 "GB/s": round(nb * 20 / (t1 - t0) / 1e9, 2)}
big = torch.empty(8 * nb, dtype=torch.uint8).pin_memory()
bigd = torch.empty(8 * nb, dtype=torch.uint8, device=dev)
bigd.copy_(big)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(5):
    bigd.copy_(big, non_blocking=True)
torch.cuda.synchronize()
res["copy_53MB"] = {"GB/s": round(5 * 8 * nb / (time.perf_counter() - t0) / 1e9, 2)}
pg = torch.empty(nb, dtype=torch.uint8)
t0 = time.perf_counter()
for i in range(10):
    u8d[0].view(-1).copy_(pg)
torch.cuda.synchronize()
res["copy_pageable"] = {"GB/s": round(10 * nb / (time.perf_counter() - t0) / 1e9, 2)}
print(json.dumps(res))
