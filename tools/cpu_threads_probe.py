"""Probe of the GPU box's host: CPU count, affinity, cgroup quota, and the CPU oracle step (config 2) at several
thread counts -- picks the thread count of bench.py's cpu_baseline leg."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle import cad_oracle as co
info = {"os_cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
    if os.path.exists(p):
        info[p] = open(p).read().strip()
torch.manual_seed(0)
from vad_amd.cad import CausalAnomalyDetector
sd = {k: v.clone() for k, v in CausalAnomalyDetector().state_dict().items()}
params = {k: v for k, v in sd.items() if "running" not in k and "num_batches" not in k}
bufs = {k: v for k, v in sd.items() if "running" in k}
B, T, H, W = 8, 16, 227, 227
x = co.synth_clips(7, 0, 0, B, T, H, W)
y = co.synth_labels(0, B)
res = {}
for th in [int(a) for a in sys.argv[1:]] or [16, 32, 64, os.cpu_count()]:
    torch.set_num_threads(th)
    co.cad_train_step(params, bufs, {}, x, y, co.CadDraws.make(1, 0, 0, B, T))
    t0 = time.perf_counter(); n = 0
    while time.perf_counter() - t0 < 6 and n < 20:
        co.cad_train_step(params, bufs, {}, x, y, co.CadDraws.make(1, n + 1, 0, B, T)); n += 1
    res[th] = round(B * n / (time.perf_counter() - t0), 3)
    print(th, res[th], flush=True)
info["clips_per_s_by_threads"] = res
print(json.dumps(info))
