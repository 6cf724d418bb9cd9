"""Per-arm step time and per-layer conv kernel times (live HIP events) of an A/B (tools/ab_knob.sh / ab_so.sh logs).
usage: python tools/ab_layers.py TAG [family-substring ...]"""
import glob
import json
import statistics
import sys

tag = sys.argv[1]
want = sys.argv[2:]
arms = {}
for v in "AB":
    runs = []
    for f in sorted(glob.glob(f"gpurun_out/{tag}_{v}_*.log")):
        try:
            runs.append(json.loads(open(f).read().strip().split("\n")[-1]))
        except Exception:
            pass
    arms[v] = runs
for v, runs in arms.items():
    ms = [r["ms_per_step"] for r in runs]
    print(v, "ms/step median", statistics.median(ms) if ms else None, ms)
keys = set()
for runs in arms.values():
    for r in runs:
        for fam in r["roofline"]["families"].values():
            keys.update(fam["per_layer_us"])
for k in sorted(keys):
    if want and not any(w in k for w in want):
        continue
    row = []
    for v, runs in arms.items():
        xs = [fam["per_layer_us"][k] for r in runs for fam in r["roofline"]["families"].values()
              if k in fam["per_layer_us"]]
        row.append(f"{statistics.median(xs):7.2f}" if xs else "    -  ")
    print(f"{k:18s} " + "  ".join(row))
