"""Print an A/B run (tools/ab_knob.sh / ab_so.sh logs) and, optionally, per-label deltas of two breakdown files."""
import glob, json, statistics, sys

tag = sys.argv[1]
for v in "AB":
    ms = [json.loads(open(f).read().strip().split("\n")[-1])["ms_per_step"] for f in sorted(glob.glob(f"gpurun_out/{tag}_{v}_*.log"))]
    print(v, statistics.median(ms) if ms else None, ms)
if len(sys.argv) > 3:
    a = json.load(open(sys.argv[2]))["per_label_ms"]
    b = json.load(open(sys.argv[3]))["per_label_ms"]
    for k in a:
        if k in b and any(s in k for s in sys.argv[4:] or [""]):
            print(f"{k:26s} {a[k][0] * 1000:8.1f} -> {b[k][0] * 1000:8.1f}")
