"""Per-family average launch duration from a rocprofv3 --stats kernel summary (to check bench.py's live HIP-event
roofline timing against the committed profile).  Usage: python tools/family_stats.py <run_kernel_stats.csv>"""
import csv
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from tools.pmc_traffic import family  # noqa: E402

agg = {}
for r in csv.DictReader(open(sys.argv[1])):
    f = family(r["Name"])
    if f is None:
        continue
    a = agg.setdefault(f, {"calls": 0, "total_ns": 0.0})
    a["calls"] += int(r["Calls"])
    a["total_ns"] += float(r["TotalDurationNs"])
out = {f: {"calls": a["calls"], "avg_launch_us": round(a["total_ns"] / a["calls"] / 1e3, 2)} for f, a in agg.items()}
json.dump(out, sys.stdout, indent=1)
