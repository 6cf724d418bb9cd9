"""Print one train step's kernel timeline from a rocprofv3 kernel trace (durations, gaps, grids) and per-kernel
totals.  Usage: python tools/timeline.py gpurun_out/<dir>/run_kernel_trace.csv [step_end_kernel]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
end_k = sys.argv[2] if len(sys.argv) > 2 else "adamw_kernel"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if end_k in r["Kernel_Name"]]
a, b = ends[-2], ends[-1]
prev = None
t0 = int(rows[a + 1]["Start_Timestamp"])
qcol = "Queue_Id" if "Queue_Id" in rows[0] else None
tot = collections.Counter()
busy = 0
for r in rows[a + 1:b + 1]:
    n = re.sub(r"\(.*", "", r["Kernel_Name"])[:80]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    prev = e
    busy += e - s
    tot[n] += (e - s) / 1e3
    q = r[qcol] if qcol else "?"
    print(f"t={(s - t0) / 1e3:7.1f} q{q:>2} {(e - s) / 1e3:7.1f} gap{gap:6.1f} g={r['Grid_Size_X']}x{r['Grid_Size_Y']} {n}")
span = int(rows[b]["End_Timestamp"]) - int(rows[a + 1]["Start_Timestamp"])
print(f"step span {span / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us, launches {b - a}")
