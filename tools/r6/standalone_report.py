"""Summarise tools/r6/gpu_standalone_ab.sh output: median us per (layer, op) per tag."""
import collections
import json
import statistics
import sys

rows = collections.defaultdict(list)
for line in open(f"gpurun_out/{sys.argv[1]}_standalone.jsonl"):
    r = json.loads(line)
    rows[(r["layer"], r["op"], r["tag"])].append((r["us"], r["tflops"]))
keys = sorted({(l, o) for l, o, _ in rows})
tags = sorted({t for _, _, t in rows})
for l, o in keys:
    print(f"L{l} {o:5s} " + "  ".join(f"{t}: {statistics.median(u for u, _ in rows[(l, o, t)]):7.2f} us "
                                      f"{statistics.median(f for _, f in rows[(l, o, t)]):6.1f} TF" for t in tags
                                      if (l, o, t) in rows))
