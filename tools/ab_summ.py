"""Summarise an A/B of tools/gpu_r4_ab.sh: ms/step per arm and config (mean of the reps)."""
import glob
import json
import sys

tag = sys.argv[1]
for cfg in ("2", "4"):
    for arm in ("A", "B"):
        v = []
        for f in sorted(glob.glob(f"gpurun_out/{tag}_c{cfg}_{arm}_*.json")):
            try:
                v.append(json.load(open(f))["ms_per_step"])
            except Exception:
                pass
        if v:
            print(f"cfg{cfg} {arm}: {sum(v) / len(v):.4f} ms  {v}")
