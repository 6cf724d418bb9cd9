"""Summarise an A/B run of tools/ab_so.sh (gpurun_out/TAG_{A,B}_k.log) into one JSON object."""
import glob, json, statistics, sys

tag, note = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
out = {"tag": tag, "note": note}
for v in "AB":
    runs = []
    for f in sorted(glob.glob(f"gpurun_out/{tag}_{v}_*.log")):
        d = json.loads(open(f).read().strip().split("\n")[-1])
        runs.append({"value": d["value"], "ms_per_step": d["ms_per_step"], "post_backbone_us": d.get("post_backbone_us")})
    out[v] = {"runs": runs, "median_ms": statistics.median(r["ms_per_step"] for r in runs)}
print(json.dumps(out, indent=1))
