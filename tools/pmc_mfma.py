"""MFMA utilisation per conv kernel family from one rocprofv3 --pmc pass of SQ_VALU_MFMA_BUSY_CYCLES,
SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE (tools/gpu_r2c.sh).

SQ_VALU_MFMA_BUSY_CYCLES counts matrix-core busy cycles summed over every SIMD (32 per v_mfma_f32_32x32x16_bf16,
MI355X_MICROARCH.md § per-instruction constants); GRBM_GUI_ACTIVE is the dispatch's busy cycles summed over the 8
XCDs.  mfma_util = busy / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the fraction of all matrix-core cycles of the chip
during the dispatch that issued MFMA work (1.0 = every SIMD's matrix pipe busy for the whole dispatch).
Usage: python tools/pmc_mfma.py gpurun_out/pmc_mfma > profiles/<round>_pmc_mfma.json
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import family  # noqa: E402

SIMDS = 1024


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))))
    per = collections.defaultdict(dict)
    names = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    fam = collections.defaultdict(lambda: {"launches": 0, "busy": 0.0, "gui": 0.0, "sq_busy": 0.0})
    kern = collections.defaultdict(lambda: {"launches": 0, "busy": 0.0, "gui": 0.0})
    for d, c in per.items():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in c or "GRBM_GUI_ACTIVE" not in c:
            continue
        n = names[d]
        f = family(n) or ("conv1" if ("conv1_kernel" in n or "stem_fused_kernel" in n) else None)
        k = kern[n.split("(")[0][:120]]
        k["launches"] += 1
        k["busy"] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        k["gui"] += c["GRBM_GUI_ACTIVE"]
        if f is None:
            continue
        a = fam[f]
        a["launches"] += 1
        a["busy"] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        a["gui"] += c["GRBM_GUI_ACTIVE"]
        a["sq_busy"] += c.get("SQ_BUSY_CYCLES", 0.0)
    out = {"method": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE (one pass, kernel-trace "
                     "only); mfma_util = MFMA busy cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)",
           "families": {}, "kernels": {}}
    for f, a in sorted(fam.items()):
        out["families"][f] = {"launches": a["launches"], "mfma_util": a["busy"] / (a["gui"] / 8 * SIMDS),
                              "mfma_busy_cycles_per_launch": a["busy"] / a["launches"],
                              "gui_active_cycles_per_launch": a["gui"] / a["launches"]}
    for n, a in sorted(kern.items(), key=lambda kv: -kv[1]["busy"]):
        if a["busy"] > 0:
            out["kernels"][n] = {"launches": a["launches"], "mfma_util": a["busy"] / (a["gui"] / 8 * SIMDS)}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
