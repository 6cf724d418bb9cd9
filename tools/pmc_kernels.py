"""Per-kernel averages of every counter in one or more rocprofv3 --pmc runs (run_counter_collection.csv), joined on
kernel name.  Usage: python tools/pmc_kernels.py <dir> [<dir> ...] [--match SUBSTR]"""
import csv
import os
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
if match in args:
    args.remove(match)
agg = {}
for d in args:
    per = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = (r["Kernel_Name"], r["Dispatch_Id"])
        per.setdefault(k, {})[r["Counter_Name"]] = per.get(k, {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for (name, _), cs in per.items():
        a = agg.setdefault(name, {})
        for c, v in cs.items():
            s = a.setdefault(c, [0.0, 0])
            s[0] += v
            s[1] += 1
for name, cs in sorted(agg.items()):
    if match not in name:
        continue
    avg = {c: s[0] / s[1] for c, s in cs.items()}
    out = []
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        out.append(f"mfma_busy={avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
    if "SQ_INSTS_VALU" in avg and "SQ_INSTS_MFMA" in avg and avg["SQ_INSTS_MFMA"] > 0:
        out.append(f"valu/mfma={(avg['SQ_INSTS_VALU'] - avg['SQ_INSTS_MFMA']) / avg['SQ_INSTS_MFMA']:.2f}")
        out.append(f"lds/mfma={avg['SQ_INSTS_LDS'] / avg['SQ_INSTS_MFMA']:.2f}")
    if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_LDS_IDX_ACTIVE", 0) > 0:
        out.append(f"bank_conf={avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE']:.3f}")
    if "FETCH_SIZE" in avg:
        out.append(f"fetch_MB={avg['FETCH_SIZE'] / 1024:.1f}")
    if "WRITE_SIZE" in avg:
        out.append(f"write_MB={avg['WRITE_SIZE'] / 1024:.1f}")
    if "SQ_WAIT_INST_ANY" in avg and avg.get("SQ_WAVE_CYCLES", 0) > 0:
        for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM",
                  "SQ_WAIT_INST_LDS"):
            out.append(f"{c[3:].lower()}={avg[c] / avg['SQ_WAVE_CYCLES']:.3f}")
    print(name[:90], " ".join(out))
