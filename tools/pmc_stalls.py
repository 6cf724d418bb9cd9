"""Where the waves of each kernel spend their cycles, from two rocprofv3 --pmc passes (tools/gpu_r2f.sh):
pass A  SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
        SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS
pass B  SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
        SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue stall) + SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES
(MI355X_MICROARCH.md § rocprofv3 PMC slots).  Prints per kernel (summed over its dispatches) the fractions of wave
cycles and the instruction mix per wave.
Usage: python tools/pmc_stalls.py gpurun_out/pmc_stallA gpurun_out/pmc_stallB > profiles/<tag>_pmc_stalls.json
"""
import collections
import csv
import json
import os
import sys


def load(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        name = r["Kernel_Name"].split("(")[0][:140]
        per[name][r["Counter_Name"]] += float(r["Counter_Value"])
        per[name]["_dispatches"] += 0  # touched
    # dispatch counts
    seen = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        seen[r["Kernel_Name"].split("(")[0][:140]].add(r["Dispatch_Id"])
    for k, v in seen.items():
        per[k]["_dispatches"] = len(v)
    return per


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    out = {}
    for k in a:
        A, B = a[k], b.get(k, {})
        wc = A.get("SQ_WAVE_CYCLES", 0.0)
        if wc <= 0:
            continue
        d = {"dispatches": int(A["_dispatches"]),
             "wait_any": A.get("SQ_WAIT_ANY", 0) / wc, "wait_inst_any": A.get("SQ_WAIT_INST_ANY", 0) / wc,
             "active_any": A.get("SQ_ACTIVE_INST_ANY", 0) / wc, "active_valu": A.get("SQ_ACTIVE_INST_VALU", 0) / wc,
             "active_lds": A.get("SQ_ACTIVE_INST_LDS", 0) / wc, "active_vmem": A.get("SQ_ACTIVE_INST_VMEM", 0) / wc,
             "wait_inst_lds": A.get("SQ_WAIT_INST_LDS", 0) / wc}
        if B:
            waves = max(1.0, B.get("SQ_INSTS_MFMA", 0))
            d.update({"valu_per_mfma": B.get("SQ_INSTS_VALU", 0) / waves, "lds_per_mfma": B.get("SQ_INSTS_LDS", 0) / waves,
                      "vmem_rd_per_mfma": B.get("SQ_INSTS_VMEM_RD", 0) / waves,
                      "lds_bank_conflict_frac": B.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, B.get("SQ_LDS_IDX_ACTIVE", 0)),
                      "mfma_util": B.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1.0, B.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024)})
        out[k] = {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in d.items()}
    json.dump(dict(sorted(out.items(), key=lambda kv: -a[kv[0]].get("SQ_WAVE_CYCLES", 0))), sys.stdout, indent=1)


if __name__ == "__main__":
    main()
