"""Summarise two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; tools/gpu_prof.sh) into HBM bytes per launch for
the conv kernel families that bench.py can name as dominant.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports
half the bytes of 16-B-per-lane streaming reads (all conv kernels stage with 16-B loads), so it is doubled;
WRITE_SIZE is exact for 16-B stores and taken as is for the 4-B epilogue stores (uncalibrated, noted).
Usage: python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write [MARKER PER_STEP]
            > profiles/<round>_cfg<N>_pmc_traffic.json
MARKER / PER_STEP: a kernel-name substring launched PER_STEP times per bench step; with them the summary also
carries the whole step's HBM bytes (every kernel of the run / the number of steps).
"""
import collections
import csv
import json
import os
import sys


def _targs(name):
    """Template arguments of a demangled kernel name, e.g. 'k<1, 2, true, 3>(...)' -> ['1', '2', 'true', '3']."""
    a = name.find("<")
    b = name.find(">", a)
    return [t.strip() for t in name[a + 1:b].split(",")] if a >= 0 and b > a else []


def family(name):
    if "conv3x3_wgrad_patch_kernel" in name or ("gemm_kernel" in name and "ConvPatchKM" in name):
        return "conv_wgrad"
    if ("conv3x3_wgrad_x3_kernel" in name or "conv3x3_wgrad_x3nt_kernel" in name or "x3_wgrad_tr_kernel" in name
            or "bfc_wgrad_kernel" in name):
        return "conv_wgrad"
    if "bfc_conv_kernel" in name:  # <S, NI, TH, TW, CB, NCT, FWD, WRES>
        return "conv_fwd" if _targs(name)[6:7] == ["true"] else "conv_dgrad"
    if "bfc_dgrad_s2_kernel" in name:
        return "conv_dgrad"
    if "conv3x3_x3_kernel" in name:  # <S, NI, TH, TW, NT, PC, FWD, NP>
        return "conv_fwd" if _targs(name)[6:7] == ["true"] else "conv_dgrad"
    if "conv3x3_patch_kernel" in name:
        return "conv_fwd" if "true" in _targs(name) else "conv_dgrad"
    if "conv3x3_x3ws_kernel" in name:  # <NI, TH, TW, PC, FWD, ...>
        return "conv_fwd" if _targs(name)[4:5] == ["true"] else "conv_dgrad"
    if "conv3x3_dgrad_s2x3_kernel" in name:
        return "conv_dgrad"
    if "conv3x3_dgrad_s2_kernel" in name or ("gemm_kernel" in name and "EpiConvDgrad" in name):
        return "conv_dgrad"
    if "gemm_kernel" in name and "EpiConvFwd" in name:
        return "conv_fwd"
    return None


def per_kernel(path, counter):
    rows = [r for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv")))
            if r["Counter_Name"] == counter]
    return {int(r["Dispatch_Id"]): (r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0) for r in rows}


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    fam = collections.defaultdict(lambda: {"launches": 0, "fetch": 0.0, "write": 0.0})
    tot = {"fetch": 0.0, "write": 0.0}
    kern = collections.defaultdict(lambda: {"launches": 0, "bytes": 0.0})
    # the two passes ran the same program: pair dispatches by kernel name in order
    wq = collections.defaultdict(list)
    for d in sorted(write):
        wq[write[d][0]].append(write[d][1])
    used = collections.Counter()
    for d in sorted(fetch):
        name, fb = fetch[d]
        f = family(name)
        k = used[name]
        used[name] += 1
        if k >= len(wq[name]):
            continue
        tot["fetch"] += 2.0 * fb
        tot["write"] += wq[name][k]
        kn = kern[name.split("(")[0][:110]]
        kn["launches"] += 1
        kn["bytes"] += 2.0 * fb + wq[name][k]
        if f is None:
            continue
        a = fam[f]
        a["launches"] += 1
        a["fetch"] += 2.0 * fb
        a["write"] += wq[name][k]
    out = {"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, --kernel-trace only); "
                     "FETCH_SIZE doubled (gfx950 16-B/lane reads), KiB -> bytes",
           "families": {}}
    for f, a in sorted(fam.items()):
        n = a["launches"]
        out["families"][f] = {"launches": n, "hbm_bytes_per_launch": (a["fetch"] + a["write"]) / n,
                              "read_bytes_per_launch": a["fetch"] / n, "write_bytes_per_launch": a["write"] / n}
    if len(sys.argv) > 4:
        marker, per_step = sys.argv[3], int(sys.argv[4])
        n = sum(1 for d in fetch.values() if marker in d[0])
        steps = n / per_step
        out["step"] = {"steps": steps, "hbm_bytes_per_step": (tot["fetch"] + tot["write"]) / steps,
                       "read_bytes_per_step": tot["fetch"] / steps, "write_bytes_per_step": tot["write"] / steps,
                       "basis": f"all kernels of the run / ({n} launches of '{marker}' / {per_step} per step)"}
        out["kernels_by_bytes_per_step"] = {k: {"launches_per_step": v["launches"] / steps,
                                                "bytes_per_step": v["bytes"] / steps}
                                            for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["bytes"])[:25]}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
