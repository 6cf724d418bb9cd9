"""Instruction mix of the MFMA loop of kernels in a device .s file (hipcc -S --cuda-device-only): for each kernel whose
symbol contains SUBSTR, the loop (by the assembler's 'Loop Header' comments) holding the most MFMAs, counted by class.
Usage: python tools/loopmix.py file.s SUBSTR [SUBSTR ...]"""
import re
import sys

L = open(sys.argv[1]).read().split("\n")
subs = sys.argv[2:]
starts = [i for i, l in enumerate(L) if re.match(r"^_Z\w+:", l)]
for a in starts:
    name = L[a][:-1]
    if not any(s in name for s in subs):
        continue
    b = next(i for i in range(a, len(L)) if L[i].startswith(".Lfunc_end"))
    seg = L[a:b]
    heads = {}
    for i, l in enumerate(seg):
        m = re.match(r"^\.LBB(\d+_\d+):.*Loop Header", l)
        if m:
            heads[m.group(1)] = [i]
    for i, l in enumerate(seg):
        m = re.search(r"in Loop: Header=BB(\d+_\d+)", l)
        if m and m.group(1) in heads:
            heads[m.group(1)].append(i)
    best = None
    for h, idx in heads.items():
        lo, hi = min(idx), max(idx)
        nxt = [i for i, l in enumerate(seg) if i > hi and re.match(r"^\.LBB\d+_\d+:", l)]
        hi = nxt[0] if nxt else len(seg)
        cnt = {}
        for l in seg[lo:hi]:
            t = l.strip().split(" ")[0]
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            k = ("mfma" if "mfma" in t else "valu" if t.startswith("v_") else "ds" if t.startswith("ds_")
                 else "salu" if t.startswith("s_") else "vmem")
            cnt[k] = cnt.get(k, 0) + 1
        if best is None or cnt.get("mfma", 0) > best.get("mfma", 0):
            best = cnt
    if best:
        print(f"{name[:100]} {best} valu/mfma={best.get('valu', 0) / max(1, best.get('mfma', 0)):.2f}")
