"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage remarks: VGPR / AGPR / scratch / occupancy / LDS per kernel."""
import re
import subprocess
import sys

txt = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cur = {}
rows = []
for line in txt.splitlines():
    for key, pat in (("name", r"Function Name: (\S+)"), ("v", r"VGPRs: (\d+)"), ("a", r"AGPRs: (\d+)"),
                     ("scr", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            if key == "name" and cur:
                rows.append(cur)
                cur = {}
            cur[key] = m.group(1)
if cur:
    rows.append(cur)
for r in rows:
    n = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip().replace("vad::", "")
    n = re.sub(r"\(.*Args\)", "", n).replace("void ", "")
    if flt and flt not in n:
        continue
    print(f"{n:70s} V{r.get('v','?'):>4} A{r.get('a','?'):>4} scr{r.get('scr','?'):>4} occ{r.get('occ','?')} lds{r.get('lds','?')}")
