"""Summarise a bench.py --breakdown-out JSON: per-family totals and per-layer conv times with TFLOP/s."""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from bench import conv_shapes  # noqa: E402

d = json.load(open(sys.argv[1]))["per_label_ms"]
B, T, H, W = 8, 16, 227, 227
cs = conv_shapes(B, T, H, W)
fam = {}
for k, (ms, n) in d.items():
    f = k.split("/L")[0]
    fam[f] = fam.get(f, 0) + ms
print("total %.1f us" % (1e3 * sum(fam.values())))
for k, v in sorted(fam.items(), key=lambda x: -x[1]):
    print(f"  {k:16s} {v * 1e3:8.1f} us")
for k, (ms, n) in d.items():
    if k.startswith("conv_"):
        NF, ci, co, oh, ow = cs[int(k.split("/L")[1])]
        fl = 2.0 * NF * oh * ow * co * ci * 9
        print(f"  {k:16s} {ms * 1e3:7.1f} us  {fl / (ms * 1e-3) / 1e12:6.1f} TF")
