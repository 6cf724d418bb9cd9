"""Stand-alone timing of the BN-backward apply pass (vad_bn_bwd_apply) at the config-2 (fp32) and config-4 (bf16)
layer shapes under knob variants; checks every variant against the default bit for bit.  GPU only."""
import json
import sys

import torch

sys.path.insert(0, ".")
import vad_amd._native as nat  # noqa: E402

lib = nat.lib()
d = torch.device("cuda")
st = nat.stream_of(d)
SHAPES = {"cfg2": (128, [(57, 32), (29, 64), (15, 128), (8, 256)], False),
          "cfg4": (256, [(64, 32), (32, 64), (16, 128), (8, 256)], True)}
VARIANTS = [dict(), dict(bn_apply_u=8), dict(bn_apply_u=2), dict(bn_apply_blocks=1024), dict(bn_apply_blocks=4096),
            dict(bn_apply_blocks=512)]


DEF = dict(bn_apply_u=4, bn_apply_blocks=2048)


def setk(kv):
    for k, v in {**DEF, **kv}.items():
        nat.check(lib.vad_set_tuning(k.encode(), v))


out = {}
g = torch.Generator(device="cpu").manual_seed(0)
for cfg, (NF, layers, bf) in SHAPES.items():
    dt = torch.bfloat16 if bf else torch.float32
    for (HW, C) in layers:
        M = NF * HW * HW
        dA = torch.randn(M, C, generator=g).to(d, dt)
        y = torch.randn(M, C, generator=g).to(d, dt)
        stats = torch.cat([torch.randn(C, generator=g) * 0.1, torch.rand(C, generator=g) + 0.5,
                           torch.randn(C, generator=g), torch.randn(C, generator=g) * 0.1,
                           torch.rand(C, generator=g), torch.randn(C, generator=g) * 1e-3,
                           torch.randn(C, generator=g) * 1e-3]).to(d)
        nbytes = 3 * M * C * (2 if bf else 4)
        ref = None
        for kv in VARIANTS:
            setk(kv)
            dY = torch.empty(M, C, device=d, dtype=dt)
            run = lambda: nat.check(lib.vad_bn_bwd_apply(dA.data_ptr(), y.data_ptr(), stats.data_ptr(), M, C,
                                                          dY.data_ptr(), 1 if bf else 0, st))
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 20
            e0.record()
            for _ in range(n):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / n
            if ref is None:
                ref = dY.clone()
            same = bool(torch.equal(ref, dY))
            key = f"{cfg}/{HW}x{HW}x{C}/" + (",".join(f"{k}={v}" for k, v in kv.items()) or "default")
            out[key] = {"us": round(us, 2), "TBps": round(nbytes / us / 1e6, 2), "bit_identical": same}
            print(key, out[key], flush=True)
setk({})
json.dump(out, open("gpurun_out/apply_bench.json", "w"), indent=1)
