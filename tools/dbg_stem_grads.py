"""Debug: gradients of the frozen-stem step with the fused stem on vs off (knob stem_fused), per tensor."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import cad_oracle as co
from tests.golden_util import make_cad_model, read_debug
from vad_amd import _native as nat
from vad_amd.train import apply_memory_efficient_training

case = dict(name="dbg", B=2, T=4, H=64, W=64, seed=3, step=0, forced=None)
x = co.synth_clips(3, 0, 0, 2, 4, 64, 64).cuda()
y = co.synth_labels(0, 2).cuda()
res = {}
for fused in (1, 0):
    nat.check(nat.lib().vad_set_tuning(b"stem_fused", fused))
    m = make_cad_model(case)
    apply_memory_efficient_training(m)
    m = m.cuda()
    eng = m.engine()
    o = eng.forward(x, True, 3, 0, 0, y)
    eng.backward(True)
    torch.cuda.synchronize()
    res[fused] = (eng.grads.cpu().numpy().copy(), o["final"].cpu().numpy().copy(),
                  read_debug(eng._last[0], "pool"), read_debug(eng._last[0], "stats", 0))
nat.check(nat.lib().vad_set_tuning(b"stem_fused", 1))
print("final", res[1][1], res[0][1])
for i, n in enumerate(eng.slot_names[:12]):
    a = res[1][0][eng.slot_offset[i]:eng.slot_offset[i] + eng.slot_numel[i]]
    b = res[0][0][eng.slot_offset[i]:eng.slot_offset[i] + eng.slot_numel[i]]
    print(n, float(np.abs(a).max()), float(np.abs(b).max()), float(np.abs(a - b).max()))
