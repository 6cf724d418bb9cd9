"""Debug: which gradient slots differ between a second backward on one forward and a fresh forward + backward."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from oracle import cad_oracle as co
from tests.golden_util import cad_cases, make_cad_model
from vad_amd import _native as nat

for gate in (1, 0):
    nat.check(nat.lib().vad_set_tuning(b"cad_det_gate", gate))
    case = cad_cases()[1]
    m = make_cad_model(case).cuda()
    eng = m.engine()
    B, T, H, W = case["B"], case["T"], case["H"], case["W"]
    x = co.synth_clips(case["seed"], case["step"], 0, B, T, H, W).cuda()
    g = torch.Generator().manual_seed(5)
    ups = [(torch.randn(B, generator=g).cuda(), torch.randn(B, 2, generator=g).cuda()) for _ in range(2)]
    eng.forward(x, True, case["seed"], case["step"], 0)
    shared = []
    for dc, dp in ups:
        eng.backward(False, d_causal=dc, d_probs=dp)
        torch.cuda.synchronize()
        shared.append(eng.grads.clone())
    fresh = []
    for dc, dp in ups:
        eng.forward(x, True, case["seed"], case["step"], 0)
        eng.backward(False, d_causal=dc, d_probs=dp)
        torch.cuda.synchronize()
        fresh.append(eng.grads.clone())
    for k in range(2):
        bad = []
        for i, n in enumerate(eng.slot_names):
            o, c = eng.slot_offset[i], eng.slot_numel[i]
            d = (shared[k][o:o + c] - fresh[k][o:o + c]).abs().max().item()
            if d > 0:
                bad.append((n, d, fresh[k][o:o + c].abs().max().item()))
        print("gate", gate, "backward", k, "differing slots:", bad[:12], "of", len(bad), flush=True)
