"""CPU checks of the mask-pinning helpers the GPU gradient tests rely on (tests/golden_util.py, oracle stem_pins)."""
import numpy as np
import torch
import torch.nn.functional as F

from oracle import cad_oracle as co
from tests.golden_util import first_max_pool_idx


def test_first_max_pool_idx_matches_torch_with_ties():
    """The window maxima rule used to pin MaxPool2d(3, 2, 1) equals torch's (first max, padding never wins),
    including ties at zero (after ReLU) and at positive values; odd and even plane sizes."""
    g = torch.Generator().manual_seed(0)
    for H, W in [(9, 11), (114, 114), (8, 8), (5, 2)]:
        z = torch.relu(torch.randn(2, 5, H, W, generator=g))
        z[0, 0, :3, :2] = 0.0
        z[1, 1, 1, 0] = z[1, 1, 1, 1] = 5.0
        out, idx = F.max_pool2d(z, 3, 2, 1, return_indices=True)
        mine = first_max_pool_idx(z.permute(0, 2, 3, 1).numpy())
        np.testing.assert_array_equal(mine, idx.permute(0, 2, 3, 1).numpy())


def test_stem_pins_reproduce_unpinned_forward_and_backward():
    """backbone_forward(stem_pins=...) with the pins taken from the same float64 forward is the unpinned stem:
    identical features and identical conv1 / bn1 gradients."""
    torch.manual_seed(3)
    from vad_amd.cad import CausalAnomalyDetector
    sd = CausalAnomalyDetector().state_dict()
    p = {k: v.double().requires_grad_(True) for k, v in sd.items() if "running" not in k and "num_batches" not in k}
    x = co.synth_clips(1, 0, 0, 1, 2, 40, 36).double()
    outs = []
    for pinned in (False, True):
        bufs = {k: v.double().clone() for k, v in sd.items() if "running" in k}
        pins = None
        if pinned:
            with torch.no_grad():
                h = F.conv2d(x.reshape(2, 1, 40, 36), p["backbone.conv1.weight"], p["backbone.conv1.bias"], 2, 3)
                h = F.batch_norm(h, None, None, p["backbone.bn1.weight"], p["backbone.bn1.bias"], True)
                z = torch.relu(h)
                pins = (h > 0, torch.from_numpy(first_max_pool_idx(z.permute(0, 2, 3, 1).numpy())).permute(0, 3, 1, 2))
        f = co.backbone_forward(p, bufs, x, True, stem_pins=pins)
        gw, gb = torch.autograd.grad(f.square().sum(), [p["backbone.conv1.weight"], p["backbone.bn1.weight"]])
        outs.append((f.detach(), gw, gb))
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=1e-12, atol=1e-12)
