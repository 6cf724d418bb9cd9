"""Golden-vector case table shared by make_golden.py and the tests (data only, no reference code)."""
from __future__ import annotations

import torch

# "forced" detector setting: the reference init (cad:186-192) puts every box out of range so every
# frame falls back to the constant box.  Forcing re-biases the last detector layer to
# logits near the x/y validity thresholds and scales its weights, so that frames carry 1..5 valid
# boxes and the detector / edge-MLP gradients are exercised.
FORCED_A = dict(
    bias=[-3.45, 0.0, 0.0, 0.0,     # det0: x near the low threshold (logit(10/360) = -3.56)
          0.0, 0.0, 0.0, 0.0,       # det1: always valid
          3.3, 0.3, 0.0, 0.0,       # det2: x near the high threshold
          0.5, -2.9, 0.0, 0.0,      # det3: y near the low threshold (logit(10/240) = -3.14)
          -3.58, 2.9, 0.0, 0.0],     # det4: both near thresholds
    weight_scale=6.0,
)


def force_detector(sd: dict, forced: dict) -> None:
    """Apply a forced-detection setting in place to a CausalAnomalyDetector state_dict."""
    with torch.no_grad():
        sd["detector.detector_net.10.bias"].copy_(torch.tensor(forced["bias"], dtype=torch.float32))
        sd["detector.detector_net.10.weight"].mul_(forced["weight_scale"])


CAD_CASES = [
    dict(name="fallback_b2t4_64", B=2, T=4, H=64, W=64, seed=0, step=0, forced=None),
    dict(name="forced_b2t4_64", B=2, T=4, H=64, W=64, seed=1, step=0, forced=FORCED_A),
    dict(name="forced_b3t5_96x80", B=3, T=5, H=96, W=80, seed=2, step=3, forced=FORCED_A),
    dict(name="fallback_b2t16_227", B=2, T=16, H=227, W=227, seed=3, step=0, forced=None),
    # edge shapes: a single clip (batch statistics over T frames only) and single-frame clips (GRU over one step)
    dict(name="forced_b1t3_64", B=1, T=3, H=64, W=64, seed=4, step=1, forced=FORCED_A),
    dict(name="forced_b2t1_64", B=2, T=1, H=64, W=64, seed=5, step=0, forced=FORCED_A),
    # config-2 frame size with live detections (N>1 trajectories, detector and edge-MLP grads)
    dict(name="forced_b2t16_227", B=2, T=16, H=227, W=227, seed=6, step=0, forced=FORCED_A),
]

# minicausal (config 1 family): scale > 1 multiplies the last classifier layer so the pre-clip grad norm exceeds 10
# and StableTrainer's clip branch (mc:304-306) runs
MC_CASES = [
    dict(name="b4t8_32", B=4, T=8, H=32, W=32, seed=10, step=0, scale=1.0),
    dict(name="b8t16_64", B=8, T=16, H=64, W=64, seed=11, step=2, scale=1.0),
    dict(name="clip_b4t8_32x48", B=4, T=8, H=32, W=48, seed=12, step=1, scale=12000.0),
]
# a2 (avenue_training_script2.py): "ckpt" starts from the reference's shipped best_improved_model.pth (stored as
# tests/golden/a2_best_improved_model.npz); seeds/steps chosen so both pseudo-label classes occur (a2:139-141)
A2_CASES = [
    dict(name="ckpt_b4t8_64", B=4, T=8, H=64, W=64, seed=22, step=0, ckpt=True),
    dict(name="ckpt_b6t8_64_pseudo", B=6, T=8, H=64, W=64, seed=21, step=0, ckpt=True),
    dict(name="init_b6t8_48x40_pseudo", B=6, T=8, H=48, W=40, seed=25, step=2, ckpt=False),
]
# bbox clip scorer (config 5): eval mode, one case per clip length of the mixed-T packing
BBOX_CASES = [
    dict(name="t8", B=3, T=8, H=64, W=64, seed=30, step=0),
    dict(name="t16", B=2, T=16, H=64, W=64, seed=31, step=0),
    dict(name="t32_48x56", B=2, T=32, H=48, W=56, seed=32, step=0),
    # a single clip: the reference's .squeeze() returns a 0-d score (bbox:101)
    dict(name="t8_b1", B=1, T=8, H=64, W=64, seed=33, step=0),
]

# cad1 memory autoencoder (causal_anomaly_detection1.py): one epoch of the reference's train_model over the label rows
# (only label-0 clips train, cad1:373-378), its validation pass and calculate_anomaly_scores.  mem: the ring state
# before training, (rows prefilled, memory_ptr) or None -- ptr >= 10 exercises the score, 498 + 3 clips the
# wrap-around of update_memory (cad1:212-219); an all-anomalous first batch exercises the skip.
AE_CASES = [
    dict(name="b4t8", B=4, T=8, seed=40, lr=1e-5, labels=[[0, 0, 1, 0], [0, 0, 0, 0], [0, 1, 0, 0]],
         val_labels=[0, 1, 0], test_labels=[0, 1, 0, 1], mem=None),
    dict(name="b3t5_wrap", B=3, T=5, seed=41, lr=5e-7, labels=[[0, 0, 0], [1, 0, 0]], val_labels=[0, 0],
         test_labels=[1, 0, 0], mem=(500, 498)),
    dict(name="b2t16_skip", B=2, T=16, seed=42, lr=2e-5, labels=[[1, 1], [0, 0]], val_labels=[0, 1],
         test_labels=[0, 1], mem=(20, 20)),
]


# frame-folder tree for the dataset-enumeration fixture (tests/golden/make_dataset_golden.py): folder -> frame count
# (UCSD Ped2 layout: TrainNNN / TestNNN folders of .tif frames, TestNNN_gt folders of .bmp masks)
DATASET_TREE = {
    "Train/Train001": 40, "Train/Train002": 23, "Train/Train003": 16, "Train/Train004": 7,
    "Test/Test001": 50, "Test/Test002": 33, "Test/Test003": 17, "Test/Test004": 64, "Test/Test005": 12,
    "Test/Test011": 45, "Test/Test001_gt": 50,
}


def build_dataset_tree(root, empty=True, frame_hw=(24, 36), seed=0):
    """Create DATASET_TREE under root: empty files (enumeration only) or small random grayscale .tif frames."""
    import os
    import numpy as np
    rs = np.random.default_rng(seed)
    for folder, n in DATASET_TREE.items():
        d = os.path.join(root, folder)
        os.makedirs(d, exist_ok=True)
        ext = ".bmp" if folder.endswith("_gt") else ".tif"
        for i in range(n):
            path = os.path.join(d, f"{i + 1:03d}{ext}")
            if empty:
                open(path, "wb").close()
            else:
                from PIL import Image
                Image.fromarray(rs.integers(0, 256, size=frame_hw, dtype=np.uint8)).save(path)
