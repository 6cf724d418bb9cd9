"""Helpers shared by the parity tests: golden fixture loading and reference-identical model construction."""
import glob
import os

import numpy as np
import torch

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# the reference's shipped a2 checkpoint (best_improved_model.pth, model_state_dict) exported as a safe .npz
A2_CKPT = "a2_best_improved_model.npz"


def load(name):
    return dict(np.load(os.path.join(GOLDEN_DIR, name), allow_pickle=False))


def cad_cases():
    from tests.golden.cases import CAD_CASES
    return CAD_CASES


def make_cad_model(case):
    """Our drop-in module under the case seed (identical init to the reference), with the forced-detector edit."""
    from vad_amd.cad import CausalAnomalyDetector
    from tests.golden.cases import force_detector
    torch.manual_seed(case["seed"])
    m = CausalAnomalyDetector(num_factors=6, reid_dim=64)
    if case["forced"]:
        force_detector(m.state_dict(), case["forced"])
    return m


def golden_names():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))
