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


def ae_memory_init(case):
    """(normal_memory (500, 64), memory_ptr) of a cad1 AE case before training."""
    mem = torch.zeros(500, 64)
    if case["mem"] is None:
        return mem, 0
    rows, ptr = case["mem"]
    mem[:rows] = torch.from_numpy(np.random.default_rng(case["seed"]).standard_normal((rows, 64)).astype(np.float32))
    return mem, ptr


def ae_case_data(case):
    """(train, val, test) lists of (clips (B, T, 1, 64, 64), int64 labels) of a cad1 AE case."""
    from oracle import ae_oracle as ae
    B, T, seed = case["B"], case["T"], case["seed"]
    lab = lambda v: torch.tensor(v, dtype=torch.int64)  # noqa: E731
    train = [(ae.synth_clips(seed, k, k * B, B, T), lab(y)) for k, y in enumerate(case["labels"])]
    val = [(ae.synth_clips(seed, 100, 0, len(case["val_labels"]), T), lab(case["val_labels"]))]
    test = [(ae.synth_clips(seed, 200, 0, len(case["test_labels"]), T), lab(case["test_labels"]))]
    return train, val, test


def golden_names():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))
