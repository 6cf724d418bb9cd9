"""Evaluation helpers: clip -> frame score broadcast and ROC-AUC, as the reference computes them
on the host (causal_anomaly_detection.py:1234-1251 `roc_auc_score(test_labels, test_scores)`, minicausal:374-390).

Every model in the reference scores whole clips; "frame-AUC" broadcasts each clip's score and label to its T
frames.  With equal-length clips that leaves the AUC unchanged (every clip is replicated T times), so frame-AUC ==
clip-AUC; with mixed T (config 5) the broadcast weights clips by length.  ``roc_auc`` is the Mann-Whitney
statistic with mid-ranks for ties, i.e. sklearn.metrics.roc_auc_score for binary labels.
"""
from __future__ import annotations

import numpy as np


def frame_scores(clip_scores, clip_lengths) -> np.ndarray:
    """Per-frame scores: clip i's score repeated clip_lengths[i] times (an int broadcasts to every clip)."""
    s = np.asarray(clip_scores, dtype=np.float64).reshape(-1)
    n = np.broadcast_to(np.asarray(clip_lengths, dtype=np.int64), s.shape)
    return np.repeat(s, n)


def roc_auc(scores, labels) -> float:
    """Binary ROC-AUC (mid-ranks for tied scores).  Raises ValueError when only one class is present, as
    roc_auc_score does."""
    s = np.asarray(scores, dtype=np.float64).reshape(-1)
    y = np.asarray(labels).reshape(-1).astype(bool)
    npos, nneg = int(y.sum()), int((~y).sum())
    if npos == 0 or nneg == 0:
        raise ValueError("Only one class present in y_true. ROC AUC score is not defined in that case.")
    order = np.argsort(s, kind="mergesort")
    ranks = np.empty(len(s), dtype=np.float64)
    ss = s[order]
    i = 0
    while i < len(ss):  # mid-ranks over runs of equal scores
        j = i
        while j + 1 < len(ss) and ss[j + 1] == ss[i]:
            j += 1
        ranks[order[i:j + 1]] = 0.5 * (i + j) + 1.0
        i = j + 1
    u = ranks[y].sum() - npos * (npos + 1) / 2.0
    return float(u / (npos * nneg))


def frame_auc(clip_scores, clip_labels, clip_lengths) -> float:
    """Frame-level AUC of clip scores and clip labels broadcast to their frames."""
    return roc_auc(frame_scores(clip_scores, clip_lengths), frame_scores(clip_labels, clip_lengths))


def evaluate_auc(model, loader) -> tuple[float, np.ndarray, np.ndarray]:
    """Scores every clip of ``loader`` with the HIP model (eval mode) and returns (frame-AUC, scores, labels), the
    quantity the reference prints after test_model (cad:1234-1251)."""
    from .train import test_model
    scores, labels, outs = test_model(model, loader)
    lengths = [len(per_clip) for o in outs for per_clip in o["detections"]]  # T frames per clip
    return frame_auc(scores, labels, lengths), np.asarray(scores), np.asarray(labels)
