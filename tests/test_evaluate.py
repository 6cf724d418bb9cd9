"""Evaluation helpers: frame-AUC against sklearn's roc_auc_score (the reference's metric,
cad:1243, minicausal:388)."""
import numpy as np
import pytest
from sklearn.metrics import roc_auc_score

from vad_amd.evaluate import frame_auc, frame_scores, roc_auc


@pytest.mark.parametrize("seed", range(5))
def test_roc_auc_matches_sklearn_with_ties(seed):
    rng = np.random.default_rng(seed)
    n = 200 + 37 * seed
    scores = np.round(rng.random(n), 2)  # many ties
    labels = rng.random(n) < 0.3
    assert roc_auc(scores, labels) == pytest.approx(roc_auc_score(labels, scores), abs=1e-12)


def test_frame_auc_equal_lengths_equals_clip_auc_and_mixed_lengths_weight_clips():
    rng = np.random.default_rng(7)
    s, y = rng.random(40), np.arange(40) % 2
    assert frame_auc(s, y, 16) == pytest.approx(roc_auc_score(y, s), abs=1e-12)
    T = rng.choice([8, 16, 32], size=40)
    fs, fy = frame_scores(s, T), frame_scores(y, T)
    assert len(fs) == T.sum()
    assert frame_auc(s, y, T) == pytest.approx(roc_auc_score(fy, fs), abs=1e-12)


def test_single_class_raises_like_sklearn():
    with pytest.raises(ValueError):
        roc_auc([0.1, 0.2], [1, 1])
