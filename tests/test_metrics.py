"""Streaming AUC (dssm_amd/metrics.py, the tf.metrics.auc of new_dssm.py:224-230) against the
oracle's restatement, including predictions exactly on thresholds, NaNs and accumulation across
batches (the reference never resets it, new_dssm.py:252)."""
import numpy as np
import pytest

from dssm_amd.metrics import StreamingAUC, dssm_labels
from oracle import dssm_oracle as O


def test_labels_match_reference_order():
    lab = dssm_labels(3, 2)
    assert lab.tolist() == [1, 1, 1, 0, 0, 0, 0, 0, 0]


def test_streaming_auc_matches_oracle():
    rng = np.random.default_rng(0)
    auc = StreamingAUC(2000)
    state = None
    thr = auc.thresholds
    for b in range(5):
        BS, NEG = 64, 4
        lab = dssm_labels(BS, NEG)
        pred = np.clip(rng.normal(0.5 + 0.2 * lab, 0.2), 0.0, 1.0)
        pred[:5] = thr[10:15]          # exactly on thresholds: '>' excludes them
        pred[-3:] = [0.0, 1.0, 0.5]
        got = auc.update(lab, pred)
        ref, state = O.auc_streaming(lab, pred, 2000, state)
        assert abs(got - ref) <= 1e-6, (b, got, ref)
        assert abs(auc.value() - ref) <= 1e-6
    for k in ("tp", "fp", "tn", "fn"):
        np.testing.assert_array_equal(getattr(auc, k), state[k].astype(np.float32))


def test_streaming_auc_nan_and_range():
    auc = StreamingAUC(10)
    lab = np.array([1, 0, 1, 0])
    pred = np.array([0.9, 0.1, np.nan, 0.2])
    auc.update(lab, pred)
    ref, _ = O.auc_streaming(lab, pred, 10)
    assert abs(auc.value() - ref) <= 1e-9
    with pytest.raises(ValueError):
        auc.update(np.array([1]), np.array([1.5]))
    with pytest.raises(ValueError):
        StreamingAUC(1)
