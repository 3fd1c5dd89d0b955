"""Side outputs of new_dssm.py:219-231: accuracy and the streaming AUC.

Accuracy comes from the device. `k_cosine_loss` writes it next to the loss.

The AUC is `tf.metrics.auc(label_tensor, cos_sim_raw, num_thresholds=2000)` (new_dssm.py:224-230).
Its semantics:

* labels are `[1]*BS + [0]*BS*NEG`, aligned with `cos_sim_raw`'s (k, j) order (new_dssm.py:163-166);
* confusion counts are accumulated at fixed thresholds. TF1.x uses
  `[-1e-7, 1/(n-1), ..., (n-2)/(n-1), 1+1e-7]`, and a prediction counts as positive when it is
  `> threshold`;
* the ROC AUC is taken by the trapezoid rule, with TF's 1e-7 smoothing;
* the counts are local variables that the reference never resets (new_dssm.py:252). One
  `StreamingAUC` object therefore accumulates for as long as the caller keeps it.

This is eval-side host logic over 5120 device-computed scores per batch. It is not on the
training hot path.
"""
from __future__ import annotations

import numpy as np

_EPS = 1e-7


class StreamingAUC:
    def __init__(self, num_thresholds: int = 2000):
        n = int(num_thresholds)
        if n < 2:
            raise ValueError("num_thresholds must be >= 2")
        self.thresholds = np.array([-_EPS] + [(i + 1) / (n - 1) for i in range(n - 2)] + [1.0 + _EPS],
                                   dtype=np.float64)
        self.reset()

    def reset(self):
        n = self.thresholds.size
        self.tp = np.zeros(n, np.float32)
        self.fp = np.zeros(n, np.float32)
        self.tn = np.zeros(n, np.float32)
        self.fn = np.zeros(n, np.float32)

    def update(self, labels: np.ndarray, predictions: np.ndarray):
        """auc_op: accumulate one batch (labels in {0,1}, predictions in [0, 1])."""
        lab = np.asarray(labels).astype(bool).ravel()
        pred = np.asarray(predictions, np.float64).ravel()
        if lab.size != pred.size:
            raise ValueError("labels and predictions differ in size")
        if pred.size and (np.nanmin(pred) < 0.0 or np.nanmax(pred) > 1.0):
            # tf.metrics.auc asserts predictions in [0, 1] (ReLU embeddings keep cosines there)
            raise ValueError("predictions must be in [0, 1]")
        # count of predictions > thr, by sorting instead of a [thresholds x n] comparison; a NaN
        # is never > thr (TF's greater), so it lands in fn / tn
        ok = ~np.isnan(pred)
        pos, neg = np.sort(pred[lab & ok]), np.sort(pred[~lab & ok])
        n_pos, n_neg = int(lab.sum()), int((~lab).sum())
        tp = pos.size - np.searchsorted(pos, self.thresholds, side="right")
        fp = neg.size - np.searchsorted(neg, self.thresholds, side="right")
        self.tp += tp.astype(np.float32)
        self.fp += fp.astype(np.float32)
        self.fn += (n_pos - tp).astype(np.float32)
        self.tn += (n_neg - fp).astype(np.float32)
        return self.value()

    def value(self) -> float:
        """auc_value: trapezoid ROC AUC of the accumulated counts."""
        tp, fp, tn, fn = (x.astype(np.float64) for x in (self.tp, self.fp, self.tn, self.fn))
        tpr = (tp + _EPS) / (tp + fn + _EPS)
        fpr = fp / (fp + tn + _EPS)
        return float(np.sum((fpr[:-1] - fpr[1:]) * (tpr[:-1] + tpr[1:]) / 2.0))


def dssm_labels(query_bs: int, neg: int) -> np.ndarray:
    """label_tensor of new_dssm.py:163-166 in cos_sim_raw's (k, j) order."""
    return np.array([1] * query_bs + [0] * query_bs * neg, np.int32)
