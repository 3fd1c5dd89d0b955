"""The CSC transpose (spmm.hip: k_csc_rank -> k_csc_scan_multi -> k_csc_scatter) against the
legacy histogram / single-block scan / fill launches (plan option CSC_RANK = 0) it replaced.

The transpose is observed through what consumes it: dW1 = [X | 1]^T dZ1 (light columns summed
one wave per column, heavy columns by 64-entry slices with fp32 atomics). Both transposes order
a column's entries by workgroup arrival, so the fp32 sums may differ in the last bits:
||a - b|| <= 1e-5 ||b|| per gradient block, and bias rows are compared like any other. The
forward pass does not read the transpose: losses must be identical. Shapes cover Zipf-hot
columns, a vocabulary small enough that every column is heavy, empty rows and a batch with
fewer rows than workgroups would get.
"""
import os

import numpy as np
import pytest
import torch

from dssm_amd.data import synth_batch
from oracle import dssm_oracle as O

pytestmark = pytest.mark.gpu

CASES = [
    # (D, widths, BS, NEG, mean_nnz)
    (30000, (300, 300, 128), 128, 4, 32),  # C2 vocabulary, Zipf-hot columns
    (50, (64, 32), 64, 4, 12),             # every column heavy
    (4000, (128, 64), 8, 1, 3),            # 24 rows: fewer rows than 32 workgroups
    (2000, (64, 32), 64, 3, 0),            # no entries at all (the ones column remains)
    (2000, (64, 32), 64, 3, 1),            # mostly empty rows
]


def _model(case, legacy, p):
    from dssm_amd.model import DSSM
    D, widths, BS, NEG, _ = case
    m = DSSM(D, widths, BS, NEG, dtype="bf16", init=False)
    m.set_option("CSC_RANK", not legacy)
    m.load_params(p)
    m.set_fused_w1_adam(False)
    return m


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"D{c[0]}_bs{c[2]}_nnz{c[4]}")
def test_rank_transpose_matches_legacy_transpose(case):
    D, widths, BS, NEG, nnz = case
    cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=3)
    a, b = _model(case, False, p), _model(case, True, p)
    for step in range(2):  # second step: counts and cursors re-armed by the first
        batch = synth_batch(D, BS, NEG, seed=50 + step, mean_nnz=nnz, lo=0 if nnz <= 1 else 4)
        for m in (a, b):
            m.set_batch(batch)
            m.forward(True)
            m.backward()
        torch.cuda.synchronize()
        assert a.loss_accuracy()[0] == b.loss_accuracy()[0]
        ga = a.named_grads()["W1"].cpu().numpy()
        gb = b.named_grads()["W1"].cpu().numpy()
        err = np.linalg.norm(ga - gb) / max(np.linalg.norm(gb), 1e-30)
        assert err <= 1e-5, err
        ba = a.named_grads()["b1"].cpu().numpy()
        bb = b.named_grads()["b1"].cpu().numpy()
        np.testing.assert_allclose(ba, bb, rtol=1e-4, atol=1e-6)
