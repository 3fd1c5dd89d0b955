"""The fused-statistics per-op schedule (csrc/bnfuse.h, default for bf16 train steps) against the
separate statistics launches (plan option FUSED_STATS = 0) and the oracle.

The fused schedule computes the same batch-norm quantities from fp64 column sums (E[z^2] - mean^2)
accumulated by the kernels that produce each layer, where the separate launches merge fp32
(mean, M2) partials. Everything downstream sees fp32 coefficients that differ in the last bits,
and bf16 roundings of the activations occasionally flip. The bars are the ones
test_gpu_dense.py uses:

* loss: rel <= 1e-3;
* cos_sim_raw / prob: <= 2e-3 abs;
* embeddings: <= 2e-2 abs;
* each gradient tensor: ||a - b|| <= 2e-2 ||b||;
* EMA and batch moments: rtol 1e-3, atol 1e-4.

Against the float64 oracle, the bf16 bars of test_gpu_parity apply.
"""
import re

import numpy as np
import pytest
import torch

from dssm_amd.data import synth_batch
from oracle import dssm_oracle as O

pytestmark = pytest.mark.gpu

CASES = [
    # (D, widths, BS, NEG)
    (5000, (300, 300, 128), 128, 4),   # C2 shape
    (1000, (100, 100), 64, 4),         # C1 widths
    (2000, (64, 64, 32), 64, 3),
    (3000, (128, 96), 64, 9),          # NEG+1 = 10: the 16-row cosine variant
    (4000, (512, 256, 256), 64, 2),    # K = 512 staging, 4 columns per lane in the cosine
]


def _model(case, fused: bool, p):
    from dssm_amd.model import DSSM
    D, widths, BS, NEG = case
    m = DSSM(D, widths, BS, NEG, dtype="bf16", init=False)
    m.set_option("FUSED_STATS", fused)
    m.load_params(p)
    m.set_fused_w1_adam(False)
    assert m.fused_stats == fused
    return m


def _is_bias(k):
    return re.fullmatch(r"b\d+", k) is not None


@pytest.mark.parametrize("case", CASES)
def test_fused_stats_match_separate_launches_and_oracle(case):
    D, widths, BS, NEG = case
    cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=21)
    batch = synth_batch(D, BS, NEG, seed=99, mean_nnz=24)
    a, b = _model(case, True, p), _model(case, False, p)
    for m in (a, b):
        m.set_batch(batch)
        m.forward(True)
        m.backward()
    torch.cuda.synchronize()
    la, lb = a.loss_accuracy()[0], b.loss_accuracy()[0]
    assert abs(la - lb) <= 1e-3 * abs(lb), (la, lb)
    for name, tol in (("cos_sim_raw", 2e-3), ("prob", 2e-3), ("embedding_all", 2e-2)):
        np.testing.assert_allclose(a.fetch(name), b.fetch(name), atol=tol, rtol=0, err_msg=name)
    ga = {k: v.cpu().numpy() for k, v in a.named_grads().items()}
    gb = {k: v.cpu().numpy() for k, v in b.named_grads().items()}
    for k in gb:
        if _is_bias(k):
            continue
        err = np.linalg.norm(ga[k] - gb[k]) / max(np.linalg.norm(gb[k]), 1e-30)
        assert err <= 2e-2, (k, err)
    for k, v in b.named_ema().items():
        np.testing.assert_allclose(a.named_ema()[k].cpu().numpy(), v.cpu().numpy(), rtol=1e-3, atol=1e-4,
                                   err_msg=k)
    for l in range(1, len(widths) + 1):
        ma, mb = a.batch_moments(l), b.batch_moments(l)
        for t in ("q", "d"):
            np.testing.assert_allclose(ma[t][0], mb[t][0], rtol=1e-3, atol=1e-4)
            np.testing.assert_allclose(ma[t][1], mb[t][1], rtol=1e-3, atol=1e-4)
    cache, _ = O.forward(cfg, p, O.make_ema(cfg), batch.as_dict(), True, np.float64)
    grads = O.backward(cfg, p, cache, np.float64)
    assert abs(la - cache["loss"]) <= 2e-2 * abs(cache["loss"])
    np.testing.assert_allclose(a.fetch("cos_sim_raw").ravel(), cache["cos_sim_raw"], atol=2e-2)
    for k, ref in grads.items():
        if _is_bias(k):
            continue
        g = ga[k].ravel().astype(np.float64)
        r = ref.ravel()
        cosd = g @ r / max(np.linalg.norm(g) * np.linalg.norm(r), 1e-30)
        assert cosd >= 0.99, (k, cosd)
    # the next train forward must start from cleared accumulators: run it twice and compare
    for m in (a, b):
        m.forward(True)
        m.backward()
    torch.cuda.synchronize()
    la2, lb2 = a.loss_accuracy()[0], b.loss_accuracy()[0]
    assert abs(la2 - lb2) <= 1e-3 * abs(lb2), (la2, lb2)
    ga2 = {k: v.cpu().numpy() for k, v in a.named_grads().items()}
    for k in ga:
        if not _is_bias(k):
            np.testing.assert_allclose(ga2[k], ga[k], rtol=1e-4, atol=1e-6, err_msg=k)


def test_fused_stats_training_steps_track_separate_launches():
    case = (5000, (300, 300, 128), 128, 4)
    D, widths, BS, NEG = case
    cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=5)
    a, b = _model(case, True, p), _model(case, False, p)
    a.set_fused_w1_adam(True)
    b.set_fused_w1_adam(True)
    la, lb = [], []
    for s in range(8):
        batch = synth_batch(D, BS, NEG, seed=300 + s % 3, mean_nnz=24)
        for m, out in ((a, la), (b, lb)):
            m.set_batch(batch)
            m.train_step()
            out.append(m.loss_accuracy()[0])
    torch.cuda.synchronize()
    la, lb = np.array(la), np.array(lb)
    assert np.all(np.isfinite(la)) and la[-1] < la[0]
    np.testing.assert_allclose(la, lb, rtol=5e-2, atol=2e-2)


def test_fused_stats_unsupported_batch_falls_back():
    from dssm_amd.model import DSSM
    m = DSSM(1000, (64, 32), 48, 4, dtype="bf16")  # 48 % 64 != 0: tiles would straddle towers
    assert not m.fused_stats
    m2 = DSSM(1000, (64, 32), 64, 4, dtype="bf16")
    assert m2.fused_stats
    m3 = DSSM(1000, (64, 32), 64, 4, dtype="fp32")  # fp32 parity mode: fused too (g32.h tiles)
    assert m3.fused_stats
    m4 = DSSM(1000, (64, 32), 48, 4, dtype="fp32")
    assert not m4.fused_stats


def test_train_forward_without_backward_reports_its_loss():
    """The fused schedule defers the loss reduction to the backward's first launch; a train
    forward read on its own (dssm_plan_finalize_loss) must report the same loss."""
    case = (2000, (64, 64, 32), 64, 3)
    D, widths, BS, NEG = case
    cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=8)
    batch = synth_batch(D, BS, NEG, seed=5, mean_nnz=16)
    a, b = _model(case, True, p), _model(case, True, p)
    a.set_batch(batch)
    a.forward(True)
    la = a.loss_accuracy()
    b.set_batch(batch)
    b.forward(True)
    b.backward()
    lb = b.loss_accuracy()
    assert la == lb, (la, lb)
    cache, _ = O.forward(cfg, p, O.make_ema(cfg), batch.as_dict(), True, np.float64)
    assert abs(la[0] - cache["loss"]) <= 2e-2 * abs(cache["loss"])
