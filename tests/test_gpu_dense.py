"""The persistent dense-stack kernels (dense.hip, default in bf16 mode) against the per-op
launches (DSSM_DENSE=0) and against the oracle.

Both paths round the same tensors to bf16 (activations, dZ, weights). They differ in fp32
summation order (whole-K vs 64-deep K steps, split-K row chunks), which occasionally flips a
bf16 rounding. The bars are:

* loss: rel <= 1e-3;
* cos_sim_raw / prob: <= 2e-3 abs;
* embeddings: <= 2e-2 abs;
* each gradient tensor: ||a - b|| <= 2e-2 ||b||;
* EMA: rtol 1e-3, atol 1e-4 (near-zero means carry bf16 rounding).

Against the float64 oracle, the bf16 bars of test_gpu_parity apply.
"""
import os
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
    (3000, (128, 96), 64, 9),          # NEG+1 = 10: the 16-wide cosine variant
    (4000, (512, 256, 256), 64, 2),    # K = 512 staging, 4 columns per lane in the cosine
]


def _model(case, dense: bool, p):
    from dssm_amd.model import DSSM
    D, widths, BS, NEG = case
    old = os.environ.get("DSSM_DENSE")
    os.environ["DSSM_DENSE"] = "1" if dense else "0"
    try:
        m = DSSM(D, widths, BS, NEG, dtype="bf16", init=False)
    finally:
        if old is None:
            os.environ.pop("DSSM_DENSE")
        else:
            os.environ["DSSM_DENSE"] = old
    m.load_params(p)
    m.set_fused_w1_adam(False)
    assert m.dense_persistent == dense
    return m


def _is_bias(k):
    return re.fullmatch(r"b\d+", k) is not None


@pytest.mark.parametrize("case", CASES)
def test_dense_matches_per_op_path_and_oracle(case):
    D, widths, BS, NEG = case
    cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=21)
    batch = synth_batch(D, BS, NEG, seed=99, mean_nnz=24)
    a, b = _model(case, True, p), _model(case, False, p)
    for m in (a, b):
        m.set_batch(batch)
        m.forward(True)
        m.backward()
    a.check()
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
    # against the float64 oracle (bf16 bars)
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
    # eval forward (EMA batch norm)
    for m in (a, b):
        m.forward(False)
    a.check()
    ea, eb = a.loss_accuracy()[0], b.loss_accuracy()[0]
    assert abs(ea - eb) <= 1e-3 * abs(eb), (ea, eb)


def test_dense_training_steps_track_per_op_path():
    case = (5000, (300, 300, 128), 128, 4)
    D, widths, BS, NEG = case
    cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=5)
    a, b = _model(case, True, p), _model(case, False, p)
    a.set_fused_w1_adam(True)  # default single-GPU path: W1 light rows + dW slabs inside Adam
    b.set_fused_w1_adam(True)
    la, lb = [], []
    for s in range(8):
        batch = synth_batch(D, BS, NEG, seed=300 + s % 3, mean_nnz=24)
        for m, out in ((a, la), (b, lb)):
            m.set_batch(batch)
            m.train_step()
            out.append(m.loss_accuracy()[0])
    a.check()
    la, lb = np.array(la), np.array(lb)
    assert np.all(np.isfinite(la)) and la[-1] < la[0]
    np.testing.assert_allclose(la, lb, rtol=5e-2, atol=2e-2)  # free-running bf16: small losses
