"""Validation of the CPU oracle itself (no GPU): finite differences, an independent torch
autograd restatement of new_dssm.py, TF-Adam/EMA update rules, and the committed goldens."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import dssm_oracle as O
from dssm_amd.data import synth_batch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def tiny(widths=(12, 16), D=40, BS=4, NEG=3):
    cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
    b = synth_batch(D, BS, NEG, seed=7, mean_nnz=6, lo=2, hi=12)
    p = O.init_params(cfg, seed=3)
    # non-trivial BN params so gamma/beta paths are exercised
    rng = np.random.default_rng(5)
    for k in p:
        if "gamma" in k:
            p[k] = (1 + 0.3 * rng.standard_normal(p[k].shape)).astype(np.float32)
        if "beta" in k:
            p[k] = (0.2 * rng.standard_normal(p[k].shape)).astype(np.float32)
    return cfg, b, p


def loss_of(cfg, p, batch):
    cache, _ = O.forward(cfg, p, O.make_ema(cfg), batch.as_dict(), train=True, dtype=np.float64)
    return cache["loss"]


@pytest.mark.parametrize("widths", [(12, 16), (10, 12, 16)])
def test_grads_match_finite_differences(widths):
    cfg, b, p = tiny(widths)
    p64 = {k: v.astype(np.float64) for k, v in p.items()}
    cache, _ = O.forward(cfg, p64, O.make_ema(cfg), b.as_dict(), True, np.float64)
    g = O.backward(cfg, p64, cache, np.float64)
    rng = np.random.default_rng(0)
    h = 1e-6
    for k, v in p64.items():
        flat = v.reshape(-1)
        picks = rng.choice(flat.size, size=min(6, flat.size), replace=False)
        if k == "W1":  # make sure touched rows are checked
            touched = np.unique(b.indices)
            picks = np.concatenate([picks, touched[:3] * v.shape[1] + 1])
        for i in picks:
            old = flat[i]
            flat[i] = old + h
            lp = loss_of(cfg, p64, b)
            flat[i] = old - h
            lm = loss_of(cfg, p64, b)
            flat[i] = old
            fd = (lp - lm) / (2 * h)
            an = g[k].reshape(-1)[i]
            assert abs(fd - an) <= 1e-6 + 1e-4 * abs(fd), (k, i, fd, an)


def torch_restatement(cfg, p, batch):
    """Independent autograd restatement of new_dssm.py:104-213 (including the literal
    Merge_Negative_Doc concat loop at :169-179) in torch float64."""
    BS, NEG = cfg.query_bs, cfg.neg
    tp = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in p.items()}
    X = torch.zeros(batch.rows, cfg.trigram_d, dtype=torch.float64)
    for r in range(batch.rows):
        s, e = batch.indptr[r], batch.indptr[r + 1]
        X[r, torch.as_tensor(batch.indices[s:e], dtype=torch.long)] = torch.as_tensor(batch.values[s:e], dtype=torch.float64)

    def bn(x, l, t):
        mean = x.mean(0)
        var = ((x - mean.detach()) ** 2).mean(0)  # tf.nn.moments stop_gradient(mean) in variance
        inv = torch.rsqrt(var + cfg.bn_eps) * tp[f"bn{l}_{t}_gamma"]
        return x * inv + (tp[f"bn{l}_{t}_beta"] - mean * inv)

    q, d = X[:BS], X[BS:]
    for l in range(1, cfg.n_layers + 1):
        W, b = tp[f"W{l}"], tp[f"b{l}"]
        q = torch.relu(bn(q @ W + b, l, "q"))
        d = torch.relu(bn(d @ W + b, l, "d"))
    pos, negs = d[:BS], d[BS:]
    doc_y = pos
    for i in range(NEG):
        for j in range(BS):
            doc_y = torch.cat([doc_y, negs[j * NEG + i:j * NEG + i + 1]], 0)
    qn = torch.sqrt((q * q).sum(1, keepdim=True)).repeat(NEG + 1, 1)
    dn = torch.sqrt((doc_y * doc_y).sum(1, keepdim=True))
    prod = (q.repeat(NEG + 1, 1) * doc_y).sum(1, keepdim=True)
    raw = prod / (qn * dn)
    cos = raw.t().reshape(NEG + 1, BS).t() * 20
    prob = torch.softmax(cos, 1)
    loss = -torch.log(prob[:, :1]).sum() / BS
    loss.backward()
    return loss.item(), raw.detach().numpy().reshape(-1), {k: v.grad.numpy() for k, v in tp.items()}


@pytest.mark.parametrize("widths", [(12, 16), (10, 12, 16)])
def test_matches_independent_torch_autograd(widths):
    cfg, b, p = tiny(widths)
    cache, _ = O.forward(cfg, p, O.make_ema(cfg), b.as_dict(), True, np.float64)
    g = O.backward(cfg, p, cache, np.float64)
    tl, traw, tg = torch_restatement(cfg, p, b)
    assert abs(cache["loss"] - tl) <= 1e-12 * max(1, abs(tl))
    np.testing.assert_allclose(cache["cos_sim_raw"], traw, rtol=1e-12, atol=1e-14)
    for k in p:
        np.testing.assert_allclose(g[k], tg[k], rtol=1e-9, atol=1e-12, err_msg=k)


def test_adam_tf_semantics():
    cfg = O.OracleConfig(trigram_d=4, widths=[2], query_bs=2)
    p = {"x": np.array([1.0, -2.0], np.float32)}
    st = O.AdamState(cfg, p)
    g = {"x": np.array([0.5, 0.0], np.float32)}
    st.step(p, g)
    # t=1: alpha = lr*sqrt(1-b2)/(1-b1); m=0.05, v=0.00025 -> update = alpha*m/(sqrt(v)+eps)
    alpha = np.float32(0.01) * np.sqrt(np.float32(1 - 0.999)) / np.float32(1 - 0.9)
    m, v = 0.1 * 0.5, 0.001 * 0.25
    assert abs(p["x"][0] - (1.0 - alpha * m / (np.sqrt(v) + 1e-8))) < 1e-6
    assert p["x"][1] == np.float32(-2.0)  # zero grad, zero slots: no move
    st.step(p, {"x": np.array([0.0, 0.0], np.float32)})
    assert p["x"][0] < 1.0 - 0.009  # momentum keeps moving it (dense Adam)


def test_ema_update_rule():
    cfg, b, p = tiny()
    ema = O.make_ema(cfg)
    c1, e1 = O.forward(cfg, p, ema, b.as_dict(), True)
    mu = c1["layers"][0]["batch_mean"]["q"]
    np.testing.assert_allclose(e1["bn1_q_mean"], (0.5 * mu).astype(np.float32), rtol=1e-6)
    c2, e2 = O.forward(cfg, p, e1, b.as_dict(), True)
    np.testing.assert_allclose(e2["bn1_q_mean"], (0.75 * mu).astype(np.float32), rtol=1e-6)
    # eval mode uses the shadows and does not update them
    c3, e3 = O.forward(cfg, p, e2, b.as_dict(), False)
    for k in e2:
        np.testing.assert_array_equal(e2[k], e3[k])


def test_bias_grad_is_rounding_noise_under_bn():
    """Every FC is followed by batch-stat BN, so d(loss)/d(b_l) = 0 in exact arithmetic."""
    cfg, b, p = tiny((12, 16))
    cache, _ = O.forward(cfg, p, O.make_ema(cfg), b.as_dict(), True, np.float64)
    g = O.backward(cfg, p, cache, np.float64)
    for l in (1, 2):
        assert np.abs(g[f"b{l}"]).max() < 1e-12


def test_golden_fixtures_reproduce():
    """The committed fixtures were made by tests/golden/make_golden.py from this oracle;
    re-running the oracle must reproduce them (guards against silent oracle drift)."""
    from tests.golden.make_golden import CASES, build_case
    files = sorted(f for f in glob.glob(os.path.join(GOLD, "*.npz"))
                   if os.path.basename(f)[:-4] in CASES)  # ref_feed.npz: the reference's own data path
    assert files, "no golden fixtures committed"
    for f in files:
        name = os.path.basename(f)[:-4]
        ref = np.load(f, allow_pickle=False)
        got = build_case(CASES[name])
        for k in ref.files:
            np.testing.assert_allclose(got[k], ref[k], rtol=1e-6, atol=1e-7, err_msg=f"{name}:{k}")
