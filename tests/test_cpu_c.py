"""The C/OpenMP CPU restatement (oracle/cpu_c, the bench's CPU baseline) against the NumPy oracle:
forward loss/accuracy in train and eval mode, every gradient, EMA, and a teacher-forced Adam step.
fp32 C vs float64 oracle: loss rel <= 1e-5, grads <= 1e-4 x max|g| (biases excluded: pure noise
under batch-stat BN, see test_oracle.py), Adam step <= 1e-5 on well-conditioned elements."""
import re

import numpy as np
import pytest

from dssm_amd.data import synth_batch
from oracle import dssm_oracle as O

cpu_c = pytest.importorskip("oracle.cpu_c")
if not cpu_c.available():
    pytest.skip("gcc/OpenMP unavailable", allow_module_level=True)

CASES = [(64, [16, 16], 8, 4), (1000, [100, 100], 64, 4), (800, [64, 64, 32], 32, 3)]


@pytest.mark.parametrize("case", CASES)
def test_cpu_c_matches_oracle(case):
    D, widths, BS, NEG = case
    cfg = O.OracleConfig(trigram_d=D, widths=widths, query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=3)
    batch = synth_batch(D, BS, NEG, seed=77, mean_nnz=min(16, D // 4)).as_dict()
    m = cpu_c.CpuDSSM(D, widths, BS, NEG, p)
    ema0 = O.make_ema(cfg)
    cache, ema1 = O.forward(cfg, p, ema0, batch, True, np.float64)
    grads = O.backward(cfg, p, cache, np.float64)
    loss = m.forward_backward(batch, train=True, backward=True)
    assert abs(loss - cache["loss"]) <= 1e-5 * abs(cache["loss"])
    assert m.accuracy() == pytest.approx(cache["accuracy"])
    for k, v in m.named_ema().items():
        np.testing.assert_allclose(v, ema1[k], rtol=1e-5, atol=1e-6, err_msg=k)
    g = m.named("g")
    for k, ref in grads.items():
        if re.fullmatch(r"b\d+", k):
            continue
        err = np.abs(g[k] - ref).max()
        assert err <= 1e-4 * np.abs(ref).max(), (k, err)
    # eval mode uses the EMA just written
    ev = O.forward_eval_loss(cfg, p, ema1, batch)
    assert abs(m.forward_backward(batch, train=False, backward=False) - ev["loss"]) <= 1e-5 * abs(ev["loss"])


def test_cpu_c_adam_step_teacher_forced():
    D, widths, BS, NEG = 1000, [100, 100], 64, 4
    cfg = O.OracleConfig(trigram_d=D, widths=widths, query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=5)
    batch = synth_batch(D, BS, NEG, seed=11, mean_nnz=16).as_dict()
    m = cpu_c.CpuDSSM(D, widths, BS, NEG, p)
    ema = O.make_ema(cfg)
    adam = O.AdamState(cfg, p)
    cache, grads, _ = O.train_step(cfg, p, ema, adam, batch, dtype=np.float64)
    loss = m.train_step(batch)
    assert abs(loss - cache["loss"]) <= 1e-5 * abs(cache["loss"])
    got = m.named("p")
    lr = 0.01
    for k, ref in p.items():
        if re.fullmatch(r"b\d+", k):
            continue
        d = np.abs(got[k] - ref)
        well = np.abs(grads[k]) > 1e-3 * np.abs(grads[k]).max()
        assert d[well].max(initial=0.0) <= 1e-5, (k, d[well].max(initial=0.0))
        assert d.max() <= 2 * lr, k
    f = np.float32
    np.testing.assert_array_equal(m.beta_powers, np.array([f(0.9) * f(0.9), f(0.999) * f(0.999)], np.float32))


@pytest.mark.parametrize("keep", [1.0, 0.5])
def test_rnn_port_matches_oracle(keep):
    """oracle/cpu_c/rnn_cpu.c (bench.py's config-4 cpu_baseline) against the float64 RNN oracle:
    embeddings, summed loss, every gradient, then one TF1.x Adam step."""
    from oracle import rnn_oracle as RO
    cfg = RO.RnnConfig(nwords=300, emb=32, hidden=32, query_bs=16, neg=4, seq_len=7, lr=1e-3)
    p = RO.init_params(cfg, seed=3)
    ids, lens = RO.synth_ids(cfg, seed=5)
    mask = RO.dropout_mask(cfg.rows, 2 * cfg.hidden, keep, seed=17, step=1)
    m = cpu_c.CpuRnnDSSM(cfg.nwords, cfg.emb, cfg.hidden, cfg.query_bs, cfg.neg, cfg.seq_len, p, lr=cfg.lr)
    loss = m.forward_backward(ids, lens, mask, keep)
    p64 = {k: v.astype(np.float64) for k, v in p.items()}
    ref = RO.forward(cfg, p64, ids, lens, mask, keep)
    np.testing.assert_allclose(m.output(), ref["y0"], rtol=1e-4, atol=1e-5)
    assert abs(loss - ref["loss"]) <= 1e-4 * abs(ref["loss"])
    g = RO.backward(cfg, p64, ids, lens, ref)
    got = m.named("g")
    for k, gr in g.items():
        assert np.abs(got[k] - gr).max() <= 1e-4 * np.abs(gr).max() + 1e-7, k
    opt = RO.Adam(cfg, {k: v.copy() for k, v in p.items()})
    pref = {k: v.copy() for k, v in p.items()}
    opt.step(pref, {k: v.copy() for k, v in got.items()})
    m2 = cpu_c.CpuRnnDSSM(cfg.nwords, cfg.emb, cfg.hidden, cfg.query_bs, cfg.neg, cfg.seq_len, p, lr=cfg.lr)
    m2.train_step(ids, lens, mask, keep)
    after = m2.named("p")
    for k in pref:
        assert np.abs(after[k] - pref[k]).max() <= 2 * cfg.lr, k
        well = np.abs(g[k]) > 1e-3 * np.abs(g[k]).max()
        assert np.abs(after[k] - pref[k])[well].max(initial=0.0) <= 1e-6, k
