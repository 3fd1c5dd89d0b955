"""RNN tower (dssm_amd/rnn.py, csrc/rnn.hip) against the NumPy oracle (oracle/rnn_oracle.py,
float64) on the same seeded inputs: forward embeddings / loss (fp32: rel 1e-5), every gradient
(<= 1e-4 * max|g|), the dropout mask, and teacher-forced TF1.x Adam steps (dense + the embedding's
IndexedSlices form; <= 1e-6 on well-conditioned elements, <= 2 lr everywhere)."""
import numpy as np
import pytest
import torch

from dssm_amd.rnn import RnnDSSM
from oracle import rnn_oracle as R

pytestmark = pytest.mark.gpu

CASES = [
    dict(nwords=300, emb=32, hidden=32, query_bs=16, neg=4, seq_len=6),
    dict(nwords=2000, emb=64, hidden=128, query_bs=32, neg=4, seq_len=12),
]


def _setup(case, keep):
    cfg = R.RnnConfig(lr=1e-3, **case)
    p = R.init_params(cfg, seed=3)
    m = RnnDSSM(cfg.nwords, cfg.emb, cfg.hidden, cfg.query_bs, cfg.neg, cfg.seq_len, lr=cfg.lr,
                keep_prob=keep, seed=17)
    m.load_params(p)
    ids, lens = R.synth_ids(cfg, seed=5)
    m.set_batch(ids, lens)
    return cfg, p, m, ids, lens


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("keep", [1.0, 0.5])
def test_rnn_forward_backward_matches_oracle(case, keep):
    cfg, p, m, ids, lens = _setup(case, keep)
    m.forward(True)
    torch.cuda.synchronize()
    mask = R.dropout_mask(cfg.rows, 2 * cfg.hidden, keep, seed=17, step=1)
    ref = R.forward(cfg, {k: v.astype(np.float64) for k, v in p.items()}, ids, lens, mask, keep)
    np.testing.assert_allclose(m.y0.cpu().numpy(), ref["y0"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(m.y.cpu().numpy(), ref["y"], rtol=1e-4, atol=1e-5)
    assert abs(m.loss() - ref["loss"]) <= 1e-4 * abs(ref["loss"]), (m.loss(), ref["loss"])
    m.backward()
    torch.cuda.synchronize()
    g = R.backward(cfg, {k: v.astype(np.float64) for k, v in p.items()}, ids, lens, ref)
    got = m.named(m.grads)
    for k, gr in g.items():
        scale = np.abs(gr).max()
        err = np.abs(got[k] - gr).max()
        assert err <= 1e-4 * scale + 1e-7, (k, err, scale)


@pytest.mark.parametrize("case", CASES[:1])
def test_rnn_adam_teacher_forced(case):
    cfg, p, m, ids, lens = _setup(case, 1.0)
    opt = R.Adam(cfg, {k: v.copy() for k, v in p.items()})
    pref = {k: v.copy() for k, v in p.items()}
    for step in range(3):
        m.load_params(pref)  # teacher forcing: same parameters, same Adam slots on both sides
        m.forward(True)
        m.backward()
        torch.cuda.synchronize()
        g = m.named(m.grads)
        m.apply_adam()
        torch.cuda.synchronize()
        opt.step(pref, g)
        got = m.named()
        for k in pref:
            d = np.abs(got[k] - pref[k])
            assert d.max() <= 2 * cfg.lr, (k, d.max())
            well = np.abs(g[k]) > 1e-3 * np.abs(g[k]).max()
            assert d[well].max(initial=0.0) <= 1e-6, (k, step, d[well].max(initial=0.0))
        pref = got


def test_rnn_trains():
    case = CASES[1]
    cfg = R.RnnConfig(lr=3e-3, **case)
    m = RnnDSSM(cfg.nwords, cfg.emb, cfg.hidden, cfg.query_bs, cfg.neg, cfg.seq_len, lr=cfg.lr,
                keep_prob=1.0)
    m.init_params(0)
    ids, lens = R.synth_ids(cfg, seed=9)
    m.set_batch(ids, lens)
    losses = []
    for _ in range(30):
        m.train_step()
        losses.append(m.loss())
    torch.cuda.synchronize()
    assert np.isfinite(losses).all() and losses[-1] < 0.5 * losses[0], losses[::5]


def test_rnn_config4_full_size_matches_oracle():
    """BASELINE.json config 4 at its full size (vocabulary 21,128, E = H = 128, T = 32, BS = 1024,
    NEG = 4: 6144 rows), dropout 0.5 and ragged lengths in [1, 32]: the forward embeddings and the
    summed loss, and every gradient, against the float64 oracle at the fp32 bars of the small cases
    (32 recurrent steps of fp32 accumulation stay inside them)."""
    case = dict(nwords=21128, emb=128, hidden=128, query_bs=1024, neg=4, seq_len=32)
    cfg, p, m, ids, lens = _setup(case, 0.5)
    m.forward(True)
    torch.cuda.synchronize()
    mask = R.dropout_mask(cfg.rows, 2 * cfg.hidden, 0.5, seed=17, step=1)
    p64 = {k: v.astype(np.float64) for k, v in p.items()}
    ref = R.forward(cfg, p64, ids, lens, mask, 0.5)
    np.testing.assert_allclose(m.y0.cpu().numpy(), ref["y0"], rtol=1e-4, atol=1e-5)
    assert abs(m.loss() - ref["loss"]) <= 1e-4 * abs(ref["loss"]), (m.loss(), ref["loss"])
    m.backward()
    torch.cuda.synchronize()
    g = R.backward(cfg, p64, ids, lens, ref)
    got = m.named(m.grads)
    for k, gr in g.items():
        err = np.abs(got[k] - gr).max()
        assert err <= 1e-4 * np.abs(gr).max() + 1e-7, (k, err, np.abs(gr).max())
