"""The RNN-tower oracle (oracle/rnn_oracle.py) pinned by float64 finite differences of its own
forward (TF is absent: parity with TF's GRUCell / bidirectional_dynamic_rnn autodiff is unpinned,
these checks pin the restatement's gradients), plus the dropout mask's statistics and the TF1.x
Adam variants."""
import numpy as np

from oracle import rnn_oracle as R


def _setup(seed=0):
    cfg = R.RnnConfig(nwords=50, emb=6, hidden=5, query_bs=3, neg=2, seq_len=4)
    p = {k: v.astype(np.float64) for k, v in R.init_params(cfg, seed).items()}
    ids, lens = R.synth_ids(cfg, seed + 1)
    lens[0] = cfg.seq_len  # full, partial and length-1 rows
    lens[1] = 1
    return cfg, p, ids, lens


def test_gradients_match_finite_differences():
    cfg, p, ids, lens = _setup()
    mask = R.dropout_mask(cfg.rows, 2 * cfg.hidden, 0.7, seed=3, step=1)
    fw = R.forward(cfg, p, ids, lens, mask, 0.7)
    g = R.backward(cfg, p, ids, lens, fw)
    rng = np.random.default_rng(0)
    h = 1e-6
    for k in ("fw_Wg", "fw_bg", "fw_Wc", "fw_bc", "bw_Wg", "bw_bc", "emb"):
        flat = p[k].reshape(-1)
        cand = np.unique(ids) * p[k].shape[1] + 2 if k == "emb" else np.arange(flat.size)
        for i in rng.choice(cand, size=min(12, len(cand)), replace=False):
            old = flat[i]
            flat[i] = old + h
            lp = R.forward(cfg, p, ids, lens, mask, 0.7)["loss"]
            flat[i] = old - h
            lm = R.forward(cfg, p, ids, lens, mask, 0.7)["loss"]
            flat[i] = old
            num = (lp - lm) / (2 * h)
            assert abs(num - g[k].reshape(-1)[i]) <= 1e-6 + 1e-5 * abs(num), (k, i, num, g[k].reshape(-1)[i])


def test_state_carried_past_length():
    """A row's final states ignore ids at and past its length (dynamic_rnn semantics)."""
    cfg, p, ids, lens = _setup(2)
    ids2 = ids.copy()
    r = 1  # length 1
    ids2[r, 1:] = (ids2[r, 1:] + 7) % cfg.nwords
    a = R.forward(cfg, p, ids, lens)["y0"][r]
    b = R.forward(cfg, p, ids2, lens)["y0"][r]
    np.testing.assert_array_equal(a, b)


def test_dropout_mask_rate():
    m = R.dropout_mask(512, 256, 0.5, seed=11, step=7)
    assert abs(m.mean() - 0.5) < 0.01
    assert not np.array_equal(m, R.dropout_mask(512, 256, 0.5, seed=11, step=8))
    assert R.dropout_mask(4, 4, 1.0, 0, 0).min() == 1.0


def test_adam_variants():
    cfg = R.RnnConfig(nwords=4, emb=2, hidden=2, query_bs=1, lr=0.1)
    p = {"emb": np.ones((4, 2), np.float32), "fw_bc": np.ones(2, np.float32)}
    opt = R.Adam(cfg, p)
    g = {"emb": np.array([[1, 0], [0, 0], [0, 0], [0, 0]], np.float32), "fw_bc": np.array([1, -1], np.float32)}
    opt.step(p, g)
    # first step moves a touched element by ~lr (m/sqrt(v) = 1), untouched ones stay
    assert abs(p["emb"][0, 0] - 0.9) < 1e-4 and p["emb"][1, 0] == 1.0
    np.testing.assert_allclose(p["fw_bc"], [0.9, 1.1], atol=1e-4)
