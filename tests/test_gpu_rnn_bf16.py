"""bf16 perf mode of the RNN tower (dssm_amd/rnn.py dtype="bf16", csrc/rnn_mfma.hip: MFMA
recurrences with register-resident weights) against the bf16-emulating NumPy oracle
(oracle/rnn_oracle.py emulate="bf16": the same operand rounding points, float64 elsewhere) on the same
seeded inputs, including BASELINE.json config 4's full size with ragged lengths and dropout.

Bars (written here, bf16 mode): final states |err| <= 1e-4 (states lie in (-1, 1); measured <= 1.2e-5);
summed loss relative <= 2e-4; every gradient ||err|| <= 5e-3 ||g|| (measured <= 1.9e-3) with cosine
>= 0.99999.  Rounding-boundary flips
of the bf16 state operand between the fp32 kernel and the float64 oracle are what the bars absorb;
the un-emulated float64 oracle is reported beside them (the bf16 mode's own error)."""
import numpy as np
import pytest
import torch

from dssm_amd.rnn import RnnDSSM
from oracle import rnn_oracle as R

pytestmark = pytest.mark.gpu

CASES = [
    dict(nwords=300, emb=32, hidden=32, query_bs=10, neg=4, seq_len=6),  # 60 rows: a partial block
    dict(nwords=2000, emb=64, hidden=128, query_bs=32, neg=4, seq_len=12),
    dict(nwords=5000, emb=128, hidden=128, query_bs=40, neg=4, seq_len=16),
]


def _setup(case, keep, seed=3):
    cfg = R.RnnConfig(lr=1e-3, **case)
    p = R.init_params(cfg, seed=seed)
    m = RnnDSSM(cfg.nwords, cfg.emb, cfg.hidden, cfg.query_bs, cfg.neg, cfg.seq_len, lr=cfg.lr,
                keep_prob=keep, seed=17, dtype="bf16")
    m.load_params(p)
    ids, lens = R.synth_ids(cfg, seed=5)
    m.set_batch(ids, lens)
    return cfg, p, m, ids, lens


def _check(cfg, p, m, ids, lens, keep):
    m.forward(True)
    torch.cuda.synchronize()
    mask = R.dropout_mask(cfg.rows, 2 * cfg.hidden, keep, seed=17, step=1)
    p64 = {k: v.astype(np.float64) for k, v in p.items()}
    ref = R.forward(cfg, p64, ids, lens, mask, keep, emulate="bf16")
    y0 = m.y0.cpu().numpy()
    err_y = np.abs(y0 - ref["y0"]).max()
    plain = R.forward(cfg, p64, ids, lens, mask, keep)
    print(f"y0 max|err| vs emulated {err_y:.2e}, vs float64 {np.abs(y0 - plain['y0']).max():.2e}")
    assert err_y <= 1e-4, err_y
    assert abs(m.loss() - ref["loss"]) <= 2e-4 * abs(ref["loss"]), (m.loss(), ref["loss"])
    m.backward()
    torch.cuda.synchronize()
    g = R.backward(cfg, p64, ids, lens, ref)
    g_plain = R.backward(cfg, p64, ids, lens, plain)
    got = m.named(m.grads)
    for k, gr in g.items():
        a, b = got[k].ravel().astype(np.float64), gr.ravel()
        rel = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
        cos = a @ b / max(np.linalg.norm(a) * np.linalg.norm(b), 1e-30)
        gp = g_plain[k].ravel()
        rel_plain = np.linalg.norm(a - gp) / max(np.linalg.norm(gp), 1e-30)
        print(f"{k}: rel {rel:.2e} cos {cos:.6f} (vs float64: rel {rel_plain:.2e})")
        assert rel <= 5e-3 and cos >= 0.99999, (k, rel, cos)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("keep", [1.0, 0.5])
def test_rnn_bf16_matches_emulating_oracle(case, keep):
    cfg, p, m, ids, lens = _setup(case, keep)
    _check(cfg, p, m, ids, lens, keep)


def test_rnn_bf16_config4_full_size():
    """BASELINE.json config 4 at full size (vocabulary 21,128, E = H = 128, T = 32, BS = 1024, NEG = 4:
    6144 rows, the timed shape), dropout 0.5, ragged lengths in [1, 32]."""
    case = dict(nwords=21128, emb=128, hidden=128, query_bs=1024, neg=4, seq_len=32)
    cfg, p, m, ids, lens = _setup(case, 0.5)
    _check(cfg, p, m, ids, lens, 0.5)


def test_rnn_bf16_trains():
    case = CASES[1]
    cfg = R.RnnConfig(lr=3e-3, **case)
    m = RnnDSSM(cfg.nwords, cfg.emb, cfg.hidden, cfg.query_bs, cfg.neg, cfg.seq_len, lr=cfg.lr,
                keep_prob=1.0, dtype="bf16")
    m.init_params(0)
    ids, lens = R.synth_ids(cfg, seed=9)
    m.set_batch(ids, lens)
    losses = []
    for _ in range(30):
        m.train_step()
        losses.append(m.loss())
    torch.cuda.synchronize()
    assert np.isfinite(losses).all() and losses[-1] < 0.5 * losses[0], losses[::5]
