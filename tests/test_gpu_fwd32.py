"""Plan option FWD32: the bf16 perf plan with the forward at the reference's precision.

new_dssm.py:111-114 declares fp32 placeholders and variables, so the north star's "loss and cosine
scores within 1e-4 of the TF reference" is a statement about the forward.  The bf16 perf mode misses
it by its bf16 weights and activations (loss 6e-4 relative, cosine 1.5e-3 absolute at C2:
bench.py's cpu_baseline.parity_vs_oracle).  FWD32 keeps the bf16 mode's backward and optimizer and
runs the forward as the fp32 parity mode does: the SpMM gathers the fp32 W1 masters, layers >= 2
run the g32 tiles (csrc/g32.h) on the fp32 W_l, and those tiles write the bf16 activations the bf16
backward reads (the bf16 NT tile's rounding of the same values).  Checked against the float64
oracle (oracle/dssm_oracle.py):

* the training forward at C2 and at a small shape: loss <= 1e-5 relative, cos_sim_raw / prob
  <= 1e-5 absolute, embeddings, BN batch moments and the EMA update at the fp32 mode's bars;
* the eval forward (EMA BN) at the same bars;
* the backward: every weight gradient's relative L2 error <= 1e-2 against the exact gradient
  (measured ~3e-3) and below the plain bf16 mode's (~7e-2);
* under DETERMINISTIC a captured multi-step graph equals the eager steps bit for bit, so the option
  composes with the timed schedule (rank pass in Adam, fused W1 Adam).
Biases are excluded from gradient comparisons (d loss / d b = 0 under batch-stat BN)."""
import numpy as np
import pytest
import torch

from dssm_amd.data import synth_batch
from oracle import dssm_oracle as O

pytestmark = pytest.mark.gpu

C2 = (30000, (300, 300, 128), 1024, 4)
SMALL = (2000, (40, 64, 32), 128, 4)


def _model(case, p, fused_w1=False):
    from dssm_amd.model import DSSM
    D, widths, BS, NEG = case
    m = DSSM(D, widths, BS, NEG, dtype="bf16", init=False)
    m.set_option("FWD32", True)
    m.load_params(p)
    m.set_fused_w1_adam(fused_w1)
    return m


def _cfg(case):
    D, widths, BS, NEG = case
    return O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)


def _rel(a, b):
    return abs(a - b) / max(abs(b), 1e-30)


@pytest.mark.parametrize("case", [C2, SMALL], ids=["C2", "small"])
def test_fwd32_forward_at_fp32_accuracy(case):
    D, widths, BS, NEG = case
    cfg = _cfg(case)
    p = O.init_params(cfg, seed=21)
    m = _model(case, p)
    f = m.schedule()
    for k in ("FWD32", "FUSED_STATS", "WHOLEK", "MERGED_CSC"):
        assert f[k], (k, f)
    batch = synth_batch(D, BS, NEG, seed=4100, mean_nnz=min(32, D // 4))
    ema0 = O.make_ema(cfg)
    cache, ema1 = O.forward(cfg, p, ema0, batch.as_dict(), True, np.float64)
    m.set_batch(batch)
    m.forward(True)
    torch.cuda.synchronize()
    loss, acc = m.loss_accuracy()
    assert _rel(loss, cache["loss"]) <= 1e-5, (loss, cache["loss"])
    assert acc == pytest.approx(cache["accuracy"])
    np.testing.assert_allclose(m.fetch("cos_sim_raw").ravel(), cache["cos_sim_raw"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(m.fetch("prob"), cache["prob"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(m.fetch("embedding_all"), cache["layers"][-1]["A"], rtol=1e-4, atol=1e-5)
    for l in range(1, len(widths) + 1):
        mo = m.batch_moments(l)
        for t in ("q", "d"):
            np.testing.assert_allclose(mo[t][0], cache["layers"][l - 1]["batch_mean"][t], rtol=1e-4, atol=1e-6)
            np.testing.assert_allclose(mo[t][1], cache["layers"][l - 1]["batch_var"][t], rtol=1e-4, atol=1e-8)
    ge = {k: v.cpu().numpy() for k, v in m.named_ema().items()}
    for k in ema1:
        np.testing.assert_allclose(ge[k], ema1[k], rtol=1e-4, atol=1e-7, err_msg=k)
    # the eval forward (EMA moments, no update) at the same accuracy
    eb = synth_batch(D, BS, NEG, seed=4200, mean_nnz=min(32, D // 4))
    ev = O.forward(cfg, p, ema1, eb.as_dict(), False, np.float64)[0]
    m.set_batch(eb)
    m.forward(False)
    torch.cuda.synchronize()
    assert _rel(m.loss_accuracy()[0], ev["loss"]) <= 1e-5
    np.testing.assert_allclose(m.fetch("cos_sim_raw").ravel(), ev["cos_sim_raw"], rtol=0, atol=1e-5)


def test_fwd32_gradients_at_bf16_accuracy():
    """The backward stays the bf16 mode's kernels, but what it backpropagates through is exact: each
    weight gradient's relative L2 error against the exact gradient is held to 1e-2 (measured 2.8e-3
    -- 3.6e-3 at C2) and below the plain bf16 mode's (6.0e-2 -- 7.7e-2, whose error is mostly its bf16
    forward's, amplified by the batch-stat BN backward)."""
    D, widths, BS, NEG = C2
    cfg = _cfg(C2)
    p = O.init_params(cfg, seed=22)
    batch = synth_batch(D, BS, NEG, seed=4300)
    cache, _ = O.forward(cfg, p, O.make_ema(cfg), batch.as_dict(), True, np.float64)
    grads = O.backward(cfg, p, cache, np.float64)
    errs = {}
    from dssm_amd.model import DSSM
    for mode in ("fwd32", "bf16"):
        m = _model(C2, p) if mode == "fwd32" else DSSM(D, widths, BS, NEG, dtype="bf16", init=False)
        if mode == "bf16":
            m.load_params(p)
            m.set_fused_w1_adam(False)
        m.set_batch(batch)
        m.forward(True)
        m.backward()
        torch.cuda.synchronize()
        gg = {k: v.cpu().numpy().astype(np.float64) for k, v in m.named_grads().items()}
        errs[mode] = {k: float(np.linalg.norm(gg[k] - grads[k]) / np.linalg.norm(grads[k]))
                      for k in ("W1", "W2", "W3")}
    print("relative L2 gradient error", errs)
    for k, e in errs["fwd32"].items():
        assert e <= 1e-2, (k, e)
        assert e <= errs["bf16"][k], (k, e, errs["bf16"][k])


def test_fwd32_graph_equals_eager_bit_for_bit():
    """DETERMINISTIC + FWD32: a captured 3-step graph (rank pass in Adam, fused W1 Adam, the timed
    schedule) equals three eager steps bit for bit."""
    D, widths, BS, NEG = 5000, (300, 300, 128), 128, 4
    case = (D, widths, BS, NEG)
    cfg = _cfg(case)
    p = O.init_params(cfg, seed=23)
    batches = []
    for i in range(3):
        b = synth_batch(D, BS, NEG, seed=4400 + i, mean_nnz=32)
        batches.append(tuple(torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values)))
    runs = []
    for mode in ("graph", "eager"):
        m = _model(case, p, fused_w1=True)
        m.set_option("DETERMINISTIC", True)
        runs.append(m)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g = runs[0].graph_build_steps(batches, probes=False)
        runs[0].graph_launch(g)
        e = runs[1]
        for ip, ix, vv in batches:
            e.set_batch(indptr=ip, indices=ix, values=vv)
            e.forward(True)
            e.backward()
            e.apply_adam(1.0)
    torch.cuda.synchronize()
    m, e = runs
    assert m.schedule()["FWD32"] and m.schedule()["DETERMINISTIC"]
    for x, y in ((m.params, e.params), (m.adam_m, e.adam_m), (m.adam_v, e.adam_v), (m.ema, e.ema)):
        assert torch.equal(x, y)
    assert m.loss_accuracy() == e.loss_accuracy()
