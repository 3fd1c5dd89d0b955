"""The fp32 parity mode's fused schedule at the headline shape, against the float64 oracle.

fp32 mode is the reference's own precision (new_dssm.py:111-114: tf.float32 placeholders and
variables).  At BASELINE config 2 (D=30000, widths 300/300/128, BS=1024, NEG=4) it runs the same
launch structure as the bf16 perf mode -- fused BN statistics (fp64 column sums in the producers,
coefficients derived by the consumers), the merged CSC transpose, dW1 inside Adam -- with the dense
layers on the fp32 tiles of csrc/g32.h.  The default build forms their products on the bf16 matrix
cores from an exact three-way split of each fp32 operand (x = h + m + l, six partial products
hh, hm, mh, hl, lh, mm on v_mfma_f32_16x16x32_bf16 with fp32 accumulation: the dropped terms are
< 2^-22 |ab|, about one fp32 rounding per product); -DDSSM_G32_SPLIT=0 builds the exact
v_mfma_f32_16x16x4_f32 FMA chains instead.  Both are held to the bars below:

1. **Kernel chain, teacher-forced** (``test_fp32_kernel_chain``): every product of one step
   recomputed by the oracle's per-op functions in float64 from the GPU's own inputs to that op
   (Z_l, A_l, dA_l, dZ_l read back through DSSM_BUF_*): max error <= 1e-5 x the row's / tensor's
   max magnitude for every output (fp32 storage and accumulation only, no bf16 rounding point);
   the cosine backward's dy, whose two terms cancel, per row at >= 1% of the tensor's max scale.
2. **The fused step against the separate-statistics fp32 schedule** (plan option FUSED_STATS off:
   fp32-partial statistics launches, the unfused GEMMs) on the same state and batch.
3. **Teacher-forced fused Adam** against the oracle's ApplyAdam on the GPU's own unfused
   gradients, from a mid-training state.
4. **One end-to-end step against the oracle** (no teacher forcing): loss and cosines <= 1e-5,
   gradients <= 1e-4 x max|g| (the north star's 1e-4 on loss and cosine scores, with margin).
Biases are excluded element-wise: under batch-stat BN d loss / d b is exactly 0 (test_oracle.py).
"""
import re

import numpy as np
import pytest
import torch

from dssm_amd import _lib
from dssm_amd.data import synth_batch
from oracle import dssm_oracle as O
from tests.test_gpu_parity import align_relu_ties

pytestmark = pytest.mark.gpu

C2 = (30000, (300, 300, 128), 1024, 4)
SMALL = (2000, (40, 64, 32), 128, 4)  # K < 64 chunks, widths not multiples of 64
CASES = [C2, SMALL]
IDS = ["C2", "small"]


def _is_bias(k):
    return re.fullmatch(r"b\d+", k) is not None


def _rel(a, b):
    return abs(a - b) / max(abs(b), 1e-30)


def _cfg(case):
    D, widths, BS, NEG = case
    return O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)


def _model(case, p, fused=False, fused_stats=True):
    from dssm_amd.model import DSSM
    D, widths, BS, NEG = case
    m = DSSM(D, widths, BS, NEG, dtype="fp32", init=False)
    m.load_params(p)
    m.set_fused_w1_adam(fused)
    m.set_option("FUSED_STATS", fused_stats)
    return m


def _expect_fused(m):
    f = m.schedule()
    want = ["FUSED_STATS", "MERGED_CSC", "HEAVY_IN_ADAM", "NT32", "DW_IN_APPLY", "SCATTER_IN_COS"]
    missing = [w for w in want if not f.get(w)]
    assert not missing, (missing, f)


def _layer(m, bid, l, n):
    ld = (n + 7) // 8 * 8
    t = m.buffer(bid, l, dtype=torch.float32)
    return t.cpu().numpy().astype(np.float64).reshape(m.rows, ld)[:, :n]


def _rowmax_err(got, ref):
    scale = np.abs(ref).max(axis=-1, keepdims=True) if np.ndim(ref) > 1 else np.abs(ref).max()
    return float((np.abs(got - ref) / np.maximum(scale, 1e-30)).max())


def _rowmax_err_floor(got, ref, floor=1e-2):
    """_rowmax_err with each row's scale floored at floor x the tensor's max: a row whose values
    are all tiny (a confidently classified query's dy) is compared at the tensor's scale."""
    scale = np.maximum(np.abs(ref).max(axis=-1, keepdims=True), floor * np.abs(ref).max())
    return float((np.abs(got - ref) / np.maximum(scale, 1e-30)).max())


def _tensor_err(got, ref):
    return float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))


def _report(tag, errs):
    bad = {k: v for k, v in errs.items() if not v[0] <= v[1]}
    worst = sorted(errs.items(), key=lambda kv: -kv[1][0] / kv[1][1])[:8]
    print(f"\n[{tag}] worst error/bar: " + ", ".join(f"{k}={e:.2e}/{b:.0e}" for k, (e, b) in worst))
    assert not bad, f"{tag}: over the bar: {bad}"


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_fp32_kernel_chain(case):
    """Each kernel of the fused fp32 step against the oracle fed that kernel's GPU inputs: 1e-5."""
    D, widths, BS, NEG = case
    cfg = _cfg(case)
    L = len(widths)
    p = O.init_params(cfg, seed=11)
    batch = synth_batch(D, BS, NEG, seed=1000, mean_nnz=min(32, D // 4))
    m = _model(case, p)
    _expect_fused(m)
    m.set_batch(batch)
    m.forward(True)
    m.backward()
    torch.cuda.synchronize()
    X = O.csr_matrix(batch.indptr, batch.indices, batch.values, cfg.rows, D, np.float64)
    W = {l: p[f"W{l}"].astype(np.float64) for l in range(1, L + 1)}
    errs = {}
    Z = [_layer(m, _lib.BUF_Z, l, widths[l]) for l in range(L)]
    A = [_layer(m, _lib.BUF_A, l, widths[l]) for l in range(L)]
    ema = O.make_ema(cfg)
    lcs = []
    for l in range(L):
        a_in = X if l == 0 else A[l - 1]
        z_ref = np.asarray(a_in @ W[l + 1]) + p[f"b{l + 1}"]
        errs[f"Z{l + 1}"] = (_rowmax_err(Z[l], z_ref), 1e-5)
        lc = O.bn_relu_forward(cfg, Z[l], p, l + 1, ema, ema)
        lcs.append(lc)
        mo = m.batch_moments(l + 1)
        for t in ("q", "d"):
            errs[f"bn{l + 1}_{t}_mean"] = (_tensor_err(mo[t][0], lc["batch_mean"][t]), 1e-5)
            errs[f"bn{l + 1}_{t}_var"] = (_tensor_err(mo[t][1], lc["batch_var"][t]), 1e-5)
        errs[f"A{l + 1}"] = (_rowmax_err(A[l], lc["A"]), 1e-5)
    ge = {k: v.cpu().numpy() for k, v in m.named_ema().items()}
    for k in ema:
        errs[f"ema_{k}"] = (_tensor_err(ge[k], ema[k]), 1e-5)
    cc = O.cosine_loss_forward(cfg, A[L - 1])
    errs["loss"] = (_rel(m.loss_accuracy()[0], cc["loss"]), 1e-5)
    errs["cos_sim_raw"] = (float(np.abs(m.fetch("cos_sim_raw").ravel() - cc["cos_sim_raw"]).max()), 1e-5)
    errs["prob"] = (float(np.abs(m.fetch("prob") - cc["prob"]).max()), 1e-5)
    errs["query_norm"] = (_tensor_err(m.fetch("query_norm_single").ravel(), cc["qn"]), 1e-5)
    dA = _layer(m, _lib.BUF_DA, L - 1, widths[-1])
    # dy = a * d - b * q per element cancels: in a row whose softmax is nearly one-hot its values
    # are tiny against the terms (measured 1.1e-5 of the row max at C2, 3.3e-5 at width 32): the
    # cosine kernel's fp32 arithmetic, shared with the bf16 mode; its rows compared at >= 1% of the
    # tensor's max
    errs["dy"] = (_rowmax_err_floor(dA, O.cosine_loss_backward(cfg, cc)), 1e-5)
    gg = {k: v.cpu().numpy().astype(np.float64) for k, v in m.named_grads().items()}
    for l in range(L - 1, -1, -1):
        dA = _layer(m, _lib.BUF_DA, l, widths[l])
        dz_exact, bg = O.bn_relu_backward(cfg, lcs[l], dA, l + 1)
        for k, g in bg.items():
            errs[f"grad_{k}"] = (_tensor_err(gg[k], g), 1e-5)
        dZ = _layer(m, _lib.BUF_DZ, l, widths[l])
        errs[f"dZ{l + 1}"] = (_rowmax_err(dZ, dz_exact), 1e-5)
        a_in = X if l == 0 else A[l - 1]
        errs[f"grad_W{l + 1}"] = (_tensor_err(gg[f"W{l + 1}"], np.asarray(a_in.T @ dZ)), 1e-5)
        db = dZ.sum(0)
        errs[f"grad_b{l + 1}"] = (float(np.abs(gg[f"b{l + 1}"] - db).max() / np.abs(dZ).sum(0).max()), 1e-5)
        if l > 0:
            da_ref = dZ @ W[l + 1].T
            errs[f"dA{l}"] = (_rowmax_err(_layer(m, _lib.BUF_DA, l - 1, widths[l - 1]), da_ref), 1e-5)
    _report(f"fp32 chain {case}", errs)


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_fp32_fused_matches_oracle_end_to_end(case):
    """One fused step against the float64 oracle with no teacher forcing."""
    D, widths, BS, NEG = case
    cfg = _cfg(case)
    p = O.init_params(cfg, seed=11)
    batch = synth_batch(D, BS, NEG, seed=1000, mean_nnz=min(32, D // 4))
    cache, _ = O.forward(cfg, p, O.make_ema(cfg), batch.as_dict(), True, np.float64)
    m = _model(case, p)
    _expect_fused(m)
    m.set_batch(batch)
    m.forward(True)
    m.backward()
    torch.cuda.synchronize()
    # elements on a ReLU boundary at fp32 resolution take the GPU's side (tests/test_gpu_parity.py)
    ties = align_relu_ties(m, cache, widths)
    assert ties <= 1e-5 * m.rows * sum(widths), ties
    grads = O.backward(cfg, p, cache, np.float64)
    errs = {"loss": (_rel(m.loss_accuracy()[0], cache["loss"]), 1e-5),
            "cos_sim_raw": (float(np.abs(m.fetch("cos_sim_raw").ravel() - cache["cos_sim_raw"]).max()), 1e-5),
            "prob": (float(np.abs(m.fetch("prob") - cache["prob"]).max()), 1e-5)}
    gg = {k: v.cpu().numpy() for k, v in m.named_grads().items()}
    for k, g in grads.items():
        if not _is_bias(k):
            errs[f"grad_{k}"] = (_tensor_err(gg[k], g), 1e-4)
    _report(f"fp32 end-to-end {case}", errs)


def test_fp32_fused_matches_separate_statistics():
    """The fused fp32 step against the separate-statistics fp32 schedule on the same state and batch:
    the forward reads no transpose, so the loss agrees to fp32 rounding of the statistics; every
    non-bias gradient <= 1e-5 x max|g|."""
    case = C2
    D, widths, BS, NEG = case
    cfg = _cfg(case)
    p = O.init_params(cfg, seed=12)
    batch = synth_batch(D, BS, NEG, seed=1002)
    a, b = _model(case, p, fused_stats=True), _model(case, p, fused_stats=False)
    _expect_fused(a)
    assert not b.schedule()["FUSED_STATS"] and not b.schedule()["NT32"]
    for m in (a, b):
        m.set_batch(batch)
        m.forward(True)
        m.backward()
    torch.cuda.synchronize()
    errs = {"loss": (_rel(a.loss_accuracy()[0], b.loss_accuracy()[0]), 2e-6)}
    ga = {k: v.cpu().numpy() for k, v in a.named_grads().items()}
    gb = {k: v.cpu().numpy() for k, v in b.named_grads().items()}
    for k in gb:
        if not _is_bias(k):
            errs[f"grad_{k}"] = (_tensor_err(ga[k], gb[k]), 1e-5)
    _report("fused vs separate fp32", errs)


def test_fp32_fused_adam_step_teacher_forced():
    """The timed fp32 step (fused statistics + dW1 / dW_l slabs inside Adam) from a mid-training
    state against the oracle's ApplyAdam on the gradients the unfused-Adam schedule computes."""
    case = C2
    D, widths, BS, NEG = case
    cfg = _cfg(case)
    p = O.init_params(cfg, seed=11)
    adam = O.AdamState(cfg, p)
    _, _, ema = O.train_step(cfg, p, O.make_ema(cfg), adam, synth_batch(D, BS, NEG, seed=999).as_dict(), np.float64)
    batch = synth_batch(D, BS, NEG, seed=1001)
    models = {}
    for fused in (False, True):
        mm = _model(case, p, fused=fused)
        mm.load_params(p, ema=ema)
        mm.load_adam_state(adam.m, adam.v, adam.beta1_power, adam.beta2_power, adam.t)
        mm.set_batch(batch)
        models[fused] = mm
    mu = models[False]
    mu.forward(True)
    mu.backward()
    torch.cuda.synchronize()
    g_gpu = {k: v.cpu().numpy().astype(np.float64) for k, v in mu.named_grads().items()}
    mf = models[True]
    _expect_fused(mf)
    assert mf.schedule()["FUSED_W1_ADAM"]
    mf.train_step()
    torch.cuda.synchronize()
    errs = {"loss_fused_vs_unfused": (_rel(mf.loss_accuracy()[0], mu.loss_accuracy()[0]), 1e-6)}
    adam.step(p, g_gpu)
    gp = {k: v.cpu().numpy() for k, v in mf.named_params().items()}
    gm, gv = mf.named_adam()
    lr = cfg.lr
    for k in p:
        if _is_bias(k):
            continue
        d = np.abs(gp[k] - p[k])
        well = np.abs(g_gpu[k]) > 1e-3 * np.abs(g_gpu[k]).max()
        errs[f"param_{k}_well"] = (float(d[well].max(initial=0.0)), 1e-6 + 1e-4 * lr)
        errs[f"param_{k}_all"] = (float(d.max()), 2 * lr)
        errs[f"m_{k}"] = (_tensor_err(gm[k].cpu().numpy(), adam.m[k]), 1e-5)
        errs[f"v_{k}"] = (_tensor_err(gv[k].cpu().numpy(), adam.v[k]), 1e-5)
    assert mf.beta_powers() == (adam.beta1_power, adam.beta2_power)
    _report("fp32 fused adam", errs)


def test_fp32_fused_deterministic_graph_bit_identical():
    """DETERMINISTIC fp32: a 3-step captured graph (rank passes inside Adam) equals 3 eager steps bit
    for bit, and two graph runs equal each other."""
    D, widths, BS, NEG = C2
    cfg = _cfg(C2)
    p = O.init_params(cfg, seed=3)
    dev = torch.device("cuda:0")
    hb = [synth_batch(D, BS, NEG, seed=40 + i) for i in range(3)]
    staged = [(torch.from_numpy(x.indptr).to(dev), torch.from_numpy(x.indices).to(dev),
               torch.from_numpy(x.values).to(dev)) for x in hb]
    runs = []
    for mode in ("graph", "eager"):
        m = _model(C2, p, fused=True)
        m.set_option("DETERMINISTIC", True)
        _expect_fused(m)
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            if mode == "graph":
                m.graph_launch(m.graph_build_steps(staged, stream=s), stream=s)
            else:
                for ip, ix, vv in staged:
                    m.set_batch(indptr=ip, indices=ix, values=vv)
                    m.train_step()
        s.synchronize()
        runs.append(m)
    a, b = runs
    for name in ("params", "adam_m", "adam_v", "ema"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert a.loss_accuracy() == b.loss_accuracy()
