"""CPU oracle for the DSSM two-tower training step — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker.  The product path (``dssm_amd``) never
imports it and fails loudly when its HIP library is missing.

What it restates (NumPy, float64 or float32) — the math of the reference graph
``semantic_matching/dssm/new_dssm.py`` with TensorFlow-1.x op semantics:

* FC1 sparse projection ``X·W1 + b1`` for q/pos/neg with one shared W1
  (new_dssm.py:117-126); dense FC layers ``A·W + b`` shared across towers
  (new_dssm.py:138-148; ``add_layer`` archive/dssm_v3.py:44-53 for the 3-layer form).
* ``batch_normalization`` (new_dssm.py:62-88): ``tf.nn.moments`` over rows (biased var),
  ``ExponentialMovingAverage(decay=0.5)`` applied to the batch moments in training
  (shadow init 0, ``zero_debias=False`` — the TF1.x default for ``apply``),
  ``tf.nn.batch_normalization`` as ``x*inv + (beta - mean*inv)``, ``inv = gamma*rsqrt(var+1e-3)``.
  Query tower and doc tower (concat[pos; neg], new_dssm.py:130) keep separate BN params.
* ReLU after every BN (new_dssm.py:134-136, :156-158).
* Merge_Negative_Doc (new_dssm.py:160-180) restated as the permutation it computes:
  ``doc(j,k) = pos[j]`` for k=0 and ``neg[j*NEG + k-1]`` otherwise.
* Cosine_Similarity (new_dssm.py:182-201): ``cos_sim_raw[k*BS+j]``, ``cos_sim = 20*c``.
* Loss (new_dssm.py:203-213): ``-sum_j log softmax(cos_sim)[j,0] / query_BS``.
* Accuracy (new_dssm.py:219-222): ``mean(argmax_k prob == 0)``.
* Backward: hand-derived gradients of the above (TF autodiff semantics: ReluGrad passes
  where the *output* is > 0; BN backward through batch mean and variance).
* ``AdamOptimizer(lr).minimize(loss)`` (new_dssm.py:215-217) as TF1.x ``ApplyAdam``:
  ``alpha = lr*sqrt(1-beta2^t)/(1-beta1^t)`` with the beta powers kept as float32
  variables multiplied once per step; ``m += (g-m)*(1-beta1)``; ``v += (g*g-v)*(1-beta2)``;
  ``var -= m*alpha/(sqrt(v)+eps)``.  Dense over every trainable variable.

Parity status: **parity unpinned** against TensorFlow.  The reference ships no tests, no
golden vectors and no fixtures, and TensorFlow is not installed (nor installable) here, so
no reference output exists to pin this restatement to.  It is cross-checked instead by
float64 central finite differences and by an independent torch-CPU autograd restatement
(tests/test_oracle.py).  The TF semantics above are documented assumptions.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional

import numpy as np
import scipy.sparse as sp


def bf16_round(x) -> np.ndarray:
    """Round to bfloat16 the way the kernels do: the value is first an fp32 (the kernels hold
    fp32), then ``(__bf16)f`` = round-to-nearest-even on the top 16 bits.  Returned as float64."""
    u = np.ascontiguousarray(np.asarray(x, np.float32)).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def _rw(a, emulate):
    """Operand as the matrix cores see it: bf16 under ``emulate == "bf16"``, unchanged otherwise."""
    return bf16_round(a) if emulate == "bf16" else a


@dataclasses.dataclass
class OracleConfig:
    trigram_d: int
    widths: List[int]
    query_bs: int
    neg: int = 4
    lr: float = 0.01
    gamma: float = 20.0
    bn_eps: float = 1e-3
    ema_decay: float = 0.5
    beta1: float = 0.9
    beta2: float = 0.999
    adam_eps: float = 1e-8

    @property
    def rows(self) -> int:
        return self.query_bs * (2 + self.neg)

    @property
    def n_layers(self) -> int:
        return len(self.widths)


def param_names(cfg: OracleConfig) -> List[str]:
    """Trainable variables in arena order (W_l, b_l per layer, then BN gamma/beta per tower)."""
    names = []
    for l in range(1, cfg.n_layers + 1):
        names += [f"W{l}", f"b{l}"]
    for l in range(1, cfg.n_layers + 1):
        for t in ("q", "d"):
            names += [f"bn{l}_{t}_gamma", f"bn{l}_{t}_beta"]
    return names


def ema_names(cfg: OracleConfig) -> List[str]:
    out = []
    for l in range(1, cfg.n_layers + 1):
        for t in ("q", "d"):
            out += [f"bn{l}_{t}_mean", f"bn{l}_{t}_var"]
    return out


def init_params(cfg: OracleConfig, seed: int = 0) -> Dict[str, np.ndarray]:
    """Reference init (new_dssm.py:118-120, :139-142, :75-76): W,b ~ U(-r, r) with
    r = sqrt(6/(fan_in+fan_out)) for the bias too; gamma=1, beta=0.  Drawn from numpy
    PCG64(seed) in the order W1, b1, W2, b2, ... as float32."""
    rng = np.random.Generator(np.random.PCG64(seed))
    p = {}
    dims = [cfg.trigram_d] + list(cfg.widths)
    for l in range(1, cfg.n_layers + 1):
        fi, fo = dims[l - 1], dims[l]
        r = np.sqrt(6.0 / (fi + fo))
        p[f"W{l}"] = rng.uniform(-r, r, size=(fi, fo)).astype(np.float32)
        p[f"b{l}"] = rng.uniform(-r, r, size=(fo,)).astype(np.float32)
    for l in range(1, cfg.n_layers + 1):
        n = dims[l]
        for t in ("q", "d"):
            p[f"bn{l}_{t}_gamma"] = np.ones(n, np.float32)
            p[f"bn{l}_{t}_beta"] = np.zeros(n, np.float32)
    return p


def csr_matrix(indptr, indices, values, rows, d, dtype):
    return sp.csr_matrix((np.asarray(values, dtype=dtype), np.asarray(indices), np.asarray(indptr)),
                         shape=(rows, d))


def towers_of(cfg: OracleConfig):
    """Row ranges of the two BN towers: query rows, then doc rows = concat[pos; neg]
    (new_dssm.py:128-132)."""
    return {"q": slice(0, cfg.query_bs), "d": slice(cfg.query_bs, cfg.rows)}


def bn_relu_forward(cfg: OracleConfig, Z, params, l: int, ema, new_ema=None, dtype=np.float64):
    """``batch_normalization`` + ReLU of layer l (new_dssm.py:62-88, :134-136) on Z [R x n] per
    tower.  ``new_ema`` given (train): batch moments, EMA update into ``new_ema``; otherwise the
    shadows in ``ema`` (new_dssm.py:85-86).  Returns the layer cache {Z, Y, A, mu, var, r, inv,
    batch_mean, batch_var}."""
    dt = dtype
    Z = np.asarray(Z, dt)
    Y = np.empty_like(Z)
    lc = {"Z": Z, "mu": {}, "var": {}, "inv": {}, "r": {}, "batch_mean": {}, "batch_var": {}}
    for t, sl in towers_of(cfg).items():
        z = Z[sl]
        bmean = z.mean(axis=0)
        bvar = ((z - bmean) ** 2).mean(axis=0)
        if new_ema is not None:
            for nm, val in (("mean", bmean), ("var", bvar)):
                key = f"bn{l}_{t}_{nm}"
                s = new_ema[key].astype(dt)
                new_ema[key] = (s - (s - val) * (1.0 - cfg.ema_decay)).astype(np.float32)
            mu, var = bmean, bvar
        else:
            mu = ema[f"bn{l}_{t}_mean"].astype(dt)
            var = ema[f"bn{l}_{t}_var"].astype(dt)
        r = 1.0 / np.sqrt(var + cfg.bn_eps)
        inv = r * params[f"bn{l}_{t}_gamma"].astype(dt)
        Y[sl] = z * inv + (params[f"bn{l}_{t}_beta"].astype(dt) - mu * inv)
        lc["mu"][t], lc["var"][t], lc["inv"][t], lc["r"][t] = mu, var, inv, r
        lc["batch_mean"][t], lc["batch_var"][t] = bmean, bvar
    lc["Y"], lc["A"] = Y, np.maximum(Y, 0)
    return lc


def cosine_loss_forward(cfg: OracleConfig, A, dtype=np.float64):
    """Merge_Negative_Doc + Cosine_Similarity + softmax loss + accuracy (new_dssm.py:160-222) on
    the embeddings A [R x n] = rows [q; pos; neg]."""
    dt = dtype
    BS, NEG = cfg.query_bs, cfg.neg
    A = np.asarray(A, dt)
    yq, yp, yn = A[:BS], A[BS:2 * BS], A[2 * BS:]
    # Merge_Negative_Doc as a permutation: doc[k][j]
    docs = [yp] + [yn[k - 1::NEG] for k in range(1, NEG + 1)]
    qn = np.sqrt((yq * yq).sum(1))
    c = np.empty((BS, NEG + 1), dt)
    dn = np.empty((BS, NEG + 1), dt)
    for k, dk in enumerate(docs):
        dn[:, k] = np.sqrt((dk * dk).sum(1))
        c[:, k] = (yq * dk).sum(1) / (qn * dn[:, k])
    cos_sim = cfg.gamma * c
    smax = cos_sim - cos_sim.max(1, keepdims=True)
    e = np.exp(smax)
    prob = e / e.sum(1, keepdims=True)
    loss = -np.log(prob[:, 0]).sum() / BS
    acc = float((np.argmax(prob, 1) == 0).mean())
    return dict(yq=yq, docs=docs, qn=qn, dn=dn, c=c, cos_sim=cos_sim, prob=prob,
                cos_sim_raw=c.T.reshape(-1).copy(), loss=float(loss), accuracy=acc,
                query_norm_single=qn)


def cosine_loss_backward(cfg: OracleConfig, cc, dtype=np.float64):
    """d loss / d embeddings [R x n] from a cosine_loss_forward result (TF autodiff of
    new_dssm.py:182-209; the merge's gradient scatters back to the pos / neg rows)."""
    BS, NEG, R = cfg.query_bs, cfg.neg, cfg.rows
    prob, c, qn, dn = cc["prob"], cc["c"], cc["qn"], cc["dn"]
    yq, docs = cc["yq"], cc["docs"]
    ds = prob.copy()
    ds[:, 0] -= 1.0
    ds /= BS
    dc = cfg.gamma * ds
    dyq = np.zeros_like(yq)
    ddocs = []
    for k, dk in enumerate(docs):
        inv_nn = 1.0 / (qn * dn[:, k])
        ck = c[:, k]
        dyq += dc[:, k:k + 1] * (dk * inv_nn[:, None] - (ck / (qn * qn))[:, None] * yq)
        ddocs.append(dc[:, k:k + 1] * (yq * inv_nn[:, None] - (ck / (dn[:, k] ** 2))[:, None] * dk))
    dA = np.empty((R, yq.shape[1]), dtype)
    dA[:BS] = dyq
    dA[BS:2 * BS] = ddocs[0]
    for k in range(1, NEG + 1):
        dA[2 * BS + (k - 1)::NEG] = ddocs[k]
    return dA


def bn_relu_backward(cfg: OracleConfig, lc, dA, l: int):
    """Backward of bn_relu_forward (train mode) for d loss / d A: ReluGrad on the output (> 0),
    then the batch-statistic BN gradient.  Returns (dZ, {bn{l}_{t}_gamma / _beta: grads})."""
    Z, Y = lc["Z"], lc["Y"]
    dY = dA * (Y > 0)
    dZ = np.empty_like(Z)
    g = {}
    for t, sl in towers_of(cfg).items():
        n = sl.stop - sl.start
        xhat = (Z[sl] - lc["mu"][t]) * lc["r"][t]
        dy = dY[sl]
        dbeta = dy.sum(0)
        dgamma = (dy * xhat).sum(0)
        g[f"bn{l}_{t}_beta"] = dbeta
        g[f"bn{l}_{t}_gamma"] = dgamma
        dZ[sl] = lc["inv"][t] * (dy - dbeta / n - xhat * (dgamma / n))
    return dZ, g


def forward(cfg: OracleConfig, params, ema, batch, train: bool = True, dtype=np.float64,
            emulate: Optional[str] = None):
    """Forward pass; returns (cache, new_ema).  ``batch`` = dict(indptr, indices, values) of the
    combined CSR over rows [q(BS); pos(BS); neg(BS*NEG)] (utils/utils.py:45-61 slicing).

    ``emulate="bf16"`` restates the GPU perf mode's roundings (not a reference behaviour: the
    reference is fp32 throughout, new_dssm.py:111-114): every weight W_l is read as its bf16
    shadow, and each hidden layer's post-BN/ReLU activation is rounded to bf16 before it feeds
    the next layer's product (the last layer's embeddings stay fp32).  Everything else --
    BN statistics, cosine, softmax, loss -- is computed as in fp32 mode."""
    dt = dtype
    X = csr_matrix(batch["indptr"], batch["indices"], batch["values"], cfg.rows, cfg.trigram_d, dt)
    cache = {"X": X, "layers": [], "emulate": emulate}
    new_ema = {k: v.copy() for k, v in ema.items()}
    A = None
    for l in range(1, cfg.n_layers + 1):
        W = _rw(params[f"W{l}"], emulate).astype(dt)
        b = params[f"b{l}"].astype(dt)
        Z = (X @ W if l == 1 else A @ W) + b
        lc = bn_relu_forward(cfg, Z, params, l, ema, new_ema if train else None, dt)
        lc["A_in"] = A
        A = lc["A"]
        if l < cfg.n_layers:
            A = _rw(A, emulate).astype(dt)  # the next product's operand (bf16 in perf mode)
        cache["layers"].append(lc)
    cache.update(cosine_loss_forward(cfg, A, dt))
    return cache, new_ema


def backward(cfg: OracleConfig, params, cache, dtype=np.float64):
    """Gradients of the loss w.r.t. every trainable variable (dict keyed like params).

    Under the forward's ``emulate="bf16"`` every dZ_l is rounded to bf16 before it enters a
    product (dW_l = A_{l-1}^T dZ_l, dA_{l-1} = dZ_l W_l^T with W_l's bf16 shadow, dW1 = X^T dZ_1),
    as the GPU perf mode stores it; BN's dgamma / dbeta use the unrounded fp32 dy."""
    dt = dtype
    emulate = cache.get("emulate")
    dA = cosine_loss_backward(cfg, cache, dt)
    grads = {}
    for l in range(cfg.n_layers, 0, -1):
        lc = cache["layers"][l - 1]
        dZ, bg = bn_relu_backward(cfg, lc, dA, l)
        grads.update(bg)
        dZ = _rw(dZ, emulate).astype(dt)
        grads[f"b{l}"] = dZ.sum(0)
        if l == 1:
            grads["W1"] = np.asarray(cache["X"].T @ dZ)
        else:
            grads[f"W{l}"] = lc["A_in"].T @ dZ
            dA = dZ @ _rw(params[f"W{l}"], emulate).astype(dt).T
    return grads


def forward_eval_loss(cfg, params, ema, batch, dtype=np.float64):
    cache, _ = forward(cfg, params, ema, batch, train=False, dtype=dtype)
    return cache


class AdamState:
    """TF1.x AdamOptimizer slots + float32 beta-power accumulators."""

    def __init__(self, cfg: OracleConfig, params):
        self.cfg = cfg
        self.m = {k: np.zeros_like(v, np.float32) for k, v in params.items()}
        self.v = {k: np.zeros_like(v, np.float32) for k, v in params.items()}
        self.beta1_power = np.float32(cfg.beta1)
        self.beta2_power = np.float32(cfg.beta2)
        self.t = 0

    def alpha(self) -> np.float32:
        cfg = self.cfg
        one = np.float32(1.0)
        return np.float32(np.float32(cfg.lr) * np.sqrt(one - self.beta2_power) / (one - self.beta1_power))

    def step(self, params, grads, grad_scale: float = 1.0, dtype=np.float32):
        """In-place ApplyAdam over every variable; float32 arithmetic like the TF kernel."""
        cfg = self.cfg
        a = self.alpha()
        one = np.float32(1.0)
        b1c = one - np.float32(cfg.beta1)  # T(1) - beta1() in the fp32 ApplyAdam functor
        b2c = one - np.float32(cfg.beta2)
        eps = np.float32(cfg.adam_eps)
        for k in params:
            g = (np.asarray(grads[k], np.float64) * grad_scale).astype(np.float32)
            m, v = self.m[k], self.v[k]
            m += (g - m) * b1c
            v += (g * g - v) * b2c
            params[k] -= (m * a) / (np.sqrt(v) + eps)
        self.beta1_power = np.float32(self.beta1_power * np.float32(cfg.beta1))
        self.beta2_power = np.float32(self.beta2_power * np.float32(cfg.beta2))
        self.t += 1


def make_ema(cfg: OracleConfig) -> Dict[str, np.ndarray]:
    ema = {}
    for l in range(1, cfg.n_layers + 1):
        for t in ("q", "d"):
            ema[f"bn{l}_{t}_mean"] = np.zeros(cfg.widths[l - 1], np.float32)
            ema[f"bn{l}_{t}_var"] = np.zeros(cfg.widths[l - 1], np.float32)
    return ema


def train_step(cfg: OracleConfig, params, ema, adam: AdamState, batch, dtype=np.float64,
               emulate: Optional[str] = None):
    """One ``sess.run(train_step)`` (new_dssm.py:267): forward (EMA update), backward, Adam.
    Mutates params/adam in place; returns (cache, grads, new_ema)."""
    cache, new_ema = forward(cfg, params, ema, batch, train=True, dtype=dtype, emulate=emulate)
    grads = backward(cfg, params, cache, dtype=dtype)
    adam.step(params, grads)
    return cache, grads, new_ema


def auc_streaming(labels: np.ndarray, preds: np.ndarray, num_thresholds: int = 2000,
                  state: Optional[dict] = None):
    """tf.metrics.auc (new_dssm.py:230) confusion-count accumulation + trapezoid AUC.
    TF1.x thresholds: [-eps, (i)/(n-1) for i in 1..n-2, 1+eps] with eps=1e-7; predictions
    are compared as ``pred > thr``.  Returns (auc, state)."""
    eps = 1e-7
    thr = np.array([-eps] + [(i + 1) / (num_thresholds - 1) for i in range(num_thresholds - 2)]
                   + [1.0 + eps])
    if state is None:
        state = {k: np.zeros(num_thresholds, np.float64) for k in ("tp", "fn", "tn", "fp")}
    lab = labels.astype(bool)
    gt = preds[None, :] > thr[:, None]
    state["tp"] += (gt & lab[None, :]).sum(1)
    state["fp"] += (gt & ~lab[None, :]).sum(1)
    state["fn"] += (~gt & lab[None, :]).sum(1)
    state["tn"] += (~gt & ~lab[None, :]).sum(1)
    e = 1e-7
    tpr = (state["tp"] + e) / (state["tp"] + state["fn"] + e)
    fpr = state["fp"] / (state["fp"] + state["tn"] + e)
    auc = float(np.sum((fpr[:-1] - fpr[1:]) * (tpr[:-1] + tpr[1:]) / 2.0))
    return auc, state
