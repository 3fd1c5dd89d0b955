"""TEST INFRASTRUCTURE ONLY: NumPy float64 restatement of the reference's multi-view DSSM
(archive/multi_view_dssm_v3.py:107-241), the checker for dssm_amd/multiview.py.

* one user tower and three item-view towers, each sparse FC1 + ReLU + FC2 + ReLU (no batch norm;
  W, b ~ U(-r, r), r = sqrt(6 / (fan_in + fan_out)), :115-185);
* the active view's item embeddings are the positives; negative i of user j is item row
  (j + rand_i) mod BS -- the in-batch rotation of Make_Negative_Item (:196-214), with the offsets
  rand_i = int((u_i + i) * BS / NEG) given as inputs;
* x20 cosine, softmax, loss = -sum_j log p[j, 0] (summed, :216-235);
* Adam (TF1.x ApplyAdam) on the user tower and the active view only: the other views' variables
  get no gradient, which TF's minimize() skips.
The reference picks the view with a Python comparison against a placeholder at graph build
(always view 3); this restatement uses the fed active view, as intended.

emulate="bf16" restates the bf16 perf mode of dssm_amd/multiview.py: the weight operands W1, W2
(the shadows), FC1's ReLU output and the backward's dz2, dz1 rounded to bfloat16 (RNE) exactly where
the kernels store them; everything else float64.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List

import numpy as np

from .dssm_oracle import bf16_round


@dataclasses.dataclass
class MvConfig:
    user_d: int
    view_d: List[int]
    l1: int
    l2: int
    bs: int
    neg: int = 4
    gamma: float = 20.0
    lr: float = 0.05


def towers(cfg: MvConfig):
    return ["user", "view1", "view2", "view3"]


def init_params(cfg: MvConfig, seed: int = 0) -> Dict[str, np.ndarray]:
    rng = np.random.Generator(np.random.PCG64(seed))
    p = {}
    for t, d in zip(towers(cfg), [cfg.user_d] + list(cfg.view_d)):
        for l, (a, b) in enumerate(((d, cfg.l1), (cfg.l1, cfg.l2)), 1):
            r = np.sqrt(6.0 / (a + b))
            p[f"{t}_W{l}"] = rng.uniform(-r, r, size=(a, b)).astype(np.float32)
            p[f"{t}_b{l}"] = rng.uniform(-r, r, size=b).astype(np.float32)
    return p


def rotations(cfg: MvConfig, seed: int) -> np.ndarray:
    u = np.random.Generator(np.random.PCG64(seed)).random(cfg.neg)
    return np.array([int((u[i] + i) * cfg.bs / cfg.neg) for i in range(cfg.neg)], np.int32)


def _dense(csr, d):
    ip, ix, vv = csr
    X = np.zeros((len(ip) - 1, d))
    for r in range(len(ip) - 1):
        X[r, ix[ip[r]:ip[r + 1]]] += vv[ip[r]:ip[r + 1]]
    return X


def _rw(a, emulate):
    return bf16_round(a) if emulate == "bf16" else a


def tower(p, t, X, emulate=None):
    z1 = X @ _rw(p[f"{t}_W1"], emulate) + p[f"{t}_b1"]
    a1 = _rw(np.maximum(z1, 0), emulate)  # bf16 mode: FC1's activation is stored bf16
    z2 = a1 @ _rw(p[f"{t}_W2"], emulate) + p[f"{t}_b2"]
    return {"X": X, "z1": z1, "a1": a1, "z2": z2, "y": np.maximum(z2, 0)}


def forward(cfg: MvConfig, p, user_csr, item_csr, view: int, rot, dtype=np.float64, sparse=False,
            emulate=None):
    """dtype float64 with dense X: the parity oracle.  float32 with sparse (scipy CSR) X: the CPU
    baseline's restatement (bench.py --model multiview).  emulate="bf16": the bf16 mode's rounding
    points (module doc)."""
    p = {k: v.astype(dtype) for k, v in p.items()}
    dims = [cfg.user_d] + list(cfg.view_d)
    if sparse:
        import scipy.sparse as sps
        X = [sps.csr_matrix((np.asarray(c[2], dtype), c[1], c[0]), shape=(cfg.bs, d))
             for c, d in ((user_csr, dims[0]), (item_csr, dims[view]))]
    else:
        X = [_dense(user_csr, dims[0]), _dense(item_csr, dims[view])]
    u = tower(p, "user", X[0], emulate)
    it = tower(p, f"view{view}", X[1], emulate)
    BS, K = cfg.bs, cfg.neg + 1
    idx = np.empty((K, BS), np.int64)
    idx[0] = np.arange(BS)
    for i in range(cfg.neg):
        idx[i + 1] = (np.arange(BS) + rot[i]) % BS
    yq, doc = u["y"], it["y"][idx]                   # doc [K, BS, L]
    qn, dn = np.linalg.norm(yq, axis=1), np.linalg.norm(doc, axis=2)
    c = np.einsum("jc,kjc->jk", yq, doc) / (qn[:, None] * dn.T)
    s = cfg.gamma * c
    e = np.exp(s - s.max(1, keepdims=True))
    prob = e / e.sum(1, keepdims=True)
    return {"u": u, "it": it, "idx": idx, "doc": doc, "qn": qn, "dn": dn, "cos": c, "prob": prob,
            "loss": -np.sum(np.log(prob[:, 0])), "view": view, "emulate": emulate}


def backward(cfg: MvConfig, p, fw) -> Dict[str, np.ndarray]:
    p = {k: v.astype(fw["u"]["y"].dtype) for k, v in p.items()}
    BS, K, g = cfg.bs, cfg.neg + 1, cfg.gamma
    yq, doc, c, qn, dn, prob = fw["u"]["y"], fw["doc"], fw["cos"], fw["qn"], fw["dn"], fw["prob"]
    dcos = (prob - np.eye(K)[0][None, :]) * g
    dyq = np.zeros_like(yq)
    dyi = np.zeros_like(fw["it"]["y"])
    for k in range(K):
        a = dcos[:, k][:, None]
        dyq += a * (doc[k] / (qn[:, None] * dn[k][:, None]) - c[:, k][:, None] * yq / qn[:, None] ** 2)
        dd = a * (yq / (qn[:, None] * dn[k][:, None]) - c[:, k][:, None] * doc[k] / dn[k][:, None] ** 2)
        np.add.at(dyi, fw["idx"][k], dd)
    grads = {}
    em = fw.get("emulate")
    for t, tw, dy in (("user", fw["u"], dyq), (f"view{fw['view']}", fw["it"], dyi)):
        dz2 = _rw(dy * (tw["z2"] > 0), em)  # bf16 mode: the bf16 dz2 the dense backward reads
        grads[f"{t}_W2"], grads[f"{t}_b2"] = tw["a1"].T @ dz2, dz2.sum(0)
        dz1 = _rw((dz2 @ _rw(p[f"{t}_W2"], em).T) * (tw["z1"] > 0), em)
        grads[f"{t}_W1"], grads[f"{t}_b1"] = np.asarray(tw["X"].T @ dz1), dz1.sum(0)
    return grads


class Adam:
    """TF1.x ApplyAdam on the variables that received a gradient this step; one shared pair of
    beta powers advanced every step (AdamOptimizer._finish)."""

    def __init__(self, cfg: MvConfig, params):
        self.cfg = cfg
        self.m = {k: np.zeros_like(v, np.float32) for k, v in params.items()}
        self.v = {k: np.zeros_like(v, np.float32) for k, v in params.items()}
        self.b1p, self.b2p = np.float32(0.9), np.float32(0.999)

    def step(self, params, grads):
        f = np.float32
        lr_t = f(self.cfg.lr) * np.sqrt(f(1) - self.b2p) / (f(1) - self.b1p)
        for k, g in grads.items():
            g = g.astype(np.float32)
            m, v = self.m[k], self.v[k]
            m[...] = m + (g - m) * f(1 - 0.9)
            v[...] = v + (g * g - v) * f(1 - 0.999)
            params[k][...] = params[k] - (m * lr_t) / (np.sqrt(v) + f(1e-8))
        self.b1p, self.b2p = f(self.b1p * f(0.9)), f(self.b2p * f(0.999))
