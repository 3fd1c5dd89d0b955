"""RNN-tower DSSM on one MI355X (BASELINE.json config 4).

The reference's semantic_matching/dssm_rnn/dssm_rnn.py:100-217: word embeddings -> one
bidirectional GRU (GRUCell(hidden), shared by query / positive / negative inputs, dynamic lengths)
-> dropout(keep) on concat(final fw state, final bw state) -> Merge_Negative_Doc -> x20 cosine ->
softmax -> loss = -sum_j log p[j, 0] (summed over queries, :214) -> AdamOptimizer(lr) (:218).

Everything runs through libdssm.so (csrc/rnn.hip for the tower and its Adam, csrc/cosine.hip's
loss kernel shared with the BoW path); torch tensors are device storage only.  dtype "fp32" (the
parity mode: fp32 FMA recurrences) or "bf16" (the perf mode, csrc/rnn_mfma.hip: the recurrences on
bf16 MFMA with register-resident weights, fp32 states / master weights / gradients / Adam).

Parameters live in one flat fp32 arena: the embedding table [nwords x E] first (its Adam update
uses TF1's IndexedSlices form), then per direction the GRU blocks [Wg; bg] ((E+H+1) x 2H) and
[Wc; bc] ((E+H+1) x H), each 64-float aligned.  Rows of a step are [q(BS); pos(BS); neg(BS*NEG)],
ids [R x T] int32 with per-row lengths.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr


def _align(n: int, a: int = 64) -> int:
    return -(-n // a) * a


class RnnDSSM:
    def __init__(self, nwords: int, emb: int, hidden: int, query_bs: int, neg: int = 4,
                 seq_len: int = 10, lr: float = 1e-5, keep_prob: float = 0.5, gamma: float = 20.0,
                 beta1: float = 0.9, beta2: float = 0.999, adam_eps: float = 1e-8, device=None,
                 seed: int = 0, dtype: str = "fp32"):
        self.lib = _lib.load()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.V, self.E, self.H = int(nwords), int(emb), int(hidden)
        self.BS, self.NEG, self.T = int(query_bs), int(neg), int(seq_len)
        self.R = self.BS * (2 + self.NEG)
        self.K = self.E + self.H
        self.lr, self.beta1, self.beta2, self.eps = lr, beta1, beta2, adam_eps
        self.keep, self.gamma, self.seed = float(keep_prob), float(gamma), int(seed)
        K, H = self.K, self.H
        self.layout = {}
        off = 0
        for name, rows, cols in (("emb", self.V, self.E), ("fw_g", K + 1, 2 * H), ("fw_c", K + 1, H),
                                 ("bw_g", K + 1, 2 * H), ("bw_c", K + 1, H)):
            self.layout[name] = (off, rows, cols)
            off = _align(off + rows * cols)
        self.n_params = off
        dev, f32 = self.device, torch.float32
        self.params = torch.zeros(off, dtype=f32, device=dev)
        self.grads = torch.zeros(off, dtype=f32, device=dev)
        self.adam_m = torch.zeros(off, dtype=f32, device=dev)
        self.adam_v = torch.zeros(off, dtype=f32, device=dev)
        self.adam_state = torch.tensor([beta1, beta2] + [0.0] * 62, dtype=f32, device=dev)
        if dtype not in ("fp32", "bf16"):
            raise ValueError("dtype is 'fp32' or 'bf16'")
        self.dtype = dtype
        if dtype == "bf16":
            if not self.lib.dssm_rnn_bf16_supported(self.E, self.H):
                raise ValueError("bf16 RNN: (E, H) in {(128, 128), (64, 128), (32, 32)}")
            ws = self.lib.dssm_rnn_bf16_ws_bytes(self.R, self.T, self.E, self.H, self.V)
            if ws == 0 or self.V > 32768:
                raise ValueError(f"bf16 RNN: vocabulary of {self.V} words exceeds the embedding-gradient "
                                 "token scan's 32768-word limit (use dtype='fp32')")
            self.ws = torch.zeros(int(ws), dtype=torch.uint8, device=dev)
        else:
            ws = self.lib.dssm_rnn_ws_floats(self.R, self.T, self.E, self.H)
            if ws == 0:
                raise ValueError("unsupported RNN shape (E, H multiples of 4; E+H <= 512; H <= 256)")
            self.ws = torch.zeros(int(ws), dtype=f32, device=dev)
        R2 = (self.R, 2 * H)
        self.y0 = torch.zeros(R2, dtype=f32, device=dev)
        self.y = torch.zeros(R2, dtype=f32, device=dev)
        self.dy = torch.zeros(R2, dtype=f32, device=dev)
        K1 = self.NEG + 1
        self.cos_raw = torch.zeros(K1 * self.BS, dtype=f32, device=dev)
        self.cos_sim = torch.zeros(self.BS * K1, dtype=f32, device=dev)
        self.prob = torch.zeros(self.BS * K1, dtype=f32, device=dev)
        self.qnorm = torch.zeros(self.BS, dtype=f32, device=dev)
        self.loss_buf = torch.zeros(2, dtype=f32, device=dev)
        self.cos_ws = torch.zeros(2 * (-(-self.BS // 4)) + 64, dtype=f32, device=dev)
        self.ids = torch.zeros((self.R, self.T), dtype=torch.int32, device=dev)
        self.lens = torch.full((self.R,), self.T, dtype=torch.int32, device=dev)
        self.global_step = 0
        self._drop_step = 0
        self._train = False
        # bf16 mode: the workspace's bf16 copy of the embedding table is bf16(emb) (written by the last
        # optimizer step), so the forward skips its conversion pass; reset when parameters are loaded
        self._emb16_ok = False

    # ---- parameters (oracle / reference names) ------------------------------------------------
    def _block(self, arena: torch.Tensor, name: str) -> torch.Tensor:
        off, rows, cols = self.layout[name]
        return arena[off:off + rows * cols].view(rows, cols)

    def mark_params_changed(self):
        """Call after writing self.params directly (arena copy, external restore, broadcast): the
        workspace's bf16 embedding copy is stale, so the next bf16 forward re-converts it."""
        self._emb16_ok = False

    def load_params(self, p: Dict[str, np.ndarray]):
        self.mark_params_changed()
        self._block(self.params, "emb").copy_(torch.from_numpy(np.asarray(p["emb"], np.float32)))
        for d in ("fw", "bw"):
            g = np.concatenate([p[f"{d}_Wg"], p[f"{d}_bg"][None, :]], 0).astype(np.float32)
            c = np.concatenate([p[f"{d}_Wc"], p[f"{d}_bc"][None, :]], 0).astype(np.float32)
            self._block(self.params, f"{d}_g").copy_(torch.from_numpy(g))
            self._block(self.params, f"{d}_c").copy_(torch.from_numpy(c))

    def named(self, arena: Optional[torch.Tensor] = None) -> Dict[str, np.ndarray]:
        a = self.params if arena is None else arena
        out = {"emb": self._block(a, "emb").cpu().numpy()}
        K = self.K
        for d in ("fw", "bw"):
            g, c = self._block(a, f"{d}_g").cpu().numpy(), self._block(a, f"{d}_c").cpu().numpy()
            out[f"{d}_Wg"], out[f"{d}_bg"] = g[:K], g[K]
            out[f"{d}_Wc"], out[f"{d}_bc"] = c[:K], c[K]
        return out

    def init_params(self, seed: int = 0):
        """tf.get_variable defaults (glorot-uniform kernels and embedding table), GRUCell's gate
        bias 1.0 and candidate bias 0 (numpy PCG64 seed)."""
        rng = np.random.Generator(np.random.PCG64(seed))

        def glorot(shape):
            r = np.sqrt(6.0 / (shape[0] + shape[1]))
            return rng.uniform(-r, r, size=shape).astype(np.float32)
        K, H = self.K, self.H
        p = {"emb": glorot((self.V, self.E))}
        for d in ("fw", "bw"):
            p[f"{d}_Wg"], p[f"{d}_bg"] = glorot((K, 2 * H)), np.ones(2 * H, np.float32)
            p[f"{d}_Wc"], p[f"{d}_bc"] = glorot((K, H)), np.zeros(H, np.float32)
        self.load_params(p)
        return p

    # ---- feed ---------------------------------------------------------------------------------
    def set_batch(self, ids, lens=None):
        """ids [R x T] (rows [q; pos; neg]); lens [R] (default: T, as dssm_rnn.py:287-289 feeds)."""
        ids = np.asarray(ids, np.int32)
        if ids.shape != (self.R, self.T):
            raise ValueError(f"ids must be [{self.R} x {self.T}]")
        if ids.min() < 0 or ids.max() >= self.V:
            raise ValueError("token id out of [0, nwords)")
        self.ids.copy_(torch.from_numpy(ids))
        if lens is None:
            self.lens.fill_(self.T)
        else:
            lens = np.asarray(lens, np.int32)
            if lens.shape != (self.R,) or lens.min() < 1 or lens.max() > self.T:
                raise ValueError("lens must be [R] in [1, T]")
            self.lens.copy_(torch.from_numpy(lens))

    # ---- step ---------------------------------------------------------------------------------
    def _w(self, arena):
        return (C.c_void_p * 4)(*[ptr(self._block(arena, n)) for n in ("fw_g", "fw_c", "bw_g", "bw_c")])

    def forward(self, train: bool = True, keep: Optional[float] = None, stream=None):
        s = stream_ptr(stream)
        keep = (self.keep if keep is None else float(keep)) if train else 1.0
        if self.dtype == "bf16":
            check(self.lib.dssm_rnn_bf16_forward_ex(ptr(self.ids), ptr(self.lens), self.R, self.T,
                                                     ptr(self._block(self.params, "emb")), self.V, self.E, self.H,
                                                     self._w(self.params), ptr(self.ws), ptr(self.y0), 2 * self.H,
                                                     int(self._emb16_ok), s), "rnn_bf16_forward")
        else:
            check(self.lib.dssm_rnn_forward(ptr(self.ids), ptr(self.lens), self.R, self.T,
                                             ptr(self._block(self.params, "emb")), self.E, self.H,
                                             self._w(self.params), ptr(self.ws), ptr(self.y0), 2 * self.H, s),
                  "rnn_forward")
        if train:
            self._drop_step += 1
        self._keep_used = keep
        # dropout(keep) on the final states fused into the cosine launch: y = y0 * m / keep, and dy
        # leaves it as d(summed loss)/dy0 (the cosine's d(mean loss)/dy x BS through the same mask)
        check(self.lib.dssm_cosine_softmax_loss_dropout(ptr(self.y0), 2 * self.H, 2 * self.H, self.BS, self.NEG,
                                                        self.gamma, keep, self.seed, self._drop_step,
                                                        float(self.BS), ptr(self.y), ptr(self.cos_raw),
                                                        ptr(self.cos_sim), ptr(self.prob), ptr(self.qnorm),
                                                        ptr(self.loss_buf), ptr(self.dy), ptr(self.cos_ws), s),
              "cosine_dropout")
        self._train = train

    def backward(self, stream=None):
        if not self._train:
            raise RuntimeError("backward needs a train-mode forward")
        s = stream_ptr(stream)
        # dy = d(sum loss)/dy0 already (the forward's fused dropout)
        gw = (C.c_void_p * 4)(*[ptr(self._block(self.grads, n)) for n in ("fw_g", "fw_c", "bw_g", "bw_c")])
        if self.dtype == "bf16":
            check(self.lib.dssm_rnn_bf16_backward(ptr(self.ids), ptr(self.lens), self.R, self.T, self.V, self.E,
                                                   self.H, self._w(self.params), ptr(self.dy), 2 * self.H,
                                                   ptr(self.ws), ptr(self._block(self.grads, "emb")), gw, s),
                  "rnn_bf16_backward")
        else:
            check(self.lib.dssm_rnn_backward(ptr(self.ids), ptr(self.lens), self.R, self.T, self.E, self.H,
                                              self._w(self.params), ptr(self.dy), 2 * self.H, ptr(self.ws),
                                              ptr(self._block(self.grads, "emb")), self.V * self.E, gw, s),
                  "rnn_backward")

    def apply_adam(self, stream=None):
        shadow = None
        if self.dtype == "bf16":  # the optimizer rewrites the recurrences' bf16 embedding copy
            shadow = ptr(self.ws) + int(self.lib.dssm_rnn_bf16_emb16_offset(self.R, self.T, self.E, self.H, self.V))
        check(self.lib.dssm_rnn_adam_ex(ptr(self.params), ptr(self.grads), ptr(self.adam_m), ptr(self.adam_v),
                                        self.V * self.E, self.n_params, ptr(self.adam_state), self.lr,
                                        self.beta1, self.beta2, self.eps, shadow, stream_ptr(stream)), "rnn_adam")
        self._emb16_ok = self.dtype == "bf16"
        self.global_step += 1

    def train_step(self, stream=None):
        self.forward(True, stream=stream)
        self.backward(stream)
        self.apply_adam(stream)

    # ---- fetches ------------------------------------------------------------------------------
    def loss(self) -> float:
        """Summed softmax loss of the last forward (dssm_rnn.py:214)."""
        return float(self.loss_buf[0].item()) * self.BS

    def dropout_mask_step(self) -> int:
        return self._drop_step

    def embeddings(self) -> np.ndarray:
        return self.y.cpu().numpy()
