"""Multi-view DSSM on one MI355X (BASELINE.json config 5).

The reference's archive/multi_view_dssm_v3.py:107-241: a user tower and three item-view towers
(sparse FC1 + ReLU + FC2 + ReLU each, no batch norm), the active view's item embeddings as
positives and in-batch rotations of them as the NEG negatives (Make_Negative_Item), x20 cosine,
softmax, summed loss, Adam on the user tower and the active view.

The user tower and the active item view run concurrently (the item tower on a second stream that
forks from and joins the caller's stream): each tower's launches are latency-bound, so the two
chains overlap on the CUs.  Composed from libdssm.so's functional C-ABI (include/dssm.h): dssm_spmm_csr_fwd /
dssm_spmm_csr_bwd_w (FC1), dssm_dense_fwd / dssm_dense_bwd (FC2) with the ReLUs in their epilogues
(dssm_spmm_csr_fwd_act / dssm_dense_fwd_act, dssm_dense_bwd_masked: FC1's ReLU backward on dA1),
dssm_rows_gather_sum (the rotation's gradient x BS with FC2's ReLU backward),
dssm_cosine_softmax_loss_mapped (the cosine kernel shared with the BoW path, reading the rotation's
merged rows through an index map), dssm_adam_step.  Torch tensors are device storage only.

Two modes, as the BoW model:
* "fp32" (parity mode): fp32 weights, activations and the fp32 MFMA 16x16x4 GEMMs;
* "bf16" (perf mode): FC1 gathers a bf16 shadow of W1 and stores its ReLU output bf16
  (dssm_spmm_csr_fwd_ex), FC2 runs on bf16 MFMA 16x16x32 tiles with a bf16 shadow of W2, the
  backward's dz2 / dz1 are bf16 (dssm_rows_gather_sum_ex, dssm_dense_bwd_ex) so the weight-gradient
  gathers read half the bytes; master weights, gradients, Adam state, the embeddings, cosine and
  loss stay fp32, and the optimizer rewrites the shadows as it updates (dssm_adam_step_shadow).

The reference chooses the view with a Python comparison against a placeholder at graph build, so
it always trains view 3; here the fed active view selects the tower.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr

TOWERS = ("user", "view1", "view2", "view3")


def _a64(n):
    return -(-n // 64) * 64


def _ld(n):
    return -(-n // 8) * 8


class MultiViewDSSM:
    def __init__(self, user_d: int, view_d: Sequence[int], l1: int, l2: int, bs: int, neg: int = 4,
                 lr: float = 0.05, gamma: float = 20.0, max_nnz_per_row: int = 96, device=None,
                 rotations: Optional[Sequence[int]] = None, seed: int = 0, dtype: str = "fp32",
                 fused_w1_adam: bool = True, csc_stream: bool = True):
        self.lib = _lib.load()
        if dtype not in ("fp32", "bf16"):
            raise ValueError("dtype: 'fp32' or 'bf16'")
        self.dtype = dtype
        self.bf16 = dtype == "bf16"
        self._dt = _lib.DSSM_BF16 if self.bf16 else _lib.DSSM_F32
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if len(view_d) != 3 or l1 % 4 or l2 % 4:
            raise ValueError("three item views; l1, l2 multiples of 4")
        self.dims = [int(user_d)] + [int(d) for d in view_d]
        self.l1, self.l2, self.bs, self.neg = int(l1), int(l2), int(bs), int(neg)
        self.ld1, self.ld2 = _ld(self.l1), _ld(self.l2)
        self.lr, self.gamma = float(lr), float(gamma)
        self.max_nnz = self.bs * int(max_nnz_per_row)
        dev, f32 = self.device, torch.float32
        # arena: per tower [W1; b1] ((D+1) x l1), [W2; b2] ((l1+1) x l2)
        self.layout: Dict[str, tuple] = {}
        off = 0
        for t, d in zip(TOWERS, self.dims):
            start = off
            for name, rows, cols in ((f"{t}_1", d + 1, self.l1), (f"{t}_2", self.l1 + 1, self.l2)):
                self.layout[name] = (off, rows, cols)
                off = _a64(off + rows * cols)
            self.layout[t] = (start, off)
        self.n_params = off
        self.params = torch.zeros(off, dtype=f32, device=dev)
        self.grads = torch.zeros(off, dtype=f32, device=dev)
        self.adam_m = torch.zeros(off, dtype=f32, device=dev)
        self.adam_v = torch.zeros(off, dtype=f32, device=dev)
        self.adam_state = torch.tensor([0.9, 0.999], dtype=f32, device=dev)
        BS, R = self.bs, self.bs * (2 + self.neg)
        act = torch.bfloat16 if self.bf16 else f32  # FC1's activation, dz2, dz1 (the MFMA operands)
        self.a1 = {k: torch.zeros((BS, self.ld1), dtype=act, device=dev) for k in ("u", "i")}
        self.ysrc = torch.zeros((2 * BS, self.ld2), dtype=f32, device=dev)   # [user_y; item_y]
        self.dz2src = torch.zeros((2 * BS, self.ld2), dtype=act, device=dev)  # FC2's dz, [user; item]
        self.dmerged = torch.zeros((R, self.ld2), dtype=f32, device=dev)
        # per-tower backward scratch: the two towers run concurrently (user tower on the caller's
        # stream, the item tower on self.aux)
        self.dz1 = {k: torch.zeros((BS, self.ld1), dtype=act, device=dev) for k in ("u", "i")}
        # bf16 mode: per tower the weight shadows the forward reads, [rows x ld] with zero pads
        self.shadow = {}
        if self.bf16:
            for t, d in zip(TOWERS, self.dims):
                self.shadow[f"{t}_1"] = torch.zeros((d, self.ld1), dtype=torch.bfloat16, device=dev)
                self.shadow[f"{t}_2"] = torch.zeros((self.l1, self.ld2), dtype=torch.bfloat16, device=dev)
        K = self.neg + 1
        self.cos_raw = torch.zeros(K * BS, dtype=f32, device=dev)
        self.cos_sim = torch.zeros(BS * K, dtype=f32, device=dev)
        self.prob = torch.zeros(BS * K, dtype=f32, device=dev)
        self.qnorm = torch.zeros(BS, dtype=f32, device=dev)
        self.loss_buf = torch.zeros(2, dtype=f32, device=dev)
        self.cos_ws = torch.zeros(2 * (-(-BS // 4)) + 64, dtype=f32, device=dev)
        slab = max(self.lib.dssm_dense_bwd_slab_floats(BS, self.l1, self.l2, self._dt), 1)
        self.slab = {k: torch.zeros(int(slab), dtype=f32, device=dev) for k in ("u", "i")}
        self.aux = torch.cuda.Stream(device=dev)
        # fused mode, csc_stream: the optimizer's CSC transposes on a third stream forked from the
        # caller's stream at the top of forward(), so the item tower's forward and backward on aux do
        # not queue behind them.  It must fork from the caller's (in a captured step: the capture's
        # origin) stream: a stream forked from aux, itself forked by an event wait, makes ROCm 7.0's
        # hipStreamEndCapture segfault with every stream joined (profiles/r05_mv_capture_probe.txt).
        # Measured at C5 bf16: 0.2400 against 0.2467 ms/step on two streams (profiles/r05_mv_streams.txt)
        self.csc_stream = bool(csc_stream)
        self.aux2 = torch.cuda.Stream(device=dev) if self.csc_stream else None
        self._csc_ev_i = None
        # one CSC-transpose workspace per tower (zero on first use, kept zero by the calls)
        self.spmm_ws = {t: torch.zeros(int(self.lib.dssm_spmm_bwd_ws_bytes(BS, d, self.max_nnz)),
                                       dtype=torch.uint8, device=dev) for t, d in zip(TOWERS, self.dims)}
        self.batch = {}
        self.view = 3
        # FC2's split-K weight-gradient partials left for the fused optimizer (per tower key)
        self._splits = {"u": C.c_int(0), "i": C.c_int(0)}
        self._fused = False
        self._adam_pending = False  # fused: backward left the towers' streams forked for apply_adam
        # the two tower launches of a fused optimizer step share these tickets: the later one to
        # finish advances the beta powers (no advance launch, no join in front of it)
        self.adam_tickets = torch.zeros(int(self.lib.dssm_adam_tickets_bytes(2)), dtype=torch.uint8, device=dev)
        self.fused_w1_adam = fused_w1_adam
        self.set_rotations(rotations if rotations is not None else self.default_rotations(seed))
        self.global_step = 0

    @property
    def fused_w1_adam(self) -> bool:
        """One GPU: each trained tower's FC1 weight gradient is never stored -- apply_adam's
        dssm_spmm_bwd_w_adam gathers it inside the optimizer launch from the batch's CSC transpose
        and dz1 (the BoW plan's fused W1 Adam), and FC2's split-K partials are summed there too.
        backward() then leaves the towers' gradients unmaterialised (W1 rows zero).  Off: backward()
        writes the whole gradient arena (data parallel: the all-reduce needs it)."""
        return self._fused

    @fused_w1_adam.setter
    def fused_w1_adam(self, on: bool):
        on = bool(on)
        if on and not self._fused:
            self.grads.zero_()  # the fused launch's heavy W1 rows accumulate into zeroed rows
        self._fused = on

    # ---- parameters ---------------------------------------------------------------------------
    def _block(self, arena, name):
        off, rows, cols = self.layout[name]
        return arena[off:off + rows * cols].view(rows, cols)

    def load_params(self, p: Dict[str, np.ndarray]):
        for t in TOWERS:
            for l in (1, 2):
                blk = np.concatenate([p[f"{t}_W{l}"], p[f"{t}_b{l}"][None, :]], 0).astype(np.float32)
                self._block(self.params, f"{t}_{l}").copy_(torch.from_numpy(blk))
        self.sync_shadows()

    def sync_shadows(self):
        """bf16 mode: the weight shadows from the fp32 parameters (RNE, as the optimizer writes
        them), after loading parameters; a setup step, not the training step."""
        for name, sh in self.shadow.items():
            w = self._block(self.params, name)[:-1]
            sh[:, :w.shape[1]].copy_(w.to(torch.bfloat16))

    def named(self, arena: Optional[torch.Tensor] = None) -> Dict[str, np.ndarray]:
        a = self.params if arena is None else arena
        out = {}
        for t in TOWERS:
            for l in (1, 2):
                blk = self._block(a, f"{t}_{l}").cpu().numpy()
                out[f"{t}_W{l}"], out[f"{t}_b{l}"] = blk[:-1], blk[-1]
        return out

    def init_params(self, seed: int = 0):
        """W, b ~ U(-r, r), r = sqrt(6 / (fan_in + fan_out)) (multi_view_dssm_v3.py:115-185)."""
        rng = np.random.Generator(np.random.PCG64(seed))
        p = {}
        for t, d in zip(TOWERS, self.dims):
            for l, (a, b) in enumerate(((d, self.l1), (self.l1, self.l2)), 1):
                r = np.sqrt(6.0 / (a + b))
                p[f"{t}_W{l}"] = rng.uniform(-r, r, size=(a, b)).astype(np.float32)
                p[f"{t}_b{l}"] = rng.uniform(-r, r, size=b).astype(np.float32)
        self.load_params(p)
        return p

    def default_rotations(self, seed: int):
        u = np.random.Generator(np.random.PCG64(seed)).random(self.neg)
        return [int((u[i] + i) * self.bs / self.neg) for i in range(self.neg)]

    def set_rotations(self, rot: Sequence[int]):
        """Make_Negative_Item's offsets (fixed at graph build in the reference): negative i of user j
        is item row (j + rot[i]) mod BS.  Sets the gather map of the merged [user; pos; neg] rows."""
        BS = self.bs
        rot = [int(r) % BS for r in rot]
        if len(rot) != self.neg:
            raise ValueError("one rotation per negative")
        m = [np.arange(BS), BS + np.arange(BS)]
        # merged neg row 2BS + j*NEG + i (the cosine kernel's layout) = item row (j + rot_i) % BS
        j = np.repeat(np.arange(BS), self.neg)
        i = np.tile(np.arange(self.neg), BS)
        m.append(BS + (j + np.array(rot)[i]) % BS)
        self.rot = rot
        mp = np.concatenate(m).astype(np.int32)
        self.map = torch.from_numpy(mp).to(self.device)
        # its inverse (each of the 2BS source rows: the merged rows it feeds, ascending) for the
        # backward's fixed-order gather-sum
        order = np.argsort(mp, kind="stable").astype(np.int32)
        offs = np.zeros(2 * BS + 1, np.int32)
        np.cumsum(np.bincount(mp, minlength=2 * BS), out=offs[1:])
        self.inv_idx = torch.from_numpy(order).to(self.device)
        self.inv_offs = torch.from_numpy(offs).to(self.device)

    # ---- feed ---------------------------------------------------------------------------------
    def set_batch(self, user_csr, item_csr, view: int):
        """user_csr, item_csr: (indptr, indices, values) host arrays of BS rows each; view in 1..3."""
        if view not in (1, 2, 3):
            raise ValueError("active view is 1, 2 or 3")
        for name, csr, d in (("u", user_csr, self.dims[0]), ("i", item_csr, self.dims[view])):
            ip, ix, vv = (np.asarray(x) for x in csr)
            if ip.size != self.bs + 1 or int(ip[-1]) > self.max_nnz:
                raise ValueError(f"{name}: {self.bs} rows, at most {self.max_nnz} non-zeros")
            if ix.size and (ix.min() < 0 or ix.max() >= d):
                raise ValueError(f"{name}: column index out of range")
            self.batch[name] = tuple(torch.from_numpy(np.ascontiguousarray(x, dt)).to(self.device)
                                     for x, dt in ((ip, np.int32), (ix, np.int32), (vv, np.float32)))
        self.view = view

    # ---- step ---------------------------------------------------------------------------------
    def _tower_fwd(self, key, tower, y_rows, s):
        ip, ix, vv = self.batch[key]
        d = self.dims[TOWERS.index(tower)]
        w1, w2 = self._block(self.params, f"{tower}_1"), self._block(self.params, f"{tower}_2")
        # FC + ReLU in one launch each (the ReLU in the producers' epilogues); bf16 mode: the weight
        # shadows, FC1's activation stored bf16 for FC2's bf16 MFMA tiles
        if self.bf16:
            ws1, ws2, ld_w1, ld_w2 = self.shadow[f"{tower}_1"], self.shadow[f"{tower}_2"], self.ld1, self.ld2
        else:
            ws1, ws2, ld_w1, ld_w2 = w1, w2, self.l1, self.l2
        check(self.lib.dssm_spmm_csr_fwd_ex(ptr(ip), ptr(ix), ptr(vv), self.bs, ptr(ws1), self._dt, ld_w1,
                                            self.l1, ptr(w1[d]), ptr(self.a1[key]), self._dt, self.ld1,
                                            _lib.DSSM_ACT_RELU, s), "spmm_fwd")
        check(self.lib.dssm_dense_fwd_act(ptr(self.a1[key]), self.ld1, ptr(ws2), ld_w2, self._dt, self.bs,
                                          self.l1, self.l2, ptr(w2[self.l1]), ptr(y_rows), self.ld2,
                                          _lib.DSSM_ACT_RELU, s), "dense_fwd")

    def _fork(self, stream):
        """The item tower's stream joins the caller's stream here."""
        main = stream if stream is not None else torch.cuda.current_stream(self.device)
        self.aux.wait_stream(main)
        return main

    def forward(self, stream=None):
        main = self._fork(stream)
        s, sa = stream_ptr(main), stream_ptr(self.aux)
        BS = self.bs
        self._csc_ev = self._csc_ev_i = None
        if self._fused and self.csc_stream:
            self.aux2.wait_stream(main)  # forked from the caller's stream, never from aux
            for key in ("u", "i"):
                for t in self.batch[key]:
                    t.record_stream(self.aux2)
            s2 = stream_ptr(self.aux2)
            self._csc("u", "user", s2)
            self._csc_ev = self.aux2.record_event()
            self._csc("i", f"view{self.view}", s2)
            self._csc_ev_i = self.aux2.record_event()
        # the towers are independent until the cosine: the item tower runs beside the user tower
        self._tower_fwd("u", "user", self.ysrc[:BS], s)
        self._tower_fwd("i", f"view{self.view}", self.ysrc[BS:], sa)
        main.wait_event(self.aux.record_event())
        if self._fused and not self.csc_stream:
            # the optimizer's CSC transposes (they depend on the batch only) on the item tower's
            # stream while the caller's stream runs the loss: off the step's critical path.  They
            # read the batch after the join above, so the batch tensors are marked in use on aux:
            # a set_batch before apply_adam (eval loops) frees them, and the caching allocator
            # must not hand their memory out again until aux's transposes have read it
            for key in ("u", "i"):
                for t in self.batch[key]:
                    t.record_stream(self.aux)
            self._csc("u", "user", sa)
            self._csc_ev = self.aux.record_event()
            self._csc("i", f"view{self.view}", sa)
        # Make_Negative_Item's merged rows read through the index map by the cosine kernel itself
        check(self.lib.dssm_cosine_softmax_loss_mapped(ptr(self.ysrc), self.ld2, ptr(self.map), self.l2, BS,
                                                       self.neg, self.gamma, ptr(self.cos_raw), ptr(self.cos_sim),
                                                       ptr(self.prob), ptr(self.qnorm), ptr(self.loss_buf),
                                                       ptr(self.dmerged), ptr(self.cos_ws), s), "cosine")

    def _tower_bwd(self, key, tower, dz2, s):
        ip, ix, vv = self.batch[key]
        d = self.dims[TOWERS.index(tower)]
        w2 = self._block(self.params, f"{tower}_2")
        ws2, ld_w2 = (self.shadow[f"{tower}_2"], self.ld2) if self.bf16 else (w2, self.l2)
        dz1 = self.dz1[key]
        # dA1 with FC1's ReLU backward fused (masked by a1 = relu(z1) > 0): dz1 directly (bf16 mode:
        # stored bf16, the operand of the weight gradient's gathers)
        check(self.lib.dssm_dense_bwd_ex(ptr(self.a1[key]), self.ld1, ptr(ws2), ld_w2, self._dt,
                                         self.bs, self.l1, self.l2, ptr(dz2), self.ld2, ptr(dz1), self._dt, self.ld1,
                                         ptr(self.a1[key]), self._dt, self.ld1,
                                         ptr(self._block(self.grads, f"{tower}_2")), ptr(self.slab[key]),
                                         C.byref(self._splits[key]) if self._fused else None, s),
              "dense_bwd")
        if self._fused:
            return  # FC1's weight gradient: inside the optimizer launch (apply_adam)
        check(self.lib.dssm_spmm_csr_bwd_w(ptr(ip), ptr(ix), ptr(vv), self.bs, d, self.max_nnz, ptr(dz1),
                                           self._dt, self.ld1, self.l1,
                                           ptr(self._block(self.grads, f"{tower}_1")), ptr(self.spmm_ws[tower]),
                                           s), "spmm_bwd")

    def backward(self, stream=None, join: bool = True):
        """join=False (fused optimizer, apply_adam next on the same streams): the item tower's stream
        is left forked so each tower's optimizer launch follows its own backward without a join and
        re-fork in between (apply_adam joins)."""
        main = stream if stream is not None else torch.cuda.current_stream(self.device)
        s = stream_ptr(main)
        BS, R = self.bs, self.bs * (2 + self.neg)
        # the cosine kernel's d(mean loss)/dy x BS = d(summed loss)/dy (multi_view_dssm_v3.py:234)
        # Merge_Negative_Doc's gradient, the x BS and FC2's ReLU backward in one launch: dz2 of both
        # towers = BS * (sum of the merged rows each source row feeds) where y > 0
        check(self.lib.dssm_rows_gather_sum_ex(ptr(self.dmerged), self.ld2, ptr(self.inv_offs), ptr(self.inv_idx),
                                               2 * BS, self.l2, float(BS), ptr(self.ysrc), self.ld2, ptr(self.dz2src),
                                               self._dt, self.ld2, s), "gather_sum")
        self._fork(main)
        self._tower_bwd("u", "user", self.dz2src[:BS], s)
        self._tower_bwd("i", f"view{self.view}", self.dz2src[BS:], stream_ptr(self.aux))
        if self._fused and not join:
            self._adam_pending = True  # each tower's optimizer launch follows on its own stream
        else:
            main.wait_stream(self.aux)

    def trained_ranges(self):
        """Arena ranges the step updates: the user tower and the active view."""
        return [self.layout[t] for t in ("user", f"view{self.view}")]

    def _csc(self, key, tower, s):
        ip, ix, vv = self.batch[key]
        check(self.lib.dssm_spmm_bwd_csc(ptr(ip), ptr(ix), ptr(vv), self.bs, self.dims[TOWERS.index(tower)],
                                         self.max_nnz, ptr(self.spmm_ws[tower]), s), "spmm_bwd_csc")

    def _tower_adam(self, key, tower, s, grad_scale, member, build_csc):
        """Fused mode: one tower's CSC transpose + ONE optimizer launch over its [W1; b1] rows (the
        gradient gathered inline) and its [W2; b2] block (FC2's split-K partials summed inline)."""
        ip, ix, vv = self.batch[key]
        d = self.dims[TOWERS.index(tower)]
        b, e = self.layout[tower]
        off2 = self.layout[f"{tower}_2"][0] - b
        segs, nseg, w1s, ld1 = None, 0, None, 0
        if self.bf16:
            sh2 = self.shadow[f"{tower}_2"]
            segs = (_lib.dssm_shadow_seg * 1)(_lib.dssm_shadow_seg(off2, self.l1, self.l2, sh2.shape[1],
                                                                  sh2.data_ptr()))
            nseg, w1s, ld1 = 1, ptr(self.shadow[f"{tower}_1"]), self.ld1
        splits = self._splits[key].value
        check(self.lib.dssm_spmm_bwd_w_adam(ptr(ip), ptr(ix), ptr(vv), self.bs, d, self.max_nnz, ptr(self.dz1[key]),
                                            self._dt, self.ld1, self.l1, ptr(self.params[b:]), ptr(self.grads[b:]),
                                            ptr(self.adam_m[b:]), ptr(self.adam_v[b:]), off2, e - b,
                                            ptr(self.slab[key]) if splits else None, (self.l1 + 1) * self.l2, splits,
                                            w1s, ld1, segs, nseg, self.lr, 0.9, 0.999, 1e-8, ptr(self.adam_state),
                                            grad_scale, 2, member, ptr(self.adam_tickets), int(build_csc),
                                            ptr(self.spmm_ws[tower]), s), "spmm_bwd_w_adam")

    def apply_adam(self, stream=None, grad_scale: float = 1.0):
        s = stream_ptr(stream)
        towers = ("user", f"view{self.view}")
        if self._fused:
            # each tower's launch on its backward's stream (the item tower's on self.aux), running
            # concurrently; the later one to finish advances the beta powers
            main = stream if stream is not None else torch.cuda.current_stream(self.device)
            if not self._adam_pending:
                self._fork(main)
            self._adam_pending = False
            # (both on one stream, each tower's transpose + launch in turn: 0.292 against 0.257 ms/step;
            # both towers in ONE launch after a join, commit history: 0.251-0.254 against 0.240-0.242)
            built = getattr(self, "_csc_ev", None) is not None  # transposed by forward() on self.aux
            if built:
                main.wait_event(self._csc_ev)
            if self._csc_ev_i is not None:  # csc_stream: the item transpose on aux2
                self.aux.wait_event(self._csc_ev_i)
            self._tower_adam("u", towers[0], stream_ptr(main), grad_scale, 0, not built)
            self._tower_adam("i", towers[1], stream_ptr(self.aux), grad_scale, 1, not built)
            main.wait_stream(self.aux)
            self._csc_ev = self._csc_ev_i = None
        elif self.bf16:
            # both trained towers in one launch, the updated weights' bf16 shadows written by the same pass
            rng = (C.c_int64 * 4)(*[x for t in towers for x in self.layout[t]])
            segs = (_lib.dssm_shadow_seg * 4)()
            for i, (t, l) in enumerate((t, l) for t in towers for l in (1, 2)):
                off, rows, cols = self.layout[f"{t}_{l}"]
                sh = self.shadow[f"{t}_{l}"]
                segs[i] = _lib.dssm_shadow_seg(off, rows - 1, cols, sh.shape[1], sh.data_ptr())
            check(self.lib.dssm_adam_step_shadow(ptr(self.params), ptr(self.grads), ptr(self.adam_m), ptr(self.adam_v),
                                                 rng, 2, self.lr, 0.9, 0.999, 1e-8, ptr(self.adam_state), grad_scale,
                                                 1, segs, 4, s), "adam")
        else:
            for k, t in enumerate(towers):
                b, e = self.layout[t]
                check(self.lib.dssm_adam_step(ptr(self.params[b:e]), ptr(self.grads[b:e]), ptr(self.adam_m[b:e]),
                                              ptr(self.adam_v[b:e]), e - b, self.lr, 0.9, 0.999, 1e-8,
                                              ptr(self.adam_state), grad_scale, k == 1, s), "adam")
        self.global_step += 1

    def train_step(self, stream=None):
        self.forward(stream)
        self.backward(stream, join=False)
        self.apply_adam(stream)

    def loss(self) -> float:
        return float(self.loss_buf[0].item()) * self.bs


class MultiViewDataParallel:
    """BASELINE config 5 across GPUs: one process per GPU, each rank trains on its own batch of BS
    users (weak scaling) with the same active view; after the backward the gradients of the user
    tower and the active view are summed over the ranks (fp32 all-reduce on libdssm.so's RCCL
    communicator, or torch.distributed: dssm_amd.dist transports, self-tested at start-up) and every
    rank applies the same Adam step with grad_scale = 1/world, the mean of the per-rank gradients,
    so the ranks stay bit-identical.  (The reference's loss is a sum over its BS users; averaging
    over ranks keeps the per-step update of the single-GPU step.)"""

    def __init__(self, model: MultiViewDSSM, comm: str = "auto"):
        import torch.distributed as dist
        from .dist import SCHEDULE_OPS, select_transport
        self.model = model
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        if self.world > 1:
            model.fused_w1_adam = False  # the all-reduce sums the materialised gradients
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.tx = None
        self.fallbacks = []
        if self.world == 1:
            return
        self.tx, self.fallbacks = select_transport(self.rank, self.world, model.device, comm,
                                                   SCHEDULE_OPS[("allreduce", "fp32")])
        if self.tx is None:
            raise RuntimeError("no working all-reduce transport: " + "; ".join(self.fallbacks))
        for note in self.fallbacks:
            import warnings
            warnings.warn(f"MultiViewDataParallel: {note}", RuntimeWarning, stacklevel=2)

    @property
    def comm(self) -> str:
        return self.tx.name if self.tx is not None else "none"

    def exchange(self):
        if self.world > 1:
            for b, e in self.model.trained_ranges():
                self.tx.all_reduce(self.model.grads[b:e])

    def train_step(self):
        self.model.forward()
        self.model.backward()
        self.exchange()
        self.model.apply_adam(grad_scale=1.0 / self.world)

    def close(self):
        if self.tx is not None:
            self.tx.destroy()
            self.tx = None
