"""Data parallelism: one process per GPU, batch sharded by query.

Two exchange schedules over the flat fp32 arenas (RCCL over xGMI):
* "zero" (default for world sizes 2, 4, 8): reduce-scatter of the gradient arena, Adam on the
  rank's shard only (p, m, v of the shard; grad_scale = 1/world), all-gather of the updated
  parameters, then the bf16 weight shadows refreshed from them.  Same bytes on the links as one
  all-reduce, but the optimizer pass (the largest kernel, HBM-bound) shrinks by the world size.
  m / v live sharded: gather_state() collects them for a checkpoint.
* "allreduce": one all-reduce of the gradient arena and replicated Adam.

The zero schedule's wire ("wire" argument; "bf16" by default for a bf16-mode model):
* "fp32": the whole padded fp32 arena is reduce-scattered and all-gathered (36.5 MB each way at
  C2), the shadows refreshed from the gathered fp32 parameters;
* "bf16": only W1's rows ([0, model.wire_extent()), 99% of the parameters) are sharded, and they
  cross the links as bf16: the backward packs bf16(dW1) into a gradient wire that is reduce-
  scattered, Adam updates the rank's fp32 W1 shard from it and writes bf16(W1) into a parameter
  wire that is all-gathered, and W1's bf16 shadow (all the bf16 forward reads of W1) is rebuilt
  from it.  The small tail ([extent, n_params): b1, W2.., BN) is all-reduced in fp32 and updated
  replicated, so every rank's biases / BN parameters stay bit-identical fp32.  Half the link
  bytes of the fp32 wire; W1's fp32 master rows outside a rank's shard are stale between
  gather_state() calls (the forward never reads them in bf16 mode).

BN statistics stay per replica (unsynced), which is the reference's BN semantics applied to a
replica's shard; EMA shadows stay rank-local and rank 0's are the ones checkpointed.

Two transports for the same collective:
* ``torch.distributed.all_reduce`` on the "nccl" backend (= RCCL on ROCm) — default;
* ``RcclComm``: libdssm.so's own RCCL communicator (dssm_comm_* in include/dssm.h), with the
  128-byte unique id shared through torch.distributed's store.
Either way the data path is one ncclAllReduce(sum) over the arena.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.distributed as dist

from . import _lib
from ._lib import check, ptr, stream_ptr


class RcclComm:
    def __init__(self, rank: int, world: int):
        lib = _lib.load()
        self.lib = lib
        buf = (C.c_char * 128)()
        if rank == 0:
            check(lib.dssm_comm_unique_id(buf), "comm_unique_id")
        obj = [bytes(buf)]
        dist.broadcast_object_list(obj, src=0)
        buf = (C.c_char * 128).from_buffer_copy(obj[0])
        check(lib.dssm_comm_init(rank, world, buf), "comm_init")

    def allreduce_(self, t: torch.Tensor, stream=None):
        assert t.dtype == torch.float32 and t.is_contiguous()
        check(self.lib.dssm_allreduce_sum_f32(ptr(t), t.numel(), stream_ptr(stream)), "allreduce")

    def destroy(self):
        self.lib.dssm_comm_destroy()


def shard_bounds(n_pad: int, n: int, rank: int, world: int):
    """Rank's optimizer shard of an arena of n elements padded to n_pad (equal shards)."""
    s = n_pad // world
    return rank * s, min((rank + 1) * s, n), s


class DataParallel:
    """Wraps a DSSM model: step = forward + backward + gradient exchange + Adam (see module doc)."""

    def __init__(self, model, comm: str = "torch", mode: str = "auto", wire: str = "auto"):
        self.model = model
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.comm = RcclComm(self.rank, self.world) if (comm == "rccl" and self.world > 1) else None
        npad = model.params.numel()
        if mode == "auto":
            mode = "zero" if (self.world > 1 and self.comm is None and npad % (64 * self.world) == 0) else "allreduce"
        if mode == "zero" and (self.comm is not None or npad % (64 * self.world)):
            raise ValueError("the zero schedule needs torch.distributed and 64-float aligned equal shards")
        self.mode = mode if self.world > 1 else "allreduce"
        self._nccl = dist.is_initialized() and dist.get_backend() == "nccl"
        if self.world > 1:
            model.set_fused_w1_adam(False)  # the exchange needs the materialized dW1
        if wire == "auto":
            wire = "bf16" if getattr(model, "dtype", "fp32") == "bf16" else "fp32"
        if wire not in ("bf16", "fp32"):
            raise ValueError("wire: 'bf16' or 'fp32'")
        if self.mode == "zero" and self._nccl and not (
                self._inplace_ok(torch.float32) and (wire == "fp32" or self._inplace_ok(torch.bfloat16))):
            self.mode = "allreduce"  # the in-place collectives misbehaved: exchange by all-reduce
        self.wire = wire if self.mode == "zero" else "fp32"
        self.grad_wire = self.param_wire = None
        if self.mode == "zero" and self.wire == "bf16":
            ext = model.wire_extent()
            self.extent = ext
            self.shard = -(-ext // (64 * self.world)) * 64
            self.begin, self.end = self.rank * self.shard, min((self.rank + 1) * self.shard, ext)
            n = self.shard * self.world
            dev = model.params.device
            self.grad_wire = torch.zeros(n, dtype=torch.bfloat16, device=dev)
            self.param_wire = torch.zeros(n, dtype=torch.bfloat16, device=dev)
            self.param_wire[:ext].copy_(model.params[:ext])
            model.set_wire(self.grad_wire, self.param_wire)
            model.set_adam_range(self.begin, max(self.begin, self.end))
        elif self.mode == "zero":
            self.begin, self.end, self.shard = shard_bounds(npad, model.n_params, self.rank, self.world)
            model.set_adam_range(self.begin, max(self.begin, self.end))

    def _inplace_ok(self, dtype) -> bool:
        """Self-test of the in-place reduce-scatter / all-gather this schedule relies on (small
        tensors with known contents, exact in bf16 too; every rank must agree), before any
        capture."""
        dev = self.model.params.device
        k = 64
        try:
            x = (torch.arange(self.world * k, device=dev) % 4 + 4 * self.rank).to(dtype)
            mine = x[self.rank * k:(self.rank + 1) * k]
            dist.reduce_scatter_tensor(mine, x)
            ref = ((torch.arange(self.rank * k, (self.rank + 1) * k, device=dev) % 4) * self.world
                   + 4 * sum(range(self.world))).to(dtype)  # every partial sum <= 256: exact in bf16
            ok = bool(torch.equal(mine, ref))
            y = torch.zeros(self.world * k, dtype=dtype, device=dev)
            y[self.rank * k:(self.rank + 1) * k] = self.rank + 1
            dist.all_gather_into_tensor(y, y[self.rank * k:(self.rank + 1) * k])
            ok = ok and bool(torch.equal(y, torch.arange(1, self.world + 1, device=dev)
                                         .to(dtype).repeat_interleave(k)))
        except Exception:
            ok = False
        flag = torch.tensor([1.0 if ok else 0.0], device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item() == 1.0)

    # ---- collectives ----------------------------------------------------------------------
    def allreduce_grads(self):
        if self.world == 1:
            return
        if self.comm is not None:
            self.comm.allreduce_(self.model.grads)
        else:
            dist.all_reduce(self.model.grads)

    def _reduce_scatter(self, g):
        """Sum over ranks, the rank's shard landing in place in its own copy of g."""
        mine = g[self.rank * self.shard:(self.rank + 1) * self.shard]
        if self._nccl:
            dist.reduce_scatter_tensor(mine, g)  # in place: output == input + rank * count
        else:
            dist.all_reduce(g)  # gloo: the shard of the full sum is the same bytes

    def _all_gather(self, p):
        mine = p[self.rank * self.shard:(self.rank + 1) * self.shard]
        if self._nccl:
            dist.all_gather_into_tensor(p, mine)  # in place: input == output + rank * count
        else:
            parts = list(p.view(self.world, self.shard).unbind(0))
            got = [torch.empty_like(x) for x in parts]
            dist.all_gather(got, mine.clone())
            for dst, src in zip(parts, got):
                dst.copy_(src)

    def reduce_scatter_grads(self):
        if self.wire == "bf16":
            self._reduce_scatter(self.grad_wire)
            dist.all_reduce(self.model.grads[self.extent:self.model.n_params])  # fp32 tail
        else:
            self._reduce_scatter(self.model.grads)

    def all_gather_params(self):
        self._all_gather(self.param_wire if self.wire == "bf16" else self.model.params)

    def refresh_shadows(self):
        if self.wire == "bf16":
            self.model.wire_shadows()
        else:
            self.model.sync_shadows()

    def exchange_before_adam(self):
        if self.mode == "zero":
            self.reduce_scatter_grads()
        else:
            self.allreduce_grads()

    def exchange_after_adam(self):
        if self.mode == "zero":
            self.all_gather_params()

    def gather_state(self):
        """Full Adam m / v on every rank (the zero schedule keeps them sharded): before a checkpoint."""
        if self.mode != "zero":
            return
        if self.wire == "bf16":
            # W1's fp32 rows (parameters too: other ranks' shards are stale on this one) through
            # a padded staging buffer; the tail is replicated already
            ext = self.extent
            for t in (self.model.params, self.model.adam_m, self.model.adam_v):
                buf = torch.zeros(self.shard * self.world, dtype=t.dtype, device=t.device)
                buf[self.begin:self.end].copy_(t[self.begin:self.end])
                self._all_gather(buf)
                t[:ext].copy_(buf[:ext])
            return
        for t in (self.model.adam_m, self.model.adam_v):
            self._all_gather(t)

    def train_step(self):
        self.model.forward(True)
        self.model.backward()
        self.exchange_before_adam()
        self.model.apply_adam(1.0 / self.world)
        if self.mode == "zero":
            self.all_gather_params()
            self.refresh_shadows()
