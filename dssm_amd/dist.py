"""Data parallelism: one process per GPU, batch sharded by query.

Two exchange schedules over the flat fp32 arenas (RCCL over xGMI):
* "zero" (default for world sizes 2, 4, 8): reduce-scatter of the gradient arena, Adam on the
  rank's shard only (p, m, v of the shard; grad_scale = 1/world), all-gather of the updated
  parameters, then the bf16 weight shadows refreshed from them.  Same bytes on the links as one
  all-reduce, but the optimizer pass (the largest kernel, HBM-bound) shrinks by the world size.
  m / v live sharded: gather_state() collects them for a checkpoint.
* "allreduce": one all-reduce of the gradient arena and replicated Adam.

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

    def __init__(self, model, comm: str = "torch", mode: str = "auto"):
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
        if self.mode == "zero" and self._nccl and not self._inplace_ok():
            self.mode = "allreduce"  # the in-place collectives misbehaved: exchange by all-reduce
        if self.mode == "zero":
            self.begin, self.end, self.shard = shard_bounds(npad, model.n_params, self.rank, self.world)
            model.set_adam_range(self.begin, max(self.begin, self.end))

    def _inplace_ok(self) -> bool:
        """Self-test of the in-place reduce-scatter / all-gather this schedule relies on (small
        tensors with known contents; every rank must agree), before any capture."""
        dev = self.model.params.device
        k = 64
        try:
            x = torch.arange(self.world * k, dtype=torch.float32, device=dev) + 1000.0 * self.rank
            mine = x[self.rank * k:(self.rank + 1) * k]
            dist.reduce_scatter_tensor(mine, x)
            ref = (torch.arange(self.rank * k, (self.rank + 1) * k, dtype=torch.float32, device=dev)
                   * self.world + 1000.0 * sum(range(self.world)))
            ok = bool(torch.equal(mine, ref))
            y = torch.zeros(self.world * k, dtype=torch.float32, device=dev)
            y[self.rank * k:(self.rank + 1) * k] = self.rank + 1
            dist.all_gather_into_tensor(y, y[self.rank * k:(self.rank + 1) * k])
            ok = ok and bool(torch.equal(y, torch.arange(1, self.world + 1, dtype=torch.float32,
                                                         device=dev).repeat_interleave(k)))
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

    def reduce_scatter_grads(self):
        """Sum of the gradient arenas, the rank's shard landing in place in its own arena."""
        g = self.model.grads
        mine = g[self.rank * self.shard:(self.rank + 1) * self.shard]
        if self._nccl:
            dist.reduce_scatter_tensor(mine, g)  # in place: output == input + rank * count
        else:
            dist.all_reduce(g)  # gloo: the shard of the full sum is the same bytes

    def all_gather_params(self):
        p = self.model.params
        mine = p[self.rank * self.shard:(self.rank + 1) * self.shard]
        if self._nccl:
            dist.all_gather_into_tensor(p, mine)  # in place: input == output + rank * count
        else:
            parts = list(p.view(self.world, self.shard).unbind(0))
            got = [torch.empty_like(x) for x in parts]
            dist.all_gather(got, mine.clone())
            for dst, src in zip(parts, got):
                dst.copy_(src)

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
        for t in (self.model.adam_m, self.model.adam_v):
            mine = t[self.rank * self.shard:(self.rank + 1) * self.shard]
            if self._nccl:
                dist.all_gather_into_tensor(t, mine)
            else:
                parts = list(t.view(self.world, self.shard).unbind(0))
                got = [torch.empty_like(x) for x in parts]
                dist.all_gather(got, mine.clone())
                for dst, src in zip(parts, got):
                    dst.copy_(src)

    def train_step(self):
        self.model.forward(True)
        self.model.backward()
        self.exchange_before_adam()
        self.model.apply_adam(1.0 / self.world)
        if self.mode == "zero":
            self.all_gather_params()
            self.model.sync_shadows()
