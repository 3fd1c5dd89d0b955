"""Data parallelism: one process per GPU, batch sharded by query, one all-reduce of
the flat gradient arena per step (RCCL over xGMI), replicated Adam with grad_scale = 1/world.

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


class DataParallel:
    """Wraps a DSSM model: step(batch) = forward + backward + all-reduce + Adam(1/world)."""

    def __init__(self, model, comm: str = "torch"):
        self.model = model
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.comm = RcclComm(self.rank, self.world) if (comm == "rccl" and self.world > 1) else None
        if self.world > 1:
            model.set_fused_w1_adam(False)  # the all-reduce needs the materialized dW1

    def allreduce_grads(self):
        if self.world == 1:
            return
        if self.comm is not None:
            self.comm.allreduce_(self.model.grads)
        else:
            dist.all_reduce(self.model.grads)

    def train_step(self):
        self.model.forward(True)
        self.model.backward()
        self.allreduce_grads()
        self.model.apply_adam(1.0 / self.world)
