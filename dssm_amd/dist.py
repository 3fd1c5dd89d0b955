"""Data parallelism: one process per GPU, batch sharded by query.

Each rank runs the whole step on its shard (its queries, their positives and negatives) with
local BN statistics (the reference's BN semantics applied per replica, new_dssm.py:62-88) and a
loss normalised by the local batch; the ranks then exchange gradients and apply the same
TF1.x Adam step (new_dssm.py:215-217), so the data-parallel step equals the oracle's mean of the
per-shard gradients followed by Adam.  EMA shadows stay rank-local (rank 0's are checkpointed).

Two exchange schedules over the flat fp32 arenas:

* "zero" (default for world sizes 2, 4, 8): the optimizer pass (the step's largest HBM-bound
  kernel) shrinks by the world size.  Each rank updates only its shard of W1's rows and then the
  updated shards are all-gathered.  The wire ("wire" argument) is
  - "bf16" (default for a bf16 model): the backward writes bf16(dW1) into a gradient wire; an
    ALL-TO-ALL delivers to every rank the bf16 gradients of ITS shard from every rank, which the
    Adam launch sums in fp32 in rank order (dssm_plan_set_wire_stage: one bf16 rounding per
    rank's gradient, no rounding per ring hop as a bf16 reduce-scatter would add); Adam writes
    bf16(W1) of the shard into a parameter wire that is all-gathered, and W1's bf16 shadow is
    rebuilt from it.  The small tail ([extent, n_params): b1, W2.., BN) is all-reduced in fp32
    and updated replicated, so every rank's biases / BN parameters stay bit-identical fp32;
  - "fp32": reduce-scatter of the fp32 gradient arena, all-gather of the fp32 parameters.
  W1's fp32 master rows / Adam m, v outside a rank's shard are stale until gather_state().
* "allreduce": one all-reduce of the gradient arena and replicated Adam.

Transports for the same collectives:

* "rccl" (default on GPUs): libdssm.so's own RCCL communicator (dssm_comm_* / dssm_all_to_all ...
  in include/dssm.h), so no torch op runs on the data path; its 128-byte unique id is broadcast
  through torch.distributed once (bootstrap only);
* "torch": torch.distributed (gloo on the CPU tests; the "nccl" backend = RCCL as a fallback).

Every collective the chosen schedule uses is self-tested at start-up on small exact patterns
(every rank must agree); a failing library transport falls back to torch.distributed, a failing
in-place schedule to "allreduce".
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.distributed as dist

from . import _lib
from ._lib import check, ptr, stream_ptr


def _dtype_id(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return _lib.DSSM_F32
    if t.dtype == torch.bfloat16:
        return _lib.DSSM_BF16
    raise TypeError(f"collectives move fp32 / bf16 tensors, not {t.dtype}")


class TorchTransport:
    """torch.distributed collectives (gloo on CPU; nccl = RCCL as a fallback)."""
    name = "torch"

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world
        self.nccl = dist.get_backend() == "nccl"

    def all_reduce(self, t):
        dist.all_reduce(t)

    def reduce_scatter_(self, t, shard: int):
        """Sum over ranks; the rank's shard lands in place in its own copy of t."""
        mine = t[self.rank * shard:(self.rank + 1) * shard]
        if self.nccl:
            dist.reduce_scatter_tensor(mine, t)  # in place: output == input + rank * count
        else:
            dist.all_reduce(t)  # gloo: the shard of the full sum is the same bytes

    def all_gather_(self, t, shard: int):
        mine = t[self.rank * shard:(self.rank + 1) * shard]
        if self.nccl:
            dist.all_gather_into_tensor(t, mine)  # in place: input == output + rank * count
        else:
            parts = list(t.view(self.world, shard).unbind(0))
            got = [torch.empty_like(x) for x in parts]
            dist.all_gather(got, mine.clone())
            for dst, src in zip(parts, got):
                dst.copy_(src)

    def all_to_all(self, send, recv):
        dist.all_to_all_single(recv, send)

    def destroy(self):
        pass


class LibTransport:
    """libdssm.so's RCCL communicator: collectives enqueued on the current stream, no torch op."""
    name = "rccl"

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world
        lib = _lib.load()
        self.lib = lib
        buf = (C.c_char * 128)()
        if rank == 0:
            check(lib.dssm_comm_unique_id(buf), "comm_unique_id")
        obj = [bytes(buf)]
        dist.broadcast_object_list(obj, src=0)
        buf = (C.c_char * 128).from_buffer_copy(obj[0])
        check(lib.dssm_comm_init(rank, world, buf), "comm_init")

    def all_reduce(self, t):
        check(self.lib.dssm_allreduce_sum(ptr(t), t.numel(), _dtype_id(t), stream_ptr()), "allreduce")

    def reduce_scatter_(self, t, shard: int):
        mine = t[self.rank * shard:(self.rank + 1) * shard]
        check(self.lib.dssm_reduce_scatter_sum(ptr(t), ptr(mine), shard, _dtype_id(t), stream_ptr()),
              "reduce_scatter")

    def all_gather_(self, t, shard: int):
        mine = t[self.rank * shard:(self.rank + 1) * shard]
        check(self.lib.dssm_all_gather(ptr(mine), ptr(t), shard, _dtype_id(t), stream_ptr()), "all_gather")

    def all_to_all(self, send, recv):
        assert send.numel() == recv.numel() and send.numel() % self.world == 0
        check(self.lib.dssm_all_to_all(ptr(send), ptr(recv), send.numel() // self.world, _dtype_id(send),
                                       stream_ptr()), "all_to_all")

    def destroy(self):
        self.lib.dssm_comm_destroy()


def shard_bounds(n_pad: int, n: int, rank: int, world: int):
    """Rank's optimizer shard of an arena of n elements padded to n_pad (equal shards)."""
    s = n_pad // world
    return rank * s, min((rank + 1) * s, n), s


class DataParallel:
    """Wraps a DSSM model: step = forward + backward + gradient exchange + Adam (see module doc)."""

    def __init__(self, model, comm: str = "auto", mode: str = "auto", wire: str = "auto"):
        self.model = model
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        npad = model.params.numel()
        if mode == "auto":
            mode = "zero" if (self.world > 1 and npad % (64 * self.world) == 0) else "allreduce"
        if mode == "zero" and npad % (64 * self.world):
            raise ValueError("the zero schedule needs 64-float aligned equal shards")
        if mode not in ("zero", "allreduce"):
            raise ValueError("mode: 'zero', 'allreduce' or 'auto'")
        self.mode = mode if self.world > 1 else "allreduce"
        if wire == "auto":
            wire = "bf16" if getattr(model, "dtype", "fp32") == "bf16" else "fp32"
        if wire not in ("bf16", "fp32"):
            raise ValueError("wire: 'bf16' or 'fp32'")
        self.wire = wire if self.mode == "zero" else "fp32"
        self.tx = None
        if self.world > 1:
            model.set_fused_w1_adam(False)  # the exchange needs the materialized dW1
            self.tx = self._transport(comm)
        self.grad_wire = self.param_wire = self.stage = None
        if self.mode == "zero" and self.wire == "bf16":
            ext = model.wire_extent()
            self.extent = ext
            self.shard = -(-ext // (64 * self.world)) * 64
            self.begin, self.end = self.rank * self.shard, min((self.rank + 1) * self.shard, ext)
            n = self.shard * self.world
            dev = model.params.device
            self.grad_wire = torch.zeros(n, dtype=torch.bfloat16, device=dev)
            self.param_wire = torch.zeros(n, dtype=torch.bfloat16, device=dev)
            self.stage = torch.zeros(n, dtype=torch.bfloat16, device=dev)
            self.param_wire[:ext].copy_(model.params[:ext])
            model.set_wire(self.grad_wire, self.param_wire)
            model.set_wire_stage(self.stage, self.world, self.shard)
            model.set_adam_range(self.begin, max(self.begin, self.end))
        elif self.mode == "zero":
            self.begin, self.end, self.shard = shard_bounds(npad, model.n_params, self.rank, self.world)
            model.set_adam_range(self.begin, max(self.begin, self.end))

    @property
    def comm(self) -> str:
        return self.tx.name if self.tx is not None else "none"

    def _transport(self, comm: str):
        """The library's RCCL communicator on GPUs (comm "auto" / "rccl"), torch.distributed
        otherwise; each candidate must pass the self-test of the collectives it will run."""
        cands = []
        gpu = self.model.params.is_cuda and dist.get_backend() == "nccl"
        if comm in ("auto", "rccl") and gpu:
            cands.append(LibTransport)
        if comm in ("auto", "torch") or not cands:
            cands.append(TorchTransport)
        for cls in cands:
            try:
                tx = cls(self.rank, self.world)
            except Exception:
                ok, tx = False, None
            else:
                ok = self._selftest(tx)
            if self._agree(ok):
                return tx
            if tx is not None:
                tx.destroy()
        if self.mode == "zero":
            self.mode, self.wire = "allreduce", "fp32"  # last resort: one all-reduce
        return TorchTransport(self.rank, self.world)

    def _agree(self, ok: bool) -> bool:
        flag = torch.tensor([1.0 if ok else 0.0], device=self.model.params.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item() == 1.0)

    def _selftest(self, tx) -> bool:
        """Small tensors with known contents (every partial sum exact in bf16) through every
        collective this schedule uses, before any capture."""
        dev = self.model.params.device
        w, r, k = self.world, self.rank, 64
        try:
            ok = True
            for dt in (torch.float32, torch.bfloat16):
                x = (torch.arange(w * k, device=dev) % 4 + 4 * r).to(dt)
                tx.reduce_scatter_(x, k)
                ref = ((torch.arange(r * k, (r + 1) * k, device=dev) % 4) * w + 4 * sum(range(w))).to(dt)
                ok = ok and bool(torch.equal(x[r * k:(r + 1) * k], ref))
                y = torch.zeros(w * k, dtype=dt, device=dev)
                y[r * k:(r + 1) * k] = r + 1
                tx.all_gather_(y, k)
                ok = ok and bool(torch.equal(y, torch.arange(1, w + 1, device=dev).to(dt).repeat_interleave(k)))
                s = (torch.arange(w, device=dev) + 8 * r).to(dt).repeat_interleave(k)  # chunk j: j + 8r
                d = torch.zeros_like(s)
                tx.all_to_all(s, d)
                want = (torch.arange(w, device=dev) * 8 + r).to(dt).repeat_interleave(k)  # from rank j: r + 8j
                ok = ok and bool(torch.equal(d, want))
                z = torch.full((k,), float(r + 1), dtype=dt, device=dev)
                tx.all_reduce(z)
                ok = ok and bool(torch.equal(z, torch.full((k,), float(w * (w + 1) // 2), dtype=dt, device=dev)))
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            return ok
        except Exception:
            return False

    # ---- collectives ----------------------------------------------------------------------
    def exchange_before_adam(self):
        if self.world == 1:
            return
        g = self.model.grads
        if self.mode != "zero":
            self.tx.all_reduce(g)
        elif self.wire == "bf16":
            self.tx.all_to_all(self.grad_wire, self.stage)  # every rank's bf16 slice of MY shard
            self.tx.all_reduce(g[self.extent:self.model.n_params])  # the fp32 tail, replicated
        else:
            self.tx.reduce_scatter_(g, self.shard)

    def exchange_after_adam(self):
        if self.mode == "zero":
            self.tx.all_gather_(self.param_wire if self.wire == "bf16" else self.model.params, self.shard)

    def refresh_shadows(self):
        if self.wire == "bf16":
            self.model.wire_shadows()
        else:
            self.model.sync_shadows()

    def gather_state(self):
        """Full parameters and Adam m / v on every rank (the zero schedule keeps W1's sharded):
        before a checkpoint."""
        if self.mode != "zero":
            return
        if self.wire == "bf16":
            # W1's fp32 rows (parameters too: other ranks' shards are stale on this one) through
            # a padded staging buffer; the tail is replicated already
            ext = self.extent
            for t in (self.model.params, self.model.adam_m, self.model.adam_v):
                buf = torch.zeros(self.shard * self.world, dtype=t.dtype, device=t.device)
                buf[self.begin:self.end].copy_(t[self.begin:self.end])
                self.tx.all_gather_(buf, self.shard)
                t[:ext].copy_(buf[:ext])
            return
        for t in (self.model.adam_m, self.model.adam_v):
            self.tx.all_gather_(t, self.shard)

    def train_step(self):
        self.model.forward(True)
        self.model.backward()
        self.exchange_before_adam()
        self.model.apply_adam(1.0 / self.world)
        if self.mode == "zero":
            self.exchange_after_adam()
            self.refresh_shadows()

    def close(self):
        if self.tx is not None:
            self.tx.destroy()
            self.tx = None
