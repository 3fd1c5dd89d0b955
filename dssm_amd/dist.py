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
    Adam launch sums in fp32 in rank order (dssm_plan_set_dp_wire: one bf16 rounding per
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

exchange="peer" (bf16 wire, one chunk; PeerBuffers below, csrc/peer.hip): no collective on the data
path at all.  The gradient pass stores each owner's bf16 W1 rows straight into that owner's stage
(HIP IPC-mapped fine-grained buffers), the fp32 tail is pushed to every rank and summed there in
rank order, and each Adam shard stores its bf16 rows into every rank's parameter wire; per-step
epoch flags order the hand-offs (DESIGN §6 "peer exchange").  The transport is then used only for
bootstrap (the IPC handles) and gather_state().

Every collective the chosen schedule uses (SCHEDULE_OPS) is self-tested at start-up on small exact
patterns and every rank must agree.  With comm="auto" a failing library transport falls back to
torch.distributed and a failing zero schedule (mode="auto") is demoted to "allreduce"; each such
fallback is warned about and listed in DataParallel.fallbacks (bench.py puts it in its JSON line).
comm="rccl" and mode="zero" are strict: a failure raises on every rank instead.
"""
from __future__ import annotations

import ctypes as C
import warnings

import torch
import torch.distributed as dist

from . import _lib
from ._lib import check, ptr, stream_ptr


def _dtype_id(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return _lib.DSSM_F32
    if t.dtype == torch.bfloat16:
        return _lib.DSSM_BF16
    if t.dtype == torch.int32:
        return _lib.DSSM_I32
    raise TypeError(f"collectives move fp32 / bf16 / int32 tensors, not {t.dtype}")


class TorchTransport:
    """torch.distributed collectives: "nccl" (= RCCL) on GPUs as a fallback, gloo on the CPU tests.
    gloo with device tensors (world-2 rehearsals sharing one GPU) stages every collective through
    host memory, so each op keeps the same in-place semantics as the device transports."""
    name = "torch"

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world
        self.nccl = dist.get_backend() == "nccl"

    def _host(self, fn, *ts):
        """Run fn on host copies of device tensors (gloo), then copy the results back."""
        if self.nccl or not any(t.is_cuda for t in ts):
            fn(*ts)
            return
        hs = [t.cpu() for t in ts]
        fn(*hs)
        for t, h in zip(ts, hs):
            t.copy_(h)

    def all_reduce(self, t):
        self._host(dist.all_reduce, t)

    def reduce_scatter_(self, t, shard: int):
        """Sum over ranks; the rank's shard lands in place in its own copy of t."""
        if self.nccl:
            mine = t[self.rank * shard:(self.rank + 1) * shard]
            dist.reduce_scatter_tensor(mine, t)  # in place: output == input + rank * count
        else:
            self._host(dist.all_reduce, t)  # gloo: the shard of the full sum is the same bytes

    def all_gather_(self, t, shard: int):
        if self.nccl:
            mine = t[self.rank * shard:(self.rank + 1) * shard]
            dist.all_gather_into_tensor(t, mine)  # in place: input == output + rank * count
            return

        def gather(x):
            parts = list(x.view(self.world, shard).unbind(0))
            got = [torch.empty_like(p) for p in parts]
            dist.all_gather(got, parts[self.rank].clone())
            for dst, src in zip(parts, got):
                dst.copy_(src)
        self._host(gather, t)

    def all_to_all(self, send, recv):
        self._host(lambda s, r: dist.all_to_all_single(r, s), send, recv)

    def all_to_all_tail(self, send, recv, tail):
        """The all-to-all and the tail's all-reduce (two calls: torch.distributed has no group)."""
        self.all_to_all(send, recv)
        self.all_reduce(tail)

    def all_to_allv(self, send, send_counts, recv, recv_counts, tail=None):
        """send_counts[j] elements of send to rank j, recv_counts[j] from rank j; tail all-reduced."""
        self._host(lambda s, r: dist.all_to_all_single(r, s, output_split_sizes=list(recv_counts),
                                                       input_split_sizes=list(send_counts)), send, recv)
        if tail is not None:
            self.all_reduce(tail)

    def info(self) -> dict:
        ver = None
        if self.nccl:
            try:
                v = torch.cuda.nccl.version()
                ver = v[0] * 10000 + v[1] * 100 + v[2] if isinstance(v, tuple) else int(v)
            except Exception:  # noqa: BLE001 - informational only
                ver = None
        return {"transport": f"torch.distributed {dist.get_backend()}", "comm_world": dist.get_world_size(),
                "comm_rank": dist.get_rank(), "rccl_version": ver}

    def destroy(self):
        pass


class LibTransport:
    """libdssm.so's RCCL communicator: collectives enqueued on the current stream, no torch op.

    Bootstrap: rank 0 creates the 128-byte unique id and broadcasts (status, id) through
    torch.distributed, so a failure on rank 0 reaches every rank in the same collective and all of
    them raise together (DataParallel's transport selection then agrees on the next candidate)."""
    name = "rccl"
    capturable = True  # RCCL calls may be captured into a hipGraph

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world
        lib = _lib.load()
        self.lib = lib
        buf = (C.c_char * 128)()
        status, msg = True, ""
        if rank == 0:
            if lib.dssm_comm_unique_id(buf) != 0:
                status, msg = False, lib.dssm_last_error().decode()
        obj = [(status, msg, bytes(buf))]
        dist.broadcast_object_list(obj, src=0)
        status, msg, raw = obj[0]
        if not status:
            raise _lib.DssmError(f"rank 0 could not create the RCCL unique id: {msg}")
        buf = (C.c_char * 128).from_buffer_copy(raw)
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

    def all_to_all_tail(self, send, recv, tail):
        """dssm_all_to_all_tail: the all-to-all with the fp32 tail's all-reduce in the same RCCL group
        (the call the step graph captures under TAIL_IN_A2A)."""
        assert send.numel() == recv.numel() and send.numel() % self.world == 0 and tail.dtype == torch.float32
        check(self.lib.dssm_all_to_all_tail(ptr(send), ptr(recv), send.numel() // self.world, _dtype_id(send),
                                            ptr(tail), tail.numel(), stream_ptr()), "all_to_all_tail")

    def all_to_allv(self, send, send_counts, recv, recv_counts, tail=None):
        """dssm_all_to_allv: grouped sends / receives of per-peer counts, the tail's all-reduce in the
        same RCCL group (tail=None: the sends / receives alone)."""
        W = self.world
        sc, rc = (C.c_int64 * W)(*send_counts), (C.c_int64 * W)(*recv_counts)
        tp, tn, td = (ptr(tail), tail.numel(), _dtype_id(tail)) if tail is not None else (None, 0, 0)
        check(self.lib.dssm_all_to_allv(ptr(send), sc, ptr(recv), rc, _dtype_id(send), tp, tn, td, stream_ptr()),
              "all_to_allv")

    def info(self) -> dict:
        """The communicator as RCCL reports it (dssm_comm_info): its rank count, this rank, version."""
        w, r, v = C.c_int(), C.c_int(), C.c_int()
        check(self.lib.dssm_comm_info(C.byref(w), C.byref(r), C.byref(v)), "comm_info")
        return {"transport": "libdssm rccl", "comm_world": w.value, "comm_rank": r.value,
                "rccl_version": v.value}

    def destroy(self):
        self.lib.dssm_comm_destroy()


# The collectives (op, dtype) each exchange schedule runs: only these are self-tested.
SCHEDULE_OPS = {
    ("allreduce", "fp32"): (("all_reduce", torch.float32),),
    ("zero", "fp32"): (("reduce_scatter", torch.float32), ("all_gather", torch.float32)),
    ("zero", "bf16"): (("all_to_all", torch.bfloat16), ("all_reduce", torch.float32),
                       ("all_gather", torch.bfloat16), ("all_gather", torch.float32)),
}


def selftest(tx, ops, device, rank: int, world: int) -> bool:
    """Small tensors with known contents (every partial sum exact in bf16) through the given
    collectives, before any capture."""
    w, r, k = world, rank, 64
    try:
        ok = True
        for op, dt in ops:
            if op == "reduce_scatter":
                x = (torch.arange(w * k, device=device) % 4 + 4 * r).to(dt)
                tx.reduce_scatter_(x, k)
                ref = ((torch.arange(r * k, (r + 1) * k, device=device) % 4) * w + 4 * sum(range(w))).to(dt)
                ok = ok and bool(torch.equal(x[r * k:(r + 1) * k], ref))
            elif op == "all_gather":
                y = torch.zeros(w * k, dtype=dt, device=device)
                y[r * k:(r + 1) * k] = r + 1
                tx.all_gather_(y, k)
                ok = ok and bool(torch.equal(y, torch.arange(1, w + 1, device=device).to(dt).repeat_interleave(k)))
            elif op == "all_to_all":
                s = (torch.arange(w, device=device) + 8 * r).to(dt).repeat_interleave(k)  # chunk j: j + 8r
                d = torch.zeros_like(s)
                tx.all_to_all(s, d)
                want = (torch.arange(w, device=device) * 8 + r).to(dt).repeat_interleave(k)  # from j: r + 8j
                ok = ok and bool(torch.equal(d, want))
            elif op == "all_reduce":
                z = torch.full((k,), float(r + 1), dtype=dt, device=device)
                tx.all_reduce(z)
                ok = ok and bool(torch.equal(z, torch.full((k,), float(w * (w + 1) // 2), dtype=dt, device=device)))
            elif op in ("all_to_all_tail", "all_to_all_tail_captured"):
                # the mixed point-to-point / collective RCCL group of TAIL_IN_A2A; "captured": recorded
                # into a graph and replayed twice (each replay re-sums the tail: r + 1, then w(w+1)/2 * w)
                s = (torch.arange(w, device=device) + 8 * r).to(dt).repeat_interleave(k)
                d = torch.zeros_like(s)
                tail = torch.full((k + 3,), float(r + 1), dtype=torch.float32, device=device)
                want = (torch.arange(w, device=device) * 8 + r).to(dt).repeat_interleave(k)
                tot = float(w * (w + 1) // 2)
                if op == "all_to_all_tail":
                    tx.all_to_all_tail(s, d, tail)
                    wt = tot
                else:
                    side = torch.cuda.Stream(device)
                    side.wait_stream(torch.cuda.current_stream(device))
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                        tx.all_to_all_tail(s, d, tail)
                    torch.cuda.current_stream(device).wait_stream(side)
                    for _ in range(2):
                        g.replay()
                    wt = tot * w
                ok = ok and bool(torch.equal(d, want))
                ok = ok and bool(torch.equal(tail, torch.full_like(tail, wt)))
            else:
                raise ValueError(op)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        return ok
    except Exception:
        return False


def agree(ok: bool, device) -> bool:
    """True on every rank iff ok on every rank (one MIN all-reduce)."""
    flag = torch.tensor([1.0 if ok else 0.0], device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item() == 1.0)


def select_transport(rank: int, world: int, device, comm: str, ops) -> "tuple":
    """The first candidate transport that every rank can build and that passes the self-test of
    `ops` on every rank: the library's RCCL communicator on GPUs under the nccl backend (comm
    "auto" / "rccl"), then torch.distributed (comm "auto" / "torch").  comm="rccl" is strict: no
    fallback, a failure raises on every rank.  Returns (transport or None, [fallback notes])."""
    if comm not in ("auto", "rccl", "torch"):
        raise ValueError("comm: 'auto', 'rccl' or 'torch'")
    gpu = device.type == "cuda" and dist.get_backend() == "nccl"
    cands = []
    if comm in ("auto", "rccl") and gpu:
        cands.append(LibTransport)
    if comm == "torch" or (comm == "auto"):
        cands.append(TorchTransport)
    notes = []
    for cls in cands:
        err = ""
        try:
            tx = cls(rank, world)
        except Exception as e:  # noqa: BLE001 - every rank learns the outcome through agree()
            ok, tx, err = False, None, repr(e)
        else:
            ok = selftest(tx, ops, device, rank, world)
            if not ok:
                err = "self-test mismatch"
        if agree(ok, device):
            return tx, notes
        if tx is not None:
            tx.destroy()
        notes.append(f"{cls.name} transport failed ({err or 'on another rank'})")
    if comm == "rccl":
        raise RuntimeError("comm='rccl' requested but libdssm.so's RCCL transport failed: " + "; ".join(notes))
    return None, notes


class _DeviceArray:
    """__cuda_array_interface__ of library-allocated device memory (for a torch view of it)."""

    def __init__(self, addr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (int(n),), "typestr": typestr, "data": (int(addr), False),
                                         "version": 2}


def device_view(addr: int, n: int, dtype, device) -> torch.Tensor:
    """A torch tensor over n elements at device address addr (not owned: keep the allocation alive)."""
    ts = {torch.bfloat16: "<i2", torch.float32: "<f4", torch.int32: "<i4"}[dtype]
    t = torch.as_tensor(_DeviceArray(addr, n, ts), device=device)
    return t.view(torch.bfloat16) if dtype == torch.bfloat16 else t


class PeerBuffers:
    """The peer-store exchange's buffers (include/dssm.h dssm_peer_alloc / dssm_ipc_*): this rank's
    fine-grained stage, parameter wire, tail stage and flags, and every other rank's, mapped through
    HIP IPC with handles exchanged once over torch.distributed (all_gather_object).  addr[kind][r]
    is rank r's buffer as seen from this process.  A barrier follows, so every rank's zeroed flags
    exist before any rank's first step."""

    KINDS = ("stage", "pwire", "tail", "flags")

    def __init__(self, world: int, rank: int, wire_n: int, tail_n: int, device):
        self.lib = _lib.load()
        self.world, self.rank = world, rank
        sizes = {"stage": 2 * wire_n, "pwire": 2 * wire_n, "tail": 4 * world * tail_n,
                 "flags": _lib.PEER_FLAG_BYTES}
        self.own, self.opened = {}, []
        try:
            for k in self.KINDS:
                p = C.c_void_p()
                check(self.lib.dssm_peer_alloc(sizes[k], C.byref(p)), f"peer_alloc {k}")
                self.own[k] = int(p.value)
            handles = {}
            for k in self.KINDS:
                h = C.create_string_buffer(64)
                check(self.lib.dssm_ipc_handle(C.c_void_p(self.own[k]), h), f"ipc_handle {k}")
                handles[k] = h.raw
            handles["device"] = torch.cuda.current_device()
            allh = [None] * world
            if world > 1:
                dist.all_gather_object(allh, handles)
            else:
                allh[0] = handles
            # every rank's device must be able to map every other rank's (hipDeviceCanAccessPeer)
            # before any handle is opened: an unsupported pair raises here, not as a GPU fault
            ok = C.c_int(0)
            bad = []
            for r in range(world):
                check(self.lib.dssm_peer_can_access(int(allh[r]["device"]), C.byref(ok)), "peer_can_access")
                if not ok.value:
                    bad.append(r)
            dev = torch.device("cuda", torch.cuda.current_device())
            all_ok = agree(not bad, dev) if world > 1 else not bad
            if not all_ok:
                raise RuntimeError(f"peer exchange: this device cannot access the devices of ranks {bad} "
                                   "(or another rank's cannot): use the collective exchange")
            self.addr = {k: [0] * world for k in self.KINDS}
            for r in range(world):
                for k in self.KINDS:
                    if r == rank:
                        self.addr[k][r] = self.own[k]
                        continue
                    p = C.c_void_p()
                    check(self.lib.dssm_ipc_open(C.create_string_buffer(allh[r][k], 64), C.byref(p)),
                          f"ipc_open rank {r} {k}")
                    self.opened.append(int(p.value))
                    self.addr[k][r] = int(p.value)
        except Exception:
            self._release()
            raise
        self.stage = device_view(self.own["stage"], wire_n, torch.bfloat16, device)
        self.param_wire = device_view(self.own["pwire"], wire_n, torch.bfloat16, device)

    def _release(self):
        for a in self.opened:
            self.lib.dssm_ipc_close(C.c_void_p(a))
        self.opened = []
        for a in self.own.values():
            self.lib.dssm_peer_free(C.c_void_p(a))
        self.own = {}

    def close(self):
        """Unmap the peers' buffers and free this rank's, after every rank is done with them."""
        if not self.own:
            return
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        self.stage = self.param_wire = None
        self._release()


class RehearsalPeers:
    """bench.py --rehearse-world W --rehearse-comm peer: rank 0 of a W-rank peer exchange on ONE GPU.
    Every rank's buffers are local allocations (so rank 0's kernels store the same bytes into W
    stages / parameter wires / tail slots as on W GPUs, at HBM instead of xGMI speed), and the other
    ranks' flags in rank 0's flags buffer are raised in advance, so its waits pass at once: the
    compute share of the per-rank step, to which DESIGN §6 adds the link time."""

    def __init__(self, world: int, wire_n: int, tail_n: int, device):
        self.lib = _lib.load()
        self.addr = {k: [] for k in PeerBuffers.KINDS}
        sizes = {"stage": 2 * wire_n, "pwire": 2 * wire_n, "tail": 4 * world * tail_n,
                 "flags": _lib.PEER_FLAG_BYTES}
        for _ in range(world):
            for k in PeerBuffers.KINDS:
                p = C.c_void_p()
                check(self.lib.dssm_peer_alloc(sizes[k], C.byref(p)), f"peer_alloc {k}")
                self.addr[k].append(int(p.value))
        self.stage = device_view(self.addr["stage"][0], wire_n, torch.bfloat16, device)
        self.param_wire = device_view(self.addr["pwire"][0], wire_n, torch.bfloat16, device)
        flags = device_view(self.addr["flags"][0], _lib.PEER_FLAG_BYTES // 4, torch.int32, device)
        for base in (0, 64):  # DSSM peer flags GRAD / PARAM (csrc/launch.h kPeerGrad / kPeerParam)
            flags[base + 1:base + world].fill_(0x7FFFFFFF)
        torch.cuda.synchronize()

    def close(self):
        torch.cuda.synchronize()
        self.stage = self.param_wire = None
        for lst in self.addr.values():
            for a in lst:
                self.lib.dssm_peer_free(C.c_void_p(a))
        self.addr = {}


def shard_bounds(n_pad: int, n: int, rank: int, world: int):
    """Rank's optimizer shard of an arena of n elements padded to n_pad (equal shards)."""
    s = n_pad // world
    return rank * s, min((rank + 1) * s, n), s


class DataParallel:
    """Wraps a DSSM model: step = forward + backward + gradient exchange + Adam (see module doc)."""

    def __init__(self, model, comm: str = "auto", mode: str = "auto", wire: str = "auto", chunks: int = 1,
                 overlap: bool = False, sparse: bool = False, tail_in_a2a="auto", verify_sparse: bool = True,
                 exchange: str = "collective", peer_timeout_ms: float = 0.0):
        """comm: "auto" (the library's RCCL communicator on GPUs, torch.distributed as the
        self-tested fallback), "rccl" (strict: no fallback) or "torch".  mode / wire: "auto" picks
        zero + bf16 wire for bf16 models; an explicit "zero" is strict (never demoted).  Every
        fallback taken is listed in .fallbacks and warned about.
        sparse (zero / bf16 wire, one chunk): the touched-row gradient exchange -- each rank sends
        to rank j only the W1 gradient rows of j's shard its batch touched (packed with their row
        ids; the counts exchanged first), the fp32 tail's all-reduce in the same RCCL group; the
        receiver scatters them into the zeroed stage, so Adam sums exactly the dense exchange's
        values.  The counts are known only on the host after the batch is read, so this exchange runs
        between captured graphs (never inside one).
        tail_in_a2a (zero / bf16 wire): the fp32 tail's all-reduce inside the last all-to-all's RCCL
        group (plan option TAIL_IN_A2A: one collective launch fewer per step).  "auto" (default):
        on when that mixed group passes its start-up self-test on every rank, eagerly and captured in
        a graph (library transport), otherwise the tail is all-reduced separately and the demotion
        is recorded in .fallbacks; True: strict (a failing self-test raises); False: off.
        verify_sparse: before the first step, one exchange of a synthetic gradient through the
        sparse path and the dense all-to-all; the stages must be bit-identical on every rank, or the
        sparse path is turned off (recorded in .fallbacks).
        exchange: "collective" (the schedules above) or "peer" (the peer-store exchange: zero / bf16
        wire in one chunk, HIP-engine models on GPUs, world <= 8; no fallback: a failure raises).
        peer_timeout_ms: the peer waits' bound (0: the library's default, 20 s)."""
        if overlap:  # removed in round 3: slower; refused before any side effect
            raise ValueError("overlap is no longer supported: the exchange runs on one captured stream")
        if exchange not in ("collective", "peer"):
            raise ValueError("exchange: 'collective' or 'peer'")
        self.model = model
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.peer = None
        if exchange == "peer":
            if mode not in ("auto", "zero") or wire not in ("auto", "bf16") or int(chunks) != 1 or sparse:
                raise ValueError("the peer exchange is the zero schedule on the bf16 wire in one chunk")
            if getattr(model, "dtype", "fp32") != "bf16" or not hasattr(model, "set_dp_peers"):
                raise ValueError("the peer exchange needs a bf16 HIP-engine model")
            if self.world > 8:
                raise ValueError("the peer exchange supports at most 8 ranks")
            mode, wire, tail_in_a2a = "zero", "bf16", False
        npad = model.params.numel()
        strict_mode = mode == "zero"
        if mode == "auto":
            mode = "zero" if (self.world > 1 and npad % (64 * self.world) == 0) else "allreduce"
        if mode == "zero" and npad % (64 * self.world):
            raise ValueError("the zero schedule needs 64-float aligned equal shards")
        if mode not in ("zero", "allreduce"):
            raise ValueError("mode: 'zero', 'allreduce' or 'auto'")
        self.mode = mode if (self.world > 1 or exchange == "peer") else "allreduce"
        if wire == "auto":
            wire = "bf16" if getattr(model, "dtype", "fp32") == "bf16" else "fp32"
        if wire not in ("bf16", "fp32"):
            raise ValueError("wire: 'bf16' or 'fp32'")
        self.wire = wire if self.mode == "zero" else "fp32"
        self.tx = None
        self.fallbacks = []
        if self.world > 1 or exchange == "peer":
            model.set_fused_w1_adam(False)  # the exchange needs the materialized dW1
        if self.world > 1:
            self.tx = self._transport(comm, strict_mode)
        self.grad_wire = self.param_wire = self.stage = None
        self.chunks, self.overlap = 1, False
        if self.mode == "zero" and self.wire == "bf16":
            # the W1 rows in `chunks` pieces (include/dssm.h dssm_plan_set_dp_wire): chunk p of each
            # collective is one contiguous block of world * sub elements
            self.chunks = max(1, int(chunks))
            n = model.dp_wire_size(self.world, self.chunks)
            dev = model.params.device
            self.grad_wire = torch.zeros(n, dtype=torch.bfloat16, device=dev)
            if exchange == "peer":  # the stage and parameter wire are the fine-grained, IPC-shared ones
                model.set_dp_wire(self.world, self.rank, 1, self.grad_wire,
                                  torch.zeros(n, dtype=torch.bfloat16, device=dev), self.grad_wire.clone())
                geo0 = model.dp_geometry()
                self.peer = PeerBuffers(self.world, self.rank, n, geo0["n_params"] - geo0["extent"], dev)
                self.param_wire, self.stage = self.peer.param_wire, self.peer.stage
            else:
                self.param_wire = torch.zeros(n, dtype=torch.bfloat16, device=dev)
                self.stage = torch.zeros(n, dtype=torch.bfloat16, device=dev)
            model.set_dp_wire(self.world, self.rank, self.chunks, self.grad_wire, self.stage, self.param_wire)
            if self.peer is not None:
                a = self.peer.addr
                model.set_dp_peers(self.world, a["stage"], a["pwire"], a["tail"], a["flags"])
                if peer_timeout_ms > 0:
                    model.set_peer_timeout(peer_timeout_ms)
                torch.cuda.synchronize()
                if self.world > 1:
                    dist.barrier()  # every rank's zeroed flags attached before any rank's first step
                # the exchange's store / release / flag / load path checked at the real world size with
                # synthetic patterns (dssm_plan_peer_selftest); any mismatch on any rank raises
                self.peer_selftest = model.peer_selftest()
                ok = self.peer_selftest == 0
                if not (agree(ok, dev) if self.world > 1 else ok):
                    raise RuntimeError(f"peer exchange self-test failed on some rank (this rank: "
                                       f"{self.peer_selftest} mismatching elements, -1 = timed out)")
            geo = model.dp_geometry()
            self.extent, self.sub = geo["extent"], geo["sub"]
            self.begin, self.end = geo["shard_begin"], geo["shard_end"]
            self.shard = self.chunks * self.sub  # W1 elements per rank (the last rank's padded)
            self.rows = geo["rows"]              # W1 rows per rank and chunk
            self.width = self.sub // self.rows   # W1 row length on the wire
        elif self.mode == "zero":
            self.begin, self.end, self.shard = shard_bounds(npad, model.n_params, self.rank, self.world)
            model.set_adam_range(self.begin, max(self.begin, self.end))
        self.sparse = bool(sparse)
        if self.sparse and not (self.mode == "zero" and self.wire == "bf16" and self.chunks == 1):
            raise ValueError("sparse exchange: the zero schedule with the bf16 wire in one chunk")
        self._staged_indices = None
        self._cur = None
        self.sparse_stats = {"steps": 0, "rows_sent": 0, "rows_dense": 0}
        self.tail_group = False
        if self.world > 1 and self.mode == "zero" and self.wire == "bf16" and tail_in_a2a is not False:
            self._select_tail_group(strict=tail_in_a2a is True)
        if self.sparse and verify_sparse and self.world > 1:
            self._verify_sparse()

    def _select_tail_group(self, strict: bool):
        """TAIL_IN_A2A on iff the mixed group passes its self-test on every rank (see __init__)."""
        dev = self.model.params.device
        ops = [("all_to_all_tail", torch.bfloat16)]
        if getattr(self.tx, "capturable", False) and dev.type == "cuda":
            ops.append(("all_to_all_tail_captured", torch.bfloat16))
        ok = agree(selftest(self.tx, ops, dev, self.rank, self.world), dev)
        if ok:
            self.tail_group = True
            if hasattr(self.model, "set_option"):  # the plan's captured step (CPU engines: eager only)
                self.model.set_option("TAIL_IN_A2A", True)
            return
        if strict:
            raise RuntimeError("tail_in_a2a=True but the mixed all-to-all + all-reduce group failed its self-test")
        note = "mixed all-to-all + tail all-reduce group failed its self-test: tail all-reduced separately"
        self.fallbacks.append(note)
        warnings.warn(f"DataParallel: {note}", RuntimeWarning, stacklevel=3)
    @property
    def comm(self) -> str:
        return self.tx.name if self.tx is not None else "none"

    @property
    def schedule(self) -> str:
        """What the exchange runs, e.g. "zero/bf16 via rccl" (bench.py's config.dp_exchange)."""
        s = f"{self.mode}/{self.wire}" if self.mode == "zero" else self.mode
        if getattr(self, "peer", None) is not None:
            return f"{s} via peer stores"
        if getattr(self, "sparse", False):
            s += " sparse"
        if getattr(self, "tail_group", False):
            s += " tail-in-a2a"
        return f"{s} via {self.comm}"

    def _transport(self, comm: str, strict_mode: bool):
        """The transport for this schedule (select_transport); with no working transport a
        non-strict zero schedule is demoted to "allreduce" (one fp32 all-reduce), whose smaller
        set of collectives is tried again.  Every fallback is recorded and warned about."""
        dev = self.model.params.device
        tx, notes = select_transport(self.rank, self.world, dev, comm, SCHEDULE_OPS[(self.mode, self.wire)])
        self.fallbacks += notes
        if tx is None and self.mode == "zero" and not strict_mode:
            self.fallbacks.append(f"zero/{self.wire} schedule demoted to allreduce")
            self.mode, self.wire = "allreduce", "fp32"
            tx, notes = select_transport(self.rank, self.world, dev, comm, SCHEDULE_OPS[("allreduce", "fp32")])
            self.fallbacks += notes
        if tx is None:
            raise RuntimeError("no working transport for the data-parallel exchange: " + "; ".join(self.fallbacks))
        for note in self.fallbacks:
            warnings.warn(f"DataParallel: {note}", RuntimeWarning, stacklevel=3)
        return tx

    # ---- collectives ----------------------------------------------------------------------
    def _sparse_exchange(self, ids=None, stats: bool = True):
        """The touched-row gradient all-to-all (see __init__): this rank's batch's W1 rows (the
        columns its CSR holds, torch.unique) split by owner rank, packed with their ids
        (dssm_rows_pack_u16), the counts all-to-all'd, the packed rows exchanged (with the tail's
        all-reduce in the same group when that group passed its self-test, tail_group; otherwise
        the tail's all-reduce follows), and scattered into the zeroed stage (dssm_rows_unpack_u16)."""
        m, W = self.model, self.world
        if ids is None:
            ids = m.touched_rows(*(self._cur or ()))  # ascending W1 rows the batch touched (int32)
        S, n, dev = self.rows, self.width, ids.device
        cut = torch.searchsorted(ids, torch.arange(1, W, device=dev, dtype=torch.int32) * S)
        bounds = torch.cat([torch.zeros(1, dtype=cut.dtype, device=dev), cut,
                            torch.full((1,), ids.numel(), dtype=cut.dtype, device=dev)])
        send_rows = (bounds[1:] - bounds[:-1]).to(torch.int32)
        recv_rows = torch.empty_like(send_rows)
        self.tx.all_to_all(send_rows, recv_rows)
        sc, rc = send_rows.tolist(), recv_rows.tolist()  # the sizes, on the host (sync)
        stride = n + 4
        sbuf = torch.empty(max(1, ids.numel()) * stride, dtype=torch.bfloat16, device=dev)
        m.rows_pack(self.grad_wire, n, ids, sbuf)
        rbuf = torch.empty(max(1, sum(rc)) * stride, dtype=torch.bfloat16, device=dev)
        tail = m.grads[self.extent:m.n_params]
        self.tx.all_to_allv(sbuf, [c * stride for c in sc], rbuf, [c * stride for c in rc],
                            tail=tail if self.tail_group else None)
        if not self.tail_group:
            self.tx.all_reduce(tail)
        self.stage.zero_()
        off = 0
        for i in range(W):  # stage block i: rank i's gradient rows of this rank's shard
            dst = self.stage[i * self.sub:(i + 1) * self.sub]
            m.rows_unpack(rbuf[off * stride:(off + rc[i]) * stride], n, rc[i], self.rank * S, S, dst)
            off += rc[i]
        if not stats:
            return
        st = self.sparse_stats
        st["steps"] += 1
        st["rows_sent"] += ids.numel()
        st["rows_dense"] += W * S

    def _verify_sparse(self):
        """The sparse exchange against the dense all-to-all at the real world size and transport (see
        __init__): a synthetic bf16 gradient (exact small integers) on a seeded subset of W1 rows,
        zero elsewhere, exchanged both ways; the two stages must be bit-identical on every rank.
        The wires, the stage and the gradient tail are cleared afterwards."""
        m, dev = self.model, self.model.params.device
        g = torch.Generator(device="cpu").manual_seed(1234 + self.rank)
        nrows = self.world * self.rows
        touched = torch.randperm(nrows, generator=g)[:max(1, nrows // 3)].sort().values
        touched = touched[touched * self.width < self.extent].to(torch.int32)
        n = self.width
        gw = self.grad_wire[:self.world * self.sub].view(-1, n)
        gw.zero_()
        vals = ((torch.arange(n, device=dev) % 7) + 1 + 8 * self.rank).to(torch.bfloat16)
        gw[touched.to(dev).long()] = vals
        tail = m.grads[self.extent:m.n_params]
        tail.fill_(float(self.rank + 1))
        blk = self.world * self.sub  # the exchanged block (the wire may carry a few slack elements)
        dense = torch.zeros_like(self.stage[:blk])
        self.tx.all_to_all(self.grad_wire[:blk], dense)
        self.tx.all_reduce(tail)
        tail_dense = tail.clone()
        tail.fill_(float(self.rank + 1))
        self._sparse_exchange(ids=touched.to(dev), stats=False)
        ok = bool(torch.equal(self.stage[:blk], dense)) and bool(torch.equal(tail, tail_dense))
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        ok = agree(ok, dev)
        self.grad_wire.zero_()
        self.stage.zero_()
        tail.zero_()
        if not ok:
            self.sparse = False
            note = "sparse exchange differed from the dense all-to-all in its start-up check: dense exchange"
            self.fallbacks.append(note)
            warnings.warn(f"DataParallel: {note}", RuntimeWarning, stacklevel=3)

    def exchange_before_adam(self):
        if self.peer is not None:  # the rows went out in the gradient pass: tail push, wait, tail sum
            self.model.peer_exchange(0)
            return
        if self.world == 1:
            return
        g = self.model.grads
        if self.sparse:
            self._sparse_exchange()
            return
        if self.mode != "zero":
            self.tx.all_reduce(g)
        elif self.wire == "bf16":
            blk = self.world * self.sub
            tail = g[self.extent:self.model.n_params]  # the fp32 tail, replicated
            for p in range(self.chunks):  # chunk p: every rank's bf16 slice of MY shard's sub-chunk p
                send, recv = self.grad_wire[p * blk:(p + 1) * blk], self.stage[p * blk:(p + 1) * blk]
                if self.tail_group and p == self.chunks - 1:  # as the captured step (TAIL_IN_A2A)
                    self.tx.all_to_all_tail(send, recv, tail)
                else:
                    self.tx.all_to_all(send, recv)
            if not self.tail_group:
                self.tx.all_reduce(tail)
        else:
            self.tx.reduce_scatter_(g, self.shard)

    def exchange_after_adam(self):
        if self.peer is not None:  # the shard's rows went out in Adam: this rank's flag, wait for all
            self.model.peer_exchange(1)
            return
        if self.mode == "zero" and self.wire == "bf16":
            blk = self.world * self.sub
            for p in range(self.chunks):
                self.tx.all_gather_(self.param_wire[p * blk:(p + 1) * blk], self.sub)
        elif self.mode == "zero":
            self.tx.all_gather_(self.model.params, self.shard)

    def refresh_shadows(self):
        if self.wire == "bf16":
            self.model.wire_shadows()
        else:
            self.model.sync_shadows()

    def gather_state(self):
        """Full parameters and Adam m / v on every rank (the zero schedule keeps W1's sharded):
        before a checkpoint."""
        if self.mode != "zero" or self.world == 1:
            return
        if self.wire == "bf16":
            # W1's fp32 rows (parameters too: other ranks' shards are stale on this one) through
            # a padded staging buffer (rank r's shard: rows [r, r+1) * chunks * S); the tail is
            # replicated already
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

    # ---- captured steps (bench.py's timed path) ----------------------------------------------
    @property
    def capturable(self) -> bool:
        """Whole steps, collectives included, can be captured into one graph: the library's RCCL
        transport with the zero / bf16-wire schedule (dssm_plan_graph_build_dp_steps)."""
        if self.peer is not None:
            return True
        return (getattr(self.tx, "capturable", False) and self.mode == "zero" and self.wire == "bf16"
                and not self.sparse)

    def build_region(self, batches, probes: bool = False) -> int:
        """len(batches) whole data-parallel steps as ONE graph, every node on one captured stream:
        per step the forward, backward, the gradient pass chunk by chunk with each chunk's
        all-to-all behind it, the fp32 tail all-reduce, Adam chunk by chunk with each chunk's
        all-gather behind it, the shadow rebuild (with one chunk only after the region's last step:
        the next step's SpMM reads the parameter wire); step i+1's CSC rank pass inside step i's
        Adam.  Replay: model.graph_launch."""
        if not self.capturable:
            raise RuntimeError(f"the {self.schedule} exchange cannot be captured (needs zero/bf16 via rccl)")
        return self.model.graph_build_dp_steps(batches, 1.0 / self.world, comm=3 if self.peer is not None else 0,
                                               overlap=self.overlap, probes=probes)

    def build_graphs(self, staged, probe_batch=None):
        """Capture, per staged device batch (indptr, indices, values), the forward + backward as a
        hipGraph (plus, under the zero schedule, a variant that first rebuilds the weight shadows
        from the previous step's all-gathered update: one graph boundary fewer per step), and one
        Adam graph.  graph_step() replays them with the exchange's collectives between the graphs.
        probe_batch: the batch whose graphs carry the plan's timing probes."""
        from . import _lib
        m = self.model
        shadow = 0
        if self.mode == "zero" and getattr(m, "dtype", "fp32") == "bf16":
            shadow = _lib.GRAPH_WIRE_SHADOWS if self.wire == "bf16" else _lib.GRAPH_SHADOWS
        self._g_plain, self._g_merged = [], []
        for b, (ip, ix, vv) in enumerate(staged):
            m.set_batch(indptr=ip, indices=ix, values=vv)
            pr = b == probe_batch
            self._g_plain.append(m.graph_build(_lib.GRAPH_FWD_BWD, probes=pr))
            if shadow:
                self._g_merged.append(m.graph_build(_lib.GRAPH_FWD_BWD | shadow, probes=pr))
        self._g_adam = m.graph_build(_lib.GRAPH_ADAM, 1.0 / self.world, probes=probe_batch is not None)
        self._g_shadow = m.graph_build(shadow) if shadow else None
        self._shadows_pending = False
        # the sparse exchange reads the replayed step's batch: its indices and nnz, known once here
        self._staged_indices = [(ix, int(ip[-1].item())) for ip, ix, _ in staged] if self.sparse else None

    def graph_step(self, i: int, events=None):
        """One step on staged batch i (mod the staged count) from the captured graphs.  events: a
        list to which (phase, start, end) torch.cuda.Event pairs recorded on the current stream are
        appended (bench.py's dp_kernels_ms for the host-issued exchange)."""
        m = self.model
        n = len(self._g_plain)

        def timed(name, fn):
            if events is None:
                return fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            events.append((name, a, b))
        timed("fwd_bwd", lambda: m.graph_launch((self._g_merged if self._shadows_pending else self._g_plain)[i % n]))
        if self._staged_indices is not None:
            self._cur = self._staged_indices[i % n]
        timed("exchange_before_adam", self.exchange_before_adam)
        self._cur = None
        timed("adam", lambda: m.graph_launch(self._g_adam))
        if self.mode == "zero":
            timed("exchange_after_adam", self.exchange_after_adam)
            self._shadows_pending = self._g_shadow is not None

    def settle(self):
        """Rebuild the weight shadows a last graph_step left pending (the next graph_step would
        have done it first thing): after the timed region, before reading or saving the model."""
        if getattr(self, "_shadows_pending", False):
            self.model.graph_launch(self._g_shadow)
            self._shadows_pending = False

    def graph_ids(self):
        """(plain fwd+bwd graphs, merged graphs, Adam graph): for reading the timing probes."""
        return self._g_plain, self._g_merged, self._g_adam

    def peer_check(self):
        """Raise if a peer wait timed out (dssm_plan_peer_status); returns the exchanged step count."""
        st = self.model.peer_status()
        if st["error"]:
            raise RuntimeError(f"peer exchange: a wait timed out (flag {st['error'] - 1}) after {st['steps']} steps")
        return st["steps"]

    def close(self):
        if self.peer is not None:
            self.model.set_dp_peers(0, None, None, None, None)
            self.model.set_dp_wire()  # detach: the stage / parameter wire are about to be freed
            self.stage = self.param_wire = None  # views of the freed buffers
            self.peer.close()
            self.peer = None
        if self.tx is not None:
            self.tx.destroy()
            self.tx = None
