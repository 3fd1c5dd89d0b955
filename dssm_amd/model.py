"""The DSSM training step on one MI355X: device arenas + the libdssm.so plan.

This is the engine behind the reference's graph (new_dssm.py:104-217).  All state lives in
torch-allocated HBM used purely as storage:

* one flat fp32 parameter arena ([W_l; b_l] blocks, then BN gamma/beta per tower), plus gradient,
  Adam m and Adam v arenas of the same layout (one RCCL all-reduce covers every gradient);
* an EMA arena for the BN moving averages (non-trainable, as in TF);
* one workspace carved by the library (activations, BN coefficients, CSC transpose, outputs).

No torch op runs on the hot path: forward/backward/Adam are three C-ABI calls that enqueue
HIP kernels on the caller's stream.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr
from .data import CSRBatch


ARENA_ALIGN = 512  # floats: equal 64-aligned shards for world sizes 1, 2, 4, 8


class DSSM:
    def __init__(self, trigram_d: int, widths, query_bs: int, neg: int = 4, lr: float = 0.01,
                 dtype: str = "bf16", max_nnz: Optional[int] = None, device=None, seed: int = 0,
                 gamma: float = 20.0, bn_eps: float = 1e-3, ema_decay: float = 0.5,
                 beta1: float = 0.9, beta2: float = 0.999, adam_eps: float = 1e-8,
                 init: bool = True):
        lib = _lib.load()
        self.lib = lib
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        widths = list(widths)
        self.trigram_d, self.widths, self.query_bs, self.neg = trigram_d, widths, query_bs, neg
        self.rows = query_bs * (2 + neg)
        self.dtype = dtype
        if max_nnz is None:
            max_nnz = self.rows * 96
        self.max_nnz = int(max_nnz)
        cfg = _lib.dssm_config()
        cfg.abi_version = _lib.DSSM_ABI_VERSION
        cfg.trigram_d = trigram_d
        cfg.n_layers = len(widths)
        for i, w in enumerate(widths):
            cfg.widths[i] = w
        cfg.query_bs, cfg.neg, cfg.max_nnz = query_bs, neg, self.max_nnz
        cfg.compute_dtype = {"bf16": _lib.DSSM_BF16, "fp32": _lib.DSSM_F32}[dtype]
        cfg.gamma, cfg.bn_eps, cfg.ema_decay = gamma, bn_eps, ema_decay
        cfg.lr, cfg.beta1, cfg.beta2, cfg.adam_eps = lr, beta1, beta2, adam_eps
        self.cfg = cfg
        self.lr, self.beta1, self.beta2 = lr, beta1, beta2
        check(lib.dssm_config_check(C.byref(cfg)), "config")
        n = lib.dssm_param_count(C.byref(cfg))
        self.n_params = int(n)
        nseg = lib.dssm_param_layout(C.byref(cfg), None, 0)
        segs = (_lib.dssm_segment * nseg)()
        lib.dssm_param_layout(C.byref(cfg), segs, nseg)
        self.segments = {s.name.decode(): (int(s.offset), int(s.rows), int(s.cols)) for s in segs}
        dev = self.device
        f32 = torch.float32
        # arenas padded to a multiple of ARENA_ALIGN floats (zeros the library never touches) so a
        # data-parallel reduce-scatter / all-gather splits them into equal 64-float-aligned shards
        npad = -(-n // ARENA_ALIGN) * ARENA_ALIGN
        self.params = torch.zeros(npad, dtype=f32, device=dev)
        self.grads = torch.zeros(npad, dtype=f32, device=dev)
        self.adam_m = torch.zeros(npad, dtype=f32, device=dev)
        self.adam_v = torch.zeros(npad, dtype=f32, device=dev)
        self.ema = torch.zeros(lib.dssm_ema_count(C.byref(cfg)), dtype=f32, device=dev)
        wsb = lib.dssm_workspace_bytes(C.byref(cfg))
        self.workspace = torch.zeros(wsb, dtype=torch.uint8, device=dev)
        self._indptr = torch.zeros(self.rows + 1, dtype=torch.int32, device=dev)
        self._indices = torch.zeros(max(1, self.max_nnz), dtype=torch.int32, device=dev)
        self._values = torch.zeros(max(1, self.max_nnz), dtype=f32, device=dev)
        h = C.c_void_p()
        check(lib.dssm_plan_create(C.byref(cfg), ptr(self.workspace), wsb, ptr(self.params),
                                   ptr(self.grads), ptr(self.adam_m), ptr(self.adam_v),
                                   ptr(self.ema), C.byref(h)), "plan_create")
        self._plan = h
        self.global_step = 0
        self._graphs = {}
        self.fused_w1_adam = True
        if init:
            self.init_params(seed)

    # ---- parameters ------------------------------------------------------------------------
    def segment(self, name: str) -> torch.Tensor:
        off, rows, cols = self.segments[name]
        return self.params[off:off + rows * cols].view(rows, cols)

    def _named_views(self, arena: torch.Tensor) -> Dict[str, torch.Tensor]:
        out = {}
        for l in range(1, len(self.widths) + 1):
            off, rows, cols = self.segments[f"fc{l}"]
            blk = arena[off:off + rows * cols].view(rows, cols)
            out[f"W{l}"] = blk[:-1]
            out[f"b{l}"] = blk[-1]
            for t in ("q", "d"):
                for k in ("gamma", "beta"):
                    o, _, c = self.segments[f"bn{l}_{t}_{k}"]
                    out[f"bn{l}_{t}_{k}"] = arena[o:o + c]
        return out

    def named_params(self) -> Dict[str, torch.Tensor]:
        """Views keyed like the reference variables: W{l}, b{l}, bn{l}_{q|d}_{gamma|beta}."""
        return self._named_views(self.params)

    def named_grads(self) -> Dict[str, torch.Tensor]:
        return self._named_views(self.grads)

    def named_ema(self) -> Dict[str, torch.Tensor]:
        out, o = {}, 0
        for l, n in enumerate(self.widths, start=1):
            for t in ("q", "d"):
                out[f"bn{l}_{t}_mean"] = self.ema[o:o + n]
                out[f"bn{l}_{t}_var"] = self.ema[o + n:o + 2 * n]
                o += 2 * n
        return out

    def init_params(self, seed: int = 0):
        """Reference init (new_dssm.py:118-120, :139-142, :75-76) from numpy PCG64(seed):
        W, b ~ U(-r, r), r = sqrt(6/(fan_in+fan_out)); gamma = 1; beta = 0."""
        rng = np.random.Generator(np.random.PCG64(seed))
        dims = [self.trigram_d] + self.widths
        host = {}
        for l in range(1, len(self.widths) + 1):
            fi, fo = dims[l - 1], dims[l]
            r = np.sqrt(6.0 / (fi + fo))
            host[f"W{l}"] = rng.uniform(-r, r, size=(fi, fo)).astype(np.float32)
            host[f"b{l}"] = rng.uniform(-r, r, size=(fo,)).astype(np.float32)
            for t in ("q", "d"):
                host[f"bn{l}_{t}_gamma"] = np.ones(fo, np.float32)
                host[f"bn{l}_{t}_beta"] = np.zeros(fo, np.float32)
        self.load_params(host)

    def load_params(self, host: Dict[str, np.ndarray], ema: Optional[Dict[str, np.ndarray]] = None):
        views = self.named_params()
        for k, v in host.items():
            views[k].copy_(torch.as_tensor(np.asarray(v, np.float32)).reshape(views[k].shape))
        if ema is not None:
            ev = self.named_ema()
            for k, v in ema.items():
                ev[k].copy_(torch.as_tensor(np.asarray(v, np.float32)))
        check(self.lib.dssm_plan_sync_shadows(self._plan, stream_ptr()), "sync_shadows")

    def load_adam_state(self, m: Dict[str, np.ndarray], v: Dict[str, np.ndarray],
                        beta1_power: float, beta2_power: float, step: int = 0):
        """Load named Adam slots (keys like named_params()) and the TF beta-power accumulators."""
        for arena, src in ((self.adam_m, m), (self.adam_v, v)):
            views = self._named_views(arena)
            for k, a in src.items():
                views[k].copy_(torch.as_tensor(np.asarray(a, np.float32)).reshape(views[k].shape))
        self.set_beta_powers(beta1_power, beta2_power)
        self.global_step = int(step)

    # TF's beta1_power/beta2_power variables live on the device (advanced by the Adam launch, so a
    # captured step needs no host scalars).
    def beta_powers(self, stream=None):
        b1, b2 = C.c_float(), C.c_float()
        check(self.lib.dssm_plan_get_adam_state(self._plan, C.byref(b1), C.byref(b2),
                                                stream_ptr(stream)), "get_adam_state")
        return np.float32(b1.value), np.float32(b2.value)

    def set_beta_powers(self, beta1_power: float, beta2_power: float, stream=None):
        check(self.lib.dssm_plan_set_adam_state(self._plan, float(beta1_power), float(beta2_power),
                                                stream_ptr(stream)), "set_adam_state")

    @property
    def beta1_power(self):
        return self.beta_powers()[0]

    @property
    def beta2_power(self):
        return self.beta_powers()[1]

    def named_adam(self):
        return self._named_views(self.adam_m), self._named_views(self.adam_v)

    # ---- feed --------------------------------------------------------------------------------
    def set_batch(self, batch: CSRBatch = None, indptr=None, indices=None, values=None,
                  non_blocking: bool = False):
        """Point the plan at one step's combined CSR.  Host batches are copied into the model's
        device staging buffers; device tensors are used in place (no copy)."""
        if batch is not None:
            if batch.rows != self.rows:
                raise ValueError(f"batch has {batch.rows} rows, model expects {self.rows}")
            if batch.nnz > self.max_nnz:
                raise ValueError(f"batch nnz {batch.nnz} exceeds max_nnz {self.max_nnz}")
            nz = batch.nnz
            if nz and (int(batch.indices.max()) >= self.trigram_d or int(batch.indices.min()) < 0):
                raise ValueError("batch column index out of [0, TRIGRAM_D)")
            if batch.indptr[0] != 0 or np.any(np.diff(batch.indptr) < 0):
                raise ValueError("batch indptr must start at 0 and be non-decreasing")
            self._indptr.copy_(torch.from_numpy(batch.indptr), non_blocking=non_blocking)
            if nz:
                self._indices[:nz].copy_(torch.from_numpy(batch.indices), non_blocking=non_blocking)
                self._values[:nz].copy_(torch.from_numpy(batch.values), non_blocking=non_blocking)
            indptr, indices, values = self._indptr, self._indices, self._values
        for t, dt in ((indptr, torch.int32), (indices, torch.int32), (values, torch.float32)):
            if t.device != self.device or t.dtype != dt or not t.is_contiguous():
                raise ValueError("device batch tensors must be contiguous int32/int32/float32 on the model device")
        self._batch_refs = (indptr, indices, values)
        check(self.lib.dssm_plan_set_batch(self._plan, ptr(indptr), ptr(indices), ptr(values)),
              "set_batch")

    def set_fused_w1_adam(self, on: bool):
        """Single-GPU fast path (default): dW1's light rows are computed inside Adam and the
        split-K slabs of dW_l (l >= 2) are summed there, so neither is materialized in the gradient
        arena.  Must be off for the data-parallel all-reduce or to read the gradients."""
        check(self.lib.dssm_plan_set_fused_w1_adam(self._plan, 1 if on else 0), "set_fused")
        self.fused_w1_adam = bool(on)

    # ---- step ---------------------------------------------------------------------------------
    def forward(self, train: bool = True, stream=None):
        check(self.lib.dssm_plan_forward(self._plan, 1 if train else 0, stream_ptr(stream)), "forward")

    def backward(self, stream=None):
        check(self.lib.dssm_plan_backward(self._plan, stream_ptr(stream)), "backward")

    def sync_shadows(self, stream=None):
        """Rewrite the bf16 weight shadows from the fp32 parameters (after an external update)."""
        check(self.lib.dssm_plan_sync_shadows(self._plan, stream_ptr(stream)), "sync_shadows")

    def set_adam_range(self, begin: int = 0, end: Optional[int] = None):
        """Optimizer shard: Adam updates arena elements [begin, end) only (data parallel)."""
        end = self.n_params if end is None else int(end)
        check(self.lib.dssm_plan_set_adam_range(self._plan, int(begin), int(end)), "set_adam_range")

    def apply_adam(self, grad_scale: float = 1.0, stream=None):
        check(self.lib.dssm_plan_adam(self._plan, float(grad_scale), stream_ptr(stream)), "adam")
        self.global_step += 1

    # ---- data-parallel bf16 wire (include/dssm.h dssm_plan_set_dp_wire) --------------------------
    def wire_extent(self) -> int:
        """Arena elements [0, extent) that cross the links as bf16 (W1's rows)."""
        return int(self.lib.dssm_plan_wire_extent(self._plan))

    def dp_wire_size(self, world: int, chunks: int = 1) -> int:
        """Elements each wire buffer needs for this world size and chunk count."""
        n = int(self.lib.dssm_plan_dp_wire_size(self._plan, int(world), int(chunks)))
        if n < 0:
            raise ValueError("world and chunks must be >= 1")
        return n

    def set_dp_wire(self, world: int = 1, rank: int = 0, chunks: int = 1, grad_wire=None, stage=None,
                    param_wire=None):
        """Attach (or detach, all None) the bf16 wire of a world-size `world` exchange in `chunks`
        pieces: backward() then ends by writing every rank's W1 gradient rows into grad_wire, the
        caller all-to-alls chunk p of grad_wire into chunk p of stage, apply_adam() updates this
        rank's W1 shard from the fp32 sum of the stage's partials and writes bf16(W1) of it into
        param_wire, the caller all-gathers param_wire chunk by chunk, wire_shadows() rebuilds W1's
        shadow from it.  Layout: dp_geometry()."""
        if grad_wire is None and stage is None and param_wire is None:
            check(self.lib.dssm_plan_set_dp_wire(self._plan, 1, 0, 1, None, None, None, 0), "set_dp_wire")
            self._wires = None
            return
        for t in (grad_wire, stage, param_wire):
            if t.dtype != torch.bfloat16 or not t.is_contiguous() or t.device != self.device:
                raise ValueError("wires are contiguous bf16 tensors on the model's device")
        n = min(grad_wire.numel(), stage.numel(), param_wire.numel())
        check(self.lib.dssm_plan_set_dp_wire(self._plan, int(world), int(rank), int(chunks), ptr(grad_wire),
                                             ptr(stage), ptr(param_wire), n), "set_dp_wire")
        self._wires = (grad_wire, stage, param_wire)

    # ---- the touched-row sparse exchange (dssm_amd/dist.py DataParallel(sparse=True)) ----------
    def touched_rows(self, indices=None, nnz=None) -> torch.Tensor:
        """Ascending W1 rows (trigram columns) the current batch -- or (indices, nnz) -- touches: the
        rows whose gradient can be non-zero (int32, on the device)."""
        if indices is None:
            ip, indices, _ = self._batch_refs
            nnz = int(ip[-1].item())
        return torch.unique(indices[:nnz]).to(torch.int32)

    def rows_pack(self, src, n: int, rows, out, stream=None):
        """dssm_rows_pack_u16: packed bf16 rows (stride n + 4, the row id in front) of src rows."""
        check(self.lib.dssm_rows_pack_u16(ptr(src), n, ptr(rows), rows.numel(), ptr(out), stream_ptr(stream)),
              "rows_pack")

    def rows_unpack(self, packed, n: int, count: int, row_base: int, nrows: int, dst, stream=None):
        """dssm_rows_unpack_u16: packed rows back into dst rows (id - row_base)."""
        check(self.lib.dssm_rows_unpack_u16(ptr(packed), n, count, row_base, nrows, ptr(dst),
                                            stream_ptr(stream)), "rows_unpack")

    def dp_geometry(self) -> Dict[str, int]:
        """The wire layout (dssm_plan_dp_geometry): world, chunks, rows per sub-chunk, elements per
        rank and chunk ('sub'), this rank's W1 shard [shard_begin, shard_end) in the arena, the wire
        extent and the parameter count."""
        out = (C.c_int64 * 8)()
        check(self.lib.dssm_plan_dp_geometry(self._plan, out), "dp_geometry")
        keys = ("world", "chunks", "rows", "sub", "shard_begin", "shard_end", "extent", "n_params")
        return {k: int(v) for k, v in zip(keys, out)}

    def set_dp_peers(self, world: int, stages, param_wires, tails, flags):
        """The peer-store exchange (dssm_plan_set_dp_peers): every rank's stage / parameter wire /
        tail stage / flags as device addresses (ints) indexed by rank, this rank's own included (its
        stage and parameter wire the ones set_dp_wire attached).  All None: off."""
        if stages is None:
            check(self.lib.dssm_plan_set_dp_peers(self._plan, 0, None, None, None, None), "set_dp_peers")
            return
        arr = [(C.c_void_p * world)(*[int(x) for x in lst]) for lst in (stages, param_wires, tails, flags)]
        check(self.lib.dssm_plan_set_dp_peers(self._plan, int(world), *arr), "set_dp_peers")

    def set_peer_timeout(self, ms: float):
        check(self.lib.dssm_plan_set_peer_timeout(self._plan, float(ms)), "set_peer_timeout")

    def peer_exchange(self, phase: int, stream=None):
        """dssm_plan_peer_exchange: phase 0 between backward and Adam, 1 after Adam."""
        check(self.lib.dssm_plan_peer_exchange(self._plan, int(phase), stream_ptr(stream)), "peer_exchange")

    def peer_selftest(self, stream=None) -> int:
        """dssm_plan_peer_selftest: mismatching elements of the synthetic exchange (-1: timed out)."""
        out = C.c_int64(0)
        check(self.lib.dssm_plan_peer_selftest(self._plan, C.byref(out), stream_ptr(stream)), "peer_selftest")
        return int(out.value)

    def peer_status(self) -> Dict[str, int]:
        """{error: 0 or 1 + the flag index a wait timed out on, steps: exchanged steps} (synchronous)."""
        out = (C.c_uint * 2)()
        check(self.lib.dssm_plan_peer_status(self._plan, out), "peer_status")
        return {"error": int(out[0]), "steps": int(out[1])}

    def wire_shadows(self, stream=None):
        check(self.lib.dssm_plan_wire_shadows(self._plan, stream_ptr(stream)), "wire_shadows")

    def train_step(self, stream=None):
        """One sess.run(train_step) (new_dssm.py:267): forward(train) + backward + Adam."""
        check(self.lib.dssm_plan_train_step(self._plan, stream_ptr(stream)), "train_step")
        self.global_step += 1

    # ---- hipGraph capture of a whole step ----------------------------------------------------
    def graph_build(self, parts: int = _lib.GRAPH_FWD_BWD | _lib.GRAPH_ADAM, grad_scale: float = 1.0,
                    probes: bool = False, stream=None) -> int:
        """Capture the step for the CURRENT batch (set_batch) into a hipGraph owned by the plan.
        Capture records work only; nothing runs until graph_launch.  Needs a non-default stream."""
        sp = stream_ptr(stream)
        if not sp:
            raise ValueError("graph capture needs a non-default stream (torch.cuda.Stream())")
        gid = C.c_int()
        check(self.lib.dssm_plan_graph_build(self._plan, int(parts), float(grad_scale),
                                             1 if probes else 0, sp, C.byref(gid)), "graph_build")
        self._graphs[gid.value] = (parts, self._batch_refs)  # keep the batch tensors alive
        return gid.value

    def graph_build_steps(self, batches, probes=False, stream=None) -> int:
        """Capture len(batches) whole training steps back to back into ONE graph, step i on the
        device CSR batch (indptr, indices, values) = batches[i]; a replay runs all of them (the
        host launch boundary is paid once per replay, not once per step).  probes: True = every
        probe (transpose / SpMM / dW1 in the first step, Adam in the last), "adam" = the Adam probe
        alone (two event-record nodes instead of eight)."""
        sp = stream_ptr(stream)
        if not sp:
            raise ValueError("graph capture needs a non-default stream (torch.cuda.Stream())")
        n = len(batches)
        arr = [(C.c_void_p * n)(*[ptr(b[k]) for b in batches]) for k in range(3)]
        gid = C.c_int()
        check(self.lib.dssm_plan_graph_build_steps(self._plan, arr[0], arr[1], arr[2], n,
                                                   2 if probes == "adam" else (1 if probes else 0), sp,
                                                   C.byref(gid)),
              "graph_build_steps")
        self._graphs[gid.value] = (_lib.GRAPH_FWD_BWD | _lib.GRAPH_ADAM, tuple(batches), n)
        return gid.value

    def graph_build_dp_steps(self, batches, grad_scale: float, comm: int = 0, link_gbps: float = 0.0,
                             latency_us: float = 0.0, overlap: bool = False, probes: bool = False,
                             stream=None) -> int:
        """len(batches) data-parallel steps on the bf16 wire (set_dp_wire) in ONE graph, collectives
        included (dssm_plan_graph_build_dp_steps); overlap must be False (the two-stream variant was
        removed in round 3).  comm 0: the library's RCCL communicator; 1 / 2: one-GPU
        rehearsals (device copies / a modelled link time of latency_us + bytes / link_gbps)."""
        sp = stream_ptr(stream)
        if not sp:
            raise ValueError("graph capture needs a non-default stream (torch.cuda.Stream())")
        n = len(batches)
        arr = [(C.c_void_p * n)(*[ptr(b[k]) for b in batches]) for k in range(3)]
        gid = C.c_int()
        check(self.lib.dssm_plan_graph_build_dp_steps(self._plan, arr[0], arr[1], arr[2], n, float(grad_scale),
                                                      int(comm), float(link_gbps), float(latency_us),
                                                      1 if overlap else 0, 1 if probes else 0, sp, C.byref(gid)),
              "graph_build_dp_steps")
        self._graphs[gid.value] = (_lib.GRAPH_FWD_BWD | _lib.GRAPH_ADAM, tuple(batches), n)
        return gid.value

    def graph_launch(self, gid: int, stream=None):
        check(self.lib.dssm_plan_graph_launch(self._plan, int(gid), stream_ptr(stream)), "graph_launch")
        g = self._graphs[gid]
        if g[0] & _lib.GRAPH_ADAM:
            self.global_step += g[2] if len(g) > 2 else 1

    def graph_probe_read(self, gid: int, probe_id: int) -> float:
        ms = C.c_float()
        check(self.lib.dssm_plan_graph_probe_read(self._plan, int(gid), int(probe_id), C.byref(ms)),
              "graph_probe_read")
        return float(ms.value)

    def graph_topology(self, gid: int) -> Dict[str, int]:
        """The captured graph's shape (dssm_plan_graph_topology): node / edge / root counts, nodes
        by type, and chain = 1 when every node is ordered after every node captured before it."""
        out = (C.c_int64 * 8)()
        check(self.lib.dssm_plan_graph_topology(self._plan, int(gid), out), "graph_topology")
        keys = ("nodes", "edges", "roots", "kernel", "memcpy", "memset", "other", "chain")
        return {k: int(v) for k, v in zip(keys, out)}

    def set_option(self, name: str, value: bool):
        """Choose a schedule alternative (dssm_plan_set_option; OPTIONS in _lib): applies to the
        steps enqueued and graphs captured afterwards.  The plan never reads the environment."""
        check(self.lib.dssm_plan_set_option(self._plan, _lib.OPTIONS[name], 1 if value else 0),
              f"set_option {name}")
        if name == "FUSED_W1_ADAM":
            self.fused_w1_adam = bool(value)

    def get_option(self, name: str) -> bool:
        v = int(self.lib.dssm_plan_get_option(self._plan, _lib.OPTIONS[name]))
        if v < 0:
            raise _lib.DssmError(f"bad option {name}")
        return bool(v)

    @property
    def fused_stats(self) -> bool:
        """True when bf16 train steps run with the BN statistics fused (csrc/bnfuse.h)."""
        return bool(self.lib.dssm_plan_fused_stats(self._plan))

    def schedule(self) -> Dict[str, bool]:
        """Which kernels a train step of this plan runs (dssm_plan_schedule, DSSM_SCHED_*)."""
        f = int(self.lib.dssm_plan_schedule(self._plan))
        return {k: bool(f & b) for k, b in _lib.SCHED_BITS.items()}

    # ---- kernel timing probes (HIP events on the launch stream) -------------------------------
    def probe_enable(self, probe_id: int, max_samples: int):
        check(self.lib.dssm_plan_probe_enable(self._plan, probe_id, max_samples), "probe_enable")

    def probe_read(self, probe_id: int):
        tot, cnt = C.c_float(), C.c_int()
        check(self.lib.dssm_plan_probe_read(self._plan, probe_id, C.byref(tot), C.byref(cnt)), "probe_read")
        return float(tot.value), int(cnt.value)

    # ---- fetches ------------------------------------------------------------------------------
    def _buf(self, bid: int, layer: int = -1):
        p, nb = C.c_void_p(), C.c_size_t()
        check(self.lib.dssm_plan_buffer(self._plan, bid, layer, C.byref(p), C.byref(nb)), "buffer")
        return p.value - self.workspace.data_ptr(), nb.value

    def buffer(self, bid: int, layer: int = -1, dtype=torch.float32) -> torch.Tensor:
        off, nb = self._buf(bid, layer)
        return self.workspace[off:off + nb].view(dtype)

    def loss_accuracy(self):
        check(self.lib.dssm_plan_finalize_loss(self._plan, stream_ptr(None)), "finalize_loss")
        la = self.buffer(_lib.BUF_LOSS).cpu().numpy()
        return float(la[0]), float(la[1])

    def fetch(self, name: str) -> np.ndarray:
        K = self.neg + 1
        BS = self.query_bs
        if name == "loss":
            return np.float32(self.loss_accuracy()[0])
        if name == "accuracy":
            return np.float32(self.loss_accuracy()[1])
        if name == "cos_sim_raw":
            return self.buffer(_lib.BUF_COS_SIM_RAW).cpu().numpy().reshape(K * BS, 1)
        if name == "cos_sim":
            return self.buffer(_lib.BUF_COS_SIM).cpu().numpy().reshape(BS, K)
        if name == "prob":
            return self.buffer(_lib.BUF_PROB).cpu().numpy().reshape(BS, K)
        if name == "query_norm_single":
            return self.buffer(_lib.BUF_QUERY_NORM).cpu().numpy().reshape(BS, 1)
        if name.startswith("embedding"):
            n = self.widths[-1]
            ld = (n + 7) // 8 * 8
            y = self.buffer(_lib.BUF_EMBED).cpu().numpy().reshape(self.rows, ld)[:, :n]
            return {"embedding_query_y": y[:BS], "embedding_doc_positive_y": y[BS:2 * BS],
                    "embedding_doc_negative_y": y[2 * BS:], "embedding_all": y}[name]
        raise KeyError(name)

    def batch_moments(self, layer: int):
        n = self.widths[layer - 1]
        m = self.buffer(_lib.BUF_BATCH_MEAN, layer - 1).cpu().numpy().reshape(2, n)
        v = self.buffer(_lib.BUF_BATCH_VAR, layer - 1).cpu().numpy().reshape(2, n)
        return {"q": (m[0], v[0]), "d": (m[1], v[1])}

    # ---- checkpoint (new_dssm.py:248,331 tf.train.Saver) ---------------------------------------
    def state_dict(self) -> Dict[str, np.ndarray]:
        n = self.n_params
        return {"params": self.params[:n].cpu().numpy(), "adam_m": self.adam_m[:n].cpu().numpy(),
                "adam_v": self.adam_v[:n].cpu().numpy(), "ema": self.ema.cpu().numpy(),
                "beta_powers": np.array(self.beta_powers(), np.float32),
                "global_step": np.array([self.global_step], np.int64)}

    def load_state_dict(self, sd: Dict[str, np.ndarray]):
        for name, t in (("params", self.params), ("adam_m", self.adam_m), ("adam_v", self.adam_v),
                        ("ema", self.ema)):
            a = np.asarray(sd[name], np.float32)
            if name != "ema" and a.shape == (self.n_params,):
                t = t[:self.n_params]  # arenas are stored without their shard padding
            if a.shape != tuple(t.shape):
                raise ValueError(f"checkpoint {name} shape {a.shape} != {tuple(t.shape)}")
            t.copy_(torch.from_numpy(a))
        self.set_beta_powers(*(float(x) for x in sd["beta_powers"]))
        self.global_step = int(sd["global_step"][0])
        check(self.lib.dssm_plan_sync_shadows(self._plan, stream_ptr()), "sync_shadows")

    def save(self, path: str):
        np.savez(path, **self.state_dict())

    def restore(self, path: str):
        with np.load(path, allow_pickle=False) as z:
            self.load_state_dict({k: z[k] for k in z.files})

    def __del__(self):
        try:
            if getattr(self, "_plan", None) is not None and self.lib is not None:
                torch.cuda.synchronize(self.device)
                self.lib.dssm_plan_destroy(self._plan)
                self._plan = None
        except Exception:
            pass
