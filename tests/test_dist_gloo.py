"""Data-parallel path on CPU: world_size 2, 4 and 8 over gloo (8 = the driver's node).

Each rank runs `dssm_amd.dist.DataParallel` (the product's DP step: forward, backward, the
gradient exchange of its schedule, Adam with grad_scale = 1/world) with the torch.distributed
transport (gloo); on GPUs the same schedules run on libdssm.so's RCCL communicator.  Its shard
comes from `dssm_amd.data.shard_batch`. The per-rank compute engine is the C/OpenMP restatement
(oracle/cpu_c), a test stand-in for the device plan, so the host-side DP logic runs without a GPU.

Schedules: "allreduce" (one fp32 all-reduce, replicated Adam), "zero" with the fp32 wire
(reduce-scatter, sharded Adam, all-gather) and "zero" with the bf16 all-to-all wire (every rank
receives the bf16 gradients of its shard from every rank and sums them in fp32 in rank order).

Parity definition (§8e): the N-rank step equals the oracle's mean of the per-shard gradients
followed by one Adam step. All ranks end bit-identical. Each rank's EMA is its own shard's
(local BN statistics).
"""
import os
import re
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dssm_amd.data import shard_batch, synth_batch
from dssm_amd.dist import DataParallel
from oracle import dssm_oracle as O

cpu_c = pytest.importorskip("oracle.cpu_c")
if not cpu_c.available():
    pytest.skip("gcc/OpenMP unavailable", allow_module_level=True)

D, WIDTHS, BS, NEG = 600, [64, 32], 32, 4


class CpuEngine:
    """The DSSM model interface DataParallel drives (forward/backward/arenas/apply_adam, the
    optimizer range and the shadow refresh of the zero schedule)."""

    def __init__(self, params, world):
        self.cpu = cpu_c.CpuDSSM(D, WIDTHS, BS // world, NEG, params, pad_to=64 * world)
        self.n_params = self.cpu.total
        self.params = torch.from_numpy(self.cpu.flat["p"])  # flat arenas (padded), shared memory
        self.grads = torch.from_numpy(self.cpu.flat["g"])
        self.adam_m = torch.from_numpy(self.cpu.flat["m"])
        self.adam_v = torch.from_numpy(self.cpu.flat["v"])
        self.range = (0, self.n_params)
        self._train = None
        self.gwire = self.pwire = self.stage = None

    # bf16 wire (include/dssm.h dssm_plan_set_dp_wire): W1's rows, arena [0, D*WIDTHS[0]), laid
    # out by sub-chunks: rank j's shard is rows [j*P*S, (j+1)*P*S), sub-chunk (p, j) at ((p*W+j)*S)*n
    def wire_extent(self):
        return D * WIDTHS[0]  # the port's arena starts with W1 [D x L1], like the device layout

    def _geo(self, world, chunks):
        return world, chunks, -(-D // (world * chunks)), WIDTHS[0]

    def dp_wire_size(self, world, chunks):
        w, p, rows, n = self._geo(world, chunks)
        return w * p * rows * n + 8  # the device wire's 8-element slack after the last row (dssm_plan_dp_wire_size)

    def set_dp_wire(self, world, rank, chunks, gw, st, pw):
        self.gwire, self.stage, self.pwire = gw, st, pw
        self.geo, self.wrank = self._geo(world, chunks), rank
        w, p, rows, n = self.geo
        r0 = min(rank * p * rows, D)
        self.range = (r0 * n, min(r0 + p * rows, D) * n)

    def dp_geometry(self):
        w, p, rows, n = self.geo
        b, e = self.range
        return {"world": w, "chunks": p, "rows": rows, "sub": rows * n, "shard_begin": b, "shard_end": e,
                "extent": self.wire_extent(), "n_params": self.n_params}

    def _wpos(self, row):
        w, p, rows, n = self.geo
        j, c, s = row // (rows * p), (row // rows) % p, row % rows
        return ((c * w + j) * rows + s) * n

    def wire_shadows(self):
        pass  # fp32 engine: the bf16 W1 shadow is the parameter wire itself

    def set_fused_w1_adam(self, on):
        pass

    def set_adam_range(self, begin, end):
        self.range = (begin, end)

    def sync_shadows(self):
        pass  # fp32 engine: no bf16 shadows

    def set_batch(self, batch):
        self.batch = batch.as_dict()

    # the touched-row sparse exchange's model hooks (dssm_amd/model.py DSSM.touched_rows / rows_pack /
    # rows_unpack; packed rows of stride n + 4 with the int32 row id in front)
    def touched_rows(self, indices=None, nnz=None):
        ix = self.batch["indices"] if indices is None else indices[:nnz]
        return torch.from_numpy(np.unique(np.asarray(ix)).astype(np.int32))

    def rows_pack(self, src, n, rows, out):
        k = rows.numel()
        o = out[:k * (n + 4)].view(k, n + 4)
        o[:, 4:] = src[:src.numel() // n * n].view(-1, n)[rows.long()]
        o.view(torch.int32)[:, 0] = rows

    def rows_unpack(self, packed, n, count, row_base, nrows, dst):
        pk = packed[:count * (n + 4)].view(count, n + 4)
        ids = pk.view(torch.int32)[:, 0].long() - row_base
        dst[:dst.numel() // n * n].view(-1, n)[ids] = pk[:, 4:]

    def forward(self, train=True):
        self._train = bool(train)

    def backward(self):
        self.loss = self.cpu.forward_backward(self.batch, train=self._train, backward=True)
        if self.gwire is not None:  # the plan's backward ends by writing W1's gradient rows
            n = WIDTHS[0]
            for row in range(D):
                o = self._wpos(row)
                self.gwire[o:o + n] = self.grads[row * n:(row + 1) * n].to(torch.bfloat16)

    def apply_adam(self, grad_scale=1.0):
        # a range step is the full step with the elements outside [begin, end) left as they were
        # (with the wire: [begin, end) from the all-to-all's stage plus the replicated tail)
        keep = {r: self.cpu.flat[r].copy() for r in ("p", "m", "v")}
        b, e = self.range
        if self.gwire is not None:
            ext = self.wire_extent()
            w, p, rows, n = self.geo
            for row in range(b // n, e // n):  # the world's bf16 partials of my rows, fp32 sum in rank order
                c, sr = (row // rows) % p, row % rows
                acc = torch.zeros(n, dtype=torch.float32)
                for k in range(w):
                    o = ((c * w + k) * rows + sr) * n
                    acc += self.stage[o:o + n].float()
                self.grads[row * n:(row + 1) * n] = acc
        self.cpu.adam(grad_scale)
        for r, old in keep.items():
            if self.gwire is not None:
                self.cpu.flat[r][:b] = old[:b]
                self.cpu.flat[r][e:ext] = old[e:ext]
            else:
                self.cpu.flat[r][:b] = old[:b]
                self.cpu.flat[r][e:] = old[e:]
        if self.pwire is not None:
            n = WIDTHS[0]
            for row in range(b // n, e // n):
                o = self._wpos(row)
                self.pwire[o:o + n] = self.params[row * n:(row + 1) * n].to(torch.bfloat16)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, out_dir, mode, wire, world, chunks, sparse=False):
    os.environ["OMP_NUM_THREADS"] = "1" if world >= 8 else "2"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        cfg = O.OracleConfig(trigram_d=D, widths=WIDTHS, query_bs=BS, neg=NEG)
        p0 = O.init_params(cfg, seed=9)
        glob = synth_batch(D, BS, NEG, seed=1234, mean_nnz=16)
        eng = CpuEngine(p0, world)
        dp = DataParallel(eng, comm="auto", mode=mode, wire=wire, chunks=chunks, sparse=sparse)
        assert dp.world == world and dp.rank == rank and dp.mode == mode and dp.comm == "torch"
        assert dp.wire == (wire if mode == "zero" else "fp32")
        # the tail's all-reduce rides in the last all-to-all's group when that group passes its
        # self-test (here: the torch transport's two calls); the sparse path passed its start-up
        # comparison with the dense all-to-all
        assert dp.tail_group == (mode == "zero" and wire == "bf16") and dp.sparse == sparse, dp.fallbacks
        assert not dp.fallbacks and ("tail-in-a2a" in dp.schedule) == dp.tail_group
        eng.set_batch(shard_batch(glob, BS, NEG, rank, world))
        dp.train_step()
        dp.gather_state()
        np.save(os.path.join(out_dir, f"p{rank}.npy"), eng.cpu.flat["p"][:eng.n_params])
        np.save(os.path.join(out_dir, f"m{rank}.npy"), eng.cpu.flat["m"][:eng.n_params])
        np.save(os.path.join(out_dir, f"ema{rank}.npy"), eng.cpu.ema)
        np.save(os.path.join(out_dir, f"loss{rank}.npy"), np.array([eng.loss]))
    finally:
        dist.destroy_process_group()


def _broken_sparse_worker(rank, port, world, q):
    """A sparse exchange that loses rows (rows_unpack drops each packet's last row) must fail the
    start-up comparison with the dense all-to-all: DataParallel turns sparse off and records it."""
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        cfg = O.OracleConfig(trigram_d=D, widths=WIDTHS, query_bs=BS, neg=NEG)
        eng = CpuEngine(O.init_params(cfg, seed=9), world)
        good = eng.rows_unpack
        eng.rows_unpack = lambda packed, n, count, row_base, nrows, dst: good(packed, n, max(0, count - 1),
                                                                              row_base, nrows, dst)
        dp = DataParallel(eng, comm="auto", mode="zero", wire="bf16", chunks=1, sparse=True)
        q.put((rank, dp.sparse, list(dp.fallbacks), float(eng.grads.abs().max()),
               float(dp.stage.float().abs().max())))
    finally:
        dist.destroy_process_group()


def test_sparse_exchange_self_check_demotes_a_broken_path():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_broken_sparse_worker, args=(r, port, 2, q)) for r in range(2)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(60)
    for rank, sparse, notes, gmax, smax in outs:
        assert sparse is False and any("sparse exchange differed" in n for n in notes), (rank, notes)
        assert gmax == 0.0 and smax == 0.0  # the check leaves the gradient tail and the stage cleared


def test_sparse_exchange_equals_dense():
    """The touched-row sparse exchange (DataParallel(sparse=True)) delivers exactly the dense
    all-to-all's stage: world 4, parameters and Adam slots bit-identical to the dense bf16 wire."""
    out = {}
    for sparse in (False, True):
        with tempfile.TemporaryDirectory() as d:
            mp.spawn(_worker, args=(_free_port(), d, "zero", "bf16", 4, 1, sparse), nprocs=4, join=True)
            out[sparse] = [np.load(os.path.join(d, f"{x}0.npy")) for x in ("p", "m")]
    for a, b in zip(out[False], out[True]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("mode,wire,chunks", [("allreduce", "fp32", 1), ("zero", "fp32", 1), ("zero", "bf16", 1),
                                              ("zero", "bf16", 3), ("zero", "bf16-sparse", 1)])
def test_data_parallel_gloo(mode, wire, chunks, world):
    """allreduce: all-reduce + replicated Adam; zero: Adam on the rank's shard + all-gather of the
    parameters, W1's rows on an fp32 (reduce-scatter) or a bf16 all-to-all wire. All must give
    the same step (the bf16 wire within Adam's insensitivity to gradient rounding: a first step
    moves each element by lr * sign(g) wherever |g| >> eps)."""
    WORLD = world
    sparse = wire == "bf16-sparse"
    wire = "bf16" if sparse else wire
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(_free_port(), d, mode, wire, world, chunks, sparse), nprocs=WORLD, join=True)
        p = [np.load(os.path.join(d, f"p{r}.npy")) for r in range(WORLD)]
        m_ = [np.load(os.path.join(d, f"m{r}.npy")) for r in range(WORLD)]
        ema = [np.load(os.path.join(d, f"ema{r}.npy")) for r in range(WORLD)]
        loss = [float(np.load(os.path.join(d, f"loss{r}.npy"))[0]) for r in range(WORLD)]
    for r in range(1, WORLD):
        np.testing.assert_array_equal(p[0], p[r])  # identical parameters on every rank
        np.testing.assert_array_equal(m_[0], m_[r])  # and identical (gathered) Adam state

    # oracle: mean of the per-shard gradients, then one Adam step
    cfg_l = O.OracleConfig(trigram_d=D, widths=WIDTHS, query_bs=BS // WORLD, neg=NEG)
    cfg_g = O.OracleConfig(trigram_d=D, widths=WIDTHS, query_bs=BS, neg=NEG)
    p0 = O.init_params(cfg_g, seed=9)
    glob = synth_batch(D, BS, NEG, seed=1234, mean_nnz=16)
    gsum = None
    for r in range(WORLD):
        cache, ema_r = O.forward(cfg_l, p0, O.make_ema(cfg_l), shard_batch(glob, BS, NEG, r, WORLD).as_dict(),
                                 True, np.float64)
        assert abs(loss[r] - cache["loss"]) <= 1e-5 * abs(cache["loss"])
        ref_ema = np.concatenate([np.concatenate([ema_r[f"bn{l}_{t}_mean"], ema_r[f"bn{l}_{t}_var"]])
                                  for l in range(1, len(WIDTHS) + 1) for t in ("q", "d")])
        np.testing.assert_allclose(ema[r], ref_ema, rtol=1e-5, atol=1e-6)
        g = O.backward(cfg_l, p0, cache, np.float64)
        gsum = g if gsum is None else {k: gsum[k] + g[k] for k in g}
    gmean = {k: v / WORLD for k, v in gsum.items()}
    pref = {k: v.copy() for k, v in p0.items()}
    O.AdamState(cfg_g, pref).step(pref, gmean)
    m = cpu_c.CpuDSSM(D, WIDTHS, BS // WORLD, NEG, p0)
    m.flat["p"][...] = p[0]
    got = m.named("p")
    for k, ref in pref.items():
        if re.fullmatch(r"b\d+", k):
            continue  # bias gradients are rounding noise under batch-stat BN (test_oracle.py)
        diff = np.abs(got[k] - ref)
        well = np.abs(gmean[k]) > 1e-3 * np.abs(gmean[k]).max()
        assert diff[well].max(initial=0.0) <= 1e-5, (k, diff[well].max(initial=0.0))
        assert diff.max() <= 2 * 0.01, k


@pytest.mark.parametrize("kw", [dict(chunks=3), dict(sparse=True), dict(wire="fp32"), dict(mode="allreduce"),
                                dict(exchange="rings")])
def test_peer_exchange_arguments_refused(kw):
    """DataParallel(exchange="peer") is the zero schedule on the bf16 wire in one chunk with a bf16
    HIP-engine model; anything else is refused before any buffer is allocated (the CPU engine,
    an fp32 model without dssm_plan_set_dp_peers, is refused too)."""
    from dssm_amd.dist import DataParallel
    eng = CpuEngine(O.init_params(O.OracleConfig(trigram_d=D, widths=WIDTHS, query_bs=BS, neg=NEG), seed=3), 1)
    args = dict(exchange="peer")
    args.update(kw)
    with pytest.raises(ValueError):
        DataParallel(eng, **args)


def test_peer_exchange_needs_a_hip_model():
    from dssm_amd.dist import DataParallel
    eng = CpuEngine(O.init_params(O.OracleConfig(trigram_d=D, widths=WIDTHS, query_bs=BS, neg=NEG), seed=3), 1)
    with pytest.raises(ValueError, match="bf16 HIP-engine"):
        DataParallel(eng, exchange="peer")
