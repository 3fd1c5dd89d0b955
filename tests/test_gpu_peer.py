"""The peer-store data-parallel exchange (include/dssm.h dssm_plan_set_dp_peers, csrc/peer.hip,
dssm_amd.dist.DataParallel(exchange="peer"); DESIGN.md §6 "peer exchange").

The exchange replaces the bf16-wire schedule's all-to-all, tail all-reduce and all-gather by stores
into the other ranks' fine-grained buffers and per-step flags, so its contract is: the same bits as
the collective schedule.  Every comparison runs under DETERMINISTIC (fixed-order reductions), and
the collective schedule is emulated exactly (rank r's block j of its gradient wire into block r of
rank j's stage, the tails summed a + b, the parameter wires' shard blocks copied to every rank):
* world 1 (one process, the buffers still IPC-exported): eager steps and two replays of a captured
  3-step region (dssm_plan_graph_build_dp_steps comm 3) bit-identical to the wire schedule's eager
  steps -- params, Adam m / v, the parameter wire, beta powers, loss;
* world 2 in ONE process (two models on two streams, the peers' buffers by plain address): each
  rank's whole step is enqueued before the other's, so the two streams run concurrently on the GPU
  and hand off through the flags -- eager steps and captured regions bit-identical to the emulated
  collectives; a run in which rank 1 never arrives times out within the bound and is reported
  (dssm_plan_peer_status), and no wait is left running;
* world 2 in TWO processes (gloo bootstrap, HIP IPC mappings of each other's buffers: the
  deployment shape): the ranks end bit-identical to each other and to the emulated collectives run
  in each process.
One GPU cannot show the cross-GPU path (xGMI); what these tests exercise is the protocol (epochs,
flags, offsets, reuse ordering) and, because the two ranks' kernels run on different CUs and XCDs
whose L2s are not coherent with each other, the release / acquire discipline across caches."""
import functools
import os
import socket
import tempfile

import numpy as np
import pytest
import torch

from dssm_amd.data import synth_batch
from tests.test_gpu_parity import make

pytestmark = pytest.mark.gpu

D, WIDTHS, BS, NEG, LR = 5000, (300, 300, 128), 96, 4, 0.01
TIMEOUT_MS = 5000.0


def _model():
    _, _, m = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    m.set_option("DETERMINISTIC", True)
    return m


def _batches(steps, seed0, rank=0):
    out = []
    for i in range(steps):
        b = synth_batch(D, BS, NEG, seed=seed0 + 97 * rank + i, mean_nnz=32)
        out.append(tuple(torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values)))
    return out


class Emulated:
    """The bf16-wire schedule of `world` ranks in one process, its collectives as device copies in the
    order the all-to-all / all-reduce / all-gather deliver (the reference the peer exchange must equal)."""

    def __init__(self, world):
        self.world = world
        self.models, self.wires = [], []
        for r in range(world):
            m = _model()
            m.set_fused_w1_adam(False)
            n = m.dp_wire_size(world, 1)
            w = [torch.zeros(n, dtype=torch.bfloat16, device="cuda") for _ in range(3)]  # grad, stage, param
            m.set_dp_wire(world, r, 1, *w)
            self.models.append(m)
            self.wires.append(w)
        geo = self.models[0].dp_geometry()
        self.sub, self.ext, self.np = geo["sub"], geo["extent"], geo["n_params"]

    def step(self, batches):
        W, sub = self.world, self.sub
        for m, (ip, ix, vv) in zip(self.models, batches):
            m.set_batch(indptr=ip, indices=ix, values=vv)
            m.forward(True)
            m.backward()
        for j in range(W):  # all-to-all: rank r's block j -> rank j's stage block r
            for r in range(W):
                self.wires[j][1][r * sub:(r + 1) * sub].copy_(self.wires[r][0][j * sub:(j + 1) * sub])
        tail = self.models[0].grads[self.ext:self.np].clone()
        for r in range(1, W):  # all-reduce of the tail, rank order
            tail += self.models[r].grads[self.ext:self.np]
        for m in self.models:
            m.grads[self.ext:self.np].copy_(tail)
            m.apply_adam(1.0 / W)
        for j in range(W):  # all-gather of the parameter wires' shard blocks
            for r in range(W):
                if r != j:
                    self.wires[j][2][r * sub:(r + 1) * sub].copy_(self.wires[r][2][r * sub:(r + 1) * sub])
        for m in self.models:
            m.wire_shadows()


def _peer_in_process(world):
    """world models with the peer exchange wired by plain addresses (no IPC: one process)."""
    from dssm_amd import _lib
    lib = _lib.load()
    models, bufs = [], []
    for r in range(world):
        m = _model()
        m.set_fused_w1_adam(False)
        models.append(m)
    n = models[0].dp_wire_size(world, 1)
    for r, m in enumerate(models):
        b = {}
        gw = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
        m.set_dp_wire(world, r, 1, gw, torch.zeros_like(gw), torch.zeros_like(gw))
        geo = m.dp_geometry()
        tail_n = geo["n_params"] - geo["extent"]
        for k, size in (("stage", 2 * n), ("pwire", 2 * n), ("tail", 4 * world * tail_n),
                        ("flags", _lib.PEER_FLAG_BYTES)):
            p = _lib.C.c_void_p()
            _lib.check(lib.dssm_peer_alloc(size, _lib.C.byref(p)), "peer_alloc")
            b[k] = int(p.value)
        from dssm_amd.dist import device_view
        b["gw"] = gw
        b["stage_t"] = device_view(b["stage"], n, torch.bfloat16, "cuda")
        b["pwire_t"] = device_view(b["pwire"], n, torch.bfloat16, "cuda")
        m.set_dp_wire(world, r, 1, gw, b["stage_t"], b["pwire_t"])
        bufs.append(b)
    for m in models:
        m.set_dp_peers(world, [b["stage"] for b in bufs], [b["pwire"] for b in bufs],
                       [b["tail"] for b in bufs], [b["flags"] for b in bufs])
        m.set_peer_timeout(TIMEOUT_MS)

    def free():
        torch.cuda.synchronize()
        for m in models:
            m.set_dp_peers(0, None, None, None, None)
        for b in bufs:
            b["stage_t"] = b["pwire_t"] = None
            for k in ("stage", "pwire", "tail", "flags"):
                lib.dssm_peer_free(_lib.C.c_void_p(b[k]))
    return models, bufs, free


def _peer_step(m, batch, world):
    ip, ix, vv = batch
    m.set_batch(indptr=ip, indices=ix, values=vv)
    m.forward(True)
    m.backward()
    m.peer_exchange(0)
    m.apply_adam(1.0 / world)
    m.peer_exchange(1)
    m.wire_shadows()


def _first_diff(name, a, b):
    if torch.equal(a, b):
        return None
    d = (a.float() - b.float()).abs()
    i = int(torch.argmax(d))
    return f"{name}: {int((d > 0).sum())} elements differ, first max at {i} ({float(d.max()):.3e})"


def _compare(m, e, pw_m, pw_e):
    msgs = [_first_diff(k, x, y) for k, x, y in
            (("params", m.params, e.params), ("adam_m", m.adam_m, e.adam_m), ("adam_v", m.adam_v, e.adam_v),
             ("param_wire", pw_m, pw_e))]
    msgs = [x for x in msgs if x]
    assert not msgs, "; ".join(msgs)
    assert m.beta_powers() == e.beta_powers()
    assert m.loss_accuracy() == e.loss_accuracy()


def test_peer_world1_eager_and_graph_equal_wire_schedule():
    from dssm_amd.dist import DataParallel
    steps, replays = 3, 2
    e = Emulated(1)
    m = _model()
    dp = DataParallel(m, exchange="peer", peer_timeout_ms=TIMEOUT_MS)
    try:
        assert dp.schedule == "zero/bf16 via peer stores" and dp.capturable
        assert dp.peer_selftest == 0
        batches = _batches(steps, 500)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for b in batches[:2]:  # eager
                m.set_batch(indptr=b[0], indices=b[1], values=b[2])
                dp.train_step()
                e.step([b])
            gid = dp.build_region(batches)
            for _ in range(replays):
                m.graph_launch(gid)
                for b in batches:
                    e.step([b])
        torch.cuda.synchronize()
        assert dp.peer_check() == 1 + 2 + steps * replays  # the start-up self-test is one exchange too
        _compare(m, e.models[0], dp.param_wire, e.wires[0][2])
        topo = m.graph_topology(gid)
        assert topo["chain"] == 1 and topo["memcpy"] == 0 and topo["memset"] == 0, topo
    finally:
        dp.close()


def test_peer_world2_in_process_equal_emulated_collectives():
    W, steps = 2, 3
    e = Emulated(W)
    models, bufs, free = _peer_in_process(W)
    try:
        streams = [torch.cuda.Stream() for _ in range(W)]
        per_rank = [_batches(steps, 700, r) for r in range(W)]
        for i in range(steps):  # eager: each rank's whole step enqueued before the next rank's
            for r in range(W):
                with torch.cuda.stream(streams[r]):
                    _peer_step(models[r], per_rank[r][i], W)
            e.step([per_rank[r][i] for r in range(W)])
        torch.cuda.synchronize()
        for r in range(W):
            assert models[r].peer_status() == {"error": 0, "steps": steps}
            _compare(models[r], e.models[r], bufs[r]["pwire_t"], e.wires[r][2])
        gids = []
        for r in range(W):  # captured regions, one per rank on its stream, replayed twice
            with torch.cuda.stream(streams[r]):
                gids.append(models[r].graph_build_dp_steps(per_rank[r], 1.0 / W, comm=3))
        for _ in range(2):
            for r in range(W):
                with torch.cuda.stream(streams[r]):
                    models[r].graph_launch(gids[r])
            for i in range(steps):
                e.step([per_rank[r][i] for r in range(W)])
        torch.cuda.synchronize()
        for r in range(W):
            assert models[r].peer_status() == {"error": 0, "steps": 3 * steps}
            _compare(models[r], e.models[r], bufs[r]["pwire_t"], e.wires[r][2])
        assert torch.equal(bufs[0]["pwire_t"], bufs[1]["pwire_t"])  # the all-gathered wires agree
    finally:
        free()


def test_peer_selftest_in_process_and_after_steps():
    """dssm_plan_peer_selftest at world 2 in one process (the two ranks' self-tests on two streams,
    each waiting for the other's flags), before and between steps: 0 mismatches, and the steps
    around it still equal the emulated collectives bit for bit."""
    import threading
    W, steps = 2, 2
    e = Emulated(W)
    models, bufs, free = _peer_in_process(W)
    try:
        streams = [torch.cuda.Stream() for _ in range(W)]
        per_rank = [_batches(steps, 1300, r) for r in range(W)]
        out = [None] * W

        def st(r):  # the self-test synchronizes its stream: the ranks run it from two host threads
            with torch.cuda.stream(streams[r]):
                out[r] = models[r].peer_selftest()
        for i in range(steps):
            th = [threading.Thread(target=st, args=(r,)) for r in range(W)]
            for t in th:
                t.start()
            for t in th:
                t.join(60)
            assert out == [0] * W, out
            for r in range(W):
                with torch.cuda.stream(streams[r]):
                    _peer_step(models[r], per_rank[r][i], W)
            e.step([per_rank[r][i] for r in range(W)])
        torch.cuda.synchronize()
        for r in range(W):
            assert models[r].peer_status()["error"] == 0
            _compare(models[r], e.models[r], bufs[r]["pwire_t"], e.wires[r][2])
    finally:
        free()


def test_peer_can_access_same_device():
    """dssm_peer_can_access: the same device is always mappable (ranks sharing one GPU)."""
    from dssm_amd import _lib
    lib = _lib.load()
    ok = _lib.C.c_int(0)
    _lib.check(lib.dssm_peer_can_access(torch.cuda.current_device(), _lib.C.byref(ok)), "peer_can_access")
    assert ok.value == 1


def test_peer_timeout_is_bounded_and_reported():
    """Rank 1 never runs: rank 0's first wait times out after the bound, records the flag it waited
    on (GRAD of rank 1 = 1 + 0 + 1), and every later wait returns at once."""
    import time
    W = 2
    models, bufs, free = _peer_in_process(W)
    try:
        models[0].set_peer_timeout(300.0)
        b = _batches(2, 900)
        s = torch.cuda.Stream()
        t0 = time.time()
        with torch.cuda.stream(s):
            for x in b:
                _peer_step(models[0], x, W)
        torch.cuda.synchronize()
        dt = time.time() - t0
        st = models[0].peer_status()
        assert st["error"] == 1 + 0 + 1 and st["steps"] == 2, st
        assert dt < 5.0, dt  # one 0.3 s timeout, not one per wait
    finally:
        free()


# ---- two processes: IPC mappings, gloo bootstrap ------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, steps, delay_rank=-1):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from dssm_amd.dist import DataParallel
        torch.cuda.set_device(0)
        s = torch.cuda.Stream()
        torch.cuda.set_stream(s)
        batches = [_batches(steps, 1100, r) for r in range(world)]  # every rank's shard (for the emulation)
        m = _model()
        dp = DataParallel(m, comm="torch", exchange="peer", peer_timeout_ms=TIMEOUT_MS)
        assert dp.peer_selftest == 0  # the synthetic exchange across the two processes
        e = Emulated(world)
        diag = []
        try:
            geo = m.dp_geometry()
            import time
            for i in range(steps):  # eager steps, then the last as a captured one-step region
                if rank == delay_rank:  # uneven arrival: the other rank's waits spin for ~50 ms
                    torch.cuda.synchronize()
                    time.sleep(0.05)
                if i < steps - 1:
                    ip, ix, vv = batches[rank][i]
                    m.set_batch(indptr=ip, indices=ix, values=vv)
                    dp.train_step()
                else:
                    m.graph_launch(dp.build_region([batches[rank][i]]))
                e.step([batches[r][i] for r in range(world)])
                torch.cuda.synchronize()
                p, q = m.params, e.models[rank].params
                regions = {"shard": (geo["shard_begin"], geo["shard_end"]), "tail": (geo["extent"], geo["n_params"])}
                diag.append({k: int((p[a:b] != q[a:b]).sum()) for k, (a, b) in regions.items()})
            nsteps = dp.peer_check()
            np.savez(os.path.join(out_dir, f"rank{rank}.npz"), params=m.params.cpu().numpy(),
                     pwire=dp.param_wire.float().cpu().numpy(), steps=nsteps,
                     ref_params=e.models[rank].params.cpu().numpy(),
                     ref_pwire=e.wires[rank][2].float().cpu().numpy(),
                     m=m.adam_m.cpu().numpy(), ref_m=e.models[rank].adam_m.cpu().numpy(),
                     diag=np.array(str(diag)))
        finally:
            dp.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("delay_rank", [-1, 0, 1])
def test_peer_world2_two_processes_ipc(delay_rank):
    """delay_rank: that rank sleeps 50 ms (idle GPU) before each of its steps, so the other rank's
    waits spin until its flags arrive late (uneven load on the hand-offs)."""
    import torch.multiprocessing as mp
    W, steps = 2, 3
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(functools.partial(_worker), args=(W, _free_port(), d, steps, delay_rank), nprocs=W,
                           start_method="spawn", join=True)
        z = [np.load(os.path.join(d, f"rank{r}.npz")) for r in range(W)]
    for r in range(W):
        assert int(z[r]["steps"]) == 1 + steps  # the start-up self-test's exchange, then the steps
        print(f"rank {r}: elements differing per step {z[r]['diag']}")
        np.testing.assert_array_equal(z[r]["params"][:len(z[r]["ref_params"])], z[r]["ref_params"])
        np.testing.assert_array_equal(z[r]["pwire"], z[r]["ref_pwire"])
        np.testing.assert_array_equal(z[r]["m"], z[r]["ref_m"])
    np.testing.assert_array_equal(z[0]["pwire"], z[1]["pwire"])
