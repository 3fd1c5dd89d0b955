"""libdssm.so's own RCCL communicator (include/dssm.h dssm_comm_* / dssm_allreduce_sum /
dssm_reduce_scatter_sum / dssm_all_gather / dssm_all_to_all; csrc/plan.hip) executed on the GPU.

RCCL refuses two ranks on one device, so on the one-GPU box the communicator runs at world size 1
(ncclCommInitRank with one rank): every collective then executes its real RCCL code path and its
result is exactly known.  Covered: the bootstrap (dssm_amd.dist.LibTransport: rank 0's unique id
broadcast through torch.distributed as a (status, id) pair), every collective in fp32 and bf16
through LibTransport, the schedule self-tests of DataParallel (SCHEDULE_OPS), and the collectives
captured into a hipGraph and replayed (the data-parallel step graph captures them).  The N>1
exchange itself is covered by tests/test_gpu_dp_bow.py (two ranks over gloo on this GPU) and
tests/test_dist_gloo.py (CPU); the reference has no data parallelism."""
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tx():
    from dssm_amd.dist import LibTransport
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    torch.cuda.set_device(0)
    t = LibTransport(0, 1)
    assert t.lib.dssm_comm_world() == 1
    yield t
    t.destroy()
    assert t.lib.dssm_comm_world() == 0
    dist.destroy_process_group()


DTYPES = [torch.float32, torch.bfloat16]


def _pattern(n, dt, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randint(-512, 512, (n,), generator=g).float() / 8).to(dt).cuda()


@pytest.mark.parametrize("dt", DTYPES, ids=["fp32", "bf16"])
def test_collectives_world1_exact(tx, dt):
    n = 4096 + 64
    x = _pattern(n, dt, 1)
    ref = x.clone()
    tx.all_reduce(x)  # one rank: the sum is the buffer itself
    torch.cuda.synchronize()
    assert torch.equal(x, ref)
    y = _pattern(n, dt, 2)
    ref = y.clone()
    tx.reduce_scatter_(y, n)  # in place: recv = send + rank * count
    tx.all_gather_(y, n)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    s, d = _pattern(n, dt, 3), torch.zeros(n, dtype=dt, device="cuda")
    tx.all_to_all(s, d)
    torch.cuda.synchronize()
    assert torch.equal(d, s)
    # distinct send / recv buffers are required by the all-to-all
    from dssm_amd._lib import DssmError
    with pytest.raises(DssmError):
        tx.all_to_all(s, s)


@pytest.mark.parametrize("sched", [("allreduce", "fp32"), ("zero", "fp32"), ("zero", "bf16")],
                         ids=lambda s: "/".join(s))
def test_schedule_selftests_world1(tx, sched):
    from dssm_amd.dist import SCHEDULE_OPS, selftest
    assert selftest(tx, SCHEDULE_OPS[sched], torch.device("cuda", 0), 0, 1)


def test_mixed_group_selftest_world1(tx):
    """The TAIL_IN_A2A group (dssm_all_to_all_tail: grouped sends / receives + the fp32 tail's
    all-reduce) through DataParallel's start-up self-test, eager and captured in a graph (the form the
    step graph replays), and a wrong answer detected."""
    from dssm_amd.dist import selftest
    dev = torch.device("cuda", 0)
    assert selftest(tx, [("all_to_all_tail", torch.bfloat16), ("all_to_all_tail_captured", torch.bfloat16)],
                    dev, 0, 1)

    class Broken:  # the tail summed twice: the self-test must say no
        def all_to_all_tail(self, s, d, t):
            tx.all_to_all_tail(s, d, t)
            t.mul_(2)
    assert not selftest(Broken(), [("all_to_all_tail", torch.bfloat16)], dev, 0, 1)


def test_collectives_captured_in_graph(tx):
    """The four collectives captured into one hipGraph on a side stream and replayed twice: each
    replay re-runs them on the buffers' current contents."""
    n = 2048
    a = torch.zeros(n, device="cuda")
    b = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
    c = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
    out = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
        tx.all_reduce(a)
        tx.reduce_scatter_(b, n)
        tx.all_gather_(b, n)
        tx.all_to_all(c, out)
    for seed in (5, 6):
        a.copy_(_pattern(n, torch.float32, seed))
        b.copy_(_pattern(n, torch.bfloat16, seed + 10))
        c.copy_(_pattern(n, torch.bfloat16, seed + 20))
        ra, rb, rc = a.clone(), b.clone(), c.clone()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(a, ra) and torch.equal(b, rb) and torch.equal(out, rc)


def test_sparse_exchange_pieces_world1(tx):
    """The touched-row sparse exchange's library pieces at world 1: dssm_rows_pack_u16 /
    dssm_rows_unpack_u16 against torch indexing (bit-exact bf16 rows, the int32 id in front), and
    dssm_all_to_allv (the own part's device copy, int32 counts, the tail's all-reduce in the same
    RCCL group), eager and captured in a hipGraph."""
    from dssm_amd import _lib
    from dssm_amd.model import DSSM
    m = DSSM(500, (300, 64), 8, 4, dtype="bf16")
    n, rows_all = 300, 400
    g = torch.Generator(device="cuda").manual_seed(5)
    src = torch.randn(rows_all * n, device="cuda", generator=g).to(torch.bfloat16)
    ids = torch.unique(torch.randint(0, rows_all, (150,), device="cuda", generator=g)).to(torch.int32)
    k = ids.numel()
    packed = torch.zeros(k * (n + 4), dtype=torch.bfloat16, device="cuda")
    m.rows_pack(src, n, ids, packed)
    pk = packed.view(k, n + 4)
    assert torch.equal(pk.view(torch.int32)[:, 0], ids)
    assert torch.equal(pk[:, 4:], src.view(-1, n)[ids.long()])
    # unpack the ids in [100, 300) into a 200-row block (others skipped)
    dst = torch.zeros(200 * n, dtype=torch.bfloat16, device="cuda")
    m.rows_unpack(packed, n, k, 100, 200, dst)
    want = torch.zeros(200, n, dtype=torch.bfloat16, device="cuda")
    sel = ids[(ids >= 100) & (ids < 300)].long()
    want[sel - 100] = src.view(-1, n)[sel]
    assert torch.equal(dst.view(200, n), want)
    # all_to_allv at world 1: the own part copied, the tail summed over one rank (unchanged)
    recv = torch.zeros_like(packed)
    tail = torch.randn(1000, device="cuda", generator=g)
    tail0 = tail.clone()
    cnt = torch.tensor([7], dtype=torch.int32, device="cuda")
    cnt_r = torch.zeros_like(cnt)
    tx.all_to_all(cnt, cnt_r)
    assert int(cnt_r.item()) == 7
    tx.all_to_allv(packed, [packed.numel()], recv, [packed.numel()], tail=tail)
    torch.cuda.synchronize()
    assert torch.equal(recv, packed) and torch.equal(tail, tail0)
    s = torch.cuda.Stream()
    recv.zero_()
    s.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        tx.all_to_allv(packed, [packed.numel()], recv, [packed.numel()], tail=tail)
    gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(recv, packed) and torch.equal(tail, tail0)
    bad = (_lib.load().dssm_rows_pack_u16(0, 6, 0, 1, 0, 0))
    assert bad != 0  # n not a multiple of 4: refused


def test_strict_rccl_without_nccl_backend_raises():
    """comm="rccl" is strict: under a backend other than nccl (here: the module's gloo group, if
    still initialised, else a fresh one) the library transport is not a candidate and the
    selection raises instead of falling back silently."""
    from dssm_amd.dist import SCHEDULE_OPS, select_transport
    made = False
    if not dist.is_initialized():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        made = True
    try:
        with pytest.raises(RuntimeError):
            select_transport(0, 1, torch.device("cuda", 0), "rccl", SCHEDULE_OPS[("allreduce", "fp32")])
    finally:
        if made:
            dist.destroy_process_group()


def _rccl_world2_worker(rank, port, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=2, device_id=torch.device("cuda", rank))
    try:
        from dssm_amd.dist import DataParallel
        from dssm_amd.model import DSSM
        m = DSSM(5000, (300, 300, 128), 128, 4, dtype="bf16", seed=0, device=torch.device("cuda", rank))
        dp = DataParallel(m, comm="rccl", sparse=True)
        q.put((rank, dp.schedule, dp.sparse, dp.tail_group, list(dp.fallbacks)))
        dp.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (RCCL refuses two ranks on one device)")
def test_sparse_exchange_and_mixed_group_rccl_world2():
    """the library transport's variable-count all-to-all across real peers.  At world 2 on
    two GPUs DataParallel's start-up checks run on RCCL: the mixed all-to-all + all-reduce group's
    self-test (eager and captured) and the sparse exchange against the dense all-to-all, bit for bit;
    both must pass on both ranks.  Skipped on one-GPU boxes."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ps = [ctx.Process(target=_rccl_world2_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(60)
    for rank, sched, sparse, tail, notes in outs:
        assert sparse and tail and not notes, (rank, sched, notes)
        assert sched == "zero/bf16 sparse tail-in-a2a via rccl"
