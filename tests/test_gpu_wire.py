"""Data-parallel bf16 wire on one GPU (include/dssm.h dssm_plan_set_dp_wire, dssm_amd/dist.py).

The wire carries W1's rows in `chunks` pieces: rank j's optimizer shard is rows [j*P*S, (j+1)*P*S)
and sub-chunk (p, j) -- rows (j*P + p)*S + [0, S) -- sits at ((p*world + j)*S)*n, so chunk p of
every collective is one contiguous block.  Checked here:
* backward() writes bf16(dW1) of every row into the grad wire at its layout position (the gradient
  pass's rows against the materialised gradient of the unwired step, to bf16 rounding);
* Adam over this rank's shard takes the fp32 sum, in rank order, of the stage's bf16 partials
  (bit-identical to the unwired Adam fed that sum), writes bf16(W1) of the shard into the
  parameter wire at its layout position and leaves the other rows alone; the replicated fp32 tail
  updates as the unwired step does;
* wire_shadows() rebuilds W1's bf16 shadow: a forward after it equals one after the fp32 refresh;
* the data-parallel step graph (dssm_plan_graph_build_dp_steps: forward, backward, the chunked
  gradient pass, the collectives, chunked Adam, chunked shadow rebuild, all on one stream) at
  world 1, with the library's RCCL communicator (comm 0) and the device-copy rehearsal (comm 1),
  against the same steps run eagerly, bit for bit under DETERMINISTIC, and its captured graph a
  single chain of nodes; the modelled-link rehearsal (comm 2) runs.
At world 1 the all-to-all and all-gather are identities; the exchange between ranks is covered by
tests/test_gpu_dp_bow.py (world 2 over gloo) and tests/test_dist_gloo.py (CPU)."""
import ctypes as C

import numpy as np
import pytest
import torch

from dssm_amd.data import synth_batch
from tests.test_gpu_parity import make

pytestmark = pytest.mark.gpu

D, WIDTHS, BS, NEG, LR = 5000, (300, 300, 128), 96, 4, 0.01


def _wires(m, world, rank, chunks, same_stage=False):
    n = m.dp_wire_size(world, chunks)
    gw = torch.zeros(n, dtype=torch.bfloat16, device=m.device)
    st = gw if same_stage else torch.zeros(n, dtype=torch.bfloat16, device=m.device)
    pw = torch.zeros(n, dtype=torch.bfloat16, device=m.device)
    m.set_dp_wire(world, rank, chunks, gw, st, pw)
    return gw, st, pw, m.dp_geometry()


def _rows(geo, wire, D_=D):
    """The wire's W1 rows in arena order ([D x n] view) from its sub-chunk layout."""
    w, p, S, n = geo["world"], geo["chunks"], geo["rows"], geo["sub"] // geo["rows"]
    out = torch.empty(D_, n, dtype=wire.dtype, device=wire.device)
    for j in range(w):
        for c in range(p):
            r0 = (j * p + c) * S
            if r0 >= D_:
                continue
            r1 = min(r0 + S, D_)
            o = (c * w + j) * S * n
            out[r0:r1] = wire[o:o + (r1 - r0) * n].view(r1 - r0, n)
    return out


def _close(a, b):
    d = (a - b).abs()
    assert float(d.max()) <= 2 * LR, float(d.max())
    assert float((d <= 1e-5).float().mean()) >= 0.999, float((d <= 1e-5).float().mean())


@pytest.mark.parametrize("chunks", [1, 3])
@pytest.mark.parametrize("grad_pass", ["1", "0"])
def test_wire_step_world1_matches_unwired(chunks, grad_pass):
    """World 1 (stage = grad wire: the all-to-all is the identity).  grad_pass 1 (default): dW1
    straight into the wire by k_adam_step's W1 roles, chunk by chunk; 0: materialised dW1 +
    k_wire_pack."""
    _, _, ref = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    _, _, m = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    m.set_option("WIRE_GRAD_PASS", grad_pass == "1")
    gw, st, pw, geo = _wires(m, 1, 0, chunks, same_stage=True)
    ext, n1 = m.wire_extent(), WIDTHS[0]
    assert ext == D * n1 and (geo["shard_begin"], geo["shard_end"]) == (0, ext)
    hb = synth_batch(D, BS, NEG, seed=77, mean_nnz=32)
    for x in (ref, m):
        x.set_batch(hb)
        x.forward(True)
        x.backward()
    torch.cuda.synchronize()
    g_rows = _rows(geo, gw).float().reshape(-1)
    g_ref = ref.grads[:ext]
    if grad_pass == "0":  # exactly RNE bf16 of this model's materialised gradient
        assert torch.equal(g_rows, m.grads[:ext].to(torch.bfloat16).float())
    else:  # the pass leaves the arena's W1 rows alone; b1's row is fp32 in the arena
        assert float(m.grads[:ext].abs().max()) == 0.0
        torch.testing.assert_close(g_rows, g_ref, rtol=2 ** -7, atol=1e-6 * float(g_ref.abs().max()))
        b_m, b_r = m.grads[ext:ext + n1], ref.grads[ext:ext + n1]
        assert float((b_m - b_r).abs().max()) <= 1e-4 * float(b_r.abs().max()) + 1e-7
    ref.apply_adam(1.0)
    m.apply_adam(1.0)
    torch.cuda.synchronize()
    n = m.n_params
    _close(m.params[:ext], ref.params[:ext])
    _close(m.params[ext:n], ref.params[ext:n])
    torch.testing.assert_close(m.adam_m[ext:n], ref.adam_m[ext:n], rtol=1e-3, atol=1e-6)
    assert torch.equal(_rows(geo, pw).reshape(-1), m.params[:ext].to(torch.bfloat16))
    assert m.beta_powers() == ref.beta_powers()


def test_wire_shadows_equal_fp32_refresh():
    _, _, m = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    _wires(m, 1, 0, 2, same_stage=True)
    hb = synth_batch(D, BS, NEG, seed=78, mean_nnz=32)
    m.set_batch(hb)
    m.forward(True)
    m.backward()
    m.apply_adam(1.0)
    m.wire_shadows()
    m.forward(False)
    torch.cuda.synchronize()
    a = m.fetch("cos_sim_raw").copy()
    m.sync_shadows()
    m.forward(False)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(m.fetch("cos_sim_raw"), a)


@pytest.mark.parametrize("world,chunks", [(2, 1), (4, 2), (8, 3)])
def test_stage_sums_rank_partials_in_fp32(world, chunks):
    """Rank 1 of `world`: Adam takes each of its shard's W1 rows as the fp32 sum, in rank order, of
    the world's bf16 partials in the stage (what the chunked all-to-all delivers).  Against the
    unwired Adam over the same rows fed that fp32 sum, the shard's parameters and Adam slots are
    bit-identical, the parameter wire holds bf16 of them at their layout positions, and every other
    W1 row is untouched."""
    _, _, ref = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    _, _, m = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    rank = 1
    gw, st, pw, geo = _wires(m, world, rank, chunks)
    S, n = geo["rows"], WIDTHS[0]
    b0, b1 = geo["shard_begin"], geo["shard_end"]
    gen = torch.Generator(device=m.device).manual_seed(5)
    st.copy_((torch.randn(st.numel(), generator=gen, device=m.device) * 1e-3).to(torch.bfloat16))
    acc = torch.zeros(b1 - b0, dtype=torch.float32, device=m.device)
    for row in range(b0 // n, b1 // n):
        c, s = (row // S) % chunks, row % S
        for k in range(world):
            o = ((c * world + k) * S + s) * n
            acc[(row * n - b0):(row * n - b0) + n] += st[o:o + n].float()
    ref.set_adam_range(b0, b1)
    ref.grads.zero_()
    ref.grads[b0:b1] = acc
    m.grads.zero_()
    p0, m0 = m.params.clone(), m.adam_m.clone()
    ref.apply_adam(1.0 / world)
    m.apply_adam(1.0 / world)
    torch.cuda.synchronize()
    for x, y in ((m.params, ref.params), (m.adam_m, ref.adam_m), (m.adam_v, ref.adam_v)):
        assert torch.equal(x[b0:b1], y[b0:b1])
    pr = _rows(geo, pw).reshape(-1)
    assert torch.equal(pr[b0:b1], m.params[b0:b1].to(torch.bfloat16))
    ext = m.wire_extent()
    assert torch.equal(m.params[:b0], p0[:b0]) and torch.equal(m.params[b1:ext], p0[b1:ext])
    assert torch.equal(m.adam_m[:b0], m0[:b0]) and torch.equal(m.adam_m[b1:ext], m0[b1:ext])


@pytest.fixture()
def comm_world1():
    """libdssm.so's RCCL communicator at world 1, bootstrapped directly (no torch.distributed)."""
    from dssm_amd import _lib
    lib = _lib.load()
    made = False
    if lib.dssm_comm_world() == 0:
        buf = (C.c_char * 128)()
        _lib.check(lib.dssm_comm_unique_id(buf), "comm_unique_id")
        _lib.check(lib.dssm_comm_init(0, 1, buf), "comm_init")
        made = True
    assert lib.dssm_comm_world() == 1
    yield
    if made:
        lib.dssm_comm_destroy()


def _staged(seeds):
    out = []
    for sd in seeds:
        b = synth_batch(D, BS, NEG, seed=sd, mean_nnz=32)
        out.append(tuple(torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values)))
    return out


def _first_mismatch(name, got, want, geo, ext):
    """Where two arenas differ: the W1 wire chunk / the tail, for the assertion message."""
    d = (got != want).nonzero().flatten()
    if d.numel() == 0:
        return ""
    i = int(d[0])
    n = geo["sub"] // geo["rows"]
    where = f"W1 row {i // n} (chunk {(i // n // geo['rows']) % geo['chunks']})" if i < ext else f"tail +{i - ext}"
    return f"{name}: {d.numel()} of {got.numel()} differ, first at {i} = {where}"


@pytest.mark.parametrize("comm,chunks,bs,memcpy,tail", [(0, 3, 96, 0, 0), (1, 3, 96, 0, 0), (0, 1, 96, 0, 0),
                                                        (0, 1, 128, 0, 0), (0, 3, 96, 1, 0), (0, 3, 96, 0, 1),
                                                        (0, 1, 128, 0, 1)])
def test_dp_step_graph_world1_matches_eager(comm, chunks, bs, memcpy, tail, comm_world1):
    """The captured data-parallel step graph (comm 0: RCCL at world 1; comm 1: device copies)
    against the same steps run eagerly on the same wire (all-to-all = copy, all-gather = identity),
    under DETERMINISTIC (every reduction in a fixed order): params, Adam m / v, beta powers and the
    wire must be BIT-identical after two replays of a 3-step graph (6 steps).  With one chunk,
    steps 2 and 3 of the graph read W1 straight from the parameter wire (tight rows of stride 300;
    bs 128 runs the merged-transpose SpMM launch, bs 96 the plain one), and Z1's pad columns must
    stay zero.  The captured graph must be one chain of nodes (dssm_plan_graph_topology), with no
    memcpy / memset nodes -- except in the MEMCPY_NODES diagnostics variant (the round-3 form of
    the own-chunk copy), which must be ordered the same way."""
    from dssm_amd import _lib
    steps, replays = 3, 2
    runs = []
    for mode in ("graph", "eager"):
        _, _, m = make(D, WIDTHS, bs, NEG, "bf16", fused=False)
        m.set_option("DETERMINISTIC", True)
        m.set_option("MEMCPY_NODES", bool(memcpy))
        m.set_option("TAIL_IN_A2A", bool(tail))  # the tail's all-reduce inside the last all-to-all's group
        gw, st, pw, geo = _wires(m, 1, 0, chunks)
        runs.append((m, gw, st, pw))
    batches = []
    for i in range(steps):
        b = synth_batch(D, bs, NEG, seed=300 + i, mean_nnz=32)
        batches.append(tuple(torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values)))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        m, gw, st, pw = runs[0]
        gid = m.graph_build_dp_steps(batches, 1.0, comm=comm)
        for _ in range(replays):
            m.graph_launch(gid)
        e, egw, est, epw = runs[1]
        for _ in range(replays):
            for ip, ix, vv in batches:
                e.set_batch(indptr=ip, indices=ix, values=vv)
                e.forward(True)
                e.backward()
                est.copy_(egw)  # the all-to-all at world 1
                e.apply_adam(1.0)
                e.wire_shadows()
    torch.cuda.synchronize()
    topo = m.graph_topology(gid)
    assert topo["chain"] == 1 and topo["roots"] == 1 and topo["nodes"] == topo["edges"] + 1, topo
    assert topo["memset"] == 0, topo
    assert (topo["memcpy"] > 0) if memcpy else (topo["memcpy"] == 0), topo
    ext = m.wire_extent()
    msgs = [_first_mismatch(k, x, y, geo, ext) for k, x, y in
            (("params", m.params, e.params), ("adam_m", m.adam_m, e.adam_m), ("adam_v", m.adam_v, e.adam_v),
             ("param_wire", pw, epw))]
    assert not any(msgs), "; ".join(x for x in msgs if x)
    assert m.beta_powers() == e.beta_powers()
    assert m.loss_accuracy() == e.loss_accuracy()
    if chunks == 1:  # the last step's SpMM read the tight wire rows: Z1's pad columns stay zero
        z1 = m.buffer(_lib.BUF_Z, 0).view(m.rows, -1)
        assert z1.shape[1] == 304 and float(z1[:, 300:].abs().max()) == 0.0
    # the replayed graph left the shadows rebuilt from its last all-gather: same forward as a refresh
    ip, ix, vv = batches[0]
    m.set_batch(indptr=ip, indices=ix, values=vv)
    m.forward(False)
    torch.cuda.synchronize()
    a = m.fetch("cos_sim_raw").copy()
    m.sync_shadows()
    m.forward(False)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(m.fetch("cos_sim_raw"), a)


def _warm_adam(m, v=1e-4):
    """A mid-training Adam state (v for every element, m = 0, beta powers at step 100)."""
    m.adam_v.fill_(v)
    m.adam_m.zero_()
    m.set_beta_powers(0.9 ** 100, 0.999 ** 100)


def _update_frac(p, q, p0, rel):
    """Fraction of elements whose update p - p0 agrees with q - p0 within rel x |q - p0| + rel x
    max |q - p0| (the floor covers the elements a step barely moves)."""
    u, w = p - p0, q - p0
    return float(((u - w).abs() <= rel * w.abs() + rel * float(w.abs().max())).float().mean())


@pytest.mark.parametrize("comm,chunks,bs,replays,warm", [(0, 3, 96, 1, False), (0, 3, 96, 2, True),
                                                         (1, 3, 96, 2, True), (0, 1, 128, 2, True)])
def test_dp_step_graph_default_schedule_matches_eager(comm, chunks, bs, replays, warm, comm_world1):
    """The DEFAULT schedule (no DETERMINISTIC: float atomics, the schedule the 8-GPU run times) of the
    captured data-parallel step graph against the same steps run eagerly, with a second eager run from
    the same state beside it and a negative control.

    Why the state matters (tools/dp_divergence.py, profiles/r06_dp_divergence.txt): the first tensor
    that differs between two eager runs is b1's gradient (47 of its 300 elements, step 0): under
    batch-stat BN d loss / d b1 is exactly zero, so it holds only rounding noise whose value depends on
    the ones column's float-atomic order.  From a FRESH Adam state ApplyAdam turns any gradient into a
    ~lr step (m / sqrt(v) = sign(g)), so the noise becomes b1 differences, Z1 differences of ~1e-7, and
    at some step one A1 element's bf16 rounding flips: one Z2 row moves by 1e-4, one layer-2 ReLU mask
    element flips, and from there every tensor diverges (after 6 steps ~10% of the parameters > 1e-4
    apart).  Whether that happens is a coin toss per run (1 of 4 eager runs, and the graph in another
    measurement), so no bar on a fresh 6-step comparison tells a race from it (round 5's 85%).  From
    a mid-training state (v = 1e-4 everywhere, step 100) an update is ~3e-5 g: rounding noise stays
    at rounding level, and every eager run and the graph applied the same update to every element
    within 1e-4 relative (measured 100%, BS 96 / 3 chunks and BS 128 / 1 chunk).  Those cases compare
    the UPDATES (p - p0) at 1e-3 relative (>= 99.9% of the elements) for graph-vs-eager and for
    eager-vs-eager; a race (a stale or half-written stage chunk) changes a whole chunk's updates by
    O(1): the negative control -- an eager run whose step 2 kept chunk 0's stage from step 1 -- must
    FAIL the same bar.  The fresh one-replay (3-step) case keeps the round-3 bar on the parameters
    (>= 99.9% within 1e-5; measured 100%)."""
    steps = 3
    runs = []
    for mode in ("graph", "eager", "eager2", "stale"):
        _, _, m = make(D, WIDTHS, bs, NEG, "bf16", fused=False)
        if warm:
            _warm_adam(m)
        gw, st, pw, geo = _wires(m, 1, 0, chunks)
        runs.append((m, gw, st, pw))
    p0 = runs[0][0].params.clone()
    blk = geo["world"] * geo["sub"]  # one chunk of the wire
    batches = []
    for i in range(steps):
        b = synth_batch(D, bs, NEG, seed=300 + i, mean_nnz=32)
        batches.append(tuple(torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values)))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        m, gw, st, pw = runs[0]
        gid = m.graph_build_dp_steps(batches, 1.0, comm=comm)
        for _ in range(replays):
            m.graph_launch(gid)
        for k, (e, egw, est, epw) in enumerate(runs[1:]):
            for rep in range(replays):
                for i, (ip, ix, vv) in enumerate(batches):
                    e.set_batch(indptr=ip, indices=ix, values=vv)
                    e.forward(True)
                    e.backward()
                    if k == 2 and rep == 0 and i == 2:  # negative control: chunk 0's stage left stale
                        est[blk:].copy_(egw[blk:])
                    else:
                        est.copy_(egw)  # the all-to-all at world 1
                    e.apply_adam(1.0)
                    e.wire_shadows()
    torch.cuda.synchronize()
    e, e2, stale = runs[1][0], runs[2][0], runs[3][0]
    assert m.beta_powers() == e.beta_powers() == e2.beta_powers()
    n = m.n_params
    if warm:
        f = lambda x, y: _update_frac(x.params[:n], y.params[:n], p0[:n], 1e-3)  # noqa: E731
        what, bar = "updates within 1e-3 relative", 0.999
    else:
        f = lambda x, y: float(((x.params[:n] - y.params[:n]).abs() <= 1e-5).float().mean())  # noqa: E731
        what, bar = "parameters within 1e-5", 0.999
    ge, ee, se = f(m, e), f(e2, e), f(stale, e)
    spread = f"{what}: graph-vs-eager {ge:.6f}, eager-vs-eager {ee:.6f}, stale-chunk control {se:.6f}"
    print(spread)
    assert ge >= bar, spread
    assert ee >= bar, spread  # the premise: this state does not amplify the schedule's noise
    assert se < bar, spread   # the bar does catch a stale chunk
    lg, le = m.loss_accuracy()[0], e.loss_accuracy()[0]
    assert abs(lg - le) <= 1e-4 * abs(le), (lg, le)


def test_single_gpu_graphs_are_chains():
    """The single-GPU multi-step graph bench.py times is one chain of kernel nodes (no memcpy /
    memset node: every device clear is a kernel)."""
    _, _, m = make(D, WIDTHS, 128, NEG, "bf16")
    batches = []
    for i in range(2):
        b = synth_batch(D, 128, NEG, seed=310 + i, mean_nnz=32)
        batches.append(tuple(torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values)))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gid = m.graph_build_steps(batches, probes=False)
        m.set_batch(indptr=batches[0][0], indices=batches[0][1], values=batches[0][2])
        gid1 = m.graph_build()
    torch.cuda.synchronize()
    for g in (gid, gid1):
        topo = m.graph_topology(g)
        assert topo["chain"] == 1 and topo["kernel"] == topo["nodes"], topo


def test_dp_step_graph_modelled_links_runs():
    """The modelled-link rehearsal (comm 2, world 8 on one GPU: the collectives are spin kernels on
    the comm stream) captures and replays; each replay advances the beta powers once per step."""
    _, _, m = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    _wires(m, 8, 0, 4)
    b1, b2 = m.beta_powers()
    batches = _staged([400, 401])
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with pytest.raises(RuntimeError):  # the two-stream variant was removed
            m.graph_build_dp_steps(batches, 1.0 / 8, comm=2, link_gbps=350.0, latency_us=10.0, overlap=True)
        gid = m.graph_build_dp_steps(batches, 1.0 / 8, comm=2, link_gbps=350.0, latency_us=10.0)
        m.graph_launch(gid)
    torch.cuda.synchronize()
    nb1, nb2 = m.beta_powers()
    assert nb1 == pytest.approx(b1 * 0.9 * 0.9, rel=1e-6) and nb2 == pytest.approx(b2 * 0.999 * 0.999, rel=1e-6)
