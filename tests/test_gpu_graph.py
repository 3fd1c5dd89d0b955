"""hipGraph replay of the training step (what bench.py times) against eager launches.

The captured graph holds the same kernels with the same arguments as the eager step, and the
Adam beta powers live on the device, so a replay must compute what the eager step computes.
The step has one source of run-to-run nondeterminism (the order of float atomics: dW1's heavy
rows and the CSC fill's per-column entry order), which free-running Adam amplifies chaotically,
so the replay is checked teacher-forced: before every step the graph model is given the eager
model's full state (parameters, Adam slots, EMA, beta powers), then both run step i on batch i.
Bar per step: bit-identical loss (the forward is deterministic), parameters <= 2 lr everywhere
and within 1e-5 on >= 99.9% of elements, EMA within 1e-5 (1e-3 relative), identical beta
powers after the step; after all steps, identical step counts.  Then a free-running stretch of
graph replays must keep training (loss finite and falling).
"""
import numpy as np
import pytest
import torch

from dssm_amd import _lib
from dssm_amd.data import synth_batch
from tests.test_gpu_parity import make

pytestmark = pytest.mark.gpu

CASES = [
    # (D, widths, BS, NEG, dtype, fused)
    (1000, (100, 100), 128, 4, "fp32", True),
    (5000, (300, 300, 128), 96, 4, "bf16", True),
    (5000, (300, 300, 128), 96, 4, "bf16", False),
]


def _batches(D, BS, NEG, k):
    return [synth_batch(D, BS, NEG, seed=2000 + i, mean_nnz=32) for i in range(k)]


def _copy_state(dst, src):
    for name in ("params", "grads", "adam_m", "adam_v", "ema"):
        getattr(dst, name).copy_(getattr(src, name))
    dst.set_beta_powers(*src.beta_powers())
    _lib.check(dst.lib.dssm_plan_sync_shadows(dst._plan, _lib.stream_ptr()), "sync_shadows")


@pytest.mark.parametrize("case", CASES)
def test_graph_replay_matches_eager(case):
    D, widths, BS, NEG, dtype, fused = case
    lr, steps = 0.01, 6
    _, _, ea = make(D, widths, BS, NEG, dtype, fused=fused)
    _, _, gr = make(D, widths, BS, NEG, dtype, fused=fused)
    batches = _batches(D, BS, NEG, 3)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        staged = []
        for hb in batches:
            staged.append(tuple(torch.from_numpy(x).cuda() for x in (hb.indptr, hb.indices, hb.values)))
        gids = []
        for ip, ix, vv in staged:
            gr.set_batch(indptr=ip, indices=ix, values=vv)
            gids.append(gr.graph_build() if fused else gr.graph_build(_lib.GRAPH_FWD_BWD))
        adam = None if fused else gr.graph_build(_lib.GRAPH_ADAM)
        # capture must not have run anything or advanced the step state
        assert gr.global_step == 0
        assert gr.beta_powers() == (np.float32(0.9), np.float32(0.999))
        for i in range(steps):
            _copy_state(gr, ea)
            ip, ix, vv = staged[i % 3]
            ea.set_batch(indptr=ip, indices=ix, values=vv)
            ea.train_step()
            gr.graph_launch(gids[i % 3])
            if adam is not None:
                gr.graph_launch(adam)
            torch.cuda.synchronize()
            la, lg = ea.loss_accuracy()[0], gr.loss_accuracy()[0]
            assert la == lg, (i, la, lg)
            d = (ea.params - gr.params).abs()
            assert float(d.max()) <= 2 * lr, (i, float(d.max()))
            assert float((d <= 1e-5).float().mean()) >= 0.999, (i, float((d <= 1e-5).float().mean()))
            torch.testing.assert_close(gr.ema, ea.ema, rtol=1e-3, atol=1e-5)
            assert ea.beta_powers() == gr.beta_powers()
        assert ea.global_step == gr.global_step == steps
        # free-running replays keep training
        losses = []
        for i in range(9):
            gr.graph_launch(gids[i % 3])
            if adam is not None:
                gr.graph_launch(adam)
            torch.cuda.synchronize()
            losses.append(gr.loss_accuracy()[0])
        assert np.all(np.isfinite(losses)) and losses[-1] < losses[0], losses


def test_graph_probes_and_eager_interleave():
    """Probe events inside a graph time the last replay; eager steps between replays see the
    device Adam state the replays advanced."""
    D, widths, BS, NEG = 2000, (64, 64, 32), 64, 4
    _, _, m = make(D, widths, BS, NEG, "bf16")
    hb = synth_batch(D, BS, NEG, seed=7, mean_nnz=24)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        m.set_batch(hb)
        g = m.graph_build(probes=True)
        m.graph_launch(g)
        m.train_step()
        m.graph_launch(g)
        torch.cuda.synchronize()
        b1, b2 = m.beta_powers()
        assert b1 == np.float32(np.float32(np.float32(np.float32(0.9) * np.float32(0.9)) * np.float32(0.9)) * np.float32(0.9))
        assert m.global_step == 3
        for pid in (_lib.PROBE_SPMM_FWD, _lib.PROBE_ADAM, _lib.PROBE_DW1, _lib.PROBE_CSC):
            ms = m.graph_probe_read(g, pid)
            # DW1 brackets no kernel when the heavy dW1 columns run inside the Adam launch
            lo = 0.0 if pid == _lib.PROBE_DW1 else 1e-6
            assert lo <= ms < 50.0, (pid, ms)
        assert np.isfinite(m.loss_accuracy()[0])


def test_graph_rejects_partial_fused_and_default_stream():
    D, widths, BS, NEG = 500, (32, 32), 16, 2
    _, _, m = make(D, widths, BS, NEG, "fp32")
    m.set_batch(synth_batch(D, BS, NEG, seed=3, mean_nnz=16))
    with pytest.raises(ValueError):
        m.graph_build(stream=torch.cuda.default_stream())
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with pytest.raises(_lib.DssmError):
            m.graph_build(_lib.GRAPH_FWD_BWD)  # fused W1 Adam: the step cannot be split


@pytest.mark.parametrize("case", CASES[:2])
@pytest.mark.parametrize("det", [False, True])
def test_multi_step_graph_matches_eager(case, det):
    """graph_build_steps: k whole steps captured back to back in one graph (bench's cycle graph)
    equal k eager steps on the same batches.  DETERMINISTIC: bit-identical.  Default schedule:
    free-running over 3 steps the atomics' order differs run to run (eager vs eager too), and Adam
    turns a rounding-noise gradient into a full step of either sign, which the next forward
    propagates (measured 93-100% of the parameters within 1e-4 across runs, tools/graph_noise.py):
    the bars are the loss, the 2 lr per step envelope and >= 80% within 1e-4."""
    D, widths, BS, NEG, dtype, fused = case
    lr, k = 0.01, 3
    _, _, ea = make(D, widths, BS, NEG, dtype, fused=fused)
    _, _, gr = make(D, widths, BS, NEG, dtype, fused=fused)
    for m in (ea, gr):
        m.set_option("DETERMINISTIC", det)
    batches = _batches(D, BS, NEG, k)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        staged = [tuple(torch.from_numpy(x).cuda() for x in (hb.indptr, hb.indices, hb.values))
                  for hb in batches]
        gid = gr.graph_build_steps(staged)
        assert gr.global_step == 0
        for ip, ix, vv in staged:
            ea.set_batch(indptr=ip, indices=ix, values=vv)
            ea.train_step()
        gr.graph_launch(gid)
        torch.cuda.synchronize()
    assert ea.global_step == gr.global_step == k
    assert ea.beta_powers() == gr.beta_powers()
    la, lg = ea.loss_accuracy()[0], gr.loss_accuracy()[0]
    assert abs(la - lg) <= 1e-3 * abs(la) + 1e-6, (la, lg)
    if det:
        assert torch.equal(ea.params, gr.params)
        return
    d = (ea.params - gr.params).abs()
    assert float(d.max()) <= 2 * k * lr, float(d.max())
    assert float((d <= 1e-4).float().mean()) >= 0.8, float((d <= 1e-4).float().mean())


TIMED = ("FUSED_STATS", "MERGED_CSC", "HEAVY_IN_ADAM", "FUSED_W1_ADAM", "WHOLEK", "DW_IN_APPLY",
         "SCATTER_IN_COS")


@pytest.mark.parametrize("hosted", [True, False])
def test_cycle_graph_with_rank_in_adam_bit_identical(hosted):
    """bench.py's timed schedule at C2 (D=30000, 300/300/128, BS=1024, NEG=4, bf16: fused
    statistics, merged transpose with its scatter in the cosine launch, dW1 light rows and heavy
    columns inside Adam, dW_l tiles in the apply launches) under DETERMINISTIC (fixed-order fused
    statistics, every CSC column in row order, heavy dW1 rows summed in item order): a multi-step
    graph of 4 steps in which step i's Adam launch also runs step i+1's CSC rank pass
    (RANK_IN_ADAM; `hosted` False: every step its own rank launch) against 4 eager steps from the
    same state -- parameters, Adam slots, EMA, beta powers and loss bit-identical.  The graph then
    replays (the hosted passes re-arm what they consume)."""
    D, widths, BS, NEG, k = 30000, (300, 300, 128), 1024, 4, 4
    runs = []
    for _ in range(2):
        _, _, m = make(D, widths, BS, NEG, "bf16")
        m.set_option("DETERMINISTIC", True)
        m.set_option("RANK_IN_ADAM", hosted)
        sch = m.schedule()
        assert sch["DETERMINISTIC"] and all(sch[x] for x in TIMED), sch
        runs.append(m)
    gr, ea = runs
    batches = _batches(D, BS, NEG, k)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        staged = [tuple(torch.from_numpy(x).cuda() for x in (hb.indptr, hb.indices, hb.values))
                  for hb in batches]
        gid = gr.graph_build_steps(staged)
        gr.graph_launch(gid)
        for ip, ix, vv in staged:
            ea.set_batch(indptr=ip, indices=ix, values=vv)
            ea.train_step()
        torch.cuda.synchronize()
    assert gr.beta_powers() == ea.beta_powers()
    assert gr.loss_accuracy() == ea.loss_accuracy()
    for name in ("params", "adam_m", "adam_v", "ema"):
        x, y = getattr(gr, name), getattr(ea, name)
        assert torch.equal(x, y), (name, float((x - y).abs().max()))
    with torch.cuda.stream(s):
        gr.graph_launch(gid)
        torch.cuda.synchronize()
    assert np.isfinite(gr.loss_accuracy()[0])


def test_shadows_first_graph_matches_separate_graphs():
    """A graph of FWD_BWD + a shadow part without ADAM runs the shadow refresh FIRST (bench.py's
    data-parallel flow: the previous step's refresh merged with the next forward + backward).
    Deterministic unfused bf16 steps: [fwd+bwd, Adam, shadows] x 3 with separate graphs equals
    fwd+bwd, Adam, then [shadows+fwd+bwd, Adam] x 2 and a final shadows graph, bit for bit."""
    D, widths, BS, NEG = 3000, (128, 128, 64), 64, 4
    batches = _batches(D, BS, NEG, 3)
    s = torch.cuda.Stream()
    out = []
    with torch.cuda.stream(s):
        staged = [tuple(torch.from_numpy(x).cuda() for x in (hb.indptr, hb.indices, hb.values)) for hb in batches]
        for merged in (False, True):
            _, _, m = make(D, widths, BS, NEG, "bf16", fused=False)
            m.set_option("DETERMINISTIC", True)
            plain, comb = [], []
            for ip, ix, vv in staged:
                m.set_batch(indptr=ip, indices=ix, values=vv)
                plain.append(m.graph_build(_lib.GRAPH_FWD_BWD))
                comb.append(m.graph_build(_lib.GRAPH_FWD_BWD | _lib.GRAPH_SHADOWS))
            adam = m.graph_build(_lib.GRAPH_ADAM)
            sh = m.graph_build(_lib.GRAPH_SHADOWS)
            for i in range(3):
                m.graph_launch(comb[i] if merged and i > 0 else plain[i])
                m.graph_launch(adam)
                if not merged:
                    m.graph_launch(sh)
            if merged:
                m.graph_launch(sh)
            torch.cuda.synchronize()
            out.append((m.params.clone(), m.loss_accuracy()[0]))
    assert out[0][1] == out[1][1]
    assert torch.equal(out[0][0], out[1][0])
