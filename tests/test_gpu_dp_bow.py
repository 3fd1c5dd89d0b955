"""BASELINE config 3's data-parallel step with the HIP engine: dssm_amd.dist.DataParallel driving
the libdssm.so plan (dssm_amd.model.DSSM, bf16 perf mode) at the per-rank C3 shape (D=30000,
widths 300/300/128, BS=1024 queries per rank, NEG=4), world size 2.

RCCL refuses two ranks on one device, so the two ranks share the box's GPU over gloo (the
torch.distributed transport, its collectives staged through host memory); the library's RCCL
collectives themselves are executed by tests/test_gpu_rccl.py.  Each schedule is covered:
"zero" with the bf16 all-to-all wire (the default for bf16), "zero" with the fp32 wire
(reduce-scatter + all-gather) and "allreduce".  Step 1 runs eagerly (DataParallel.train_step),
step 2 through the captured graphs bench.py times (build_graphs / graph_step / settle).

Parity: the N-rank step equals one Adam step on the mean of the per-shard
gradients.
* Every rank ends each step with bit-identical parameters and Adam slots (after gather_state).
* Teacher-forced: from the state the ranks started the step in, a single-process engine computes
  each shard's gradient with the same kernels (unfused schedule); the exchange is emulated exactly
  (bf16 rounding of each rank's W1 rows summed in fp32 in rank order for the bf16 wire, fp32 sums
  otherwise) and TF1.x ApplyAdam is applied in float64.  Parameters and slots must match on all
  non-bias elements: 99.99% within 1e-6 + 1e-4*lr (parameters) / 1e-6 of max|m| (first slot), all
  within 0.05*lr / 1e-3 of max|m| (heavy W1 columns sum with float atomics in a different order,
  which can move a bf16-wire element by one bf16 ulp).
* Against the oracle (step 1): each rank's loss against the bf16-emulating float64 oracle on its
  shard (rel 1e-4), and the parameter update against oracle Adam on the oracle's mean of shard
  gradients (per weight tensor, ||dp - dp_ref|| <= 1e-2 ||dp_ref||).
Biases are excluded: under batch-stat BN their gradient is rounding noise."""
import functools
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dssm_amd.data import shard_batch, synth_batch
from oracle import dssm_oracle as O

pytestmark = pytest.mark.gpu

D, WIDTHS, BS, NEG, WORLD = 30000, [300, 300, 128], 1024, 4, 2
LR = 0.01
SCHEDULES = [("zero", "bf16"), ("zero", "bf16-sparse"), ("zero", "fp32"), ("allreduce", "fp32")]


def _global_batch(step):
    return synth_batch(D, BS * WORLD, NEG, seed=2000 + step)


def _shard(step, rank):
    return shard_batch(_global_batch(step), BS * WORLD, NEG, rank, WORLD)


def _model(fused=True):
    from dssm_amd.model import DSSM
    m = DSSM(D, WIDTHS, BS, NEG, lr=LR, dtype="bf16", init=False, device="cuda:0")
    if not fused:
        m.set_fused_w1_adam(False)
    return m


def _load(m, sd):
    m.load_state_dict(sd)
    torch.cuda.synchronize()


def _worker(rank, port, out_dir, mode, wire):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=WORLD)
    try:
        from dssm_amd.dist import DataParallel
        torch.cuda.set_device(0)
        s = torch.cuda.Stream()
        torch.cuda.set_stream(s)
        m = _model()
        with np.load(os.path.join(out_dir, "state0.npz")) as z:
            _load(m, {k: z[k] for k in z.files})
        sparse = wire == "bf16-sparse"  # the touched-row sparse gradient all-to-all
        wire = "bf16" if sparse else wire
        dp = DataParallel(m, comm="auto", mode=mode, wire=wire, sparse=sparse)
        assert (dp.world, dp.rank, dp.mode, dp.wire, dp.comm) == (WORLD, rank, mode, wire, "torch"), dp.schedule
        assert not dp.fallbacks, dp.fallbacks
        # step 1: eager
        m.set_batch(_shard(1, rank))
        dp.train_step()
        loss1 = m.loss_accuracy()[0]
        dp.gather_state()
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, f"s1_r{rank}.npz"), loss=np.array([loss1]), **m.state_dict())
        # step 2: the captured graphs bench.py replays, collectives between them
        b = _shard(2, rank)
        staged = [tuple(torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values))]
        dp.build_graphs(staged)
        dp.graph_step(0)
        dp.settle()
        loss2 = m.loss_accuracy()[0]
        dp.gather_state()
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, f"s2_r{rank}.npz"), loss=np.array([loss2]), **m.state_dict())
        dp.close()
    finally:
        dist.destroy_process_group()


@functools.lru_cache(maxsize=1)
def _state0():
    """A mid-training state (one fused single-GPU step from the reference init): non-zero Adam
    slots, so an update is a smooth function of the gradient rather than lr * sign(g)."""
    cfg = O.OracleConfig(trigram_d=D, widths=WIDTHS, query_bs=BS, neg=NEG, lr=LR)
    m = _model()
    # fixed-order reductions: the same state every run (the default schedule's fp32 atomics move
    # small-v Adam slots, to which step 1's update direction against the oracle is sensitive)
    m.set_option("DETERMINISTIC", True)
    m.load_params(O.init_params(cfg, seed=11))
    m.set_batch(synth_batch(D, BS, NEG, seed=999))
    m.train_step()
    torch.cuda.synchronize()
    return m.state_dict()


def _nonbias_mask(m):
    mask = np.ones(m.n_params, bool)
    for name, (off, rows, cols) in m.segments.items():
        if name.startswith("fc"):
            mask[off + (rows - 1) * cols: off + rows * cols] = False  # the bias row of [W; b]
    return mask


def _shard_grads(sd, step):
    """Each shard's flat gradient, computed from state sd by a single-process engine (unfused)."""
    e = _model(fused=False)
    _load(e, sd)
    out = []
    for r in range(WORLD):
        e.grads.zero_()
        e.set_batch(_shard(step, r))
        e.forward(True)
        e.backward()
        torch.cuda.synchronize()
        out.append(e.grads[:e.n_params].cpu().numpy().copy())
    return out, e


def _bf16(x):
    return O.bf16_round(x).astype(np.float32)


def _exchanged(gs, mode, wire, ext):
    """The gradient the rank's Adam sees (before its 1/world scale): the exchange emulated (the
    sparse exchange delivers the dense one's values: untouched rows are zero)."""
    g = np.zeros_like(gs[0])
    for gr in gs:  # fp32 sums in rank order
        if mode == "zero" and wire in ("bf16", "bf16-sparse"):
            g[:ext] += _bf16(gr[:ext])
            g[ext:] += gr[ext:]
        else:
            g += gr
    return g


def _adam64(sd, g):
    """TF1.x ApplyAdam (new_dssm.py:215-217) in float64 on the flat arenas, grad_scale 1/world."""
    n = g.size
    b1p, b2p = (float(x) for x in sd["beta_powers"])
    alpha = np.float32(LR) * np.sqrt(np.float32(1) - np.float32(b2p)) / (np.float32(1) - np.float32(b1p))
    gg = g.astype(np.float64) * (1.0 / WORLD)
    m = sd["adam_m"][:n].astype(np.float64)
    v = sd["adam_v"][:n].astype(np.float64)
    m = m + (gg - m) * (1 - 0.9)
    v = v + (gg * gg - v) * (1 - 0.999)
    p = sd["params"][:n].astype(np.float64) - float(alpha) * m / (np.sqrt(v) + 1e-8)
    return p, m, v


def _check_teacher_forced(tag, got, ref, mask, errs):
    p_ref, m_ref, _ = ref
    n = p_ref.size
    dp = np.abs(got["params"][:n] - p_ref)[mask]
    dm = np.abs(got["adam_m"][:n] - m_ref)[mask]
    mmax = np.abs(m_ref[mask]).max()
    errs[f"{tag}_param_q9999"] = (float(np.quantile(dp, 0.9999)), 1e-6 + 1e-4 * LR)
    errs[f"{tag}_param_max"] = (float(dp.max()), 0.05 * LR)
    errs[f"{tag}_m_q9999"] = (float(np.quantile(dm, 0.9999) / mmax), 1e-6)
    errs[f"{tag}_m_max"] = (float(dm.max() / mmax), 1e-3)


def _report(tag, errs):
    bad = {k: v for k, v in errs.items() if not v[0] <= v[1]}
    print(tag, {k: f"{v[0]:.3e}/{v[1]:.0e}" for k, v in errs.items()})
    assert not bad, (tag, bad)


@pytest.mark.parametrize("mode,wire", SCHEDULES, ids=[f"{a}-{b}" for a, b in SCHEDULES])
def test_bow_data_parallel_world2(mode, wire):
    sd0 = _state0()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as d:
        np.savez(os.path.join(d, "state0.npz"), **sd0)
        mp.spawn(_worker, args=(port, d, mode, wire), nprocs=WORLD, join=True)
        res = {}
        for k in (1, 2):
            for r in range(WORLD):
                with np.load(os.path.join(d, f"s{k}_r{r}.npz")) as z:
                    res[k, r] = {x: z[x] for x in z.files}
    errs = {}
    for k in (1, 2):  # bit-identical ranks (EMA aside: local BN statistics by design)
        for x in ("params", "adam_m", "adam_v", "beta_powers"):
            assert np.array_equal(res[k, 0][x], res[k, 1][x]), (k, x)
    prev = sd0
    for k in (1, 2):
        gs, eng = _shard_grads(prev, k)
        mask = _nonbias_mask(eng)
        ext = eng.wire_extent()
        ref = _adam64(prev, _exchanged(gs, mode, wire, ext))
        _check_teacher_forced(f"step{k}", res[k, 0], ref, mask, errs)
        prev = res[k, 0]
        del eng

    # step 1 against the float64 oracle (bf16-emulating): losses and the update's direction
    cfg = O.OracleConfig(trigram_d=D, widths=WIDTHS, query_bs=BS, neg=NEG, lr=LR)
    e = _model(fused=False)
    _load(e, sd0)
    p0 = {k: v.cpu().numpy().astype(np.float64) for k, v in e.named_params().items()}
    m0 = {k: v.cpu().numpy().astype(np.float64) for k, v in e.named_adam()[0].items()}
    v0 = {k: v.cpu().numpy().astype(np.float64) for k, v in e.named_adam()[1].items()}
    gsum = None
    for r in range(WORLD):
        cache, _ = O.forward(cfg, p0, O.make_ema(cfg), _shard(1, r).as_dict(), True, np.float64, emulate="bf16")
        lr_ = abs(float(res[1, r]["loss"][0]) - cache["loss"]) / abs(cache["loss"])
        errs[f"loss_rank{r}_vs_oracle"] = (lr_, 1e-4)
        g = O.backward(cfg, p0, cache, np.float64)
        gsum = g if gsum is None else {x: gsum[x] + g[x] for x in g}
    b1p, b2p = (float(x) for x in sd0["beta_powers"])
    alpha = LR * np.sqrt(1 - b2p) / (1 - b1p)
    e.load_state_dict(res[1, 0])
    p1 = {k: v.cpu().numpy().astype(np.float64) for k, v in e.named_params().items()}
    for x in ("W1", "W2", "W3"):
        g = gsum[x] / WORLD
        mm = m0[x] + (g - m0[x]) * 0.1
        vv = v0[x] + (g * g - v0[x]) * 0.001
        upd_ref = -alpha * mm / (np.sqrt(vv) + 1e-8)
        upd = p1[x] - p0[x]
        errs[f"update_{x}_vs_oracle"] = (float(np.linalg.norm(upd - upd_ref) / np.linalg.norm(upd_ref)), 1e-2)
    _report(f"dp {mode}/{wire}", errs)
