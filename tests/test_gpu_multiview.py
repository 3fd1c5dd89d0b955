"""Multi-view DSSM (dssm_amd/multiview.py, functional C-ABI) against the float64 oracle on the same
seeded inputs: loss (rel 1e-5), cosines, every gradient of the user tower and the active view
(<= 1e-4 * max|g|; the other views get none), teacher-forced Adam (<= 2 lr everywhere, 1e-6 on
well-conditioned elements), and a short training run.  The fused optimizer (fused_w1_adam: each
tower's FC1 weight gradient gathered inside its Adam launch, FC2's split-K partials summed there) is
checked against the oracle's Adam on the materialised gradients of the unfused path, fp32 and bf16,
at a batch whose ones column and head trigrams span several 256-entry work items."""
import numpy as np
import pytest
import torch

from dssm_amd.data import ZipfColumns, synth_rows
from dssm_amd.multiview import TOWERS, MultiViewDSSM
from oracle import multiview_oracle as M

pytestmark = pytest.mark.gpu


def _setup(view, bs=64, fused=False, dtype="fp32", csc_stream=True):
    cfg = M.MvConfig(user_d=3000, view_d=[2000, 2500, 1500], l1=64, l2=32, bs=bs, neg=4, lr=0.01)
    p = M.init_params(cfg, 1)
    rot = M.rotations(cfg, 3)
    m = MultiViewDSSM(cfg.user_d, cfg.view_d, cfg.l1, cfg.l2, cfg.bs, cfg.neg, lr=cfg.lr, rotations=rot,
                      fused_w1_adam=fused, dtype=dtype, csc_stream=csc_stream)
    m.load_params(p)
    rng = np.random.Generator(np.random.PCG64(view))
    u = synth_rows(rng, ZipfColumns(cfg.user_d), cfg.bs, 16.0)
    it = synth_rows(rng, ZipfColumns(cfg.view_d[view - 1]), cfg.bs, 16.0)
    m.set_batch(u, it, view)
    return cfg, p, rot, m, u, it


@pytest.mark.parametrize("view", [1, 3])
def test_multiview_matches_oracle(view):
    cfg, p, rot, m, u, it = _setup(view)
    m.forward()
    m.backward()
    torch.cuda.synchronize()
    fw = M.forward(cfg, p, u, it, view, rot)
    assert abs(m.loss() - fw["loss"]) <= 1e-5 * abs(fw["loss"]), (m.loss(), fw["loss"])
    np.testing.assert_allclose(m.cos_raw.cpu().numpy().reshape(cfg.neg + 1, cfg.bs).T, fw["cos"],
                               rtol=1e-4, atol=1e-5)
    g = M.backward(cfg, p, fw)
    got = m.named(m.grads)
    for k, ref in g.items():
        err = np.abs(got[k] - ref).max()
        assert err <= 1e-4 * np.abs(ref).max() + 1e-7, (k, err, np.abs(ref).max())


def test_multiview_adam_and_training():
    cfg, p, rot, m, u, it = _setup(2)
    opt = M.Adam(cfg, {k: v.copy() for k, v in p.items()})
    pref = {k: v.copy() for k, v in p.items()}
    m.forward()
    m.backward()
    torch.cuda.synchronize()
    g = {k: v for k, v in m.named(m.grads).items() if k.startswith(("user", "view2"))}
    m.apply_adam()
    torch.cuda.synchronize()
    opt.step(pref, g)
    got = m.named()
    for k in pref:
        d = np.abs(got[k] - pref[k])
        assert d.max() <= 2 * cfg.lr, (k, d.max())
        if k in g:
            well = np.abs(g[k]) > 1e-3 * np.abs(g[k]).max()
            assert d[well].max(initial=0.0) <= 1e-6, (k, d[well].max(initial=0.0))
        else:
            assert d.max() == 0.0, k  # views without a gradient are not updated
    losses = []
    for _ in range(20):
        m.train_step()
        losses.append(m.loss())
    assert np.isfinite(losses).all() and losses[-1] < losses[0], losses[::5]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_multiview_fused_w1_adam(dtype):
    """One step with the fused optimizer vs the oracle's ApplyAdam on the unfused path's gradients
    (same params, batch and dtype): <= 2 lr everywhere, <= 1e-6 on well-conditioned elements,
    untrained views unchanged, the W1 gradient rows left zero, bf16 shadows = bf16(weights); then a
    short fused training run."""
    cfg, p, rot, ref, u, it = _setup(2, bs=512, fused=False, dtype=dtype)
    _, _, _, m, _, _ = _setup(2, bs=512, fused=True, dtype=dtype)
    for x in (ref, m):
        x.forward()
        x.backward()
    torch.cuda.synchronize()
    assert abs(m.loss() - ref.loss()) <= 1e-6 * abs(ref.loss())
    g = {k: v for k, v in ref.named(ref.grads).items() if k.startswith(("user", "view2"))}
    pref = {k: v.copy() for k, v in p.items()}
    M.Adam(cfg, pref).step(pref, g)
    m.apply_adam()
    torch.cuda.synchronize()
    got = m.named()
    for k in pref:
        d = np.abs(got[k] - pref[k])
        assert d.max() <= 2 * cfg.lr, (k, d.max())
        if k in g:
            well = np.abs(g[k]) > 1e-3 * np.abs(g[k]).max()
            assert d[well].max(initial=0.0) <= 1e-6, (k, d[well].max(initial=0.0))
        else:
            assert d.max() == 0.0, k
    for t in TOWERS:  # heavy columns' atomics target: consumed and cleared
        assert not torch.any(m._block(m.grads, f"{t}_1")), t
    assert np.allclose(m.adam_state.cpu().numpy(), [0.9 ** 2, 0.999 ** 2], rtol=1e-6)
    if dtype == "bf16":
        for name, sh in m.shadow.items():
            w = m._block(m.params, name)[:-1]
            assert torch.equal(sh[:, :w.shape[1]], w.to(torch.bfloat16)), name
    losses = []
    for _ in range(10):
        m.train_step()
        losses.append(m.loss())
    assert np.isfinite(losses).all() and losses[-1] < losses[0], losses[::3]


def test_multiview_fused_forward_only_set_batch_loop():
    """Eval-style loop in fused mode (set_batch, forward, loss; no backward / Adam): forward()
    leaves the optimizer's CSC transposes running on their own stream (aux2; aux when csc_stream is
    off) never joined, and set_batch frees the previous batch tensors.  The batch tensors are marked
    in use on that stream (record_stream), so
    their memory is not handed out again while the transposes read them: every loss equals the
    unfused model's on the same batch, and a train step after the loop still matches."""
    cfg, p, rot, ref, _, _ = _setup(2, bs=512, fused=False)
    _, _, _, m, _, _ = _setup(2, bs=512, fused=True)
    rng = np.random.Generator(np.random.PCG64(5))
    for i in range(8):
        view = 1 + i % 3
        uu = synth_rows(rng, ZipfColumns(cfg.user_d), cfg.bs, 16.0)
        ii = synth_rows(rng, ZipfColumns(cfg.view_d[view - 1]), cfg.bs, 16.0)
        for x in (ref, m):
            x.set_batch(uu, ii, view)
            x.forward()
        # allocations on the caller's stream while aux may still read the freed batch
        junk = [torch.full((4096,), -1, dtype=torch.int32, device=m.device) for _ in range(8)]
        assert abs(m.loss() - ref.loss()) <= 1e-6 * abs(ref.loss()), (i, m.loss(), ref.loss())
        del junk
    for x in (ref, m):
        x.backward()
        x.apply_adam()
    torch.cuda.synchronize()
    pa, pb = ref.params.cpu().numpy(), m.params.cpu().numpy()
    d = np.abs(pa - pb)
    assert d.max() <= 2 * cfg.lr and (d <= 1e-5).mean() >= 0.999, (d.max(), (d > 1e-5).sum())


@pytest.mark.parametrize("dtype,csc_stream", [("fp32", True), ("bf16", True), ("bf16", False)])
def test_multiview_fused_graph_matches_eager(dtype, csc_stream):
    """The fused step's stream structure (item tower and transposes on self.aux, the optimizer launches
    chained on the backward streams, the beta powers advanced by the later launch) captured as ONE
    graph of 4 steps over 2 alternating feeds (views 1 and 3), as bench.py times it, against the same
    4 steps run eagerly: losses rel <= 1e-5, beta powers exact, parameters within 1e-5 on 99.99% of the
    elements and 2 lr everywhere (the heavy W1 columns' fp32 atomics may add in another order).
    csc_stream: the transposes on a third stream forked from the capture's origin stream (a fork
    from self.aux segfaulted capture_end, profiles/r05_mv_capture_probe.txt)."""
    cfg, p, rot, a, u, it = _setup(1, bs=512, fused=True, dtype=dtype, csc_stream=csc_stream)
    _, _, _, b, _, _ = _setup(1, bs=512, fused=True, dtype=dtype, csc_stream=csc_stream)
    rng = np.random.Generator(np.random.PCG64(77))
    feeds = []
    for view in (1, 3):
        uu = synth_rows(rng, ZipfColumns(cfg.user_d), cfg.bs, 16.0)
        ii = synth_rows(rng, ZipfColumns(cfg.view_d[view - 1]), cfg.bs, 16.0)
        a.set_batch(uu, ii, view)
        feeds.append((dict(a.batch), view))
    la, lb = [], []
    for i in range(4):
        a.batch, a.view = dict(feeds[i % 2][0]), feeds[i % 2][1]
        a.train_step()
        la.append(a.loss())
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(4):
            b.batch, b.view = dict(feeds[i % 2][0]), feeds[i % 2][1]
            b.forward()
            b.backward(join=False)
            b.apply_adam()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    lb.append(b.loss())
    assert abs(lb[-1] - la[-1]) <= 1e-5 * abs(la[-1]), (la, lb)
    assert torch.equal(a.adam_state, b.adam_state)
    pa, pb = a.params.cpu().numpy(), b.params.cpu().numpy()
    d = np.abs(pa - pb)
    assert d.max() <= 2 * cfg.lr, d.max()
    assert (d <= 1e-5).mean() >= 0.9999, (d > 1e-5).sum()
    if dtype == "bf16":
        for name, sh in b.shadow.items():
            w = b._block(b.params, name)[:-1]
            assert torch.equal(sh[:, :w.shape[1]], w.to(torch.bfloat16)), name
