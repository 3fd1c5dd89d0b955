"""Multi-view DSSM at BASELINE config 5's size (archive/multi_view_dssm_v3.py:107-241): one user
tower and three item views, 30k-wide sparse inputs, FC 300 -> 128, BS = 4096, NEG = 4 -- the shape
`bench.py --model multiview` times -- against the float64 oracle (oracle/multiview_oracle.py,
scipy CSR inputs) on the same Zipf batches, for active views 1 and 3:
* loss (summed over the batch, as the reference) rel <= 1e-5; every cosine <= 1e-4 rel + 1e-5;
* every gradient of the user tower and the active view <= 1e-4 * max|g| (the other views get none),
  with the oracle's ReLU masks teacher-forced to the GPU's: at this size (1.2M pre-activations per
  layer and tower) a few pre-activations lie within fp32 rounding of zero, where the fp32 kernels and
  the float64 oracle legitimately take opposite ReLU branches (a whole row's contribution to one
  gradient column then differs); such flips must be rare (<= 20 per layer and tower) and each at
  |z| <= 1e-5 max|z|;
* one teacher-forced Adam step (the oracle's TF1.x ApplyAdam on the GPU's gradients): <= 1e-6 on
  well-conditioned elements (|g| > 1e-3 max|g|), <= 2 lr everywhere, untouched views unchanged.
The bf16 perf mode (bf16 W shadows, bf16 FC1 activation, bf16 dz2 / dz1, MFMA 16x16x32) is checked
against the bf16-emulating oracle (emulate="bf16": the same rounding points, float64 elsewhere):
loss rel <= 1e-4 (the north star's bar), cosines <= 1e-3 abs, every gradient ||err|| <= 5e-3 ||g||
(rounding-boundary flips of bf16 values, RNE ties); the optimizer's shadows equal bf16(weights) bit for
bit after a step and the untrained views' shadows are untouched.  The fused optimizer (the bench's
default: FC1's weight gradient gathered inside each tower's Adam launch, FC2's split-K partials summed
there) against the oracle's ApplyAdam on the unfused path's gradients, both dtypes."""
import numpy as np
import pytest
import torch

from dssm_amd.data import ZipfColumns, synth_rows
from dssm_amd.multiview import MultiViewDSSM
from oracle import multiview_oracle as M

pytestmark = pytest.mark.gpu

CFG = M.MvConfig(user_d=30000, view_d=[30000, 30000, 30000], l1=300, l2=128, bs=4096, neg=4, lr=0.05)


def _setup(view, dtype="fp32", fused=False):
    cfg = CFG
    p = M.init_params(cfg, 5)
    rot = M.rotations(cfg, 7)
    m = MultiViewDSSM(cfg.user_d, cfg.view_d, cfg.l1, cfg.l2, cfg.bs, cfg.neg, lr=cfg.lr, rotations=rot,
                      dtype=dtype, fused_w1_adam=fused)
    m.load_params(p)
    rng = np.random.Generator(np.random.PCG64(40 + view))
    u = synth_rows(rng, ZipfColumns(cfg.user_d), cfg.bs, 32.0)
    it = synth_rows(rng, ZipfColumns(cfg.view_d[view - 1]), cfg.bs, 32.0)
    m.set_batch(u, it, view)
    return cfg, p, rot, m, u, it


def _force_masks(m, fw, view):
    """Set the oracle's ReLU decisions (z > 0 of FC1 and FC2, both towers) to the GPU forward's
    (a1 > 0, y > 0) where they differ; return the flip counts after checking each flip lies at
    the fp32 rounding boundary."""
    BS, l1, l2 = m.bs, m.l1, m.l2
    gpu = {"u": (m.a1["u"][:, :l1], m.ysrc[:BS, :l2]), "it": (m.a1["i"][:, :l1], m.ysrc[BS:, :l2])}
    flips = {}
    for key in ("u", "it"):
        tw = fw[key]
        for z, a, pos in (("z1", "a1", gpu[key][0]), ("z2", "y", gpu[key][1])):
            gpos = pos.cpu().numpy() > 0
            zz = tw[z]
            bad = gpos != (zz > 0)
            n = int(bad.sum())
            flips[f"{key}_{z}"] = n
            assert n <= 20, (key, z, n)
            if n:
                scale = np.abs(zz).max()
                assert np.abs(zz[bad]).max() <= 1e-5 * scale, (key, z, np.abs(zz[bad]).max() / scale)
                zz[bad] = np.where(gpos[bad], 1e-30, -1e-30)  # the GPU's branch, at |z| ~ 0
                tw[a] = np.maximum(zz, 0)
    return flips


@pytest.mark.parametrize("view", [1, 3])
def test_multiview_config5_matches_oracle(view):
    cfg, p, rot, m, u, it = _setup(view)
    m.forward()
    m.backward()
    torch.cuda.synchronize()
    fw = M.forward(cfg, p, u, it, view, rot, dtype=np.float64, sparse=True)
    assert abs(m.loss() - fw["loss"]) <= 1e-5 * abs(fw["loss"]), (m.loss(), fw["loss"])
    cos = m.cos_raw.cpu().numpy().reshape(cfg.neg + 1, cfg.bs).T
    np.testing.assert_allclose(cos, fw["cos"], rtol=1e-4, atol=1e-5)
    flips = _force_masks(m, fw, view)
    print("config-5 view", view, "ReLU boundary flips", flips)
    g = M.backward(cfg, p, fw)
    got = m.named(m.grads)
    errs = {}
    for k, ref in g.items():
        errs[k] = float(np.abs(got[k] - ref).max() / np.abs(ref).max())
    print("config-5 view", view, {k: f"{v:.2e}" for k, v in errs.items()})
    assert all(v <= 1e-4 for v in errs.values()), errs
    for k, v in got.items():  # views without a gradient this step
        if not k.startswith(("user", f"view{view}")):
            assert not np.any(v), k

    # one teacher-forced Adam step on the GPU's own gradients
    gg = {k: v for k, v in got.items() if k.startswith(("user", f"view{view}"))}
    pref = {k: v.copy() for k, v in p.items()}
    M.Adam(cfg, pref).step(pref, gg)
    m.apply_adam()
    torch.cuda.synchronize()
    after = m.named()
    for k in pref:
        d = np.abs(after[k] - pref[k])
        assert d.max() <= 2 * cfg.lr, (k, d.max())
        if k in gg:
            well = np.abs(gg[k]) > 1e-3 * np.abs(gg[k]).max()
            assert d[well].max(initial=0.0) <= 1e-6, (k, d[well].max(initial=0.0))
        else:
            assert d.max() == 0.0, k


@pytest.mark.parametrize("view", [1, 3])
def test_multiview_config5_bf16_matches_emulating_oracle(view):
    cfg, p, rot, m, u, it = _setup(view, "bf16")
    m.forward()
    m.backward()
    torch.cuda.synchronize()
    fw = M.forward(cfg, p, u, it, view, rot, dtype=np.float64, sparse=True, emulate="bf16")
    assert abs(m.loss() - fw["loss"]) <= 1e-4 * abs(fw["loss"]), (m.loss(), fw["loss"])
    cos = m.cos_raw.cpu().numpy().reshape(cfg.neg + 1, cfg.bs).T
    assert float(np.abs(cos - fw["cos"]).max()) <= 1e-3
    g = M.backward(cfg, p, fw)
    got = m.named(m.grads)
    errs = {k: float(np.linalg.norm(got[k] - ref) / np.linalg.norm(ref)) for k, ref in g.items()}
    print("config-5 bf16 view", view, {k: f"{v:.2e}" for k, v in errs.items()})
    assert all(v <= 5e-3 for v in errs.values()), errs
    for k, v in got.items():
        if not k.startswith(("user", f"view{view}")):
            assert not np.any(v), k
    sh0 = {k: t.clone() for k, t in m.shadow.items()}
    m.apply_adam()
    torch.cuda.synchronize()
    for name, sh in m.shadow.items():
        w = m._block(m.params, name)[:-1]
        if name.startswith(("user", f"view{view}")):  # rewritten by the optimizer: bf16(RNE) of the weights
            assert torch.equal(sh[:, :w.shape[1]], w.to(torch.bfloat16)), name
            assert not torch.any(sh[:, w.shape[1]:].float()), name  # zero pads kept
        else:
            assert torch.equal(sh, sh0[name]), name


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_multiview_config5_fused_w1_adam(dtype):
    cfg, p, rot, ref, u, it = _setup(3, dtype, fused=False)
    _, _, _, m, _, _ = _setup(3, dtype, fused=True)
    for x in (ref, m):
        x.forward()
        x.backward()
    torch.cuda.synchronize()
    assert m._splits["u"].value > 1 and m._splits["i"].value > 1  # FC2's partials summed by the optimizer
    g = {k: v for k, v in ref.named(ref.grads).items() if k.startswith(("user", "view3"))}
    pref = {k: v.copy() for k, v in p.items()}
    M.Adam(cfg, pref).step(pref, g)
    m.apply_adam()
    torch.cuda.synchronize()
    after = m.named()
    for k in pref:
        d = np.abs(after[k] - pref[k])
        assert d.max() <= 2 * cfg.lr, (k, d.max())
        if k in g:
            well = np.abs(g[k]) > 1e-3 * np.abs(g[k]).max()
            assert d[well].max(initial=0.0) <= 1e-6, (k, d[well].max(initial=0.0))
        else:
            assert d.max() == 0.0, k
    for t in ("user", "view1", "view2", "view3"):
        assert not torch.any(m._block(m.grads, f"{t}_1")), t
    if dtype == "bf16":
        for name, sh in m.shadow.items():
            w = m._block(m.params, name)[:-1]
            assert torch.equal(sh[:, :w.shape[1]], w.to(torch.bfloat16)), name
