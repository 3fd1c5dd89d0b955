"""Multi-view oracle (oracle/multiview_oracle.py) pinned by float64 finite differences."""
import numpy as np

from dssm_amd.data import ZipfColumns, synth_rows
from oracle import multiview_oracle as M


def test_multiview_gradients_fd():
    cfg = M.MvConfig(user_d=40, view_d=[30, 35, 25], l1=8, l2=6, bs=6, neg=3)
    p = {k: v.astype(np.float64) for k, v in M.init_params(cfg, 1).items()}
    rng = np.random.Generator(np.random.PCG64(2))
    u = synth_rows(rng, ZipfColumns(40), cfg.bs, 6.0, 2, 10)
    it = synth_rows(rng, ZipfColumns(35), cfg.bs, 6.0, 2, 10)
    rot = M.rotations(cfg, 3)
    fw = M.forward(cfg, p, u, it, 2, rot)
    g = M.backward(cfg, p, fw)
    assert set(g) == {f"{t}_{w}" for t in ("user", "view2") for w in ("W1", "b1", "W2", "b2")}
    h = 1e-6
    for k in g:
        flat = p[k].reshape(-1)
        for i in np.random.default_rng(0).choice(flat.size, size=min(10, flat.size), replace=False):
            old = flat[i]
            flat[i] = old + h
            lp = M.forward(cfg, p, u, it, 2, rot)["loss"]
            flat[i] = old - h
            lm = M.forward(cfg, p, u, it, 2, rot)["loss"]
            flat[i] = old
            num = (lp - lm) / (2 * h)
            assert abs(num - g[k].reshape(-1)[i]) <= 1e-6 + 1e-5 * abs(num), (k, i, num)


def test_multiview_sparse_f32_matches_f64():
    """The CPU baseline's restatement (float32, scipy CSR FC1) against the float64 dense oracle."""
    cfg = M.MvConfig(user_d=300, view_d=[200, 250, 280], l1=24, l2=16, bs=64, neg=4)
    p = M.init_params(cfg, 5)
    rng = np.random.Generator(np.random.PCG64(6))
    u = synth_rows(rng, ZipfColumns(300), cfg.bs, 12.0)
    it = synth_rows(rng, ZipfColumns(280), cfg.bs, 12.0)
    rot = M.rotations(cfg, 7)
    f64 = M.forward(cfg, p, u, it, 3, rot)
    f32 = M.forward(cfg, p, u, it, 3, rot, dtype=np.float32, sparse=True)
    assert abs(f32["loss"] - f64["loss"]) <= 1e-4 * abs(f64["loss"])
    np.testing.assert_allclose(f32["cos"], f64["cos"], atol=1e-5)
    g64, g32 = M.backward(cfg, p, f64), M.backward(cfg, p, f32)
    assert set(g64) == set(g32)
    for k in g64:
        assert np.abs(g32[k] - g64[k]).max() <= 1e-4 * np.abs(g64[k]).max(), k
