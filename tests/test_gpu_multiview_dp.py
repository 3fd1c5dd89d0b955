"""Multi-view data parallelism (dssm_amd.multiview.MultiViewDataParallel, BASELINE config 5 across
GPUs) at world size 2: two processes on the one GPU of the box over gloo (the torch.distributed
transport; RCCL itself needs a GPU per rank).  Each rank trains on its own batch with the same
active view.  Parity: after one step both ranks' parameters are bit-identical, their exchanged
gradients equal the sum of the two per-batch gradients computed by one process (fp32, 1e-6 of the
tensor's largest), and the parameters equal one Adam step on the mean of those gradients on the
well-conditioned elements (|g| > 1e-3 max|g|: elsewhere Adam's first step is ±lr of a rounding-level
gradient, whose sign the dW1 atomics' summation order decides)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFGS = {"toy": dict(user_d=2000, view_d=[1800, 1900, 2000], l1=64, l2=32, bs=64, neg=4, nnz=12.0),
        # BASELINE config 5 per rank (bench.py --model multiview): 30k views, 300 -> 128, BS = 4096
        "config5": dict(user_d=30000, view_d=[30000, 30000, 30000], l1=300, l2=128, bs=4096, neg=4, nnz=32.0)}
VIEW = 2


def _batch(cfg, rank):
    from dssm_amd.data import ZipfColumns, synth_rows
    rng = np.random.Generator(np.random.PCG64(100 + rank))
    u = synth_rows(rng, ZipfColumns(cfg["user_d"]), cfg["bs"], cfg["nnz"])
    it = synth_rows(rng, ZipfColumns(cfg["view_d"][VIEW - 1]), cfg["bs"], cfg["nnz"])
    return u, it


def _model(cfg):
    from dssm_amd.multiview import MultiViewDSSM
    m = MultiViewDSSM(cfg["user_d"], cfg["view_d"], cfg["l1"], cfg["l2"], cfg["bs"], cfg["neg"], lr=0.01,
                      device=torch.device("cuda", 0), fused_w1_adam=False)
    m.init_params(4)
    return m


def _worker(rank, port, out_dir, name):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        from dssm_amd.multiview import MultiViewDataParallel
        torch.cuda.set_device(0)
        cfg = CFGS[name]
        m = _model(cfg)
        m.set_batch(*_batch(cfg, rank), VIEW)
        dp = MultiViewDataParallel(m, comm="auto")
        assert dp.world == 2 and dp.comm == "torch"
        m.forward()
        m.backward()
        dp.exchange()
        torch.cuda.synchronize()
        g = m.grads.cpu().numpy().copy()
        m.apply_adam(grad_scale=0.5)
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), params=m.params.cpu().numpy(), grads=g)
        dp.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", list(CFGS))
def test_multiview_dp_world2_matches_mean_gradient_step(name):
    cfg = CFGS[name]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(port, d, name), nprocs=2, join=True)
        r0, r1 = (np.load(os.path.join(d, f"r{r}.npz")) for r in (0, 1))
        # one process: each batch's gradient, their sum, one Adam step on the mean
        m = _model(cfg)
        gs = []
        for rank in (0, 1):
            m.grads.zero_()
            m.set_batch(*_batch(cfg, rank), VIEW)
            m.forward()
            m.backward()
            torch.cuda.synchronize()
            gs.append(m.grads.clone())
        m.grads.copy_(gs[0] + gs[1])
        m.apply_adam(grad_scale=0.5)
        torch.cuda.synchronize()
        gsum = (gs[0] + gs[1]).cpu().numpy()
        p_ref = m.params.cpu().numpy()
        ranges = m.trained_ranges()
    assert np.array_equal(r0["params"], r1["params"]), "ranks diverged"
    for b, e in ranges:
        got, ref = r0["grads"][b:e], gsum[b:e]
        assert np.abs(got - ref).max() <= 1e-6 * np.abs(ref).max(), (b, e)
        well = np.abs(ref) > 1e-3 * np.abs(ref).max()
        dp_ = np.abs(r0["params"][b:e] - p_ref[b:e])
        assert dp_[well].max() <= 1e-6, (b, e, dp_[well].max())
        assert dp_.max() <= 2 * 0.01 + 1e-6
