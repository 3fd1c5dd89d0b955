"""Lazy W1 Adam (plan option LAZY_ADAM, include/dssm.h): inside a multi-step graph a W1
row with no entry in this step's batch nor the next one is left behind, and its zero-gradient steps
are replayed -- the dense ApplyAdam arithmetic of new_dssm.py:215-217, in order, each with its own
alpha -- when a batch next reads it, once it is kLazyCap (16) steps behind, and by the graph's last
step.  So wherever the caller can see them, parameters, Adam slots, bf16 shadows and beta powers
must equal dense Adam's BIT FOR BIT.  Checked under DETERMINISTIC (every reduction in a fixed
order) against eager dense steps from the same state, with a small batch over a 30k-wide
vocabulary (most rows untouched on most steps: long gaps, rows hitting the cap) and enough steps
that the alpha ring (64 lazy steps) wraps."""
import numpy as np
import pytest
import torch

from dssm_amd.data import synth_batch
from tests.test_gpu_parity import make

pytestmark = pytest.mark.gpu

D, WIDTHS, NEG = 30000, (300, 300, 128), 4


def _staged(BS, k, seed0, mean_nnz):
    out = []
    for i in range(k):
        b = synth_batch(D, BS, NEG, seed=seed0 + i, mean_nnz=mean_nnz)
        out.append(tuple(torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values)))
    return out


@pytest.mark.parametrize("BS,nbatch,steps,replays,mean_nnz", [(128, 10, 40, 2, 8), (1024, 6, 12, 1, 32)])
def test_lazy_graph_equals_dense_eager(BS, nbatch, steps, replays, mean_nnz):
    runs = []
    for lazy in (True, False, None):  # graph lazy, graph dense, eager dense
        _, _, m = make(D, WIDTHS, BS, NEG, "bf16")
        m.set_option("DETERMINISTIC", True)
        if lazy is not None:
            m.set_option("LAZY_ADAM", lazy)
        runs.append(m)
    gl, gd, ea = runs
    assert gl.schedule()["LAZY_ADAM"] and not gd.schedule()["LAZY_ADAM"]
    staged = _staged(BS, nbatch, 4100, mean_nnz)
    order = [staged[i % nbatch] for i in range(steps)]
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g1 = gl.graph_build_steps(order)
        g2 = gd.graph_build_steps(order)
        for _ in range(replays):
            gl.graph_launch(g1)
            gd.graph_launch(g2)
            for ip, ix, vv in order:
                ea.set_batch(indptr=ip, indices=ix, values=vv)
                ea.train_step()
        torch.cuda.synchronize()
    for other in (gd, ea):
        assert gl.beta_powers() == other.beta_powers()
        assert gl.loss_accuracy() == other.loss_accuracy()
        for name in ("params", "adam_m", "adam_v", "ema"):
            x, y = getattr(gl, name), getattr(other, name)
            d = (x != y).nonzero().flatten()
            assert d.numel() == 0, (name, d.numel(), int(d[0]) if d.numel() else -1,
                                    float((x - y).abs().max()))
    # the graph left every W1 shadow row current: an eval forward equals one after a refresh
    ip, ix, vv = staged[0]
    gl.set_batch(indptr=ip, indices=ix, values=vv)
    with torch.cuda.stream(s):
        gl.forward(False)
        torch.cuda.synchronize()
        a = gl.fetch("cos_sim_raw").copy()
        gl.sync_shadows()
        gl.forward(False)
        torch.cuda.synchronize()
    np.testing.assert_array_equal(gl.fetch("cos_sim_raw"), a)
