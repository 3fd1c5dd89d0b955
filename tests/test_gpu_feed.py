"""Native asynchronous feeder (dssm_feeder_*, dssm_amd/feed.py Feeder): the device CSR it hands the
plan is the batch pull_batch would feed -- eval forwards fed by it are bit-identical to forwards fed
through DSSM.set_batch(feeds_to_csr(pull_batch(...))) -- and a training loop driven by it (slots
reused while earlier steps are in flight, eager and graph-captured per slot) keeps training."""
import numpy as np
import pytest
import scipy.sparse as sps
import torch

from dssm_amd import _lib
from dssm_amd.data import ZipfColumns, feeds_to_csr, pull_batch, synth_rows
from dssm_amd.feed import Feeder
from tests.test_gpu_parity import make

pytestmark = pytest.mark.gpu

D, WIDTHS, BS, NEG, NB = 2000, (64, 64, 32), 64, 4, 6


class _Conf:
    NEG = NEG


def _mats():
    cols = ZipfColumns(D)
    rng = np.random.Generator(np.random.PCG64(21))
    out = []
    for rows in (NB * BS, NB * BS, NB * BS * NEG):
        ip, ix, vv = synth_rows(rng, cols, rows, 24.0)
        out.append(sps.csr_matrix((vv, ix, ip), shape=(rows, D)))
    return out


def test_feeder_matches_pull_batch_eval():
    q, d, n = _mats()
    _, _, a = make(D, WIDTHS, BS, NEG, "fp32")
    _, _, b = make(D, WIDTHS, BS, NEG, "fp32")
    f = Feeder(q, d, n, BS, NEG, max_nnz=a.max_nnz)
    order = [3, 0, 5, 1, 1, 4]
    f.start(order[0])
    for i, bi in enumerate(order):
        got = f.next(a, next_batch=order[i + 1] if i + 1 < len(order) else None)
        assert got == bi
        a.forward(False)
        f.done()
        feed = pull_batch(False, q, d, n, bi, BS, "q", "p", "n", "t", _Conf)
        b.set_batch(feeds_to_csr(feed["q"], feed["p"], feed["n"], D))
        b.forward(False)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(a.fetch("cos_sim_raw"), b.fetch("cos_sim_raw"))
        assert a.loss_accuracy() == b.loss_accuracy()
    f.close()


@pytest.mark.parametrize("graph", [False, True])
def test_feeder_training_loop(graph):
    q, d, n = _mats()
    _, _, m = make(D, WIDTHS, BS, NEG, "bf16")
    f = Feeder(q, d, n, BS, NEG, max_nnz=m.max_nnz)
    s = torch.cuda.Stream()
    losses = []
    with torch.cuda.stream(s):
        gids = None
        if graph:  # one captured step per slot (the slot's device pointers are fixed)
            gids = []
            for slot in range(2):
                f.start(slot)
                f.next(m)
                gids.append(m.graph_build())
                f.done()
            torch.cuda.synchronize()
        f.start(0)
        for i in range(3 * NB):
            slot = i % 2
            f.next(m, next_batch=(i + 1) % NB)
            if graph:
                m.graph_launch(gids[slot])
            else:
                m.train_step()
            f.done()
            if i % NB == NB - 1:
                torch.cuda.synchronize()
                losses.append(m.loss_accuracy()[0])
        torch.cuda.synchronize()
    f.close()
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses
