"""fp32 parity mode's merged step (round 4: the CSC rank transpose's scan beside the SpMM rows, its
scatter as workgroups of the cosine launch, the rank pass inside the previous Adam, the last BN
applied by the cosine, the loss reduced inside the first BN-backward launch) against the separate
schedule (plan option MERGED_CSC off: the three transpose launches) on the
same batches, eager steps and a multi-step graph.

The forward does not read the transpose, so the first step's loss / accuracy are identical; a
column's CSC entries are ordered by workgroup arrival in both schedules, so dW1 differs in the last
bits and Adam amplifies that on near-zero gradients (up to lr per element and step): ||a - b|| <=
1e-4 ||b|| and max |a - b| <= 2 lr per step, per weight / BN parameter block; later losses within
1e-5 relative."""
import re

import numpy as np
import pytest
import torch

from dssm_amd.data import synth_batch
from oracle import dssm_oracle as O

pytestmark = pytest.mark.gpu

D, WIDTHS, BS, NEG = 30000, (300, 300, 128), 128, 4


def _model(merged, p):
    from dssm_amd.model import DSSM
    m = DSSM(D, WIDTHS, BS, NEG, dtype="fp32", init=False)
    m.set_option("MERGED_CSC", merged)
    m.load_params(p)
    return m


def _close(a, b, steps, lr=0.01):
    # FC biases feed a batch-stat BN, so their gradient is zero up to rounding noise and Adam moves
    # them by the noise's sign (test_gpu_parity skips them the same way)
    for k in b:
        if re.fullmatch(r"b\d+", k):
            continue
        x, y = a[k].cpu().numpy(), b[k].cpu().numpy()
        err = np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-30)
        assert err <= 1e-4, (k, err)
        assert np.abs(x - y).max() <= 2 * lr * steps, k


def test_fp32_merged_schedule_matches_separate():
    cfg = O.OracleConfig(trigram_d=D, widths=list(WIDTHS), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=4)
    a, b = _model(True, p), _model(False, p)
    assert a.schedule()["MERGED_CSC"] and not b.schedule()["MERGED_CSC"]
    batches = [synth_batch(D, BS, NEG, seed=70 + i) for i in range(3)]
    for i, batch in enumerate(batches):
        for m in (a, b):
            m.set_batch(batch)
            m.train_step()
        torch.cuda.synchronize()
        la, lb = a.loss_accuracy(), b.loss_accuracy()
        if i == 0:
            assert la == lb
        else:
            assert abs(la[0] - lb[0]) <= 1e-5 * abs(lb[0])
        _close(a.named_params(), b.named_params(), i + 1)


def test_fp32_merged_multistep_graph_matches_separate():
    """Three steps as ONE captured graph (the merged schedule's rank passes ride in the previous
    step's Adam) against the separate schedule's eager steps."""
    cfg = O.OracleConfig(trigram_d=D, widths=list(WIDTHS), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=6)
    a, b = _model(True, p), _model(False, p)
    dev = torch.device("cuda:0")
    hb = [synth_batch(D, BS, NEG, seed=80 + i) for i in range(3)]
    staged = [(torch.from_numpy(x.indptr).to(dev), torch.from_numpy(x.indices).to(dev),
               torch.from_numpy(x.values).to(dev)) for x in hb]
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        gid = a.graph_build_steps(staged, stream=s)
        a.graph_launch(gid, stream=s)
    s.synchronize()
    for x in hb:
        b.set_batch(x)
        b.train_step()
    torch.cuda.synchronize()
    assert abs(a.loss_accuracy()[0] - b.loss_accuracy()[0]) <= 1e-5 * abs(b.loss_accuracy()[0])
    _close(a.named_params(), b.named_params(), len(hb))


def test_fp32_forward_loss_without_backward():
    """A train forward leaves its loss to the backward's first launch; finalize_loss (loss_accuracy)
    reduces it when no backward follows, and an eval forward reduces it in place."""
    cfg = O.OracleConfig(trigram_d=D, widths=list(WIDTHS), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=5)
    a, b = _model(True, p), _model(False, p)
    batch = synth_batch(D, BS, NEG, seed=90)
    for m in (a, b):
        m.set_batch(batch)
        m.forward(True)
    torch.cuda.synchronize()
    assert a.loss_accuracy() == b.loss_accuracy()
    for m in (a, b):
        m.forward(False)
    torch.cuda.synchronize()
    assert a.loss_accuracy() == b.loss_accuracy()
