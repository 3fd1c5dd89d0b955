"""The RNN tower's dropout fused into the cosine launch (dssm_cosine_softmax_loss_dropout) against the
unfused launches it replaces -- dssm_rnn_dropout on the final states, dssm_cosine_softmax_loss, then
dssm_rnn_dropout on dy with the summed loss's BS scale (dssm_rnn.py:139-153, 214) -- on the same inputs.
Bar: bit-identical dropped rows, dy, cosine scores, probabilities and loss (same mask, same fp32
arithmetic), for keep < 1, keep = 1 (eval) and the config-4 shape."""
import ctypes as C

import numpy as np
import pytest
import torch

from dssm_amd import _lib

pytestmark = pytest.mark.gpu


def _p(t):
    return C.c_void_p(t.data_ptr())


@pytest.mark.parametrize("bs,neg,n,keep", [(40, 4, 256, 0.8), (33, 4, 64, 0.5), (1024, 4, 256, 0.9),
                                           (40, 4, 256, 1.0)])
def test_cosine_dropout_matches_unfused(bs, neg, n, keep):
    lib = _lib.load()
    dev = torch.device("cuda:0")
    R = bs * (2 + neg)
    g = torch.Generator().manual_seed(bs * 7 + n)
    x = (torch.rand(R, n, generator=g) * 2 - 1).to(dev)
    seed, step, gamma = 17, 5, 20.0
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def bufs():
        f = dict(device=dev, dtype=torch.float32)
        return dict(y=torch.full((R, n), 3.0, **f), raw=torch.zeros((neg + 1) * bs, **f),
                    sim=torch.zeros(bs * (neg + 1), **f), prob=torch.zeros(bs * (neg + 1), **f),
                    qn=torch.zeros(bs, **f), loss=torch.zeros(2, **f), dy=torch.full((R, n), 5.0, **f),
                    ws=torch.zeros(2 * ((bs + 3) // 4) + 64, **f))

    a = bufs()
    assert lib.dssm_rnn_dropout(_p(x), _p(a["y"]), R, n, n, C.c_float(keep), seed, step, C.c_float(1.0), s) == 0
    assert lib.dssm_cosine_softmax_loss(_p(a["y"]), n, n, bs, neg, C.c_float(gamma), _p(a["raw"]), _p(a["sim"]),
                                        _p(a["prob"]), _p(a["qn"]), _p(a["loss"]), _p(a["dy"]), _p(a["ws"]), s) == 0
    assert lib.dssm_rnn_dropout(_p(a["dy"]), _p(a["dy"]), R, n, n, C.c_float(keep), seed, step,
                                C.c_float(float(bs)), s) == 0
    b = bufs()
    assert lib.dssm_cosine_softmax_loss_dropout(_p(x), n, n, bs, neg, C.c_float(gamma), C.c_float(keep), seed, step,
                                                C.c_float(float(bs)), _p(b["y"]), _p(b["raw"]), _p(b["sim"]),
                                                _p(b["prob"]), _p(b["qn"]), _p(b["loss"]), _p(b["dy"]),
                                                _p(b["ws"]), s) == 0
    torch.cuda.synchronize()
    for k in ("y", "raw", "sim", "prob", "qn", "loss", "dy"):
        assert torch.equal(a[k], b[k]), (k, int((a[k] != b[k]).sum()))
    if keep < 1.0:  # the mask really dropped something
        assert float((b["y"] == 0).float().mean()) > 0.5 * (1 - keep)
