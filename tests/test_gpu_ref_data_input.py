"""Training steps on feeds the reference's utils/data_input.py produced (tests/golden/
ref_data_input.npz: get_data_by_dssm2 over a fixed 21,128-word vocabulary, then pull_batch; see
tests/test_ref_data_input.py) against the oracle.  As tests/test_gpu_ref_feed.py: the oracle's
CSR is assembled from the fixture's COO triplets with scipy, the GPU is fed through
dssm_amd.data.feeds_to_csr; fp32 bars (loss rel 1e-5, cosines 1e-5, gradients 1e-4 x max|g|)
over three teacher-forced steps at D = nwords = 21128, widths 32/32, BS = 4, NEG = 4."""
import numpy as np
import pytest
import scipy.sparse as sps
import torch

from oracle import dssm_oracle as O
from tests.test_gpu_parity import is_bias, make, rel
from tests.test_ref_data_input import load_ref, ref_feeds

pytestmark = pytest.mark.gpu


def _oracle_batch(ref, b):
    mats = []
    for k in ("q", "p", "n"):
        idx = np.asarray(ref[f"b{b}_{k}_indices"])
        shp = tuple(int(x) for x in ref[f"b{b}_{k}_shape"])
        mats.append(sps.coo_matrix((ref[f"b{b}_{k}_values"].astype(np.float64), (idx[:, 0], idx[:, 1])),
                                   shape=shp).tocsr())
    m = sps.vstack(mats).tocsr()
    return {"indptr": m.indptr, "indices": m.indices, "values": m.data}


def test_steps_on_data_input_feeds():
    from dssm_amd.data import feeds_to_csr
    ref = load_ref()
    D, BS, NEG = int(ref["nwords"][0]), int(ref["bs"][0]), int(ref["neg"][0])
    cfg, p, m = make(D, (32, 32), BS, NEG, "fp32", fused=False)
    ema = O.make_ema(cfg)
    adam = O.AdamState(cfg, p)
    for b in range(3):
        m.load_params(p, ema=ema)
        m.load_adam_state(adam.m, adam.v, adam.beta1_power, adam.beta2_power, b)
        cache, ema = O.forward(cfg, p, ema, _oracle_batch(ref, b), True, np.float64)
        grads = O.backward(cfg, p, cache, np.float64)
        m.set_batch(feeds_to_csr(*ref_feeds(ref, b), trigram_d=D))
        m.forward(True)
        m.backward()
        torch.cuda.synchronize()
        assert rel(m.loss_accuracy()[0], cache["loss"]) <= 1e-5, b
        np.testing.assert_allclose(m.fetch("cos_sim_raw").ravel(), cache["cos_sim_raw"], rtol=1e-4, atol=1e-5)
        gg = {k: v.cpu().numpy() for k, v in m.named_grads().items()}
        for k, g in grads.items():
            if not is_bias(k):
                assert np.abs(gg[k] - g).max() <= 1e-4 * np.abs(g).max(), (b, k)
        adam.step(p, grads)
        m.apply_adam()
        torch.cuda.synchronize()
        gp = {k: v.cpu().numpy() for k, v in m.named_params().items()}
        for k in p:
            if not is_bias(k):
                d = np.abs(gp[k] - p[k])
                well = np.abs(grads[k]) > 1e-3 * np.abs(grads[k]).max()
                assert d[well].max(initial=0.0) <= 1e-5 and d.max() <= 2 * cfg.lr, (b, k)
