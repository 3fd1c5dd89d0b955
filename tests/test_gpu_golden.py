"""GPU path (through the C-ABI, fp32 parity mode) against the committed golden fixtures
(tests/golden/*.npz, produced by make_golden.py from the oracle).

Tolerances.  Forward: loss rel <= 1e-5, cosine/prob abs <= 1e-5.  Gradients: <= 1e-4 x max|g|
per tensor.  One Adam step from an identical state (teacher forced): params within 1e-5 on
every element whose gradient exceeds 1e-3 x max|g| and within 2 lr everywhere (Adam maps a
rounding-level gradient g to a step lr*g/(|g|+eps*sqrt(1-b2^t)) whose size is noise); Adam m/v
within 1e-4 / 1e-3 of their tensor maxima; EMA shadows rel 1e-4.  Free-running 3 steps: the same
rounding-level elements move by O(lr) and perturb later steps chaotically, so only the loss
trajectory (rel 1e-4), the EMA variances and a 3 lr envelope are checked.  Biases are
excluded from element checks: under batch-stat BN d loss/d b == 0 exactly, so both sides hold
only rounding noise (tests/test_oracle.py pins that)."""
import glob
import os
import re

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
FILES = sorted(f for f in glob.glob(os.path.join(GOLD, "*.npz"))
               if not os.path.basename(f).startswith("ref_"))  # ref_*: the reference's data path (test_ref_feed)
IDS = [os.path.basename(f) for f in FILES]
LR = 0.01


def load(path):
    from tests.golden.make_golden import CASES
    name = os.path.basename(path)[:-4]
    z = np.load(path, allow_pickle=False)
    return CASES[name], {k: z[k] for k in z.files}


def group(d, prefix):
    return {k[len(prefix) + 2:]: v for k, v in d.items() if k.startswith(prefix + "__")}


def is_bias(k):
    return re.fullmatch(r"b\d+", k) is not None


def batch_of(d, b, c):
    from dssm_amd.data import CSRBatch
    return CSRBatch(d[f"batch{b}__indptr"], d[f"batch{b}__indices"], d[f"batch{b}__values"],
                    c["BS"] * (2 + c["NEG"]), c["D"])


def model(c, fused):
    from dssm_amd.model import DSSM
    m = DSSM(c["D"], c["widths"], c["BS"], c["NEG"], dtype="fp32", init=False)
    m.set_fused_w1_adam(fused)
    return m


def check_update(m, d, s, label):
    """Compare the GPU state after step s with the oracle's (p{s}, m{s}, v{s}, ema{s})."""
    got = {k: v.cpu().numpy() for k, v in m.named_params().items()}
    gm, gv = m.named_adam()
    wells = group(d, f"well{s}")
    for k, ref in group(d, f"p{s}").items():
        if is_bias(k):
            continue
        diff = np.abs(got[k] - ref)
        well = np.unpackbits(wells[k])[:ref.size].astype(bool).reshape(ref.shape)
        assert diff[well].max(initial=0.0) <= 1e-5, (label, k, diff[well].max(initial=0.0))
        assert diff.max() <= 2 * LR, (label, k, diff.max())
        mref, vref = d[f"m{s}__{k}"], d[f"v{s}__{k}"]
        assert np.abs(gm[k].cpu().numpy() - mref).max() <= 1e-4 * np.abs(mref).max() + 1e-12, (label, k)
        assert np.abs(gv[k].cpu().numpy() - vref).max() <= 1e-3 * np.abs(vref).max() + 1e-20, (label, k)
    ema = {k: v.cpu().numpy() for k, v in m.named_ema().items()}
    for k, ref in group(d, f"ema{s}").items():
        np.testing.assert_allclose(ema[k], ref, rtol=1e-4, atol=1e-6, err_msg=f"{label} {k}")


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_step1_outputs_and_grads(path):
    c, d = load(path)
    m = model(c, fused=False)
    m.load_params(group(d, "p0"))
    m.set_batch(batch_of(d, 0, c))
    m.forward(True)
    m.backward()
    torch.cuda.synchronize()
    loss, acc = m.loss_accuracy()
    assert abs(loss - d["s1__loss"]) <= 1e-5 * abs(d["s1__loss"])
    assert acc == pytest.approx(float(d["s1__accuracy"]))
    np.testing.assert_allclose(m.fetch("cos_sim_raw").ravel(), d["s1__cos_sim_raw"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(m.fetch("prob"), d["s1__prob"], rtol=1e-4, atol=1e-5)
    for l in range(1, len(c["widths"]) + 1):
        mo = m.batch_moments(l)
        for t in ("q", "d"):
            np.testing.assert_allclose(mo[t][0], d[f"s1__bn{l}_{t}_batch_mean"], rtol=1e-4, atol=1e-6)
            np.testing.assert_allclose(mo[t][1], d[f"s1__bn{l}_{t}_batch_var"], rtol=1e-4, atol=1e-8)
    g = {k: v.cpu().numpy() for k, v in m.named_grads().items()}
    for k, ref in group(d, "g1").items():
        if is_bias(k):
            continue
        err = np.abs(g[k] - ref).max()
        assert err <= 1e-4 * np.abs(ref).max(), (k, err)


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_adam_steps_teacher_forced(path, fused):
    c, d = load(path)
    m = model(c, fused)
    # step 1 from the initial state (m = v = 0, beta powers = beta)
    m.load_params(group(d, "p0"))
    m.set_batch(batch_of(d, 0, c))
    m.train_step()
    torch.cuda.synchronize()
    check_update(m, d, 1, "step1")
    # step 2 from the oracle's exact step-1 state
    m.load_params(group(d, "p1"), ema=group(d, "ema1"))
    m.load_adam_state(group(d, "m1"), group(d, "v1"), 0.9 ** 2, 0.999 ** 2, step=1)
    m.set_batch(batch_of(d, 1, c))
    m.train_step()
    torch.cuda.synchronize()
    assert abs(m.loss_accuracy()[0] - d["losses"][1]) <= 1e-5 * abs(d["losses"][1])
    check_update(m, d, 2, "step2")


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_free_running_three_steps_then_eval(path):
    c, d = load(path)
    m = model(c, fused=True)
    m.load_params(group(d, "p0"))
    for s in range(3):
        m.set_batch(batch_of(d, s, c))
        m.train_step()
        torch.cuda.synchronize()
        assert abs(m.loss_accuracy()[0] - d["losses"][s]) <= 1e-4 * abs(d["losses"][s])
    got = {k: v.cpu().numpy() for k, v in m.named_params().items()}
    for k, ref in group(d, "p3").items():
        if not is_bias(k):
            assert np.abs(got[k] - ref).max() <= 3 * LR, k
    ema = {k: v.cpu().numpy() for k, v in m.named_ema().items()}
    for k, ref in group(d, "ema3").items():
        if k.endswith("_var"):
            np.testing.assert_allclose(ema[k], ref, rtol=1e-3, atol=1e-6, err_msg=k)
    # eval forward (on_train=False) from the fixture's own step-3 state
    m.load_params(group(d, "p3"), ema=group(d, "ema3"))
    m.set_batch(batch_of(d, 3, c))
    m.forward(False)
    torch.cuda.synchronize()
    assert abs(m.loss_accuracy()[0] - d["eval__loss"]) <= 1e-5 * abs(d["eval__loss"])
    np.testing.assert_allclose(m.fetch("cos_sim_raw").ravel(), d["eval__cos_sim_raw"], rtol=1e-4, atol=1e-5)
