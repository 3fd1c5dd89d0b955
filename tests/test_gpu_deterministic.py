"""Deterministic mode (plan option DETERMINISTIC; SURVEY.md §5 "deterministic-reduction mode for
parity").

The default schedule has two run-to-run noise sources (DESIGN.md §3 "Numerics"): the CSC
transpose's per-column entry order (per-block slot reservations by atomics) and dW1's multi-item
heavy columns (fp32 atomics), plus the fused BN statistics' fp64 atomics.  Under DETERMINISTIC the
plan keeps the timed schedule but sums the fused statistics in a fixed order (each producer
workgroup's partials in a slab row, summed in row order by the last arrival: bnfuse.h DetAcc),
puts every CSC column in row order (k_csc_sort_rows, also after the merged transpose's scatter)
and sums heavy dW1 rows through per-item slabs in item order.  Checks:

* two runs from the same state over the same batches leave parameters, Adam slots, EMA shadows and
  gradients bit-identical (torch.equal), at the headline shape C2 (D=30000, 300/300/128, BS=1024,
  NEG=4 -- hundreds of heavy columns, the 6144-entry ones column) in bf16 and fp32, fused and
  unfused, and with the histogram transpose (CSC_RANK = 0);
* the two transposes (rank / histogram) agree to fp32 summation order (the rank path splits
  heavy columns into 256-entry items, the histogram path sums every column in one chain);
* the deterministic step computes the same step as the default one, teacher-forced.  Its BN
  sums are added in another order than the default's fp64 atomics, so an fp32-ulp difference can
  tip a bf16 rounding of an activation (tests/test_gpu_c2_bf16.py): the bars are those of the bf16
  end-to-end check there (loss rel 1e-4, gradients 3e-3 in norm); in fp32 it matches the oracle at
  test_gpu_parity.py's bars.
The multi-step graph of the timed schedule with the rank pass inside Adam against eager steps,
bit for bit, is tests/test_gpu_graph.py's.
"""
import numpy as np
import pytest
import torch

from dssm_amd.data import synth_batch
from oracle import dssm_oracle as O
from tests.test_gpu_parity import grad_check, is_bias, make, rel

pytestmark = pytest.mark.gpu

C2 = (30000, (300, 300, 128), 1024, 4)
SMALL = (5000, (300, 300, 128), 128, 4)


def _state(m):
    return [t.clone() for t in (m.params, m.adam_m, m.adam_v, m.ema, m.grads)]


def _run(case, dtype, fused, steps, csc_rank=True, graph=False):
    D, widths, BS, NEG = case
    _, _, m = make(D, widths, BS, NEG, dtype, fused=fused)
    m.set_option("DETERMINISTIC", True)
    m.set_option("CSC_RANK", csc_rank)
    sch = m.schedule()
    # both dtypes keep the timed schedule (fused statistics; the merged transpose at batch % 128)
    timed = csc_rank and case[2] % 128 == 0
    assert sch["DETERMINISTIC"] and sch["FUSED_STATS"] and sch["MERGED_CSC"] == timed, sch
    batches = [synth_batch(D, BS, NEG, seed=4000 + i, mean_nnz=32) for i in range(steps)]
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        staged = [tuple(torch.from_numpy(x).cuda() for x in (hb.indptr, hb.indices, hb.values))
                  for hb in batches]
        if graph:
            m.graph_launch(m.graph_build_steps(staged))
        else:
            for ip, ix, vv in staged:
                m.set_batch(indptr=ip, indices=ix, values=vv)
                if fused:
                    m.train_step()
                else:
                    m.forward(True)
                    m.backward()
                    m.apply_adam()
        torch.cuda.synchronize()
    return _state(m), m.loss_accuracy()[0]


@pytest.mark.parametrize("dtype,fused,csc_rank", [
    ("bf16", True, True), ("bf16", False, True), ("fp32", True, True), ("fp32", False, True),
    ("bf16", True, False)])
def test_repeated_runs_are_bit_identical(dtype, fused, csc_rank):
    a, la = _run(C2, dtype, fused, 3, csc_rank)
    b, lb = _run(C2, dtype, fused, 3, csc_rank)
    assert la == lb
    for name, x, y in zip(("params", "adam_m", "adam_v", "ema", "grads"), a, b):
        assert torch.equal(x, y), (name, float((x - y).abs().max()))


def test_graph_equals_eager_bit_for_bit():
    """bench's cycle graph (whole steps captured back to back) against eager steps: without
    order-dependent reductions the two are bit-identical, not just within a rounding bar."""
    a, la = _run(C2, "bf16", True, 2, graph=True)
    b, lb = _run(C2, "bf16", True, 2, graph=False)
    assert la == lb
    for x, y in zip(a[:4], b[:4]):  # the fused step leaves no materialised gradient to compare
        assert torch.equal(x, y)


def test_rank_and_histogram_transposes_agree():
    D, widths, BS, NEG = C2
    ms = []
    for rank in (True, False):
        _, _, m = make(D, widths, BS, NEG, "bf16", fused=False)
        m.set_option("DETERMINISTIC", True)
        m.set_option("CSC_RANK", rank)
        m.set_batch(synth_batch(D, BS, NEG, seed=4200, mean_nnz=32))
        m.forward(True)
        m.backward()
        ms.append(m)
    torch.cuda.synchronize()
    ga, gb = ms[0].grads, ms[1].grads
    assert float((ga - gb).abs().max()) <= 1e-5 * float(ga.abs().max())


@pytest.mark.parametrize("fused", [True, False])
def test_deterministic_step_matches_default(fused):
    """Teacher-forced: before every step the deterministic model gets the default model's state."""
    D, widths, BS, NEG = SMALL
    lr = 0.01
    _, _, ref = make(D, widths, BS, NEG, "bf16", fused=fused)
    _, _, det = make(D, widths, BS, NEG, "bf16", fused=fused)
    det.set_option("DETERMINISTIC", True)
    for i in range(3):
        for name in ("params", "grads", "adam_m", "adam_v", "ema"):
            getattr(det, name).copy_(getattr(ref, name))
        det.set_beta_powers(*ref.beta_powers())
        det.sync_shadows()
        hb = synth_batch(D, BS, NEG, seed=4100 + i, mean_nnz=32)
        for m in (ref, det):
            m.set_batch(hb)
            if fused:
                m.train_step()
            else:
                m.forward(True)
                m.backward()
        torch.cuda.synchronize()
        la, ld = ref.loss_accuracy()[0], det.loss_accuracy()[0]
        assert rel(ld, la) <= 1e-4, (i, la, ld)
        if not fused:
            for k, g in ref.named_grads().items():
                if k.startswith("W"):
                    err = float((g - det.named_grads()[k]).norm() / g.norm())
                    assert err <= 3e-3, (i, k, err)
            for m in (ref, det):
                m.apply_adam()
            torch.cuda.synchronize()
        d = (ref.params - det.params).abs()
        assert float(d.max()) <= 2 * lr, float(d.max())
        assert float((d <= 1e-4).float().mean()) >= 0.99


def test_deterministic_fp32_matches_oracle():
    D, widths, BS, NEG = SMALL
    cfg, p, m = make(D, widths, BS, NEG, "fp32", fused=False)
    m.set_option("DETERMINISTIC", True)
    batch = synth_batch(D, BS, NEG, seed=1000, mean_nnz=32)
    cache, _ = O.forward(cfg, p, O.make_ema(cfg), batch.as_dict(), True, np.float64)
    grads = O.backward(cfg, p, cache, np.float64)
    m.set_batch(batch)
    m.forward(True)
    m.backward()
    torch.cuda.synchronize()
    assert rel(m.loss_accuracy()[0], cache["loss"]) <= 1e-5
    np.testing.assert_allclose(m.fetch("cos_sim_raw").ravel(), cache["cos_sim_raw"], rtol=1e-4, atol=1e-5)
    gg = {k: v.cpu().numpy() for k, v in m.named_grads().items()}
    for k, g in grads.items():
        if not is_bias(k):
            grad_check(k, gg[k], g, 1e-4)


def test_tf_checkpoint_resume_is_bit_identical(tmp_path):
    """tf.train.Saver round trip (dssm_amd/tfckpt.py, new_dssm.py:248,331): save after two steps,
    train two more, restore into a fresh model and replay them -- parameters, Adam slots, EMA and
    beta powers end bit-identical (deterministic mode, so the replay has no atomics noise)."""
    from dssm_amd import tfckpt
    from dssm_amd.model import DSSM
    D, widths, BS, NEG = SMALL
    batches = [synth_batch(D, BS, NEG, seed=1000 + i) for i in range(4)]

    def model():
        m = DSSM(D, widths, BS, NEG, dtype="bf16", init=False)
        m.set_option("DETERMINISTIC", True)
        return m

    a = model()
    a.init_params(seed=5)
    for b in batches[:2]:
        a.set_batch(b)
        a.train_step()
    prefix = tfckpt.save_model(a, str(tmp_path / "model" / "model_1.ckpt"))
    for b in batches[2:]:
        a.set_batch(b)
        a.train_step()
    torch.cuda.synchronize()
    c = model()
    tfckpt.restore_model(c, tfckpt.latest_checkpoint(str(tmp_path / "model")))
    assert c.global_step == 2
    for b in batches[2:]:
        c.set_batch(b)
        c.train_step()
    torch.cuda.synchronize()
    n = a.n_params
    for x, y in ((a.params, c.params), (a.adam_m, c.adam_m), (a.adam_v, c.adam_v), (a.ema, c.ema)):
        assert torch.equal(x[:n] if x.numel() > n else x, y[:n] if y.numel() > n else y)
    assert a.beta_powers() == c.beta_powers()
