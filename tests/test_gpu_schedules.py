"""The step's launch schedules against each other (same arithmetic, different launches).

Two placements of work are plan options (dssm_plan_set_option):

* DW_IN_APPLY: dW_l's split-K tiles run in the BN_{l-1} backward-apply launch (default,
  tn.h tn_chunk_body, 64 x 64 tiles) or in the backward pair launch (0, 128 x 64 tiles);
* SCATTER_IN_COS: the CSC transpose's scatter runs as a role of the cosine launch
  (default, csc.h) or beside the BN1 sums (0);
* BNB_IN_PAIR: the last layer's BN backward is formed while its dA pair launch stages the A
  operand (default, gemm.hip launch_bwd_pair_bnb, which also writes dZ_L for dW_L, dgamma / dbeta
  and the loss) or by its own BN-backward apply launch (0).

Both tile shapes sum every split in the same k order, and the scatter writes every entry to
the slot its rank reserved, so the schedules compute the same step.  The check is teacher-forced
like tests/test_gpu_graph.py (dW1's heavy-column float atomics are the step's one source of
run-to-run noise): before every step the variant gets the default model's state, both run the
step on the same batch, and then:

* the loss must be bit-identical (the forward does not depend on either option);
* unfused models (materialised gradients, the data-parallel path) must have gradients within
  1e-5 of the largest;
* parameters must be within 2 lr everywhere and within 1e-5 on >= 99.9% of the elements.
"""
import numpy as np
import pytest
import torch

from dssm_amd import _lib
from dssm_amd.data import synth_batch
from tests.test_gpu_parity import make

pytestmark = pytest.mark.gpu

VARIANTS = [{"DW_IN_APPLY": False}, {"SCATTER_IN_COS": False},
            {"DW_IN_APPLY": False, "SCATTER_IN_COS": False}, {"BNB_IN_PAIR": False}]
CASES = [
    # (D, widths, BS, NEG, fused); BS a multiple of 128: the whole-K backward pair path
    (5000, (300, 300, 128), 128, 4, True),
    (5000, (300, 300, 128), 128, 4, False),
    (3000, (200, 96), 256, 3, True),
]


def _copy_state(dst, src):
    for name in ("params", "grads", "adam_m", "adam_v", "ema"):
        getattr(dst, name).copy_(getattr(src, name))
    dst.set_beta_powers(*src.beta_powers())
    _lib.check(dst.lib.dssm_plan_sync_shadows(dst._plan, _lib.stream_ptr()), "sync_shadows")


@pytest.mark.parametrize("variant", VARIANTS, ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items()))
@pytest.mark.parametrize("case", CASES)
def test_schedule_matches_default(case, variant):
    D, widths, BS, NEG, fused = case
    lr, steps = 0.01, 3
    _, _, ref = make(D, widths, BS, NEG, "bf16", fused=fused)
    _, _, var = make(D, widths, BS, NEG, "bf16", fused=fused)
    for k, x in variant.items():
        var.set_option(k, x)
    assert ref.schedule()["BNB_IN_PAIR"] and not (var.schedule()["BNB_IN_PAIR"] and "BNB_IN_PAIR" in variant)
    batches = [synth_batch(D, BS, NEG, seed=3000 + i, mean_nnz=32) for i in range(steps)]
    for i, hb in enumerate(batches):
        _copy_state(var, ref)
        for m in (ref, var):
            m.set_batch(hb)
            if fused:
                m.train_step()
            else:
                m.forward(True)
                m.backward()
        torch.cuda.synchronize()
        lr_, lv = ref.loss_accuracy()[0], var.loss_accuracy()[0]
        assert lr_ == lv, (i, lr_, lv)
        if not fused:
            scale = float(ref.grads.abs().max())
            err = float((ref.grads - var.grads).abs().max())
            assert err <= 1e-5 * scale, (i, err, scale)
            for m in (ref, var):
                m.apply_adam()
            torch.cuda.synchronize()
        d = (ref.params - var.params).abs()
        assert float(d.max()) <= 2 * lr, (i, float(d.max()))
        assert float((d <= 1e-5).float().mean()) >= 0.999, (i, float((d <= 1e-5).float().mean()))
        assert ref.beta_powers() == var.beta_powers()
