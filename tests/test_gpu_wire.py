"""Data-parallel bf16 wire kernels on one GPU (include/dssm.h dssm_plan_set_wire).

The collectives are the caller's (dssm_amd/dist.py, covered over gloo in test_dist_gloo.py);
what runs on the device is checked here with world = 1, where the reduce-scatter and
all-gather are identities:
* backward() ends by packing bf16(dW1) into the gradient wire (exactly torch's RNE rounding of
  the materialized fp32 gradient);
* Adam over a W1 shard reads the wire, updates the shard only, writes bf16(W1) into the
  parameter wire, and updates the fp32 tail (b1, W2.., BN) as the unwired step does;
* wire_shadows() rebuilds W1's bf16 shadow: a forward after it equals one after the fp32
  shadow refresh.
"""
import numpy as np
import pytest
import torch

from dssm_amd.data import synth_batch
from tests.test_gpu_parity import make

pytestmark = pytest.mark.gpu

D, WIDTHS, BS, NEG, LR = 5000, (300, 300, 128), 96, 4, 0.01


def _wired(m):
    ext = m.wire_extent()
    assert ext == D * WIDTHS[0]
    n = -(-ext // 512) * 512
    gw = torch.zeros(n, dtype=torch.bfloat16, device=m.device)
    pw = torch.zeros(n, dtype=torch.bfloat16, device=m.device)
    pw[:ext].copy_(m.params[:ext])
    m.set_wire(gw, pw)
    return ext, gw, pw


def _close(a, b):
    d = (a - b).abs()
    assert float(d.max()) <= 2 * LR, float(d.max())
    assert float((d <= 1e-5).float().mean()) >= 0.999, float((d <= 1e-5).float().mean())


@pytest.mark.parametrize("bs", [BS, 128])
@pytest.mark.parametrize("shard,grad_pass", [("all", "1"), ("first_half", "1"), ("all", "0")])
def test_wire_step_matches_unwired(shard, grad_pass, bs):
    """grad_pass 1 (default): dW1 straight into the wire by k_adam_step's W1 roles; 0: materialised
    dW1 + k_wire_pack.  bs 128 (a multiple of 128) takes the whole-K backward pair, whose dW_l tiles
    ride in the apply launches with the slabs reduced after them (the data-parallel schedule)."""
    BS = bs
    _, _, ref = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    _, _, m = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    m.set_option("WIRE_GRAD_PASS", grad_pass == "1")
    ext, gw, pw = _wired(m)
    end = ext if shard == "all" else (ext // 2) // 64 * 64
    m.set_adam_range(0, end)
    p0, m0 = m.params.clone(), m.adam_m.clone()
    hb = synth_batch(D, BS, NEG, seed=77, mean_nnz=32)
    for x in (ref, m):
        x.set_batch(hb)
        x.forward(True)
        x.backward()
    torch.cuda.synchronize()
    if grad_pass == "0":
        assert torch.equal(gw[:ext], m.grads[:ext].to(torch.bfloat16))
    else:  # the pass leaves the arena's W1 rows alone; the wire holds bf16(dW1), b1's row is fp32
        assert float(m.grads[:ext].abs().max()) == 0.0
        g_ref = ref.grads[:ext]
        torch.testing.assert_close(gw[:ext].float(), g_ref, rtol=2 ** -7, atol=1e-6 * float(g_ref.abs().max()))
        # b1's row (fp32, in the arena): under batch-stat BN dloss/db1 is exactly 0 and both sides
        # hold the same bf16-dZ1 summation noise (test_oracle.py), up to float-atomic order
        n1 = WIDTHS[0]
        b_m, b_r = m.grads[ext:ext + n1], ref.grads[ext:ext + n1]
        assert float((b_m - b_r).abs().max()) <= 1e-4 * float(b_r.abs().max()) + 1e-7
    ref.apply_adam(1.0)
    m.apply_adam(1.0)
    torch.cuda.synchronize()
    n = m.n_params
    _close(m.params[:end], ref.params[:end])
    _close(m.params[ext:n], ref.params[ext:n])
    torch.testing.assert_close(m.adam_m[ext:n], ref.adam_m[ext:n], rtol=1e-3, atol=1e-6)
    assert torch.equal(pw[:end], m.params[:end].to(torch.bfloat16))
    if end < ext:  # outside the shard: untouched
        assert torch.equal(m.params[end:ext], p0[end:ext])
        assert torch.equal(m.adam_m[end:ext], m0[end:ext])
    assert m.beta_powers() == ref.beta_powers()


def test_wire_shadows_equal_fp32_refresh():
    _, _, m = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    ext, gw, pw = _wired(m)
    m.set_adam_range(0, ext)
    hb = synth_batch(D, BS, NEG, seed=78, mean_nnz=32)
    m.set_batch(hb)
    m.forward(True)
    m.backward()
    m.apply_adam(1.0)
    m.wire_shadows()
    m.forward(False)
    torch.cuda.synchronize()
    a = m.fetch("cos_sim_raw").copy()
    m.sync_shadows()
    m.forward(False)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(m.fetch("cos_sim_raw"), a)


@pytest.mark.parametrize("parts", [2, 4, 8])
def test_wire_stage_sums_rank_partials_in_fp32(parts):
    """The all-to-all wire (dssm_plan_set_wire_stage, the default data-parallel exchange): Adam
    takes the shard's W1 gradient as the fp32 sum, in rank order, of `parts` bf16 partials (what
    dssm_all_to_all delivers).  Against the unwired Adam over the same range fed that fp32 sum,
    the shard's parameters and Adam slots are bit-identical."""
    _, _, ref = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    _, _, m = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    ext, gw, pw = _wired(m)
    stride = -(-ext // (64 * parts)) * 64
    s0, s1 = stride, min(2 * stride, ext)  # the shard of rank 1
    stage = torch.zeros(parts * stride, dtype=torch.bfloat16, device=m.device)
    gen = torch.Generator(device=m.device).manual_seed(5)
    for k in range(parts):  # rank k's bf16 gradient of this shard
        stage[k * stride:k * stride + (s1 - s0)] = (
            torch.randn(s1 - s0, generator=gen, device=m.device) * 1e-3).to(torch.bfloat16)
    m.set_wire_stage(stage, parts, stride)
    m.set_adam_range(s0, s1)
    ref.set_adam_range(s0, s1)
    acc = torch.zeros(s1 - s0, dtype=torch.float32, device=m.device)
    for k in range(parts):
        acc += stage[k * stride:k * stride + (s1 - s0)].float()
    ref.grads.zero_()
    ref.grads[s0:s1] = acc
    m.grads.zero_()
    ref.apply_adam(1.0 / parts)
    m.apply_adam(1.0 / parts)
    torch.cuda.synchronize()
    assert torch.equal(m.params[s0:s1], ref.params[s0:s1])
    assert torch.equal(m.adam_m[s0:s1], ref.adam_m[s0:s1])
    assert torch.equal(m.adam_v[s0:s1], ref.adam_v[s0:s1])
    assert torch.equal(pw[s0:s1], m.params[s0:s1].to(torch.bfloat16))
