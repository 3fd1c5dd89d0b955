"""Diagnostics (not collected by pytest): where the bf16 step with the last layer's BN backward
folded into the pair launch (BNB_IN_PAIR, default) differs from the apply-launch schedule, per
buffer and gradient tensor, on one step from the same state (tests/test_gpu_schedules.py case 1).
    python tools/diag_bnb.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from dssm_amd import _lib
    from dssm_amd.data import synth_batch
    from tests.test_gpu_parity import make

    D, widths, BS, NEG = 5000, (300, 300, 128), 128, 4
    models = []
    for fold in (True, True, False, False):
        _, _, m = make(D, widths, BS, NEG, "bf16", fused=False)
        m.set_option("BNB_IN_PAIR", fold)
        models.append(m)
    hb = synth_batch(D, BS, NEG, seed=3000, mean_nnz=32)
    for m in models:
        m.set_batch(hb)
        m.forward(True)
        m.backward()
    torch.cuda.synchronize()
    for i, j in ((0, 1), (2, 3), (0, 2), (1, 3)):
        a = models[i].buffer(_lib.BUF_DZ, 2, dtype=torch.bfloat16).float()
        b = models[j].buffer(_lib.BUF_DZ, 2, dtype=torch.bfloat16).float()
        ga, gb = models[i].named_grads()["W1"], models[j].named_grads()["W1"]
        print(f"models {i} vs {j} (fold {i < 2} / {j < 2}): dZ3 differ {int((a != b).sum())}, "
              f"grad W1 max diff {float((ga - gb).abs().max()):.3e}", flush=True)
    ref, var = models[0], models[2]
    L = len(widths)
    for name, bid, dt in (("Z", _lib.BUF_Z, torch.float32), ("A", _lib.BUF_A, torch.bfloat16),
                          ("dA", _lib.BUF_DA, torch.float32), ("dZ", _lib.BUF_DZ, torch.bfloat16)):
        for l in range(L):
            a = ref.buffer(bid, l, dtype=dt).float().cpu().numpy()
            b = var.buffer(bid, l, dtype=dt).float().cpu().numpy()
            d = np.abs(a - b)
            i = int(d.argmax())
            print(f"{name}{l + 1}: differ {int((d > 0).sum())} of {d.size}, max {d.max():.3e} at {i} "
                  f"(ld {(widths[l] + 7) // 8 * 8}: row {i // ((widths[l] + 7) // 8 * 8)}, col {i % ((widths[l] + 7) // 8 * 8)}) "
                  f"values {a.ravel()[i]:.6e} / {b.ravel()[i]:.6e}", flush=True)
    ga, gb = ref.named_grads(), var.named_grads()
    for k in ga:
        d = (ga[k] - gb[k]).abs()
        print(f"grad {k}: max {float(d.max()):.3e} (scale {float(ga[k].abs().max()):.3e}), differ {int((d > 0).sum())}",
              flush=True)


if __name__ == "__main__":
    main()
