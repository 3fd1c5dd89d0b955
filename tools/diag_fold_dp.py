"""Diagnostics (not collected by pytest): tests/test_gpu_dp_bow.py's state and shard, single
process: the unfused backward's gradients with and without BNB_IN_PAIR, bitwise and against the
bf16-emulating oracle.   python tools/diag_fold_dp.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from dssm_amd.data import shard_batch, synth_batch
    from dssm_amd.model import DSSM
    from oracle import dssm_oracle as O

    D, WIDTHS, BS, NEG, WORLD, LR = 30000, [300, 300, 128], 1024, 4, 2, 0.01
    cfg = O.OracleConfig(trigram_d=D, widths=WIDTHS, query_bs=BS, neg=NEG, lr=LR)
    out = {}
    for fold in (True, False):
        m = DSSM(D, WIDTHS, BS, NEG, lr=LR, dtype="bf16", init=False, device="cuda:0")
        m.set_option("BNB_IN_PAIR", fold)
        m.load_params(O.init_params(cfg, seed=11))
        m.set_batch(synth_batch(D, BS, NEG, seed=999))
        m.train_step()
        torch.cuda.synchronize()
        sd0 = m.state_dict()
        e = DSSM(D, WIDTHS, BS, NEG, lr=LR, dtype="bf16", init=False, device="cuda:0")
        e.set_option("BNB_IN_PAIR", fold)
        e.set_fused_w1_adam(False)
        e.load_state_dict(sd0)
        b = shard_batch(synth_batch(D, BS * WORLD, NEG, seed=2001), BS * WORLD, NEG, 0, WORLD)
        e.set_batch(b)
        e.forward(True)
        e.backward()
        torch.cuda.synchronize()
        p0 = {k: v.cpu().numpy().astype(np.float64) for k, v in e.named_params().items()}
        gg = {k: v.cpu().numpy().astype(np.float64) for k, v in e.named_grads().items()}
        cache, _ = O.forward(cfg, p0, O.make_ema(cfg), b.as_dict(), True, np.float64, emulate="bf16")
        g_ref = O.backward(cfg, p0, cache, np.float64)
        out[fold] = (sd0, gg)
        print(f"fold {fold}: " + " ".join(
            f"{k} {np.linalg.norm(gg[k] - g_ref[k]) / np.linalg.norm(g_ref[k]):.3e}" for k in ("W1", "W2", "W3")),
            flush=True)
    for k in ("params", "adam_m", "adam_v"):
        a, c = out[True][0][k], out[False][0][k]
        print(f"state0 {k}: differ {(a != c).sum()} max {np.abs(a - c).max():.3e}", flush=True)
    for k in ("W1", "W2", "W3"):
        a, c = out[True][1][k], out[False][1][k]
        print(f"grad {k}: differ {(a != c).sum()} max {np.abs(a - c).max():.3e} scale {np.abs(c).max():.3e}", flush=True)


if __name__ == "__main__":
    main()
