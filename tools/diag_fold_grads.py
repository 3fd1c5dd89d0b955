"""Diagnostics (not collected by pytest): the bf16 step's gradients against the bf16-emulating
float64 oracle at the C3 shard shape of tests/test_gpu_dp_bow.py, with the BN backward folded into
the pairs (BNB_IN_PAIR = 1, default) and with the apply launches (0): relative L2 error per weight.
    python tools/diag_fold_grads.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from dssm_amd.data import shard_batch, synth_batch
    from dssm_amd.model import DSSM
    from oracle import dssm_oracle as O

    D, WIDTHS, BS, NEG, WORLD = 30000, [300, 300, 128], 1024, 4, 2
    cfg = O.OracleConfig(trigram_d=D, widths=WIDTHS, query_bs=BS, neg=NEG, lr=0.01)
    p0 = O.init_params(cfg, seed=11)
    glob = synth_batch(D, BS * WORLD, NEG, seed=2001)
    b = shard_batch(glob, BS * WORLD, NEG, 0, WORLD)
    cache, _ = O.forward(cfg, p0, O.make_ema(cfg), b.as_dict(), True, np.float64, emulate="bf16")
    g_ref = O.backward(cfg, p0, cache, np.float64)
    for fold in (True, False):
        m = DSSM(D, WIDTHS, BS, NEG, lr=0.01, dtype="bf16", init=False)
        m.load_params(p0)
        m.set_fused_w1_adam(False)
        m.set_option("BNB_IN_PAIR", fold)
        m.set_batch(b)
        m.forward(True)
        m.backward()
        torch.cuda.synchronize()
        gg = {k: v.cpu().numpy().astype(np.float64) for k, v in m.named_grads().items()}
        errs = {k: float(np.linalg.norm(gg[k] - g_ref[k]) / np.linalg.norm(g_ref[k]))
                for k in ("W1", "W2", "W3", "bn1_d_beta", "bn2_d_beta", "bn3_d_beta")}
        print(f"fold {fold} schedule {sorted(k for k, v in m.schedule().items() if v)}", flush=True)
        print("  " + " ".join(f"{k} {v:.3e}" for k, v in errs.items()), flush=True)
    # one fused train step (fused W1 Adam, deferred dW slabs) with and without the fold
    res = {}
    for fold in (True, False):
        m = DSSM(D, WIDTHS, BS, NEG, lr=0.01, dtype="bf16", init=False)
        m.load_params(p0)
        m.set_option("BNB_IN_PAIR", fold)
        m.set_option("DETERMINISTIC", True)
        m.set_batch(b)
        m.train_step()
        torch.cuda.synchronize()
        res[fold] = {k: v.cpu().numpy().astype(np.float64) for k, v in m.named_params().items()}
    for k in res[True]:
        d = np.abs(res[True][k] - res[False][k])
        if d.max() > 0:
            print(f"  fused step param {k}: max diff {d.max():.3e}, differ {(d > 0).sum()} of {d.size}", flush=True)
    print("fused step compared", flush=True)


if __name__ == "__main__":
    main()
