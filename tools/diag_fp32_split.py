"""Diagnostics (not collected by pytest): the fp32 parity mode's end-to-end C2 step against the
float64 oracle, per layer (Z, A, dA, dZ) and per gradient, for the library named by DSSM_LIB_PATH
(the split-product tiles, DSSM_G32_SPLIT=1, or the exact FMA-chain tiles, =0).  Usage, on a GPU:
    DSSM_LIB_PATH=dssm_amd/libdssm.so python tools/diag_fp32_split.py
    python tools/diag_fp32_split.py both      # both libraries, each in a child process"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run():
    import numpy as np
    import torch

    from dssm_amd import _lib
    from dssm_amd.data import synth_batch
    from dssm_amd.model import DSSM
    from oracle import dssm_oracle as O

    D, widths, BS, NEG = 30000, (300, 300, 128), 1024, 4
    cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=11)
    batch = synth_batch(D, BS, NEG, seed=1000, mean_nnz=32)
    cache, _ = O.forward(cfg, p, O.make_ema(cfg), batch.as_dict(), True, np.float64)
    grads = O.backward(cfg, p, cache, np.float64)
    m = DSSM(D, widths, BS, NEG, dtype="fp32", init=False)
    m.load_params(p)
    m.set_fused_w1_adam(False)
    m.set_batch(batch)
    m.forward(True)
    m.backward()
    torch.cuda.synchronize()

    def layer(bid, l, n):
        ld = (n + 7) // 8 * 8
        return m.buffer(bid, l, dtype=torch.float32).cpu().numpy().astype(np.float64).reshape(m.rows, ld)[:, :n]

    def err(g, r):
        return float(np.abs(g - r).max() / max(np.abs(r).max(), 1e-30))

    lib = os.environ.get("DSSM_LIB_PATH", "libdssm.so")
    out = []
    dA_ref = O.cosine_loss_backward(cfg, cache, np.float64)
    dAs = {}
    for l in range(len(widths), 0, -1):
        lc = cache["layers"][l - 1]
        dZ, _ = O.bn_relu_backward(cfg, lc, dA_ref, l)
        dAs[l] = dA_ref
        if l > 1:
            dA_ref = dZ @ p[f"W{l}"].astype(np.float64).T
    for l in range(len(widths)):
        lc = cache["layers"][l]
        out.append(f"Z{l + 1} {err(layer(_lib.BUF_Z, l, widths[l]), lc['Z']):.2e} "
                   f"A{l + 1} {err(layer(_lib.BUF_A, l, widths[l]), lc['A']):.2e} "
                   f"dA{l + 1} {err(layer(_lib.BUF_DA, l, widths[l]), dAs[l + 1]):.2e}")
    out.append(f"loss rel {abs(m.loss_accuracy()[0] - cache['loss']) / abs(cache['loss']):.2e}")
    gg = {k: v.cpu().numpy() for k, v in m.named_grads().items()}
    out.append(" ".join(f"{k} {err(gg[k], g):.2e}" for k, g in sorted(grads.items())))
    for line in out:
        print(f"[{os.path.basename(lib)}] {line}", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "both":
        for so in ("dssm_amd/libdssm.so", "dssm_amd/libdssmexact.so"):
            env = dict(os.environ, DSSM_LIB_PATH=os.path.join(ROOT, so))
            r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True,
                               text=True, timeout=300)
            print(r.stdout + "\n".join(r.stderr.splitlines()[-5:]), flush=True)
        return
    run()


if __name__ == "__main__":
    main()
