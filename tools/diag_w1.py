"""Diagnostic: per-step W1 gradient agreement (unfused) for the C1 case."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from oracle import dssm_oracle as O
from dssm_amd.data import synth_batch
from dssm_amd.model import DSSM
D, widths, BS, NEG = 1000, (100, 100), 128, 4
cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
p = O.init_params(cfg, seed=11)
m = DSSM(D, widths, BS, NEG, dtype="fp32", init=False)
m.load_params(p); m.set_fused_w1_adam(False)
ema = O.make_ema(cfg); adam = O.AdamState(cfg, p)
for step in range(3):
    batch = synth_batch(D, BS, NEG, seed=2000 + step, mean_nnz=32)
    cache, ema = O.forward(cfg, p, ema, batch.as_dict(), True, np.float64)
    g = O.backward(cfg, p, cache, np.float64)
    m.set_batch(batch); m.forward(True); m.backward(); torch.cuda.synchronize()
    gg = {k: v.cpu().numpy().copy() for k, v in m.named_grads().items()}
    pre = {k: v.cpu().numpy().copy() for k, v in m.named_params().items()}
    for k in ("W1", "W2", "bn1_q_gamma", "bn2_d_gamma"):
        ref, got = g[k], gg[k]
        well = np.abs(ref) > 1e-4 * np.abs(ref).max()
        rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30)
        i = np.argmax(np.where(well, rel, 0))
        print(f"step{step} {k}: max|g|={np.abs(ref).max():.3e} worst well rel={rel.flat[i]:.3e} at {np.unravel_index(i, ref.shape)} ref={ref.flat[i]:.4e} got={got.flat[i]:.4e}  n_rel>1e-3={(well & (rel>1e-3)).sum()}")
    dparam = {k: np.abs(pre[k] - p[k]).max() for k in ("W1", "W2")}
    print(f"step{step} pre-update param maxdiff {dparam}")
    adam.step(p, g)
    m.apply_adam(1.0); torch.cuda.synchronize()
    # resync biases
    views = m.named_params()
    for l in (1, 2):
        views[f"b{l}"].copy_(torch.from_numpy(p[f"b{l}"]))
    post = {k: v.cpu().numpy() for k, v in m.named_params().items()}
    d = np.abs(post["W1"] - p["W1"]); i = np.argmax(d)
    print(f"step{step} post W1 maxdiff {d.max():.3e} at {np.unravel_index(i, d.shape)} m_gpu={m.adam_m[i].item():.4e} m_ref={adam.m['W1'].flat[i]:.4e} v_gpu={m.adam_v[i].item():.4e} v_ref={adam.v['W1'].flat[i]:.4e}")
