"""Diagnostics: where the bf16 timed path departs from the bf16-emulating oracle (per-row error
quantiles per layer; flips of a bf16 rounding show up as a few rows with large errors)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from dssm_amd import _lib
from dssm_amd.data import synth_batch
from dssm_amd.model import DSSM
from oracle import dssm_oracle as O

case = (30000, (300, 300, 128), 1024, 4) if len(sys.argv) < 2 else eval(sys.argv[1])
D, widths, BS, NEG = case
cfg = O.OracleConfig(D, list(widths), BS, NEG)
p = O.init_params(cfg, 11)
b = synth_batch(D, BS, NEG, seed=1000)
cache, _ = O.forward(cfg, p, O.make_ema(cfg), b.as_dict(), True, np.float64, emulate="bf16")
grads = O.backward(cfg, p, cache)
m = DSSM(D, widths, BS, NEG, dtype="bf16", init=False)
m.load_params(p)
m.set_fused_w1_adam(False)
print("schedule", m.schedule())
m.set_batch(b)
m.forward(True)
m.backward()
torch.cuda.synchronize()
q = [0.5, 0.9, 0.99, 0.999, 1.0]
for l, n in enumerate(widths):
    ld = (n + 7) // 8 * 8
    z = m.buffer(_lib.BUF_Z, l).cpu().numpy().reshape(-1, ld)[:, :n]
    zr = cache["layers"][l]["Z"]
    e = np.abs(z - zr).max(1) / np.abs(zr).max(1)
    print(f"Z{l+1} row rel err quantiles", np.quantile(e, q), "rows>1e-5:", int((e > 1e-5).sum()))
y = m.fetch("embedding_all")
yr = cache["layers"][-1]["A"]
e = np.abs(y - yr).max(1) / (np.abs(yr).max(1) + 1e-30)
print("emb row rel err quantiles", np.quantile(e, q), "rows>1e-4:", int((e > 1e-4).sum()))
c = np.abs(m.fetch("cos_sim_raw").ravel() - cache["cos_sim_raw"])
print("cos abs err quantiles", np.quantile(c, q))
print("loss", m.loss_accuracy()[0], cache["loss"])
gg = {k: v.cpu().numpy() for k, v in m.named_grads().items()}
for k in ("W1", "W2", "W3"):
    g = grads[k]
    e = np.abs(gg[k] - g) / np.abs(g).max()
    print(k, "grad err quantiles", np.quantile(e, q))
