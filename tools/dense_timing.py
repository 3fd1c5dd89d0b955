"""Phase timeline of the persistent dense kernels (block 0's s_memrealtime stamps, 100 MHz).
Run on the GPU box: DSSM_DENSE_TIMING=1 python tools/dense_timing.py"""
import os
import sys

os.environ.setdefault("DSSM_DENSE_TIMING", "1")
os.environ.setdefault("DSSM_DENSE", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from dssm_amd import _lib
from dssm_amd.data import ZipfColumns, synth_batch
from dssm_amd.model import DSSM

D, W, BS, NEG = 30000, (300, 300, 128), 1024, 4
m = DSSM(D, W, BS, NEG, dtype="bf16")
b = synth_batch(D, BS, NEG, seed=1000, cols=ZipfColumns(D))
m.set_batch(b)
for _ in range(5):
    m.train_step()
m.check()
print("dense grid:", m.lib.dssm_plan_dense_enabled(m._plan))
t = m.buffer(_lib.BUF_DENSE_TIMING, dtype=torch.int64).cpu().numpy().reshape(4, 64)
for k, name in enumerate(("fwd | pair_l2 tn tile", "bwd", "fwd_item0 | pair_l2 dA tile", "nt_l2_tile")):
    row = t[k]
    n = int(np.argmax(row == 0)) if np.any(row == 0) else 64
    st = row[:n].astype(np.int64)
    if st.size < 2:
        continue
    d = np.diff(st) * 0.01  # us
    print(name, "total %.1f us" % ((st[-1] - st[0]) * 0.01))
    print("  segments (us): " + " ".join("%.1f" % x for x in d))
