"""Diagnostics (GPU box): which W1 rows of the multi-view item tower disagree with the oracle at
config-5 size, their CSC entry counts, and whether repeated backward passes agree."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_multiview_c5 import _setup  # noqa: E402
from oracle import multiview_oracle as M  # noqa: E402

view = int(sys.argv[1]) if len(sys.argv) > 1 else 1
cfg, p, rot, m, u, it = _setup(view)
fw = M.forward(cfg, p, u, it, view, rot, dtype=np.float64, sparse=True)
g = M.backward(cfg, p, fw)
counts = np.bincount(it[1], minlength=cfg.view_d[view - 1])
for rep in range(3):
    m.grads.zero_()
    m.forward()
    m.backward()
    torch.cuda.synchronize()
    got = m.named(m.grads)
    for k in (f"view{view}_W1", f"view{view}_b1", "user_W1"):
        ref = g[k]
        e = np.abs(got[k] - ref)
        if e.ndim == 1:
            print(rep, k, "max err", e.max() / np.abs(ref).max(), "argmax", e.argmax(), flush=True)
            continue
        rows = np.where(e.max(1) > 1e-5 * np.abs(ref).max())[0]
        print(rep, k, "bad rows", rows.size, "max rel", e.max() / np.abs(ref).max(), flush=True)
        if rows.size:
            print("   rows", rows[:20], "counts", counts[rows[:20]] if k.startswith("view") else "", flush=True)
            r0 = rows[0]
            cols = np.where(e[r0] > 1e-5 * np.abs(ref).max())[0]
            print("   row", r0, "bad cols", cols.size, cols[:16], "got", got[k][r0, cols[:4]], "ref", ref[r0, cols[:4]])
    if rep == 0:
        # heavy columns: entries > 64
        print("heavy cols", int((counts > 64).sum()), "max count", int(counts.max()), "nnz", int(counts.sum()))
