"""Where the Adam launch's time goes at the C2 shape: probe averages (HIP events around the
launches) for the default fused step, heavy columns outside Adam, the unfused optimizer pass, and
near-empty batches (the streaming floor).  Run on the GPU box: python tools/adam_split.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from dssm_amd import _lib
from dssm_amd.data import ZipfColumns, synth_batch
from dssm_amd.model import DSSM

D, W, BS, NEG = 30000, (300, 300, 128), 1024, 4
zipf = ZipfColumns(D)
full = synth_batch(D, BS, NEG, seed=1000, cols=zipf)
tiny = synth_batch(D, BS, NEG, seed=1000, cols=zipf, mean_nnz=1.0, lo=1, hi=2)
CASES = [
    ("default", full, {}),
    ("heavy outside adam", full, {"HEAVY_IN_ADAM": False}),
    ("unfused (dw1 materialised)", full, {"FUSED_W1_ADAM": False}),
    ("default, 1 nnz/row", tiny, {}),
    ("unfused, 1 nnz/row", tiny, {"FUSED_W1_ADAM": False}),
]
for name, b, opts in CASES:
    m = DSSM(D, W, BS, NEG, dtype="bf16")
    for k, v in opts.items():
        m.set_option(k, v)
    m.set_batch(b)
    for _ in range(3):
        m.train_step()
    torch.cuda.synchronize()
    for p in (_lib.PROBE_ADAM, _lib.PROBE_DW1, _lib.PROBE_SPMM_FWD, _lib.PROBE_CSC):
        m.probe_enable(p, 50)
    for _ in range(20):
        m.train_step()
    torch.cuda.synchronize()
    out = []
    for nm, p in (("adam", _lib.PROBE_ADAM), ("dw1", _lib.PROBE_DW1), ("spmm", _lib.PROBE_SPMM_FWD),
                  ("csc", _lib.PROBE_CSC)):
        t, n = m.probe_read(p)
        out.append(f"{nm} {1e3 * t / max(n, 1):6.1f} us")
    print(f"{name:30s} nnz={b.nnz:7d} " + "  ".join(out), flush=True)
    del m
