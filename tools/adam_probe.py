"""Adam kernel time with the fused W1 rows vs the flat (unfused) optimizer pass, C2 shape.
Run on the GPU box: python tools/adam_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from dssm_amd import _lib
from dssm_amd.data import ZipfColumns, synth_batch
from dssm_amd.model import DSSM

D, W, BS, NEG = 30000, (300, 300, 128), 1024, 4
b = synth_batch(D, BS, NEG, seed=1000, cols=ZipfColumns(D))
for fused in (True, False):
    m = DSSM(D, W, BS, NEG, dtype="bf16")
    m.set_fused_w1_adam(fused)
    m.set_batch(b)
    for _ in range(3):
        m.train_step()
    torch.cuda.synchronize()
    m.probe_enable(_lib.PROBE_ADAM, 50)
    m.probe_enable(_lib.PROBE_DW1, 50)
    for _ in range(20):
        m.train_step()
    torch.cuda.synchronize()
    ta, na = m.probe_read(_lib.PROBE_ADAM)
    td, nd = m.probe_read(_lib.PROBE_DW1)
    print(f"fused={fused}: adam {1e3 * ta / max(na, 1):.1f} us, dw1 {1e3 * td / max(nd, 1):.1f} us")
