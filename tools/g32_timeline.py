"""Per-workgroup phase timeline of the fp32 parity mode's GEMM tiles (csrc/g32.h; diagnostics build).

On the GPU box:  DSSM_EXTRA_CFLAGS=-DDSSM_G32_TL DSSM_BUILD_TAG=_g32tl python -m dssm_amd.build &&
                 DSSM_LIB_PATH=dssm_amd/libdssm_g32tl.so python tools/g32_timeline.py
Slots: 0 = forward N=300 (layer 2), 1 = forward N=128 (layer 3), 2 = dA K=128 (layer 3),
3 = dA K=300 (layer 2).  Stamps of wave 0 (s_memrealtime, 100 MHz): start, prologue done, per chunk
c staged (after its barrier) and MFMAs issued, epilogue done."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from dssm_amd import _lib
from dssm_amd.data import ZipfColumns, synth_batch
from dssm_amd.model import DSSM

D, W, BS, NEG = 30000, (300, 300, 128), 1024, 4
m = DSSM(D, W, BS, NEG, dtype="fp32")
m.set_batch(synth_batch(D, BS, NEG, seed=1000, cols=ZipfColumns(D)))
for _ in range(5):
    m.train_step()
torch.cuda.synchronize()
f = _lib.load().dssm_debug_g32_timeline
f.restype = C.c_int
f.argtypes = [C.c_int, C.c_void_p, C.c_int]
for slot, (name, nch) in enumerate((("fwd L2 (N=300, K=300)", 10), ("fwd L3 (N=128, K=300)", 10),
                                    ("dA L3 (N=300, K=128)", 4), ("dA L2 (N=300, K=300)", 10))):
    buf = np.zeros((2048, 32), np.uint64)
    assert f(slot, buf.ctypes.data, 2048) == 0
    n = int(np.sum(buf[:, 0] > 0))
    t = buf[:n].astype(np.int64)
    t0 = t[:, 0].min()
    rel = (t - t[:, :1]) * 0.01  # us from the workgroup's start
    st = (t[:, 0] - t0) * 0.01
    end = rel[:, 30]
    print(f"{name}: {n} WGs, span {(st + end).max():.2f} us, start spread {st.max():.2f}, "
          f"WG duration median {np.median(end):.2f} max {end.max():.2f}")
    clk = (t[:, 29] - t[:, 28]) / np.maximum(t[:, 30] - t[:, 0], 1) * 0.1  # s_memtime cycles / 10 ns ticks
    print(f"  shader clock over the WG (s_memtime / s_memrealtime): median {np.median(clk):.2f} GHz")
    print(f"  prologue {np.median(rel[:, 1]):.2f}; per chunk (staged / MFMA done) medians: " +
          " ".join(f"{np.median(rel[:, 2 + 2 * c]):.2f}/{np.median(rel[:, 3 + 2 * c]):.2f}" for c in range(nch)))
