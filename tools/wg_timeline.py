"""Per-workgroup start/end timeline of the dense GEMM launches (diagnostics build only).

On the GPU box:  DSSM_EXTRA_CFLAGS=-DDSSM_WG_TL python -m dssm_amd.build --force &&
                 python tools/wg_timeline.py
Slots: 0 = forward NT GEMM N=300 (layer 2), 1 = forward NT GEMM N=128 (layer 3),
2 = backward pair of layer 3 (dA K=128), 3 = backward pair of layer 2 (K=300)."""
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
m = DSSM(D, W, BS, NEG, dtype="bf16")
b = synth_batch(D, BS, NEG, seed=1000, cols=ZipfColumns(D))
batch = b
m.set_batch(b)
for _ in range(5):
    m.train_step()
torch.cuda.synchronize()
lib = _lib.load()
f = lib.dssm_debug_wg_timeline
f.restype = C.c_int
f.argtypes = [C.c_int, C.c_void_p, C.c_int]
grids = {0: 5 * 48, 1: 2 * 48, 2: None, 3: None}
for slot, name in enumerate(("nt L2 (N=300)", "nt L3 (N=128)", "pair L3", "pair L2")):
    buf = np.zeros((2048, 6), np.uint64)
    assert f(slot, buf.ctypes.data, 2048) == 0
    n = int(np.sum(buf[:, 0] > 0))
    if n == 0:
        print(f"{name}: no stamps")
        continue
    t = buf[:n].astype(np.int64)
    ph = t[:, 2:6]
    if (ph > 0).all():  # phase stamps (tiles only; the materialising block has none)
        rel = (ph - t[:, :1]) * 0.01
        tiles = (t[:, 2] > 0)
        print(f"{name}: phase medians from WG start (us): operands landed {np.median(rel[:, 0]):.2f}, "
              f"LDS images {np.median(rel[:, 1]):.2f}, MFMA done {np.median(rel[:, 2]):.2f}, "
              f"stats published {np.median(rel[:, 3]):.2f}, end {np.median((t[:, 1] - t[:, 0]) * 0.01):.2f}")
    else:
        ok = t[:, 2] > 0
        if ok.any():
            rel = (t[ok][:, 2:6] - t[ok][:, :1]) * 0.01
            print(f"{name}: phase medians over {int(ok.sum())} tiles (us): operands landed {np.median(rel[:, 0]):.2f}, "
                  f"LDS images {np.median(rel[:, 1]):.2f}, MFMA done {np.median(rel[:, 2]):.2f}, "
                  f"stats published {np.median(rel[:, 3]):.2f}, end {np.median((t[ok][:, 1] - t[ok][:, 0]) * 0.01):.2f}")
    t = t[:, :2]
    t0 = t[:, 0].min()
    st, en = (t[:, 0] - t0) * 0.01, (t[:, 1] - t0) * 0.01
    dur = en - st
    print(f"{name}: {n} WGs, span {en.max():.2f} us; start spread {st.max():.2f} us; "
          f"WG duration min/median/max {dur.min():.2f}/{np.median(dur):.2f}/{dur.max():.2f} us; "
          f"last end {en.max():.2f}")
    order = np.argsort(st)
    print("   starts (us, by start order, every 16th):", " ".join(f"{x:.1f}" for x in st[order][::16]))
    print("   ends   (us, same WGs):                ", " ".join(f"{x:.1f}" for x in en[order][::16]))

# k_adam_step: roles by block index (heavy items, W1 rows, flat/dense streaming), as
# k_adam_step assigns them
g = lib.dssm_debug_adam_timeline
g.restype = C.c_int
g.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros((8192, 2), np.uint64)
assert g(buf.ctypes.data, 8192) == 0
n = int(np.sum(buf[:, 0] > 0))
t = buf[:n].astype(np.int64)
t0 = t[:, 0].min()
st, en = (t[:, 0] - t0) * 0.01, (t[:, 1] - t0) * 0.01
items, w1 = 512, 2048  # kAdamItemBlocks, kAdamW1Blocks: roles contiguous in block order
b = np.arange(n, dtype=np.int64)
heavy = b < items
w1r = (b >= items) & (b < items + w1)
for name, sel in (("heavy items", heavy), ("W1 rows", w1r), ("flat/dense", ~heavy & ~w1r)):
    if not sel.any():
        continue
    d = en[sel] - st[sel]
    print(f"adam {name}: blocks {int(sel.sum())}, start {st[sel].min():.1f}..{st[sel].max():.1f} us, "
          f"end {en[sel].min():.1f}..{en[sel].max():.1f} us, duration median {np.median(d):.2f} max {d.max():.2f}")
print(f"adam span {en.max():.1f} us over {n} blocks")
hist = np.histogram(en, bins=12)[0]
print("  block ends histogram (12 bins over the span):", hist.tolist())

# SpMM row waves: duration against the row's nnz
h = lib.dssm_debug_spmm_timeline
h.restype = C.c_int
h.argtypes = [C.c_void_p, C.c_int]
R = m.rows if hasattr(m, "rows") else 6144
buf = np.zeros((R, 2), np.uint64)
assert h(buf.ctypes.data, R) == 0
t = buf.astype(np.int64)
t0 = t[:, 0].min()
st, en = (t[:, 0] - t0) * 0.01, (t[:, 1] - t0) * 0.01
nnz = np.diff(batch.indptr)[:R]
d = en - st
print(f"spmm rows: span {en.max():.1f} us; start spread {st.max():.1f}; wave duration median {np.median(d):.2f} "
      f"max {d.max():.2f}; nnz median {np.median(nnz)} max {nnz.max()}")
for lo, hi in ((0, 24), (24, 32), (32, 40), (40, 48), (48, 200)):
    sel = (nnz >= lo) & (nnz < hi)
    if sel.any():
        print(f"   nnz [{lo},{hi}): {int(sel.sum())} rows, duration median {np.median(d[sel]):.2f} max {d[sel].max():.2f}, "
              f"end median {np.median(en[sel]):.2f} max {en[sel].max():.2f}")
hist = np.histogram(st, bins=10)[0]
print("   wave starts histogram (10 bins):", hist.tolist(), f"over {st.max():.1f} us")
late = np.where(st > 2.0)[0]
if late.size:
    print(f"   late-starting rows: {late.size}, rows {late.min()}..{late.max()}, "
          f"blocks {sorted(set((late // 4).tolist()))[:40]}")
print("   duration percentiles 50/90/99/max:", [round(float(np.percentile(d, q)), 2) for q in (50, 90, 99, 100)])
blk = np.arange(R) // 4
for name, key in (("xcd (block % 8)", blk % 8), ("block // 256", blk // 256)):
    print(f"   by {name}:", " ".join(f"{int(k)}:{np.median(d[key == k]):.1f}/{np.percentile(d[key == k], 99):.1f}"
                                      for k in np.unique(key)))
slow = np.argsort(d)[-12:]
print("   slowest rows:", [(int(r), int(nnz[r]), round(float(st[r]), 1), round(float(d[r]), 1)) for r in slow])

# fused cosine launch: query blocks, then the materialising block, then the CSC scatter blocks
h = lib.dssm_debug_cos_timeline
h.restype = C.c_int
h.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros((1024, 8), np.uint64)
assert h(buf.ctypes.data, 1024) == 0
n = int(np.sum(buf[:, 0] > 0))
t = buf[:n].astype(np.int64)
nq0 = BS // 16
ph = (t[:nq0, 2:7] - t[:nq0, :1]) * 0.01
print("cosine query-block phase medians from start (us): rows landed %.2f, coefficients %.2f, forward %.2f, "
      "backward %.2f, statistics %.2f, end %.2f" % tuple(list(np.median(ph, axis=0)) + [np.median((t[:nq0, 1] - t[:nq0, 0]) * 0.01)]))
t = t[:, :2]
t0 = t[:, 0].min()
st, en = (t[:, 0] - t0) * 0.01, (t[:, 1] - t0) * 0.01
nq = BS // 16
for name, sel in (("query blocks", slice(0, nq)), ("materialise", slice(nq, nq + 1)), ("scatter blocks", slice(nq + 1, n))):
    d = en[sel] - st[sel]
    if d.size:
        print(f"cosine {name}: {d.size} blocks, start {st[sel].min():.1f}..{st[sel].max():.1f}, end "
              f"{en[sel].min():.1f}..{en[sel].max():.1f} us, duration median {np.median(d):.2f} max {d.max():.2f}")

# the two bf16 BN-backward apply launches (bn.hip, g_apply_tl): dW tile blocks vs element blocks
fa = getattr(lib, "dssm_debug_apply_timeline", None)
if fa is not None:
    fa.restype = C.c_int
    fa.argtypes = [C.c_int, C.c_void_p, C.c_int]
    for slot, name in enumerate(("apply hosting dW3 (N=128)", "apply (other)")):
        buf = np.zeros((2048, 4), np.uint64)
        assert fa(slot, buf.ctypes.data, 2048) == 0
        ok = buf[:, 0] > 0
        if not ok.any():
            print(f"{name}: no stamps")
            continue
        t = buf[ok].astype(np.int64)
        t0 = t[:, 0].min()
        st, en = (t[:, 0] - t0) * 0.01, (t[:, 1] - t0) * 0.01
        print(f"{name}: {int(ok.sum())} WGs, span {en.max():.2f} us")
        for role, rn in enumerate(("dW tiles", "second dW set", "element blocks", "extra block")):
            m = t[:, 2] == role
            if not m.any():
                continue
            d = en[m] - st[m]
            line = (f"   {rn}: {int(m.sum())} WGs, start {st[m].min():.2f}..{st[m].max():.2f}, end "
                    f"{np.median(en[m]):.2f} median / {en[m].max():.2f} max, duration median {np.median(d):.2f} max {d.max():.2f}")
            if role == 2:
                pro = (t[m][:, 3] - t[m][:, 0]) * 0.01
                line += f"; prologue median {np.median(pro):.2f} max {pro.max():.2f}"
            print(line)
