"""Diagnostics: the deterministic mode's CSC row sort (spmm.hip k_csc_sort_rows) timed alone on the
bench's C2 batch: dssm_csc_transpose with row_order 1 minus row_order 0, HIP events around each
call, averaged.  Side builds of the sort with parts skipped (DSSM_SORT_DIAG, wrong results) are
loaded through DSSM_LIB_PATH.
    DSSM_LIB_PATH=dssm_amd/libdssm<tag>.so python3 tools/sort_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from dssm_amd import _lib
from dssm_amd._lib import check, ptr
from dssm_amd.data import ZipfColumns, synth_batch

D, BS, NEG = 30000, 1024, 4
lib = _lib.load()
b = synth_batch(D, BS, NEG, seed=1000, cols=ZipfColumns(D))
rows, max_nnz = b.rows, b.nnz
ws = torch.zeros(lib.dssm_spmm_bwd_ws_bytes(rows, D, max_nnz), dtype=torch.uint8, device="cuda")
t = [torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values)]
ent = max_nnz + rows
cp = torch.zeros(D + 2, dtype=torch.int32, device="cuda")
cr, cc = (torch.zeros(ent, dtype=torch.int32, device="cuda") for _ in range(2))
cv = torch.zeros(ent, dtype=torch.float32, device="cuda")


def call(order):
    check(lib.dssm_csc_transpose(ptr(t[0]), ptr(t[1]), ptr(t[2]), rows, D, max_nnz, order, ptr(cp), ptr(cr),
                                 ptr(cv), ptr(cc), ptr(ws), _lib.stream_ptr()), "csc_transpose")


out = {}
for order in (0, 1, 0, 1):
    for _ in range(5):
        call(order)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(50):
        call(order)
    ev[1].record()
    torch.cuda.synchronize()
    out.setdefault(order, []).append(ev[0].elapsed_time(ev[1]) / 50 * 1e3)
print(f"{os.path.basename(_lib.LIB_PATH)}: transpose {min(out[0]):.2f} us, with the row sort {min(out[1]):.2f} us, "
      f"sort {min(out[1]) - min(out[0]):.2f} us")
