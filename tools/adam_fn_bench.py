"""Time dssm_spmm_bwd_w_adam's optimizer launch alone (HIP-event probe) at a given batch shape, to
compare the functional fused optimizer with the plan's (bench.py kernels_ms.adam).
Usage: python tools/adam_fn_bench.py [rows] [nnz_per_row] [D] [n] [reps]"""
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dssm_amd import _lib  # noqa: E402
from dssm_amd._lib import check, ptr  # noqa: E402
from dssm_amd.data import ZipfColumns, synth_rows  # noqa: E402


def main(rows=6144, nnz=32.0, D=30000, n=300, reps=50):
    rows, D, n, reps, nnz = int(rows), int(D), int(n), int(reps), float(nnz)
    lib = _lib.load()
    rng = np.random.Generator(np.random.PCG64(3))
    ip, ix, vv = synth_rows(rng, ZipfColumns(D), rows, nnz)
    ld = -(-n // 8) * 8
    w1 = (D + 1) * n
    rb = -(-w1 // 64) * 64
    n2 = 128
    re = rb + -(-((n + 1) * n2) // 64) * 64
    t = [torch.from_numpy(x).cuda() for x in (ip, ix, vv)]
    dz = (torch.randn(rows, ld, device="cuda") * 0.01).to(torch.bfloat16)
    p = torch.randn(re, device="cuda") * 0.01
    g, m, v = (torch.zeros(re, device="cuda") for _ in range(3))
    g[rb:] = torch.randn(re - rb, device="cuda")
    st = torch.tensor([0.9, 0.999], device="cuda")
    tk = torch.zeros(int(lib.dssm_adam_tickets_bytes(1)), dtype=torch.uint8, device="cuda")
    ws = torch.zeros(int(lib.dssm_spmm_bwd_ws_bytes(rows, D, int(ip[-1]))), dtype=torch.uint8, device="cuda")
    sh1 = torch.zeros((D, ld), dtype=torch.bfloat16, device="cuda")
    sh2 = torch.zeros((n, n2), dtype=torch.bfloat16, device="cuda")
    seg = (_lib.dssm_shadow_seg * 1)(_lib.dssm_shadow_seg(rb, n, n2, n2, sh2.data_ptr()))

    def call():
        check(lib.dssm_spmm_bwd_w_adam(ptr(t[0]), ptr(t[1]), ptr(t[2]), rows, D, int(ip[-1]), ptr(dz), _lib.DSSM_BF16,
                                       ld, n, ptr(p), ptr(g), ptr(m), ptr(v), rb, re, None, 0, 0, ptr(sh1), ld, seg, 1,
                                       0.01, 0.9, 0.999, 1e-8, ptr(st), 1.0, 1, 0, ptr(tk), 1, ptr(ws),
                                       _lib.stream_ptr()), "adam")
    for _ in range(5):
        call()
    torch.cuda.synchronize()
    lib.dssm_adam_probe(reps)
    for _ in range(reps):
        call()
    torch.cuda.synchronize()
    avg, cnt = C.c_double(), C.c_int()
    check(lib.dssm_adam_probe_read(C.byref(avg), C.byref(cnt)), "probe")
    lib.dssm_adam_probe(0)
    touched = int((np.bincount(ix, minlength=D) > 0).sum())
    print(f"rows {rows} nnz {int(ip[-1])} D {D} n {n}: adam {avg.value * 1e3:.2f} us over {cnt.value}, "
          f"touched rows {touched / D:.3f}", flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
