"""Diagnostics: time the XCD-sliced FC1 SpMM prototype (tools/proto/spmm_slice.hip) against the
library's row-major bf16 SpMM (dssm_spmm_csr_fwd) on the bench's batch shape, and check the outputs
are bit-identical (same per-element FMA order)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from dssm_amd import _lib  # noqa: E402
from dssm_amd.data import synth_batch  # noqa: E402

D, N, LD, BS, NEG = 30000, 300, 304, 1024, 4
SW, NS = 40, 8


def main():
    lib = _lib.load()
    pl = C.CDLL(os.path.join(os.path.dirname(__file__), "libspmm_slice.so"))
    dev = torch.device("cuda:0")
    b = synth_batch(D, BS, NEG, seed=1000)
    ip = torch.from_numpy(b.indptr.astype(np.int32)).to(dev)
    ix = torch.from_numpy(b.indices.astype(np.int32)).to(dev)
    vv = torch.from_numpy(b.values.astype(np.float32)).to(dev)
    R = b.rows
    g = torch.Generator().manual_seed(0)
    w = (torch.rand(D, N, generator=g) * 0.2 - 0.1).to(torch.bfloat16)
    wpad = torch.zeros(D, LD, dtype=torch.bfloat16)
    wpad[:, :N] = w
    wsl = torch.zeros(NS, D, SW, dtype=torch.bfloat16)
    for x in range(NS):
        c0, c1 = x * SW, min(N, (x + 1) * SW)
        if c1 > c0:
            wsl[x, :, :c1 - c0] = w[:, c0:c1]
    wpad = wpad.to(dev)
    wsl = wsl.to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    z0 = torch.zeros(R, LD, device=dev)
    z1 = torch.full((R, LD), 7.0, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731

    def base():
        rc = lib.dssm_spmm_csr_fwd(P(ip), P(ix), P(vv), R, P(wpad), 1, LD, N, P(bias), P(z0), LD, C.c_void_p(s))
        assert rc == 0, rc

    def sliced(u, xsel):
        def f():
            rc = pl.proto_spmm_sliced(P(ip), P(ix), P(vv), R, P(wsl), D, N, P(bias), P(z1), LD, u, xsel, C.c_void_p(s))
            assert rc == 0, rc
        return f

    base()
    sliced(8, 0)()
    torch.cuda.synchronize()
    same = torch.equal(z0, z1)
    print("nnz", int(b.indptr[-1]), "rows", R, "bit-identical", same, "max abs diff", float((z0 - z1).abs().max()))

    def t(fn, reps=200):
        for _ in range(10):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return 1e3 * e0.elapsed_time(e1) / reps

    # interleave the variants twice; with a 256 MB write in between to evict the caches (cold) or not
    junk = torch.empty(64 * 1024 * 1024, device=dev)
    for rnd in range(2):
        for name, fn in [("row-major (library)", base), ("sliced U=8", sliced(8, 0)), ("sliced U=4", sliced(4, 0)),
                         ("sliced U=8, slices spread (control)", sliced(8, 1))]:
            warm = t(fn)

            def cold():
                junk.fill_(1.0)
                fn()
            c = t(cold, 50) - t(lambda: junk.fill_(1.0), 50)
            print(f"[{rnd}] {name:40s} back-to-back {warm:7.2f} us   after a 256 MB write {c:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
