"""Diagnostics: dssm_dense_bwd_ex (dA + split-K dW of one dense layer) in isolation at the multi-view
tower's FC2 shape (BS rows, 300 -> 128, bf16 operands, bf16 dA masked by the bf16 activation), to
separate the kernels' own duration from the two-stream step's sharing.  Run under
rocprofv3 --kernel-trace --stats for the per-kernel split.
Usage: python tools/dense_bwd_bench.py [rows] [K] [N]"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from dssm_amd import _lib  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    lib = _lib.load()
    dev = torch.device("cuda:0")
    ldk = (K + 7) // 8 * 8
    g = torch.Generator().manual_seed(0)
    bf = torch.bfloat16
    A = torch.rand(M, ldk, generator=g).to(bf).to(dev)
    W = (torch.rand(ldk, N, generator=g) - 0.5).to(bf).to(dev)
    dZ = (torch.rand(M, N, generator=g) - 0.5).to(bf).to(dev)
    dA = torch.empty(M, ldk, dtype=bf, device=dev)
    dWb = torch.zeros(K + 1, N, device=dev)
    nslab = int(lib.dssm_dense_bwd_slab_floats(M, K, N, 1))
    slab = torch.zeros(max(1, nslab), device=dev)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731

    def call():
        rc = lib.dssm_dense_bwd_ex(P(A), ldk, P(W), N, 1, M, K, N, P(dZ), N, P(dA), 1, ldk, P(A), 1, ldk, P(dWb),
                                   P(slab), None, s)
        assert rc == 0, rc

    for _ in range(10):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 200
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    print(f"dense_bwd_ex M={M} K={K} N={N}: {1e3 * e0.elapsed_time(e1) / reps:.2f} us per call "
          f"(dA + dW{' + split reduce' if nslab else ''})", flush=True)


if __name__ == "__main__":
    main()
