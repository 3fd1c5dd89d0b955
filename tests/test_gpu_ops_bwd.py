"""Functional backward entry points of include/dssm.h against float64 NumPy of the
same inputs: dssm_spmm_csr_bwd_w ([X|1]^T dZ, dense, fp32 and bf16 dZ), dssm_dense_bwd (dZ W^T,
[A|1]^T dZ), dssm_bn_relu_bwd (the oracle's batch-stat BN + ReLU backward formula), dssm_adam_step
(TF1.x ApplyAdam).  Tolerances: fp32 1e-5 relative to the output scale; bf16 inputs 1e-2."""
import ctypes as C

import numpy as np
import pytest
import torch

from dssm_amd import _lib
from dssm_amd._lib import check, ptr
from dssm_amd.data import ZipfColumns, synth_rows

pytestmark = pytest.mark.gpu


def _close(got, ref, tol):
    scale = max(np.abs(ref).max(), 1e-30)
    assert np.abs(got - ref).max() <= tol * scale, (np.abs(got - ref).max(), scale)


@pytest.mark.parametrize("D,rows,n,dt", [(5000, 768, 300, "fp32"), (30000, 1536, 304, "bf16"), (700, 64, 64, "fp32")])
def test_spmm_csr_bwd_w(D, rows, n, dt):
    lib = _lib.load()
    rng = np.random.Generator(np.random.PCG64(1))
    ip, ix, vv = synth_rows(rng, ZipfColumns(D), rows, 24.0)
    dZ = rng.standard_normal((rows, n)).astype(np.float32)
    ldz = -(-n // 8) * 8
    dZp = np.zeros((rows, ldz), np.float32)
    dZp[:, :n] = dZ
    tdz = torch.from_numpy(dZp).cuda()
    if dt == "bf16":
        tdz = tdz.to(torch.bfloat16)
        dZ = tdz.float().cpu().numpy()[:, :n]
    max_nnz = int(ip[-1])
    ws = torch.zeros(lib.dssm_spmm_bwd_ws_bytes(rows, D, max_nnz), dtype=torch.uint8, device="cuda")
    out = torch.zeros((D + 1, n), dtype=torch.float32, device="cuda")
    t = [torch.from_numpy(x).cuda() for x in (ip, ix, vv)]
    for _ in range(2):  # the scratch must be re-armed by the call itself
        check(lib.dssm_spmm_csr_bwd_w(ptr(t[0]), ptr(t[1]), ptr(t[2]), rows, D, max_nnz, ptr(tdz),
                                      _lib.DSSM_BF16 if dt == "bf16" else _lib.DSSM_F32, ldz, n, ptr(out),
                                      ptr(ws), _lib.stream_ptr()), "spmm_bwd")
        torch.cuda.synchronize()
        X = np.zeros((rows, D + 1))
        for r in range(rows):
            X[r, ix[ip[r]:ip[r + 1]]] += vv[ip[r]:ip[r + 1]]
        X[:, D] = 1.0
        _close(out.cpu().numpy(), X.T @ dZ.astype(np.float64), 1e-5)


def _csc_expected(ip, ix, vv, rows, D):
    """[X | 1]^T as CSC with every column in ascending row order (ties: value bits), NumPy."""
    r = np.repeat(np.arange(rows, dtype=np.int64), np.diff(ip))
    c = np.concatenate([ix.astype(np.int64), np.full(rows, D)])
    rr = np.concatenate([r, np.arange(rows)])
    v = np.concatenate([vv, np.ones(rows, np.float32)])
    order = np.lexsort((v.view(np.uint32), rr, c))
    ptr = np.zeros(D + 2, np.int64)
    np.add.at(ptr, c + 1, 1)
    return np.cumsum(ptr), rr[order], v[order], c[order]


@pytest.mark.parametrize("D,rows,dups", [(30000, 6144, False), (5000, 9000, False), (700, 64, False),
                                         (3000, 4096, True)])
@pytest.mark.parametrize("row_order", [1, 0])
def test_csc_transpose(D, rows, dups, row_order):
    """dssm_csc_transpose: row_order 1 (the deterministic mode's wave-per-column row sort, one and two
    8192-row windows) equals NumPy's row-ordered transpose exactly; row_order 0 holds the same
    entries per column.  `dups`: CSR rows repeating a column (a hot one included), the sort's
    (row, value, slot) ranking path."""
    lib = _lib.load()
    rng = np.random.Generator(np.random.PCG64(7))
    ip, ix, vv = synth_rows(rng, ZipfColumns(D), rows, 24.0)
    if dups:  # every 7th row repeats its first column with another value, every 11th column 0 twice
        parts = []
        for r in range(rows):
            cols, vals = list(ix[ip[r]:ip[r + 1]]), list(vv[ip[r]:ip[r + 1]])
            if r % 7 == 0:
                cols.append(cols[0]), vals.append(5.0)
            if r % 11 == 0:
                cols += [0, 0]
                vals += [1.0, 7.0]
            parts.append((cols, vals))
        ip = np.concatenate([[0], np.cumsum([len(c) for c, _ in parts])]).astype(np.int32)
        ix = np.concatenate([c for c, _ in parts]).astype(np.int32)
        vv = np.concatenate([v for _, v in parts]).astype(np.float32)
    max_nnz = int(ip[-1])
    ptr_e, row_e, val_e, col_e = _csc_expected(ip, ix, vv, rows, D)
    ws = torch.zeros(lib.dssm_spmm_bwd_ws_bytes(rows, D, max_nnz), dtype=torch.uint8, device="cuda")
    t = [torch.from_numpy(x).cuda() for x in (ip, ix, vv)]
    ent = max_nnz + rows
    cp = torch.zeros(D + 2, dtype=torch.int32, device="cuda")
    cr, cc = (torch.zeros(ent, dtype=torch.int32, device="cuda") for _ in range(2))
    cv = torch.zeros(ent, dtype=torch.float32, device="cuda")
    for _ in range(2):  # the scratch must be re-armed by the call itself
        check(lib.dssm_csc_transpose(ptr(t[0]), ptr(t[1]), ptr(t[2]), rows, D, max_nnz, row_order, ptr(cp),
                                     ptr(cr), ptr(cv), ptr(cc), ptr(ws), _lib.stream_ptr()), "csc_transpose")
        torch.cuda.synchronize()
        gp, gr, gv, gc = (x.cpu().numpy() for x in (cp, cr, cv, cc))
        assert np.array_equal(gp, ptr_e)
        assert np.array_equal(gc, col_e)
        if row_order:
            assert np.array_equal(gr, row_e) and np.array_equal(gv.view(np.uint32), val_e.view(np.uint32))
        else:
            o = np.lexsort((gv.view(np.uint32), gr, gc))
            assert np.array_equal(gr[o], row_e) and np.array_equal(gv[o], val_e)


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_dense_bwd(dt):
    lib = _lib.load()
    M, K, N = 1536, 300, 128
    rng = np.random.Generator(np.random.PCG64(2))
    A, W, dZ = (rng.standard_normal(s).astype(np.float32) for s in ((M, K), (K, N), (M, N)))
    lda, ldw = -(-K // 8) * 8, -(-N // 8) * 8
    tt = torch.bfloat16 if dt == "bf16" else torch.float32

    def dev(x, ld):
        y = np.zeros((x.shape[0], ld), np.float32)
        y[:, :x.shape[1]] = x
        return torch.from_numpy(y).cuda().to(tt)
    tA, tW, tZ = dev(A, lda), dev(W, ldw), dev(dZ, ldw)
    if dt == "bf16":
        A, W, dZ = (t.float().cpu().numpy()[:, :s] for t, s in ((tA, K), (tW, N), (tZ, N)))
    dtype = _lib.DSSM_BF16 if dt == "bf16" else _lib.DSSM_F32
    slab = torch.zeros(max(1, lib.dssm_dense_bwd_slab_floats(M, K, N, dtype)), device="cuda")
    dA = torch.zeros((M, lda), device="cuda")
    dWb = torch.zeros((K + 1, N), device="cuda")
    check(lib.dssm_dense_bwd(ptr(tA), lda, ptr(tW), ldw, dtype, M, K, N, ptr(tZ), ldw, ptr(dA), lda,
                             ptr(dWb), ptr(slab), _lib.stream_ptr()), "dense_bwd")
    torch.cuda.synchronize()
    tol = 1e-5 if dt == "fp32" else 1e-2
    _close(dA.cpu().numpy()[:, :K], dZ.astype(np.float64) @ W.T.astype(np.float64), tol)
    A1 = np.concatenate([A, np.ones((M, 1), np.float32)], 1).astype(np.float64)
    _close(dWb.cpu().numpy(), A1.T @ dZ.astype(np.float64), tol)


def test_dense_bwd_masked_and_fused_relu_forwards():
    """dssm_dense_bwd_masked (ReluGrad through the layer input fused into dA: exact zeros where the
    mask is <= 0, the plain dA elsewhere, same dW), dssm_dense_fwd_act / dssm_spmm_csr_fwd_act with
    DSSM_ACT_RELU against the unfused entry points + dssm_relu (bit-identical: the same arithmetic
    with the max in the epilogue)."""
    lib = _lib.load()
    M, K, N = 1024, 300, 128
    rng = np.random.Generator(np.random.PCG64(5))
    lda, ldw = 304, 128
    A = torch.zeros((M, lda), device="cuda")
    A[:, :K] = torch.from_numpy(np.maximum(rng.standard_normal((M, K)), 0).astype(np.float32)).cuda()
    W = torch.from_numpy(rng.standard_normal((K + 1, ldw)).astype(np.float32) * 0.1).cuda()
    dZ = torch.from_numpy(rng.standard_normal((M, ldw)).astype(np.float32)).cuda()
    slab = torch.zeros(max(1, lib.dssm_dense_bwd_slab_floats(M, K, N, _lib.DSSM_F32)), device="cuda")
    s = _lib.stream_ptr()
    dA, dWb = torch.zeros((M, lda), device="cuda"), torch.zeros((K + 1, N), device="cuda")
    check(lib.dssm_dense_bwd(ptr(A), lda, ptr(W), ldw, _lib.DSSM_F32, M, K, N, ptr(dZ), ldw, ptr(dA), lda,
                             ptr(dWb), ptr(slab), s), "dense_bwd")
    dAm, dWbm = torch.zeros((M, lda), device="cuda"), torch.zeros((K + 1, N), device="cuda")
    check(lib.dssm_dense_bwd_masked(ptr(A), lda, ptr(W), ldw, _lib.DSSM_F32, M, K, N, ptr(dZ), ldw, ptr(dAm),
                                    lda, ptr(A), lda, ptr(dWbm), ptr(slab), s), "dense_bwd_masked")
    torch.cuda.synchronize()
    assert torch.equal(dWbm, dWb)
    assert torch.equal(dAm[:, :K], torch.where(A[:, :K] > 0, dA[:, :K], torch.zeros_like(dA[:, :K])))
    assert float((A[:, :K] <= 0).float().mean()) > 0.3  # the mask does cut
    # the masked form rejects a mask without dA
    assert lib.dssm_dense_bwd_masked(ptr(A), lda, ptr(W), ldw, _lib.DSSM_F32, M, K, N, ptr(dZ), ldw, None,
                                     lda, ptr(A), lda, ptr(dWbm), ptr(slab), s) != 0
    # forward GEMM + ReLU
    Z, Zr = torch.zeros((M, ldw), device="cuda"), torch.zeros((M, ldw), device="cuda")
    check(lib.dssm_dense_fwd(ptr(A), lda, ptr(W), ldw, _lib.DSSM_F32, M, K, N, ptr(W[K]), ptr(Z), ldw, s), "fwd")
    check(lib.dssm_relu(ptr(Z), ldw, M, N, ptr(Z), ldw, s), "relu")
    check(lib.dssm_dense_fwd_act(ptr(A), lda, ptr(W), ldw, _lib.DSSM_F32, M, K, N, ptr(W[K]), ptr(Zr), ldw,
                                 _lib.DSSM_ACT_RELU, s), "fwd_act")
    torch.cuda.synchronize()
    assert torch.equal(Z, Zr) and float((Zr[:, :N] == 0).float().mean()) > 0.3
    ref = torch.relu(A[:, :K].double() @ W[:K, :N].double() + W[K, :N].double())
    assert float((Zr[:, :N].double() - ref).abs().max()) <= 1e-5 * float(ref.abs().max())
    # sparse FC1 + ReLU
    D, n = 5000, 300
    ip, ix, vv = synth_rows(rng, ZipfColumns(D), M, 24.0)
    t = [torch.from_numpy(x).cuda() for x in (ip, ix, vv)]
    W1 = torch.from_numpy(rng.standard_normal((D + 1, n)).astype(np.float32) * 0.1).cuda()
    Y, Yr = torch.zeros((M, lda), device="cuda"), torch.zeros((M, lda), device="cuda")
    check(lib.dssm_spmm_csr_fwd(ptr(t[0]), ptr(t[1]), ptr(t[2]), M, ptr(W1), _lib.DSSM_F32, n, n, ptr(W1[D]),
                                ptr(Y), lda, s), "spmm")
    check(lib.dssm_relu(ptr(Y), lda, M, n, ptr(Y), lda, s), "relu")
    check(lib.dssm_spmm_csr_fwd_act(ptr(t[0]), ptr(t[1]), ptr(t[2]), M, ptr(W1), _lib.DSSM_F32, n, n,
                                    ptr(W1[D]), ptr(Yr), lda, _lib.DSSM_ACT_RELU, s), "spmm_act")
    torch.cuda.synchronize()
    assert torch.equal(Y[:, :n], Yr[:, :n])
    assert lib.dssm_spmm_csr_fwd_act(ptr(t[0]), ptr(t[1]), ptr(t[2]), M, ptr(W1), _lib.DSSM_F32, n, n,
                                     ptr(W1[D]), ptr(Yr), lda, 7, s) != 0


def test_rows_gather_sum_is_the_scatter_add_inverse():
    """dssm_rows_gather_sum over the inverse of a map == scale x dssm_rows_scatter_add over the map
    (up to summation order), masked by ReluGrad where a mask is given."""
    lib = _lib.load()
    rng = np.random.Generator(np.random.PCG64(9))
    n_src, n, cols, ld = 300, 1500, 128, 128
    mp = rng.integers(0, n_src, n).astype(np.int32)
    order = np.argsort(mp, kind="stable").astype(np.int32)
    offs = np.zeros(n_src + 1, np.int32)
    np.cumsum(np.bincount(mp, minlength=n_src), out=offs[1:])
    src = torch.from_numpy(rng.standard_normal((n, ld)).astype(np.float32)).cuda()
    mask = torch.from_numpy(rng.standard_normal((n_src, ld)).astype(np.float32)).cuda()
    t_map, t_idx, t_off = (torch.from_numpy(x).cuda() for x in (mp, order, offs))
    ref = torch.zeros((n_src, ld), device="cuda")
    s = _lib.stream_ptr()
    check(lib.dssm_rows_scatter_add(ptr(src), ld, ptr(t_map), n, cols, ptr(ref), ld, n_src, s), "scatter_add")
    got, gotm = torch.zeros_like(ref), torch.zeros_like(ref)
    check(lib.dssm_rows_gather_sum(ptr(src), ld, ptr(t_off), ptr(t_idx), n_src, cols, 3.0, None, 0, ptr(got), ld, s),
          "gather_sum")
    check(lib.dssm_rows_gather_sum(ptr(src), ld, ptr(t_off), ptr(t_idx), n_src, cols, 3.0, ptr(mask), ld, ptr(gotm),
                                   ld, s), "gather_sum masked")
    torch.cuda.synchronize()
    torch.testing.assert_close(got, 3.0 * ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gotm, torch.where(mask > 0, 3.0 * ref, torch.zeros_like(ref)), rtol=1e-5, atol=1e-5)
    # a source row no merged row maps to gets exact zeros
    empty = np.flatnonzero(np.bincount(mp, minlength=n_src) == 0)
    if empty.size:
        assert float(got[torch.from_numpy(empty).cuda()].abs().max()) == 0.0


@pytest.mark.parametrize("relu", [1, 0])
def test_bn_relu_bwd(relu):
    lib = _lib.load()
    rows, n, eps = 1000, 100, 1e-3
    rng = np.random.Generator(np.random.PCG64(3))
    Z = (rng.standard_normal((rows, n)) * 2 + 0.5).astype(np.float32)
    g = rng.uniform(0.5, 1.5, n).astype(np.float32)
    b = rng.uniform(-0.3, 0.3, n).astype(np.float32)
    dout = rng.standard_normal((rows, n)).astype(np.float32)
    mu, var = Z.astype(np.float64).mean(0), Z.astype(np.float64).var(0)
    t = {k: torch.from_numpy(np.ascontiguousarray(v, np.float32)).cuda()
         for k, v in dict(Z=Z, g=g, b=b, mu=mu, var=var, d=dout).items()}
    dz = torch.zeros((rows, n), device="cuda")
    dg, db = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    check(lib.dssm_bn_relu_bwd(ptr(t["Z"]), n, rows, n, ptr(t["g"]), ptr(t["b"]), ptr(t["mu"]), ptr(t["var"]),
                               eps, relu, ptr(t["d"]), n, ptr(dz), n, ptr(dg), ptr(db), _lib.stream_ptr()), "bn_bwd")
    torch.cuda.synchronize()
    # float64 reference: y = g xhat + b, out = relu(y)
    Zd = Z.astype(np.float64)
    xh = (Zd - mu) / np.sqrt(var + eps)
    dy = dout.astype(np.float64) * ((g * xh + b > 0) if relu else 1.0)
    ref_db, ref_dg = dy.sum(0), (dy * xh).sum(0)
    ref_dz = g / np.sqrt(var + eps) * (dy - dy.mean(0) - xh * (dy * xh).mean(0))
    _close(db.cpu().numpy(), ref_db, 1e-5)
    _close(dg.cpu().numpy(), ref_dg, 1e-5)
    _close(dz.cpu().numpy(), ref_dz, 1e-4)
    # finite-difference spot check of dz through the full batch-stat BN + ReLU in float64
    def f(Zx):
        m, v = Zx.mean(0), Zx.var(0)
        y = g * (Zx - m) / np.sqrt(v + eps) + b
        return float(((np.maximum(y, 0) if relu else y) * dout).sum())
    for (r, c) in ((3, 7), (500, 42)):
        e = np.zeros_like(Zd)
        e[r, c] = 1e-6
        num = (f(Zd + e) - f(Zd - e)) / 2e-6
        assert abs(num - ref_dz[r, c]) <= 1e-4 * max(1.0, abs(num))


def test_adam_step():
    lib = _lib.load()
    n = 10000
    rng = np.random.Generator(np.random.PCG64(4))
    p0 = rng.standard_normal(n).astype(np.float32)
    g = rng.standard_normal(n).astype(np.float32)
    tp, tg = torch.from_numpy(p0.copy()).cuda(), torch.from_numpy(g).cuda()
    tm, tv = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    st = torch.tensor([0.9, 0.999], device="cuda")
    f = np.float32
    p, m, v, b1p, b2p = p0.copy(), np.zeros(n, f), np.zeros(n, f), f(0.9), f(0.999)
    for _ in range(3):
        check(lib.dssm_adam_step(ptr(tp), ptr(tg), ptr(tm), ptr(tv), n, 0.01, 0.9, 0.999, 1e-8, ptr(st), 0.5, 1,
                                 _lib.stream_ptr()), "adam")
        lr_t = f(0.01) * np.sqrt(f(1) - b2p) / (f(1) - b1p)
        gs = g * f(0.5)
        m = m + (gs - m) * f(1 - 0.9)
        v = v + (gs * gs - v) * f(1 - 0.999)
        p = p - (m * lr_t) / (np.sqrt(v) + f(1e-8))
        b1p, b2p = f(b1p * f(0.9)), f(b2p * f(0.999))
    torch.cuda.synchronize()
    np.testing.assert_allclose(tp.cpu().numpy(), p, rtol=0, atol=1e-6)
    np.testing.assert_allclose(st.cpu().numpy(), [b1p, b2p], rtol=1e-7)


def _adam_ref(p, g, m, v, b1p, b2p, lr=0.01):
    f = np.float32
    lr_t = f(lr) * np.sqrt(f(1) - b2p) / (f(1) - b1p)
    m = m + (g - m) * f(1 - 0.9)
    v = v + (g * g - v) * f(1 - 0.999)
    return p - (m * lr_t) / (np.sqrt(v) + f(1e-8)), m, v


@pytest.mark.parametrize("D,rows,n,dt", [(700, 200, 64, "fp32"), (5000, 768, 300, "bf16"), (30000, 1536, 304, "bf16")])
def test_spmm_bwd_w_adam(D, rows, n, dt):
    """dssm_spmm_bwd_w_adam: two towers (separate arenas, batches and workspaces) on two streams, one
    optimizer step group of 2 sharing the beta powers, 2 steps.  Reference: float32 ApplyAdam on
    [X | 1]^T dZ (float64, then float32) for [W1; b1] and on the sum of 3 split-K partials for the
    rest block.  W1's rows where the gradient is well-conditioned (|g| > 1e-3 max|g|) <= 2e-6, every
    element <= 2 lr; the W1 gradient rows stay zero; bf16 shadows = bf16(p) bit for bit; the beta
    powers advance once per step.  Batches include an empty row, columns past 64 and 256 entries."""
    lib = _lib.load()
    rng = np.random.Generator(np.random.PCG64(11))
    bf = dt == "bf16"
    n2, r2, splits = 32, 20, 3
    w1 = (D + 1) * n
    rb = -(-w1 // 64) * 64
    re = rb + -(-(r2 * n2) // 64) * 64
    ldz = -(-n // 8) * 8
    st = torch.tensor([0.9, 0.999], device="cuda")
    tickets = torch.zeros(int(lib.dssm_adam_tickets_bytes(2)), dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    towers = []
    for k in range(2):
        ip, ix, vv = synth_rows(rng, ZipfColumns(D), rows, 24.0)
        ip = np.concatenate([ip[:3], ip[2:]]).astype(np.int32)[:rows + 1]  # row 2 empty
        ip[-1] = min(ip[-1], len(ix))
        ix, vv = ix[:ip[-1]], vv[:ip[-1]]
        import scipy.sparse as sp
        X = sp.csr_matrix((vv.astype(np.float64), ix, ip), shape=(rows, D + 1)).tolil()
        X[:, D] = 1.0
        X = X.tocsr()
        dZp = np.zeros((rows, ldz), np.float32)
        dZp[:, :n] = rng.standard_normal((rows, n))
        tdz = torch.from_numpy(dZp).cuda()
        if bf:
            tdz = tdz.to(torch.bfloat16)
            dZp = tdz.float().cpu().numpy()
        slab = rng.standard_normal((splits, r2 * n2)).astype(np.float32)
        g1 = np.asarray(X.T @ dZp[:, :n].astype(np.float64)).astype(np.float32).ravel()
        g2 = slab[0] + slab[1] + slab[2]  # the optimizer's fixed split order
        p0 = rng.standard_normal(re).astype(np.float32) * 0.1
        T = dict(ip=ip, ix=ix, vv=vv, g1=g1, g2=g2, p0=p0,
                 t=[torch.from_numpy(x).cuda() for x in (ip, ix, vv)], dz=tdz,
                 slab=torch.from_numpy(slab.ravel()).cuda(), p=torch.from_numpy(p0.copy()).cuda(),
                 g=torch.zeros(re, device="cuda"), m=torch.zeros(re, device="cuda"), v=torch.zeros(re, device="cuda"),
                 ws=torch.zeros(int(lib.dssm_spmm_bwd_ws_bytes(rows, D, int(ip[-1]))), dtype=torch.uint8, device="cuda"),
                 sh1=torch.zeros((D, ldz), dtype=torch.bfloat16, device="cuda"),
                 sh2=torch.zeros((r2 - 1, n2), dtype=torch.bfloat16, device="cuda"))
        cnt = np.bincount(ix, minlength=D)
        assert cnt.max() > (256 if rows >= 768 else 64) and int(ip[3] - ip[2]) == 0
        towers.append(T)
    torch.cuda.synchronize()
    for step in range(2):
        for k, T in enumerate(towers):
            streams[k].wait_stream(streams[0])
            seg = (_lib.dssm_shadow_seg * 1)(_lib.dssm_shadow_seg(rb, r2 - 1, n2, n2, T["sh2"].data_ptr()))
            check(lib.dssm_spmm_bwd_w_adam(ptr(T["t"][0]), ptr(T["t"][1]), ptr(T["t"][2]), rows, D, int(T["ip"][-1]),
                                           ptr(T["dz"]), _lib.DSSM_BF16 if bf else _lib.DSSM_F32, ldz, n,
                                           ptr(T["p"]), ptr(T["g"]), ptr(T["m"]), ptr(T["v"]), rb, re,
                                           ptr(T["slab"]), r2 * n2, splits,
                                           ptr(T["sh1"]) if bf else None, ldz, seg if bf else None, 1 if bf else 0,
                                           0.01, 0.9, 0.999, 1e-8, ptr(st), 1.0, 2, k, ptr(tickets), 1, ptr(T["ws"]),
                                           streams[k].cuda_stream), "spmm_bwd_w_adam")
        streams[0].wait_stream(streams[1])
    torch.cuda.synchronize()
    f = np.float32
    np.testing.assert_allclose(st.cpu().numpy(), [f(f(0.9 * 0.9) * 0.9), f(f(0.999 * 0.999) * 0.999)], rtol=1e-7)
    for T in towers:
        g = np.zeros(re, np.float32)
        g[:w1] = T["g1"]
        g[rb:rb + r2 * n2] = T["g2"]
        p, m, v = T["p0"].copy(), np.zeros(re, f), np.zeros(re, f)
        b1p, b2p = f(0.9), f(0.999)
        for _ in range(2):
            p, m, v = _adam_ref(p, g, m, v, b1p, b2p)
            b1p, b2p = f(b1p * f(0.9)), f(b2p * f(0.999))
        got = T["p"].cpu().numpy()
        assert np.abs(got - p).max() <= 2 * 2 * 0.01
        well = np.abs(g) > 1e-3 * np.abs(g).max()
        assert np.abs(got - p)[well].max() <= 2e-6, np.abs(got - p)[well].max()
        assert np.array_equal(got[w1:rb], p[w1:rb]) and np.array_equal(got[rb + r2 * n2:], p[rb + r2 * n2:])
        assert not torch.any(T["g"][:w1])
        if bf:
            pw = T["p"][:D * n].view(D, n)
            assert torch.equal(T["sh1"][:, :n], pw.to(torch.bfloat16))
            assert torch.equal(T["sh2"], T["p"][rb:rb + (r2 - 1) * n2].view(r2 - 1, n2).to(torch.bfloat16))
