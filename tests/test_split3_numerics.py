"""The fp32 parity mode's split products (dssm_amd/csrc/g32.h, DSSM_G32_SPLIT): every fp32 operand is
split into three bf16 planes x = h + m + l while staging, and the tile sums the six partial
products hh + hm + mh + hl + lh + mm on the bf16 matrix cores with fp32 accumulation.

CPU restatement of the arithmetic (bf16 = round-to-nearest-even of the fp32 bit pattern's top 16
bits, as v_cvt_pk_bf16_f32 does), checking the two claims the design rests on:
* the split is exact for normal fp32 values (h + m + l == x, each step exact in fp32);
* the six kept products differ from the exact product a*b by less than 2^-22 |a b| (the dropped
  ml + lm + ll), i.e. below two fp32 roundings of the product; a K=320 dot product of them stays
  within fp32 accumulation error of the float64 result."""
import numpy as np


def bf16(x: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 (RNE) -> fp32."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def split3(x: np.ndarray):
    x = np.asarray(x, np.float32)
    h = bf16(x)
    with np.errstate(invalid="ignore"):
        r = (x - h).astype(np.float32)
    m = bf16(r)
    q = (r - m).astype(np.float32)
    l = bf16(q)
    return h, m, l


def test_split_is_exact():
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(200000) * np.exp(rng.uniform(-20, 20, 200000))).astype(np.float32)
    h, m, l = split3(x)
    assert np.array_equal(bf16(l), l)  # l needs no rounding
    back = (h.astype(np.float64) + m.astype(np.float64) + l.astype(np.float64))
    np.testing.assert_array_equal(back, x.astype(np.float64))


def test_six_term_product_error():
    rng = np.random.default_rng(1)
    a = rng.standard_normal(100000).astype(np.float32)
    b = rng.standard_normal(100000).astype(np.float32)
    (ah, am, al), (bh, bm, bl) = split3(a), split3(b)
    f = lambda u, v: u.astype(np.float64) * v.astype(np.float64)  # noqa: E731  bf16 x bf16: exact
    six = f(ah, bh) + f(ah, bm) + f(am, bh) + f(ah, bl) + f(al, bh) + f(am, bm)
    exact = a.astype(np.float64) * b.astype(np.float64)
    rel = np.abs(six - exact) / np.maximum(np.abs(exact), 1e-300)
    assert rel.max() < 2.0 ** -22, rel.max()


def test_split_dot_product_within_fp32_accumulation():
    """K = 320 dot products (the forward's widest K): six-term products accumulated in fp32 (two
    accumulators, as the tile does) against float64; the error is of the order of fp32 summation."""
    rng = np.random.default_rng(2)
    K, n = 320, 2000
    A = rng.standard_normal((n, K)).astype(np.float32)
    B = rng.standard_normal((n, K)).astype(np.float32)
    (ah, am, al), (bh, bm, bl) = split3(A), split3(B)
    acc = np.zeros(n, np.float32)
    acc2 = np.zeros(n, np.float32)
    for k0 in range(0, K, 32):  # per 32-deep chunk: each MFMA adds a chunk's products to fp32
        s = slice(k0, k0 + 32)
        pr = lambda u, v: (u[:, s].astype(np.float64) * v[:, s].astype(np.float64)).sum(1)  # noqa: E731
        acc = (acc + pr(ah, bh).astype(np.float32)).astype(np.float32)
        for u, v in ((ah, bm), (am, bh), (ah, bl), (al, bh), (am, bm)):
            acc2 = (acc2 + pr(u, v).astype(np.float32)).astype(np.float32)
    got = (acc2 + acc).astype(np.float64)
    ref = (A.astype(np.float64) * B.astype(np.float64)).sum(1)
    scale = np.sqrt((A.astype(np.float64) ** 2 * B.astype(np.float64) ** 2).sum(1))
    err = np.abs(got - ref) / scale
    # fp32 sequential accumulation of K terms: ~sqrt(K) * 2^-24 relative to the terms' norm
    assert err.max() < 4 * np.sqrt(K) * 2.0 ** -24, err.max()


def test_non_finite_operand_gives_nan():
    """g32.h's documented range: an Inf operand makes the split product NaN (not Inf).  Its
    residual x - h is NaN; and even a residual forced to zero would leave h_a * m_b = Inf * 0 = NaN
    for a bf16-exact b, whose m and l planes are zero."""
    a = np.array([np.inf, -np.inf, 1.5], np.float32)
    b = np.array([2.0, 2.0, 2.0], np.float32)
    (ah, am, al), (bh, bm, bl) = split3(a), split3(b)
    assert not np.any(bm) and not np.any(bl)
    with np.errstate(invalid="ignore"):
        six = ah * bh + ah * bm + am * bh + ah * bl + al * bh + am * bm
        forced = ah * bh + ah * bm  # m_a = l_a = 0
    assert np.isnan(six[:2]).all() and np.isnan(forced[:2]).all() and six[2] == 3.0
