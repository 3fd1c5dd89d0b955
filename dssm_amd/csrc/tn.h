// The split-K "TN" tile of the dW GEMMs, shared by gemm.hip (k_gemm_tn, k_bwd_pair) and bn.hip
// (the dW tiles that ride in the BN-backward apply launch): 64 x 64 output per 256-thread
// workgroup, 64-deep k-steps double-buffered in LDS (2 x 2 x kTnTile u16 = 36 KiB).
#pragma once
#include "common.h"

namespace dssm {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int kTnBK = 64, kTnLd = kTnBK + 8;  // [k][m] / [k][n] tiles, 144-B rows
constexpr int kTnTile = 64 * kTnLd;            // one LDS operand buffer (u16)

// C[M x N] (+ split slab tz at C + tz*M*ldc) = A^T . B over k in [tz*k_per_split, ...): A [K x lda]
// (m contiguous), B [K x ldb] (n contiguous); ones_row: virtual all-ones A column at m == M-1.
struct TnParams {
  int M, N, K;
  const u16* A;
  int lda;
  const u16* B;
  int ldb;
  float* C;
  int ldc, ones_row, k_per_split;
};

namespace {

// "TN" (dW): C[M x N] (+ split slab) = A^T . B over K batch rows, A [K x lda] (m contiguous),
// B [K x ldb] (n contiguous), both bf16.  Both tiles are staged exactly as they lie in memory
// ([k][m], [k][n]: 16-B loads and 16-B LDS writes) and the MFMA fragments, which need 8
// consecutive k per lane, come from ds_read_b64_tr_b16 (4 k x 16 columns per 16-lane group,
// delivered column-major).  ones_row: virtual all-ones A column at m == M-1 (-> bias grad).

__device__ __forceinline__ bf16x8 tn_frag(const u16* tile, int row0, int col0, int lane) {
  // lanes 16g+4q+p read rows (row0 + 8g + q [+4]) at columns col0 + 4p..4p+3
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const u16* a0 = tile + (row0 + 8 * g + q) * kTnLd + col0 + 4 * p;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a0);
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0 + 4 * kTnLd));
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}


__device__ __forceinline__ void tn_body(const TnParams& p, int tx, int ty, int tz, u16* sA, u16* sB) {
  const int M = p.M, N = p.N, lda = p.lda, ldb = p.ldb;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int bm = ty * 64, bn = tx * 64;
  const int kbeg = tz * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int Mload = p.ones_row ? M - 1 : M;
  int sk[2], sc[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int e = t + 256 * g;
    sk[g] = e >> 3;
    sc[g] = (e & 7) * 8;
  }
  uint4 ra[2], rb[2];
  auto load = [&](int k0) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int gk = k0 + sk[g], gm = bm + sc[g], gn = bn + sc[g];
      uint4 va = make_uint4(0u, 0u, 0u, 0u), vb = make_uint4(0u, 0u, 0u, 0u);
      if (gk < kend) {
        if (gm + 8 <= Mload) {
          va = *reinterpret_cast<const uint4*>(p.A + (size_t)gk * lda + gm);
        } else {
          u16 x[8];
#pragma unroll
          for (int i = 0; i < 8; ++i)
            x[i] = (gm + i < Mload) ? p.A[(size_t)gk * lda + gm + i]
                                    : ((p.ones_row && gm + i == Mload) ? (u16)0x3f80 : (u16)0);
          va.x = x[0] | ((unsigned)x[1] << 16); va.y = x[2] | ((unsigned)x[3] << 16);
          va.z = x[4] | ((unsigned)x[5] << 16); va.w = x[6] | ((unsigned)x[7] << 16);
        }
        if (gn + 8 <= N) {
          vb = *reinterpret_cast<const uint4*>(p.B + (size_t)gk * ldb + gn);
        } else {
          u16 x[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = (gn + i < N) ? p.B[(size_t)gk * ldb + gn + i] : (u16)0;
          vb.x = x[0] | ((unsigned)x[1] << 16); vb.y = x[2] | ((unsigned)x[3] << 16);
          vb.z = x[4] | ((unsigned)x[5] << 16); vb.w = x[6] | ((unsigned)x[7] << 16);
        }
      }
      ra[g] = va;
      rb[g] = vb;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      *reinterpret_cast<uint4*>(&sA[buf * kTnTile + sk[g] * kTnLd + sc[g]]) = ra[g];
      *reinterpret_cast<uint4*>(&sB[buf * kTnTile + sk[g] * kTnLd + sc[g]]) = rb[g];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (kbeg < kend) {
    load(kbeg);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += kTnBK, buf ^= 1) {
    const bool more = k0 + kTnBK < kend;
    if (more) load(k0 + kTnBK);
#pragma unroll
    for (int ks = 0; ks < kTnBK; ks += 32) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = tn_frag(sA + buf * kTnTile, ks, wm * 32 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = tn_frag(sB + buf * kTnTile, ks, wn * 32 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }
  float* out = p.C + (size_t)tz * M * p.ldc;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = bn + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = bm + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (m < M && n < N) out[(size_t)m * p.ldc + n] = acc[i][j][r];
      }
    }
  }
}

// Whole-split variant of tn_body (same tile, same k order, so the same sums): every load of the
// split's k_per_split <= 128 * NSUB rows is issued at once (one round trip instead of one per
// 64-row k-step), then staged through the same 2 x 2 x kTnTile LDS 128 rows at a time.
// Needs lda >= Mload, ldb >= N, both multiples of 8 (the callers' padded strides).
template <int NSUB>
__device__ __forceinline__ void tn_chunk_body(const TnParams& p, int tx, int ty, int tz, u16* sA,
                                              u16* sB) {
  const int M = p.M;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int bm = ty * 64, bn = tx * 64;
  const int kbeg = tz * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int Mload = p.ones_row ? M - 1 : M;
  const int sc = (t & 7) * 8;  // group g of a sub-chunk: row (t >> 3) + 32 g
  // Every load unconditional, from a clamped in-bounds address (lda, ldb: multiples of 8 that
  // cover Mload, N), so all of them are in flight before the first wait; edge tiles then fix
  // their out-of-range elements (zero; the ones column) with selects.
  const int gm = bm + sc, gn = bn + sc;
  const int gmc = min(gm, p.lda - 8), gnc = min(gn, p.ldb - 8);
  uint4 ra[NSUB][4], rb[NSUB][4];
#pragma unroll
  for (int s = 0; s < NSUB; ++s)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int gk = min(kbeg + 128 * s + (t >> 3) + 32 * g, kend - 1);
      ra[s][g] = *reinterpret_cast<const uint4*>(p.A + (size_t)gk * p.lda + gmc);
      rb[s][g] = *reinterpret_cast<const uint4*>(p.B + (size_t)gk * p.ldb + gnc);
    }
  // Edge tiles: this thread's 8 columns get a keep mask (column < lim) and the ones-row pattern
  // (column == lim), formed once; each operand vector is written to LDS as (v & keep) | ones, or zero
  // for a row past the split.  (A per-element extract / select / insert right after the loads cost
  // ~50 VALU instructions per vector and made the edge tiles the apply launch's longest.)
  const bool edge = !(bm + 64 <= Mload && bn + 64 <= p.N && kbeg + 128 * NSUB <= kend);
  uint4 ka = make_uint4(~0u, ~0u, ~0u, ~0u), oa = make_uint4(0u, 0u, 0u, 0u), kb = ka, ob = oa;
  if (edge) {
    auto masks = [](int g0, int lim, bool ones, uint4& keep, uint4& one) {
      unsigned kk[4], oo[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int lo = g0 + 2 * q, hi = lo + 1;
        kk[q] = (lo < lim ? 0xffffu : 0u) | (hi < lim ? 0xffff0000u : 0u);
        oo[q] = ((ones && lo == lim) ? 0x3f80u : 0u) | ((ones && hi == lim) ? 0x3f800000u : 0u);
      }
      keep = make_uint4(kk[0], kk[1], kk[2], kk[3]);
      one = make_uint4(oo[0], oo[1], oo[2], oo[3]);
    };
    masks(gm, Mload, p.ones_row != 0, ka, oa);
    masks(gn, p.N, false, kb, ob);
  }
  auto fix = [](uint4 v, uint4 keep, uint4 one, bool rowok) {
    return rowok ? make_uint4((v.x & keep.x) | one.x, (v.y & keep.y) | one.y, (v.z & keep.z) | one.z,
                              (v.w & keep.w) | one.w)
                 : make_uint4(0u, 0u, 0u, 0u);
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NSUB; ++s) {
    if (kbeg + 128 * s >= kend) break;
    if (s) __syncthreads();  // every wave is past the previous sub-chunk's fragment reads
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int r = (t >> 3) + 32 * g;
      uint4 va = ra[s][g], vb = rb[s][g];
      if (edge) {
        const bool rowok = kbeg + 128 * s + r < kend;
        va = fix(va, ka, oa, rowok);
        vb = fix(vb, kb, ob, rowok);
      }
      *reinterpret_cast<uint4*>(&sA[r * kTnLd + sc]) = va;
      *reinterpret_cast<uint4*>(&sB[r * kTnLd + sc]) = vb;
    }
    __syncthreads();
    const int kc = min(128, ((kend - kbeg - 128 * s) + 31) & ~31);
    for (int ks = 0; ks < kc; ks += 32) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = tn_frag(sA, ks, wm * 32 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = tn_frag(sB, ks, wn * 32 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  float* out = p.C + (size_t)tz * M * p.ldc;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = bn + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = bm + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (m < M && n < p.N) out[(size_t)m * p.ldc + n] = acc[i][j][r];
      }
    }
  }
}

}  // namespace
}  // namespace dssm
