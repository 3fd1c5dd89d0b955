// fp32 parity mode's dense-layer tiles on the f32-input matrix cores (v_mfma_f32_16x16x4_f32: each
// result is the k-ordered fp32 fmaf chain, no reduced-precision path), shared by gemm32.hip (the
// forward / dA launches) and bn.hip (the dW split-K tiles that ride in the BN-backward apply launch).
// Same fusion as the bf16 path (bnfuse.h): the forward tile applies the previous layer's BN + ReLU
// while staging its A operand and adds its output's per-tower column sums; the dA tile adds the
// previous layer's backward sums (sum dy, sum dy * xhat).
//
// One 256-thread workgroup computes a 64 x 64 tile (4 waves of 32 x 32 = 2 x 2 MFMA 16 x 16 blocks).
// K runs in 32-deep chunks: every chunk's global loads go to registers D chunks ahead (a ring of
// D + 1 register sets, the chunk loop fully unrolled so every index is compile-time), the current
// chunk is written to one of two LDS images and read back one fp32 per lane per MFMA operand
// (64 FLOP/clk/SIMD at 32 cycles per MFMA leaves the LDS idle).  Images are stored as the operand
// lies in memory:
//   RK ([row][k], 36-float rows): 16 rows x 4 consecutive k per read -> 64 distinct banks
//   KR ([k][row], 80-float rows): 4 k rows x 16 consecutive columns -> 64 distinct banks
// FWD: A = Z_{l-1} [M x lda] (RK, BN + ReLU applied while staging), B = W_l [K x ldb] (KR)
// DA : A = dZ_l  [M x lda] (RK), B^T = W_l [N x ldb], i.e. W's rows (RK)
// DW : A^T of A_{l-1} [K x lda] (KR, a virtual ones column at m == M - 1 gives db), B = dZ_l (KR)
#pragma once
#include "bnfuse.h"
#include "common.h"

namespace dssm {

constexpr int kG32KC = 32;                    // k per chunk
constexpr int kG32LdRK = kG32KC + 4;          // 36
constexpr int kG32LdKR = 64 + 16;             // 80
constexpr int kG32Img = 64 * kG32LdRK > kG32KC * kG32LdKR ? 64 * kG32LdRK : kG32KC * kG32LdKR;
constexpr int kG32SmemFloats = 2 * 2 * kG32Img;  // two chunk buffers of (A, B) images: 40 KB
constexpr int kG32MaxK = 320;                 // FWD / DA: the whole K in NCH = 10 chunks
constexpr int kG32DwSplit = 384;              // DW: batch rows per split-K slab (12 chunks)
constexpr int kG32Depth = 3;                  // chunks in flight ahead of the one being written

enum { G32_FWD = 0, G32_DA = 1, G32_DW = 2 };

struct G32Params {
  int M, N, K;
  const float* A;
  int lda;
  const float* B;
  int ldb;
  float* C;  // DW: slab base (split tz at C + tz * M * ldc)
  int ldc;
  const float* bias;  // FWD
  float* a_out;       // FWD: relu(BN(A)) (ld lda), written by the column-tile-0 workgroups
  const float* coef;  // FWD without sums: the A layer's materialised coefficients [4][2][lda]
  int row_split;      // tower boundary (multiple of 64)
  int ones_row, k_per_split;  // DW
};

struct G32Fuse {
  int in_from_sums;    // FWD: the A operand's BN coefficients from `in`'s sums
  BnSide in;
  double* out_sum;     // FS: [2 towers][2][ldc]
  const float* zb;     // DA: pre-BN activations of the output layer [M x ldc]
  const float* coefb;  // DA: its coefficients [4][2][ldc]
  DetAcc det;          // deterministic mode: per-row-tile slab rows + fixed-order sums
  int det_rows;
};

namespace {

// LDS beside the chunk images: the A layer's (inv, shift) per tower [2][2][kG32MaxK] (FWD) and the
// column-sum reduction [2 wm][64][2] (FS)
struct G32Lds {
  float img[kG32SmemFloats];
  float coef[4 * kG32MaxK];
  double red[2 * 64 * 2];
};

// NCH: FWD / DA ceil(K / kG32KC) exactly (the launchers dispatch on it); DW kG32DwSplit / kG32KC
template <int MODE, int FS, int NCH>
__device__ __forceinline__ void g32_body(const G32Params& p, const G32Fuse& f, int tx, int ty, int tz,
                                         G32Lds& L) {
  constexpr bool A_RK = MODE != G32_DW;
  constexpr bool B_RK = MODE == G32_DA;
  constexpr bool BN_A = MODE == G32_FWD;
  constexpr int D = kG32Depth, S = kG32Depth + 1;
  const int M = p.M, N = p.N;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int bm = ty * 64, bn = tx * 64;
  const int kbeg = MODE == G32_DW ? tz * p.k_per_split : 0;
  const int kend = MODE == G32_DW ? min(p.K, kbeg + p.k_per_split) : p.K;
  const int tower = bm < p.row_split ? 0 : 1;
  const int Mload = p.ones_row ? M - 1 : M;  // DW: rows of A^T stored in memory
  // the A operand's coefficient inputs first (they return ahead of the bulk loads)
  constexpr int NPC = (2 * kG32MaxK + 255) / 256;
  FsCoefStage<NPC> cst;
  const bool from_sums = BN_A && f.in_from_sums;
  if (from_sums) cst.load(f.in, t, 256);
  // ---- thread -> staged groups (two float4 of one row / k-row per operand and chunk)
  //   RK: row t >> 2, k (t & 3) * 8 .. + 8;  KR: k-row t >> 3, columns (t & 7) * 8 .. + 8
  const int rk_r = t >> 2, rk_k = (t & 3) * 8;
  const int kr_k = t >> 3, kr_c = (t & 7) * 8;
  float4 ra[S][2], rb[S][2];
  // Every load is unconditional, from its own address when in range and from the operand's base
  // otherwise (a select, no branch: a masked load in a branch makes the compiler drain vmcnt at
  // the merge); stage() zeroes the out-of-range groups.  Widths are multiples of 4, so a float4
  // is all in range or all out.
  auto a_ok = [&](int c, int h) {
    const int k0 = kbeg + c * kG32KC;
    if constexpr (A_RK) return bm + rk_r < M && k0 + rk_k + 4 * h < kend;
    else return k0 + kr_k < kend && bm + kr_c + 4 * h < Mload;
  };
  auto b_ok = [&](int c, int h) {
    const int k0 = kbeg + c * kG32KC;
    if constexpr (B_RK) return bn + rk_r < N && k0 + rk_k + 4 * h < kend;
    else return k0 + kr_k < kend && bn + kr_c + 4 * h < N;
  };
  auto load = [&](int c, float4 (&xa)[2], float4 (&xb)[2]) {
    const int k0 = kbeg + c * kG32KC;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const size_t oa = A_RK ? (size_t)(bm + rk_r) * p.lda + k0 + rk_k + 4 * h   // A [M x lda]
                             : (size_t)(k0 + kr_k) * p.lda + bm + kr_c + 4 * h;  // A^T from A [K x lda]
      const size_t ob = B_RK ? (size_t)(bn + rk_r) * p.ldb + k0 + rk_k + 4 * h   // B^T [N x ldb]
                             : (size_t)(k0 + kr_k) * p.ldb + bn + kr_c + 4 * h;  // B [K x ldb]
      xa[h] = *reinterpret_cast<const float4*>(p.A + (a_ok(c, h) ? oa : 0));
      xb[h] = *reinterpret_cast<const float4*>(p.B + (b_ok(c, h) ? ob : 0));
    }
  };
  // the first D chunks' loads in flight before anything waits
#pragma unroll
  for (int c = 0; c < D; ++c)
    if (c < NCH) load(c, ra[c], rb[c]);
  // the epilogue's bias columns (FWD) and pre-BN values / coefficients (DA), loaded with the operands
  float bcol[2] = {0.f, 0.f};
  if constexpr (MODE == G32_FWD) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = bn + wn * 32 + j * 16 + (lane & 15);
      bcol[j] = (p.bias && n < N) ? p.bias[n] : 0.f;
    }
  }
  float zb[2][2][4], cb[2][4];
  if constexpr (FS == 2) {
    const size_t plane = (size_t)2 * p.ldc;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = bn + wn * 32 + j * 16 + (lane & 15);
      const size_t o = (size_t)tower * p.ldc + (n < N ? n : 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) cb[j][q] = f.coefb[q * plane + o];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = bm + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
          zb[i][j][r] = f.zb[(size_t)(m < M ? m : 0) * p.ldc + (n < N ? n : 0)];
        }
    }
  }
  // ---- the A layer's BN coefficients (FWD), zero beyond its width
  const int Kc = NCH * kG32KC;  // staged k extent (<= kG32MaxK for FWD)
  if constexpr (BN_A) {
    if (from_sums) {
      cst.finish(f.in, t, 256, [&](int tw, int k, float, float, float inv, float sh) {
        if (k < Kc) {
          L.coef[(tw * 2 + 0) * kG32MaxK + k] = inv;
          L.coef[(tw * 2 + 1) * kG32MaxK + k] = sh;
        }
      });
      for (int i = t; i < 2 * (Kc - p.lda); i += 256) {
        const int tw = i / (Kc - p.lda), k = p.lda + i % (Kc - p.lda);
        L.coef[(tw * 2 + 0) * kG32MaxK + k] = 0.f;
        L.coef[(tw * 2 + 1) * kG32MaxK + k] = 0.f;
      }
    } else {
      const size_t plane = (size_t)2 * p.lda;
      for (int i = t; i < 2 * Kc; i += 256) {
        const int tw = i / Kc, k = i - tw * Kc;
        const bool ok = k < p.lda;
        L.coef[(tw * 2 + 0) * kG32MaxK + k] = ok ? p.coef[2 * plane + (size_t)tw * p.lda + k] : 0.f;
        L.coef[(tw * 2 + 1) * kG32MaxK + k] = ok ? p.coef[3 * plane + (size_t)tw * p.lda + k] : 0.f;
      }
    }
    __syncthreads();
  }
  const bool write_a = BN_A && p.a_out != nullptr && tx == 0;
  // chunk c's registers -> LDS image buf (BN + ReLU on A for FWD; the ones column for DW)
  auto stage = [&](int c, float4 (&xa)[2], float4 (&xb)[2], int buf) {
    float* sa = L.img + buf * 2 * kG32Img;
    float* sb = sa + kG32Img;
    const int k0 = kbeg + c * kG32KC;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!a_ok(c, h)) xa[h] = z4;
      if (!b_ok(c, h)) xb[h] = z4;
    }
    if constexpr (BN_A) {
      const int r = bm + rk_r;
      const float* ci = &L.coef[(tower * 2) * kG32MaxK + k0 + rk_k];
      const float* ch = ci + kG32MaxK;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float4& v = xa[h];
        v.x = fmaxf(bn_affine(v.x, ci[4 * h + 0], ch[4 * h + 0]), 0.f);
        v.y = fmaxf(bn_affine(v.y, ci[4 * h + 1], ch[4 * h + 1]), 0.f);
        v.z = fmaxf(bn_affine(v.z, ci[4 * h + 2], ch[4 * h + 2]), 0.f);
        v.w = fmaxf(bn_affine(v.w, ci[4 * h + 3], ch[4 * h + 3]), 0.f);
        const int k = k0 + rk_k + 4 * h;
        if (write_a && r < M && k < p.lda) *reinterpret_cast<float4*>(p.a_out + (size_t)r * p.lda + k) = v;
      }
    }
    if constexpr (MODE == G32_DW) {
      if (p.ones_row) {
        const int k = k0 + kr_k;
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (bm + kr_c + 4 * h == Mload && k < kend) xa[h].x = 1.0f;
      }
    }
    if constexpr (A_RK) {
#pragma unroll
      for (int h = 0; h < 2; ++h) *reinterpret_cast<float4*>(&sa[rk_r * kG32LdRK + rk_k + 4 * h]) = xa[h];
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) *reinterpret_cast<float4*>(&sa[kr_k * kG32LdKR + kr_c + 4 * h]) = xa[h];
    }
    if constexpr (B_RK) {
#pragma unroll
      for (int h = 0; h < 2; ++h) *reinterpret_cast<float4*>(&sb[rk_r * kG32LdRK + rk_k + 4 * h]) = xb[h];
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) *reinterpret_cast<float4*>(&sb[kr_k * kG32LdKR + kr_c + 4 * h]) = xb[h];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fk = lane >> 4;  // fragment row / column and k within the 4-deep step
  // ---- the chunk pipeline: load c + D, stage c, barrier, MFMA c (one barrier per chunk: the image
  // staged at c was last read at c - 2, before every wave passed barrier c - 1).  NCH is the
  // chunk count (FWD / DA: exactly ceil(K / 32); DW: the split's, chunks past its rows staged as
  // zeros), so the unrolled pipeline is straight-line code and the compiler's vmcnt waits are exact
  // (a runtime chunk bound around the loads made it drain every load at each branch merge).
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    {
      if (c + D < NCH) load(c + D, ra[(c + D) % S], rb[(c + D) % S]);
      const int buf = c & 1;
      stage(c, ra[c % S], rb[c % S], buf);
      __syncthreads();
      const float* sa = L.img + buf * 2 * kG32Img;
      const float* sb = sa + kG32Img;
      const int kv = kend - (kbeg + c * kG32KC);  // valid k of this chunk (the rest are zeros)
#pragma unroll
      for (int kk = 0; kk < kG32KC; kk += 4) {
        if (kk < kv) {
          float av[2], bv[2];
#pragma unroll
          for (int i = 0; i < 2; ++i)
            av[i] = A_RK ? sa[(wm * 32 + i * 16 + fr) * kG32LdRK + kk + fk]
                         : sa[(kk + fk) * kG32LdKR + wm * 32 + i * 16 + fr];
#pragma unroll
          for (int j = 0; j < 2; ++j)
            bv[j] = B_RK ? sb[(wn * 32 + j * 16 + fr) * kG32LdRK + kk + fk]
                         : sb[(kk + fk) * kG32LdKR + wn * 32 + j * 16 + fr];
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
      }
    }
  }
  // ---- epilogue: C/D map col = lane & 15, row = (lane >> 4) * 4 + r
  if constexpr (MODE == G32_DW) {
    float* out = p.C + (size_t)tz * M * p.ldc;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = bn + wn * 32 + j * 16 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = bm + wm * 32 + i * 16 + fk * 4 + r;
          if (m < M && n < N) out[(size_t)m * p.ldc + n] = acc[i][j][r];
        }
      }
    return;
  }
  double cs[2] = {0.0, 0.0}, cq[2] = {0.0, 0.0};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = bn + wn * 32 + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = bm + wm * 32 + i * 16 + fk * 4 + r;
        if (m < M && n < p.ldc) {
          const float v = acc[i][j][r];
          const float x = (n < N) ? v + bcol[j] : 0.f;
          p.C[(size_t)m * p.ldc + n] = x;
          if constexpr (FS == 1) {
            cs[j] += x;
            cq[j] += (double)x * x;
          } else if constexpr (FS == 2) {
            const float z = zb[i][j][r];
            // the forward's ReLU mask (bn.hip bwd_terms): dy = dA where BN(z) > 0
            const float dy = (n < N && bn_affine(z, cb[j][2], cb[j][3]) > 0.f) ? x : 0.f;
            const float xh = (z - cb[j][0]) * cb[j][1];
            cs[j] += dy;
            cq[j] += (double)dy * xh;
          }
        }
      }
    }
  }
  if constexpr (FS != 0) {
    // the wave's 4 row groups by shuffles, the two wm halves through LDS, one atomic per statistic
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      cs[j] += __shfl_xor(cs[j], 16);
      cs[j] += __shfl_xor(cs[j], 32);
      cq[j] += __shfl_xor(cq[j], 16);
      cq[j] += __shfl_xor(cq[j], 32);
    }
    if (wm == 1 && lane < 16) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        L.red[(wn * 32 + j * 16 + lane) * 2] = cs[j];
        L.red[(wn * 32 + j * 16 + lane) * 2 + 1] = cq[j];
      }
    }
    __syncthreads();
    if (wm == 0 && lane < 16) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = wn * 32 + j * 16 + lane, n = bn + c;
        if (n < N) {
          const double s1 = cs[j] + L.red[c * 2], s2 = cq[j] + L.red[c * 2 + 1];
          if (f.det.slab) {  // deterministic: this row tile's slab row, the other tower zero
            double* row = f.det.slab + (size_t)ty * 4 * p.ldc;
            row[(size_t)(tower * 2) * p.ldc + n] = s1;
            row[(size_t)(tower * 2 + 1) * p.ldc + n] = s2;
            row[(size_t)((1 - tower) * 2) * p.ldc + n] = 0.0;
            row[(size_t)((1 - tower) * 2 + 1) * p.ldc + n] = 0.0;
          } else {
            atomic_add_f64(f.out_sum + (size_t)(tower * 2) * p.ldc + n, s1);
            atomic_add_f64(f.out_sum + (size_t)(tower * 2 + 1) * p.ldc + n, s2);
          }
        }
      }
    }
    if (f.det.slab) {
      __shared__ int s_det;
      det_publish(f.det, tx, ty, f.det_rows, p.ldc, bn, min(bn + 64, N), f.out_sum, &s_det);
    }
  }
}

}  // namespace
}  // namespace dssm
