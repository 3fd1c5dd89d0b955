// fp32 parity mode's dense-layer tiles, shared by gemm32.hip (the forward / dA launches) and bn.hip
// (the dW split-K tiles that ride in the BN-backward apply launch).  The DEFAULT build
// (DSSM_G32_SPLIT=1, below) forms the products on the bf16 matrix cores from an exact three-way
// split of each fp32 operand; -DDSSM_G32_SPLIT=0 builds the k-ordered fp32 fmaf chains on
// v_mfma_f32_16x16x4_f32 (no reduced-precision path) that the rest of this paragraph describes.
// Same fusion as the bf16 path (bnfuse.h): the forward tile applies the previous layer's BN + ReLU
// while staging its A operand and adds its output's per-tower column sums; the dA tile adds the
// previous layer's backward sums (sum dy, sum dy * xhat).
//
// One 256-thread workgroup computes a 64 x 64 tile (4 waves of 32 x 32 = 2 x 2 MFMA 16 x 16 blocks).
// K runs in 32-deep chunks: every chunk's global loads go to registers D chunks ahead (a ring of
// D + 1 register sets, the chunk loop fully unrolled so every index is compile-time), the current
// chunk is written to one of two LDS images and read back in 8-deep k steps: two MFMAs per step,
// MFMA q taking k = kk + 2 g + q from lane group g = lane >> 4 (the same permutation for A and B, so
// each lane holds two consecutive k of its row / column).  Images are stored as the operand lies in
// memory (MI355X_MICROARCH.md LDS banking):
//   RK ([row][k], 36-float rows): one ds_read_b64 per lane, 16 rows x 2 groups -> 64 distinct banks
//   KR ([k][row], 72-float rows): one ds_read2_b32 (rows kk + 2g, + 1) per lane; each of its reads
//       covers 16 columns x 2 groups on 32 distinct banks
// FWD: A = Z_{l-1} [M x lda] (RK, BN + ReLU applied while staging), B = W_l [K x ldb] (KR)
// DA : A = dZ_l  [M x lda] (RK), B^T = W_l [N x ldb], i.e. W's rows (RK)
// DW : A^T of A_{l-1} [K x lda] (KR, a virtual ones column at m == M - 1 gives db), B = dZ_l (KR)
//
// DSSM_G32_SPLIT (default 1): the products on the bf16 matrix cores instead, each fp32 operand
// split EXACTLY into three bf16 planes while staging (x = h + m + l: h = bf16(x), m = bf16(x - h),
// l = x - h - m, each step exact in fp32 for normal x), and per 32-deep chunk the six partial
// products down to 2^-16 relative (hh; hm, mh; hl, lh, mm) on v_mfma_f32_16x16x32_bf16, fp32
// accumulate, the hh chain and the small-term chain in separate accumulators summed in the
// epilogue.  The dropped ml, lm, ll terms are below 2^-24 |a b|: every product is accurate to about
// one fp32 rounding, and 6 bf16 MFMAs cost 6/16 of the 8 fp32 MFMAs they replace (the fp32 matrix
// rate is 1/16 of bf16's, MI355X_MICROARCH.md).  LDS images hold the three planes as bf16: RK
// [row][k] rows of 40 (ds_read_b128 fragments), KR [k][col] rows of 72 (ds_read_b64_tr_b16
// fragments, tn.h).  DSSM_G32_SPLIT=0 builds the exact fp32 FMA-chain tiles described above.
// Range: the split is exact for normal and zero x below bf16's largest finite value.  A non-finite
// operand makes the product NaN, not Inf: its residual x - h is NaN, and even with the residual
// forced to zero the partial product h_a * m_b (m_b = 0 for a bf16-exact b) is Inf * 0 = NaN
// (tests/test_split3_numerics.py restates this).  Either way the step's loss turns non-finite, as
// the reference's would; DSSM_G32_SPLIT=0 keeps IEEE Inf.  Subnormal x: bf16 shares fp32's exponent
// range, so h / m / l of a subnormal are subnormal bf16 and the matrix core may flush them (the
// product then loses < 2^-126 in absolute terms, far below every tolerance here).
#pragma once
#include "bnfuse.h"
#include "common.h"
#include "tn.h"

#ifndef DSSM_G32_SPLIT
#define DSSM_G32_SPLIT 1
#endif

namespace dssm {

constexpr int kG32KC = 32;                    // k per chunk
constexpr int kG32LdRK = kG32KC + 4;          // 36
constexpr int kG32LdKR = 64 + 8;              // 72
constexpr int kG32Img = 64 * kG32LdRK > kG32KC * kG32LdKR ? 64 * kG32LdRK : kG32KC * kG32LdKR;
constexpr bool kG32Split = DSSM_G32_SPLIT != 0;
constexpr int kS3LdRK = kG32KC + 8;           // split planes, RK: 40 bf16 (80-B rows)
constexpr int kS3LdKR = kTnLd;                // split planes, KR: 72 bf16 (tn.h's stride)
constexpr int kS3Plane = 64 * kS3LdRK > kG32KC * kS3LdKR ? 64 * kS3LdRK : kG32KC * kS3LdKR;  // u16
constexpr int kS3Img = 3 * kS3Plane;          // one operand's three planes (u16)
// two chunk buffers of (A, B) images: exact 36 KB; split 60 KB
constexpr int kG32SmemFloats = kG32Split ? 2 * 2 * kS3Img / 2 : 2 * 2 * kG32Img;
constexpr int kG32MaxK = 320;                 // FWD / DA: the whole K in NCH = 10 chunks
constexpr int kG32DwSplit = 384;              // DW: batch rows per split-K slab (12 chunks)
#ifndef DSSM_G32_DEPTH
#define DSSM_G32_DEPTH 4
#endif
constexpr int kG32Depth = DSSM_G32_DEPTH;     // chunks in flight ahead of the one being computed
#ifndef DSSM_G32_FRAGALL
#define DSSM_G32_FRAGALL 0  // 1: a chunk's fragments all read before its staging / MFMAs (A/B option)
#endif

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
  u16* a_out16;       // FWD (bf16 plan, DSSM_OPT_FWD32): relu(BN(A)) written bf16 instead of a_out
};

struct G32Fuse {
  int in_from_sums;    // FWD: the A operand's BN coefficients from `in`'s sums
  BnSide in;
  double* out_sum;     // FS: [2 towers][2][ldc]
  const float* zb;     // DA: pre-BN activations of the output layer [M x ldc]
  const float* coefb;  // DA: its coefficients [4][2][ldc]
  DetAcc det;          // deterministic mode: per-row-tile slab rows + fixed-order sums
  int det_rows;
  int tl_slot;         // diagnostics build (G32_TL): the launch's timeline slot, -1 none
};

// Diagnostics build only (-DDSSM_G32_TL, gemm32.hip's forward / dA launches): per-workgroup
// s_memrealtime stamps (100 MHz) of wave 0: [0] start, [1] prologue done, [2 + 2c] chunk c staged
// (after its barrier), [3 + 2c] chunk c's MFMAs issued, [30] epilogue done; read back by
// dssm_debug_g32_timeline (tools/g32_timeline.py).
#if defined(DSSM_G32_TL) && defined(DSSM_G32_TL_HOST)
#define G32_TL(slot, idx)                                                                        \
  do {                                                                                           \
    if (threadIdx.x == 0 && (slot) >= 0)                                                         \
      g_g32_tl[slot][blockIdx.x & 2047][idx] = __builtin_amdgcn_s_memrealtime();                 \
  } while (0)
#else
#define G32_TL(slot, idx) \
  do {                    \
  } while (0)
#endif

namespace {

// LDS beside the chunk images: the A layer's (inv, shift) per tower [2][2][kG32MaxK] (FWD) and the
// column-sum reduction [2 wm][64][2] (FS)
struct G32Lds {
  float img[kG32SmemFloats];
  float coef[4 * kG32MaxK];
  double red[2 * 64 * 2];
};

// 4 fp32 values -> their three bf16 planes, 4 bf16 each (x = h + m + l exactly for normal x)
__device__ __forceinline__ void split3(const float4 v, uint2& h, uint2& m, uint2& l) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  float r[4], q[4];
  u16 a[4], b[4], c[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a[e] = f2bf(x[e]);
    r[e] = x[e] - bf2f(a[e]);
    b[e] = f2bf(r[e]);
    q[e] = r[e] - bf2f(b[e]);
    c[e] = f2bf(q[e]);
  }
  h = make_uint2(a[0] | ((unsigned)a[1] << 16), a[2] | ((unsigned)a[3] << 16));
  m = make_uint2(b[0] | ((unsigned)b[1] << 16), b[2] | ((unsigned)b[3] << 16));
  l = make_uint2(c[0] | ((unsigned)c[1] << 16), c[2] | ((unsigned)c[3] << 16));
}

// NCH: FWD / DA ceil(K / kG32KC) exactly (the launchers dispatch on it); DW kG32DwSplit / kG32KC.
// WN: waves along the tile's 64 columns (2: 4 waves of 32 x 32; 4: 8 waves of 32 x 16, two per
// SIMD, for launches that give a CU one tile: a lone wave per SIMD waits out every LDS and barrier
// latency with the matrix core idle, two interleave).  Threads: 128 WN.
template <int MODE, int FS, int NCH, int WN = 2>
__device__ __forceinline__ void g32_body(const G32Params& p, const G32Fuse& f, int tx, int ty, int tz,
                                         G32Lds& L) {
  constexpr bool A_RK = MODE != G32_DW;
  constexpr bool B_RK = MODE == G32_DA;
  constexpr bool BN_A = MODE == G32_FWD;
  constexpr int D = kG32Depth, S = kG32Depth + 1;
  constexpr int NT = 128 * WN;    // threads
  constexpr int JN = 4 / WN;      // 16-column MFMA blocks per wave
  constexpr int WC = 64 / WN;     // columns per wave
  constexpr int G = 512 / NT;     // staged float4 per thread, operand and chunk
  const int M = p.M, N = p.N;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w / WN, wn = w % WN;
  const int bm = ty * 64, bn = tx * 64;
  const int kbeg = MODE == G32_DW ? tz * p.k_per_split : 0;
  const int kend = MODE == G32_DW ? min(p.K, kbeg + p.k_per_split) : p.K;
  const int tower = bm < p.row_split ? 0 : 1;
  const int Mload = p.ones_row ? M - 1 : M;  // DW: rows of A^T stored in memory
  G32_TL(f.tl_slot, 0);
#if defined(DSSM_G32_TL) && defined(DSSM_G32_TL_HOST)
  if (threadIdx.x == 0 && f.tl_slot >= 0) g_g32_tl[f.tl_slot][blockIdx.x & 2047][28] = __builtin_amdgcn_s_memtime();
#endif
  // the A operand's coefficient inputs first (they return ahead of the bulk loads)
  constexpr int NPC = (2 * kG32MaxK + NT - 1) / NT;
  FsCoefStage<NPC> cst;
  const bool from_sums = BN_A && f.in_from_sums;
  if (from_sums) cst.load(f.in, t, NT);
  // ---- thread -> staged groups: G float4 per operand and chunk, each wave instruction reading
  // whole 128-B lines (RK: 8 lanes per 32-float row, rows rk_r + (NT / 8) h; KR: 16 lanes per
  // 64-float k-row, k-rows kr_k + (NT / 16) h)
  const int rk_r = t >> 3, rk_k = (t & 7) * 4;
  const int kr_k = t >> 4, kr_c = (t & 15) * 4;
  constexpr int RKH = NT / 8, KRH = NT / 16;
  float4 ra[S][G], rb[S][G];
  // Each staged group's row / column part of its address is computed once; a chunk adds its k
  // offset (RK: along the row, a compile-time offset for FWD / DA; KR: k rows of stride ld).  Loads
  // are unconditional (a masked load in a branch makes the compiler drain vmcnt at the merge):
  // out-of-range rows / columns read row / column 0, and in a chunk that reaches past kend the k
  // index is clamped to the operand's stored extent.  stage() zeroes the groups outside, under
  // uniform conditions (edge tiles, the tail chunk) that interior tiles and full chunks skip.
  // Every tile walks K in order: each result is a fixed sequence of fp32 accumulations.
  const int kdim = MODE == G32_DW ? p.K : kend;  // k extent in memory (DW: every batch row)
  size_t a_off[G], b_off[G];
  bool a_in[G], b_in[G];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    if constexpr (A_RK) {
      const int r = bm + rk_r + RKH * h;
      a_in[h] = r < M;
      a_off[h] = (size_t)(a_in[h] ? r : 0) * p.lda + rk_k;
    } else {
      const int c = bm + kr_c;
      a_in[h] = c < Mload;
      a_off[h] = (size_t)(kr_k + KRH * h) * p.lda + (a_in[h] ? c : 0);
    }
    if constexpr (B_RK) {
      const int r = bn + rk_r + RKH * h;
      b_in[h] = r < N;
      b_off[h] = (size_t)(b_in[h] ? r : 0) * p.ldb + rk_k;
    } else {
      const int c = bn + kr_c;
      b_in[h] = c < N;
      b_off[h] = (size_t)(kr_k + KRH * h) * p.ldb + (b_in[h] ? c : 0);
    }
  }
  const bool edge = bm + 64 > (A_RK ? M : Mload) || bn + 64 > N;  // uniform
  auto kofs = [&](int c) { return kbeg + c * kG32KC; };
  auto a_ok = [&](int c, int h) {
    const int k0 = kofs(c);
    if constexpr (A_RK) return a_in[h] && k0 + rk_k < kend;
    else return a_in[h] && k0 + kr_k + KRH * h < kend;
  };
  auto b_ok = [&](int c, int h) {
    const int k0 = kofs(c);
    if constexpr (B_RK) return b_in[h] && k0 + rk_k < kend;
    else return b_in[h] && k0 + kr_k + KRH * h < kend;
  };
  auto load = [&](int c, float4 (&xa)[G], float4 (&xb)[G]) {
#ifdef DSSM_G32_SAMECHUNK  // diagnostics (wrong results): every chunk's loads from chunk 0's lines
    const int k0 = kofs(0);
#else
    const int k0 = kofs(c);
#endif
    // uniform; FWD / DA: only the last chunk (compile-time) can reach past K
    const bool tail = (MODE == G32_DW || c == NCH - 1) && k0 + kG32KC > kend;
    const float* pa = p.A + (A_RK ? (size_t)k0 : (size_t)k0 * p.lda);
    const float* pb = p.B + (B_RK ? (size_t)k0 : (size_t)k0 * p.ldb);
#pragma unroll
    for (int h = 0; h < G; ++h) {
      size_t oa = a_off[h], ob = b_off[h];
      if (tail) {  // clamp k into the stored extent (rows past kend are zeroed by stage())
        if constexpr (A_RK) oa -= (size_t)max(0, k0 + rk_k - (kdim - 4));
        else oa -= (size_t)max(0, k0 + kr_k + KRH * h - (kdim - 1)) * p.lda;
        if constexpr (B_RK) ob -= (size_t)max(0, k0 + rk_k - (kdim - 4));
        else ob -= (size_t)max(0, k0 + kr_k + KRH * h - (kdim - 1)) * p.ldb;
      }
      xa[h] = *reinterpret_cast<const float4*>(pa + oa);
      xb[h] = *reinterpret_cast<const float4*>(pb + ob);
    }
  };
  // the first D chunks' loads in flight before anything waits
#pragma unroll
  for (int c = 0; c < D; ++c)
    if (c < NCH) load(c, ra[c], rb[c]);
  const int fr = lane & 15, fk = lane >> 4;  // fragment row / column, k group of the lane
  // the epilogue's bias columns (FWD) and pre-BN values / coefficients (DA), loaded with the operands
  float bcol[JN];
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const int n = bn + wn * WC + j * 16 + fr;
    bcol[j] = (MODE == G32_FWD && p.bias && n < N) ? p.bias[n] : 0.f;
  }
  float zb[2][JN][4], cb[JN][4];
  if constexpr (FS == 2) {
    const size_t plane = (size_t)2 * p.ldc;
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int n = bn + wn * WC + j * 16 + fr;
      const size_t o = (size_t)tower * p.ldc + (n < N ? n : 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) cb[j][q] = f.coefb[q * plane + o];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = bm + wm * 32 + i * 16 + fk * 4 + r;
          zb[i][j][r] = f.zb[(size_t)(m < M ? m : 0) * p.ldc + (n < N ? n : 0)];
        }
    }
  }
  // ---- the A layer's BN coefficients (FWD), zero beyond its width
  const int Kc = NCH * kG32KC;  // staged k extent (<= kG32MaxK for FWD)
  if constexpr (BN_A) {
    if (from_sums) {
      cst.finish(f.in, t, NT, [&](int tw, int k, float, float, float inv, float sh) {
        if (k < Kc) {
          L.coef[(tw * 2 + 0) * kG32MaxK + k] = inv;
          L.coef[(tw * 2 + 1) * kG32MaxK + k] = sh;
        }
      });
      for (int i = t; i < 2 * (Kc - p.lda); i += NT) {
        const int tw = i / (Kc - p.lda), k = p.lda + i % (Kc - p.lda);
        L.coef[(tw * 2 + 0) * kG32MaxK + k] = 0.f;
        L.coef[(tw * 2 + 1) * kG32MaxK + k] = 0.f;
      }
    } else {
      const size_t plane = (size_t)2 * p.lda;
      for (int i = t; i < 2 * Kc; i += NT) {
        const int tw = i / Kc, k = i - tw * Kc;
        const bool ok = k < p.lda;
        L.coef[(tw * 2 + 0) * kG32MaxK + k] = ok ? p.coef[2 * plane + (size_t)tw * p.lda + k] : 0.f;
        L.coef[(tw * 2 + 1) * kG32MaxK + k] = ok ? p.coef[3 * plane + (size_t)tw * p.lda + k] : 0.f;
      }
    }
    __syncthreads();
  }
  const bool write_a = BN_A && p.a_out != nullptr && tx == 0;
  const bool write_a16 = BN_A && p.a_out16 != nullptr && tx == 0;
  // chunk c's registers -> LDS image buf (BN + ReLU on A for FWD; the ones column for DW)
  auto stage = [&](int c, float4 (&xa)[G], float4 (&xb)[G], int buf) {
    float* sa = L.img + buf * 2 * kG32Img;
    float* sb = sa + kG32Img;
    const int k0 = kofs(c);
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (edge || ((MODE == G32_DW || c == NCH - 1) && k0 + kG32KC > kend)) {  // uniform: edge tiles, tail chunk
#pragma unroll
      for (int h = 0; h < G; ++h) {
        if (!a_ok(c, h)) xa[h] = z4;
        if (!b_ok(c, h)) xb[h] = z4;
      }
    }
    if constexpr (BN_A) {
      const float* ci = &L.coef[(tower * 2) * kG32MaxK + k0 + rk_k];
      const float4 inv = *reinterpret_cast<const float4*>(ci);
      const float4 sh = *reinterpret_cast<const float4*>(ci + kG32MaxK);
      const int k = k0 + rk_k;
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float4& v = xa[h];
        v.x = fmaxf(bn_affine(v.x, inv.x, sh.x), 0.f);
        v.y = fmaxf(bn_affine(v.y, inv.y, sh.y), 0.f);
        v.z = fmaxf(bn_affine(v.z, inv.z, sh.z), 0.f);
        v.w = fmaxf(bn_affine(v.w, inv.w, sh.w), 0.f);
        const int r = bm + rk_r + RKH * h;
        if (write_a && r < M && k < p.lda) *reinterpret_cast<float4*>(p.a_out + (size_t)r * p.lda + k) = v;
        if (write_a16 && r < M && k < p.lda)  // the bf16 NT tile's rounding of the same activation
          *reinterpret_cast<uint2*>(p.a_out16 + (size_t)r * p.lda + k) = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
      }
    }
    if constexpr (MODE == G32_DW) {
      if (p.ones_row && bm + kr_c == Mload) {
#pragma unroll
        for (int h = 0; h < G; ++h)
          if (k0 + kr_k + KRH * h < kend) xa[h].x = 1.0f;
      }
    }
    if constexpr (kG32Split) {
      u16* pa = reinterpret_cast<u16*>(L.img) + buf * 2 * kS3Img;
      u16* pb = pa + kS3Img;
#pragma unroll
      for (int h = 0; h < G; ++h) {
        const int oa = A_RK ? (rk_r + RKH * h) * kS3LdRK + rk_k : (kr_k + KRH * h) * kS3LdKR + kr_c;
        const int ob = B_RK ? (rk_r + RKH * h) * kS3LdRK + rk_k : (kr_k + KRH * h) * kS3LdKR + kr_c;
        uint2 x0, x1, x2;
        split3(xa[h], x0, x1, x2);
        *reinterpret_cast<uint2*>(pa + oa) = x0;
        *reinterpret_cast<uint2*>(pa + kS3Plane + oa) = x1;
        *reinterpret_cast<uint2*>(pa + 2 * kS3Plane + oa) = x2;
        split3(xb[h], x0, x1, x2);
        *reinterpret_cast<uint2*>(pb + ob) = x0;
        *reinterpret_cast<uint2*>(pb + kS3Plane + ob) = x1;
        *reinterpret_cast<uint2*>(pb + 2 * kS3Plane + ob) = x2;
      }
      return;
    }
#pragma unroll
    for (int h = 0; h < G; ++h) {
      if constexpr (A_RK) *reinterpret_cast<float4*>(&sa[(rk_r + RKH * h) * kG32LdRK + rk_k]) = xa[h];
      else *reinterpret_cast<float4*>(&sa[(kr_k + KRH * h) * kG32LdKR + kr_c]) = xa[h];
      if constexpr (B_RK) *reinterpret_cast<float4*>(&sb[(rk_r + RKH * h) * kG32LdRK + rk_k]) = xb[h];
      else *reinterpret_cast<float4*>(&sb[(kr_k + KRH * h) * kG32LdKR + kr_c]) = xb[h];
    }
  };
  f32x4 acc[2][JN], acc2[2][JN];  // split: hh; the five small terms
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  G32_TL(f.tl_slot, 1);
  // ---- the chunk pipeline.  Iteration c: load chunk c + D, stage chunk c + 1 into the other LDS
  // image, the MFMAs of chunk c, one barrier.  Staging (the wait for c + 1's loads, BN + ReLU, the
  // LDS writes) and the MFMAs share a basic block, so the compiler interleaves them.  The image
  // staged at c + 1 was last read by the MFMAs of c - 1, which every wave finished before the barrier
  // ending iteration c - 1; the register set chunk c + D loads into held chunk c - 1 (ring of D + 1),
  // staged at iteration c - 2.  NCH is the chunk count (FWD / DA: exactly ceil(K / 32); DW: the
  // split's, chunks past its rows staged as zeros), so the unrolled pipeline is straight-line code
  // and the compiler's vmcnt waits are exact (a runtime chunk bound around the loads made it drain
  // every load at each branch merge).
  stage(0, ra[0], rb[0], 0);
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const float* sa = L.img + (c & 1) * 2 * kG32Img;
    const float* sb = sa + kG32Img;
    // the whole chunk (k past the operand's end staged as zeros: exact no-ops on the sums); 8-deep
    // steps, MFMA q of a step taking k = kk + 2 fk + q; step kk + 8's fragments read ahead of step
    // kk's MFMAs, so the LDS latency overlaps them
    auto frag = [&](int kk, float2 (&av)[2], float2 (&bv)[JN]) {
      const int k2 = kk + 2 * fk;
#ifdef DSSM_G32_NOFRAG  // diagnostics (wrong results): MFMA operands from registers only
      for (int i = 0; i < 2; ++i) av[i] = make_float2((float)k2, (float)i);
      for (int j = 0; j < JN; ++j) bv[j] = make_float2((float)j, (float)k2);
      return;
#endif
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = wm * 32 + i * 16 + fr;
        if constexpr (A_RK) av[i] = *reinterpret_cast<const float2*>(&sa[r * kG32LdRK + k2]);
        else av[i] = make_float2(sa[k2 * kG32LdKR + r], sa[(k2 + 1) * kG32LdKR + r]);
      }
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const int r = wn * WC + j * 16 + fr;
        if constexpr (B_RK) bv[j] = *reinterpret_cast<const float2*>(&sb[r * kG32LdRK + k2]);
        else bv[j] = make_float2(sb[k2 * kG32LdKR + r], sb[(k2 + 1) * kG32LdKR + r]);
      }
    };
#if DSSM_G32_FRAGALL
    // every fragment of the chunk read first (4 steps x (2 + JN) float2), behind them the next
    // chunk's loads and staging, then the MFMAs back to back
    float2 av[kG32KC / 8][2], bv[kG32KC / 8][JN];
#pragma unroll
    for (int st = 0; st < kG32KC / 8; ++st) frag(8 * st, av[st], bv[st]);
#endif
    if constexpr (kG32Split) {
      // the chunk's fragments: per operand block its three planes (RK: one ds_read_b128 of 8
      // consecutive k; KR: tn.h's transposing pair of ds_read_b64_tr_b16), read before the next
      // chunk's loads and staging, then the 6 x 2 x JN MFMAs term by term (independent chains
      // back to back)
      const u16* pa = reinterpret_cast<const u16*>(L.img) + (c & 1) * 2 * kS3Img;
      const u16* pb = pa + kS3Img;
      bf16x8 af[2][3], bf[JN][3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = wm * 32 + i * 16;
          if constexpr (A_RK)
            af[i][q] = *reinterpret_cast<const bf16x8*>(pa + q * kS3Plane + (r + fr) * kS3LdRK + 8 * fk);
          else
            af[i][q] = tn_frag(pa + q * kS3Plane, 0, r, lane);
        }
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int r = wn * WC + j * 16;
          if constexpr (B_RK)
            bf[j][q] = *reinterpret_cast<const bf16x8*>(pb + q * kS3Plane + (r + fr) * kS3LdRK + 8 * fk);
          else
            bf[j][q] = tn_frag(pb + q * kS3Plane, 0, r, lane);
        }
      }
#ifndef DSSM_G32_NOSTAGE
      if (c + D < NCH) load(c + D, ra[(c + D) % S], rb[(c + D) % S]);
      if (c + 1 < NCH) stage(c + 1, ra[(c + 1) % S], rb[(c + 1) % S], (c + 1) & 1);
#endif
      G32_TL(f.tl_slot, 2 + 2 * c);
#pragma unroll
      for (int u = 0; u < 6; ++u) {  // (a plane, b plane): hh, hm, mh, hl, lh, mm
        const int qa = u == 2 || u == 5 ? 1 : (u == 4 ? 2 : 0);
        const int qb = u == 1 || u == 5 ? 1 : (u == 3 ? 2 : 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < JN; ++j) {
            if (u == 0) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[j][0], acc[i][j], 0, 0, 0);
            else acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][qa], bf[j][qb], acc2[i][j], 0, 0, 0);
          }
      }
      __syncthreads();
      G32_TL(f.tl_slot, 3 + 2 * c);
      continue;
    }
#ifndef DSSM_G32_NOSTAGE  // diagnostics (wrong results): the loop without its loads and staging
    if (c + D < NCH) load(c + D, ra[(c + D) % S], rb[(c + D) % S]);
    if (c + 1 < NCH) stage(c + 1, ra[(c + 1) % S], rb[(c + 1) % S], (c + 1) & 1);
#endif
    G32_TL(f.tl_slot, 2 + 2 * c);
#if DSSM_G32_FRAGALL
#pragma unroll
    for (int st = 0; st < kG32KC / 8; ++st) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[st][i].x, bv[st][j].x, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[st][i].y, bv[st][j].y, acc[i][j], 0, 0, 0);
    }
#else
    float2 av[2], bv[JN];
    frag(0, av, bv);
#pragma unroll
    for (int kk = 0; kk < kG32KC; kk += 8) {
      float2 an[2], bnx[JN];
      if (kk + 8 < kG32KC) frag(kk + 8, an, bnx);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].x, bv[j].x, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].y, bv[j].y, acc[i][j], 0, 0, 0);
      if (kk + 8 < kG32KC) {
#pragma unroll
        for (int i = 0; i < 2; ++i) av[i] = an[i];
#pragma unroll
        for (int j = 0; j < JN; ++j) bv[j] = bnx[j];
      }
    }
#endif
#ifndef DSSM_G32_NOBAR  // diagnostics (wrong results): no barrier per chunk
    __syncthreads();
#endif
    G32_TL(f.tl_slot, 3 + 2 * c);
  }
  // ---- epilogue: C/D map col = lane & 15, row = (lane >> 4) * 4 + r.  The tile goes to LDS (the
  // chunk images are free after the loop's last barrier) and leaves as float4 row segments: whole
  // 256-B rows per 16 lanes instead of the accumulator layout's scattered 4-B stores.
  constexpr int kCld = 68;
  float* sC = L.img;  // [64][kCld]
  double cs[JN], cq[JN];
#pragma unroll
  for (int j = 0; j < JN; ++j) cs[j] = cq[j] = 0.0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int cl = wn * WC + j * 16 + fr, n = bn + cl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 32 + i * 16 + fk * 4 + r, m = bm + rl;
        const float v = kG32Split ? acc2[i][j][r] + acc[i][j][r] : acc[i][j][r];
        const float x = (n < N) ? v + bcol[j] : 0.f;  // DW / DA: no bias (bcol zero)
        sC[rl * kCld + cl] = x;
        if constexpr (FS == 1) {
          if (m < M) {
            cs[j] += x;
            cq[j] += (double)x * x;
          }
        } else if constexpr (FS == 2) {
          if (m < M) {
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
  __syncthreads();
  {
    float* out = MODE == G32_DW ? p.C + (size_t)tz * M * p.ldc : p.C;
    const int ncols = MODE == G32_DW ? min(64, N - bn) : min(64, p.ldc - bn);  // multiples of 4
#pragma unroll
    for (int k = 0; k < 1024 / NT; ++k) {
      const int idx = t + NT * k, r = idx >> 4, q = (idx & 15) * 4;
      if (bm + r < M && q < ncols)
        *reinterpret_cast<float4*>(out + (size_t)(bm + r) * p.ldc + bn + q) =
            *reinterpret_cast<const float4*>(&sC[r * kCld + q]);
    }
  }
  if constexpr (MODE == G32_DW) return;
  if constexpr (FS != 0) {
    // the wave's 4 row groups by shuffles, the two wm halves through LDS, one atomic per statistic
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      cs[j] = sum_xor32(sum_xor16(cs[j]));
      cq[j] = sum_xor32(sum_xor16(cq[j]));
    }
    if (wm == 1 && lane < 16) {
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        L.red[(wn * WC + j * 16 + lane) * 2] = cs[j];
        L.red[(wn * WC + j * 16 + lane) * 2 + 1] = cq[j];
      }
    }
    __syncthreads();
    if (wm == 0 && lane < 16) {
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const int c = wn * WC + j * 16 + lane, n = bn + c;
        if (n < N) {
          const double s1 = cs[j] + L.red[c * 2], s2 = cq[j] + L.red[c * 2 + 1];
          if (f.det.slab) {  // deterministic: this row tile's slab row, the other tower zero
            double* row = f.det.slab + (size_t)ty * 4 * p.ldc;
            det_st(row + (size_t)(tower * 2) * p.ldc + n, s1);
            det_st(row + (size_t)(tower * 2 + 1) * p.ldc + n, s2);
            det_st(row + (size_t)((1 - tower) * 2) * p.ldc + n, 0.0);
            det_st(row + (size_t)((1 - tower) * 2 + 1) * p.ldc + n, 0.0);
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
#if defined(DSSM_G32_TL) && defined(DSSM_G32_TL_HOST)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  G32_TL(f.tl_slot, 30);
  if (threadIdx.x == 0 && f.tl_slot >= 0) g_g32_tl[f.tl_slot][blockIdx.x & 2047][29] = __builtin_amdgcn_s_memtime();
#endif
}

}  // namespace
}  // namespace dssm
