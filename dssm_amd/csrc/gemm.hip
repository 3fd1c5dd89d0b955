// Dense FC layers of the DSSM towers on gfx950 matrix cores (new_dssm.py:146-148 MatMul and its
// autodiff: dA = dZ*W^T, dW = A^T*dZ, db = colsum(dZ)).
//
// One 256-thread workgroup computes a 64x64 output tile; its 4 waves each own 32x32 = 2x2
// MFMA 16x16 tiles.  K is staged through a double-buffered LDS ring (64-deep for bf16, 32 for
// fp32) with the next step's global loads issued into registers before the current step's
// MFMAs (one barrier per K-step).  Both operands are stored k-contiguous ([row][k] for A,
// [col][k] for B) so every MFMA fragment is one contiguous LDS read: bf16 ->
// v_mfma_f32_16x16x32_bf16 (8 elements per lane, one ds_read_b128), fp32 (parity mode) ->
// v_mfma_f32_16x16x4_f32 (exact f32 FMA chain).  fp32 accumulate.
//
// dW is a split-K GEMM over the batch rows (K = R = 6144 at C2); each split writes a plain fp32
// partial slab and k_splitk_reduce sums the slabs in fixed order (deterministic, no atomics, no
// zero-init).  The bias gradient rides along: the A^T operand gets a virtual all-ones row at
// m = K_in, so row K_in of the [K_in+1 x N] output (the arena's [W; b] block) is colsum(dZ).
#include <cstdlib>
#include <type_traits>

#include "bnfuse.h"
#include "common.h"
#include "launch.h"
#include "tn.h"

namespace dssm {
namespace {

constexpr int BM = 64, BN = 64;

// Diagnostics build only (-DDSSM_WG_TL): per-workgroup start / end / phase stamps (s_memrealtime,
// 100 MHz) of the dense GEMM launches, read back by dssm_debug_wg_timeline (tools/wg_timeline.py).
#ifdef DSSM_WG_TL
constexpr int kTlStamps = 6;  // 0 start, 1 end; NT / pair tiles: 2 operands landed, 3 LDS images
                              // written, 4 MFMA done, 5 statistics published
__device__ unsigned long long g_wg_tl[4][2048][kTlStamps];
#define WG_TL(slot, idx)                                                                    \
  do {                                                                                      \
    if (threadIdx.x == 0)                                                                   \
      g_wg_tl[slot][(blockIdx.y * gridDim.x + blockIdx.x) & 2047][idx] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define WG_TL(slot, idx) \
  do {                   \
  } while (0)
#endif

template <typename T> struct Cfg;
template <> struct Cfg<u16> { static constexpr int BK = 64, PAD = 8; };    // 144-B LDS rows
template <> struct Cfg<float> { static constexpr int BK = 32, PAD = 4; };  // 144-B LDS rows

template <typename T> __device__ __forceinline__ T one_v();
template <> __device__ __forceinline__ float one_v<float>() { return 1.0f; }
template <> __device__ __forceinline__ u16 one_v<u16>() { return (u16)0x3f80; }

// Load 8 consecutive elements p[0..8) where only the first `nv` are in range.
template <typename T>
__device__ __forceinline__ void ld8(const T* p, int nv, T (&x)[8]) {
  if (nv >= 8) {
    if constexpr (sizeof(T) == 2) {
      uint4 a = *reinterpret_cast<const uint4*>(p);
      x[0] = a.x & 0xffff; x[1] = a.x >> 16; x[2] = a.y & 0xffff; x[3] = a.y >> 16;
      x[4] = a.z & 0xffff; x[5] = a.z >> 16; x[6] = a.w & 0xffff; x[7] = a.w >> 16;
    } else {
      float4 a = *reinterpret_cast<const float4*>(p);
      float4 b = *reinterpret_cast<const float4*>(p + 4);
      x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
      x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (i < nv) ? p[i] : T(0);
  }
}

// 8 contiguous elements into LDS (16-B aligned destination)
template <typename T>
__device__ __forceinline__ void st8(T* d, const T (&x)[8]) {
  if constexpr (sizeof(T) == 2) {
    uint4 a;
    a.x = (unsigned)x[0] | ((unsigned)x[1] << 16);
    a.y = (unsigned)x[2] | ((unsigned)x[3] << 16);
    a.z = (unsigned)x[4] | ((unsigned)x[5] << 16);
    a.w = (unsigned)x[6] | ((unsigned)x[7] << 16);
    *reinterpret_cast<uint4*>(d) = a;
  } else {
    *reinterpret_cast<float4*>(d) = make_float4(x[0], x[1], x[2], x[3]);
    *reinterpret_cast<float4*>(d + 4) = make_float4(x[4], x[5], x[6], x[7]);
  }
}

template <typename T, int MODE>
__global__ __launch_bounds__(256) void k_gemm(int M, int N, int K, const T* __restrict__ A,
                                              int lda, const T* __restrict__ B, int ldb,
                                              void* __restrict__ Cv, int ldc,
                                              const float* __restrict__ bias, int ones_row,
                                              int k_per_split, int relu,
                                              const void* __restrict__ maskv, int ldmask, int flags) {
  // relu (FWD): the layer's ReLU in the epilogue; mask (DA): dA zeroed where mask <= 0 (the ReLU
  // backward through the layer's input activation, ReluGrad).  flags (FWD / DA): bit 0 = C stored
  // as bf16 (RNE) instead of fp32, bit 1 = the mask is bf16 (the bf16 activation itself)
  const bool c_bf16 = MODE != GEMM_DW && (flags & 1);
  const bool mask_bf16 = (flags & 2) != 0;
  auto mask_pos = [&](size_t o) {
    return mask_bf16 ? bf2f(static_cast<const u16*>(maskv)[o]) > 0.f : static_cast<const float*>(maskv)[o] > 0.f;
  };
  const bool mask = maskv != nullptr;
  constexpr bool TA = (MODE == GEMM_DW);
  constexpr bool TB = (MODE == GEMM_DA);
  constexpr int BK = Cfg<T>::BK;
  constexpr int LDK = BK + Cfg<T>::PAD;
  constexpr int G = (BM * BK / 256) / 8;  // 8-element groups per thread per operand
  __shared__ __attribute__((aligned(16))) T sA[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) T sB[2][BN * LDK];

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  // XCD-grouped tile order over the whole grid (x fastest): consecutive tiles share a row block's
  // A panel (FWD / DA) or a split's batch-row chunk (DW), so they run on one XCD
  const int gx = gridDim.x, gxy = gridDim.x * gridDim.y;
  const int lin = blockIdx.x + gx * (blockIdx.y + gridDim.y * blockIdx.z);
  const int tile = xcd_tile(lin, gxy * gridDim.z);
  const int tbx = tile % gx, tby = (tile % gxy) / gx, tbz = tile / gxy;
  const int bm = tby * BM, bn = tbx * BN;
  const int kbeg = tbz * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int Mload = ones_row ? M - 1 : M;
  float bcol[2] = {0.f, 0.f};  // GEMM_FWD: the epilogue's bias columns, loaded ahead of the K loop
  if constexpr (MODE == GEMM_FWD) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = bn + wn * 32 + j * 16 + (lane & 15);
      bcol[j] = n < N ? bias[n] : 0.f;
    }
  }

  T ra[G][8], rb[G][8];
  auto load = [&](int k0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int e = t + 256 * g;
      if constexpr (!TA) {  // A[m][k]
        const int m = e / (BK / 8), kk = (e % (BK / 8)) * 8;
        const int gm = bm + m, gk = k0 + kk;
        ld8(A + (size_t)gm * lda + gk, (gm < Mload) ? min(8, kend - gk) : 0, ra[g]);
      } else {  // A^T: A[k][m]
        const int k = e / (BM / 8), mm = (e % (BM / 8)) * 8;
        const int gk = k0 + k, gm = bm + mm;
        ld8(A + (size_t)gk * lda + gm, (gk < kend) ? min(8, Mload - gm) : 0, ra[g]);
        if (ones_row && gk < kend) {
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if (gm + i == Mload) ra[g][i] = one_v<T>();
        }
      }
      if constexpr (!TB) {  // B[k][n]
        const int k = e / (BN / 8), nn = (e % (BN / 8)) * 8;
        const int gk = k0 + k, gn = bn + nn;
        ld8(B + (size_t)gk * ldb + gn, (gk < kend) ? min(8, N - gn) : 0, rb[g]);
      } else {  // B^T: B[n][k]
        const int n = e / (BK / 8), kk = (e % (BK / 8)) * 8;
        const int gn = bn + n, gk = k0 + kk;
        ld8(B + (size_t)gn * ldb + gk, (gn < N) ? min(8, kend - gk) : 0, rb[g]);
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int e = t + 256 * g;
      if constexpr (!TA) {
        const int m = e / (BK / 8), kk = (e % (BK / 8)) * 8;
        st8(&sA[buf][m * LDK + kk], ra[g]);
      } else {
        const int k = e / (BM / 8), mm = (e % (BM / 8)) * 8;
#pragma unroll
        for (int i = 0; i < 8; ++i) sA[buf][(mm + i) * LDK + k] = ra[g][i];
      }
      if constexpr (!TB) {
        const int k = e / (BN / 8), nn = (e % (BN / 8)) * 8;
#pragma unroll
        for (int i = 0; i < 8; ++i) sB[buf][(nn + i) * LDK + k] = rb[g][i];
      } else {
        const int n = e / (BK / 8), kk = (e % (BK / 8)) * 8;
        st8(&sB[buf][n * LDK + kk], rb[g]);
      }
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // GEMM_DA with a mask: the epilogue's 16 mask values per lane loaded behind the first K-step's
  // operands and kept as bits (bit (i*2+j)*4+r: keep), not loaded after the K loop
  unsigned keep_bits = 0xffffu;
  if (kbeg < kend) {
    load(kbeg);
    if constexpr (MODE == GEMM_DA) {
      if (mask) {
        keep_bits = 0u;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int n = bn + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int m = bm + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
              const bool k = m < M && n < N && mask_pos((size_t)m * ldmask + n);
              keep_bits |= (k ? 1u : 0u) << ((i * 2 + j) * 4 + r);
            }
          }
      }
    }
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += BK, buf ^= 1) {
    const bool more = k0 + BK < kend;
    if (more) load(k0 + BK);  // next step's global loads in flight during this step's MFMAs
    const T* a = sA[buf];
    const T* b = sB[buf];
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int ks = 0; ks < BK; ks += 32) {
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(&a[(wm * 32 + i * 16 + (lane & 15)) * LDK + ks + 8 * (lane >> 4)]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(&b[(wn * 32 + j * 16 + (lane & 15)) * LDK + ks + 8 * (lane >> 4)]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        float af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = a[(wm * 32 + i * 16 + (lane & 15)) * LDK + kk + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bfr[j] = b[(wn * 32 + j * 16 + (lane & 15)) * LDK + kk + (lane >> 4)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: C/D map col = lane&15, row = (lane>>4)*4 + r
  float* out = static_cast<float*>(Cv);
  if constexpr (MODE == GEMM_DW) out += (size_t)tbz * M * ldc;  // this split's slab
  u16* out16 = static_cast<u16*>(Cv);
  auto put = [&](size_t o, float x) {
    if (c_bf16) out16[o] = f2bf(x);
    else out[o] = x;
  };
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = bn + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = bm + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        const float v = acc[i][j][r];
        if (m >= M) continue;
        if constexpr (MODE == GEMM_FWD) {
          float x = v + bcol[j];
          if (relu) x = fmaxf(x, 0.f);
          if (n < ldc) put((size_t)m * ldc + n, (n < N) ? x : 0.f);
        } else if constexpr (MODE == GEMM_DA) {
          const bool keep = n < N && (kbeg < kend ? ((keep_bits >> ((i * 2 + j) * 4 + r)) & 1u)
                                                  : (!mask || mask_pos((size_t)m * ldmask + n)));
          if (n < ldc) put((size_t)m * ldc + n, keep ? v : 0.f);
        } else {
          if (n < N) out[(size_t)m * ldc + n] = v;
        }
      }
    }
  }
}

// ---- bf16 specialised GEMMs (perf mode) ------------------------------------------------------
// Shared geometry: 64x64 output tile, 4 waves (2x2 of 32x32), BK = 64, double-buffered LDS with
// the next K-step's global loads issued into registers before the current step's MFMAs.
// The tile bodies take their tile coordinates and LDS buffers explicitly so one launch can run
// tiles of two GEMMs (k_bwd_pair).
constexpr int NBK = 64, NLD = NBK + 8;  // k-contiguous tiles: [row][k], 144-B rows
constexpr int kNtMaxK = 512;            // BN-staged A: max K (LDS coefficient cache)
constexpr int kTileElems = 64 * NLD;    // one LDS operand buffer (u16)

// "NT": C[M x ldc] = A[M x K] . B where B is given k-contiguous as BT[N x ldb] (BT[n][k]).
// Forward (BT = transposed weight shadow, + bias) and dA (BT = the weight shadow itself).
// BN_A: A = relu(Z*inv + shift) from the fp32 pre-BN activations Z [M x lda] and the layer's
// BN coefficients (per row tower), converted to bf16 while staging; the column-tile-0 blocks
// also write that activation (bf16, ld lda) to a_out for the dW GEMM.
// FS (bnfuse.h): 1 = forward, add the output tile's per-column sum / sum of squares (+ bias) to
// f.out_sum; 2 = dA, add sum dy / sum dy*xhat of the output layer (mask and xhat from f.zb /
// f.coefb) to f.out_sum.  Tiles never straddle the tower boundary (row_split % 64 == 0).
struct NtParams {
  int M, N, K;
  const void* A;
  int lda;
  const float* coef;
  int row_split;
  const u16* BT;
  int ldb;
  float* C;
  int ldc;
  const float* bias;
  u16* a_out;
};
struct NtFuse {
  int in_from_sums;  // BN_A: derive the A operand's coefficients from `in`'s sums
  BnSide in;
  double* out_sum;   // [2 towers][2][ldc]
  const float* zb;   // FS == 2: pre-BN activations of the output layer [M x ldc]
  const float* coefb;  // FS == 2: its coefficients [4][2][ldc]
  int lds_epi;             // whole-K tiles: C staged through LDS, stored as 16-B row segments
  DetAcc det;              // deterministic mode: out_sum by slab rows + fixed-order last-arrival sum
  int det_rows;            // the launch's row tiles (arrivals per column tile)
  // BN-backward A (dA pair of the last layer): A = dZ_l formed while staging from dA_l (a.A, fp32),
  // the layer's pre-BN Z_l (zA), coefficients and backward sums (inb); dZ_l also written (bf16) by
  // the column-tile-0 workgroups to a.a_out for dW_l.  One extra workgroup: the forward's deferred
  // loss (loss_part) and BN_l's dgamma / dbeta.
  BnSide inb;
  const float* zA;
  const float* loss_part;
  int loss_blocks;
  float* loss_out;
};

template <bool BN_A, int FS>
__device__ __forceinline__ void nt_body(const NtParams& a, const NtFuse& f, int tx, int ty,
                                        u16* sA, u16* sB, float* sCoef, double* sRed) {
  const int M = a.M, N = a.N, K = a.K, lda = a.lda, ldb = a.ldb, ldc = a.ldc;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int bm = ty * 64, bn = tx * 64;
  const int tower = bm < a.row_split ? 0 : 1;
  const bool write_a = BN_A && a.a_out != nullptr && tx == 0;
  float bcol[2];  // the epilogue's bias columns, loaded ahead of the K loop
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = bn + wn * 32 + j * 16 + (lane & 15);
    bcol[j] = (a.bias && n < N) ? a.bias[n] : 0.f;
  }
  // BN_A: the layer's (inv, shift) for both towers staged in LDS once; the raw fp32 Z loads of
  // the next K-step stay in flight across this step's MFMAs and are transformed in store().
  if constexpr (BN_A) {
    if (FS == 1 && f.in_from_sums) {
      fs_coef_stage<(2 * kNtMaxK) / 256>(f.in, t, 256, [&](int tw, int k, float, float, float inv, float sh) {
        sCoef[(tw * 2 + 0) * kNtMaxK + k] = inv;
        sCoef[(tw * 2 + 1) * kNtMaxK + k] = sh;
      });
      if (tx == 0 && ty == 0) fs_materialize_fwd(f.in);
    } else {
      const size_t plane = (size_t)2 * lda;
      for (int i = t; i < 2 * lda; i += 256) {
        const int tw = i / lda, k = i - tw * lda;
        sCoef[(tw * 2 + 0) * kNtMaxK + k] = a.coef[2 * plane + (size_t)tw * lda + k];
        sCoef[(tw * 2 + 1) * kNtMaxK + k] = a.coef[3 * plane + (size_t)tw * lda + k];
      }
    }
    __syncthreads();
  }
  // FS == 2: the epilogue's pre-BN values and coefficients, loaded before the K loop
  float zb[2][2][4], cb[2][4];
  if constexpr (FS == 2) {
    const size_t plane = (size_t)2 * ldc;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = bn + wn * 32 + j * 16 + (lane & 15);
      const bool okn = n < N;
      const size_t o = (size_t)tower * ldc + (okn ? n : 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) cb[j][q] = f.coefb[q * plane + o];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = bm + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
          zb[i][j][r] = f.zb[(size_t)(m < M ? m : 0) * ldc + (okn ? n : 0)];
        }
    }
  }
  // thread -> (row, 8-wide k group) for the two staging groups of each operand
  int am[2], ak[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int e = t + 256 * g;
    am[g] = e >> 3;
    ak[g] = (e & 7) * 8;
  }
  uint4 ra[2], rb[2];
  float4 rz[2][2];
  int kcur = 0;
  auto load = [&](int k0) {
    kcur = k0;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int gm = bm + am[g], gk = k0 + ak[g];
      const bool ok = gm < M && gk < lda;
      if constexpr (BN_A) {
        const float* z = (const float*)a.A + (size_t)gm * lda + gk;
        rz[g][0] = ok ? *reinterpret_cast<const float4*>(z) : make_float4(0.f, 0.f, 0.f, 0.f);
        rz[g][1] = ok ? *reinterpret_cast<const float4*>(z + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        ra[g] = ok ? *reinterpret_cast<const uint4*>((const u16*)a.A + (size_t)gm * lda + gk)
                   : make_uint4(0u, 0u, 0u, 0u);
      }
      const int gn = bn + am[g];
      rb[g] = (gn < N && gk < ldb) ? *reinterpret_cast<const uint4*>(a.BT + (size_t)gn * ldb + gk)
                                   : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if constexpr (BN_A) {
        const int gm = bm + am[g], gk = kcur + ak[g];
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (gm < M && gk < lda) {
          const float* ci = &sCoef[((gm < a.row_split ? 0 : 1) * 2) * kNtMaxK + gk];
          const float* ch = ci + kNtMaxK;
          const float z[8] = {rz[g][0].x, rz[g][0].y, rz[g][0].z, rz[g][0].w,
                              rz[g][1].x, rz[g][1].y, rz[g][1].z, rz[g][1].w};
          float y[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) y[i] = fmaxf(bn_affine(z[i], ci[i], ch[i]), 0.f);
          v.x = pack2bf(y[0], y[1]); v.y = pack2bf(y[2], y[3]);
          v.z = pack2bf(y[4], y[5]); v.w = pack2bf(y[6], y[7]);
          if (write_a) *reinterpret_cast<uint4*>(a.a_out + (size_t)gm * lda + gk) = v;
        }
        ra[g] = v;
      }
      *reinterpret_cast<uint4*>(&sA[buf * kTileElems + am[g] * NLD + ak[g]]) = ra[g];
      *reinterpret_cast<uint4*>(&sB[buf * kTileElems + am[g] * NLD + ak[g]]) = rb[g];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(0);
  store(0);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += NBK, buf ^= 1) {
    const bool more = k0 + NBK < K;
    if (more) load(k0 + NBK);
    const u16* ta = sA + buf * kTileElems;
    const u16* tb = sB + buf * kTileElems;
#pragma unroll
    for (int ks = 0; ks < NBK; ks += 32) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(&ta[(wm * 32 + i * 16 + (lane & 15)) * NLD + ks + 8 * (lane >> 4)]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(&tb[(wn * 32 + j * 16 + (lane & 15)) * NLD + ks + 8 * (lane >> 4)]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }
  double cs[2] = {0.0, 0.0}, cq[2] = {0.0, 0.0};  // FS: this lane's column partials per j
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = bn + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = bm + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (m < M && n < ldc) {
          const float v = acc[i][j][r];
          const float x = (n < N) ? (a.bias ? v + bcol[j] : v) : 0.f;
          a.C[(size_t)m * ldc + n] = x;
          if constexpr (FS == 1) {
            cs[j] += x;
            cq[j] += (double)x * x;
          } else if constexpr (FS == 2) {
            const float z = zb[i][j][r];
            // same mask / xhat as bn.hip's bwd_terms: dy = dA where BN(z) > 0
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
    // reduce the 4 row groups of the wave, then the two wm halves through LDS
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      cs[j] = sum_xor32(sum_xor16(cs[j]));
      cq[j] = sum_xor32(sum_xor16(cq[j]));
    }
    if (wm == 1 && lane < 16) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        sRed[(wn * 32 + j * 16 + lane) * 2] = cs[j];
        sRed[(wn * 32 + j * 16 + lane) * 2 + 1] = cq[j];
      }
    }
    __syncthreads();
    if (wm == 0 && lane < 16) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = wn * 32 + j * 16 + lane, n = bn + c;
        if (n < N) {
          if (f.det.slab) {  // deterministic: this row tile's slab row, the other tower zero
            double* row = f.det.slab + (size_t)ty * 4 * ldc;
            det_st(row + (size_t)(tower * 2) * ldc + n, cs[j] + sRed[c * 2]);
            det_st(row + (size_t)(tower * 2 + 1) * ldc + n, cq[j] + sRed[c * 2 + 1]);
            det_st(row + (size_t)((1 - tower) * 2) * ldc + n, 0.0);
            det_st(row + (size_t)((1 - tower) * 2 + 1) * ldc + n, 0.0);
          } else {
            double* os = f.out_sum;
            atomic_add_f64(os + (size_t)(tower * 2) * ldc + n, cs[j] + sRed[c * 2]);
            atomic_add_f64(os + (size_t)(tower * 2 + 1) * ldc + n, cq[j] + sRed[c * 2 + 1]);
          }
        }
      }
    }
    if (f.det.slab) {
      __shared__ int s_det;
      det_publish(f.det, tx, ty, f.det_rows, ldc, bn, min(bn + 64, N), f.out_sum, &s_det);
    }
  }
}

template <bool BN_A, int FS>
__global__ __launch_bounds__(256) void k_gemm_nt(NtParams a, NtFuse f) {
  __shared__ __attribute__((aligned(16))) u16 sA[2 * kTileElems];
  __shared__ __attribute__((aligned(16))) u16 sB[2 * kTileElems];
  __shared__ float sCoef[BN_A ? 4 * kNtMaxK : 1];  // [tower][inv|shift][k]
  __shared__ double sRed[FS ? 128 : 1];
  nt_body<BN_A, FS>(a, f, blockIdx.x, blockIdx.y, sA, sB, sCoef, sRed);
}

// ---- whole-K NT GEMM (K <= 352): one load round per tile -----------------------------------
// (32 WM) x 64 output tile per (128 WM)-thread workgroup (2 WM waves = WM x 2 of 32 x 32), the
// tile's WHOLE K panel of A (32 WM rows) and BT (64 rows) staged once: every global load of the
// tile is issued before the first LDS write, so a tile costs one memory round trip instead of
// one per 64-deep K step; the A panel is converted to bf16 (with BN+ReLU when BN_A) on the way
// into LDS.  WM = 4: 128-row tiles, 512 threads (240 tiles at C2, one per CU); WM = 2: 64-row
// tiles, 256 threads, half the LDS, so two tiles share a CU and overlap their load / MFMA /
// epilogue chains.  FS epilogues as nt_body's (tiles never straddle the tower boundary:
// row_split % (32 WM) == 0).
constexpr int kWkMaxK = 352;
#ifndef DSSM_NT_COLMAP
#define DSSM_NT_COLMAP 1
#endif
#ifndef DSSM_WK_ROWS
#define DSSM_WK_ROWS 128
#endif
constexpr int kWkRows = DSSM_WK_ROWS;  // whole-K tile height of the forward / dA launches (64 or 128)
constexpr int kWkMaxG = kWkMaxK / 32;  // 8-element A groups per thread: (32 WM) rows x Kp/8 / (128 WM)
__host__ __device__ constexpr int wk_ldk(int Kp) { return Kp + 8; }
// LDS: A / B panels, BN coefficients, then the column-sum reduction.  The LDS epilogue stages a
// [32 WM][68] fp32 tile over the panels, so for small K the reduction moves past that tile.
// BN-backward A: the widest K it stages.  A K <= 320 instance (both hidden layers of C2 folded)
// measured slower: 18.1 us against 10.3 + 10.15 for the pair and apply it replaced, with 256 VGPRs
// and spills for the fp32 dA / Z panels, and +3.3 us in the apply that then hosts both dW sets.
constexpr int kBnbMaxK = 128;
__host__ __device__ inline size_t wk_red_offset(int Kp, int lds_epi, int WM = 4, int coef_rows = 4) {
  const size_t panels = (size_t)(32 * WM + 64) * wk_ldk(Kp) * 2 + (size_t)coef_rows * Kp * 4;
  const size_t epi = (size_t)32 * WM * 68 * 4;
  return (lds_epi && panels < epi) ? epi : panels;
}
__host__ __device__ inline size_t wk_smem_bytes(int Kp, int lds_epi = 0, int WM = 4, int coef_rows = 4) {
  return wk_red_offset(Kp, lds_epi, WM, coef_rows) + (size_t)WM * 64 * 2 * 8;
}

// BNBK > 0: the BN-backward A operand, K <= BNBK (its fp32 dA / Z groups sized for BNBK).
// KGA > 0: the A groups per thread for K <= 32 KGA (default: kWkMaxK's), so no load is issued past Kp.
template <bool BN_A, int FS, int WM = 4, int BNBK = 0, int KGA = 0>
__device__ __forceinline__ void nt_wk_body(const NtParams& a, const NtFuse& f, int tx, int ty,
                                           u16* wk_smem) {
  constexpr bool BNB = BNBK > 0;
  constexpr int NT = 128 * WM, ROWS = 32 * WM, BT = NT / 64;  // threads, tile rows, B threads / row
  const int M = a.M, N = a.N, K = a.K, lda = a.lda, ldb = a.ldb, ldc = a.ldc;
  const int Kp = (K + 31) & ~31, LDK = wk_ldk(Kp);
  u16* sA = wk_smem;                                     // [ROWS][LDK]
  u16* sB = sA + ROWS * LDK;                             // [64][LDK]
  // [tower][inv|shift][Kp]; BNB: [tower][mu|rstd|inv|shift|m1|m2][Kp]
  float* sCoef = reinterpret_cast<float*>(sB + 64 * LDK);
  double* sRed = reinterpret_cast<double*>(reinterpret_cast<char*>(wk_smem) +
                                           wk_red_offset(Kp, f.lds_epi, WM, BNB ? 12 : 4));  // [WM][64][2]
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int bm = ty * ROWS, bn = tx * 64;
  const int tower = bm < a.row_split ? 0 : 1;
  // the A operand's BN coefficient inputs (sums, gamma, beta) first: they return ahead of the
  // tile's bulk loads
  constexpr int NPC = (2 * kWkMaxK + NT - 1) / NT;
  FsCoefStage<NPC> cst;
  const bool from_sums = BN_A && FS == 1 && f.in_from_sums;
  if (from_sums) cst.load(f.in, t, NT);
  // ---- every global load of the tile, issued first.  A: 4 threads per row (groups t%4 + 4i),
  // B: BT threads per row (groups t%BT + BT i): 128-B row segments per 4 / BT lanes.  (Measured
  // neutral in round 3: 8 threads per row with whole-line instructions, and a per-column-tile
  // rotation of the K groups' issue order.)
  const int arow = t >> 2, ag0 = t & 3;
  const int brow = t / BT, bg0 = t % BT;
  // >= ceil(Kp/8 / 4), ceil(Kp/8 / BT)
  constexpr int NGA = BNB ? BNBK / 32 : (KGA ? KGA : kWkMaxG), NGB = (4 * NGA + BT - 1) / BT;
  // CM (BN_A, exact-K instances): the fp32 A panel by fixed column group -- thread t stages group
  // t % CG of rows t / CG + CP j -- so each thread reads its group's BN coefficients from LDS once
  // instead of once per group (4 ds_read_b128 per 8 elements, ~1 KiB of LDS reads per wave-group)
  // (BNB: six coefficient planes per group)
  constexpr bool CM = ((BN_A && KGA > 0) || BNB) && DSSM_NT_COLMAP;
  constexpr int CG = 4 * (BNB ? BNBK / 32 : (KGA ? KGA : 1)), CP = NT / CG, CR = (ROWS + CP - 1) / CP;
  constexpr int NFA = CM ? CR : NGA;
  float4 fa[NFA][2];  // fp32 A groups (BN_A: Z; BNB: dA)
  float4 fz[BNB ? NFA : 1][2];  // BNB: the A layer's Z
  uint4 ua[NGA];      // bf16 A groups
  uint4 ub[NGB];
  const int cg = t % CG, cr0 = t / CG;  // CM: this thread's column group and first row
  if constexpr (CM) {
    const int kg = cg * 8;
#pragma unroll
    for (int j = 0; j < CR; ++j) {
      const int row = cr0 + CP * j;
      const bool ok = row < ROWS && bm + row < M && kg < lda;
      const size_t off = ok ? (size_t)(bm + row) * lda + kg : 0;
      fa[j][0] = *reinterpret_cast<const float4*>((const float*)a.A + off);
      fa[j][1] = *reinterpret_cast<const float4*>((const float*)a.A + off + 4);
      if constexpr (BNB) {
        fz[j][0] = *reinterpret_cast<const float4*>(f.zA + off);
        fz[j][1] = *reinterpret_cast<const float4*>(f.zA + off + 4);
      }
    }
  }
  if constexpr (!CM) {
    const bool rok = bm + arow < M;
    const size_t rbase = (size_t)(rok ? bm + arow : 0) * lda;
#pragma unroll
    for (int i = 0; i < NGA; ++i) {
      const int kg = (ag0 + 4 * i) * 8;
      const size_t off = (rok && kg < lda) ? rbase + kg : 0;
      if constexpr (BN_A || BNB) {
        fa[i][0] = *reinterpret_cast<const float4*>((const float*)a.A + off);
        fa[i][1] = *reinterpret_cast<const float4*>((const float*)a.A + off + 4);
        if constexpr (BNB) {
          fz[i][0] = *reinterpret_cast<const float4*>(f.zA + off);
          fz[i][1] = *reinterpret_cast<const float4*>(f.zA + off + 4);
        }
      } else {
        ua[i] = *reinterpret_cast<const uint4*>((const u16*)a.A + off);
      }
    }
  }
#ifndef DSSM_DIAG_NT_NOB  // diagnostics build (wrong results): the B panel neither loaded nor staged
  {
    const bool bok = bn + brow < N;
    const size_t bbase = (size_t)(bok ? bn + brow : 0) * ldb;
#pragma unroll
    for (int i = 0; i < NGB; ++i) {
      const int kg = (bg0 + BT * i) * 8;
      ub[i] = *reinterpret_cast<const uint4*>(a.BT + ((bok && kg < ldb) ? bbase + kg : 0));
    }
  }
#endif
  // the epilogue's bias columns, loaded with the operands (a load issued after the MFMA loop would
  // put its latency into the epilogue)
  float bcol[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = bn + wn * 32 + j * 16 + (lane & 15);
    bcol[j] = (a.bias && n < N) ? a.bias[n] : 0.f;
  }
  float zb[2][2][4], cb[2][4];  // FS == 2: the epilogue's pre-BN values and coefficients
  auto load_epi = [&]() {
    const size_t plane = (size_t)2 * ldc;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = bn + wn * 32 + j * 16 + (lane & 15);
      const size_t o = (size_t)tower * ldc + (n < N ? n : 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) cb[j][q] = f.coefb[q * plane + o];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = bm + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
          zb[i][j][r] = f.zb[(size_t)(m < M ? m : 0) * ldc + (n < N ? n : 0)];
        }
    }
  };
  // with the operands (their latency hidden by the staging); BNB's fp32 panels leave no registers
  // for them there, so it loads them after the staging (hidden by the MFMA loop)
  if constexpr (FS == 2 && !BNB) load_epi();
#ifdef DSSM_WG_TL
  const int tl_slot = FS == 1 ? (a.N == 300 ? 0 : 1) : (a.K == 300 ? 3 : 2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  WG_TL(tl_slot, 2);
#endif
  // ---- BN coefficients of the A operand (from the sums or the materialised coefficients)
  if constexpr (BN_A) {
    if (FS == 1 && f.in_from_sums) {
      cst.finish(f.in, t, NT, [&](int tw, int k, float, float, float inv, float sh) {
        if (k < Kp) {
          sCoef[(tw * 2 + 0) * Kp + k] = inv;
          sCoef[(tw * 2 + 1) * Kp + k] = sh;
        }
      });
      for (int i = t; i < 2 * (Kp - lda); i += NT) {  // K pad beyond the stored width
        const int tw = i / (Kp - lda), k = lda + i % (Kp - lda);
        sCoef[(tw * 2 + 0) * Kp + k] = 0.f;
        sCoef[(tw * 2 + 1) * Kp + k] = 0.f;
      }
    } else {
      const size_t plane = (size_t)2 * lda;
      for (int i = t; i < 2 * Kp; i += NT) {
        const int tw = i / Kp, k = i - tw * Kp;
        const bool ok = k < lda;
        sCoef[(tw * 2 + 0) * Kp + k] = ok ? a.coef[2 * plane + (size_t)tw * lda + k] : 0.f;
        sCoef[(tw * 2 + 1) * Kp + k] = ok ? a.coef[3 * plane + (size_t)tw * lda + k] : 0.f;
      }
    }
    __syncthreads();
  }
  if constexpr (BNB) {  // the A layer's forward coefficients and backward means (pad columns zero)
    const BnSide& b = f.inb;
    const size_t plane = (size_t)2 * b.ld;
    for (int i = t; i < 2 * Kp; i += NT) {
      const int tw = i / Kp, k = i - tw * Kp;
      const bool ok = k < b.n;
      const size_t o = (size_t)tw * b.ld + (ok ? k : 0);
      float v[6];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = ok ? b.coef[q * plane + o] : 0.f;
      float m1 = 0.f, m2 = 0.f;
      if (ok) fs_dcoef(b, tw, k, m1, m2);
      v[4] = m1;
      v[5] = m2;
#pragma unroll
      for (int q = 0; q < 6; ++q) sCoef[(tw * 6 + q) * Kp + k] = v[q];
    }
    __syncthreads();
  }
  // ---- LDS images (bf16); out-of-range groups zeroed here, after every load was issued
  const bool write_a = (BN_A || BNB) && a.a_out != nullptr && tx == 0;
  if constexpr (CM) {
    const int kg = cg * 8;
    if (cr0 < CP && kg < Kp) {  // threads past CP * CG, and groups past Kp (BNB: K < BNBK), stage nothing
      constexpr int NC = BNB ? 6 : 2;  // BN_A: inv, shift; BNB: mu, rstd, inv, shift, m1, m2
      float cf[NC][8];
      const float* cp = &sCoef[(tower * NC) * Kp + kg];
#pragma unroll
      for (int u = 0; u < NC; ++u)
#pragma unroll
        for (int q = 0; q < 8; ++q) cf[u][q] = cp[u * Kp + q];
#pragma unroll
      for (int j = 0; j < CR; ++j) {
        const int row = cr0 + CP * j;
        if (row < ROWS) {
          uint4 v = make_uint4(0u, 0u, 0u, 0u);
          if (bm + row < M && kg < lda) {
            const float z[8] = {fa[j][0].x, fa[j][0].y, fa[j][0].z, fa[j][0].w,
                                fa[j][1].x, fa[j][1].y, fa[j][1].z, fa[j][1].w};
            float y[8];
            if constexpr (BNB) {  // bn.hip's k_bn_bwd_apply_fs arithmetic: dZ = inv * (dy - m1 - xhat * m2)
              const float zz[8] = {fz[j][0].x, fz[j][0].y, fz[j][0].z, fz[j][0].w,
                                   fz[j][1].x, fz[j][1].y, fz[j][1].z, fz[j][1].w};
#pragma unroll
              for (int q = 0; q < 8; ++q)
                y[q] = bn_bwd_dz(zz[q], z[q], cf[0][q], cf[1][q], cf[2][q], cf[3][q], cf[4][q], cf[5][q]);
            } else {
#pragma unroll
              for (int q = 0; q < 8; ++q) y[q] = fmaxf(bn_affine(z[q], cf[0][q], cf[1][q]), 0.f);
            }
            v.x = pack2bf(y[0], y[1]); v.y = pack2bf(y[2], y[3]);
            v.z = pack2bf(y[4], y[5]); v.w = pack2bf(y[6], y[7]);
            if (write_a) *reinterpret_cast<uint4*>(a.a_out + (size_t)(bm + row) * lda + kg) = v;
          }
          *reinterpret_cast<uint4*>(&sA[row * LDK + kg]) = v;
        }
      }
    }
  }
  if constexpr (!CM) {
    const bool rok = bm + arow < M;
#pragma unroll
    for (int i = 0; i < NGA; ++i) {
      const int kg = (ag0 + 4 * i) * 8;
      if (kg < Kp) {
        const bool ok = rok && kg < lda;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if constexpr (BN_A) {
          if (ok) {
            const float* ci = &sCoef[(tower * 2) * Kp + kg];
            const float* ch = ci + Kp;
            const float z[8] = {fa[i][0].x, fa[i][0].y, fa[i][0].z, fa[i][0].w,
                                fa[i][1].x, fa[i][1].y, fa[i][1].z, fa[i][1].w};
            float y[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) y[q] = fmaxf(bn_affine(z[q], ci[q], ch[q]), 0.f);
            v.x = pack2bf(y[0], y[1]); v.y = pack2bf(y[2], y[3]);
            v.z = pack2bf(y[4], y[5]); v.w = pack2bf(y[6], y[7]);
            if (write_a) *reinterpret_cast<uint4*>(a.a_out + (size_t)(bm + arow) * lda + kg) = v;
          }
        } else if constexpr (BNB) {
          if (ok) {  // bn.hip's k_bn_bwd_apply_fs arithmetic: dZ = inv * (dy - m1 - xhat * m2)
            const float* cm = &sCoef[(tower * 6) * Kp + kg];
            const float z[8] = {fz[i][0].x, fz[i][0].y, fz[i][0].z, fz[i][0].w,
                                fz[i][1].x, fz[i][1].y, fz[i][1].z, fz[i][1].w};
            const float d[8] = {fa[i][0].x, fa[i][0].y, fa[i][0].z, fa[i][0].w,
                                fa[i][1].x, fa[i][1].y, fa[i][1].z, fa[i][1].w};
            float y[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
              y[q] = bn_bwd_dz(z[q], d[q], cm[q], cm[Kp + q], cm[2 * Kp + q], cm[3 * Kp + q], cm[4 * Kp + q],
                               cm[5 * Kp + q]);
            v.x = pack2bf(y[0], y[1]); v.y = pack2bf(y[2], y[3]);
            v.z = pack2bf(y[4], y[5]); v.w = pack2bf(y[6], y[7]);
            if (write_a) *reinterpret_cast<uint4*>(a.a_out + (size_t)(bm + arow) * lda + kg) = v;
          }
        } else {
          v = ok ? ua[i] : make_uint4(0u, 0u, 0u, 0u);
        }
        *reinterpret_cast<uint4*>(&sA[arow * LDK + kg]) = v;
      }
    }
  }
#ifndef DSSM_DIAG_NT_NOB
  {
    const bool bok = bn + brow < N;
#pragma unroll
    for (int i = 0; i < NGB; ++i) {
      const int kg = (bg0 + BT * i) * 8;
      if (kg < Kp)
        *reinterpret_cast<uint4*>(&sB[brow * LDK + kg]) =
            (bok && kg < ldb) ? ub[i] : make_uint4(0u, 0u, 0u, 0u);
    }
  }
#endif
  if constexpr (FS == 2 && BNB) load_epi();
  __syncthreads();
#ifdef DSSM_WG_TL
  WG_TL(tl_slot, 3);
#endif
  // ---- MFMA over the whole K (fragments of the next k-step read ahead of this step's MFMAs)
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const u16* pa0 = sA + (wm * 32 + (lane & 15)) * LDK + 8 * (lane >> 4);
  const u16* pb0 = sB + (wn * 32 + (lane & 15)) * LDK + 8 * (lane >> 4);
  bf16x8 af[2], bfr[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) af[i] = *reinterpret_cast<const bf16x8*>(pa0 + i * 16 * LDK);
#pragma unroll
  for (int j = 0; j < 2; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(pb0 + j * 16 * LDK);
  for (int ks = 0; ks < Kp; ks += 32) {
    bf16x8 an[2], bnx[2];
    const int kn = ks + 32 < Kp ? ks + 32 : ks;
#pragma unroll
    for (int i = 0; i < 2; ++i) an[i] = *reinterpret_cast<const bf16x8*>(pa0 + i * 16 * LDK + kn);
#pragma unroll
    for (int j = 0; j < 2; ++j) bnx[j] = *reinterpret_cast<const bf16x8*>(pb0 + j * 16 * LDK + kn);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = an[i];
#pragma unroll
    for (int j = 0; j < 2; ++j) bfr[j] = bnx[j];
  }
#ifdef DSSM_WG_TL
  WG_TL(tl_slot, 4);
#endif
  // ---- epilogue
  // lds_epi: the tile's values go to LDS (the A panel's space, free once every wave is past its
  // last MFMA) and leave as 16-B row segments (full 256-B rows) instead of the accumulator
  // layout's 4-B scattered stores
  const bool lds_epi = f.lds_epi != 0;
  float* sC = reinterpret_cast<float*>(sA);  // [ROWS][68]
  constexpr int kCld = 68;
  if (lds_epi) __syncthreads();
  double cs[2] = {0.0, 0.0}, cq[2] = {0.0, 0.0};
  // The store target (LDS or global) and the tile's row bound are workgroup-uniform: one loop
  // instance per case, so the unrolled loop carries no per-element branch (the per-element form
  // compiled to 16 exec-mask regions and uniform branches); per j, the column bound per lane.
  // Each column's sums add its values in the same (i, r) order as before.
  auto epi = [&](auto lds_c, auto rows_c) {
    constexpr bool LDS = decltype(lds_c)::value, RF = decltype(rows_c)::value;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = bn + wn * 32 + j * 16 + (lane & 15);
      if (n < ldc) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = bm + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
            if (RF || m < M) {
              const float v = acc[i][j][r];
              const float x = (n < N) ? (a.bias ? v + bcol[j] : v) : 0.f;
              if constexpr (LDS)
                sC[(wm * 32 + i * 16 + (lane >> 4) * 4 + r) * kCld + wn * 32 + j * 16 + (lane & 15)] = x;
              else
                a.C[(size_t)m * ldc + n] = x;
              if constexpr (FS == 1) {
                cs[j] += x;
                cq[j] += (double)x * x;
              } else if constexpr (FS == 2) {
                const float z = zb[i][j][r];
                const float dy = (n < N && bn_affine(z, cb[j][2], cb[j][3]) > 0.f) ? x : 0.f;
                const float xh = (z - cb[j][0]) * cb[j][1];
                cs[j] += dy;
                cq[j] += (double)dy * xh;
              }
            }
          }
        }
      }
    }
  };
  {
    using T = std::true_type;
    using F = std::false_type;
    const bool rows_full = bm + ROWS <= M;
    if (lds_epi) {
      if (rows_full) epi(T{}, T{}); else epi(T{}, F{});
    } else {
      if (rows_full) epi(F{}, T{}); else epi(F{}, F{});
    }
  }
  if constexpr (FS != 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      cs[j] = sum_xor32(sum_xor16(cs[j]));
      cq[j] = sum_xor32(sum_xor16(cq[j]));
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = wn * 32 + j * 16 + lane;
        sRed[(wm * 64 + c) * 2] = cs[j];
        sRed[(wm * 64 + c) * 2 + 1] = cq[j];
      }
    }
    __syncthreads();
    if (t < 128) {
      const int c = t >> 1, st = t & 1, n = bn + c;
      if (n < N) {
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < WM; ++q) v += sRed[(q * 64 + c) * 2 + st];
        if (f.det.slab) {  // deterministic: this row tile's slab row, the other tower zero
          double* row = f.det.slab + (size_t)ty * 4 * ldc;
          det_st(row + (size_t)(tower * 2 + st) * ldc + n, v);
          det_st(row + (size_t)((1 - tower) * 2 + st) * ldc + n, 0.0);
        } else {
          atomic_add_f64(f.out_sum + (size_t)(tower * 2 + st) * ldc + n, v);
        }
      }
    }
    if (f.det.slab) {
      __shared__ int s_det;
      det_publish(f.det, tx, ty, f.det_rows, ldc, bn, min(bn + 64, N), f.out_sum, &s_det);
    }
  }
#ifdef DSSM_WG_TL
  WG_TL(tl_slot, 5);
#endif
  if (lds_epi) {
    __syncthreads();
    const int ncols = min(64, ldc - bn);  // multiple of 8: ldc = ldp8(N)
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // ROWS x 16 float4 = 4 per thread
      const int idx = t + NT * k, r = idx >> 4, q = (idx & 15) * 4;
      if (bm + r < M && q < ncols)
        *reinterpret_cast<float4*>(a.C + (size_t)(bm + r) * ldc + bn + q) =
            *reinterpret_cast<const float4*>(&sC[r * kCld + q]);
    }
  }
}


// Whole-K forward NT GEMM: blocks [0, ntiles) compute tiles (XCD-grouped row blocks); with the
// A coefficients derived from the sums, one extra block materialises them (coef, batch moments,
// EMA update) off the tiles' critical path.
template <bool BN_A, int FS, int WM, int KGA = 0>
__global__ __launch_bounds__(128 * WM) void k_gemm_nt_wk(NtParams a, NtFuse f, int nx, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) u16 wk_smem[];
  WG_TL(a.N == 300 ? 0 : 1, 0);
  if ((int)blockIdx.x >= ntiles) {
    if (BN_A && FS == 1 && f.in_from_sums) fs_materialize_fwd(f.in);
    return;
  }
  const int tile = xcd_tile(blockIdx.x, ntiles);
  nt_wk_body<BN_A, FS, WM, 0, KGA>(a, f, tile % nx, tile / nx, wk_smem);
#ifdef DSSM_WG_TL
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  WG_TL(a.N == 300 ? 0 : 1, 1);
#endif
}

__global__ __launch_bounds__(256) void k_gemm_tn(TnParams p) {
  __shared__ __attribute__((aligned(16))) u16 sA[2 * kTileElems];  // [k][m]
  __shared__ __attribute__((aligned(16))) u16 sB[2 * kTileElems];  // [k][n]
  tn_body(p, blockIdx.x, blockIdx.y, blockIdx.z, sA, sB);
}

// ---- whole-K-chunk TN (dW) tile: 128 (m) x 64 (n) per 512-thread workgroup ------------------
// The tile's whole chunk of kTwKc batch rows of both operands is loaded at once (one round
// trip) and staged as it lies in memory ([k][m], [k][n]); fragments by ds_read_b64_tr_b16.
// At C2: 16 splits of 384 rows x 15 tiles = 240 workgroups for dW2 (one per CU).
constexpr int kTwKc = 384;
constexpr int kTwLdA = 136, kTwLdB = 72;  // LDS row strides (u16)
__host__ __device__ inline size_t tw_smem_bytes() { return (size_t)kTwKc * (kTwLdA + kTwLdB) * 2; }

__device__ __forceinline__ bf16x8 tr_frag_s(const u16* tile, int ld, int row0, int col0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const u16* a0 = tile + (row0 + 8 * g + q) * ld + col0 + 4 * p;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a0);
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0 + 4 * ld));
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ void tn_wk_body(const TnParams& p, int tx, int ty, int tz, u16* smem) {
  const int M = p.M, N = p.N, lda = p.lda, ldb = p.ldb;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int bm = ty * 128, bn = tx * 64;
  const int kbeg = tz * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int Mload = p.ones_row ? M - 1 : M;
  u16* sA = smem;                    // [kTwKc][kTwLdA]  ([k][m])
  u16* sB = smem + kTwKc * kTwLdA;   // [kTwKc][kTwLdB]  ([k][n])
  // A: 16 threads per k-row (8 m each), rows (t>>4) + 32 i; B: 8 per row, rows (t>>3) + 64 i
  const int ar = t >> 4, am = bm + (t & 15) * 8;
  const int br = t >> 3, bnn = bn + (t & 7) * 8;
  constexpr int NA = kTwKc / 32, NB = kTwKc / 64;
  uint4 ra[NA], rb[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int k = kbeg + ar + 32 * i;
    const bool ok = k < kend && am < lda;
    ra[i] = *reinterpret_cast<const uint4*>(p.A + (ok ? (size_t)k * lda + am : 0));
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int k = kbeg + br + 64 * i;
    const bool ok = k < kend && bnn < ldb;
    rb[i] = *reinterpret_cast<const uint4*>(p.B + (ok ? (size_t)k * ldb + bnn : 0));
  }
  // stage; the group holding m == Mload gets the virtual ones column, m > Mload zeros
  const bool aedge = am + 8 > Mload;
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int k = kbeg + ar + 32 * i;
    uint4 v = (k < kend && am < lda) ? ra[i] : make_uint4(0u, 0u, 0u, 0u);
    if (aedge) {
      unsigned e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int m = am + q;
        const unsigned keep = m < Mload ? ((e[q >> 1] >> (16 * (q & 1))) & 0xffffu)
                                        : ((p.ones_row && m == Mload && k < kend) ? 0x3f80u : 0u);
        e[q >> 1] = (e[q >> 1] & ~(0xffffu << (16 * (q & 1)))) | (keep << (16 * (q & 1)));
      }
      v = make_uint4(e[0], e[1], e[2], e[3]);
    }
    *reinterpret_cast<uint4*>(&sA[(ar + 32 * i) * kTwLdA + (t & 15) * 8]) = v;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int k = kbeg + br + 64 * i;
    *reinterpret_cast<uint4*>(&sB[(br + 64 * i) * kTwLdB + (t & 7) * 8]) =
        (k < kend && bnn < ldb) ? rb[i] : make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kc = min(kTwKc, ((kend - kbeg) + 31) & ~31);
  for (int ks = 0; ks < kc; ks += 32) {
    bf16x8 af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = tr_frag_s(sA, kTwLdA, ks, wm * 32 + i * 16, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) bfr[j] = tr_frag_s(sB, kTwLdB, ks, wn * 32 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
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

// Whole-K backward pair, dA tiles only (the dW_l tiles ride in the next BN-backward apply launch).
// BNB: the A operand dZ_l formed from dA_l while staging (NtFuse::inb); block nt_blocks: the loss
// and BN_l's dgamma / dbeta.
template <int WM, int BNBK = 0, int KGA = 0>
__global__ __launch_bounds__(128 * WM) void k_pair_da_wk(NtParams a, NtFuse f, int nt_x, int nt_blocks) {
  extern __shared__ __attribute__((aligned(16))) u16 pw_smem[];
  WG_TL(a.K == 300 ? 3 : 2, 0);
  if constexpr (BNBK > 0) {
    if ((int)blockIdx.x >= nt_blocks) {
      if (f.loss_part) loss_reduce(f.loss_part, f.loss_blocks, f.inb.rows_q, f.loss_out);
      fs_materialize_bwd(f.inb);
      return;
    }
  }
  const int tile = xcd_tile(blockIdx.x, nt_blocks);
  nt_wk_body<false, 2, WM, BNBK, KGA>(a, f, tile % nt_x, tile / nt_x, pw_smem);
#ifdef DSSM_WG_TL
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  WG_TL(a.K == 300 ? 3 : 2, 1);
#endif
}

// Whole-K backward pair: the dA tiles (nt_wk_body, FS == 2) first, then the dW chunk tiles.
__global__ __launch_bounds__(512) void k_bwd_pair_wk(NtParams a, NtFuse f, int nt_x, int nt_blocks,
                                                     TnParams p, int tn_x, int tn_y) {
  extern __shared__ __attribute__((aligned(16))) u16 pw_smem[];
  const int b = blockIdx.x;
  WG_TL(a.K == 300 ? 3 : 2, 0);
  if (b < nt_blocks) {
    const int tile = xcd_tile(b, nt_blocks);
    nt_wk_body<false, 2, 4>(a, f, tile % nt_x, tile / nt_x, pw_smem);
  } else {
    // XCD grouping of the dW tiles needs the dA range to end on a multiple of 8
    const int nr = (int)gridDim.x - nt_blocks;
    const int r = (nt_blocks % 8) ? b - nt_blocks : xcd_tile(b - nt_blocks, nr);
    tn_wk_body(p, r % tn_x, (r / tn_x) % tn_y, r / (tn_x * tn_y), pw_smem);
  }
#ifdef DSSM_WG_TL
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  WG_TL(a.K == 300 ? 3 : 2, 1);
#endif
}

// One launch for the two backward GEMMs of layer l that both consume dZ_l: the dA tiles
// (critical path: they feed BN_{l-1}'s backward, with its sums fused) come first, then the
// split-K dW tiles.  Same 256-thread geometry and LDS buffers.
__global__ __launch_bounds__(256) void k_bwd_pair(NtParams a, NtFuse f, int nt_x, int nt_blocks,
                                                  TnParams p, int tn_x, int tn_y) {
  __shared__ __attribute__((aligned(16))) u16 sA[2 * kTileElems];
  __shared__ __attribute__((aligned(16))) u16 sB[2 * kTileElems];
  __shared__ double sRed[128];
  const int b = blockIdx.x;
  if (b < nt_blocks) {
    nt_body<false, 2>(a, f, b % nt_x, b / nt_x, sA, sB, nullptr, sRed);
  } else {
    const int r = b - nt_blocks;
    tn_body(p, r % tn_x, (r / tn_x) % tn_y, r / (tn_x * tn_y), sA, sB);
  }
}

// dst[i] = sum_s slab[s][i] in fixed split order.
__global__ __launch_bounds__(256) void k_splitk_reduce(const float* __restrict__ slab, int splits,
                                                       int64_t n, float* __restrict__ dst) {
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 acc = reinterpret_cast<const float4*>(slab)[i];
    for (int s = 1; s < splits; ++s) {
      const float4 v = reinterpret_cast<const float4*>(slab + (size_t)s * n)[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<float4*>(dst)[i] = acc;
  }
  // tail (n % 4)
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = n4 * 4 + threadIdx.x;
    float acc = slab[i];
    for (int s = 1; s < splits; ++s) acc += slab[(size_t)s * n + i];
    dst[i] = acc;
  }
}

int dw_splits(int M, int N, int K, int BK) {
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  int splits = max(1, min(cdiv(384, tiles), cdiv(K, 4 * BK)));
  splits = min(splits, kMaxDwSplits);
  const int kps = cdiv(cdiv(K, splits), BK) * BK;
  return cdiv(K, kps);
}

template <typename T>
hipError_t launch_t(GemmMode mode, int M, int N, int K, const T* A, int lda, const T* B, int ldb,
                    void* C, int ldc, const float* bias, bool ones_row, float* slab,
                    hipStream_t s, int* deferred_splits, int relu, const void* mask, int ldmask, int flags) {
  dim3 block(256);
  constexpr int BK = Cfg<T>::BK;
  if (mode == GEMM_DW) {
    const int splits = dw_splits(M, N, K, BK);
    const int kps = cdiv(cdiv(K, splits), BK) * BK;
    dim3 grid(cdiv(N, BN), cdiv(M, BM), splits);
    float* target = splits > 1 ? slab : static_cast<float*>(C);
    if constexpr (sizeof(T) == 2) {
      if ((lda % 8) == 0 && (ldb % 8) == 0)
        hipLaunchKernelGGL(k_gemm_tn, grid, block, 0, s,
                           TnParams{M, N, K, (const u16*)A, lda, (const u16*)B, ldb, target, ldc,
                                    ones_row ? 1 : 0, kps});
      else
        hipLaunchKernelGGL((k_gemm<T, GEMM_DW>), grid, block, 0, s, M, N, K, A, lda, B, ldb,
                           target, ldc, bias, ones_row ? 1 : 0, kps, 0, nullptr, 0, 0);
    } else {
      hipLaunchKernelGGL((k_gemm<T, GEMM_DW>), grid, block, 0, s, M, N, K, A, lda, B, ldb, target,
                         ldc, bias, ones_row ? 1 : 0, kps, 0, nullptr, 0, 0);
    }
    if (deferred_splits) *deferred_splits = splits > 1 ? splits : 0;
    if (splits > 1 && !deferred_splits) {
      const int64_t n = (int64_t)M * ldc;
      const int rg = (int)std::min<int64_t>((n / 4 + 255) / 256 + 1, 2048);
      hipLaunchKernelGGL(k_splitk_reduce, dim3(rg), block, 0, s, slab, splits, n, static_cast<float*>(C));
    }
  } else {
    dim3 grid(cdiv(ldc, BN), cdiv(M, BM), 1);
    const int kps = cdiv(K, BK) * BK;
    if (mode == GEMM_FWD)
      hipLaunchKernelGGL((k_gemm<T, GEMM_FWD>), grid, block, 0, s, M, N, K, A, lda, B, ldb, C,
                         ldc, bias, 0, kps, relu, nullptr, 0, flags);
    else
      hipLaunchKernelGGL((k_gemm<T, GEMM_DA>), grid, block, 0, s, M, N, K, A, lda, B, ldb, C,
                         ldc, bias, 0, kps, 0, mask, ldmask, flags);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_gemm_nt(int M, int N, int K, const void* A, int lda, bool bn_a,
                          const float* coef, int row_split, const uint16_t* BT, int ldb, float* C,
                          int ldc, const float* bias, uint16_t* a_out, hipStream_t s) {
  if ((lda % 8) || (ldb % 8) || K > lda || K > ldb || (bn_a && lda > kNtMaxK))
    return hipErrorInvalidValue;
  dim3 grid(cdiv(ldc, 64), cdiv(M, 64)), block(256);
  const NtParams a{M, N, K, A, lda, coef, row_split, (const u16*)BT, ldb, C, ldc, bias, (u16*)a_out};
  const NtFuse f{};
  if (bn_a)
    hipLaunchKernelGGL((k_gemm_nt<true, 0>), grid, block, 0, s, a, f);
  else
    hipLaunchKernelGGL((k_gemm_nt<false, 0>), grid, block, 0, s, a, f);
  return hipGetLastError();
}

// deterministic statistics: the launch's producer rows fit the slab, its column tiles the tickets
static bool det_fits(const NtFuse& f, int ld) {
  return !f.det.slab || (f.det_rows <= f.det.cap && cdiv(ld, 64) <= kDetTiles);
}

hipError_t launch_gemm_nt_fwd_fused(int M, int N, int K, const float* Z, int lda, const float* coef,
                                    const BnSide* in_from_sums, int row_split, const uint16_t* BT,
                                    int ldb, float* C, int ldc, const float* bias, uint16_t* a_out,
                                    double* out_sum, hipStream_t s, const DetAcc* det) {
  if ((lda % 8) || (ldb % 8) || K > lda || K > ldb || lda > kNtMaxK || (row_split % 64))
    return hipErrorInvalidValue;
  const NtParams a{M, N, K, Z, lda, coef, row_split, (const u16*)BT, ldb, C, ldc, bias, (u16*)a_out};
  NtFuse f{};
  if (in_from_sums) {
    f.in_from_sums = 1;
    f.in = *in_from_sums;
  }
  f.out_sum = out_sum;
  f.lds_epi = 1;  // measured: 14.4 (LDS-staged epilogue) vs 16.2 us per NT launch
  if (det) f.det = *det;
  if (K <= kWkMaxK && (row_split % 64) == 0) {
    const int Kp = (K + 31) & ~31;
    const int nx = cdiv(ldc, 64);
#define DSSM_NTWK(WM)                                                                         \
  {                                                                                           \
    f.det_rows = cdiv(M, 32 * WM);                                                            \
    if (!det_fits(f, ldc)) return hipErrorInvalidValue;                                       \
    const int ntiles = nx * cdiv(M, 32 * WM);                                                 \
    if (Kp == 320)                                                                            \
      hipLaunchKernelGGL((k_gemm_nt_wk<true, 1, WM, 10>), dim3(ntiles + (in_from_sums ? 1 : 0)), \
                         dim3(128 * WM), wk_smem_bytes(Kp, f.lds_epi, WM), s, a, f, nx, ntiles); \
    else                                                                                      \
    hipLaunchKernelGGL((k_gemm_nt_wk<true, 1, WM>), dim3(ntiles + (in_from_sums ? 1 : 0)),    \
                       dim3(128 * WM), wk_smem_bytes(Kp, f.lds_epi, WM), s, a, f, nx, ntiles); \
  }
    if (kWkRows == 64 || (row_split % 128)) DSSM_NTWK(2) else DSSM_NTWK(4)
#undef DSSM_NTWK
    return hipGetLastError();
  }
  f.det_rows = cdiv(M, 64);
  if (!det_fits(f, ldc)) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_gemm_nt<true, 1>), dim3(cdiv(ldc, 64), cdiv(M, 64)), dim3(256), 0, s, a, f);
  return hipGetLastError();
}

hipError_t launch_splitk_reduce(const float* slab, int splits, int64_t n, float* dst, hipStream_t s) {
  const int rg = (int)std::min<int64_t>((n / 4 + 255) / 256 + 1, 2048);
  hipLaunchKernelGGL(k_splitk_reduce, dim3(rg), dim3(256), 0, s, slab, splits, n, dst);
  return hipGetLastError();
}

// The last layer's pair with its BN backward folded into the dA tiles' A staging (no apply launch
// for BN_l): dZ_l = BN_l backward of (dA_l, Z_l) formed per element while staging, written bf16 to
// dZ_out by the column-tile-0 tiles for dW_l, whose split-K tiles are handed over (dw_out) to the next
// apply launch; one extra workgroup writes BN_l's dgamma / dbeta and the deferred loss.
hipError_t launch_bwd_pair_bnb(int M, int kin, int n, const float* dA_l, const float* Z_l, const BnSide& b,
                               uint16_t* dZ_out, int lddz, const uint16_t* W, int ldw, float* dA, int ldda,
                               const float* z_prev, const float* coef_prev, double* bsum_prev, int row_split,
                               const uint16_t* A_prev, int lda_prev, float* slab, float* gw, bool defer,
                               hipStream_t s, int* deferred_splits, TnParams* dw_out, const DetAcc* det,
                               const float* loss_part, int loss_blocks, float* loss_out) {
  if ((lddz % 8) || (ldw % 8) || (lda_prev % 8) || n > lddz || n > ldw || n > kBnbMaxK || (row_split % 128) ||
      lda_prev < kin || b.ld != lddz || b.n != n || !dw_out || kWkRows != 128)
    return hipErrorInvalidValue;
  const NtParams a{M, kin, n, dA_l, lddz, nullptr, row_split, W, ldw, dA, ldda, nullptr, dZ_out};
  NtFuse f{};
  f.out_sum = bsum_prev;
  f.zb = z_prev;
  f.coefb = coef_prev;
  f.lds_epi = 0;
  if (det) f.det = *det;
  f.inb = b;
  f.zA = Z_l;
  f.loss_part = loss_part;
  f.loss_blocks = loss_blocks;
  f.loss_out = loss_out;
  const int Kp = (n + 31) & ~31;
  const int nt_x = cdiv(ldda, 64), nt_blocks = nt_x * cdiv(M, 128);
  const int Mw = kin + 1;
  const int nsplit = cdiv(M, kTwKc);
  *dw_out = TnParams{Mw, n, M, A_prev, lda_prev, dZ_out, lddz, nsplit > 1 ? slab : gw, n, 1, kTwKc};
  f.det_rows = cdiv(M, 128);
  if (!det_fits(f, ldda)) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_pair_da_wk<4, kBnbMaxK>), dim3(nt_blocks + 1), dim3(512), wk_smem_bytes(Kp, 0, 4, 12), s, a,
                     f, nt_x, nt_blocks);
  *deferred_splits = (defer && nsplit > 1) ? nsplit : 0;
  return hipGetLastError();
}

hipError_t launch_bwd_pair(int M, int kin, int n, const uint16_t* dZ, int lddz, const uint16_t* W,
                           int ldw, float* dA, int ldda, const float* z_prev, const float* coef_prev,
                           double* bsum_prev, int row_split, const uint16_t* A_prev, int lda_prev,
                           float* slab, float* gw, bool defer, hipStream_t s, int* deferred_splits,
                           TnParams* dw_out, const DetAcc* det) {
  if ((lddz % 8) || (ldw % 8) || (lda_prev % 8) || n > lddz || n > ldw || (row_split % 64))
    return hipErrorInvalidValue;
  // dA_{l-1} = dZ_l . W_l^T (the weight shadow rows are k-contiguous), BN_{l-1} bwd sums fused
  const NtParams a{M, kin, n, dZ, lddz, nullptr, row_split, W, ldw, dA, ldda, nullptr, nullptr};
  NtFuse f{};
  f.out_sum = bsum_prev;
  f.zb = z_prev;
  f.coefb = coef_prev;
  f.lds_epi = 0;  // measured: 18.1 (register epilogue) vs 18.3 us (LDS-staged) per pair launch
  if (det) f.det = *det;
  if (n <= kWkMaxK && (row_split % 128) == 0 && lda_prev >= kin) {
    const int Kp = (n + 31) & ~31;
    const int nt_x = cdiv(ldda, 64), nt_blocks = nt_x * cdiv(M, 128);
    const int nt_blocks64 = nt_x * cdiv(M, 64);
    const int Mw = kin + 1;
    const int nsplit = cdiv(M, kTwKc);
    const TnParams p{Mw, n, M, A_prev, lda_prev, dZ, lddz, nsplit > 1 ? slab : gw, n, 1, kTwKc};
    if (dw_out) {
      // dA tiles alone (one round at one workgroup per CU); dW_l's tiles ride in the next
      // BN-backward apply launch (bn.hip), same splits and slabs.  Without defer the caller sums
      // the slabs (launch_splitk_reduce) after that launch.
      *dw_out = TnParams{Mw, n, M, A_prev, lda_prev, dZ, lddz, nsplit > 1 ? slab : gw, n, 1, kTwKc};
      f.det_rows = cdiv(M, kWkRows == 64 ? 64 : 128);
      if (!det_fits(f, ldda)) return hipErrorInvalidValue;
      if (kWkRows == 64)
        hipLaunchKernelGGL(k_pair_da_wk<2>, dim3(nt_blocks64), dim3(256), wk_smem_bytes(Kp, f.lds_epi, 2),
                           s, a, f, nt_x, nt_blocks64);
      else if (Kp == 320)  // every A load inside K (10 groups per thread)
        hipLaunchKernelGGL((k_pair_da_wk<4, 0, 10>), dim3(nt_blocks), dim3(512), wk_smem_bytes(Kp, f.lds_epi, 4),
                           s, a, f, nt_x, nt_blocks);
      else if (Kp == 128)
        hipLaunchKernelGGL((k_pair_da_wk<4, 0, 4>), dim3(nt_blocks), dim3(512), wk_smem_bytes(Kp, f.lds_epi, 4),
                           s, a, f, nt_x, nt_blocks);
      else
        hipLaunchKernelGGL(k_pair_da_wk<4>, dim3(nt_blocks), dim3(512), wk_smem_bytes(Kp, f.lds_epi, 4),
                           s, a, f, nt_x, nt_blocks);
      *deferred_splits = (defer && nsplit > 1) ? nsplit : 0;
      return hipGetLastError();
    }
    const int tn_x = cdiv(n, 64), tn_y = cdiv(Mw, 128);
    const int tn_blocks = tn_x * tn_y * nsplit;
    const size_t smem = std::max(wk_smem_bytes(Kp, f.lds_epi), tw_smem_bytes());
    f.det_rows = cdiv(M, 128);
    if (!det_fits(f, ldda)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_bwd_pair_wk, dim3(nt_blocks + tn_blocks), dim3(512), smem, s, a, f, nt_x,
                       nt_blocks, p, tn_x, tn_y);
    *deferred_splits = 0;
    if (nsplit > 1) {
      if (defer) {
        *deferred_splits = nsplit;
      } else {
        const int64_t cnt = (int64_t)Mw * n;
        const int rg = (int)std::min<int64_t>((cnt / 4 + 255) / 256 + 1, 2048);
        hipLaunchKernelGGL(k_splitk_reduce, dim3(rg), dim3(256), 0, s, slab, nsplit, cnt, gw);
      }
    }
    return hipGetLastError();
  }
  const int nt_x = cdiv(ldda, 64), nt_blocks = nt_x * cdiv(M, 64);
  // dW_l = [A_{l-1}; 1]^T . dZ_l, split-K slabs left for the Adam step to sum
  const int Mw = kin + 1;
  const int splits = dw_splits(Mw, n, M, NBK);
  const int kps = cdiv(cdiv(M, splits), NBK) * NBK;
  const int nsplit = cdiv(M, kps);
  const TnParams p{Mw, n, M, A_prev, lda_prev, dZ, lddz, nsplit > 1 ? slab : gw, n, 1, kps};
  const int tn_x = cdiv(n, BN), tn_y = cdiv(Mw, BM);
  const int tn_blocks = tn_x * tn_y * nsplit;
  f.det_rows = cdiv(M, 64);
  if (!det_fits(f, ldda)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bwd_pair, dim3(nt_blocks + tn_blocks), dim3(256), 0, s, a, f, nt_x,
                     nt_blocks, p, tn_x, tn_y);
  *deferred_splits = 0;
  if (nsplit > 1) {
    if (defer) {
      *deferred_splits = nsplit;  // summed inside the Adam step
    } else {
      const int64_t cnt = (int64_t)Mw * n;
      const int rg = (int)std::min<int64_t>((cnt / 4 + 255) / 256 + 1, 2048);
      hipLaunchKernelGGL(k_splitk_reduce, dim3(rg), dim3(256), 0, s, slab, nsplit, cnt, gw);
    }
  }
  return hipGetLastError();
}

size_t gemm_dw_slab_floats(int M, int N, int K, bool bf16) {
  int splits = dw_splits(M, N, K, bf16 ? Cfg<u16>::BK : Cfg<float>::BK);
  if (bf16) splits = std::max(splits, cdiv(K, kTwKc));  // the whole-K pair's chunk count
  else splits = std::max(splits, g32_dw_splits(K));      // the fp32 pair's (gemm32.hip)
  return splits > 1 ? (size_t)splits * M * N : 0;
}

hipError_t launch_gemm(GemmMode mode, bool bf16, int M, int N, int K, const void* A, int lda,
                       const void* B, int ldb, void* C, int ldc, const float* bias, bool ones_row,
                       float* slab, hipStream_t s, int* deferred_splits, int relu,
                       const void* mask, int ldmask, int flags) {
  if (bf16)
    return launch_t<u16>(mode, M, N, K, (const u16*)A, lda, (const u16*)B, ldb, C, ldc, bias,
                         ones_row, slab, s, deferred_splits, relu, mask, ldmask, flags);
  return launch_t<float>(mode, M, N, K, (const float*)A, lda, (const float*)B, ldb, C, ldc, bias,
                         ones_row, slab, s, deferred_splits, relu, mask, ldmask, flags);
}

}  // namespace dssm

#ifdef DSSM_WG_TL
extern "C" int dssm_debug_wg_timeline(int slot, unsigned long long* out, int n) {
  if (slot < 0 || slot >= 4 || n > 2048) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dssm::g_wg_tl), sizeof(unsigned long long) * dssm::kTlStamps * n,
                             sizeof(unsigned long long) * dssm::kTlStamps * 2048 * slot) == hipSuccess ? 0 : -2;
}
#endif
