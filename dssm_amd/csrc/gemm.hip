// Dense FC layers of the DSSM towers on gfx950 matrix cores (new_dssm.py:146-148 MatMul and its
// autodiff: dA = dZ*W^T, dW = A^T*dZ, db = colsum(dZ)).
//
// One 256-thread workgroup computes a 64x64 output tile; its 4 waves each own 32x32 = 2x2
// MFMA 16x16 tiles.  K is staged through LDS in 32-deep steps, both operands stored
// k-contiguous ([row][k] for A, [col][k] for B) so every MFMA fragment is one contiguous LDS
// read: bf16 -> v_mfma_f32_16x16x32_bf16 (8 elements per lane, one ds_read_b128 each),
// fp32 (parity mode) -> v_mfma_f32_16x16x4_f32 (exact f32 FMA chain).  fp32 accumulate.
//
// The bias gradient rides along with dW: the A^T operand gets a virtual all-ones row at
// m = K_in, so row K_in of the [K_in+1 x N] output (the arena's [W; b] block) is colsum(dZ).
#include "common.h"
#include "launch.h"

namespace dssm {
namespace {

constexpr int BM = 64, BN = 64, BK = 32;

template <typename T> struct LdsPad;
template <> struct LdsPad<u16> { static constexpr int v = 8; };    // 80-B rows
template <> struct LdsPad<float> { static constexpr int v = 4; };  // 144-B rows

template <typename T> __device__ __forceinline__ T zero_v() { return T(0); }
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
    for (int i = 0; i < 8; ++i) x[i] = (i < nv) ? p[i] : zero_v<T>();
  }
}

template <typename T, int MODE>
__global__ __launch_bounds__(256) void k_gemm(int M, int N, int K, const T* __restrict__ A,
                                              int lda, const T* __restrict__ B, int ldb,
                                              float* __restrict__ C, int ldc,
                                              const float* __restrict__ bias, int ones_row,
                                              int k_per_split) {
  constexpr bool TA = (MODE == GEMM_DW);
  constexpr bool TB = (MODE == GEMM_DA);
  constexpr int LDK = BK + LdsPad<T>::v;
  __shared__ __attribute__((aligned(16))) T sA[BM * LDK];
  __shared__ __attribute__((aligned(16))) T sB[BN * LDK];

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int bm = blockIdx.y * BM, bn = blockIdx.x * BN;
  const int kbeg = blockIdx.z * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int Mload = ones_row ? M - 1 : M;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    // ---- stage A tile (BM x BK) as sA[m][k]
    if constexpr (!TA) {
      const int m = t >> 2, kk = (t & 3) * 8;
      T x[8];
      const int gm = bm + m, gk = k0 + kk;
      const int nv = (gm < Mload) ? min(8, kend - gk) : 0;
      ld8(A + (size_t)gm * lda + gk, nv, x);
#pragma unroll
      for (int i = 0; i < 8; ++i) sA[m * LDK + kk + i] = x[i];
    } else {
      const int k = t >> 3, mm = (t & 7) * 8;
      T x[8];
      const int gk = k0 + k, gm = bm + mm;
      const int nv = (gk < kend) ? min(8, Mload - gm) : 0;
      ld8(A + (size_t)gk * lda + gm, nv, x);
      if (ones_row && gk < kend) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (gm + i == Mload) x[i] = one_v<T>();
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) sA[(mm + i) * LDK + k] = x[i];
    }
    // ---- stage B tile (BK x BN) as sB[n][k]
    if constexpr (!TB) {
      const int k = t >> 3, nn = (t & 7) * 8;
      T x[8];
      const int gk = k0 + k, gn = bn + nn;
      const int nv = (gk < kend) ? min(8, N - gn) : 0;
      ld8(B + (size_t)gk * ldb + gn, nv, x);
#pragma unroll
      for (int i = 0; i < 8; ++i) sB[(nn + i) * LDK + k] = x[i];
    } else {
      const int n = t >> 2, kk = (t & 3) * 8;
      T x[8];
      const int gn = bn + n, gk = k0 + kk;
      const int nv = (gn < N) ? min(8, kend - gk) : 0;
      ld8(B + (size_t)gn * ldb + gk, nv, x);
#pragma unroll
      for (int i = 0; i < 8; ++i) sB[n * LDK + kk + i] = x[i];
    }
    __syncthreads();

    if constexpr (sizeof(T) == 2) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(&sA[(wm * 32 + i * 16 + (lane & 15)) * LDK + 8 * (lane >> 4)]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(&sB[(wn * 32 + j * 16 + (lane & 15)) * LDK + 8 * (lane >> 4)]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        float af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = sA[(wm * 32 + i * 16 + (lane & 15)) * LDK + kk + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bfr[j] = sB[(wn * 32 + j * 16 + (lane & 15)) * LDK + kk + (lane >> 4)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- epilogue: C/D map col = lane&15, row = (lane>>4)*4 + r
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
          if (n < ldc) C[(size_t)m * ldc + n] = (n < N) ? v + bias[n] : 0.f;
        } else if constexpr (MODE == GEMM_DA) {
          if (n < ldc) C[(size_t)m * ldc + n] = (n < N) ? v : 0.f;
        } else {
          if (n < N) atomicAdd(&C[(size_t)m * ldc + n], v);
        }
      }
    }
  }
}

template <typename T>
hipError_t launch_t(GemmMode mode, int M, int N, int K, const T* A, int lda, const T* B, int ldb,
                    float* C, int ldc, const float* bias, bool ones_row, hipStream_t s) {
  dim3 block(256);
  if (mode == GEMM_DW) {
    const int tiles = cdiv(M, BM) * cdiv(N, BN);
    int splits = max(1, min(cdiv(1024, tiles), cdiv(K, 128)));
    int kps = cdiv(cdiv(K, splits), BK) * BK;
    splits = cdiv(K, kps);
    dim3 grid(cdiv(N, BN), cdiv(M, BM), splits);
    hipLaunchKernelGGL((k_gemm<T, GEMM_DW>), grid, block, 0, s, M, N, K, A, lda, B, ldb, C, ldc,
                       bias, ones_row ? 1 : 0, kps);
  } else {
    dim3 grid(cdiv(ldc, BN), cdiv(M, BM), 1);
    const int kps = cdiv(K, BK) * BK;
    if (mode == GEMM_FWD)
      hipLaunchKernelGGL((k_gemm<T, GEMM_FWD>), grid, block, 0, s, M, N, K, A, lda, B, ldb, C,
                         ldc, bias, 0, kps);
    else
      hipLaunchKernelGGL((k_gemm<T, GEMM_DA>), grid, block, 0, s, M, N, K, A, lda, B, ldb, C,
                         ldc, bias, 0, kps);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_gemm(GemmMode mode, bool bf16, int M, int N, int K, const void* A, int lda,
                       const void* B, int ldb, float* C, int ldc, const float* bias, bool ones_row,
                       hipStream_t s) {
  if (bf16)
    return launch_t<u16>(mode, M, N, K, (const u16*)A, lda, (const u16*)B, ldb, C, ldc, bias,
                         ones_row, s);
  return launch_t<float>(mode, M, N, K, (const float*)A, lda, (const float*)B, ldb, C, ldc, bias,
                         ones_row, s);
}

}  // namespace dssm
