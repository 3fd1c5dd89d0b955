// fp32 parity mode's fused dense layers (new_dssm.py:62-88, 138-148 and their autodiff, at the
// reference's own precision, new_dssm.py:111-114): the g32.h tiles on v_mfma_f32_16x16x4_f32.
//   k_g32_fwd : Z_l = relu(BN_{l-1}(Z_{l-1})) . W_l + b_l, the activation written for dW_l, Z_l's
//               per-tower column sums (fused statistics); + 1 workgroup materialising BN_{l-1}
//   k_g32_da  : dA_{l-1} = dZ_l . W_l^T with BN_{l-1}'s backward sums in the epilogue
//   k_g32_dw  : dW_l split-K slabs (when they do not ride in the BN-backward apply launch, bn.hip)
#define DSSM_G32_TL_HOST 1
#ifdef DSSM_G32_TL
namespace dssm {
__device__ unsigned long long g_g32_tl[4][2048][32];
}
#endif
#include "g32.h"
#include "launch.h"

namespace dssm {
namespace {

#ifndef DSSM_G32_WN
#define DSSM_G32_WN (DSSM_G32_SPLIT ? 2 : 4)  // forward / dA tiles: 2 = 4 waves of 32 x 32, 4 = 8 of 32 x 16
#endif
constexpr int kWN = DSSM_G32_WN;

template <int NCH>
__global__ __launch_bounds__(128 * kWN) void k_g32_fwd(G32Params p, G32Fuse f, int nx, int ntiles) {
  __shared__ G32Lds L;
  if ((int)blockIdx.x >= ntiles) {  // the extra workgroup: BN_{l-1}'s coef, batch moments, EMA
    if (f.in_from_sums) fs_materialize_fwd(f.in);
    return;
  }
  const int tile = xcd_tile(blockIdx.x, ntiles);  // a row block's column tiles on one XCD
  g32_body<G32_FWD, 1, NCH, kWN>(p, f, tile % nx, tile / nx, 0, L);
}

template <int NCH>
__global__ __launch_bounds__(128 * kWN) void k_g32_da(G32Params p, G32Fuse f, int nx, int ntiles) {
  __shared__ G32Lds L;
  const int tile = xcd_tile(blockIdx.x, ntiles);
  g32_body<G32_DA, 2, NCH, kWN>(p, f, tile % nx, tile / nx, 0, L);
}

// the kernel instance for K: NCH = ceil(K / 32) chunks (K <= kG32MaxK)
template <template <int> class KS>
void g32_by_chunks(int K, dim3 grid, hipStream_t s, const G32Params& p, const G32Fuse& f, int nx, int nt) {
  switch ((K + kG32KC - 1) / kG32KC) {
#define DSSM_G32_NCH(n) \
    case n: hipLaunchKernelGGL(KS<n>::fn, grid, dim3(128 * kWN), 0, s, p, f, nx, nt); break;
    DSSM_G32_NCH(1) DSSM_G32_NCH(2) DSSM_G32_NCH(3) DSSM_G32_NCH(4) DSSM_G32_NCH(5)
    DSSM_G32_NCH(6) DSSM_G32_NCH(7) DSSM_G32_NCH(8) DSSM_G32_NCH(9) DSSM_G32_NCH(10)
#undef DSSM_G32_NCH
    default: break;
  }
}
template <int n> struct FwdK { static constexpr auto fn = k_g32_fwd<n>; };
template <int n> struct DaK { static constexpr auto fn = k_g32_da<n>; };

__global__ __launch_bounds__(256) void k_g32_dw(G32Params p, int nx, int ny, int nblocks) {
  __shared__ G32Lds L;
  const int r = xcd_tile(blockIdx.x, nblocks);  // one batch-row chunk's tiles on one XCD
  G32Fuse f{};
  f.tl_slot = -1;
  g32_body<G32_DW, 0, kG32DwSplit / kG32KC>(p, f, r % nx, (r / nx) % ny, r / (nx * ny), L);
}

bool g32_det_fits(const G32Fuse& f, int ld) {
  return !f.det.slab || (f.det_rows <= f.det.cap && cdiv(ld, 64) <= kDetTiles);
}

}  // namespace

int g32_dw_splits(int rows) { return cdiv(rows, kG32DwSplit); }

hipError_t launch_g32_fwd(int M, int N, int K, const float* Z, int lda, const float* coef,
                          const BnSide* in_from_sums, int row_split, const float* W, int ldw, float* C,
                          int ldc, const float* bias, float* a_out, double* out_sum, hipStream_t s,
                          const DetAcc* det, uint16_t* a_out16) {
  if (K < 1 || K > kG32MaxK || K > lda || (lda % 4) || (ldw % 4) || (ldc % 4) || (K % 4) || (N % 4) || ldw < N ||
      (row_split % 64) || (!in_from_sums && !coef))
    return hipErrorInvalidValue;
  G32Params p{M, N, K, Z, lda, W, ldw, C, ldc, bias, a_out, coef, row_split, 0, 0};
  p.a_out16 = a_out16;
  G32Fuse f{};
  if (in_from_sums) {
    f.in_from_sums = 1;
    f.in = *in_from_sums;
  }
  f.out_sum = out_sum;
  if (det) f.det = *det;
  f.det_rows = cdiv(M, 64);
  f.tl_slot = N > 128 ? 0 : 1;
  if (!g32_det_fits(f, ldc)) return hipErrorInvalidValue;
  const int nx = cdiv(ldc, 64), ntiles = nx * cdiv(M, 64);
  g32_by_chunks<FwdK>(K, dim3(ntiles + (in_from_sums ? 1 : 0)), s, p, f, nx, ntiles);
  return hipGetLastError();
}

hipError_t launch_g32_dw(const G32Params& dw, hipStream_t s) {
  const int nx = cdiv(dw.N, 64), ny = cdiv(dw.M, 64), nz = cdiv(dw.K, dw.k_per_split);
  if (dw.k_per_split > kG32DwSplit) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_g32_dw, dim3(nx * ny * nz), dim3(256), 0, s, dw, nx, ny, nx * ny * nz);
  return hipGetLastError();
}

hipError_t launch_g32_pair(int M, int kin, int n, const float* dZ, int lddz, const float* W, int ldw,
                           float* dA, int ldda, const float* z_prev, const float* coef_prev, double* bsum_prev,
                           int row_split, const float* A_prev, int lda_prev, float* slab, float* gw, bool defer,
                           hipStream_t s, int* deferred_splits, G32Params* dw_out, const DetAcc* det) {
  if (n < 1 || n > kG32MaxK || n > lddz || (lddz % 4) || (ldw % 4) || ldw < n || (ldda % 4) || (lda_prev % 4) ||
      (n % 4) || (kin % 4) || lda_prev < kin || (row_split % 64))
    return hipErrorInvalidValue;
  // dA_{l-1} = dZ_l . W_l^T: W_l [kin x n] row-major is B^T, its rows k-contiguous
  const G32Params a{M, kin, n, dZ, lddz, W, ldw, dA, ldda, nullptr, nullptr, nullptr, row_split, 0, 0};
  G32Fuse f{};
  f.out_sum = bsum_prev;
  f.zb = z_prev;
  f.coefb = coef_prev;
  if (det) f.det = *det;
  f.det_rows = cdiv(M, 64);
  f.tl_slot = n > 128 ? 3 : 2;
  if (!g32_det_fits(f, ldda)) return hipErrorInvalidValue;
  const int nx = cdiv(ldda, 64), ntiles = nx * cdiv(M, 64);
  g32_by_chunks<DaK>(n, dim3(ntiles), s, a, f, nx, ntiles);
  // dW_l = [A_{l-1}; 1]^T . dZ_l over the batch rows in kG32DwSplit-row slabs: handed to the next
  // BN-backward apply launch (dw_out), or launched here
  const int nsplit = g32_dw_splits(M);
  const G32Params d{kin + 1, n, M, A_prev, lda_prev, dZ, lddz, nsplit > 1 ? slab : gw, n, nullptr, nullptr,
                    nullptr, 0, 1, kG32DwSplit};
  *deferred_splits = (defer && nsplit > 1) ? nsplit : 0;
  if (dw_out) {
    *dw_out = d;
    return hipGetLastError();
  }
  if (hipError_t e = launch_g32_dw(d, s)) return e;
  if (nsplit > 1 && !defer) return launch_splitk_reduce(slab, nsplit, (int64_t)(kin + 1) * n, gw, s);
  return hipGetLastError();
}

}  // namespace dssm

#ifdef DSSM_G32_TL
extern "C" int dssm_debug_g32_timeline(int slot, unsigned long long* out, int n) {
  if (slot < 0 || slot >= 4 || n > 2048) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dssm::g_g32_tl), sizeof(unsigned long long) * 32 * n,
                             sizeof(unsigned long long) * 32 * 2048 * slot) == hipSuccess ? 0 : -2;
}
#endif
