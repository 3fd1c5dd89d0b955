// Functional backward entry points of the C-ABI: the per-op gradients a caller
// composes when it drives the layers itself (dssm_amd/api.py's functional ops, the multi-view
// towers) instead of the fused training-step plan.
//   dssm_spmm_csr_bwd_w : [dW1; db1] = [X | 1]^T dZ1 (TF's SparseTensorDenseMatMul gradient,
//                         dense), via the plan's CSC transpose + dW1 kernels
//   dssm_dense_bwd      : dA = dZ W^T and [dW; db] = [A | 1]^T dZ (tf.matmul + bias autodiff);
//                         _masked: dA zeroed where the layer input (a ReLU output) is <= 0
//   dssm_bn_relu_bwd    : batch-statistics batch_normalization + ReLU backward (new_dssm.py:62-88)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/dssm.h"
#include "common.h"
#include "launch.h"

namespace dssm {
int report_error(int code, const char* msg);
bool adam_probe_begin(hipStream_t s);  // rnn.hip
void adam_probe_end(hipStream_t s);
}

namespace {

int oerr(int code, const char* m) { return dssm::report_error(code, m); }

int hip_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DSSM_OK : oerr(DSSM_E_HIP, hipGetErrorString(e));
}

struct SpmmWs {
  size_t scratch, col_ptr, row, val, col, total;
};

SpmmWs spmm_ws(int rows, int D, int max_nnz) {
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  SpmmWs w{};
  size_t o = 0;
  w.scratch = o;
  o += al(dssm::csc_scratch_ints(D, rows, max_nnz) * 4);
  w.col_ptr = o;
  o += al((size_t)(D + 2) * 4);
  const size_t ent = (size_t)max_nnz + rows;
  w.row = o;
  o += al(ent * 4);
  w.val = o;
  o += al(ent * 4);
  w.col = o;
  o += al(ent * 4);
  w.total = o;
  return w;
}

// Column sums of the batch-norm backward: dbeta = sum dy, dgamma = sum dy * xhat (dy through the
// ReLU mask).  One block per 64 columns, 4 row groups reduced through LDS (fixed order).
__global__ __launch_bounds__(256) void k_bnr_bwd_sums(const float* __restrict__ Z, int ldz, int rows,
                                                      int n, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ var, float eps, int relu,
                                                      const float* __restrict__ dout, int ldd,
                                                      float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float s1[4][64], s2[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), grp = threadIdx.x >> 6;
  float a = 0.f, b = 0.f;
  if (c < n) {
    const float mu = mean[c], rstd = 1.0f / sqrtf(var[c] + eps), gm = gamma[c], bt = beta[c];
    for (int r = grp; r < rows; r += 4) {
      const float xh = (Z[(size_t)r * ldz + c] - mu) * rstd;
      float dy = dout[(size_t)r * ldd + c];
      if (relu && !(gm * xh + bt > 0.f)) dy = 0.f;
      a += dy;
      b += dy * xh;
    }
  }
  s1[grp][threadIdx.x & 63] = a;
  s2[grp][threadIdx.x & 63] = b;
  __syncthreads();
  if (grp == 0 && c < n) {
    const int l = threadIdx.x;
    dbeta[c] = s1[0][l] + s1[1][l] + s1[2][l] + s1[3][l];
    dgamma[c] = s2[0][l] + s2[1][l] + s2[2][l] + s2[3][l];
  }
}

// dz = gamma * rstd * (dy - mean(dy) - xhat * mean(dy * xhat))
__global__ __launch_bounds__(256) void k_bnr_bwd_apply(const float* __restrict__ Z, int ldz, int rows,
                                                       int n, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ var, float eps, int relu,
                                                       const float* __restrict__ dout, int ldd,
                                                       const float* __restrict__ dgamma,
                                                       const float* __restrict__ dbeta,
                                                       float* __restrict__ dz, int lddz) {
  const int64_t total = (int64_t)rows * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / n), c = (int)(i - (int64_t)r * n);
    const float rstd = 1.0f / sqrtf(var[c] + eps), gm = gamma[c];
    const float xh = (Z[(size_t)r * ldz + c] - mean[c]) * rstd;
    float dy = dout[(size_t)r * ldd + c];
    if (relu && !(gm * xh + beta[c] > 0.f)) dy = 0.f;
    const float m1 = dbeta[c] / rows, m2 = dgamma[c] / rows;
    dz[(size_t)r * lddz + c] = gm * rstd * (dy - m1 - xh * m2);
  }
}

__global__ void k_rows_gather(const float* __restrict__ src, int lds, const int* __restrict__ map, int n,
                              int cols, float* __restrict__ dst, int ldd) {
  const int64_t total = (int64_t)n * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i - (int64_t)r * cols);
    dst[(size_t)r * ldd + c] = src[(size_t)map[r] * lds + c];
  }
}

__global__ void k_rows_scatter_add(const float* __restrict__ src, int lds, const int* __restrict__ map,
                                   int n, int cols, float* __restrict__ dst, int ldd) {
  using gfloat = __attribute__((address_space(1))) float;
  const int64_t total = (int64_t)n * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i - (int64_t)r * cols);
    __hip_atomic_fetch_add((gfloat*)(dst + (size_t)map[r] * ldd + c), src[(size_t)r * lds + c],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// dst[r] = scale * sum of src rows idx[offs[r] .. offs[r+1]) in list order (the scatter-add's
// inverse: fixed order, no atomics, no clearing pass); with mask, zero where mask[r] <= 0 (ReluGrad)
template <typename TD>
__global__ void k_rows_gather_sum(const float* __restrict__ src, int lds, const int* __restrict__ offs,
                                  const int* __restrict__ idx, int n, int cols, float scale,
                                  const float* __restrict__ mask, int ldm, TD* __restrict__ dst, int ldd) {
  const int64_t total = (int64_t)n * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i - (int64_t)r * cols);
    float acc = 0.f;
    for (int j = offs[r]; j < offs[r + 1]; ++j) acc += src[(size_t)idx[j] * lds + c];
    acc *= scale;
    if (mask && !(mask[(size_t)r * ldm + c] > 0.f)) acc = 0.f;
    dst[(size_t)r * ldd + c] = from_f<TD>(acc);
  }
}

__global__ void k_relu(const float* __restrict__ x, int ldx, int rows, int cols, float* __restrict__ y,
                       int ldy) {
  const int64_t total = (int64_t)rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i - (int64_t)r * cols);
    y[(size_t)r * ldy + c] = fmaxf(x[(size_t)r * ldx + c], 0.f);
  }
}

// ReLU'(0) = 0 (TF1.x ReluGrad): dx = y > 0 ? dy : 0
__global__ void k_relu_bwd(const float* __restrict__ y, int ldy, const float* __restrict__ dy, int lddy,
                           int rows, int cols, float* __restrict__ dx, int lddx) {
  const int64_t total = (int64_t)rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i - (int64_t)r * cols);
    dx[(size_t)r * lddx + c] = y[(size_t)r * ldy + c] > 0.f ? dy[(size_t)r * lddy + c] : 0.f;
  }
}

int ew_grid(int64_t total) { return (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 2048)); }

}  // namespace

extern "C" {

int dssm_rows_gather(const float* src, int lds, const int32_t* map, int n, int cols, float* dst, int ldd,
                     void* stream) {
  if (!src || !map || !dst || n < 0 || cols < 0 || lds < cols || ldd < cols)
    return oerr(DSSM_E_INVALID, "rows_gather: bad argument");
  hipLaunchKernelGGL(k_rows_gather, dim3(ew_grid((int64_t)n * cols)), dim3(256), 0, (hipStream_t)stream, src,
                     lds, map, n, cols, dst, ldd);
  return hip_status();
}

int dssm_rows_scatter_add(const float* src, int lds, const int32_t* map, int n, int cols, float* dst,
                          int ldd, int dst_rows, void* stream) {
  if (!src || !map || !dst || n < 0 || cols < 0 || lds < cols || ldd < cols || dst_rows < 0)
    return oerr(DSSM_E_INVALID, "rows_scatter_add: bad argument");
  hipStream_t s = (hipStream_t)stream;
  if (zero_bytes_async(dst, sizeof(float) * (size_t)dst_rows * ldd, s) != hipSuccess)
    return oerr(DSSM_E_HIP, "rows_scatter_add: zero fill");
  hipLaunchKernelGGL(k_rows_scatter_add, dim3(ew_grid((int64_t)n * cols)), dim3(256), 0, s, src, lds, map, n,
                     cols, dst, ldd);
  return hip_status();
}

int dssm_rows_gather_sum_ex(const float* src, int lds, const int32_t* offs, const int32_t* idx, int n, int cols,
                            float scale, const float* mask, int ldm, void* dst, int dst_dtype, int ldd,
                            void* stream) {
  if (!src || !offs || !idx || !dst || n < 0 || cols < 0 || lds < cols || ldd < cols || (mask && ldm < cols) ||
      (dst_dtype != DSSM_F32 && dst_dtype != DSSM_BF16))
    return oerr(DSSM_E_INVALID, "rows_gather_sum: bad argument");
  if (dst_dtype == DSSM_BF16)
    hipLaunchKernelGGL(k_rows_gather_sum<u16>, dim3(ew_grid((int64_t)n * cols)), dim3(256), 0, (hipStream_t)stream,
                       src, lds, offs, idx, n, cols, scale, mask, ldm, static_cast<u16*>(dst), ldd);
  else
    hipLaunchKernelGGL(k_rows_gather_sum<float>, dim3(ew_grid((int64_t)n * cols)), dim3(256), 0,
                       (hipStream_t)stream, src, lds, offs, idx, n, cols, scale, mask, ldm, static_cast<float*>(dst),
                       ldd);
  return hip_status();
}

int dssm_rows_gather_sum(const float* src, int lds, const int32_t* offs, const int32_t* idx, int n, int cols,
                         float scale, const float* mask, int ldm, float* dst, int ldd, void* stream) {
  return dssm_rows_gather_sum_ex(src, lds, offs, idx, n, cols, scale, mask, ldm, dst, DSSM_F32, ldd, stream);
}

int dssm_relu(const float* x, int ldx, int rows, int cols, float* y, int ldy, void* stream) {
  if (!x || !y || rows < 0 || cols < 0 || ldx < cols || ldy < cols) return oerr(DSSM_E_INVALID, "relu: bad argument");
  hipLaunchKernelGGL(k_relu, dim3(ew_grid((int64_t)rows * cols)), dim3(256), 0, (hipStream_t)stream, x, ldx,
                     rows, cols, y, ldy);
  return hip_status();
}

int dssm_relu_bwd(const float* y, int ldy, const float* dy, int lddy, int rows, int cols, float* dx, int lddx,
                  void* stream) {
  if (!y || !dy || !dx || rows < 0 || cols < 0 || ldy < cols || lddy < cols || lddx < cols)
    return oerr(DSSM_E_INVALID, "relu_bwd: bad argument");
  hipLaunchKernelGGL(k_relu_bwd, dim3(ew_grid((int64_t)rows * cols)), dim3(256), 0, (hipStream_t)stream, y,
                     ldy, dy, lddy, rows, cols, dx, lddx);
  return hip_status();
}


size_t dssm_spmm_bwd_ws_bytes(int rows, int D, int max_nnz) {
  if (rows <= 0 || D <= 0 || max_nnz < 0) return 0;
  return spmm_ws(rows, D, max_nnz).total;
}

int dssm_spmm_csr_bwd_w(const int32_t* indptr, const int32_t* indices, const float* values, int rows,
                        int D, int max_nnz, const void* dZ, int dz_dtype, int lddz, int n, float* dWb,
                        void* ws, void* stream) {
  if (!indptr || !dZ || !dWb || !ws || rows <= 0 || D <= 0 || n <= 0 || lddz < n || (lddz % 8) ||
      (max_nnz && (!indices || !values)))
    return oerr(DSSM_E_INVALID, "spmm_csr_bwd_w: bad argument (lddz must be a multiple of 8)");
  hipStream_t s = (hipStream_t)stream;
  const SpmmWs w = spmm_ws(rows, D, max_nnz);
  char* b = static_cast<char*>(ws);
  int* scratch = reinterpret_cast<int*>(b + w.scratch);
  int* col_ptr = reinterpret_cast<int*>(b + w.col_ptr);
  int* crow = reinterpret_cast<int*>(b + w.row);
  float* cval = reinterpret_cast<float*>(b + w.val);
  int* ccol = reinterpret_cast<int*>(b + w.col);
  const bool rank = dssm::csc_rank_supported(D);
  hipError_t e = dssm::launch_csc_build(indptr, indices, values, rows, D, max_nnz, scratch, col_ptr, crow,
                                        cval, ccol, s, nullptr, 0, rank, false);
  if (e == hipSuccess)
    e = dssm::launch_dw1(col_ptr, crow, cval, ccol, D, rows, max_nnz, dZ, dz_dtype == DSSM_BF16, lddz, n,
                         dWb, true, s, rank ? scratch : nullptr);
  return e == hipSuccess ? DSSM_OK : oerr(DSSM_E_HIP, hipGetErrorString(e));
}

int dssm_csc_transpose(const int32_t* indptr, const int32_t* indices, const float* values, int rows, int D,
                       int max_nnz, int row_order, int32_t* col_ptr, int32_t* csc_row, float* csc_val,
                       int32_t* csc_col, void* ws, void* stream) {
  if (!indptr || !col_ptr || !csc_row || !csc_val || !csc_col || !ws || rows <= 0 || D <= 0 || max_nnz < 0 ||
      (max_nnz && (!indices || !values)))
    return oerr(DSSM_E_INVALID, "csc_transpose: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const SpmmWs w = spmm_ws(rows, D, max_nnz);
  char* b = static_cast<char*>(ws);
  int* scratch = reinterpret_cast<int*>(b + w.scratch);
  // row order: the transpose lands in the workspace's arrays, the row sort writes the caller's
  int* srow = row_order ? reinterpret_cast<int*>(b + w.row) : nullptr;
  float* sval = row_order ? reinterpret_cast<float*>(b + w.val) : nullptr;
  const hipError_t e = dssm::launch_csc_build(indptr, indices, values, rows, D, max_nnz, scratch, col_ptr, csc_row,
                                              csc_val, csc_col, s, nullptr, 0, dssm::csc_rank_supported(D), false,
                                              srow, sval);
  return e == hipSuccess ? DSSM_OK : oerr(DSSM_E_HIP, hipGetErrorString(e));
}

size_t dssm_dense_bwd_slab_floats(int M, int K, int N, int dtype) {
  return dssm::gemm_dw_slab_floats(K + 1, N, M, dtype == DSSM_BF16);
}

int dssm_dense_bwd_ex(const void* A, int lda, const void* W, int ldw, int dtype, int M, int K, int N,
                      const void* dZ, int lddz, void* dA, int da_dtype, int ldda, const void* mask, int mask_dtype,
                      int ldmask, float* dWb, float* slab, int* deferred_splits, void* stream) {
  if (!A || !W || !dZ || !dWb || M <= 0 || K <= 0 || N <= 0 || lda < K || ldw < N || lddz < N ||
      (dA && ldda < K) || (dtype != DSSM_F32 && dtype != DSSM_BF16) || (lda % 4) || (ldw % 4) ||
      (lddz % 4) || (mask && (!dA || ldmask < K)) || (da_dtype != DSSM_F32 && da_dtype != DSSM_BF16) ||
      (mask_dtype != DSSM_F32 && mask_dtype != DSSM_BF16))
    return oerr(DSSM_E_INVALID, "dense_bwd: bad argument");
  if (dssm_dense_bwd_slab_floats(M, K, N, dtype) && !slab)
    return oerr(DSSM_E_INVALID, "dense_bwd: this shape needs a split-K slab");
  hipStream_t s = (hipStream_t)stream;
  const bool bf = dtype == DSSM_BF16;
  const int flags = (da_dtype == DSSM_BF16 ? dssm::kGemmOutBf16 : 0) | (mask_dtype == DSSM_BF16 ? dssm::kGemmMaskBf16 : 0);
  hipError_t e = hipSuccess;
  if (dA)
    e = dssm::launch_gemm(dssm::GEMM_DA, bf, M, K, N, dZ, lddz, W, ldw, dA, ldda, nullptr, false, nullptr,
                          s, nullptr, 0, mask, ldmask, flags);
  if (e == hipSuccess)
    e = dssm::launch_gemm(dssm::GEMM_DW, bf, K + 1, N, M, A, lda, dZ, lddz, dWb, N, nullptr, true, slab, s,
                          deferred_splits);
  return e == hipSuccess ? DSSM_OK : oerr(DSSM_E_HIP, hipGetErrorString(e));
}

int dssm_spmm_bwd_csc(const int32_t* indptr, const int32_t* indices, const float* values, int rows, int D,
                      int max_nnz, void* ws, void* stream) {
  if (!indptr || !ws || rows <= 0 || D <= 0 || max_nnz < 0 || (max_nnz && (!indices || !values)))
    return oerr(DSSM_E_INVALID, "spmm_bwd_csc: bad argument");
  if (!dssm::csc_rank_supported(D)) return oerr(DSSM_E_INVALID, "spmm_bwd_csc: D beyond the CSC rank path");
  const SpmmWs w = spmm_ws(rows, D, max_nnz);
  char* b = static_cast<char*>(ws);
  const hipError_t e = dssm::launch_csc_build(
      indptr, indices, values, rows, D, max_nnz, reinterpret_cast<int*>(b + w.scratch),
      reinterpret_cast<int*>(b + w.col_ptr), reinterpret_cast<int*>(b + w.row), reinterpret_cast<float*>(b + w.val),
      reinterpret_cast<int*>(b + w.col), (hipStream_t)stream, nullptr, 0, true, false);
  return e == hipSuccess ? DSSM_OK : oerr(DSSM_E_HIP, hipGetErrorString(e));
}

size_t dssm_adam_tickets_bytes(int group) {
  return group <= 0 ? 0 : (64 + (size_t)group * dssm::kAdamTicketUints) * sizeof(unsigned);
}

}  // extern "C"

namespace {
// One tower's optimizer step (validated; its CSC transpose built first when asked) as an AdamStep.
int tower_step(const dssm_tower_adam& t, float lr, float beta1, float beta2, float eps, float* state,
               float grad_scale, int group, int member, void* tickets, hipStream_t s, dssm::AdamStep& a) {
  const int D = t.D, n = t.n, rows = t.rows, max_nnz = t.max_nnz;
  const int64_t w1_end = (int64_t)(D + 1) * n, rest_begin = t.rest_begin, rest_end = t.rest_end;
  if (!t.indptr || !t.dZ || !t.p || !t.g || !t.m || !t.v || !state || !t.ws || rows <= 0 || D <= 0 || n <= 0 ||
      (n % 4) || t.lddz < n || (t.lddz % 8) || (max_nnz && (!t.indices || !t.values)) ||
      (t.dz_dtype != DSSM_F32 && t.dz_dtype != DSSM_BF16) || rest_begin % 4 || rest_end % 4 || rest_begin < w1_end ||
      rest_end < rest_begin || t.splits < 0 ||
      (t.splits && (!t.slab || t.slab_count <= 0 || t.slab_count % 4 || rest_begin + t.slab_count > rest_end)) ||
      (t.w1_shadow && (t.ld_shadow < n || t.ld_shadow % 4)) || t.nseg < 0 || t.nseg > 4 || (t.nseg && !t.segs) ||
      group < 0 || (group && (!tickets || member < 0 || member >= group)))
    return oerr(DSSM_E_INVALID, "spmm_bwd_w_adam: bad argument");
  if (!dssm::csc_rank_supported(D)) return oerr(DSSM_E_INVALID, "spmm_bwd_w_adam: D beyond the CSC rank path");
  if ((reinterpret_cast<uintptr_t>(t.p) | reinterpret_cast<uintptr_t>(t.g) | reinterpret_cast<uintptr_t>(t.m) |
       reinterpret_cast<uintptr_t>(t.v)) % 16)
    return oerr(DSSM_E_INVALID, "spmm_bwd_w_adam: arrays must be 16-B aligned");
  const SpmmWs w = spmm_ws(rows, D, max_nnz);
  char* b = static_cast<char*>(t.ws);
  int* scratch = reinterpret_cast<int*>(b + w.scratch);
  int* col_ptr = reinterpret_cast<int*>(b + w.col_ptr);
  int* crow = reinterpret_cast<int*>(b + w.row);
  float* cval = reinterpret_cast<float*>(b + w.val);
  int* ccol = reinterpret_cast<int*>(b + w.col);
  if (t.build_csc) {
    const hipError_t e = dssm::launch_csc_build(t.indptr, t.indices, t.values, rows, D, max_nnz, scratch, col_ptr,
                                                crow, cval, ccol, s, nullptr, 0, true, false);
    if (e != hipSuccess) return oerr(DSSM_E_HIP, hipGetErrorString(e));
  }
  a = dssm::AdamStep{};
  a.p = t.p;
  a.g = t.g;
  a.m = t.m;
  a.v = t.v;
  a.st = state;
  if (group) {  // member's own two-level ticket after the group counter (dssm_adam_tickets_bytes)
    unsigned* tk = static_cast<unsigned*>(tickets);
    a.group_ticket = tk;
    a.group_n = group;
    a.ticket = tk + 64 + (size_t)member * dssm::kAdamTicketUints;
  } else {
    a.no_advance = 1;
  }
  a.lr = lr;
  a.beta1 = beta1;
  a.beta2 = beta2;
  a.eps = eps;
  a.gs = grad_scale;
  a.w1_blocks = 1;  // sized by the launcher
  a.D = D;
  a.n = n;
  a.col_ptr = col_ptr;
  a.csc_row = crow;
  a.csc_val = cval;
  a.dZ = t.dZ;
  a.lddz = t.lddz;
  a.shadow = t.w1_shadow;
  a.ldsh = t.ld_shadow;
  a.item_blocks = dssm::kAdamItemBlocks;
  a.heavy_n = dssm::csc_heavy_count(scratch, D, max_nnz);
  a.heavy_items = reinterpret_cast<const int2*>(a.heavy_n + 64);
  a.heavy_ticket = dssm::csc_heavy_tickets(scratch, D, rows, max_nnz);
  a.d4_begin = rest_begin / 4;
  a.d4_end = rest_end / 4;
  a.clear_from = rest_end;  // the rest's gradient is rewritten by the next backward
  a.sh.count = t.nseg;
  for (int i = 0; i < t.nseg; ++i) {
    const dssm_shadow_seg& q = t.segs[i];
    if (!q.ptr || q.offset < rest_begin || q.rows < 0 || q.cols <= 0 || q.ld < q.cols || q.offset % 4 || q.cols % 4 ||
        q.ld % 4 || q.offset + q.rows * q.cols > rest_end)
      return oerr(DSSM_E_INVALID, "spmm_bwd_w_adam: bad shadow segment");
    a.sh.seg[i] = dssm::ShadowSeg{q.offset, q.rows, q.cols, q.ld, q.ptr, nullptr, 0};
  }
  if (t.splits) {
    a.slabs.count = 1;
    a.slabs.seg[0] = dssm::SlabSeg{rest_begin, t.slab_count, t.splits, t.slab};
  }
  return DSSM_OK;
}
}  // namespace

extern "C" {

int dssm_spmm_bwd_w_adam(const int32_t* indptr, const int32_t* indices, const float* values, int rows, int D,
                         int max_nnz, const void* dZ, int dz_dtype, int lddz, int n, float* p, float* g, float* m,
                         float* v, int64_t rest_begin, int64_t rest_end, const float* slab, int64_t slab_count,
                         int splits, uint16_t* w1_shadow, int ld_shadow, const dssm_shadow_seg* segs, int nseg,
                         float lr, float beta1, float beta2, float eps, float* state, float grad_scale,
                         int group, int member, void* tickets, int build_csc, void* ws, void* stream) {
  const dssm_tower_adam t{indptr, indices, values, rows, D, max_nnz, dZ, dz_dtype, lddz, n, p, g, m, v,
                          rest_begin, rest_end, slab, slab_count, splits, w1_shadow, ld_shadow, segs, nseg,
                          build_csc, ws};
  hipStream_t s = (hipStream_t)stream;
  dssm::AdamStep a;
  const int rc = tower_step(t, lr, beta1, beta2, eps, state, grad_scale, group, member, tickets, s, a);
  if (rc != DSSM_OK) return rc;
  const bool probe = dssm::adam_probe_begin(s);
  const hipError_t e = dssm::launch_adam_step(a, dz_dtype == DSSM_BF16, s);
  if (probe) dssm::adam_probe_end(s);
  return e == hipSuccess ? DSSM_OK : oerr(DSSM_E_HIP, hipGetErrorString(e));
}

int dssm_dense_bwd_masked(const void* A, int lda, const void* W, int ldw, int dtype, int M, int K, int N,
                          const void* dZ, int lddz, float* dA, int ldda, const float* mask, int ldmask,
                          float* dWb, float* slab, void* stream) {
  if (!A || !W || !dZ || !dWb || M <= 0 || K <= 0 || N <= 0 || lda < K || ldw < N || lddz < N ||
      (dA && ldda < K) || (dtype != DSSM_F32 && dtype != DSSM_BF16) || (lda % 4) || (ldw % 4) ||
      (lddz % 4) || (mask && (!dA || ldmask < K)))
    return oerr(DSSM_E_INVALID, "dense_bwd: bad argument");
  if (dssm_dense_bwd_slab_floats(M, K, N, dtype) && !slab)
    return oerr(DSSM_E_INVALID, "dense_bwd: this shape needs a split-K slab");
  hipStream_t s = (hipStream_t)stream;
  const bool bf = dtype == DSSM_BF16;
  hipError_t e = hipSuccess;
  if (dA)
    e = dssm::launch_gemm(dssm::GEMM_DA, bf, M, K, N, dZ, lddz, W, ldw, dA, ldda, nullptr, false, nullptr,
                          s, nullptr, 0, mask, ldmask);
  if (e == hipSuccess)
    e = dssm::launch_gemm(dssm::GEMM_DW, bf, K + 1, N, M, A, lda, dZ, lddz, dWb, N, nullptr, true, slab, s,
                          nullptr);
  return e == hipSuccess ? DSSM_OK : oerr(DSSM_E_HIP, hipGetErrorString(e));
}

int dssm_dense_bwd(const void* A, int lda, const void* W, int ldw, int dtype, int M, int K, int N,
                   const void* dZ, int lddz, float* dA, int ldda, float* dWb, float* slab, void* stream) {
  return dssm_dense_bwd_masked(A, lda, W, ldw, dtype, M, K, N, dZ, lddz, dA, ldda, nullptr, 0, dWb, slab,
                               stream);
}

int dssm_bn_relu_bwd(const float* Z, int ldz, int rows, int n, const float* gamma, const float* beta,
                     const float* batch_mean, const float* batch_var, float eps, int relu,
                     const float* dout, int ldd, float* dz, int lddz, float* dgamma, float* dbeta,
                     void* stream) {
  if (!Z || !gamma || !beta || !batch_mean || !batch_var || !dout || !dz || !dgamma || !dbeta || rows <= 0 ||
      n <= 0 || ldz < n || ldd < n || lddz < n)
    return oerr(DSSM_E_INVALID, "bn_relu_bwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_bnr_bwd_sums, dim3((n + 63) / 64), dim3(256), 0, s, Z, ldz, rows, n, gamma, beta,
                     batch_mean, batch_var, eps, relu, dout, ldd, dgamma, dbeta);
  const int64_t total = (int64_t)rows * n;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 2048));
  hipLaunchKernelGGL(k_bnr_bwd_apply, dim3(grid), dim3(256), 0, s, Z, ldz, rows, n, gamma, beta, batch_mean,
                     batch_var, eps, relu, dout, ldd, dgamma, dbeta, dz, lddz);
  return hip_status();
}

}  // extern "C"

// ---- touched-row sparse gradient exchange (dssm_amd/dist.py DataParallel(sparse=True)) --------
// A packed row: [row id (int32, 2 u16)][2 u16 pad][n u16 of the row], stride n + 4 (8-B aligned).
namespace {
__global__ __launch_bounds__(256) void k_rows_pack_u16(const uint16_t* __restrict__ src, int64_t n,
                                                       const int32_t* __restrict__ rows, int64_t count,
                                                       uint16_t* __restrict__ out) {
  const int64_t q = n / 4, stride = n + 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count * (q + 1);
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = i / (q + 1), g = i - k * (q + 1);
    const int32_t r = rows[k];
    uint2 v;
    if (g == 0) {
      v.x = (uint32_t)r;
      v.y = 0u;
    } else {
      v = *reinterpret_cast<const uint2*>(src + (int64_t)r * n + 4 * (g - 1));
    }
    *reinterpret_cast<uint2*>(out + k * stride + 4 * g) = v;
  }
}
__global__ __launch_bounds__(256) void k_rows_unpack_u16(const uint16_t* __restrict__ in, int64_t n,
                                                         int64_t count, int64_t row_base, int64_t nrows,
                                                         uint16_t* __restrict__ dst) {
  const int64_t q = n / 4, stride = n + 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count * q;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = i / q, g = i - k * q;
    const int64_t r = (int64_t)*reinterpret_cast<const int32_t*>(in + k * stride) - row_base;
    if (r < 0 || r >= nrows) continue;  // not this rank's row: never sent here
    *reinterpret_cast<uint2*>(dst + r * n + 4 * g) = *reinterpret_cast<const uint2*>(in + k * stride + 4 + 4 * g);
  }
}
int rows_grid(int64_t work) { return (int)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 4096)); }
}  // namespace

extern "C" {

int dssm_rows_pack_u16(const uint16_t* src, int64_t n, const int32_t* rows, int64_t count, uint16_t* out,
                       void* stream) {
  if (count < 0 || n <= 0 || (n % 4) || (count && (!src || !rows || !out)))
    return oerr(DSSM_E_INVALID, "rows_pack_u16: bad argument (n a multiple of 4)");
  if (count)
    hipLaunchKernelGGL(k_rows_pack_u16, dim3(rows_grid(count * (n / 4 + 1))), dim3(256), 0, (hipStream_t)stream,
                       src, n, rows, count, out);
  return hip_status();
}

int dssm_rows_unpack_u16(const uint16_t* in, int64_t n, int64_t count, int64_t row_base, int64_t nrows,
                         uint16_t* dst, void* stream) {
  if (count < 0 || n <= 0 || (n % 4) || nrows < 0 || (count && (!in || !dst)))
    return oerr(DSSM_E_INVALID, "rows_unpack_u16: bad argument (n a multiple of 4)");
  if (count)
    hipLaunchKernelGGL(k_rows_unpack_u16, dim3(rows_grid(count * (n / 4))), dim3(256), 0, (hipStream_t)stream,
                       in, n, count, row_base, nrows, dst);
  return hip_status();
}

}  // extern "C"

