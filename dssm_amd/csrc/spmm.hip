// Sparse side of the DSSM step on gfx950:
//   * FC1 forward  Z1 = X*W1 + b1           (new_dssm.py:124-126, SparseTensorDenseMatMul)
//   * CSR -> CSC transpose of [X | 1]       (TF's adjoint_a gradient needs X^T)
//   * dW1 (+db1)  = [X | 1]^T * dZ1         (TF1.x SparseTensorDenseMatMul grad + BiasAddGrad)
//
// Mapping: one wave per CSR row (forward) or per CSC column (backward).  Lane l owns output
// columns [8l, 8l+8): each gathered W1 / dZ1 row is read with one 16-B load per lane (bf16)
// or two (fp32), so a 300-wide bf16 row is one 608-B wave-instruction.  Column indices and
// values are loaded coalesced by lane and broadcast with v_readlane (scalar address math).
#include "common.h"
#include "launch.h"

namespace dssm {
namespace {

constexpr int kUnroll = 8;
constexpr int kChunk = 64;  // CSC entries per wave in the dW1 kernels

__device__ __forceinline__ void store8n(float* p, const float (&x)[8], int nvalid) {
  *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
  if (nvalid > 4) *reinterpret_cast<float4*>(p + 4) = make_float4(x[4], x[5], x[6], x[7]);
}

// Accumulate sum_j val_j * M[idx_j, c..c+8) for entries [s, e) into acc.
template <typename T>
__device__ __forceinline__ void gather_accumulate(const int* __restrict__ idx,
                                                  const float* __restrict__ val, int s, int e,
                                                  const T* __restrict__ M, int ldm, int c,
                                                  int nvalid, float (&acc)[8]) {
  const int lane = lane_id();
  for (int base = s; base < e; base += 64) {
    const int cnt = min(64, e - base);
    int my_i = 0;
    float my_v = 0.f;
    if (lane < cnt) {
      my_i = idx[base + lane];
      my_v = val[base + lane];
    }
    int j = 0;
    for (; j + kUnroll <= cnt; j += kUnroll) {
      float x[kUnroll][8];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int r = bcast_i(my_i, j + u);
        if (nvalid > 0) load8(M + (size_t)r * ldm + c, nvalid, x[u]);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const float v = bcast_f(my_v, j + u);
        if (nvalid > 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[i] = __fmaf_rn(v, x[u][i], acc[i]);
        }
      }
    }
    for (; j < cnt; ++j) {
      const int r = bcast_i(my_i, j);
      const float v = bcast_f(my_v, j);
      if (nvalid > 0) {
        float x[8];
        load8(M + (size_t)r * ldm + c, nvalid, x);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __fmaf_rn(v, x[i], acc[i]);
      }
    }
  }
}

template <typename TW>
__global__ __launch_bounds__(256) void k_spmm_fwd(const int* __restrict__ indptr,
                                                  const int* __restrict__ indices,
                                                  const float* __restrict__ values, int rows,
                                                  const TW* __restrict__ W, int ldw, int n,
                                                  const float* __restrict__ bias,
                                                  float* __restrict__ Z, int ldz) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = lane_id();
  const int s = indptr[row], e = indptr[row + 1];
  for (int c0 = 0; c0 < ldz; c0 += 512) {
    // All 64 lanes stay active through gather_accumulate: its index broadcasts read every
    // lane's register (v_readlane ignores EXEC), so out-of-range lanes only skip the loads.
    const int c = c0 + lane * 8;
    const int nvalid = (c < ldz) ? n - c : 0;  // >= 8 full, 4 half, <= 0 pad-only/idle
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = (c + i < n) ? bias[c + i] : 0.f;
    gather_accumulate(indices, values, s, e, W, ldw, c, nvalid, acc);
    if (c < ldz) store8(Z + (size_t)row * ldz + c, acc);
  }
}

__global__ void k_csc_count(const int* __restrict__ indptr, const int* __restrict__ indices,
                            int rows, int* __restrict__ cnt) {
  const int nnz = indptr[rows];
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < nnz; e += gridDim.x * blockDim.x)
    atomicAdd(&cnt[indices[e]], 1);
}

// Single-workgroup exclusive scan of the D+1 column counts (column D = virtual ones column
// holding every row).  Also turns cnt[] into per-column fill cursors.
__global__ __launch_bounds__(1024) void k_csc_scan(int* __restrict__ cnt, int D, int rows,
                                                   int* __restrict__ col_ptr) {
  __shared__ int wave_tot[16];
  const int ncols = D + 1;
  const int t = threadIdx.x;
  const int per = cdiv(ncols, 1024);
  const int c0 = min(t * per, ncols), c1 = min(c0 + per, ncols);
  int sum = 0;
  for (int c = c0; c < c1; ++c) sum += (c == D) ? rows : cnt[c];
  // inclusive wave scan
  const int lane = t & 63, w = t >> 6;
  int x = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wave_tot[w] = x;
  __syncthreads();
  if (t == 0) {
    int run = 0;
    for (int i = 0; i < 16; ++i) {
      int v = wave_tot[i];
      wave_tot[i] = run;
      run += v;
    }
  }
  __syncthreads();
  int run = wave_tot[w] + x - sum;  // exclusive prefix of this thread's chunk
  for (int c = c0; c < c1; ++c) {
    const int v = (c == D) ? rows : cnt[c];
    col_ptr[c] = run;
    cnt[c] = run;  // fill cursor
    run += v;
  }
  if (t == 1023) col_ptr[ncols] = run;
}

__global__ __launch_bounds__(256) void k_csc_fill(const int* __restrict__ indptr,
                                                  const int* __restrict__ indices,
                                                  const float* __restrict__ values, int rows, int D,
                                                  int* __restrict__ cursor,
                                                  const int* __restrict__ col_ptr,
                                                  int* __restrict__ csc_row,
                                                  float* __restrict__ csc_val,
                                                  int* __restrict__ csc_col) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = lane_id();
  const int s = indptr[row], e = indptr[row + 1];
  for (int k = s + lane; k < e; k += 64) {
    const int c = indices[k];
    const int pos = atomicAdd(&cursor[c], 1);
    csc_row[pos] = row;
    csc_val[pos] = values[k];
    csc_col[pos] = c;
  }
  if (lane == 0) {
    const int pos = col_ptr[D] + row;
    csc_row[pos] = row;
    csc_val[pos] = 1.0f;
    csc_col[pos] = D;
  }
}

// Columns' first kChunk entries: plain store of the row of G (zero for untouched columns).
template <typename TZ>
__global__ __launch_bounds__(256) void k_dw1_light(const int* __restrict__ col_ptr,
                                                   const int* __restrict__ csc_row,
                                                   const float* __restrict__ csc_val, int D,
                                                   const TZ* __restrict__ dZ, int lddz, int n,
                                                   float* __restrict__ G) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c > D) return;
  const int lane = lane_id();
  const int s = col_ptr[c];
  const int e = min(col_ptr[c + 1], s + kChunk);
  for (int c0 = 0; c0 < n; c0 += 512) {
    const int cc = c0 + lane * 8;
    const int nvalid = n - cc;  // lanes with nvalid <= 0 stay active for the broadcasts
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    gather_accumulate(csc_row, csc_val, s, e, dZ, lddz, cc, nvalid, acc);
    if (nvalid > 0) store8n(G + (size_t)c * n + cc, acc, nvalid);
  }
}

// Remaining entries of heavy columns: fixed kChunk-entry slices of the CSC arrays, summed per
// column run and added with fp32 atomics (after k_dw1_light has stored the first slice).
template <typename TZ>
__global__ __launch_bounds__(256) void k_dw1_heavy(const int* __restrict__ col_ptr,
                                                   const int* __restrict__ csc_row,
                                                   const float* __restrict__ csc_val,
                                                   const int* __restrict__ csc_col, int D,
                                                   const TZ* __restrict__ dZ, int lddz, int n,
                                                   float* __restrict__ G) {
  const int chunk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int total = col_ptr[D + 1];
  const int j0 = chunk * kChunk;
  if (j0 >= total) return;
  const int j1 = min(j0 + kChunk, total);
  const int lane = lane_id();
  int j = j0;
  while (j < j1) {
    const int c = csc_col[j];
    const int cs = col_ptr[c];
    const int ce = min(col_ptr[c + 1], j1);
    const int first = max(j, cs + kChunk);
    if (first < ce) {
      for (int c0 = 0; c0 < n; c0 += 512) {
        const int cc = c0 + lane * 8;
        const int nvalid = n - cc;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        gather_accumulate(csc_row, csc_val, first, ce, dZ, lddz, cc, nvalid, acc);
        if (nvalid > 0) {
          float* g = G + (size_t)c * n + cc;
          const int m = nvalid >= 8 ? 8 : 4;
          for (int i = 0; i < m; ++i) atomicAdd(g + i, acc[i]);
        }
      }
    }
    j = ce;
  }
}

}  // namespace

hipError_t launch_spmm_fwd(const int* indptr, const int* indices, const float* values, int rows,
                           const void* W, bool w_bf16, int ldw, int n, const float* bias, float* Z,
                           int ldz, hipStream_t s) {
  dim3 grid(cdiv(rows, 4)), block(256);
  if (w_bf16)
    hipLaunchKernelGGL(k_spmm_fwd<u16>, grid, block, 0, s, indptr, indices, values, rows,
                       (const u16*)W, ldw, n, bias, Z, ldz);
  else
    hipLaunchKernelGGL(k_spmm_fwd<float>, grid, block, 0, s, indptr, indices, values, rows,
                       (const float*)W, ldw, n, bias, Z, ldz);
  return hipGetLastError();
}

hipError_t launch_csc_build(const int* indptr, const int* indices, const float* values, int rows,
                            int D, int max_nnz, int* cnt, int* col_ptr, int* csc_row,
                            float* csc_val, int* csc_col, hipStream_t s) {
  hipError_t err = hipMemsetAsync(cnt, 0, sizeof(int) * (size_t)(D + 1), s);
  if (err != hipSuccess) return err;
  const int cblocks = max(1, min(cdiv(max_nnz, 256), 2048));
  hipLaunchKernelGGL(k_csc_count, dim3(cblocks), dim3(256), 0, s, indptr, indices, rows, cnt);
  hipLaunchKernelGGL(k_csc_scan, dim3(1), dim3(1024), 0, s, cnt, D, rows, col_ptr);
  hipLaunchKernelGGL(k_csc_fill, dim3(cdiv(rows, 4)), dim3(256), 0, s, indptr, indices, values,
                     rows, D, cnt, col_ptr, csc_row, csc_val, csc_col);
  return hipGetLastError();
}

hipError_t launch_dw1(const int* col_ptr, const int* csc_row, const float* csc_val,
                      const int* csc_col, int D, int rows, int max_nnz, const void* dZ,
                      bool dz_bf16, int lddz, int n, float* G, hipStream_t s) {
  dim3 block(256);
  dim3 g1(cdiv(D + 1, 4));
  dim3 g2(max(1, cdiv(cdiv(max_nnz + rows, kChunk), 4)));
  if (dz_bf16) {
    hipLaunchKernelGGL(k_dw1_light<u16>, g1, block, 0, s, col_ptr, csc_row, csc_val, D,
                       (const u16*)dZ, lddz, n, G);
    hipLaunchKernelGGL(k_dw1_heavy<u16>, g2, block, 0, s, col_ptr, csc_row, csc_val, csc_col, D,
                       (const u16*)dZ, lddz, n, G);
  } else {
    hipLaunchKernelGGL(k_dw1_light<float>, g1, block, 0, s, col_ptr, csc_row, csc_val, D,
                       (const float*)dZ, lddz, n, G);
    hipLaunchKernelGGL(k_dw1_heavy<float>, g2, block, 0, s, col_ptr, csc_row, csc_val, csc_col,
                       D, (const float*)dZ, lddz, n, G);
  }
  return hipGetLastError();
}

}  // namespace dssm
