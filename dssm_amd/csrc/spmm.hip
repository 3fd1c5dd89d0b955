// Sparse side of the DSSM step on gfx950:
//   * FC1 forward  Z1 = X*W1 + b1           (new_dssm.py:124-126, SparseTensorDenseMatMul)
//   * CSR -> CSC transpose of [X | 1]       (TF's adjoint_a gradient needs X^T)
//   * dW1 (+db1)  = [X | 1]^T * dZ1         (TF1.x SparseTensorDenseMatMul grad + BiasAddGrad)
//
// Mapping: one wave per CSR row (forward) or per CSC column (backward).  Lane l owns output
// columns [8l, 8l+8): each gathered W1 / dZ1 row is read with one 16-B load per lane (bf16)
// or two (fp32), so a 300-wide bf16 row is one 608-B wave-instruction.  Column indices and
// values are loaded coalesced by lane and broadcast with v_readlane (scalar address math).
//
// The transpose never puts a Zipf-hot column on one global atomic: each 1024-thread block
// histograms its rows' columns in LDS (D+1 bins fit the 160 KiB LDS for D <= 38k), then adds
// or reserves whole per-block counts with one global atomic per (block, column).
//
// dW1 splits columns by count: "heavy" columns (> kLight entries, incl. the virtual bias column
// with every row) are summed by fixed 64-entry slices and added with coalesced fp32 atomics
// (each atomic wave-instruction covers 256 contiguous bytes); "light" columns are summed by
// one wave each, either here (materialized dW1 for the all-reduce) or inside the fused
// W1 Adam kernel (adam.hip), which then never writes or re-reads a dense dW1.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "bnfuse.h"
#include "common.h"
#include "gather.h"
#include "launch.h"
#include "csc.h"

#ifndef DSSM_SPMM_U  // rows in flight per lane in the SpMM's gather batches
#define DSSM_SPMM_U 8
#endif

namespace dssm {
namespace {

__device__ __forceinline__ void store8n(float* p, const float (&x)[8], int nvalid) {
  *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
  if (nvalid > 4) *reinterpret_cast<float4*>(p + 4) = make_float4(x[4], x[5], x[6], x[7]);
}

}  // namespace

namespace {

template <typename TW, typename TO = float>
__device__ __forceinline__ void spmm_rows(const int* __restrict__ indptr,
                                          const int* __restrict__ indices,
                                          const float* __restrict__ values, int rows,
                                          const TW* __restrict__ W, int ldw, int n,
                                          const float* __restrict__ bias, TO* __restrict__ Z,
                                          int ldz, int b, bool relu = false) {
  const int row = b * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  if (row >= rows) return;
  const int lane = lane_id();
  const int s = indptr[row], e = indptr[row + 1];
  for (int c0 = 0; c0 < ldz; c0 += 512) {
    const int c = c0 + lane * 8;
    const int nvalid = (c < ldz) ? n - c : 0;  // >= 8 full, 4 half, <= 0 pad-only/idle
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = (c + i < n) ? bias[c + i] : 0.f;
    gather_accumulate<TW, 1, DSSM_SPMM_U>(indices, values, s, e, W, ldw, c, nvalid, acc);
    if constexpr (std::is_same<TW, u16t>::value) {  // tight rows: the half group's upper sums
#pragma unroll
      for (int i = 4; i < 8; ++i) acc[i] = (c + i < n) ? acc[i] : 0.f;  // read the next row (gather.h)
    }
    if (relu) {  // the layer's ReLU fused (functional API: FC1 + tf.nn.relu)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaxf(acc[i], 0.f);
    }
    if (c < ldz) store8(Z + (size_t)row * ldz + c, acc);
  }
}

// Eval BN coefficients, item i of all layers' (column, tower) pairs: the arithmetic of
// k_bn_stats' eval finalize (rstd = 1 / sqrt(var + eps), inv = rstd * gamma, shift = beta - mu * inv;
// pad columns zero).
__device__ __forceinline__ void eval_coef_item(const EvalCoef& e, int i) {
  for (int l = 0; l < e.L; ++l) {
    const int items = 2 * e.ld[l];
    if (i >= items) {
      i -= items;
      continue;
    }
    const int t = i / e.ld[l], c = i - t * e.ld[l];
    const size_t plane = (size_t)2 * e.ld[l], o = (size_t)t * e.ld[l] + c;
    float* coef = e.coef[l];
    if (c >= e.n[l]) {
      coef[o] = 0.f; coef[plane + o] = 0.f; coef[2 * plane + o] = 0.f; coef[3 * plane + o] = 0.f;
    } else {
      const float mu = e.ema_mean[l][t][c], var = e.ema_var[l][t][c];
      const float rstd = 1.0f / sqrtf(var + e.eps);
      const float inv = rstd * e.gamma[l][t][c];
      coef[o] = mu;
      coef[plane + o] = rstd;
      coef[2 * plane + o] = inv;
      coef[3 * plane + o] = e.beta[l][t][c] - mu * inv;
    }
    return;
  }
}

// blocks [0, ne): eval coefficients (first in dispatch order); the rest: one wave per CSR row.
// TO: the output's storage (fp32, or bf16 RNE: the multi-view model's bf16 FC1 activation)
template <typename TW, typename TO = float>
__global__ __launch_bounds__(256) void k_spmm_fwd(const int* __restrict__ indptr,
                                                  const int* __restrict__ indices,
                                                  const float* __restrict__ values, int rows,
                                                  const TW* __restrict__ W, int ldw, int n,
                                                  const float* __restrict__ bias,
                                                  TO* __restrict__ Z, int ldz, EvalCoef ec,
                                                  int ne, int relu) {
  if ((int)blockIdx.x < ne) {
    eval_coef_item(ec, (int)blockIdx.x * 256 + threadIdx.x);
    return;
  }
  spmm_rows<TW, TO>(indptr, indices, values, rows, W, ldw, n, bias, Z, ldz, (int)blockIdx.x - ne, relu != 0);
}

// ---- CSR -> CSC ------------------------------------------------------------------------------
// Blocks own contiguous row ranges; wave w of a block walks rows r0+w, r0+w+16, ... and its
// lanes the row's entries (a row's columns are distinct, so a wave-instruction never collides).
constexpr int kTB = 1024;  // threads per transpose block

constexpr int kTU = 8;  // entries per thread in flight

__global__ __launch_bounds__(kTB) void k_csc_hist(const int* __restrict__ indptr,
                                                  const int* __restrict__ indices, int rows, int D,
                                                  int rows_per_block, int* __restrict__ gcnt,
                                                  double* __restrict__ zero, int nzero) {
  extern __shared__ int hist[];
  // the first launch of a train step also clears the step's fused BN accumulators (bnfuse.h)
  for (int i = blockIdx.x * kTB + threadIdx.x; i < nzero; i += gridDim.x * kTB) zero[i] = 0.0;
  for (int c = threadIdx.x; c < D; c += kTB) hist[c] = 0;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  const int e0 = indptr[r0], e1 = indptr[r1];  // the block's rows own a contiguous entry range
  __syncthreads();
  for (int base = e0; base < e1; base += kTB * kTU) {
    int c[kTU];
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int e = base + u * kTB + (int)threadIdx.x;
      c[u] = e < e1 ? indices[e] : -1;
    }
#pragma unroll
    for (int u = 0; u < kTU; ++u)
      if (c[u] >= 0) atomicAdd(&hist[c[u]], 1);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += kTB) {
    const int v = hist[c];
    if (v) atomicAdd(&gcnt[c], v);
  }
}

// Fallback when D+1 bins do not fit LDS: direct global atomics.
__global__ void k_csc_count_global(const int* __restrict__ indptr, const int* __restrict__ indices,
                                   int rows, int* __restrict__ cnt) {
  const int nnz = indptr[rows];
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < nnz; e += gridDim.x * blockDim.x)
    atomicAdd(&cnt[indices[e]], 1);
}

// Single-workgroup exclusive scan of the D+1 column counts (column D = the virtual ones column
// holding every row).  Counts are staged through LDS with coalesced loads/stores (thread t owns
// 16 consecutive bins of each 16K-bin tile).  Writes col_ptr and the fill cursors, and
// re-zeroes the counts for the next step (so no memset is needed on the stream).
constexpr int kScanPer = 16, kScanTile = 1024 * kScanPer;
__global__ __launch_bounds__(1024) void k_csc_scan(int* __restrict__ cnt, int D, int rows,
                                                   int* __restrict__ col_ptr,
                                                   int* __restrict__ cursor) {
  __shared__ int tile[kScanTile + kScanTile / 32];  // +1 int per 32: breaks the stride-16 conflicts
  __shared__ int wave_tot[16];
  __shared__ int carry_s;
  const int ncols = D + 1;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  auto pad = [](int i) { return i + (i >> 5); };
  if (t == 0) carry_s = 0;
  for (int base = 0; base < ncols; base += kScanTile) {
    {
      int ld[kScanPer];  // all 16 loads in flight before the LDS writes
#pragma unroll
      for (int k = 0; k < kScanPer; ++k) {
        const int c = base + k * 1024 + t;
        ld[k] = (c < D) ? cnt[c] : (c == D ? rows : 0);
      }
#pragma unroll
      for (int k = 0; k < kScanPer; ++k) tile[pad(k * 1024 + t)] = ld[k];
    }
    __syncthreads();
    int v[kScanPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      v[k] = tile[pad(t * kScanPer + k)];
      sum += v[k];
    }
    int x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) wave_tot[w] = x;
    __syncthreads();
    if (t == 0) {
      int run = carry_s;
      for (int i = 0; i < 16; ++i) {
        const int a = wave_tot[i];
        wave_tot[i] = run;
        run += a;
      }
      carry_s = run;
    }
    __syncthreads();
    int run = wave_tot[w] + x - sum;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      tile[pad(t * kScanPer + k)] = run;
      run += v[k];
    }
    __syncthreads();
    for (int i = t; i < kScanTile; i += 1024) {
      const int c = base + i;
      if (c < ncols) {
        const int o = tile[pad(i)];
        col_ptr[c] = o;
        cursor[c] = o;
        if (c < D) cnt[c] = 0;
      }
    }
    __syncthreads();
  }
  if (t == 0) col_ptr[ncols] = carry_s;
}

// Fill: local rank per entry from an LDS histogram, one returning global atomic per
// (block, column) to reserve the block's slot range, then scatter (row, value, column).  Rows of
// entries come from a binary search of the block's indptr slice staged in LDS.
__global__ __launch_bounds__(kTB) void k_csc_fill(const int* __restrict__ indptr,
                                                  const int* __restrict__ indices,
                                                  const float* __restrict__ values, int rows,
                                                  int D, int rows_per_block,
                                                  int* __restrict__ cursor,
                                                  const int* __restrict__ col_ptr,
                                                  int* __restrict__ rank_tmp,
                                                  int* __restrict__ csc_row,
                                                  float* __restrict__ csc_val,
                                                  int* __restrict__ csc_col) {
  extern __shared__ int hist[];  // D bins, then the block's indptr slice
  int* sptr = hist + D;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  const int nr = r1 - r0;
  for (int c = threadIdx.x; c < D; c += kTB) hist[c] = 0;
  for (int i = threadIdx.x; i <= nr; i += kTB) sptr[i] = indptr[r0 + i];
  __syncthreads();
  const int e0 = sptr[0], e1 = sptr[nr];
  for (int base = e0; base < e1; base += kTB * kTU) {
    int c[kTU];
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int e = base + u * kTB + (int)threadIdx.x;
      c[u] = e < e1 ? indices[e] : -1;
    }
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int e = base + u * kTB + (int)threadIdx.x;
      if (c[u] >= 0) rank_tmp[e] = atomicAdd(&hist[c[u]], 1);
    }
  }
  __syncthreads();
  for (int base = 0; base < D; base += kTB * kTU) {  // reserve: independent returning atomics
    int v[kTU], got[kTU];
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int c = base + u * kTB + (int)threadIdx.x;
      v[u] = c < D ? hist[c] : 0;
    }
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int c = base + u * kTB + (int)threadIdx.x;
      got[u] = v[u] ? atomicAdd(&cursor[c], v[u]) : 0;
    }
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int c = base + u * kTB + (int)threadIdx.x;
      if (v[u]) hist[c] = got[u];
    }
  }
  __syncthreads();
  for (int base = e0; base < e1; base += kTB * kTU) {
    int c[kTU], rk[kTU];
    float val[kTU];
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int e = base + u * kTB + (int)threadIdx.x;
      const bool ok = e < e1;
      c[u] = ok ? indices[e] : -1;
      rk[u] = ok ? rank_tmp[e] : 0;
      val[u] = ok ? values[e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      if (c[u] < 0) continue;
      const int e = base + u * kTB + (int)threadIdx.x;
      int lo = 0, hi = nr;  // largest i with sptr[i] <= e
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (sptr[mid] <= e) lo = mid; else hi = mid;
      }
      const int pos = hist[c[u]] + rk[u];
      csc_row[pos] = r0 + lo;
      csc_val[pos] = val[u];
      csc_col[pos] = c[u];
    }
  }
  const int vbase = col_ptr[D];
  for (int r = r0 + threadIdx.x; r < r1; r += kTB) {
    csc_row[vbase + r] = r;
    csc_val[vbase + r] = 1.0f;
    csc_col[vbase + r] = D;
  }
}

// ---- three-launch transpose without re-histogramming -----------------------------------------
// k_csc_rank (workgroups own row ranges; one per CU: the histogram fills LDS): every entry's rank
// among the block's entries of its column comes from an LDS histogram; ONE returning global
// atomic per distinct column of the block reserves the block's range inside the column (hot
// Zipf columns see one atomic per block, never one per entry); each entry's position inside its
// column (block base + rank) is stored in place of its rank.
// k_csc_scan_multi: column pointers; every workgroup sums the counts before its chunk itself
// (all its loads in flight at once) and scans its chunk.
// k_csc_scatter: one wave per CSR row scatters (row, value, column) to col_ptr[c] + position, and
// re-zeroes the counts for the next step.
// Kernel boundaries (~1.5-2 us) are cheaper than in-kernel grid barriers on MI355X
// (MI355X_MICROARCH.md: boundary vs barrier-xcd / barrier-counter rows).
constexpr int kCscRankBlocks = 128;
constexpr int kCscListMax = 4096;  // LDS list of the block's distinct columns
__global__ __launch_bounds__(kTB) void k_csc_rank(const int* __restrict__ indptr,
                                                  const int* __restrict__ indices, int rows, int D,
                                                  int rows_per_block, int* __restrict__ cnt,
                                                  int* __restrict__ pos_tmp,
                                                  double* __restrict__ zero, int nzero,
                                                  int* __restrict__ heavy_n) {
  extern __shared__ int hist[];  // D bins
  __shared__ int s_list[kCscListMax];
  __shared__ int s_nlist;
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  // the first launch of a train step also clears the step's fused BN accumulators (bnfuse.h)
  for (int i = blockIdx.x * kTB + t; i < nzero; i += gridDim.x * kTB) zero[i] = 0.0;
  for (int c = t; c < D; c += kTB) hist[c] = 0;
  if (t == 0) s_nlist = 0;
  // this step's heavy-item list (k_csc_scan_multi); null when the previous step's Adam re-arms it
  if (heavy_n && blockIdx.x == 0 && t == 0) *heavy_n = 0;
  __syncthreads();
  const int e0 = indptr[r0], e1 = indptr[max(r0, r1)];
  for (int base = e0; base < e1; base += kTB * kTU) {
    int c[kTU];
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int e = base + u * kTB + t;
      c[u] = e < e1 ? indices[e] : -1;
    }
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int e = base + u * kTB + t;
      if (c[u] >= 0) {
        const int r = atomicAdd(&hist[c[u]], 1);
        pos_tmp[e] = r;
        if (r == 0) s_list[min(atomicAdd(&s_nlist, 1), kCscListMax - 1)] = c[u];  // first touch
      }
    }
  }
  __syncthreads();
  const int nl = s_nlist;
  if (nl < kCscListMax) {  // every distinct column listed: all reservations in flight at once
    for (int i0 = 0; i0 < nl; i0 += kTB * 4) {
      int cc[4], got[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * kTB + t;
        cc[u] = i < nl ? s_list[i] : -1;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) got[u] = cc[u] >= 0 ? atomicAdd(&cnt[cc[u]], hist[cc[u]]) : 0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (cc[u] >= 0) hist[cc[u]] = got[u];
    }
  } else {
    for (int base = 0; base < D; base += kTB * kTU) {
      int v[kTU], got[kTU];
#pragma unroll
      for (int u = 0; u < kTU; ++u) {
        const int c = base + u * kTB + t;
        v[u] = c < D ? hist[c] : 0;
      }
#pragma unroll
      for (int u = 0; u < kTU; ++u) {
        const int c = base + u * kTB + t;
        got[u] = v[u] ? atomicAdd(&cnt[c], v[u]) : 0;
      }
#pragma unroll
      for (int u = 0; u < kTU; ++u) {
        const int c = base + u * kTB + t;
        if (v[u]) hist[c] = got[u];
      }
    }
  }
  __syncthreads();
  for (int base = e0; base < e1; base += kTB * kTU) {  // rank -> position inside the column
    int c[kTU], rk[kTU];
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int e = base + u * kTB + t;
      const bool ok = e < e1;
      c[u] = ok ? indices[e] : 0;
      rk[u] = ok ? pos_tmp[e] : 0;
    }
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int e = base + u * kTB + t;
      if (e < e1) pos_tmp[e] = hist[c[u]] + rk[u];
    }
  }
}

// block-wide exclusive scan of one value per thread (NT threads); returns the block total too
template <int NT = kTB>
__device__ __forceinline__ int block_excl_scan(int v, int* s_wave, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wave[w] = x;
  __syncthreads();
  int before = 0;
  total = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    const int t = s_wave[i];
    before += i < w ? t : 0;
    total += t;
  }
  __syncthreads();
  return before + x - v;
}

constexpr int kScanMultiCols = 4096;  // columns per scan workgroup (4 per thread)
// Heavy columns (> kLightEntries entries, the ones column included) are also listed as
// kHeavyItem-entry work items {column, item} for k_dw1_heavy_items (one returning atomic per
// workgroup reserves its slots).
template <int NT>
__device__ __forceinline__ void scan_chunk(const int* __restrict__ cnt, int D, int rows,
                                           int* __restrict__ col_ptr, int* __restrict__ heavy_n,
                                           int2* __restrict__ heavy_items, int chunk, int* s_wave,
                                           int* s_hbase) {
  constexpr int COLS = NT * 4;
  const int t = threadIdx.x;
  const int ncols = D + 1;
  const int c0 = chunk * COLS, c1 = min(ncols, c0 + COLS);
  int pre = 0;  // all counts before the chunk (< D: column D is the last), 32 loads per thread
  for (int b = 0; b < c0; b += NT * 32) {
    int x[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int c = b + u * NT + t;
      x[u] = cnt[c < c0 ? c : 0];
    }
#pragma unroll
    for (int u = 0; u < 32; ++u) pre += (b + u * NT + t < c0) ? x[u] : 0;
  }
  int tot;
  (void)block_excl_scan<NT>(pre, s_wave, tot);
  const int base = tot;
  int v[4], sum = 0;
  const int cb = c0 + t * 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = cb + k;
    v[k] = c < c1 ? (c < D ? cnt[c] : rows) : 0;
    sum += v[k];
  }
  int run = base + block_excl_scan<NT>(sum, s_wave, tot);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (cb + k < c1) col_ptr[cb + k] = run;
    run += v[k];
  }
  if (c1 == ncols && t == 0) col_ptr[ncols] = base + tot;
  // heavy work items of this chunk
  int hi[4], hsum = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    hi[k] = v[k] > kLightEntries ? cdiv(v[k], kHeavyItem) : 0;
    hsum += hi[k];
  }
  int htot;
  int hrun = block_excl_scan<NT>(hsum, s_wave, htot);
  if (t == 0) *s_hbase = htot ? atomicAdd(heavy_n, htot) : 0;
  __syncthreads();
  hrun += *s_hbase;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    for (int i = 0; i < hi[k]; ++i) heavy_items[hrun++] = make_int2(cb + k, i);
}

__global__ __launch_bounds__(kTB) void k_csc_scan_multi(const int* __restrict__ cnt, int D, int rows,
                                                        int* __restrict__ col_ptr,
                                                        int* __restrict__ heavy_n,
                                                        int2* __restrict__ heavy_items) {
  __shared__ int s_wave[kTB / 64];
  __shared__ int s_hbase;
  scan_chunk<kTB>(cnt, D, rows, col_ptr, heavy_n, heavy_items, blockIdx.x, s_wave, &s_hbase);
}

// rows 4b .. 4b+3 of the scatter (one wave each); cnt cleared grid-stride over the nb blocks
__device__ __forceinline__ void scatter_rows(const int* __restrict__ indptr,
                                             const int* __restrict__ indices,
                                             const float* __restrict__ values, int rows, int D,
                                             const int* __restrict__ col_ptr,
                                             const int* __restrict__ pos_tmp, int* __restrict__ cnt,
                                             int* __restrict__ csc_row, float* __restrict__ csc_val,
                                             int* __restrict__ csc_col, int b, int nb) {
  for (int c = b * 256 + threadIdx.x; c < D; c += nb * 256) cnt[c] = 0;
  const int row = b * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  if (row >= rows) return;
  const int lane = lane_id();
  const int s = indptr[row], e = indptr[row + 1];
  for (int k = s + lane; k < e; k += 64) {
    const int c = indices[k];
    const float v = values[k];
    const int pos = col_ptr[c] + pos_tmp[k];
    csc_row[pos] = row;
    csc_val[pos] = v;
    if (csc_col) csc_col[pos] = c;  // null on the rank path: only k_dw1_heavy's slices read it
  }
  if (lane == 0) {
    const int pos = col_ptr[D] + row;
    csc_row[pos] = row;
    csc_val[pos] = 1.0f;
    if (csc_col) csc_col[pos] = D;
  }
}

__global__ __launch_bounds__(256) void k_csc_scatter(const int* __restrict__ indptr,
                                                     const int* __restrict__ indices,
                                                     const float* __restrict__ values, int rows,
                                                     int D, const int* __restrict__ col_ptr,
                                                     const int* __restrict__ pos_tmp,
                                                     int* __restrict__ cnt,
                                                     int* __restrict__ csc_row,
                                                     float* __restrict__ csc_val,
                                                     int* __restrict__ csc_col) {
  scatter_rows(indptr, indices, values, rows, D, col_ptr, pos_tmp, cnt, csc_row, csc_val, csc_col,
               blockIdx.x, gridDim.x);
}

// ---- independent launches sharing one grid (fused-statistics train step) -----------------------
// k_spmm_scan: the FC1 SpMM rows beside the transpose's column scan (both depend only on
// k_csc_rank / the batch); k_sums_scatter: BN1's column sums beside the transpose's scatter.  One
// launch each instead of two: a kernel boundary saved, and the small scan / scatter work fills the
// gaps of the latency-bound SpMM / sums.  The scan and sums workgroups come first.
constexpr int kScanSmallNT = 256;
#ifndef DSSM_SCAN_LAST
#define DSSM_SCAN_LAST 0
#endif
#ifdef DSSM_WG_TL
// Diagnostics build only: per-wave start / end stamps of the training SpMM's row waves (row index)
__device__ unsigned long long g_spmm_tl[8192][2];
#endif
template <typename TW>
__global__ __launch_bounds__(256) void k_spmm_scan(const int* __restrict__ indptr,
                                                   const int* __restrict__ indices,
                                                   const float* __restrict__ values, int rows,
                                                   const TW* __restrict__ W, int ldw, int n,
                                                   const float* __restrict__ bias,
                                                   float* __restrict__ Z, int ldz,
                                                   const int* __restrict__ cnt, int D,
                                                   int* __restrict__ col_ptr,
                                                   int* __restrict__ heavy_n,
                                                   int2* __restrict__ heavy_items, int nscan) {
  __shared__ int s_wave[kScanSmallNT / 64];
  __shared__ int s_hbase;
  const int bxm = (int)blockIdx.x;
#if DSSM_SCAN_LAST  // the scan workgroups after the row workgroups in dispatch order
  const int nrow_blocks = (int)gridDim.x - nscan;
  if (bxm >= nrow_blocks)
    scan_chunk<kScanSmallNT>(cnt, D, rows, col_ptr, heavy_n, heavy_items, bxm - nrow_blocks, s_wave,
                             &s_hbase);
  else {
    const int rb = bxm;
#else
  if (bxm < nscan)
    scan_chunk<kScanSmallNT>(cnt, D, rows, col_ptr, heavy_n, heavy_items, bxm, s_wave, &s_hbase);
  else {
    const int rb = bxm - nscan;
#endif
#ifdef DSSM_WG_TL
    const int row = rb * 4 + (threadIdx.x >> 6);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#endif
    spmm_rows<TW>(indptr, indices, values, rows, W, ldw, n, bias, Z, ldz, rb);
#ifdef DSSM_WG_TL
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0 && row < rows && row < 8192) {
      g_spmm_tl[row][0] = t0;
      g_spmm_tl[row][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
  }
}

__global__ __launch_bounds__(256) void k_sums_scatter(const float* __restrict__ Z, int ldz, int ncol,
                                                      int row_split, double* __restrict__ fsum,
                                                      int nsum_x, int nsum,
                                                      const int* __restrict__ indptr,
                                                      const int* __restrict__ indices,
                                                      const float* __restrict__ values, int rows,
                                                      int D, const int* __restrict__ col_ptr,
                                                      const int* __restrict__ pos_tmp,
                                                      int* __restrict__ cnt,
                                                      int* __restrict__ csc_row,
                                                      float* __restrict__ csc_val,
                                                      int* __restrict__ csc_col, DetAcc det) {
  __shared__ double s_red[2][4][64];
  const int b = blockIdx.x;
  if (b < nsum)
    bn_sums_block<256>(Z, ldz, ncol, row_split, rows, fsum, b % nsum_x, b / nsum_x, s_red, det, nsum / nsum_x);
  else
    scatter_rows(indptr, indices, values, rows, D, col_ptr, pos_tmp, cnt, csc_row, csc_val,
                 csc_col, b - nsum, (int)gridDim.x - nsum);
}

// Fallback fill with per-entry global atomics (one wave per row).
__global__ __launch_bounds__(256) void k_csc_fill_global(const int* __restrict__ indptr,
                                                         const int* __restrict__ indices,
                                                         const float* __restrict__ values,
                                                         int rows, int D, int* __restrict__ cursor,
                                                         const int* __restrict__ col_ptr,
                                                         int* __restrict__ csc_row,
                                                         float* __restrict__ csc_val,
                                                         int* __restrict__ csc_col) {
  const int row = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
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

// Deterministic mode: the transpose's entries of every column put in row order.  The scatter /
// fill place a column's entries in an order set by atomics (per-block slot reservations, LDS
// histogram arrival), which changes the fp32 summation order of dW1 from run to run; this pass
// rewrites each column [col_ptr[c], col_ptr[c+1]) of (row_in, val_in) sorted by row into
// (row_out, val_out).  Every entry's slot is its rank by the key (row, value bits, input slot): a
// column holding a row once (always, from CountVectorizer) is thus in row order, and a column
// repeating a row (legal input) still gets an order that is a function of the batch alone (equal
// keys are identical entries).  Wave g of the grid's G waves takes the kSortCols columns g + k G
// (lane k loads column k's bounds; interleaved so the Zipf-hot columns spread out) and handles each
// by its length n (at C2: 8k of the 30k columns hold 1 entry, 10k 2..8, all but ~350 <= 64):
// * n <= kSortSmall: all the wave's such columns at once, one 8-lane group per column: lane r of
//   group k holds entry r and counts the group's entries with a smaller key (8 shuffles);
// * n <= 64, one column at a time: lane i holds entry i and counts the lanes with a smaller key (n
//   v_readlane steps); no LDS, no barrier;
// * n <= kSortWaveMax: the wave's own LDS bitmap of the column's rows (a window of kSortWin rows at a
//   time), a wave prefix count of the bitmap words gives every entry its slot; wave-synchronous
//   (fences, no workgroup barrier).  A window with fewer bits than entries (a repeated row) falls
//   back to the key rank, O(n^2);
// * longer (the Zipf-hot columns): listed, then the whole workgroup per listed column, the same
//   bitmap scheme over all the waves' words (a kSortWinWg-row window) with barriers.
// The virtual ones column (already in row order: slot col_ptr[D] + row) is copied by the whole grid.
// Round 6: the previous form gave every column a wave of 512-thread workgroups and ran the bitmap
// windows (four workgroup barriers each) for every column, empty ones included: 27.6 us at C2.
constexpr int kSortWaves = 4;
constexpr int kSortNT = 64 * kSortWaves;
constexpr int kSortCols = 8;                         // columns per wave
constexpr int kSortSmall = 8;                        // longest column of the 8-lane group path
constexpr int kSortWords = 4;                        // bitmap words per lane
constexpr int kSortWin = 64 * 32 * kSortWords;       // rows per window of a wave
constexpr int kSortWinWg = kSortWaves * kSortWin;    // rows per window of the workgroup
constexpr int kSortWaveMax = 512;
constexpr int kSortU = 8;                            // long columns: entries in flight per thread
static_assert(kSortCols * kSortSmall == 64, "one 8-lane group per column");
// diagnostics builds (wrong results), bits: 1 skip the group path, 2 the <= 64 path, 4 the
// wave-bitmap path, 8 the in-workgroup long path, 16 the long-column role (tools/sort_bench.py)
#ifndef DSSM_SORT_DIAG
#define DSSM_SORT_DIAG 0
#endif

__host__ __device__ inline int csc_sort_grid(int D) { return (D + kSortWaves * kSortCols - 1) / (kSortWaves * kSortCols); }

// rank of entry i among [s, e) by (row, value bits, slot): the duplicate-row fallback
__device__ __forceinline__ int sort_rank_slow(const int* __restrict__ row_in, const float* __restrict__ val_in,
                                              int s, int e, int i, int ri, unsigned bi) {
  int p = s;
  for (int j = s; j < e; ++j) {
    const int rj = row_in[j];
    const unsigned bj = __float_as_uint(val_in[j]);
    p += rj < ri || (rj == ri && (bj < bi || (bj == bi && j < i)));
  }
  return p;
}

// LDS written by some lanes of this wave and read by others: the wave's LDS operations execute in
// order, so a compiler fence is all the ordering needed
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The workgroup path for one long column c (every wave of the workgroup; block-uniform call).
__device__ __forceinline__ void sort_long_column(const int* __restrict__ col_ptr, int c, int rows,
                                                 const int* __restrict__ row_in, const float* __restrict__ val_in,
                                                 int* __restrict__ row_out, float* __restrict__ val_out,
                                                 unsigned* bits, int* wpre, int* s_wave) {
  const int t = threadIdx.x;
  const int s = col_ptr[c], e = col_ptr[c + 1];
  bool dup = false;
  int base = s;
  for (int w0 = 0; w0 < rows; w0 += kSortWinWg) {
#pragma unroll
    for (int j = 0; j < kSortWords; ++j) bits[t * kSortWords + j] = 0u;
    __syncthreads();
    int nin = 0;
    for (int i0 = s + t; i0 < e; i0 += kSortNT * kSortU) {  // kSortU loads in flight per thread
      int rr[kSortU];
#pragma unroll
      for (int u = 0; u < kSortU; ++u) {
        const int i = i0 + kSortNT * u;
        rr[u] = i < e ? row_in[i] - w0 : -1;
      }
#pragma unroll
      for (int u = 0; u < kSortU; ++u)
        if (rr[u] >= 0 && rr[u] < kSortWinWg) {
          atomicOr(&bits[rr[u] >> 5], 1u << (rr[u] & 31));
          ++nin;
        }
    }
    __syncthreads();
    unsigned m[kSortWords];
    int own = 0;
#pragma unroll
    for (int j = 0; j < kSortWords; ++j) {
      m[j] = bits[t * kSortWords + j];
      own += __popc(m[j]);
    }
    int total, nin_total;
    int run = block_excl_scan<kSortNT>(own, s_wave, total);
    (void)block_excl_scan<kSortNT>(nin, s_wave, nin_total);
#pragma unroll
    for (int j = 0; j < kSortWords; ++j) {
      wpre[t * kSortWords + j] = run;
      run += __popc(m[j]);
    }
    dup = dup || nin_total != total;
    __syncthreads();
    if (!dup)
      for (int i0 = s + t; i0 < e; i0 += kSortNT * kSortU) {
        int rr[kSortU];
        float vv[kSortU];
#pragma unroll
        for (int u = 0; u < kSortU; ++u) {
          const int i = i0 + kSortNT * u;
          rr[u] = i < e ? row_in[i] - w0 : -1;
          vv[u] = i < e ? val_in[i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kSortU; ++u) {
          const int r = rr[u];
          if (r >= 0 && r < kSortWinWg) {
            const int wd = r >> 5;
            const int p = base + wpre[wd] + __popc(bits[wd] & ((1u << (r & 31)) - 1u));
            row_out[p] = r + w0;
            val_out[p] = vv[u];
          }
        }
      }
    base += total;
    __syncthreads();
  }
  if (dup)
    for (int i = s + t; i < e; i += kSortNT) {
      const int ri = row_in[i];
      const float vi = val_in[i];
      const int p = sort_rank_slow(row_in, val_in, s, e, i, ri, __float_as_uint(vi));
      row_out[p] = ri;
      val_out[p] = vi;
    }
  __syncthreads();  // the LDS bitmap is reused by the next long column
}

// heavy_n / heavy_items (the rank transpose's heavy-column work list, csc_heavy_count): when given,
// the long columns (> kSortWaveMax entries) are sorted by kSortLongWgs extra workgroups that find
// them in the list (item 0 of each), so the column waves never wait for them; without the list a
// column wave hands its long columns to its own workgroup after its other columns.
constexpr int kSortLongWgs = 64;
// one pass of the long-column role lists at most ceil(kSortNT / kSortLongWgs) columns per workgroup
static_assert((kSortNT + kSortLongWgs - 1) / kSortLongWgs <= kSortWaves * kSortCols, "s_long holds a pass");
__global__ __launch_bounds__(kSortNT) void k_csc_sort_rows(const int* __restrict__ col_ptr, int D, int rows,
                                                           const int* __restrict__ row_in,
                                                           const float* __restrict__ val_in,
                                                           int* __restrict__ row_out,
                                                           float* __restrict__ val_out,
                                                           const int* __restrict__ heavy_n,
                                                           const int2* __restrict__ heavy_items,
                                                           int ncol_blocks) {
  __shared__ unsigned bits[kSortWaves * 64 * kSortWords];
  __shared__ int wpre[kSortWaves * 64 * kSortWords];
  __shared__ int s_wave[kSortWaves];
  __shared__ int s_long[kSortWaves * kSortCols];
  __shared__ int s_nlong;
  const int t = threadIdx.x, lane = t & 63;
  if ((int)blockIdx.x >= ncol_blocks) {  // the long-column role (workgroup-uniform)
    if (DSSM_SORT_DIAG & 16) return;
    // Every role workgroup walks the whole list (kSortNT items per pass, all loads in flight) and
    // numbers the long columns in list order -- item 0 of a column longer than kSortWaveMax, not the
    // ones column -- with a workgroup prefix count; workgroup j sorts those numbered j mod the role's
    // size, one at a time, so the Zipf-hot columns (often adjacent in the list) spread over the role
    const int nh = *heavy_n, nlw = (int)gridDim.x - ncol_blocks, j = (int)blockIdx.x - ncol_blocks;
    int seen = 0;  // long columns numbered in earlier passes (uniform)
    for (int b0 = 0; b0 < nh; b0 += kSortNT) {
      if (t == 0) s_nlong = 0;
      const int it = b0 + t;
      int c = -1;
      if (it < nh) {
        const int2 item = heavy_items[it];
        if (item.y == 0 && item.x < D && col_ptr[item.x + 1] - col_ptr[item.x] > kSortWaveMax) c = item.x;
      }
      int total;
      const int idx = seen + block_excl_scan<kSortNT>(c >= 0 ? 1 : 0, s_wave, total);
      if (c >= 0 && idx % nlw == j) s_long[min(atomicAdd(&s_nlong, 1), kSortWaves * kSortCols - 1)] = c;
      __syncthreads();
      const int nl = min(s_nlong, kSortWaves * kSortCols);  // <= ceil(kSortNT / nlw) = 4 at 64 workgroups
      for (int k = 0; k < nl; ++k)
        sort_long_column(col_ptr, s_long[k], rows, row_in, val_in, row_out, val_out, bits, wpre, s_wave);
      seen += total;
      __syncthreads();
    }
    return;
  }
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  unsigned* wbits = bits + wv * 64 * kSortWords;
  int* wp = wpre + wv * 64 * kSortWords;
  if (t == 0) s_nlong = 0;
  {  // the virtual ones column (in row order already), copied by the column workgroups
    const int o0 = col_ptr[D], on = col_ptr[D + 1] - o0;
    for (int i = blockIdx.x * kSortNT + t; i < on; i += ncol_blocks * kSortNT) {
      row_out[o0 + i] = row_in[o0 + i];
      val_out[o0 + i] = val_in[o0 + i];
    }
  }
  const int G = ncol_blocks * kSortWaves, gw = blockIdx.x * kSortWaves + wv;
  int cs = 0, cn = 0;  // lane k < kSortCols: column gw + k G
  if (lane < kSortCols) {
    const int c = gw + lane * G;
    if (c < D) {
      cs = col_ptr[c];
      cn = col_ptr[c + 1] - cs;
    }
  }
  {  // the short columns, one 8-lane group each (every lane runs the shuffles: no inactive sources)
    const int q = lane >> 3, r = lane & 7;
    const int s = __shfl(cs, q, 64), n = __shfl(cn, q, 64);
    const bool own = n <= kSortSmall && r < n;
    const int ri = own ? row_in[s + r] : 0;
    const unsigned bi = own ? __float_as_uint(val_in[s + r]) : 0u;
    int p = 0;
#pragma unroll
    for (int j = 0; j < kSortSmall; ++j) {
      const int rj = __shfl(ri, (q << 3) + j, 64);
      const unsigned bj = (unsigned)__shfl((int)bi, (q << 3) + j, 64);
      p += j < n && (rj < ri || (rj == ri && (bj < bi || (bj == bi && j < r))));
    }
    if (own && !(DSSM_SORT_DIAG & 1)) {
      row_out[s + p] = ri;
      val_out[s + p] = __uint_as_float(bi);
    }
  }
  // the entries of every column of 9..64 entries, loaded at once (lane i: entry i of column k), so
  // the one-column-at-a-time loop below waits for no load of them
  int pr[kSortCols];
  unsigned pb[kSortCols];
#pragma unroll
  for (int k = 0; k < kSortCols; ++k) {
    const int s = __builtin_amdgcn_readlane(cs, k), n = __builtin_amdgcn_readlane(cn, k);
    const bool own = n > kSortSmall && n <= 64 && lane < n;
    pr[k] = own ? row_in[s + lane] : 0;
    pb[k] = own ? __float_as_uint(val_in[s + lane]) : 0u;
  }
#pragma unroll
  for (int k = 0; k < kSortCols; ++k) {  // the longer ones, one at a time (wave-uniform bounds)
    const int s = __builtin_amdgcn_readlane(cs, k), n = __builtin_amdgcn_readlane(cn, k);
    const int e = s + n;
    if (n <= kSortSmall) continue;
    if ((DSSM_SORT_DIAG & 2) && n <= 64) continue;
    if ((DSSM_SORT_DIAG & 4) && n > 64 && n <= kSortWaveMax) continue;
    if ((DSSM_SORT_DIAG & 8) && n > kSortWaveMax) continue;
    if (n <= 64) {
      const bool own = lane < n;
      const int ri = pr[k];
      const unsigned bi = pb[k];
      int p = 0;
      for (int j = 0; j < n; ++j) {
        const int rj = __builtin_amdgcn_readlane(ri, j);
        const unsigned bj = (unsigned)__builtin_amdgcn_readlane((int)bi, j);
        p += rj < ri || (rj == ri && (bj < bi || (bj == bi && j < lane)));
      }
      if (own) {
        row_out[s + p] = ri;
        val_out[s + p] = __uint_as_float(bi);
      }
    } else if (n <= kSortWaveMax) {
      bool dup = false;  // wave-uniform
      int base = s;
      for (int w0 = 0; w0 < rows && !dup; w0 += kSortWin) {
#pragma unroll
        for (int j = 0; j < kSortWords; ++j) wbits[lane * kSortWords + j] = 0u;
        wave_lds_sync();
        int nin = 0;  // the column's entries in this window (a repeated row: more than its bits)
        int rr[kSortWaveMax / 64];  // a lane's entries, every load in flight first
#pragma unroll
        for (int u = 0; u < kSortWaveMax / 64; ++u) {
          const int i = s + lane + 64 * u;
          rr[u] = i < e ? row_in[i] - w0 : -1;
        }
#pragma unroll
        for (int u = 0; u < kSortWaveMax / 64; ++u)
          if (rr[u] >= 0 && rr[u] < kSortWin) {
            atomicOr(&wbits[rr[u] >> 5], 1u << (rr[u] & 31));
            ++nin;
          }
        wave_lds_sync();
        unsigned m[kSortWords];
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < kSortWords; ++j) {
          m[j] = wbits[lane * kSortWords + j];
          cnt += __popc(m[j]);
        }
        int inc = cnt;  // wave inclusive scan of the lanes' counts
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int y = __shfl_up(inc, d, 64);
          if (lane >= d) inc += y;
        }
        int run = inc - cnt;
#pragma unroll
        for (int j = 0; j < kSortWords; ++j) {
          wp[lane * kSortWords + j] = run;
          run += __popc(m[j]);
        }
        const int total = __shfl(inc, 63, 64);
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) nin += __shfl_xor(nin, d, 64);
        dup = nin != total;
        wave_lds_sync();
        if (!dup) {
          float vv[kSortWaveMax / 64];
#pragma unroll
          for (int u = 0; u < kSortWaveMax / 64; ++u) {
            const int i = s + lane + 64 * u;
            vv[u] = i < e ? val_in[i] : 0.f;
          }
#pragma unroll
          for (int u = 0; u < kSortWaveMax / 64; ++u) {
            const int r = rr[u];
            if (r >= 0 && r < kSortWin) {
              const int wd = r >> 5;
              const int p = base + wp[wd] + __popc(wbits[wd] & ((1u << (r & 31)) - 1u));
              row_out[p] = r + w0;
              val_out[p] = vv[u];
            }
          }
        }
        base += total;
        wave_lds_sync();
      }
      if (dup)  // every entry ranked by its key (earlier windows' slots are rewritten the same way)
        for (int i = s + lane; i < e; i += 64) {
          const int ri = row_in[i];
          const float vi = val_in[i];
          const int p = sort_rank_slow(row_in, val_in, s, e, i, ri, __float_as_uint(vi));
          row_out[p] = ri;
          val_out[p] = vi;
        }
    } else if (!heavy_n && lane == 0) {  // with the heavy list the long-column role takes it
      s_long[atomicAdd(&s_nlong, 1)] = gw + k * G;  // the workgroup's pass below (order irrelevant)
    }
  }
  __syncthreads();
  const int nlong = s_nlong;  // workgroup-uniform
  for (int k = 0; k < nlong; ++k)  // the long columns, one at a time with every wave
    sort_long_column(col_ptr, s_long[k], rows, row_in, val_in, row_out, val_out, bits, wpre, s_wave);
}

// ---- dW1 ---------------------------------------------------------------------------------------
// Light columns (<= kLight entries): one wave sums and stores the whole row; heavy rows get 0
// here (the heavy kernel adds into them afterwards).
template <typename TZ>
__global__ __launch_bounds__(256) void k_dw1_light(const int* __restrict__ col_ptr,
                                                   const int* __restrict__ csc_row,
                                                   const float* __restrict__ csc_val, int D,
                                                   const TZ* __restrict__ dZ, int lddz, int n,
                                                   float* __restrict__ G, int mode) {
  const int c = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  if (c > D) return;
  const int lane = lane_id();
  const int s = col_ptr[c], e = col_ptr[c + 1];
  // mode 0: light rows summed, heavy rows zeroed (the heavy kernels add into them); deterministic
  // mode without the heavy-item list, one wave per column in CSC order: 1 every row, 2 the heavy
  // rows only (the fused W1 Adam gathers the light ones itself)
  if (mode == 2 && e - s <= kLightEntries) return;
  const bool heavy = mode == 0 && e - s > kLightEntries;
  for (int c0 = 0; c0 < n; c0 += 512) {
    const int cc = c0 + lane * 8;
    const int nvalid = n - cc;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (!heavy) gather_accumulate(csc_row, csc_val, s, e, dZ, lddz, cc, nvalid, acc);
    if (nvalid > 0) store8n(G + (size_t)c * n + cc, acc, nvalid);
  }
}

// Heavy columns: fixed 64-entry slices of the CSC arrays, summed per column run, transposed
// through LDS so each fp32 atomic wave-instruction covers 64 consecutive floats.
template <typename TZ>
__global__ __launch_bounds__(256) void k_dw1_heavy(const int* __restrict__ col_ptr,
                                                   const int* __restrict__ csc_row,
                                                   const float* __restrict__ csc_val,
                                                   const int* __restrict__ csc_col, int D,
                                                   const TZ* __restrict__ dZ, int lddz, int n,
                                                   float* __restrict__ G) {
  __shared__ float sbuf[4][512];
  const int wv = threadIdx.x >> 6;
  const int chunk = blockIdx.x * 4 + wv;
  const int total = col_ptr[D + 1];
  const int j0 = chunk * 64;
  if (j0 >= total) return;
  const int j1 = min(j0 + 64, total);
  const int lane = lane_id();
  int j = j0;
  while (j < j1) {
    const int c = csc_col[j];
    const int cs = col_ptr[c], cend = col_ptr[c + 1];
    const int ce = min(cend, j1);
    if (cend - cs > kLightEntries) {
      for (int c0 = 0; c0 < n; c0 += 512) {
        const int cc = c0 + lane * 8;
        const int nvalid = n - cc;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        gather_accumulate(csc_row, csc_val, j, ce, dZ, lddz, cc, nvalid, acc);
        if (nvalid > 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) sbuf[wv][lane * 8 + i] = acc[i];
        }
        __builtin_amdgcn_wave_barrier();
        const int m = min(512, n - c0);
        float* g = G + (size_t)c * n + c0;
        for (int i = lane; i < m; i += 64) atomicAdd(g + i, sbuf[wv][i]);
        __builtin_amdgcn_wave_barrier();
      }
    }
    j = ce;
  }
}

// Heavy columns by work items of kHeavyItem entries: 16 waves x 16 entries each (two gather
// batches), the 16 partial rows summed through LDS; a column that is one item is STORED (no
// atomics), longer columns add their items' rows with fp32 atomics (ones column, Zipf-hot
// trigrams: cdiv(count, 256) atomic row-adds instead of one per 64 entries).
constexpr int kHeavyWaves = 16, kHeavyPerWave = kHeavyItem / kHeavyWaves;
template <typename TZ>
__global__ __launch_bounds__(1024) void k_dw1_heavy_items(const int* __restrict__ col_ptr,
                                                         const int* __restrict__ csc_row,
                                                         const float* __restrict__ csc_val,
                                                         const int* __restrict__ heavy_n,
                                                         const int2* __restrict__ items,
                                                         const TZ* __restrict__ dZ, int lddz, int n,
                                                         float* __restrict__ G, float* __restrict__ slab) {
  __shared__ float part[kHeavyWaves][512];
  const int wv = threadIdx.x >> 6, lane = lane_id();
  const int nitems = *heavy_n;
  for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
    const int2 item = items[it];
    const int c = item.x;
    const int cs = col_ptr[c], ce = col_ptr[c + 1];
    const int i0 = cs + item.y * kHeavyItem;
    const int s = min(ce, i0 + wv * kHeavyPerWave), e = min(ce, s + kHeavyPerWave);
    const bool single = ce - cs <= kHeavyItem;
    for (int c0 = 0; c0 < n; c0 += 512) {
      const int cc = c0 + lane * 8;
      const int nvalid = n - cc;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (s < e) gather_accumulate(csc_row, csc_val, s, e, dZ, lddz, cc, nvalid, acc);
#pragma unroll
      for (int i = 0; i < 8; ++i) part[wv][lane * 8 + i] = acc[i];
      __syncthreads();
      const int m = min(512, n - c0);
      for (int i = threadIdx.x; i < m; i += 1024) {
        float a = 0.f;
#pragma unroll
        for (int w = 0; w < kHeavyWaves; ++w) a += part[w][i];
        float* g = G + (size_t)c * n + c0 + i;
        if (single) *g = a;
        else if (slab) slab[(size_t)it * n + c0 + i] = a;  // deterministic: summed in item order
        else atomicAdd(g, a);
      }
      __syncthreads();
    }
  }
}

// Deterministic mode: the multi-item heavy columns' rows from their items' partial rows, summed in
// item order (one workgroup per column, at its first item).
__global__ __launch_bounds__(256) void k_dw1_heavy_reduce(const int* __restrict__ col_ptr,
                                                          const int* __restrict__ heavy_n,
                                                          const int2* __restrict__ items, int n,
                                                          const float* __restrict__ slab,
                                                          float* __restrict__ G) {
  const int nitems = *heavy_n;
  for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
    const int2 item = items[it];
    if (item.y != 0) continue;
    const int c = item.x;
    const int nit = cdiv(col_ptr[c + 1] - col_ptr[c], kHeavyItem);
    if (nit < 2) continue;
    for (int j = threadIdx.x; j < n; j += 256) {
      float a = 0.f;
      for (int k = 0; k < nit; ++k) a += slab[(size_t)(it + k) * n + j];
      G[(size_t)c * n + j] = a;
    }
  }
}

}  // namespace

int eval_coef_blocks(const EvalCoef& e) {
  int items = 0;
  for (int l = 0; l < e.L; ++l) items += 2 * e.ld[l];
  return cdiv(items, 256);
}

// bf16 weight rows: padded to a multiple of 8 elements with zero pads (the shadows), or tight at
// stride n (the parameter wire), whose last row the u16t instances read 8 B past (gather.h)
static bool bf16_rows_ok(int ldw, int n) {
  if (ldw % 8 == 0) return ldw >= n;
  return ldw == n && n % 4 == 0 && n >= 8;
}

hipError_t launch_spmm_fwd(const int* indptr, const int* indices, const float* values, int rows,
                           const void* W, bool w_bf16, int ldw, int n, const float* bias, float* Z,
                           int ldz, hipStream_t s, const EvalCoef* ec, bool relu, bool z_bf16) {
  EvalCoef e{};
  const int ne = ec ? eval_coef_blocks(*ec) : 0;
  if (ec) e = *ec;
  dim3 grid(ne + cdiv(rows, 4)), block(256);
  if (w_bf16 && !bf16_rows_ok(ldw, n)) return hipErrorInvalidValue;
  if (z_bf16) {  // bf16 output (functional API: bf16 W, no eval coefficients)
    if (!w_bf16 || ldw % 8 || ec || ldz % 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_spmm_fwd<u16, u16>), grid, block, 0, s, indptr, indices, values, rows, (const u16*)W,
                       ldw, n, bias, reinterpret_cast<u16*>(Z), ldz, e, ne, relu ? 1 : 0);
    return hipGetLastError();
  }
  if (w_bf16 && ldw % 8)  // the parameter wire's tight rows
    hipLaunchKernelGGL(k_spmm_fwd<u16t>, grid, block, 0, s, indptr, indices, values, rows,
                       (const u16t*)W, ldw, n, bias, Z, ldz, e, ne, relu ? 1 : 0);
  else if (w_bf16)
    hipLaunchKernelGGL(k_spmm_fwd<u16>, grid, block, 0, s, indptr, indices, values, rows,
                       (const u16*)W, ldw, n, bias, Z, ldz, e, ne, relu ? 1 : 0);
  else
    hipLaunchKernelGGL(k_spmm_fwd<float>, grid, block, 0, s, indptr, indices, values, rows,
                       (const float*)W, ldw, n, bias, Z, ldz, e, ne, relu ? 1 : 0);
  return hipGetLastError();
}

bool csc_rank_supported(int D) {
  return (size_t)D * sizeof(int) + (kCscListMax + 64) * sizeof(int) <= 160 * 1024 &&
         D + 1 <= 1024 * kScanMultiCols;
}

hipError_t launch_spmm_scan(const int* indptr, const int* indices, const float* values, int rows,
                            const void* W, bool w_bf16, int ldw, int n, const float* bias, float* Z, int ldz,
                            int D, int max_nnz, int* scratch, int* col_ptr, hipStream_t s) {
  int* cnt = scratch;
  int* heavy_n = csc_heavy_count(scratch, D, max_nnz);
  int2* heavy_items = reinterpret_cast<int2*>(heavy_n + 64);
  const int nscan = cdiv(D + 1, kScanSmallNT * 4);
  if (w_bf16 ? !bf16_rows_ok(ldw, n) : (ldw < n || ldw % 4)) return hipErrorInvalidValue;
  const dim3 grid(nscan + cdiv(rows, 4));
  if (!w_bf16)  // fp32 parity mode
    hipLaunchKernelGGL(k_spmm_scan<float>, grid, dim3(256), 0, s, indptr, indices, values, rows,
                       (const float*)W, ldw, n, bias, Z, ldz, cnt, D, col_ptr, heavy_n, heavy_items,
                       nscan);
  else if (ldw % 8)  // the parameter wire's tight rows (RawRow8<u16t>)
    hipLaunchKernelGGL(k_spmm_scan<u16t>, grid, dim3(256), 0, s, indptr, indices, values, rows,
                       (const u16t*)W, ldw, n, bias, Z, ldz, cnt, D, col_ptr, heavy_n, heavy_items,
                       nscan);
  else
    hipLaunchKernelGGL(k_spmm_scan<u16>, grid, dim3(256), 0, s, indptr, indices, values, rows,
                       (const u16*)W, ldw, n, bias, Z, ldz, cnt, D, col_ptr, heavy_n, heavy_items,
                       nscan);
  return hipGetLastError();
}

CscScatter csc_scatter_args(const int* indptr, const int* indices, const float* values, int rows, int D,
                            int* scratch, const int* col_ptr, int* csc_row, float* csc_val, int* csc_col) {
  constexpr int nb = 384;  // scatter workgroups beside the cosine launch
  // cnt and the per-entry ranks where launch_csc_build keeps them
  return CscScatter{indptr, indices, values, rows, D, col_ptr, scratch + 2 * (D + 1 + 64), scratch,
                    csc_row, csc_val, csc_col, std::min(nb, cdiv(rows, 4))};
}

hipError_t launch_sums_scatter(const float* Z, int ldz, int n, int row_split, double* fsum,
                               const int* indptr, const int* indices, const float* values, int rows,
                               int D, int max_nnz, int* scratch, const int* col_ptr, int* csc_row,
                               float* csc_val, int* csc_col, hipStream_t s, CscScatter* scatter_out,
                               const DetAcc* det) {
  (void)max_nnz;
  if (row_split % kSumsRows) return hipErrorInvalidValue;
  int* cnt = scratch;
  int* pos_tmp = scratch + 2 * (D + 1 + 64);
  const int nsum_x = cdiv(ldz, 64), nsum = nsum_x * cdiv(rows, kSumsRows);
  if (det && det->slab && (cdiv(rows, kSumsRows) > det->cap || nsum_x > kDetTiles)) return hipErrorInvalidValue;
  if (scatter_out)
    *scatter_out = csc_scatter_args(indptr, indices, values, rows, D, scratch, col_ptr, csc_row, csc_val, csc_col);
  hipLaunchKernelGGL(k_sums_scatter, dim3(nsum + (scatter_out ? 0 : cdiv(rows, 4))), dim3(256), 0, s, Z, ldz, n,
                     row_split, fsum, nsum_x, nsum, indptr, indices, values, rows, D, col_ptr, pos_tmp, cnt,
                     csc_row, csc_val, csc_col, det ? *det : DetAcc{});
  return hipGetLastError();
}

size_t csc_heavy_cap(int rows, int max_nnz) { return (size_t)(max_nnz + rows) / 32 + 64; }

CscRankRole csc_rank_role_args(const int* indptr, const int* indices, int rows, int D, int* scratch,
                               double* zero, int nzero) {
  // cnt and the per-entry ranks where launch_csc_build keeps them
  return CscRankRole{indptr, indices, rows, scratch, scratch + 2 * (D + 1 + 64), zero, nzero,
                     cdiv(rows, kRankRoleRows)};
}

size_t csc_scratch_ints(int D, int rows, int max_nnz) {
  // cnt (D+1, padded) + cursor (D+1) + rank / position per entry (max_nnz) + heavy-item count
  // (64, padded) + heavy items (int2 each) + per-column heavy tickets (D+1, padded)
  return (size_t)2 * (D + 1 + 64) + (size_t)max_nnz + 64 + 64 + 2 * csc_heavy_cap(rows, max_nnz) +
         (D + 1 + 64);
}

unsigned* csc_heavy_tickets(int* scratch, int D, int rows, int max_nnz) {
  return reinterpret_cast<unsigned*>(csc_heavy_count(scratch, D, max_nnz) + 64 +
                                     2 * csc_heavy_cap(rows, max_nnz));
}

int* csc_heavy_count(int* scratch, int D, int max_nnz) {
  return scratch + 2 * (D + 1 + 64) + max_nnz + 64;
}

hipError_t launch_csc_sort(const int* col_ptr, int rows, int D, const int* row_in, const float* val_in,
                           int* row_out, float* val_out, hipStream_t s, int* scratch, int max_nnz) {
  // scratch (the rank transpose's): its heavy-column list routes the long columns to their own role
  const int* hn = scratch ? csc_heavy_count(scratch, D, max_nnz) : nullptr;
  const int2* hi = hn ? reinterpret_cast<const int2*>(hn + 64) : nullptr;
  const int nb = csc_sort_grid(D);
  hipLaunchKernelGGL(k_csc_sort_rows, dim3(nb + (hn ? kSortLongWgs : 0)), dim3(kSortNT), 0, s, col_ptr, D,
                     rows, row_in, val_in, row_out, val_out, hn, hi, nb);
  return hipGetLastError();
}

hipError_t launch_csc_build(const int* indptr, const int* indices, const float* values, int rows,
                            int D, int max_nnz, int* scratch, int* col_ptr, int* csc_row,
                            float* csc_val, int* csc_col, hipStream_t s, double* zero,
                            int nzero, bool rank_path, bool rank_only, int* sort_row,
                            float* sort_val) {
  // deterministic mode (sort_row != null): the scatter / fill write into (sort_row, sort_val),
  // then k_csc_sort_rows puts every column in row order into (csc_row, csc_val)
  if (sort_row && (!sort_val || rank_only)) return hipErrorInvalidValue;
  int* out_row = sort_row ? sort_row : csc_row;
  float* out_val = sort_row ? sort_val : csc_val;
  int* cnt = scratch;  // zero between steps (re-zeroed by k_csc_scan / k_csc_scatter)
  int* cursor = scratch + (D + 1 + 64);
  int* rank_tmp = cursor + (D + 1 + 64);
  int* heavy_n = csc_heavy_count(scratch, D, max_nnz);
  int2* heavy_items = reinterpret_cast<int2*>(heavy_n + 64);
  const size_t lds = (size_t)D * sizeof(int);
  if (rank_path && csc_rank_supported(D)) {
    const int rpb = cdiv(rows, kCscRankBlocks);
    const int grid = cdiv(rows, rpb);
    hipLaunchKernelGGL(k_csc_rank, dim3(grid), dim3(kTB), lds, s, indptr, indices, rows, D, rpb, cnt,
                       rank_tmp, zero, nzero, heavy_n);
    if (rank_only) return hipGetLastError();  // scan and scatter ride in later launches
    hipLaunchKernelGGL(k_csc_scan_multi, dim3(cdiv(D + 1, kScanMultiCols)), dim3(kTB), 0, s, cnt, D,
                       rows, col_ptr, heavy_n, heavy_items);
    hipLaunchKernelGGL(k_csc_scatter, dim3(cdiv(rows, 4)), dim3(256), 0, s, indptr, indices, values,
                       rows, D, col_ptr, rank_tmp, cnt, out_row, out_val, csc_col);
  } else if (lds + (size_t)(cdiv(rows, max(1, min(32, cdiv(rows, 64)))) + 1) * sizeof(int) <= 156 * 1024) {
    // Few fat blocks (one CU each: the LDS histogram takes 120 KB): enough to keep the transpose
    // short while leaving most CUs to the forward pass it overlaps on the main stream.
    const int nblk = max(1, min(32, cdiv(rows, 64)));
    const int rpb = cdiv(rows, nblk);
    const int grid = cdiv(rows, rpb);
    hipLaunchKernelGGL(k_csc_hist, dim3(grid), dim3(kTB), lds, s, indptr, indices, rows, D, rpb,
                       cnt, zero, nzero);
    hipLaunchKernelGGL(k_csc_scan, dim3(1), dim3(1024), 0, s, cnt, D, rows, col_ptr, cursor);
    hipLaunchKernelGGL(k_csc_fill, dim3(grid), dim3(kTB), lds + (size_t)(rpb + 1) * sizeof(int), s,
                       indptr, indices, values, rows, D, rpb, cursor, col_ptr, rank_tmp, out_row,
                       out_val, csc_col);
  } else {
    if (nzero) {
      const hipError_t e = zero_bytes_async(zero, (size_t)nzero * sizeof(double), s);
      if (e != hipSuccess) return e;
    }
    const int cblocks = max(1, min(cdiv(max_nnz, 256), 2048));
    hipLaunchKernelGGL(k_csc_count_global, dim3(cblocks), dim3(256), 0, s, indptr, indices, rows,
                       cnt);
    hipLaunchKernelGGL(k_csc_scan, dim3(1), dim3(1024), 0, s, cnt, D, rows, col_ptr, cursor);
    hipLaunchKernelGGL(k_csc_fill_global, dim3(cdiv(rows, 4)), dim3(256), 0, s, indptr, indices,
                       values, rows, D, cursor, col_ptr, out_row, out_val, csc_col);
  }
  if (sort_row)  // the rank path's scan listed the heavy columns: the long ones get their own role
    return launch_csc_sort(col_ptr, rows, D, sort_row, sort_val, csc_row, csc_val, s,
                           rank_path && csc_rank_supported(D) ? scratch : nullptr, max_nnz);
  return hipGetLastError();
}

hipError_t launch_dw1(const int* col_ptr, const int* csc_row, const float* csc_val,
                      const int* csc_col, int D, int rows, int max_nnz, const void* dZ,
                      bool dz_bf16, int lddz, int n, float* G, bool light, hipStream_t s,
                      int* scratch, float* heavy_slab) {
  dim3 block(256);
  dim3 g1(cdiv(D + 1, 4));
  dim3 g2(max(1, cdiv(cdiv(max_nnz + rows, 64), 4)));
  // heavy-item list of the rank transpose (scratch != null), else 64-entry slices
  const int* heavy_n = scratch ? csc_heavy_count(scratch, D, max_nnz) : nullptr;
  const int2* items = scratch ? reinterpret_cast<const int2*>(heavy_n + 64) : nullptr;
  const int gi = 512;
  // deterministic (heavy_slab != null): multi-item columns through the slab and an ordered sum;
  // without the item list every column is summed by one wave
  const bool serial = heavy_slab && !items;
  const int mode = serial ? (light ? 1 : 2) : 0;
#define DSSM_DW1(T)                                                                             \
  if (light || serial)                                                                          \
    hipLaunchKernelGGL(k_dw1_light<T>, g1, block, 0, s, col_ptr, csc_row, csc_val, D,           \
                       (const T*)dZ, lddz, n, G, mode);                                         \
  if (items) {                                                                                  \
    hipLaunchKernelGGL(k_dw1_heavy_items<T>, dim3(gi), dim3(1024), 0, s, col_ptr, csc_row,      \
                       csc_val, heavy_n, items, (const T*)dZ, lddz, n, G, heavy_slab);          \
    if (heavy_slab)                                                                             \
      hipLaunchKernelGGL(k_dw1_heavy_reduce, dim3(gi), dim3(256), 0, s, col_ptr, heavy_n,       \
                         items, n, heavy_slab, G);                                              \
  } else if (!serial) {                                                                         \
    hipLaunchKernelGGL(k_dw1_heavy<T>, g2, block, 0, s, col_ptr, csc_row, csc_val, csc_col, D,  \
                       (const T*)dZ, lddz, n, G);                                               \
  }
  if (dz_bf16) {
    DSSM_DW1(u16)
  } else {
    DSSM_DW1(float)
  }
#undef DSSM_DW1
  return hipGetLastError();
}

}  // namespace dssm

#ifdef DSSM_WG_TL
extern "C" int dssm_debug_spmm_timeline(unsigned long long* out, int n) {
  if (n > 8192) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dssm::g_spmm_tl), sizeof(unsigned long long) * 2 * n, 0) == hipSuccess
             ? 0 : -2;
}
#endif
