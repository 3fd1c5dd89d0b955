// The CSC transpose's scatter (dW1 = [X | 1]^T dZ1 needs X^T) as a workgroup role
// that can ride in any launch between the column scan and the Adam step (by default the cosine
// launch, whose 257 latency-bound workgroups leave most CU slots free): entry k of CSR row r goes
// to col_ptr[c] + rank[k] (its slot reserved by k_csc_rank), the virtual ones column's entry of
// row r to col_ptr[D] + r; the histogram counts are re-zeroed for the next step's transpose.
#pragma once
#include "common.h"

namespace dssm {

struct CscScatter {
  const int* indptr;
  const int* indices;
  const float* values;
  int rows, D;
  const int* col_ptr;
  const int* rank;  // per-entry slot within its column (k_csc_rank)
  int* cnt;         // per-column counts, cleared here
  int* csc_row;
  float* csc_val;
  int* csc_col;
  int nblocks;      // workgroups given to the role (0: none)
};

// Workgroup b of the role's nblocks: one wave per CSR row, grid-stride over rows.
__device__ __forceinline__ void csc_scatter_role(const CscScatter& s, int b) {
  const int nt = blockDim.x, nw = nt >> 6;
  for (int c = b * nt + (int)threadIdx.x; c < s.D; c += s.nblocks * nt) s.cnt[c] = 0;
  const int lane = threadIdx.x & 63;
  for (int row = b * nw + (int)(threadIdx.x >> 6); row < s.rows; row += s.nblocks * nw) {
    const int st = s.indptr[row], e = s.indptr[row + 1];
    for (int k = st + lane; k < e; k += 64) {
      const int c = s.indices[k];
      const float v = s.values[k];
      const int pos = s.col_ptr[c] + s.rank[k];
      s.csc_row[pos] = row;
      s.csc_val[pos] = v;
      if (s.csc_col) s.csc_col[pos] = c;  // null on the plan's rank path (nothing reads it)
    }
    if (lane == 0) {
      const int pos = s.col_ptr[s.D] + row;
      s.csc_row[pos] = row;
      s.csc_val[pos] = 1.0f;
      if (s.csc_col) s.csc_col[pos] = s.D;
    }
  }
}

}  // namespace dssm

namespace dssm {

// The rank pass of the CSC transpose (k_csc_rank's result: rank[k] = entry k's slot within its
// column, cnt[c] += the column's count) as a workgroup role of another launch of 256-thread
// workgroups, which cannot give the D-bin LDS histogram k_csc_rank uses: kRankRoleRows CSR rows
// per workgroup, the workgroup's distinct columns in an LDS hash table (open addressing, one
// 32-bit word per slot: column << 16 | count) that counts them, then ONE returning global atomic
// per (workgroup, distinct column) reserves the workgroup's range inside the column, as
// k_csc_rank does.  Fewer, fatter workgroups keep the same-address atomic chains on the Zipf-hot
// columns short.  A workgroup with more than kRankCap entries (the table would fill) takes its
// slots with one global atomic per entry instead: any mix of the two paths hands out distinct
// slots in [0, count).  Also clears `zero` (the next step's fused BN sums).  The role rides in
// the previous step's Adam launch (multi-step graphs), so the transpose's first launch leaves
// the step.  Needs D < 65535 (column ids in 16 bits).
#ifndef DSSM_RANK_ROWS
#define DSSM_RANK_ROWS 64
#endif
constexpr int kRankRoleRows = DSSM_RANK_ROWS;
constexpr int kRankHash = 4096;  // LDS slots, 16 KiB
constexpr int kRankCap = 2816;   // entries per workgroup on the hash path (table load <= 0.69)
constexpr int kRankPerThread = (kRankCap + 255) / 256;
constexpr int kRankMaxD = 65534;

struct CscRankRole {
  const int* indptr;
  const int* indices;
  int rows;
  int* cnt;      // per-column counts (zero on entry: cleared by the previous step's scatter)
  int* rank;     // per-entry slot within its column
  double* zero;  // cleared here
  int nzero;
  int nblocks;   // workgroups given to the role (0: none)
};

__device__ __forceinline__ void csc_rank_role(const CscRankRole& r, int b, unsigned* slot) {
  constexpr unsigned kEmpty = 0xffffffffu;
  const int t = threadIdx.x;
  for (int i = b * 256 + t; i < r.nzero; i += r.nblocks * 256) r.zero[i] = 0.0;
  const int r0 = b * kRankRoleRows, r1 = min(r.rows, r0 + kRankRoleRows);
  if (r0 >= r1) return;  // uniform over the workgroup
  const int e0 = r.indptr[r0], e1 = r.indptr[r1];
  if (e1 - e0 > kRankCap) {
    for (int e = e0 + t; e < e1; e += 256) r.rank[e] = atomicAdd(&r.cnt[r.indices[e]], 1);
    return;
  }
  for (int i = t; i < kRankHash; i += 256) slot[i] = kEmpty;
  __syncthreads();
  int hs[kRankPerThread], rk[kRankPerThread];
  int c[kRankPerThread];
#pragma unroll
  for (int u = 0; u < kRankPerThread; ++u) {  // every index load in flight first
    const int e = e0 + t + 256 * u;
    c[u] = e < e1 ? r.indices[e] : -1;
  }
#pragma unroll
  for (int u = 0; u < kRankPerThread; ++u) {
    hs[u] = -1;
    if (c[u] >= 0) {
      const unsigned key = (unsigned)c[u] << 16;
      unsigned h = ((unsigned)c[u] * 2654435761u) >> 20;  // 12 bits
      for (;;) {
        const unsigned k = atomicCAS(&slot[h], kEmpty, key);
        if (k == kEmpty || (k >> 16) == (unsigned)c[u]) break;
        h = (h + 1) & (kRankHash - 1);
      }
      hs[u] = (int)h;
      rk[u] = (int)(atomicAdd(&slot[h], 1u) & 0xffffu);
    }
  }
  __syncthreads();
  // every distinct column: its count -> the workgroup's base inside the column (all in flight)
  int got[kRankHash / 256];
#pragma unroll
  for (int u = 0; u < kRankHash / 256; ++u) {
    const unsigned v = slot[t + 256 * u];
    got[u] = v != kEmpty ? atomicAdd(&r.cnt[v >> 16], (int)(v & 0xffffu)) : 0;
  }
#pragma unroll
  for (int u = 0; u < kRankHash / 256; ++u) slot[t + 256 * u] = (unsigned)got[u];  // own slots only
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kRankPerThread; ++u)
    if (hs[u] >= 0) r.rank[e0 + t + 256 * u] = (int)slot[hs[u]] + rk[u];
}

}  // namespace dssm
