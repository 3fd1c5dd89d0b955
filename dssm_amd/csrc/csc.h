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
      s.csc_col[pos] = c;
    }
    if (lane == 0) {
      const int pos = s.col_ptr[s.D] + row;
      s.csc_row[pos] = row;
      s.csc_val[pos] = 1.0f;
      s.csc_col[pos] = s.D;
    }
  }
}

}  // namespace dssm
