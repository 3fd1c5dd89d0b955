// The decay-only Adam update of W1's untouched rows (TF1.x ApplyAdam is dense,
// so a row with no CSC entry this step still gets m, v decayed and p moved with g = 0): the Adam
// launch's flat streaming role (adam.hip), every lane busy instead of a wave per row.  It needs only
// the batch's column pointers and the step's beta powers.  (Spreading it as extra workgroups over
// the step's latency-bound launches was measured slower: the host launches grew by more than the
// Adam launch shrank, 205 -> 211 us/step.)
#pragma once
#include "common.h"

namespace dssm {

__device__ __forceinline__ void adam1(float& p, float& m, float& v, float g, float alpha, float b1c,
                                      float b2c, float eps) {
  m += (g - m) * b1c;
  v += (g * g - v) * b2c;
  p -= (m * alpha) / (sqrtf(v) + eps);
}

struct FlatSlice {
  float* p;
  float* m;
  float* v;
  uint16_t* shadow;  // W1's bf16 shadow [D x ldsh] (null: none)
  int ldsh;
  int n, D;          // W1 row length, rows of W1 (the [W1; b1] block has D + 1)
  const int* col_ptr;
  const float* st;   // {beta1_power, beta2_power} of this step
  float lr, b1c, b2c, eps;
  int64_t i4_begin, i4_end;  // float4 range of the [W1; b1] block
  int nblocks;               // workgroups given to the slice
};

// Workgroup bi of the slice's nblocks: float4 streaming over the untouched rows of its range.
__device__ __forceinline__ void flat_untouched(const FlatSlice& f, int bi) {
  const float alpha = f.lr * sqrtf(1.0f - f.st[1]) / (1.0f - f.st[0]);
  for (int64_t i = f.i4_begin + (int64_t)bi * blockDim.x + threadIdx.x; i < f.i4_end;
       i += (int64_t)f.nblocks * blockDim.x) {
    const int c = (int)((i * 4) / f.n);
    if (f.col_ptr[c + 1] != f.col_ptr[c]) continue;
    float4 pp = ld_stream4(f.p + i * 4);
    float4 mm = ld_stream4(f.m + i * 4);
    float4 vv = ld_stream4(f.v + i * 4);
    adam1(pp.x, mm.x, vv.x, 0.f, alpha, f.b1c, f.b2c, f.eps);
    adam1(pp.y, mm.y, vv.y, 0.f, alpha, f.b1c, f.b2c, f.eps);
    adam1(pp.z, mm.z, vv.z, 0.f, alpha, f.b1c, f.b2c, f.eps);
    adam1(pp.w, mm.w, vv.w, 0.f, alpha, f.b1c, f.b2c, f.eps);
    st_stream4(f.p + i * 4, pp);
    st_stream4(f.m + i * 4, mm);
    st_stream4(f.v + i * 4, vv);
    if (f.shadow && c < f.D) {
      uint2 q;
      q.x = pack2bf(pp.x, pp.y);
      q.y = pack2bf(pp.z, pp.w);
      *reinterpret_cast<uint2*>(f.shadow + (size_t)c * f.ldsh + (i * 4 - (int64_t)c * f.n)) = q;
    }
  }
}

}  // namespace dssm
