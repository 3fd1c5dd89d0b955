// Sparse row-gather accumulation shared by the SpMM, the dW1 kernels and the fused W1 Adam.
#pragma once
#include "common.h"

namespace dssm {

// Columns with at most this many CSC entries are "light": one wave sums the whole dW1 row.
constexpr int kLightEntries = 64;

// One gathered 8-column slice kept in its storage format until it is consumed, so a batch of
// in-flight bf16 rows costs 4 VGPRs each (not 8).
template <typename T> struct RawRow8;
template <> struct RawRow8<u16> {
  uint4 a;
  __device__ __forceinline__ void load(const u16* p, int) { a = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void fma(float v, float (&acc)[8]) const {
    acc[0] = __fmaf_rn(v, __uint_as_float(a.x << 16), acc[0]);
    acc[1] = __fmaf_rn(v, __uint_as_float(a.x & 0xffff0000u), acc[1]);
    acc[2] = __fmaf_rn(v, __uint_as_float(a.y << 16), acc[2]);
    acc[3] = __fmaf_rn(v, __uint_as_float(a.y & 0xffff0000u), acc[3]);
    acc[4] = __fmaf_rn(v, __uint_as_float(a.z << 16), acc[4]);
    acc[5] = __fmaf_rn(v, __uint_as_float(a.z & 0xffff0000u), acc[5]);
    acc[6] = __fmaf_rn(v, __uint_as_float(a.w << 16), acc[6]);
    acc[7] = __fmaf_rn(v, __uint_as_float(a.w & 0xffff0000u), acc[7]);
  }
};
// bf16 rows at a stride that is NOT a multiple of 8 elements (the data-parallel parameter wire:
// W1 row-major at stride n = 300, read directly by the forward SpMM).  Such rows have no zero pads:
// a half group (nvalid == 4: the row's last 4 columns) loads the full 16 B, whose upper 8 B are the
// next row's first columns (for the buffer's last row: the 8-element slack dssm_plan_dp_wire_size
// includes, and that dssm_spmm_csr_fwd documents for tight bf16 rows).  The lane's upper 4 sums are
// garbage and spmm_rows zeroes them once per row after the gather.  Measured alternatives, both
// slower because they add work to every gathered row: loading the 16 B that END at the row's end
// (the compiler narrowed every gather to two 8-B loads: SpMM 19.8 -> 27.2 us) and masking the
// upper half per load (25.9 us; the plain load: 20.2 us).  Loads are 8-B aligned.
struct u16t {
  u16 bits;
};
template <> struct RawRow8<u16t> {
  RawRow8<u16> r;
  __device__ __forceinline__ void load(const u16t* p, int) { r.a = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void fma(float v, float (&acc)[8]) const { r.fma(v, acc); }
};
template <> struct RawRow8<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p, int nvalid) {
    a = *reinterpret_cast<const float4*>(p);
    b = nvalid > 4 ? *reinterpret_cast<const float4*>(p + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __device__ __forceinline__ void fma(float v, float (&acc)[8]) const {
    acc[0] = __fmaf_rn(v, a.x, acc[0]); acc[1] = __fmaf_rn(v, a.y, acc[1]);
    acc[2] = __fmaf_rn(v, a.z, acc[2]); acc[3] = __fmaf_rn(v, a.w, acc[3]);
    acc[4] = __fmaf_rn(v, b.x, acc[4]); acc[5] = __fmaf_rn(v, b.y, acc[5]);
    acc[6] = __fmaf_rn(v, b.z, acc[6]); acc[7] = __fmaf_rn(v, b.w, acc[7]);
  }
};

// One batch of cnt <= 64 entries whose (index, value) pairs lane j already holds in my_i, my_v.
// All 64 lanes must be active (the index broadcast reads every lane's register; v_readlane
// ignores EXEC); lanes with nvalid <= 0 only skip their loads.
// REM: rows in flight in the remainder (< U) loop: 2 for the short CSC columns of dW1 (most light
// columns have a handful of entries: their chain is the remainder), 1 for the SpMM's ~32-entry rows
// (measured: the wider remainder costs it occupancy).
// U: rows in flight per lane in the main loop.
template <typename T, int REM = 1, int U = sizeof(T) == 2 ? 8 : 4>
__device__ __forceinline__ void gather_batch(int my_i, float my_v, int cnt, const T* __restrict__ M,
                                             int ldm, int c, int nvalid, float (&acc)[8]) {
  {
    int j = 0;
    for (; j + U <= cnt; j += U) {
      RawRow8<T> x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = bcast_i(my_i, j + u);
        if (nvalid > 0) x[u].load(M + (size_t)r * ldm + c, nvalid);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float v = bcast_f(my_v, j + u);
        if (nvalid > 0) x[u].fma(v, acc);
      }
    }
    for (; REM == 2 && j + 2 <= cnt; j += 2) {  // remainder: two rows in flight, FMAs in entry order
      RawRow8<T> x0, x1;
      const int r0 = bcast_i(my_i, j), r1 = bcast_i(my_i, j + 1);
      if (nvalid > 0) {
        x0.load(M + (size_t)r0 * ldm + c, nvalid);
        x1.load(M + (size_t)r1 * ldm + c, nvalid);
        x0.fma(bcast_f(my_v, j), acc);
        x1.fma(bcast_f(my_v, j + 1), acc);
      }
    }
    for (; j < cnt; ++j) {
      const int r = bcast_i(my_i, j);
      const float v = bcast_f(my_v, j);
      if (nvalid > 0) {
        RawRow8<T> x;
        x.load(M + (size_t)r * ldm + c, nvalid);
        x.fma(v, acc);
      }
    }
  }
}

// Accumulate sum_j val_j * M[idx_j, c..c+8) for entries [s, e) into acc (gather_batch per 64).
template <typename T, int REM = 1, int U = sizeof(T) == 2 ? 8 : 4>
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
    gather_batch<T, REM, U>(my_i, my_v, cnt, M, ldm, c, nvalid, acc);
  }
}

}  // namespace dssm
