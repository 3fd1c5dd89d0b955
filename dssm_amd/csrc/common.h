// Shared device helpers for the gfx950 DSSM kernels (wave64, bf16 storage = uint16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned short u16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define DSSM_WAVE 64

__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float(((unsigned)h) << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Butterfly all-sum stages on the VALU (no LDS-pipe ds_bpermute): stage S of wave_allsum_step
// adds the partner value of the lane's 2^S-block neighbour.  Stages run in order 0..5; stages 2
// and 3 use the row half-mirror / mirror permutations, which pair each lane with a lane of the
// other half-block -- the same partner value as lane ^ 4 / lane ^ 8, because after the earlier
// stages every lane of a half-block holds the same partial sum -- and stages 4 / 5 the gfx950
// row / half-wave swaps.  Every lane ends with the same bits.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// v + v[lane ^ 16] / v + v[lane ^ 32] in every lane (the same bits as a __shfl_xor butterfly stage:
// each lane adds the even-row / low-half value and the odd-row / high-half value), on the VALU
__device__ __forceinline__ float sum_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                  false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
__device__ __forceinline__ float sum_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                  false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
__device__ __forceinline__ double sum_xor16(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double d0 = __builtin_bit_cast(double, (unsigned long long)(unsigned)a[0] | ((unsigned long long)(unsigned)b[0] << 32));
  const double d1 = __builtin_bit_cast(double, (unsigned long long)(unsigned)a[1] | ((unsigned long long)(unsigned)b[1] << 32));
  return d0 + d1;
}
__device__ __forceinline__ double sum_xor32(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const double d0 = __builtin_bit_cast(double, (unsigned long long)(unsigned)a[0] | ((unsigned long long)(unsigned)b[0] << 32));
  const double d1 = __builtin_bit_cast(double, (unsigned long long)(unsigned)a[1] | ((unsigned long long)(unsigned)b[1] << 32));
  return d0 + d1;
}

template <int S>
__device__ __forceinline__ float wave_allsum_step(float v) {
  if constexpr (S == 0) return v + dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
  if constexpr (S == 1) return v + dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
  if constexpr (S == 2) return v + dpp_mov<0x141>(v);  // row_half_mirror
  if constexpr (S == 3) return v + dpp_mov<0x140>(v);  // row_mirror
  if constexpr (S == 4) return sum_xor16(v);  // rows 0 <-> 1, 2 <-> 3
  if constexpr (S == 5) return sum_xor32(v);  // half-waves
}

// Broadcast lane j's value (j wave-uniform) -> scalar register.
__device__ __forceinline__ int bcast_i(int v, int j) { return __builtin_amdgcn_readlane(v, j); }
__device__ __forceinline__ float bcast_f(float v, int j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

// ---- cache policy of the optimizer's once-per-step state streams (p, m, v) ------------------
// Those 219 MB per step (C2) pass through the XCD L2s between the gathers of dZ1 rows (3.7 MB,
// re-read by every XCD) that share the launch.  DSSM_STREAM_POLICY (build-time A/B):
//   bit 0: nt loads;  bit 1: nt stores;  bit 2: sc1 (write-through) stores, which drop the line
//   from the XCD's L2 (MI355X_MICROARCH.md, store flavours).
#ifndef DSSM_STREAM_POLICY
#define DSSM_STREAM_POLICY 0
#endif
typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_stream4(const float* p) {
#if DSSM_STREAM_POLICY & 1
  const f32x4v v = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(p));
  return make_float4(v[0], v[1], v[2], v[3]);
#else
  return *reinterpret_cast<const float4*>(p);
#endif
}
__device__ __forceinline__ void st_stream4(float* p, float4 x) {
#if DSSM_STREAM_POLICY & 4
  const f32x4v v = {x.x, x.y, x.z, x.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
#elif DSSM_STREAM_POLICY & 2
  const f32x4v v = {x.x, x.y, x.z, x.w};
  __builtin_nontemporal_store(v, reinterpret_cast<f32x4v*>(p));
#else
  *reinterpret_cast<float4*>(p) = x;
#endif
}
// the lane's 8-column group of a stream (nvalid in {4, 8})
__device__ __forceinline__ void ld_stream8(const float* p, int nvalid, float (&x)[8]) {
  const float4 a = ld_stream4(p);
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  if (nvalid > 4) {
    const float4 b = ld_stream4(p + 4);
    x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  } else {
    x[4] = x[5] = x[6] = x[7] = 0.f;
  }
}

// ---- 8-column vector loads/stores (lane owns 8 consecutive columns) ------------------------
// nvalid in {4, 8}: widths are multiples of 4, so a lane's group is either full or half.
__device__ __forceinline__ void load8(const float* p, int nvalid, float (&x)[8]) {
  float4 a = *reinterpret_cast<const float4*>(p);
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  if (nvalid > 4) {
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  } else {
    x[4] = x[5] = x[6] = x[7] = 0.f;
  }
}
// bf16 rows are padded to ldp(n) (multiple of 8) with zero pads: always a full 16-B load.
__device__ __forceinline__ void load8(const u16* p, int /*nvalid*/, float (&x)[8]) {
  uint4 a = *reinterpret_cast<const uint4*>(p);
  x[0] = __uint_as_float(a.x << 16); x[1] = __uint_as_float(a.x & 0xffff0000u);
  x[2] = __uint_as_float(a.y << 16); x[3] = __uint_as_float(a.y & 0xffff0000u);
  x[4] = __uint_as_float(a.z << 16); x[5] = __uint_as_float(a.z & 0xffff0000u);
  x[6] = __uint_as_float(a.w << 16); x[7] = __uint_as_float(a.w & 0xffff0000u);
}

__device__ __forceinline__ void store8(float* p, const float (&x)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(x[4], x[5], x[6], x[7]);
}
// One v_cvt_pk_bf16_f32 (RNE, as f2bf): the two-scalar form compiles to a pair of packed converts
// and four shift / mask / or instructions to re-pair their halves.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack2bf(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2{a, b}), bf16x2));
}
__device__ __forceinline__ void store8(u16* p, const float (&x)[8]) {
  uint4 a;
  a.x = pack2bf(x[0], x[1]); a.y = pack2bf(x[2], x[3]);
  a.z = pack2bf(x[4], x[5]); a.w = pack2bf(x[6], x[7]);
  *reinterpret_cast<uint4*>(p) = a;
}

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<u16>(u16 v) { return bf2f(v); }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ u16 from_f<u16>(float v) { return f2bf(v); }

// BatchNorm affine exactly as tf.nn.batch_normalization: x*inv + (beta - mean*inv).
// The forward and the backward's ReLU mask both call this, so the mask is bit-identical.
__device__ __forceinline__ float bn_affine(float z, float inv, float shift) {
  return __fmaf_rn(z, inv, shift);
}

// Publish this block's partials and return true in every thread of the LAST block to arrive
// for ticket `cnt` (expected arrivals: `arrivals`).  Producer: every wave drains its stores,
// workgroup barrier, one agent-scope release, relaxed agent ticket.  Last block: one agent
// acquire before any thread reads other blocks' partials.  The last block re-arms the ticket.
__device__ __forceinline__ bool last_block_arrival(unsigned* cnt, unsigned arrivals,
                                                   int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t == arrivals - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag != 0;
}

// The same arrival WITHOUT agent-scope fences, for hand-offs whose every store was write-through
// (sc1: an agent-scope relaxed atomic store) and every read of which is an sc1 load (agent-scope
// relaxed atomic load): each wave drains its stores, then one lane's agent-scope ticket add; the
// last adder's workgroup reads after the barrier (MI355X_MICROARCH.md, inter-workgroup visibility,
// the measured fence-free form).  The release fence of last_block_arrival writes back the whole
// XCD L2's dirty lines, which is what made the deterministic heavy-column slab cost ~20 us.
__device__ __forceinline__ bool last_block_arrival_wt(unsigned* cnt, unsigned arrivals, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t == arrivals - 1);
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag != 0;
}

// Block b -> tile: tiles [x n/8, (x+1) n/8) go to the blocks b = x (mod 8), which the observed
// round-robin dispatch places on one XCD (speed only, never correctness: any placement computes
// the same tiles).  Consecutive tiles share their A rows (a row block's column tiles) or their
// batch-row chunk (dW), so those re-reads hit that XCD's L2 instead of the Infinity Cache.
// (measured in round 3 with the grouping off: +4.5 us/step, so the row block's A panel is shared
// through the XCD's L2)
#ifndef DSSM_XCD_TILE
#define DSSM_XCD_TILE 1
#endif
__device__ __forceinline__ int xcd_tile(int b, int n) {
  return (!DSSM_XCD_TILE || (n % 8)) ? b : (b % 8) * (n / 8) + b / 8;
}

__host__ __device__ inline int ldp8(int n) { return (n + 7) & ~7; }
__host__ __device__ inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// Loss / accuracy of the step from the cosine kernel's per-workgroup partials: wave 0 of the
// calling workgroup, fixed order (lane-strided partial sums, then a shuffle tree).
// Inverted-dropout mask of element i (row-major index r * cols + c): kept when the hash < thr,
// thr = keep * 2^32 (oracle/rnn_oracle.py dropout_mask); shared by k_dropout and the fused cosine.
__device__ __forceinline__ unsigned dropout_hash(unsigned i, unsigned seed, unsigned step) {
  unsigned x = i * 0x9E3779B1u + seed * 0x85EBCA77u + step * 0xC2B2AE3Du;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ void loss_reduce(const float* __restrict__ part, int nblk, int bs,
                                            float* __restrict__ loss_out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (wv == 0) {
    float a = 0.f, b = 0.f;
    int i = lane;
    // eight partials' loads in flight per lane before the (in-order) adds: the launch is one
    // wave, so its time is the load latency chain
    for (; i + 7 * 64 < nblk; i += 8 * 64) {
      float pa[8], pb[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        pa[k] = part[2 * (i + 64 * k)];
        pb[k] = part[2 * (i + 64 * k) + 1];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a += pa[k];
        b += pb[k];
      }
    }
    for (; i < nblk; i += 64) {
      a += part[2 * i];
      b += part[2 * i + 1];
    }
    // fixed-order tree over the 64 lane partials
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_down(a, o);
      b += __shfl_down(b, o);
    }
    if (lane == 0) {
      loss_out[0] = a / (float)bs;
      loss_out[1] = b / (float)bs;
    }
  }
}

// ---- zero fill as a kernel node -------------------------------------------------------------------
// Every device-side clear that can enter a captured graph is a kernel (not a hipMemsetAsync node), so
// a captured stream is a chain of kernel nodes whose ordering is the stream's.  A
// template so each translation unit may instantiate it (COMDAT).  4-B words; a byte tail if any.
template <int kUnused = 0>
__global__ __launch_bounds__(256) void k_zero_bytes(unsigned char* __restrict__ p, size_t bytes) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool aligned = ((uintptr_t)p % 4) == 0;
  const size_t words = aligned ? bytes / 4 : 0;
  for (size_t i = t; i < words; i += stride) reinterpret_cast<unsigned*>(p)[i] = 0u;
  for (size_t i = words * 4 + t; i < bytes; i += stride) p[i] = 0;
}
inline hipError_t zero_bytes_async(void* p, size_t bytes, hipStream_t s) {
  if (!bytes) return hipSuccess;
  const size_t items = (bytes + 3) / 4;
  const unsigned grid = (unsigned)(items / 256 + 1 < 2048 ? items / 256 + 1 : 2048);
  hipLaunchKernelGGL(k_zero_bytes<0>, dim3(grid), dim3(256), 0, s, static_cast<unsigned char*>(p), bytes);
  return hipGetLastError();
}
