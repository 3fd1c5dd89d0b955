// The dense part of the DSSM step as two persistent kernels (bf16 perf mode), on gfx950.
//
// After the SpMM has written Z1, everything up to dZ1 runs in k_dense_fwd + k_dense_bwd:
//   BN1..BN_L (new_dssm.py:62-88), FC2..FC_L (:146-148), Merge + Cosine + Loss (:160-213) and
//   their backward, including dW_l (split-K slabs) and dgamma/dbeta.
// One grid of one 512-thread workgroup per CU walks the phases, separated by grid barriers:
//   fwd : BN1 sums | GEMM_2 (+BN_2 sums) | ... | GEMM_L (+BN_L sums) |
//         cosine + loss + dy_L + BN_L backward sums; last block: loss, EMA, coefficients
//   bwd : dA_{L-1} (dZ_L staged) + BN_{L-1} bwd sums | dW_L + dA_{L-2} + ... |
//         dW_2 + dZ1; last block: dgamma, dbeta
// (L=3: 3 + 2 grid barriers per step; a barrier costs about what a kernel boundary does, ~4 us).
// Batch-norm statistics are accumulated as fp64 column sums (sum z, sum z^2; sum dy,
// sum dy*xhat) with hardware fp64 atomics by the producing phase, and every consumer derives the
// coefficients it needs in-block, so no separate finalize phase (and barrier) is needed.  fp64
// sums of fp32 terms: the order of the atomics changes the result by ~1e-16 relative, below
// the fp32 rounding of every derived coefficient.
// GEMM items are 32 batch rows x ALL output columns: the whole-K A panel (<= 512) is staged once
// with the BN+ReLU (forward) or the BN backward of dZ (backward) applied while staging, then the
// 64-column weight panels stream through a double-buffered LDS ring.
//
// Grid barrier: one workgroup per CU, all co-resident (the plan sizes the grid by the CU count
// and the occupancy API).  Arrival: drain stores, workgroup barrier, agent-scope release,
// relaxed agent atomic count; the last arrival bumps a generation word (release); waiters poll
// it with s_sleep, then agent-scope acquire (cdna_hip_programming.md §6 G16).  Every spin is
// bounded: on timeout the block sets a sticky error word, every later barrier returns at once,
// the kernel drains, and the host reports it (dssm_plan_check).
#define DSSM_GAS __attribute__((address_space(1)))
#include "common.h"
#include "dense.h"
#include "launch.h"

#include <algorithm>

namespace dssm {
namespace {

constexpr int TM = 64;       // output column tile (one MFMA 16x16 column block per wave)
constexpr int RT = 32;       // batch rows per GEMM item
constexpr int NTH = 512;     // threads per workgroup (8 waves)
constexpr int NW = NTH / 64;
constexpr int MAXG_A = 4;    // A staging groups (8 elements) per thread: RT * 512 / 8 / NTH
constexpr int MAXG_B = 8;    // B staging groups per thread: TM * 512 / 8 / NTH
constexpr int DW_K = 256;    // batch rows per dW split
constexpr int TLD = 72;      // dW chunk LDS row stride (64 + 8)
constexpr unsigned kSpinLimit = 1u << 21;  // >= ~0.3 s of polling before declaring a failure

// ---- timing stamps and grid barrier --------------------------------------------------------
// DSSM_DENSE_TIMING=1: block 0 stamps the 100 MHz s_memrealtime clock at kernel start, on
// arrival at and exit from every grid barrier, and at the end.
__device__ __forceinline__ void stamp(unsigned long long DSSM_GAS* t, int& i) {
  if (t && blockIdx.x == 0 && threadIdx.x == 0 && i < 64) t[i] = __builtin_amdgcn_s_memrealtime();
  ++i;
}

__device__ __forceinline__ bool grid_sync(unsigned DSSM_GAS* bar, unsigned& gen, int* s_ok,
                                          unsigned long long DSSM_GAS* tm, int& ti) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp(tm, ti);
  if (threadIdx.x == 0) {
    unsigned DSSM_GAS* cnt = bar;
    unsigned DSSM_GAS* g = bar + 64;
    unsigned DSSM_GAS* err = bar + 128;
    int ok = 1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned target = gen + 1;
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(g, target, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != target) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        if (++spins > kSpinLimit) {
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    *s_ok = ok;
  }
  __syncthreads();
  stamp(tm, ti);
  gen += 1;
  return *s_ok != 0;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops (lgkmcnt) but not for
// its outstanding global loads / stores / atomics, so prefetches and write-backs stay in flight
// across it (__syncthreads would drain vmcnt as well).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ unsigned read_gen(unsigned DSSM_GAS* bar) {
  return __hip_atomic_load(bar + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 16/8-byte global accesses through native vector types (HIP's uint4/float4 classes cannot be
// address-space qualified)
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gload_u4(const void DSSM_GAS* p) {
  const v4u x = *(const v4u DSSM_GAS*)p;
  return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ float4 gload_f4(const void DSSM_GAS* p) {
  const v4f x = *(const v4f DSSM_GAS*)p;
  return make_float4(x.x, x.y, x.z, x.w);
}
// Branch-free guarded loads: always load (from `p` when ok, else from the always-valid `safe`)
// and select.  Loads inside divergent branches make the waitcnt pass serialize them
// (s_waitcnt vmcnt(0) at every join), so guarded loads never branch.
__device__ __forceinline__ uint4 ld_u4(bool ok, const void DSSM_GAS* p, const void DSSM_GAS* safe) {
  const uint4 v = gload_u4(ok ? p : safe);
  return ok ? v : make_uint4(0u, 0u, 0u, 0u);
}
__device__ __forceinline__ float4 ld_f4(bool ok, const void DSSM_GAS* p, const void DSSM_GAS* safe) {
  const float4 v = gload_f4(ok ? p : safe);
  return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}
template <typename T>
__device__ __forceinline__ T ld1(bool ok, const T DSSM_GAS* p, const T DSSM_GAS* safe) {
  const T v = *(ok ? p : safe);
  return ok ? v : T(0);
}
__device__ __forceinline__ void gstore_u4(void DSSM_GAS* p, uint4 v) {
  *(v4u DSSM_GAS*)p = v4u{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void gstore_u2(void DSSM_GAS* p, uint2 v) {
  *(v2u DSSM_GAS*)p = v2u{v.x, v.y};
}
__device__ __forceinline__ void gstore_f4(void DSSM_GAS* p, float4 v) {
  *(v4f DSSM_GAS*)p = v4f{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ int tower_of(int r, int bs) { return r < bs ? 0 : 1; }
__device__ __forceinline__ int round32(int k) { return (k + 31) & ~31; }
__device__ __forceinline__ void atomic_addd(double DSSM_GAS* p, double v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- batch-norm coefficients ---------------------------------------------------------------
// Forward coefficients of column c, tower t: batch moments from the step's fp64 sums (train,
// biased variance) or the EMA shadows (eval).  Columns >= n (row padding) get all zeros.
__device__ __forceinline__ void bn_coef(const DenseArgs& a, const DenseLayer& C, int t, int c,
                                        int train, float& mu, float& var, float& rstd, float& inv,
                                        float& shift) {
  if (c >= C.n) {
    mu = var = rstd = inv = shift = 0.f;
    return;
  }
  if (train) {
    const double N = t == 0 ? a.BS : a.R - a.BS;
    const double m = C.fsum[(t * 2) * C.ld + c] / N;
    const double v = C.fsum[(t * 2 + 1) * C.ld + c] / N - m * m;
    mu = (float)m;
    var = (float)(v > 0.0 ? v : 0.0);
  } else {
    mu = C.ema_mean[t][c];
    var = C.ema_var[t][c];
  }
  rstd = 1.0f / sqrtf(var + a.eps);
  inv = rstd * C.gamma[t][c];
  shift = C.beta[t][c] - mu * inv;
}

// Backward coefficients of column c, tower t: dz = inv*dy + c1*z + c0 with
// dz = inv*(dy - mean(dy) - xhat*mean(dy*xhat)), xhat = (z - mu)*rstd.
__device__ __forceinline__ void bn_dcoef(const DenseArgs& a, const DenseLayer& C, int t, int c,
                                         float& inv, float& c1, float& c0) {
  if (c >= C.n) {
    inv = c1 = c0 = 0.f;
    return;
  }
  const double N = t == 0 ? a.BS : a.R - a.BS;
  const float m1 = (float)(C.bsum[(t * 2) * C.ld + c] / N);
  const float m2 = (float)(C.bsum[(t * 2 + 1) * C.ld + c] / N);
  const size_t plane = (size_t)2 * C.ld, o = (size_t)t * C.ld + c;
  const float mu = C.coef[o], rstd = C.coef[plane + o];
  inv = C.coef[2 * plane + o];
  c1 = -inv * rstd * m2;
  c0 = -inv * m1 - c1 * mu;
}

// ---- GEMM building blocks --------------------------------------------------------------------
// One 16x16 fp32 block of A[r0..r0+16) . B[c0..c0+16)^T over Kp (k-contiguous bf16 panels).
__device__ __forceinline__ f32x4 mfma16(const u16* sA, int r0, const u16* sB, int c0, int ldk,
                                        int Kp, int lane) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const u16* pa = sA + (r0 + (lane & 15)) * ldk + 8 * (lane >> 4);
  const u16* pb = sB + (c0 + (lane & 15)) * ldk + 8 * (lane >> 4);
  for (int ks = 0; ks < Kp; ks += 32) {
    const bf16x8 af = *reinterpret_cast<const bf16x8*>(pa + ks);
    const bf16x8 bf = *reinterpret_cast<const bf16x8*>(pb + ks);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc, 0, 0, 0);
  }
  return acc;
}

// B panel rows [b0, b0+64) x K columns [0, Kp) of a k-contiguous bf16 matrix [nrows x ldb]
// (zero beyond nrows / klim): global -> registers, registers -> LDS.
struct BRegs {
  uint4 v[MAXG_B];
  unsigned ok;  // bit g: group g is in range (else it is stored as zeros)
};
// All loads are issued unconditionally (out-of-range groups read the always-valid base) and
// zeroed only when stored, so no select sits between two loads (a select right after a load
// makes the waitcnt pass drain vmcnt there and serializes the whole panel).
__device__ __forceinline__ void load_b(BRegs& r, const u16 DSSM_GAS* __restrict__ Bm, int ldb, int nrows,
                                       int klim, int b0, int Kp) {
  const int gpr = Kp >> 3, tot = TM * gpr;
  r.ok = 0;
#pragma unroll
  for (int g = 0; g < MAXG_B; ++g) {
    const int e = threadIdx.x + NTH * g;
    const int ee = e < tot ? e : 0;
    const int row = ee / gpr, kg = (ee - row * gpr) * 8;
    const int gr = b0 + row;
    const bool ok = e < tot && gr < nrows && kg < klim;
    r.ok |= (ok ? 1u : 0u) << g;
    r.v[g] = gload_u4(ok ? (const void DSSM_GAS*)(Bm + (size_t)gr * ldb + kg) : (const void DSSM_GAS*)Bm);
  }
}
__device__ __forceinline__ void store_b(const BRegs& r, u16* sB, int ldk, int Kp) {
  const int gpr = Kp >> 3, tot = TM * gpr;
#pragma unroll
  for (int g = 0; g < MAXG_B; ++g) {
    const int e = threadIdx.x + NTH * g;
    if (e < tot) {
      const int row = e / gpr, kg = (e - row * gpr) * 8;
      *reinterpret_cast<uint4*>(&sB[row * ldk + kg]) =
          ((r.ok >> g) & 1u) ? r.v[g] : make_uint4(0u, 0u, 0u, 0u);
    }
  }
}


// Column sums of the 32-row tile held as acc rows (lane>>4)*4 + r of the wm = 0 / 1 waves:
// reduce over r and the 4 lane groups, combine the two wm halves through LDS, and add the
// result to the fp64 accumulators (s -> dst0[n], q -> dst1[n]) when n is valid.
__device__ __forceinline__ void tile_colsum_add(double s, double q, int wm, int wn, int lane,
                                                double* dred, double DSSM_GAS* dst0,
                                                double DSSM_GAS* dst1, bool ok) {
  s += __shfl_xor(s, 16);
  s += __shfl_xor(s, 32);
  q += __shfl_xor(q, 16);
  q += __shfl_xor(q, 32);
  if (wm == 1 && lane < 16) {
    dred[(wn * 16 + lane) * 2] = s;
    dred[(wn * 16 + lane) * 2 + 1] = q;
  }
  lds_barrier();
  if (wm == 0 && lane < 16 && ok) {
    atomic_addd(dst0, s + dred[(wn * 16 + lane) * 2]);
    atomic_addd(dst1, q + dred[(wn * 16 + lane) * 2 + 1]);
  }
}

// ---- weight-stationary GEMM phases -----------------------------------------------------------
// A block owns a column part of the layer's weights (<= ~105 KB bf16, whole K) in LDS for the
// whole phase and streams 32-row A panels through it: every weight byte is read once per block,
// every A row once per part, and a row tile's whole part is one MFMA pass (no per-column-tile
// round trips).  Parts: nparts = ceil(ld_out / pc_max), pc = columns per part (multiple of 16);
// blocks b = part (mod nparts) share a part and split the row tiles.
constexpr int kDenseSmem = 144 * 1024;  // dynamic LDS per workgroup

struct WsGeom {
  int K, Kp, ldk, nparts, pc, part, c0, cols, nsub, bi, nb;
};

__device__ __forceinline__ WsGeom ws_geom(int K, int ld_out, int coef_floats) {
  WsGeom g;
  g.K = K;
  g.Kp = round32(K);
  g.ldk = g.Kp + 8;
  const int fixed = RT * g.ldk * 2 + coef_floats * g.Kp * 4 + 1024;
  const int percol = g.ldk * 2 + 8 * 4 + 4 * 8 + 4;  // W row, coefficients, fp64 sums, bias
  int pcmax = ((kDenseSmem - fixed) / percol) & ~15;
  if (pcmax < 16) pcmax = 16;
  g.nparts = cdiv(ld_out, pcmax);
  g.pc = (cdiv(cdiv(ld_out, g.nparts), 16)) * 16;
  g.part = blockIdx.x % g.nparts;
  g.c0 = g.part * g.pc;
  g.cols = min(g.pc, ld_out - g.c0);
  g.nsub = cdiv(g.cols, 16);
  g.bi = blockIdx.x / g.nparts;
  g.nb = ((int)gridDim.x - g.part + g.nparts - 1) / g.nparts;
  return g;
}

// stage rows [c0, c0 + pc) x K of a k-contiguous bf16 matrix [nrows x ldb] into sW [pc][ldk]
__device__ __forceinline__ void ws_load_w(u16* sW, const WsGeom& g, const u16 DSSM_GAS* Bm, int ldb,
                                          int nrows) {
  const int gpr = g.Kp >> 3, tot = g.pc * gpr;
  for (int base = 0; base < tot; base += NTH * 8) {
    uint4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = base + threadIdx.x + NTH * i;
      const int ee = e < tot ? e : 0;
      const int row = ee / gpr, kg = (ee - row * gpr) * 8;
      const int gr = g.c0 + row;
      const bool ok = e < tot && gr < nrows && kg < g.K;
      v[i] = gload_u4(ok ? (const void DSSM_GAS*)(Bm + (size_t)gr * ldb + kg) : (const void DSSM_GAS*)Bm);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // zero out-of-range groups only now (no select between loads)
      const int e = base + threadIdx.x + NTH * i;
      if (e < tot) {
        const int row = e / gpr, kg = (e - row * gpr) * 8;
        const bool ok = g.c0 + row < nrows && kg < g.K;
        *reinterpret_cast<uint4*>(&sW[row * g.ldk + kg]) = ok ? v[i] : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  }
}

// A-panel registers: 32 rows x Kp fp32 (x2 in the backward: Z and dy), 8-element groups
struct APanel {
  float4 z[MAXG_A][2], d[MAXG_A][2];
};
template <bool BWD>
__device__ __forceinline__ void ws_load_a(APanel& r, const float DSSM_GAS* Z, const float DSSM_GAS* D,
                                          int bm, const WsGeom& g) {
  const int gpr = g.Kp >> 3, totA = RT * gpr;
#pragma unroll
  for (int i = 0; i < MAXG_A; ++i) {
    const int e = threadIdx.x + NTH * i;
    const int ee = e < totA ? e : 0;
    const int row = ee / gpr, kg = (ee - row * gpr) * 8;
    const bool ok = e < totA && kg < g.K;  // zeroed when staged
    const size_t off = ok ? (size_t)(bm + row) * g.K + kg : 0;
    r.z[i][0] = gload_f4(Z + off);
    r.z[i][1] = gload_f4(Z + off + 4);
    if (BWD) {
      r.d[i][0] = gload_f4(D + off);
      r.d[i][1] = gload_f4(D + off + 4);
    }
  }
}

// Column sums of the pass: every wave's 16-row partials (lanes 0..15 per 16-column subtile) go
// to ps[wm][col] / pq[wm][col]; after a barrier the block adds the two halves to the fp64
// accumulators (column c0 + c of tower `tower`).
__device__ __forceinline__ void ws_sums_flush(double* ps, double* pq, const WsGeom& g, int ncols_valid,
                                              double DSSM_GAS* dst, int ld, int tower) {
  for (int c = threadIdx.x; c < g.cols; c += NTH) {
    const int n = g.c0 + c;
    if (n < ncols_valid) {
      atomic_addd(dst + (size_t)(tower * 2) * ld + n, ps[c] + ps[g.pc + c]);
      atomic_addd(dst + (size_t)(tower * 2 + 1) * ld + n, pq[c] + pq[g.pc + c]);
    }
  }
}

__device__ __forceinline__ void fwd_phase(const DenseArgs& a, int l, int train, u16* smem, double*) {
  const DenseLayer& P = a.ly[l - 1];
  const DenseLayer& C = a.ly[l];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 2, wn = w & 3;
  const WsGeom g = ws_geom(P.ld, C.ld, 4);
  const int nrt = a.R / RT;
  if (g.bi >= nrt) return;
  unsigned long long DSSM_GAS* ftm = (a.timing && l == 1 && blockIdx.x == 0) ? a.timing + 128 : nullptr;
  int fti = 0;
  stamp(ftm, fti);
  u16* sW = smem;                                   // [pc][ldk]
  u16* sA = sW + g.pc * g.ldk;                      // [RT][ldk]
  float* sc = reinterpret_cast<float*>(sA + RT * g.ldk);  // [tower][inv | shift][Kp]
  float* sb = sc + 4 * g.Kp;                        // [pc] bias
  double* ps = reinterpret_cast<double*>(sb + g.pc + (g.pc & 1));  // [2][pc] sums, [2][pc] squares
  double* pq = ps + 2 * g.pc;
  for (int i = t; i < 2 * g.Kp; i += NTH) {
    const int tw = i / g.Kp, k = i - tw * g.Kp;
    float mu, var, rs, inv, sh;
    bn_coef(a, P, tw, k, train, mu, var, rs, inv, sh);
    sc[(tw * 2) * g.Kp + k] = inv;
    sc[(tw * 2 + 1) * g.Kp + k] = sh;
  }
  for (int c = t; c < g.pc; c += NTH) sb[c] = *(g.c0 + c < C.n ? C.bias + g.c0 + c : C.bias) * (g.c0 + c < C.n ? 1.f : 0.f);
  stamp(ftm, fti);
  APanel r;
  ws_load_a<false>(r, P.Z, nullptr, g.bi * RT, g);
  stamp(ftm, fti);
  ws_load_w(sW, g, C.WT, g.K, C.n);
  stamp(ftm, fti);
  const int gpr = g.Kp >> 3, totA = RT * gpr;
  lds_barrier();  // sc, sb, sW
  stamp(ftm, fti);
  for (int rt = g.bi; rt < nrt; rt += g.nb) {
    const int bm = rt * RT;
    const int tower = tower_of(bm, a.BS);
    const float* si = sc + (tower * 2) * g.Kp;
    const float* ss = si + g.Kp;
#pragma unroll
    for (int i = 0; i < MAXG_A; ++i) {
      const int e = t + NTH * i;
      if (e < totA) {
        const int row = e / gpr, kg = (e - row * gpr) * 8;
        const bool okk = kg < g.K;
        const float zz[8] = {r.z[i][0].x, r.z[i][0].y, r.z[i][0].z, r.z[i][0].w,
                             r.z[i][1].x, r.z[i][1].y, r.z[i][1].z, r.z[i][1].w};
        float y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) y[k] = okk ? fmaxf(bn_affine(zz[k], si[kg + k], ss[kg + k]), 0.f) : 0.f;
        uint4 v;
        v.x = pack2bf(y[0], y[1]); v.y = pack2bf(y[2], y[3]);
        v.z = pack2bf(y[4], y[5]); v.w = pack2bf(y[6], y[7]);
        *reinterpret_cast<uint4*>(&sA[row * g.ldk + kg]) = v;
        if (g.part == 0 && P.A && okk) gstore_u4(P.A + (size_t)(bm + row) * g.K + kg, v);
      }
    }
    lds_barrier();
    stamp(ftm, fti);
    if (rt + g.nb < nrt) ws_load_a<false>(r, P.Z, nullptr, (rt + g.nb) * RT, g);  // next tile in flight
    stamp(ftm, fti);
    // MFMA: wave (wm, wn) -> rows wm*16, subtiles j = wn, wn + 4, wn + 8
    const u16* pa = sA + (wm * 16 + (lane & 15)) * g.ldk + 8 * (lane >> 4);
    for (int j = wn; j < g.nsub; j += 4) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const u16* pb = sW + (j * 16 + (lane & 15)) * g.ldk + 8 * (lane >> 4);
      for (int ks = 0; ks < g.Kp; ks += 32)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(pa + ks),
                                                      *reinterpret_cast<const bf16x8*>(pb + ks), acc, 0, 0, 0);
      if (ftm && j == wn) { asm volatile("s_nop 0" :: "v"(acc[0]), "v"(acc[3])); stamp(ftm, fti); }
      const int cl = j * 16 + (lane & 15), n = g.c0 + cl;
      const float b = sb[cl];
      double s = 0.0, q = 0.0;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int m = bm + wm * 16 + (lane >> 4) * 4 + rr;
        const float x = n < C.n ? acc[rr] + b : 0.f;
        if (cl < g.cols) C.Z[(size_t)m * C.ld + n] = x;
        s += x;
        q += (double)x * x;
      }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      if (lane < 16) {
        ps[wm * g.pc + cl] = s;
        pq[wm * g.pc + cl] = q;
      }
      if (ftm && j == wn) { asm volatile("s_nop 0" :: "v"(s), "v"(q)); stamp(ftm, fti); }
    }
    stamp(ftm, fti);
    lds_barrier();
    stamp(ftm, fti);
    if (train) ws_sums_flush(ps, pq, g, C.n, C.fsum, C.ld, tower);
    stamp(ftm, fti);
  }
}

__device__ __forceinline__ void bwd_phase(const DenseArgs& a, int l, u16* smem, double*) {
  const DenseLayer& C = a.ly[l];      // dZ_l staged from (dy_l, Z_l)
  const DenseLayer& P = a.ly[l - 1];  // produces dy_{l-1}
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 2, wn = w & 3;
  const WsGeom g = ws_geom(C.ld, P.ld, 6);
  const int nrt = a.R / RT;
  if (g.bi >= nrt) return;
  u16* sW = smem;
  u16* sA = sW + g.pc * g.ldk;
  float* sc = reinterpret_cast<float*>(sA + RT * g.ldk);  // [tower][inv | c1 | c0][Kp]
  float* se = sc + 6 * g.Kp;                          // [tower][mu | rstd | inv | shift][pc]
  double* ps = reinterpret_cast<double*>(se + 8 * g.pc);
  double* pq = ps + 2 * g.pc;
  for (int i = t; i < 2 * g.Kp; i += NTH) {
    const int tw = i / g.Kp, k = i - tw * g.Kp;
    float inv, c1, c0;
    bn_dcoef(a, C, tw, k, inv, c1, c0);
    sc[(tw * 3) * g.Kp + k] = inv;
    sc[(tw * 3 + 1) * g.Kp + k] = c1;
    sc[(tw * 3 + 2) * g.Kp + k] = c0;
  }
  const size_t pplane = (size_t)2 * P.ld;
  for (int i = t; i < 2 * g.pc; i += NTH) {
    const int tw = i / g.pc, c = i - tw * g.pc, n = g.c0 + c;
    const bool ok = n < P.ld;
    const size_t o = ok ? (size_t)tw * P.ld + n : 0;
    se[(tw * 4 + 0) * g.pc + c] = ok ? P.coef[o] : 0.f;
    se[(tw * 4 + 1) * g.pc + c] = ok ? P.coef[pplane + o] : 0.f;
    se[(tw * 4 + 2) * g.pc + c] = ok ? P.coef[2 * pplane + o] : 0.f;
    se[(tw * 4 + 3) * g.pc + c] = ok ? P.coef[3 * pplane + o] : 0.f;
  }
  APanel r;
  ws_load_a<true>(r, C.Z, C.dy, g.bi * RT, g);
  ws_load_w(sW, g, C.W, g.K, P.n);
  const int gpr = g.Kp >> 3, totA = RT * gpr;
  lds_barrier();
  for (int rt = g.bi; rt < nrt; rt += g.nb) {
    const int bm = rt * RT;
    const int tower = tower_of(bm, a.BS);
    const float* k0 = sc + (tower * 3) * g.Kp;
    const float* k1 = k0 + g.Kp;
    const float* k2 = k1 + g.Kp;
#pragma unroll
    for (int i = 0; i < MAXG_A; ++i) {
      const int e = t + NTH * i;
      if (e < totA) {
        const int row = e / gpr, kg = (e - row * gpr) * 8;
        const bool okk = kg < g.K;
        const float zz[8] = {r.z[i][0].x, r.z[i][0].y, r.z[i][0].z, r.z[i][0].w,
                             r.z[i][1].x, r.z[i][1].y, r.z[i][1].z, r.z[i][1].w};
        const float dd[8] = {r.d[i][0].x, r.d[i][0].y, r.d[i][0].z, r.d[i][0].w,
                             r.d[i][1].x, r.d[i][1].y, r.d[i][1].z, r.d[i][1].w};
        float y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
          y[k] = okk ? __fmaf_rn(k0[kg + k], dd[k], __fmaf_rn(k1[kg + k], zz[k], k2[kg + k])) : 0.f;
        uint4 v;
        v.x = pack2bf(y[0], y[1]); v.y = pack2bf(y[2], y[3]);
        v.z = pack2bf(y[4], y[5]); v.w = pack2bf(y[6], y[7]);
        *reinterpret_cast<uint4*>(&sA[row * g.ldk + kg]) = v;
        if (g.part == 0 && okk) gstore_u4(C.dZ + (size_t)(bm + row) * g.K + kg, v);
      }
    }
    lds_barrier();
    if (rt + g.nb < nrt) ws_load_a<true>(r, C.Z, C.dy, (rt + g.nb) * RT, g);
    const u16* pa = sA + (wm * 16 + (lane & 15)) * g.ldk + 8 * (lane >> 4);
    const int m0 = bm + wm * 16 + (lane >> 4) * 4;
    for (int j = wn; j < g.nsub; j += 4) {
      const int cl = j * 16 + (lane & 15), n = g.c0 + cl;
      const bool okn = cl < g.cols;
      float z[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) z[rr] = *(okn ? P.Z + (size_t)(m0 + rr) * P.ld + n : P.Z);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const u16* pb = sW + (j * 16 + (lane & 15)) * g.ldk + 8 * (lane >> 4);
      for (int ks = 0; ks < g.Kp; ks += 32)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(pa + ks),
                                                      *reinterpret_cast<const bf16x8*>(pb + ks), acc, 0, 0, 0);
      const float mu = se[(tower * 4 + 0) * g.pc + cl], rs = se[(tower * 4 + 1) * g.pc + cl];
      const float inv = se[(tower * 4 + 2) * g.pc + cl], sh = se[(tower * 4 + 3) * g.pc + cl];
      double s = 0.0, q = 0.0;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float dy = (okn && bn_affine(z[rr], inv, sh) > 0.f) ? acc[rr] : 0.f;
        const float xh = (z[rr] - mu) * rs;
        if (okn) P.dy[(size_t)(m0 + rr) * P.ld + n] = dy;
        s += dy;
        q += (double)dy * xh;
      }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      if (lane < 16) {
        ps[wm * g.pc + cl] = s;
        pq[wm * g.pc + cl] = q;
      }
    }
    lds_barrier();
    ws_sums_flush(ps, pq, g, P.n, P.bsum, P.ld, tower);
  }
}

// ---- BN1 sums of Z1 (written by the SpMM): item = 64 rows x 64 columns --------------------
__device__ __forceinline__ void stats_item(const DenseArgs& a, int item, double* dsum) {
  const DenseLayer& C = a.ly[0];
  const int t = threadIdx.x, lane = t & 63, g = t >> 6;
  const int ncol = cdiv(C.ld, TM);
  const int rt = item / ncol, ct = item - rt * ncol;
  const int c = ct * TM + lane;
  const int tower = tower_of(rt * TM, a.BS);
  float x[TM / NW];
#pragma unroll
  for (int i = 0; i < TM / NW; ++i) {
    const int r = rt * TM + g + NW * i;
    x[i] = ld1(c < C.ld, C.Z + (size_t)r * C.ld + c, C.Z);
  }
  double s = 0.0, q = 0.0;
#pragma unroll
  for (int i = 0; i < TM / NW; ++i) {
    s += x[i];
    q += (double)x[i] * x[i];
  }
  dsum[(g * 64 + lane) * 2] = s;
  dsum[(g * 64 + lane) * 2 + 1] = q;
  lds_barrier();
  if (g == 0 && c < C.n) {
    double ts = 0.0, tq = 0.0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      ts += dsum[(k * 64 + lane) * 2];
      tq += dsum[(k * 64 + lane) * 2 + 1];
    }
    atomic_addd(C.fsum + (size_t)(tower * 2) * C.ld + c, ts);
    atomic_addd(C.fsum + (size_t)(tower * 2 + 1) * C.ld + c, tq);
  }
  lds_barrier();
}

// ---- dW_l split-K item: slab[s] = [A_{l-1}; 1]^T . dZ_l over DW_K batch rows -------------
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

__device__ __forceinline__ bf16x8 tr_frag72(const u16* tile, int row0, int col0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const u16* a0 = tile + (row0 + 8 * g + q) * TLD + col0 + 4 * p;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a0);
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0 + 4 * TLD));
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ void dw_item(const DenseArgs& a, int l, int item, u16* smem) {
  const DenseLayer& C = a.ly[l];
  const DenseLayer& P = a.ly[l - 1];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;
  const int M = P.n + 1, N = C.n;  // [W; b] block rows / cols
  const int mt_n = cdiv(M, TM), nt_n = cdiv(N, TM);
  const int split = item / (mt_n * nt_n);
  const int rem = item - split * mt_n * nt_n;
  const int mt = rem / nt_n, nt = rem - mt * nt_n;
  const int bm = mt * TM, bn = nt * TM;
  const int r0 = split * DW_K;
  u16* sA = smem;
  u16* sB = smem + DW_K * TLD;
  constexpr int G = DW_K * 8 / NTH;
  uint4 ra[G], rb[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int e = t + NTH * g;
    const int k = e >> 3, c8 = (e & 7) * 8;
    const int r = r0 + k;
    const bool okr = r < a.R;
    const int gm = bm + c8, gn = bn + c8;
    // A rows are stored to ld >= n with zero pads, so a whole 8-group loads whenever it starts
    // inside the row; the virtual ones column m == n (bias gradient) is patched in after.
    uint4 va = ld_u4(okr && gm < P.ld, P.A + (size_t)r * P.ld + gm, P.A);
    if (gm <= P.n && P.n < gm + 8) {  // the group holding m == n: ones there, zeros after
      u16 x[8];
      const unsigned w4[4] = {va.x, va.y, va.z, va.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = gm + i;
        const u16 cur = (u16)(w4[i >> 1] >> (16 * (i & 1)));
        x[i] = m < P.n ? cur : (m == P.n && okr ? (u16)0x3f80 : (u16)0);
      }
      va.x = x[0] | ((unsigned)x[1] << 16); va.y = x[2] | ((unsigned)x[3] << 16);
      va.z = x[4] | ((unsigned)x[5] << 16); va.w = x[6] | ((unsigned)x[7] << 16);
    } else if (gm > P.n) {
      va = make_uint4(0u, 0u, 0u, 0u);
    }
    ra[g] = va;
    rb[g] = ld_u4(okr && gn < C.ld, C.dZ + (size_t)r * C.ld + gn, C.dZ);
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int e = t + NTH * g;
    const int k = e >> 3, c8 = (e & 7) * 8;
    *reinterpret_cast<uint4*>(&sA[k * TLD + c8]) = ra[g];
    *reinterpret_cast<uint4*>(&sB[k * TLD + c8]) = rb[g];
  }
  lds_barrier();
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll 2
  for (int ks = 0; ks < DW_K; ks += 32) {
    const bf16x8 af = tr_frag72(sA, ks, wm * 16, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bf16x8 bfr = tr_frag72(sB, ks, wn * 32 + j * 16, lane);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[j], 0, 0, 0);
    }
  }
  float DSSM_GAS* out = C.slab + (size_t)split * M * N;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = bn + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = bm + wm * 16 + (lane >> 4) * 4 + r;
      if (m < M && n < N) out[(size_t)m * N + n] = acc[j][r];
    }
  }
  lds_barrier();
}

// ---- cosine / softmax / loss for query j (one wave), BN_L + ReLU fused, dy_L masked -------
// KMAX >= NEG + 1 (8 or 16) bounds the per-lane arrays; the pre-BN values needed for xhat in
// the backward are re-read (L2-resident) instead of being held across the forward.
// sco: LDS coefficients of layer L, [tower][mu | rstd | inv | shift][ld].
template <int EPL, int KMAX>
__device__ __forceinline__ void cosine_query(const DenseArgs& a, int j, int train, const float* sco,
                             float (&s1)[2][EPL], float (&s2)[2][EPL], float& lj, float& cj) {
  const DenseLayer& C = a.ly[a.L - 1];
  const int lane = threadIdx.x & 63;
  const int n = C.n, ld = C.ld, bs = a.BS, neg = a.NEG, K = neg + 1;
  auto co = [&](int t, int which, int c) { return sco[(t * 4 + which) * ld + c]; };
  auto doc_row = [&](int k) { return k == 0 ? bs + j : 2 * bs + j * neg + (k - 1); };
  float q[EPL], d[KMAX][EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int c = lane + 64 * e;
    q[e] = ld1(c < n, C.Z + (size_t)j * ld + c, C.Z);
  }
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int c = lane + 64 * e;
      d[k][e] = ld1(k < K && c < n, C.Z + (size_t)doc_row(k < K ? k : 0) * ld + c, C.Z);
    }
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int c = lane + 64 * e;
    if (c < n) {
      q[e] = fmaxf(bn_affine(q[e], co(0, 2, c), co(0, 3, c)), 0.f);
      const float inv = co(1, 2, c), sh = co(1, 3, c);
#pragma unroll
      for (int k = 0; k < KMAX; ++k) d[k][e] = (k < K) ? fmaxf(bn_affine(d[k][e], inv, sh), 0.f) : 0.f;
    }
  }
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int c = lane + 64 * e;
    if (c < ld) {
      C.Y[(size_t)j * ld + c] = q[e];
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < K) C.Y[(size_t)doc_row(k) * ld + c] = d[k][e];
    }
  }
  float qq = 0.f;
#pragma unroll
  for (int e = 0; e < EPL; ++e) qq = __fmaf_rn(q[e], q[e], qq);
  qq = wave_sum(qq);
  const float qn = sqrtf(qq);
  float cs[KMAX], dn[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    cs[k] = 0.f;
    dn[k] = 1.f;
    if (k < K) {
      float dd = 0.f, qd = 0.f;
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        dd = __fmaf_rn(d[k][e], d[k][e], dd);
        qd = __fmaf_rn(q[e], d[k][e], qd);
      }
      dd = wave_sum(dd);
      qd = wave_sum(qd);
      dn[k] = sqrtf(dd);
      cs[k] = qd / (qn * dn[k]);
    }
  }
  const float gamma = a.gamma_cos;
  float mx = gamma * cs[0];
#pragma unroll
  for (int k = 1; k < KMAX; ++k)
    if (k < K) mx = fmaxf(mx, gamma * cs[k]);
  float p[KMAX], sum = 0.f;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    p[k] = (k < K) ? expf(gamma * cs[k] - mx) : 0.f;
    sum += p[k];
  }
  int amax = 0;
  float pbest = -1.f;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    p[k] = p[k] / sum;
    if (k < K && p[k] > pbest) { pbest = p[k]; amax = k; }
  }
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (k < K && k == lane) {
      a.cos_raw[(size_t)k * bs + j] = cs[k];
      a.cos_sim[(size_t)j * K + k] = gamma * cs[k];
      a.prob[(size_t)j * K + k] = p[k];
    }
  if (lane == 0) a.qnorm[j] = qn;
  lj += -logf(p[0]);
  cj += (amax == 0) ? 1.f : 0.f;
  if (!train) return;
  // backward of cosine/softmax: d loss / d cos_sim[j,k] = (p_k - [k==0]) / BS; ReLU mask
  float dq[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) dq[e] = 0.f;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (k < K) {
      const float g = gamma * (p[k] - (k == 0 ? 1.f : 0.f)) / (float)bs;
      const float ak = g / (qn * dn[k]);
      const float bq = g * cs[k] / (qn * qn);
      const float bd = g * cs[k] / (dn[k] * dn[k]);
      const size_t row = (size_t)doc_row(k) * ld;
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int c = lane + 64 * e;
        dq[e] += ak * d[k][e] - bq * q[e];
        if (c < ld) {
          float dy = 0.f;
          if (c < n && d[k][e] > 0.f) {
            dy = ak * q[e] - bd * d[k][e];
            const float xh = (C.Z[row + c] - co(1, 0, c)) * co(1, 1, c);
            s1[1][e] += dy;
            s2[1][e] = __fmaf_rn(dy, xh, s2[1][e]);
          }
          C.dy[row + c] = dy;
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int c = lane + 64 * e;
    if (c < ld) {
      float dy = 0.f;
      if (c < n && q[e] > 0.f) {
        dy = dq[e];
        const float xh = (C.Z[(size_t)j * ld + c] - co(0, 0, c)) * co(0, 1, c);
        s1[0][e] += dy;
        s2[0][e] = __fmaf_rn(dy, xh, s2[0][e]);
      }
      C.dy[(size_t)j * ld + c] = dy;
    }
  }
}

// cosine phase + (last block) loss, EMA, batch moments and materialized coefficients
template <int EPL, int KMAX>
__device__ __forceinline__ void cosine_phase(const DenseArgs& a, int train, float* smemf, float* s_red, int* s_flag) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const DenseLayer& C = a.ly[a.L - 1];
  const int ld = C.ld;
  float* sco = smemf;                   // [2][4][ld]
  float* base = smemf + 8 * ld;         // [NW][2][2][64*EPL]
  for (int i = threadIdx.x; i < 2 * ld; i += NTH) {
    const int t = i / ld, c = i - t * ld;
    float mu, var, rs, inv, sh;
    bn_coef(a, C, t, c, train, mu, var, rs, inv, sh);
    sco[(t * 4 + 0) * ld + c] = mu;
    sco[(t * 4 + 1) * ld + c] = rs;
    sco[(t * 4 + 2) * ld + c] = inv;
    sco[(t * 4 + 3) * ld + c] = sh;
  }
  lds_barrier();
  float s1[2][EPL], s2[2][EPL];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < EPL; ++e) s1[t][e] = s2[t][e] = 0.f;
  float lj = 0.f, cj = 0.f;
  for (int j = blockIdx.x * NW + w; j < a.BS; j += gridDim.x * NW)
    cosine_query<EPL, KMAX>(a, j, train, sco, s1, s2, lj, cj);
  if (lane == 0) {
    s_red[w] = lj;
    s_red[NW + w] = cj;
  }
  if (train) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        base[((w * 2 + t) * 2 + 0) * 64 * EPL + e * 64 + lane] = s1[t][e];
        base[((w * 2 + t) * 2 + 1) * 64 * EPL + e * 64 + lane] = s2[t][e];
      }
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    float x = 0.f, y = 0.f;
    for (int k = 0; k < NW; ++k) {
      x += s_red[k];
      y += s_red[NW + k];
    }
    a.loss_part[2 * blockIdx.x] = x;
    a.loss_part[2 * blockIdx.x + 1] = y;
  }
  if (train && (int)blockIdx.x * NW < a.BS) {  // blocks that processed queries add BN_L sums
    for (int idx = threadIdx.x; idx < 2 * 2 * C.n; idx += NTH) {
      const int ts = idx / C.n, c = idx - ts * C.n;  // ts = tower*2 + s
      float acc = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) acc += base[(ww * 4 + ts) * 64 * EPL + c];
      atomic_addd(C.bsum + (size_t)ts * ld + c, (double)acc);
    }
  }
  if (!last_block_arrival((unsigned*)a.tickets, gridDim.x, s_flag)) return;
  // ---- last block: loss / accuracy, then per layer: EMA, batch moments, coefficients ------
  if (threadIdx.x < 64) {
    float x = 0.f, y = 0.f;
    for (int i = lane; i < (int)gridDim.x; i += 64) {
      x += a.loss_part[2 * i];
      y += a.loss_part[2 * i + 1];
    }
    x = bcast_f(wave_sum(x), 0);
    y = bcast_f(wave_sum(y), 0);
    if (lane == 0) {
      a.loss[0] = x / (float)a.BS;
      a.loss[1] = y / (float)a.BS;
    }
  }
  for (int l = 0; l < a.L; ++l) {
    const DenseLayer& D = a.ly[l];
    const size_t plane = (size_t)2 * D.ld;
    for (int i = threadIdx.x; i < 2 * D.ld; i += NTH) {
      const int t = i / D.ld, c = i - t * D.ld;
      float mu, var, rs, inv, sh;
      bn_coef(a, D, t, c, train, mu, var, rs, inv, sh);
      const size_t o = (size_t)t * D.ld + c;
      D.coef[o] = mu;
      D.coef[plane + o] = rs;
      D.coef[2 * plane + o] = inv;
      D.coef[3 * plane + o] = sh;
      if (train) {
        if (c < D.n) {
          D.bmean[t * D.n + c] = mu;
          D.bvar[t * D.n + c] = var;
          // ExponentialMovingAverage(decay).apply: shadow -= (shadow - value) * (1 - decay)
          float DSSM_GAS* em = D.ema_mean[t];
          float DSSM_GAS* ev = D.ema_var[t];
          const float one_m = 1.0f - a.decay;
          em[c] = em[c] - (em[c] - mu) * one_m;
          ev[c] = ev[c] - (ev[c] - var) * one_m;
        }
        D.fsum[(size_t)(t * 2) * D.ld + c] = 0.0;
        D.fsum[(size_t)(t * 2 + 1) * D.ld + c] = 0.0;
      }
    }
  }
}

// ---- the kernels ---------------------------------------------------------------------------
template <int EPL, int KMAX>
__global__ __launch_bounds__(NTH) void k_dense_fwd(const DenseArgs* __restrict__ ap, int train) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  __shared__ double dred[2 * NTH];
  __shared__ float s_red[2 * NW];
  __shared__ int s_flag;
  const DenseArgs& a = *ap;
  unsigned gen = read_gen(a.bar);
  unsigned long long DSSM_GAS* tm = a.timing;
  int ti = 0;
  stamp(tm, ti);
  if (train) {
    // the cosine phase below starts the backward sums of this step: clear all of them first
    for (int l = 0; l < a.L; ++l)
      for (int i = blockIdx.x * NTH + threadIdx.x; i < 4 * a.ly[l].ld; i += gridDim.x * NTH)
        a.ly[l].bsum[i] = 0.0;
    const int items = (a.R / TM) * cdiv(a.ly[0].ld, TM);
    for (int it = blockIdx.x; it < items; it += gridDim.x) stats_item(a, it, dred);
    if (!grid_sync(a.bar, gen, &s_flag, tm, ti)) return;
  }
  for (int l = 1; l < a.L; ++l) {
    fwd_phase(a, l, train, smem, dred);
    if (!grid_sync(a.bar, gen, &s_flag, tm, ti)) return;
  }
  cosine_phase<EPL, KMAX>(a, train, reinterpret_cast<float*>(smem), s_red, &s_flag);
  stamp(tm, ti);
}

__global__ __launch_bounds__(NTH) void k_dense_bwd(const DenseArgs* __restrict__ ap) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  __shared__ double dred[2 * 64];
  __shared__ int s_flag;
  const DenseArgs& a = *ap;
  unsigned gen = read_gen(a.bar);
  const int L = a.L;
  unsigned long long DSSM_GAS* tm = a.timing ? a.timing + 64 : nullptr;
  int ti = 0;
  stamp(tm, ti);
  // phase for layer l (L-1 .. 1): dA items (dZ_l staged) + dW_{l+1} items (dZ_{l+1} complete)
  for (int l = L - 1; l >= 1; --l) {
    const int dw_items =
        l < L - 1 ? a.ly[l + 1].splits * cdiv(a.ly[l].n + 1, TM) * cdiv(a.ly[l + 1].n, TM) : 0;
    for (int it = blockIdx.x; it < dw_items; it += gridDim.x) dw_item(a, l + 1, it, smem);
    bwd_phase(a, l, smem, dred);
    if (!grid_sync(a.bar, gen, &s_flag, tm, ti)) return;
  }
  // last phase: dW_2 and dZ1 = inv*dy + c1*z + c0 (bf16, for the dW1 gathers)
  {
    const int dw_items = a.ly[1].splits * cdiv(a.ly[0].n + 1, TM) * cdiv(a.ly[1].n, TM);
    for (int it = blockIdx.x; it < dw_items; it += gridDim.x) dw_item(a, 1, it, smem);
    const DenseLayer& C = a.ly[0];
    float* sk = reinterpret_cast<float*>(smem);  // [tower][inv | c1 | c0][ld]
    const int ld = C.ld;
    for (int i = threadIdx.x; i < 2 * ld; i += NTH) {
      const int t = i / ld, c = i - t * ld;
      float inv, c1, c0;
      bn_dcoef(a, C, t, c, inv, c1, c0);
      sk[(t * 3 + 0) * ld + c] = inv;
      sk[(t * 3 + 1) * ld + c] = c1;
      sk[(t * 3 + 2) * ld + c] = c0;
    }
    lds_barrier();
    const int q = ld >> 2;
    const size_t total = (size_t)a.R * q;
    for (size_t i = (size_t)blockIdx.x * NTH + threadIdx.x; i < total; i += (size_t)gridDim.x * NTH) {
      const int r = (int)(i / q);
      const int c = (int)(i - (size_t)r * q) * 4;
      const float* k = sk + tower_of(r, a.BS) * 3 * ld + c;
      const float4 z = gload_f4(C.Z + (size_t)r * ld + c);
      const float4 dy = gload_f4(C.dy + (size_t)r * ld + c);
      uint2 pk;
      pk.x = pack2bf(__fmaf_rn(k[0], dy.x, __fmaf_rn(k[ld], z.x, k[2 * ld])),
                     __fmaf_rn(k[1], dy.y, __fmaf_rn(k[ld + 1], z.y, k[2 * ld + 1])));
      pk.y = pack2bf(__fmaf_rn(k[2], dy.z, __fmaf_rn(k[ld + 2], z.z, k[2 * ld + 2])),
                     __fmaf_rn(k[3], dy.w, __fmaf_rn(k[ld + 3], z.w, k[2 * ld + 3])));
      gstore_u2(C.dZ + (size_t)r * ld + c, pk);
    }
  }
  if (!last_block_arrival((unsigned*)(a.tickets + 64), gridDim.x, &s_flag)) {
    stamp(tm, ti);
    return;
  }
  // ---- last block: dgamma / dbeta of every layer from the sums; re-zero the sums ----------
  for (int l = 0; l < L; ++l) {
    const DenseLayer& D = a.ly[l];
    for (int i = threadIdx.x; i < 2 * D.ld; i += NTH) {
      const int t = i / D.ld, c = i - t * D.ld;
      if (c < D.n) {
        D.dbeta[t][c] = (float)D.bsum[(size_t)(t * 2) * D.ld + c];
        D.dgamma[t][c] = (float)D.bsum[(size_t)(t * 2 + 1) * D.ld + c];
      }
      D.bsum[(size_t)(t * 2) * D.ld + c] = 0.0;
      D.bsum[(size_t)(t * 2 + 1) * D.ld + c] = 0.0;
    }
  }
  stamp(tm, ti);
}

// dW slab reduction (non-deferred mode): gW = sum_s slab[s] in fixed order
__global__ __launch_bounds__(256) void k_dense_slab_reduce(const DenseArgs* __restrict__ ap) {
  const DenseArgs& a = *ap;
  for (int l = 1; l < a.L; ++l) {
    const DenseLayer& D = a.ly[l];
    const size_t cnt = (size_t)(a.ly[l - 1].n + 1) * D.n;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < cnt / 4; i += (size_t)gridDim.x * 256) {
      float4 acc = gload_f4(D.slab + 4 * i);
      for (int s = 1; s < D.splits; ++s) {
        const float4 x = gload_f4(D.slab + (size_t)s * cnt + 4 * i);
        acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
      }
      gstore_f4(D.gW + 4 * i, acc);
    }
  }
}

#define COMMA ,
#define DSSM_DENSE_FWD_E(X, K)                                                              \
  X(k_dense_fwd<1 COMMA K>) X(k_dense_fwd<2 COMMA K>) X(k_dense_fwd<4 COMMA K>)            \
  X(k_dense_fwd<8 COMMA K>)
#define DSSM_DENSE_KERNELS(X) DSSM_DENSE_FWD_E(X, 8) DSSM_DENSE_FWD_E(X, 16) X(k_dense_bwd)
#define DSSM_KPTR(k) (const void*)k,
const void* const kDenseKernels[] = {DSSM_DENSE_KERNELS(DSSM_KPTR)};
#undef DSSM_KPTR

}  // namespace

int dense_dw_splits(int R) { return cdiv(R, DW_K); }

size_t dense_smem_bytes(const int* ld, int L) {
  // the weight-stationary GEMM phases size their parts to kDenseSmem; the dW chunk (74 KB),
  // cosine (<= 64 KB) and dZ1 coefficients fit inside it
  (void)ld;
  (void)L;
  return (size_t)kDenseSmem;
}

bool dense_supported(int L, const int* n, const int* ld, int BS, int NEG) {
  if (L < 2 || BS % TM || NEG + 1 > 16) return false;
  for (int l = 0; l < L; ++l)
    if (ld[l] > 512 || n[l] % 4) return false;
  return true;
}

hipError_t dense_prepare(size_t smem) {
  for (const void* f : kDenseKernels) {
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_dense_fwd(const DenseArgs* dev_args, int last_ld, int kmax, int neg, int train,
                            int grid, size_t smem, hipStream_t s) {
  (void)kmax;
  const int epl = last_ld <= 64 ? 1 : last_ld <= 128 ? 2 : last_ld <= 256 ? 4 : 8;
  const bool k8 = neg + 1 <= 8;
#define DSSM_DF(E)                                                                              \
  if (k8)                                                                                       \
    hipLaunchKernelGGL((k_dense_fwd<E, 8>), dim3(grid), dim3(NTH), smem, s, dev_args, train);  \
  else                                                                                          \
    hipLaunchKernelGGL((k_dense_fwd<E, 16>), dim3(grid), dim3(NTH), smem, s, dev_args, train)
  if (epl == 1) { DSSM_DF(1); }
  else if (epl == 2) { DSSM_DF(2); }
  else if (epl == 4) { DSSM_DF(4); }
  else { DSSM_DF(8); }
#undef DSSM_DF
  return hipGetLastError();
}

hipError_t launch_dense_bwd(const DenseArgs* dev_args, int kmax, int defer, int grid, size_t smem,
                            hipStream_t s) {
  (void)kmax;
  hipLaunchKernelGGL(k_dense_bwd, dim3(grid), dim3(NTH), smem, s, dev_args);
  if (!defer) hipLaunchKernelGGL(k_dense_slab_reduce, dim3(512), dim3(256), 0, s, dev_args);
  return hipGetLastError();
}

int dense_max_grid(size_t smem) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (dense_prepare(smem) != hipSuccess) return 0;
  for (const void* k : kDenseKernels) {
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, NTH, smem) != hipSuccess || per < 1)
      return 0;
  }
  return cus;  // one workgroup per CU: every workgroup of the grid is co-resident
}

}  // namespace dssm
