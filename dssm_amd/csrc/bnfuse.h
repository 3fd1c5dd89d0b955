// Fused batch-norm statistics for the per-op bf16 path (gemm.hip, cosine.hip, bn.hip).
//
// The reference's tf.nn.moments (new_dssm.py:62-88) is a full reduction over the batch rows
// between a layer's MatMul and its normalisation.  Instead of a separate statistics launch per
// layer and direction, the kernel that PRODUCES a layer's pre-BN activations (the NT GEMM
// epilogue) or its backward input (the dA GEMM epilogue, the cosine kernel) adds per-column
// fp64 sums of its tile to a small accumulator with hardware fp64 atomics:
//   forward : sum z, sum z^2                   -> mean, biased variance (E[z^2] - mean^2 in fp64)
//   backward: sum dy, sum dy*xhat (dy = ReLU-masked dA, xhat = (z - mean) * rstd)
// and the kernel that CONSUMES the layer derives the coefficients it needs from the sums in its
// prologue (every workgroup redundantly: <= 2 x 512 columns).  One designated workgroup of the
// consumer also materialises them (coef / batch moments / EMA update, or dgamma / dbeta), so
// the rest of the step and the host read exactly what the unfused path writes.
//
// The sums are fp64 accumulations of fp32 values: the result does not depend on the atomic
// order beyond fp64 rounding, far below the fp32 outputs' resolution.  They are zeroed by the
// first launch of the next train step (the CSC histogram, spmm.hip).  Same-address fp64 atomics
// serialise (measured on MI355X: ~23 ns each; tools/micro/atomics.hip): producers keep the chains
// short by summing many rows per workgroup before their one atomic per (statistic, column).
#pragma once
#include "common.h"

namespace dssm {

// Deterministic mode (DSSM_OPT_DETERMINISTIC) of the fused statistics.  Instead of fp64 atomics
// (exact up to fp64 rounding, whose order then varies), producer row r of a launch stores its
// per-column partials of the accumulator [2 towers][2][ld] into slab row r -- zeros for the tower
// it does not cover -- and the rows are summed by a two-level tree fixed by row index
// (det_publish): the last arrival of each group of consecutive rows sums them in order into a
// level-2 row, the last group's arrival sums the level-2 rows in order into the accumulator.
// Most of the summing happens while other producers still run; the launch's tail is one short sum.
constexpr int kDetTiles = 8;     // column tiles of 64 (ld <= 512)
constexpr int kDetTickets = 32;  // tickets per column tile: [0] level 2, [1 + g] group g
struct DetAcc {
  double* slab;      // [cap + cap / 8 + 1][4][ld]: level-1 rows, then level-2 rows (null: atomics)
  unsigned* ticket;  // [kDetTiles][kDetTickets], zero-initialised, re-armed by the last arrivals
  int cap;           // level-1 rows (producer rows of one launch) the slab holds
};
// rows per level-1 group for a launch of `nrows` producer rows (at most kDetTickets - 1 groups)
__host__ __device__ inline int det_group(int nrows) {
  const int g = (nrows + kDetTickets - 2) / (kDetTickets - 1);
  return g > 8 ? g : 8;
}
__host__ __device__ inline size_t det_slab_rows(int cap) { return (size_t)cap + cap / 8 + 1; }

struct BnSide {
  int n, ld;        // width, padded row stride
  int rows_q, rows_d;  // rows of the query / doc tower (row_split, rows - row_split)
  float eps, decay;
  const float* gamma[2];
  const float* beta[2];
  float* ema_mean[2];
  float* ema_var[2];
  float* coef;      // [4][2][ld]: mean, rstd, inv = gamma*rstd, shift = beta - mean*inv
  float* bmean;     // [2][n] batch moments (train)
  float* bvar;
  double* fsum;     // [2 towers][2][ld]: sum z, sum z^2
  double* bsum;     // [2 towers][2][ld]: sum dy, sum dy*xhat
  float* dgamma[2];
  float* dbeta[2];
  DetAcc fdet, bdet;  // deterministic mode: the producers' slabs of fsum / bsum (slab null: atomics)
};

// Element t (0 / 1) of a two-pointer array of a kernel argument, as a select of the two (uniform)
// pointers: indexing the array with a lane-varying t makes the compiler fetch the pointer from the
// argument segment with a vector load, a dependent round trip before the data load.
template <typename P>
__device__ __forceinline__ P pick2(P const (&a)[2], int t) {
  return t ? a[1] : a[0];
}

__device__ __forceinline__ void atomic_add_f64(double* p, double v) {
#ifdef DSSM_DIAG_NO_STAT_ATOMICS  // diagnostics (wrong results): plain stores, to time the chains
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

// The slab rows are handed from workgroup to workgroup inside one launch WITHOUT agent-scope
// fences: every slab store is write-through (sc1: an agent-scope relaxed atomic store, the line
// leaves the XCD's L2) and drained by its wave before the arrival, and every read of a slab row is
// an sc1 load (an agent-scope relaxed atomic load).  That is MI355X_MICROARCH.md's measured
// fence-free hand-off form (inter-workgroup visibility, "Valid forms": sc1 stores drained before
// one lane's agent-scope ticket add, the last adder's sc1 loads).  Round 6: the release fence it
// replaces wrote back the XCD L2's dirty lines -- the producer's whole output tile -- in every
// producer workgroup (+6.5 us per statistics launch in deterministic mode).
__device__ __forceinline__ void det_st(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double det_ld(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every storing thread's write-through slab stores drained, then one lane's arrival on
// ticket[tile]: true (block-uniform) in the workgroup that arrived last of `expected`.
__device__ __forceinline__ bool det_arrive(unsigned* ticket, unsigned expected, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old == expected - 1;
    if (last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
    *s_flag = last ? 1 : 0;
  }
  __syncthreads();
  return *s_flag != 0;
}

// Fixed-order sum of nr consecutive slab rows from row r0: dst[k * ld + c] = sum over rows (in
// order) of src[((r0 + r) * 4 + k) * ld + c], k < 4, c in [c0, c1); 16 loads in flight per thread.
// A level-2 destination is itself handed off (handoff = true: write-through stores); the final
// accumulator is read by the next launch (plain stores).
__device__ __forceinline__ void det_sum_rows(const double* src, int r0, int nr, int ld, int c0, int c1,
                                             double* dst, bool handoff) {
  const int w = c1 - c0;
  for (int i = threadIdx.x; i < 4 * w; i += blockDim.x) {
    const int k = i / w, c = c0 + i - k * w;
    const double* p = src + ((size_t)r0 * 4 + k) * ld + c;
    double a = 0.0;
    for (int r = 0; r < nr; r += 16) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = r + u < nr ? det_ld(p + (size_t)(r + u) * 4 * ld) : 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u) a += v[u];
    }
    if (handoff) det_st(dst + (size_t)k * ld + c, a);
    else dst[(size_t)k * ld + c] = a;
  }
}

// Producer `row` of `nrows` (block-uniform call) has stored its slab row for column tile `tile`
// (columns [c0, c1)): arrive, and sum what this workgroup arrived last for (module comment).
__device__ __forceinline__ void det_publish(const DetAcc& d, int tile, int row, int nrows, int ld, int c0, int c1,
                                            double* out, int* s_flag) {
  unsigned* tk = d.ticket + tile * kDetTickets;
  const int G = det_group(nrows), ng = (nrows + G - 1) / G;
  if (ng == 1) {
    if (det_arrive(tk, (unsigned)nrows, s_flag)) det_sum_rows(d.slab, 0, nrows, ld, c0, c1, out, false);
    return;
  }
  const int g = row / G, gn = min(G, nrows - g * G);
  if (!det_arrive(tk + 1 + g, (unsigned)gn, s_flag)) return;
  double* lvl2 = d.slab + (size_t)nrows * 4 * ld;
  det_sum_rows(d.slab, g * G, gn, ld, c0, c1, lvl2 + (size_t)g * 4 * ld, true);
  if (det_arrive(tk, (unsigned)ng, s_flag)) det_sum_rows(lvl2, 0, ng, ld, c0, c1, out, false);
}

// Forward coefficients of column c (< n), tower t, from the step's sums s = sum z, q = sum z^2
// (biased variance).
__device__ __forceinline__ void fs_coef_from(const BnSide& b, int t, int c, double s, double q,
                                             float& mu, float& var, float& rstd, float& inv,
                                             float& shift) {
  const double N = t == 0 ? b.rows_q : b.rows_d;
  const double m = s / N;
  const double v = q / N - m * m;
  mu = (float)m;
  var = (float)(v > 0.0 ? v : 0.0);
  rstd = 1.0f / sqrtf(var + b.eps);
  inv = rstd * pick2(b.gamma, t)[c];
  shift = pick2(b.beta, t)[c] - mu * inv;
}
__device__ __forceinline__ void fs_coef(const BnSide& b, int t, int c, float& mu, float& var,
                                        float& rstd, float& inv, float& shift) {
  const double s = b.fsum[(t * 2) * b.ld + c], q = b.fsum[(t * 2 + 1) * b.ld + c];
  fs_coef_from(b, t, c, s, q, mu, var, rstd, inv, shift);
}

// Every thread of the workgroup derives the coefficients of items i = tid + nthreads*u
// (u < NPER, i < 2*ld; tower i / ld, column i % ld) with all loads in flight at once:
// load() issues the loads (call it before a kernel's bulk loads so these return first),
// finish() calls out(tower, column, mu, rstd, inv, shift) (zeros for pad columns >= n).
template <int NPER>
struct FsCoefStage {
  double s[NPER], q[NPER];
  float gm[NPER], bt[NPER];
  __device__ __forceinline__ void load(const BnSide& b, int tid, int nthreads) {
    int off[NPER];
#pragma unroll
    for (int u = 0; u < NPER; ++u) {
      const int i = tid + nthreads * u;
      const int ic = i < 2 * b.ld ? i : 0;  // clamped: every load issued, unconditionally
      const int t = ic / b.ld, c = ic - t * b.ld;
      const int cn = c < b.n ? c : 0;
      off[u] = (t * 2) * b.ld + c;
      gm[u] = pick2(b.gamma, t)[cn];
      bt[u] = pick2(b.beta, t)[cn];
    }
#pragma unroll
    for (int u = 0; u < NPER; ++u) {
      s[u] = b.fsum[off[u]];
      q[u] = b.fsum[off[u] + b.ld];
    }
  }
  template <typename F>
  __device__ __forceinline__ void finish(const BnSide& b, int tid, int nthreads, F&& out) const {
#pragma unroll
    for (int u = 0; u < NPER; ++u) {
      const int i = tid + nthreads * u;
      if (i < 2 * b.ld) {
        const int t = i / b.ld, c = i - t * b.ld;
        float mu = 0.f, rs = 0.f, inv = 0.f, sh = 0.f;
        if (c < b.n) {
          const double N = t == 0 ? b.rows_q : b.rows_d;
          const double m = s[u] / N;
          const double v = q[u] / N - m * m;
          mu = (float)m;
          const float var = (float)(v > 0.0 ? v : 0.0);
          rs = 1.0f / sqrtf(var + b.eps);
          inv = rs * gm[u];
          sh = bt[u] - mu * inv;
        }
        out(t, c, mu, rs, inv, sh);
      }
    }
  }
};
template <int NPER, typename F>
__device__ __forceinline__ void fs_coef_stage(const BnSide& b, int tid, int nthreads, F&& out) {
  FsCoefStage<NPER> st;
  st.load(b, tid, nthreads);
  st.finish(b, tid, nthreads, out);
}

// Per-tower column sums of z and z^2 of one kSumsRows x 64 block (NT threads: NT/64 row groups),
// fp64 atomics into fsum [2 towers][2][ldz]; blocks never straddle the tower boundary.
#ifndef DSSM_SUMS_ROWS
#define DSSM_SUMS_ROWS 128
#endif
constexpr int kSumsRows = DSSM_SUMS_ROWS;  // 256-row blocks measured +0.4 us/step (round 3)
template <int NT>
__device__ __forceinline__ void bn_sums_block(const float* __restrict__ Z, int ldz, int ncol,
                                              int row_split, int rows, double* __restrict__ fsum,
                                              int bx, int by, double (*s_red)[NT / 64][64],
                                              DetAcc det = DetAcc{}, int nby = 0) {
  constexpr int NG = NT / 64, RPT = kSumsRows / NG;
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = bx * 64 + lane;
  const int r0 = by * kSumsRows, r1 = min(rows, r0 + kSumsRows);
  const int tower = r0 < row_split ? 0 : 1;
  float x[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {  // all loads issued before any arithmetic
    const int r = r0 + g + NG * i;
    x[i] = Z[(size_t)(r < r1 ? r : r0) * ldz + (c < ldz ? c : 0)];
  }
  double s = 0.0, q = 0.0;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const float v = (r0 + g + NG * i < r1) ? x[i] : 0.f;
    s += v;
    q += (double)v * v;
  }
  s_red[0][g][lane] = s;
  s_red[1][g][lane] = q;
  __syncthreads();
  if (g < 2 && c < ncol) {
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < NG; ++k) a += s_red[g][k][lane];
    if (det.slab) {  // this row block's partials, the other tower's zero (deterministic mode)
      double* row = det.slab + (size_t)by * 4 * ldz;
      det_st(row + (size_t)(tower * 2 + g) * ldz + c, a);
      det_st(row + (size_t)((1 - tower) * 2 + g) * ldz + c, 0.0);
    } else {
      atomic_add_f64(fsum + (size_t)(tower * 2 + g) * ldz + c, a);
    }
  }
  if (det.slab) {
    __shared__ int s_last;
    det_publish(det, bx, by, nby, ldz, bx * 64, min(bx * 64 + 64, ncol), fsum, &s_last);
  }
}

// Materialise layer b's forward coefficients, batch moments and EMA update (one workgroup; its
// sums, gamma/beta and EMA loads all in flight at once).
__device__ __forceinline__ void fs_materialize_fwd(const BnSide& b) {
  constexpr int NPER = 4;  // 2 * 512 (max ld) / 256 threads; larger workgroups loop
  const size_t plane = (size_t)2 * b.ld;
  for (int base = 0; base < 2 * b.ld; base += NPER * (int)blockDim.x) {
    FsCoefStage<NPER> st;
    st.load(b, base + threadIdx.x, blockDim.x);
    float em[NPER], ev[NPER];
#pragma unroll
    for (int u = 0; u < NPER; ++u) {
      const int i = base + threadIdx.x + blockDim.x * u;
      const int ic = i < 2 * b.ld ? i : 0;
      const int t = ic / b.ld, c = ic - t * b.ld;
      const int cn = c < b.n ? c : 0;
      em[u] = pick2(b.ema_mean, t)[cn];
      ev[u] = pick2(b.ema_var, t)[cn];
    }
    // the coefficient arithmetic of FsCoefStage::finish, unrolled here so that the sums are read by
    // compile-time index (a counter in finish's callback indexed them at run time: scratch memory
    // for every workgroup of the producing launch)
#pragma unroll
    for (int u = 0; u < NPER; ++u) {
      const int i = base + threadIdx.x + blockDim.x * u;
      if (i < 2 * b.ld) {
        const int t = i / b.ld, c = i - t * b.ld;
        float mu = 0.f, var = 0.f, rstd = 0.f, inv = 0.f, shift = 0.f;
        if (c < b.n) {
          const double N = t == 0 ? b.rows_q : b.rows_d;
          const double m = st.s[u] / N;
          const double v = st.q[u] / N - m * m;
          mu = (float)m;
          var = (float)(v > 0.0 ? v : 0.0);
          rstd = 1.0f / sqrtf(var + b.eps);
          inv = rstd * st.gm[u];
          shift = st.bt[u] - mu * inv;
        }
        const size_t o = (size_t)t * b.ld + c;
        b.coef[o] = mu;
        b.coef[plane + o] = rstd;
        b.coef[2 * plane + o] = inv;
        b.coef[3 * plane + o] = shift;
        if (c < b.n) {
          b.bmean[t * b.n + c] = mu;
          b.bvar[t * b.n + c] = var;
          // ExponentialMovingAverage(decay).apply: shadow -= (shadow - value) * (1 - decay)
          const float one_m = 1.0f - b.decay;
          pick2(b.ema_mean, t)[c] = em[u] - (em[u] - mu) * one_m;
          pick2(b.ema_var, t)[c] = ev[u] - (ev[u] - var) * one_m;
        }
      }
    }
  }
}

// Backward means of column c, tower t: m1 = mean(dy), m2 = mean(dy*xhat).
__device__ __forceinline__ void fs_bsums(const BnSide& b, int t, int c, double& s1, double& s2) {
  s1 = b.bsum[(t * 2) * b.ld + c];
  s2 = b.bsum[(t * 2 + 1) * b.ld + c];
}
__device__ __forceinline__ void fs_dcoef(const BnSide& b, int t, int c, float& m1, float& m2) {
  const double N = t == 0 ? b.rows_q : b.rows_d;
  double s1, s2;
  fs_bsums(b, t, c, s1, s2);
  m1 = (float)(s1 / N);
  m2 = (float)(s2 / N);
}

// BN + ReLU backward of one element: dZ = inv * (dy - m1 - xhat * m2), dy = da where BN(z) > 0
// (ReluGrad), xhat = (z - mu) * rstd, m1 / m2 the column's mean(dy) / mean(dy * xhat).  Every
// operation rounded on its own (no FMA contraction), so each kernel that forms dZ -- bn.hip's apply
// launches, gemm.hip's pair with the BN backward folded into its staging -- gets the same fp32 value.
__device__ __forceinline__ float bn_bwd_dz(float z, float da, float mu, float rstd, float inv, float sh,
                                           float m1, float m2) {
#pragma clang fp contract(off)  // (HIP's __fmul_rn / __fsub_rn are plain operators: contractible)
  const float dy = (bn_affine(z, inv, sh) > 0.f) ? da : 0.f;
  const float xh = (z - mu) * rstd;
  return inv * ((dy - m1) - xh * m2);
}

// dbeta = sum dy, dgamma = sum dy*xhat per tower (one workgroup).
__device__ __forceinline__ void fs_materialize_bwd(const BnSide& b) {
  for (int i = threadIdx.x; i < 2 * b.n; i += blockDim.x) {
    const int t = i / b.n, c = i - t * b.n;
    double s1, s2;
    fs_bsums(b, t, c, s1, s2);
    pick2(b.dbeta, t)[c] = (float)s1;
    pick2(b.dgamma, t)[c] = (float)s2;
  }
}

}  // namespace dssm
