// batch_normalization + ReLU (new_dssm.py:62-88, :128-136, :150-158) and its backward on gfx950.
//
// Towers: rows [0, row_split) are the query tower, [row_split, rows) the doc tower
// (concat[pos; neg], new_dssm.py:130) — each gets its own moments / gamma / beta / EMA.
//
// Statistics are ONE launch per layer and direction: blocks of 256 rows (never straddling a
// tower) x 64 columns (1024 threads: 16 row groups) compute per-column partials with all their loads in flight at once
// (thread <-> column, so every access is a coalesced 256-B row segment per wave), publish them,
// and the last block to finish a column chunk (agent-scope release/acquire ticket, per
// cdna_hip_programming.md §6 G16) merges the partials of that chunk in a fixed order and writes
// the per-column coefficients.  Results are deterministic: no float atomics, fixed merge order.
//   forward : partial (mean, M2) by two-pass over the block's rows; merge by the parallel-axis
//             formula (no E[x^2]-E[x]^2 cancellation); EMA update + affine coefficients.
//   backward: partial sum(dy), sum(dy*xhat) with dy = dA*[y>0]; finals are dbeta, dgamma and the
//             two means the input gradient needs.
// The affine+ReLU itself is applied by the consumers (GEMM A-operand staging, cosine kernel) or
// by k_bn_apply / k_bn_bwd_apply where a materialized tensor is needed.
#include <algorithm>
#include <cstdlib>

#include "bnfuse.h"
#include "common.h"
#include "launch.h"
#include "tn.h"
#include "g32.h"

namespace dssm {
namespace {

constexpr int NG = 16;        // row groups per block: 1024 threads = 16 groups x 64 columns
constexpr int RB = 256;       // rows per statistics block
constexpr int RPT = RB / NG;  // rows per thread

struct RowBlocks {
  int nq, nd;
  __host__ __device__ RowBlocks(BnTowers t)
      : nq(cdiv(t.row_split, RB)), nd(cdiv(t.rows - t.row_split, RB)) {}
  __host__ __device__ int total() const { return nq + nd; }
  __device__ void range(BnTowers t, int rb, int& r0, int& r1, int& tower) const {
    if (rb < nq) {
      r0 = rb * RB; r1 = min(r0 + RB, t.row_split); tower = 0;
    } else {
      r0 = t.row_split + (rb - nq) * RB; r1 = min(r0 + RB, t.rows); tower = 1;
    }
  }
};

struct BnParams {
  const float* gamma[2];
  const float* beta[2];
  float* ema_mean[2];
  float* ema_var[2];
};

// ---- forward statistics ----------------------------------------------------------------
// part layout: [rb][2][ldz] = (mean, M2) of the block's rows.  coef: [4][2][ldz] = mean_used,
// rstd, inv = gamma*rstd, shift = beta - mean*inv per tower.
__global__ __launch_bounds__(1024) void k_bn_stats(const float* __restrict__ Z, int ldz, int ncol,
                                                  BnTowers tw, BnParams P, float eps, float decay,
                                                  int train, float* __restrict__ part,
                                                  unsigned* __restrict__ tickets,
                                                  float* __restrict__ batch_mean,
                                                  float* __restrict__ batch_var,
                                                  float* __restrict__ coef,
                                                  double* __restrict__ zero, int nzero) {
  // partials, then the last block to arrive finalizes
  // zero: fused-statistics accumulators of this step's later layers (bnfuse.h), cleared here
  if (zero) {
    const int nb = gridDim.x * gridDim.y;
    for (int i = (blockIdx.y * gridDim.x + blockIdx.x) * 1024 + threadIdx.x; i < nzero; i += nb * 1024)
      zero[i] = 0.0;
  }
  __shared__ float s_a[NG][64], s_b[NG][64];
  __shared__ int s_flag;
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int rb = blockIdx.y;
  const RowBlocks blk(tw);
  const size_t plane = (size_t)2 * ldz;
  if (train) {
    int r0, r1, tower;
    blk.range(tw, rb, r0, r1, tower);
    float x[RPT];
    int n = 0;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {  // all loads issued before any arithmetic
      const int r = r0 + g + NG * i;
      x[i] = (r < r1 && c < ldz) ? Z[(size_t)r * ldz + c] : 0.f;
      n += (r < r1) ? 1 : 0;
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < RPT; ++i) s += x[i];
    const float mean = n ? s / (float)n : 0.f;
    float m2 = 0.f;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = r0 + g + NG * i;
      const float d = (r < r1) ? x[i] - mean : 0.f;
      m2 = __fmaf_rn(d, d, m2);
    }
    // merge the 4 row groups (counts n_g) with the parallel-axis formula
    s_a[g][lane] = s;
    s_b[g][lane] = m2;
    __syncthreads();
    if (g == 0 && c < ldz) {
      const int nb = r1 - r0;
      float tot = 0.f;
      for (int k = 0; k < NG; ++k) tot += s_a[k][lane];
      const float mu = tot / (float)nb;
      float M2 = 0.f;
      for (int k = 0; k < NG; ++k) {
        const int nk = max(0, min(RPT, (nb - k + NG - 1) / NG));
        const float mk = nk ? s_a[k][lane] / (float)nk : 0.f;
        const float dk = mk - mu;
        M2 += s_b[k][lane] + (float)nk * dk * dk;
      }
      part[((size_t)rb * 2) * ldz + c] = mu;
      part[((size_t)rb * 2 + 1) * ldz + c] = M2;
    }
    if (!last_block_arrival(&tickets[blockIdx.x], (unsigned)gridDim.y, &s_flag)) return;
  } else if (rb != 0) {
    return;  // eval: one block per column chunk just builds the coefficients from the EMA
  }
  // ---- finalize this column chunk (both towers) -------------------------------------------
  for (int tower = 0; tower < 2; ++tower) {
    const int first = tower == 0 ? 0 : blk.nq;
    const int count = tower == 0 ? blk.nq : blk.nd;
    const int nrows = tower == 0 ? tw.row_split : tw.rows - tw.row_split;
    if (count == 0) continue;
    float mu = 0.f, var = 0.f;
    if (train) {
      // pass 1: global mean = sum_i n_i mean_i / N
      // every partial this thread merges is loaded up front (one round of loads)
      constexpr int KMAX = 4;
      float pm[KMAX], pv[KMAX], pn[KMAX];
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        const int k = g + NG * j;
        pm[j] = pv[j] = pn[j] = 0.f;
        if (k < count && c < ldz) {
          const int rbk = first + k;
          int r0, r1, tt;
          blk.range(tw, rbk, r0, r1, tt);
          pn[j] = (float)(r1 - r0);
          pm[j] = part[((size_t)rbk * 2) * ldz + c];
          pv[j] = part[((size_t)rbk * 2 + 1) * ldz + c];
        }
      }
      float a = 0.f;
      for (int k = g + NG * KMAX; k < count; k += NG) {  // only for > KMAX*NG partials
        const int rbk = first + k;
        int r0, r1, tt;
        blk.range(tw, rbk, r0, r1, tt);
        if (c < ldz) a = __fmaf_rn((float)(r1 - r0), part[((size_t)rbk * 2) * ldz + c], a);
      }
#pragma unroll
      for (int j = 0; j < KMAX; ++j) a = __fmaf_rn(pn[j], pm[j], a);
      __syncthreads();
      s_a[g][lane] = a;
      __syncthreads();
      float tot = 0.f;
      for (int k = 0; k < NG; ++k) tot += s_a[k][lane];
      mu = tot / (float)nrows;
      // pass 2: M2 = sum_i M2_i + n_i (mean_i - mu)^2
      float b = 0.f;
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        const float d = pm[j] - mu;
        b += pv[j] + pn[j] * d * d;
      }
      for (int k = g + NG * KMAX; k < count; k += NG) {
        const int rbk = first + k;
        int r0, r1, tt;
        blk.range(tw, rbk, r0, r1, tt);
        if (c < ldz) {
          const float d = part[((size_t)rbk * 2) * ldz + c] - mu;
          b += part[((size_t)rbk * 2 + 1) * ldz + c] + (float)(r1 - r0) * d * d;
        }
      }
      s_b[g][lane] = b;
      __syncthreads();
      float tv = 0.f;
      for (int k = 0; k < NG; ++k) tv += s_b[k][lane];
      var = tv / (float)nrows;
    }
    if (g == 0 && c < ldz) {
      const size_t o = (size_t)tower * ldz + c;
      if (c >= ncol) {
        coef[o] = 0.f; coef[plane + o] = 0.f; coef[2 * plane + o] = 0.f; coef[3 * plane + o] = 0.f;
      } else {
        if (train) {
          if (batch_mean) {
            batch_mean[tower * ncol + c] = mu;
            batch_var[tower * ncol + c] = var;
          }
          // ExponentialMovingAverage(decay).apply: shadow -= (shadow - value) * (1 - decay)
          float* em = P.ema_mean[tower];
          float* ev = P.ema_var[tower];
          const float one_m = 1.0f - decay;
          em[c] = em[c] - (em[c] - mu) * one_m;
          ev[c] = ev[c] - (ev[c] - var) * one_m;
        } else {
          mu = P.ema_mean[tower][c];
          var = P.ema_var[tower][c];
        }
        const float rstd = 1.0f / sqrtf(var + eps);
        const float inv = rstd * pick2(P.gamma, tower)[c];
        coef[o] = mu;
        coef[plane + o] = rstd;
        coef[2 * plane + o] = inv;
        coef[3 * plane + o] = pick2(P.beta, tower)[c] - mu * inv;
      }
    }
  }
}

// Fused-statistics schedule (bnfuse.h): per-tower column sums of z and z^2 in fp64, one
// atomic per (column, statistic) per 256-row block; no partials, no finalize (the consumer
// derives the coefficients).
__global__ __launch_bounds__(1024) void k_bn_sums(const float* __restrict__ Z, int ldz, int ncol,
                                                 BnTowers tw, double* __restrict__ fsum, DetAcc det) {
  __shared__ double s_a[NG][64], s_b[NG][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const RowBlocks blk(tw);
  int r0, r1, tower;
  blk.range(tw, blockIdx.y, r0, r1, tower);
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
  s_a[g][lane] = s;
  s_b[g][lane] = q;
  __syncthreads();
  if (g < 2 && c < ncol) {
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < NG; ++k) a += g == 0 ? s_a[k][lane] : s_b[k][lane];
    if (det.slab) {  // deterministic: this row block's slab row, the other tower zero
      double* row = det.slab + (size_t)blockIdx.y * 4 * ldz;
      det_st(row + (size_t)(tower * 2 + g) * ldz + c, a);
      det_st(row + (size_t)((1 - tower) * 2 + g) * ldz + c, 0.0);
    } else {
      __hip_atomic_fetch_add(fsum + (size_t)(tower * 2 + g) * ldz + c, a, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (det.slab) {
    __shared__ int s_last;
    det_publish(det, blockIdx.x, blockIdx.y, gridDim.y, ldz, blockIdx.x * 64, min((int)blockIdx.x * 64 + 64, ncol),
                fsum, &s_last);
  }
}

template <typename TO>
__global__ __launch_bounds__(256) void k_bn_apply(const float* __restrict__ Z, int ldz,
                                                  BnTowers tw, const float* __restrict__ coef,
                                                  int relu, TO* __restrict__ out) {
  const int q = ldz >> 2;
  const size_t total = (size_t)tw.rows * q;
  const size_t plane = (size_t)2 * ldz;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / q);
    const int c = (int)(i - (size_t)r * q) * 4;
    const int tower = r < tw.row_split ? 0 : 1;
    const size_t o = (size_t)tower * ldz + c;
    const float4 z = *reinterpret_cast<const float4*>(Z + (size_t)r * ldz + c);
    const float4 inv = *reinterpret_cast<const float4*>(coef + 2 * plane + o);
    const float4 sh = *reinterpret_cast<const float4*>(coef + 3 * plane + o);
    float y[4] = {bn_affine(z.x, inv.x, sh.x), bn_affine(z.y, inv.y, sh.y),
                  bn_affine(z.z, inv.z, sh.z), bn_affine(z.w, inv.w, sh.w)};
    if (relu) {
#pragma unroll
      for (int k = 0; k < 4; ++k) y[k] = fmaxf(y[k], 0.f);
    }
    if constexpr (sizeof(TO) == 4) {
      *reinterpret_cast<float4*>((float*)out + (size_t)r * ldz + c) = make_float4(y[0], y[1], y[2], y[3]);
    } else {
      uint2 p;
      p.x = pack2bf(y[0], y[1]);
      p.y = pack2bf(y[2], y[3]);
      *reinterpret_cast<uint2*>((u16*)out + (size_t)r * ldz + c) = p;
    }
  }
}

// ---- backward ----------------------------------------------------------------------------
__device__ __forceinline__ void bwd_terms(float z, float da, float mu, float rstd, float inv,
                                          float shift, float& dy, float& xhat) {
  dy = (bn_affine(z, inv, shift) > 0.f) ? da : 0.f;  // ReluGrad: pass where output > 0
  xhat = (z - mu) * rstd;
}

struct BnGrads {
  float* dgamma[2];
  float* dbeta[2];
};

// part: [rb][2][ldz] = (sum dy, sum dy*xhat); bcoef: [2][2][ldz] = (mean dy, mean dy*xhat).
__global__ __launch_bounds__(1024) void k_bn_bwd_stats(const float* __restrict__ Z,
                                                      const float* __restrict__ dA, int ldz,
                                                      int ncol, BnTowers tw,
                                                      const float* __restrict__ coef, BnGrads G,
                                                      float* __restrict__ part,
                                                      unsigned* __restrict__ tickets,
                                                      float* __restrict__ bcoef,
                                                      const float* __restrict__ loss_part, int loss_nblk,
                                                      float* __restrict__ loss_out) {
  __shared__ float s_a[NG][64], s_b[NG][64];
  __shared__ int s_flag;
  if (loss_part && (int)blockIdx.x == (int)gridDim.x - 1) {  // the forward's deferred loss
    if (blockIdx.y == 0) loss_reduce(loss_part, loss_nblk, tw.row_split, loss_out);
    return;
  }
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int rb = blockIdx.y;
  const RowBlocks blk(tw);
  const size_t plane = (size_t)2 * ldz;
  {
    int r0, r1, tower;
    blk.range(tw, rb, r0, r1, tower);
    float zz[RPT], dd[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = r0 + g + NG * i;
      const bool ok = r < r1 && c < ldz;
      zz[i] = ok ? Z[(size_t)r * ldz + c] : 0.f;
      dd[i] = ok ? dA[(size_t)r * ldz + c] : 0.f;
    }
    float s1 = 0.f, s2 = 0.f;
    if (c < ldz) {
      const size_t o = (size_t)tower * ldz + c;
      const float mu = coef[o], rstd = coef[plane + o], inv = coef[2 * plane + o],
                  sh = coef[3 * plane + o];
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        float dy, xh;
        bwd_terms(zz[i], dd[i], mu, rstd, inv, sh, dy, xh);  // dd = 0 on padded rows
        s1 += dy;
        s2 = __fmaf_rn(dy, xh, s2);
      }
    }
    s_a[g][lane] = s1;
    s_b[g][lane] = s2;
    __syncthreads();
    if (g == 0 && c < ldz) {
      float t1 = 0.f, t2 = 0.f;
      for (int k = 0; k < NG; ++k) { t1 += s_a[k][lane]; t2 += s_b[k][lane]; }
      part[((size_t)rb * 2) * ldz + c] = t1;
      part[((size_t)rb * 2 + 1) * ldz + c] = t2;
    }
  }
  if (!last_block_arrival(&tickets[blockIdx.x], (unsigned)gridDim.y, &s_flag)) return;
  for (int tower = 0; tower < 2; ++tower) {
    const int first = tower == 0 ? 0 : blk.nq;
    const int count = tower == 0 ? blk.nq : blk.nd;
    if (count == 0) continue;
    float a = 0.f, b = 0.f;
    if (c < ldz) {
#pragma unroll 4
      for (int k = g; k < count; k += NG) {
        a += part[((size_t)(first + k) * 2) * ldz + c];
        b += part[((size_t)(first + k) * 2 + 1) * ldz + c];
      }
    }
    __syncthreads();
    s_a[g][lane] = a;
    s_b[g][lane] = b;
    __syncthreads();
    if (g == 0 && c < ldz) {
      float s1 = 0.f, s2 = 0.f;
      for (int k = 0; k < NG; ++k) { s1 += s_a[k][lane]; s2 += s_b[k][lane]; }
      const float nrows = (float)(tower == 0 ? tw.row_split : tw.rows - tw.row_split);
      const size_t o = (size_t)tower * ldz + c;
      if (c < ncol) {
        G.dbeta[tower][c] = s1;
        G.dgamma[tower][c] = s2;
        bcoef[o] = s1 / nrows;
        bcoef[plane + o] = s2 / nrows;
      } else {
        bcoef[o] = 0.f;
        bcoef[plane + o] = 0.f;
      }
    }
  }
}

template <typename TO>
__global__ __launch_bounds__(256) void k_bn_bwd_apply(const float* __restrict__ Z,
                                                      const float* __restrict__ dA, int ldz,
                                                      BnTowers tw, const float* __restrict__ coef,
                                                      const float* __restrict__ bcoef,
                                                      TO* __restrict__ dZ) {
  const int q = ldz >> 2;
  const size_t total = (size_t)tw.rows * q;
  const size_t plane = (size_t)2 * ldz;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / q);
    const int c = (int)(i - (size_t)r * q) * 4;
    const int tower = r < tw.row_split ? 0 : 1;
    const size_t o = (size_t)tower * ldz + c;
    const float4 z = *reinterpret_cast<const float4*>(Z + (size_t)r * ldz + c);
    const float4 da = *reinterpret_cast<const float4*>(dA + (size_t)r * ldz + c);
    const float4 mu = *reinterpret_cast<const float4*>(coef + o);
    const float4 rs = *reinterpret_cast<const float4*>(coef + plane + o);
    const float4 inv = *reinterpret_cast<const float4*>(coef + 2 * plane + o);
    const float4 sh = *reinterpret_cast<const float4*>(coef + 3 * plane + o);
    const float4 m1 = *reinterpret_cast<const float4*>(bcoef + o);
    const float4 m2 = *reinterpret_cast<const float4*>(bcoef + plane + o);
    const float zz[4] = {z.x, z.y, z.z, z.w}, dd[4] = {da.x, da.y, da.z, da.w};
    const float mm[4] = {mu.x, mu.y, mu.z, mu.w}, rr[4] = {rs.x, rs.y, rs.z, rs.w};
    const float ii[4] = {inv.x, inv.y, inv.z, inv.w}, ss[4] = {sh.x, sh.y, sh.z, sh.w};
    const float a1[4] = {m1.x, m1.y, m1.z, m1.w}, a2[4] = {m2.x, m2.y, m2.z, m2.w};
    float out[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      out[k] = bn_bwd_dz(zz[k], dd[k], mm[k], rr[k], ii[k], ss[k], a1[k], a2[k]);
    }
    if constexpr (sizeof(TO) == 4) {
      *reinterpret_cast<float4*>((float*)dZ + (size_t)r * ldz + c) = make_float4(out[0], out[1], out[2], out[3]);
    } else {
      uint2 p;
      p.x = pack2bf(out[0], out[1]);
      p.y = pack2bf(out[2], out[3]);
      *reinterpret_cast<uint2*>((u16*)dZ + (size_t)r * ldz + c) = p;
    }
  }
}

// Fused-statistics backward apply (bnfuse.h): the workgroup derives mean(dy), mean(dy*xhat)
// from the layer's fp64 sums into LDS along with the forward coefficients; workgroup 0 also
// writes dbeta / dgamma.  Same arithmetic per element as k_bn_bwd_apply.
constexpr int kApplyMaxLd = 512;
// LDS of the launch: the coefficient cache of the element blocks, or the double-buffered operand
// tiles of the dW blocks (tn.h)
static_assert(kTnTile * 2 >= 128 * kTnLd, "a 128-row sub-chunk per operand");
// TO = u16 (bf16 dZ; hosted dW tiles: tn.h) or float (fp32 parity mode; hosted tiles: g32.h)
template <typename TO>
struct ApplyDw;
template <>
struct ApplyDw<u16> {
  using P = TnParams;
  static constexpr int kFloats = kTnTile * 2;
  __device__ static void run(const P& dw, int r, int dw_x, int dw_y, float* smem) {
    u16* sA = reinterpret_cast<u16*>(smem);
    tn_chunk_body<3>(dw, r % dw_x, (r / dw_x) % dw_y, r / (dw_x * dw_y), sA, sA + 2 * kTnTile);
  }
};
template <>
struct ApplyDw<float> {
  using P = G32Params;
  static constexpr int kFloats = (int)(sizeof(G32Lds) / 4);
  __device__ static void run(const P& dw, int r, int dw_x, int dw_y, float* smem) {
    G32Fuse f{};
    f.tl_slot = -1;
    g32_body<G32_DW, 0, kG32DwSplit / kG32KC>(dw, f, r % dw_x, (r / dw_x) % dw_y, r / (dw_x * dw_y),
                                              *reinterpret_cast<G32Lds*>(smem));
  }
};
template <typename TO>
constexpr int apply_smem_floats() {
  return 2 * 6 * kApplyMaxLd > ApplyDw<TO>::kFloats ? 2 * 6 * kApplyMaxLd : ApplyDw<TO>::kFloats;
}

// The element blocks of the bf16 launch are the critical path once the dW tiles' edge handling is
// cheap (per-workgroup timeline): their loads for kApplyPf grid-stride iterations go out up front,
// and the launch is compiled for 4 waves per SIMD (128 VGPRs, no spill) so all of its workgroups
// (400 dW tiles + 512 element blocks at C2) are resident at once instead of the last ~145 element
// blocks starting ~6 us late.  154.6 vs 155.7 us/step, four alternations.
#ifndef DSSM_APPLY_PF  // grid-stride iterations of an element block whose loads are issued up front
#define DSSM_APPLY_PF 4
#endif
constexpr int kApplyPf = DSSM_APPLY_PF;
#ifndef DSSM_APPLY_WAVES  // waves per SIMD the bf16 apply launch is compiled for (its VGPR budget)
#define DSSM_APPLY_WAVES 4
#endif
#ifdef DSSM_WG_TL
// Diagnostics build only: per-workgroup stamps of the bf16 apply launches, slot 0 = the one hosting
// an N = 128 dW (layer 3's), 1 = the other; [0] start [1] end [2] role (0 dW, 1 second dW set,
// 2 element block, 3 extra block) [3] element blocks: coefficient prologue done
__device__ unsigned long long g_apply_tl[2][2048][4];
#define APPLY_TL(idx, v)                                                                             \
  do {                                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < 2048) g_apply_tl[tl_slot][blockIdx.x][idx] = (v);           \
  } while (0)
#else
#define APPLY_TL(idx, v) \
  do {                   \
  } while (0)
#endif

template <typename TO>
__global__ __launch_bounds__(256, sizeof(TO) == 2 ? DSSM_APPLY_WAVES : 1) void k_bn_bwd_apply_fs(const float* __restrict__ Z,
                                                         const float* __restrict__ dA, BnSide b,
                                                         TO* __restrict__ dZ,
                                                         const float* __restrict__ loss_part,
                                                         int loss_blocks,
                                                         float* __restrict__ loss_out,
                                                         int nwork, typename ApplyDw<TO>::P dw,
                                                         int dw_x, int dw_y, int dw_blocks,
                                                         typename ApplyDw<TO>::P dw2, int dw2_x, int dw2_y,
                                                         int dw2_blocks) {
  __shared__ __attribute__((aligned(16))) float smem[apply_smem_floats<TO>()];
#ifdef DSSM_WG_TL
  const int tl_slot = (sizeof(TO) == 2 && dw_blocks && dw.N == 128) ? 0 : 1;
  const unsigned long long tl0 = __builtin_amdgcn_s_memrealtime();
  auto tl_end = [&](int role) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    APPLY_TL(0, tl0);
    APPLY_TL(1, __builtin_amdgcn_s_memrealtime());
    APPLY_TL(2, (unsigned long long)role);
  };
#else
  auto tl_end = [](int) {};
#endif
  // blocks [0, dw_blocks): the previous backward pair's dW split-K tiles (the longest chains,
  // first in dispatch order), then [dw_blocks, + dw2_blocks) a second pair's (the one before it,
  // when that pair's BN-backward apply was folded into the next pair: BNB_IN_PAIR); they read dZ of
  // the layers above and the forward's activations, so they are independent of this launch's work
  if ((int)blockIdx.x < dw_blocks + dw2_blocks) {
    // XCD-grouped: the tiles of one batch-row chunk share its A / dZ sub-panels through one L2
#ifndef DSSM_XCD_DW_APPLY
#define DSSM_XCD_DW_APPLY 1
#endif
    if ((int)blockIdx.x < dw_blocks) {
      const int r = DSSM_XCD_DW_APPLY ? xcd_tile(blockIdx.x, dw_blocks) : (int)blockIdx.x;
      ApplyDw<TO>::run(dw, r, dw_x, dw_y, smem);
    } else {
      const int b2 = (int)blockIdx.x - dw_blocks;
      const int r = DSSM_XCD_DW_APPLY ? xcd_tile(b2, dw2_blocks) : b2;
      ApplyDw<TO>::run(dw2, r, dw2_x, dw2_y, smem);
    }
    tl_end((int)blockIdx.x < dw_blocks ? 0 : 1);
    return;
  }
  const int bid = (int)blockIdx.x - dw_blocks - dw2_blocks;
  // one extra block past the element blocks: the step's loss / accuracy from the cosine kernel's
  // partials (deferred finalize: no cross-workgroup ticket in the cosine launch) and dgamma /
  // dbeta, off the element blocks' critical path
  if (bid >= nwork) {
    if (loss_part) loss_reduce(loss_part, loss_blocks, b.rows_q, loss_out);
    fs_materialize_bwd(b);
    tl_end(3);
    return;
  }
  float (*sc)[6][kApplyMaxLd] = reinterpret_cast<float (*)[6][kApplyMaxLd]>(smem);  // mu rstd inv shift m1 m2
  const int ld = b.ld;
  const size_t plane = (size_t)2 * ld;
  const int q = ld >> 2;
  const int rows = b.rows_q + b.rows_d;
  const size_t total = (size_t)rows * q;
  // the first kApplyPf grid-stride elements' loads go out before the coefficient prologue (a
  // dependent load per iteration would put one memory latency per iteration on the block)
  const size_t i0 = (size_t)bid * 256 + threadIdx.x, stride = (size_t)nwork * 256;
  float4 zp[kApplyPf], dp[kApplyPf];
#pragma unroll
  for (int u = 0; u < kApplyPf; ++u) {
    const size_t i = i0 + u * stride;
    zp[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    dp[u] = zp[u];
    if (i < total) {
      const int r = (int)(i / q);
      const int c = (int)(i - (size_t)r * q) * 4;
      zp[u] = *reinterpret_cast<const float4*>(Z + (size_t)r * ld + c);
      dp[u] = *reinterpret_cast<const float4*>(dA + (size_t)r * ld + c);
    }
  }
  {  // coefficients of all 2*ld (tower, column) items: every load in flight at once
    constexpr int NPER = 2 * kApplyMaxLd / 256;
    float cf[NPER][4];
    double s1[NPER], s2[NPER];
#pragma unroll
    for (int u = 0; u < NPER; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int ic = i < 2 * ld ? i : 0;
      const int t = ic / ld, c = ic - t * ld;
      const size_t o = (size_t)t * ld + c;
#pragma unroll
      for (int k = 0; k < 4; ++k) cf[u][k] = b.coef[k * plane + o];
      fs_bsums(b, t, c < b.n ? c : 0, s1[u], s2[u]);
    }
#pragma unroll
    for (int u = 0; u < NPER; ++u) {
      const int i = threadIdx.x + 256 * u;
      if (i < 2 * ld) {
        const int t = i / ld, c = i - t * ld;
        const double N = t == 0 ? b.rows_q : b.rows_d;
        const bool ok = c < b.n;
#pragma unroll
        for (int k = 0; k < 4; ++k) sc[t][k][c] = cf[u][k];
        sc[t][4][c] = ok ? (float)(s1[u] / N) : 0.f;
        sc[t][5][c] = ok ? (float)(s2[u] / N) : 0.f;
      }
    }
  }
  __syncthreads();
  APPLY_TL(3, __builtin_amdgcn_s_memrealtime());
  auto element = [&](size_t i, float4 z, float4 da) {
    const int r = (int)(i / q);
    const int c = (int)(i - (size_t)r * q) * 4;
    const int t = r < b.rows_q ? 0 : 1;
    const float zz[4] = {z.x, z.y, z.z, z.w}, dd[4] = {da.x, da.y, da.z, da.w};
    float out[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      out[k] = bn_bwd_dz(zz[k], dd[k], sc[t][0][c + k], sc[t][1][c + k], sc[t][2][c + k], sc[t][3][c + k],
                         sc[t][4][c + k], sc[t][5][c + k]);
    }
    if constexpr (sizeof(TO) == 2) {
      uint2 p;
      p.x = pack2bf(out[0], out[1]);
      p.y = pack2bf(out[2], out[3]);
      *reinterpret_cast<uint2*>(dZ + (size_t)r * ld + c) = p;
    } else {
      *reinterpret_cast<float4*>(dZ + (size_t)r * ld + c) = make_float4(out[0], out[1], out[2], out[3]);
    }
  };
#pragma unroll
  for (int u = 0; u < kApplyPf; ++u)
    if (i0 + u * stride < total) element(i0 + u * stride, zp[u], dp[u]);
  for (size_t i = i0 + kApplyPf * stride; i < total; i += stride) {
    const int r = (int)(i / q);
    const int c = (int)(i - (size_t)r * q) * 4;
    element(i, *reinterpret_cast<const float4*>(Z + (size_t)r * ld + c),
            *reinterpret_cast<const float4*>(dA + (size_t)r * ld + c));
  }
  tl_end(2);
}

int ew_grid(size_t total) {
  size_t g = (total + 255) / 256;
  return (int)(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

}  // namespace

size_t bn_partial_floats(int rows, int ldz, int row_split) {
  BnTowers t{row_split, rows};
  RowBlocks b(t);
  return (size_t)b.total() * 2 * ldz;
}

size_t bn_ticket_count(int ldz) { return (size_t)cdiv(ldz, 64); }

hipError_t launch_bn_fwd_stats(const float* Z, int ldz, int n, BnTowers t, const float* gamma_q,
                               const float* beta_q, const float* gamma_d, const float* beta_d,
                               float* ema_q_mean, float* ema_q_var, float* ema_d_mean,
                               float* ema_d_var, float eps, float decay, bool train,
                               float* batch_mean, float* batch_var, float* partial,
                               unsigned* tickets, float* coef, hipStream_t s, double* zero,
                               int nzero) {
  RowBlocks b(t);
  BnParams P;
  P.gamma[0] = gamma_q; P.gamma[1] = gamma_d;
  P.beta[0] = beta_q; P.beta[1] = beta_d;
  P.ema_mean[0] = ema_q_mean; P.ema_mean[1] = ema_d_mean;
  P.ema_var[0] = ema_q_var; P.ema_var[1] = ema_d_var;
  hipLaunchKernelGGL(k_bn_stats, dim3(cdiv(ldz, 64), train ? b.total() : 1), dim3(1024), 0, s, Z,
                     ldz, n, t, P, eps, decay, train ? 1 : 0, partial, tickets, batch_mean, batch_var,
                     coef, zero, nzero);
  return hipGetLastError();
}

hipError_t launch_bn_apply(const float* Z, int ldz, int n, BnTowers t, const float* coef,
                           bool relu, void* out, bool out_bf16, hipStream_t s) {
  (void)n;
  const int grid = ew_grid((size_t)t.rows * (ldz / 4));
  if (out_bf16)
    hipLaunchKernelGGL(k_bn_apply<u16>, dim3(grid), dim3(256), 0, s, Z, ldz, t, coef,
                       relu ? 1 : 0, (u16*)out);
  else
    hipLaunchKernelGGL(k_bn_apply<float>, dim3(grid), dim3(256), 0, s, Z, ldz, t, coef,
                       relu ? 1 : 0, (float*)out);
  return hipGetLastError();
}

hipError_t launch_bn_bwd(const float* Z, const float* dA, int ldz, int n, BnTowers t,
                         const float* coef, float* dgamma_q, float* dbeta_q, float* dgamma_d,
                         float* dbeta_d, float* partial, unsigned* tickets, float* bcoef,
                         void* dZ, bool dz_bf16, hipStream_t s, const float* loss_part, int loss_nblk,
                         float* loss_out) {
  RowBlocks b(t);
  BnGrads G;
  G.dgamma[0] = dgamma_q; G.dgamma[1] = dgamma_d;
  G.dbeta[0] = dbeta_q; G.dbeta[1] = dbeta_d;
  if (loss_part && (!loss_out || loss_nblk < 1)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bn_bwd_stats, dim3(cdiv(ldz, 64) + (loss_part ? 1 : 0), b.total()), dim3(1024), 0, s, Z,
                     dA, ldz, n, t, coef, G, partial, tickets, bcoef, loss_part, loss_nblk, loss_out);
  const int grid = ew_grid((size_t)t.rows * (ldz / 4));
  if (dz_bf16)
    hipLaunchKernelGGL(k_bn_bwd_apply<u16>, dim3(grid), dim3(256), 0, s, Z, dA, ldz, t, coef,
                       bcoef, (u16*)dZ);
  else
    hipLaunchKernelGGL(k_bn_bwd_apply<float>, dim3(grid), dim3(256), 0, s, Z, dA, ldz, t, coef,
                       bcoef, (float*)dZ);
  return hipGetLastError();
}

hipError_t launch_bn_sums(const float* Z, int ldz, int n, BnTowers t, double* fsum, hipStream_t s,
                          const DetAcc* det) {
  RowBlocks b(t);
  if (det && det->slab && (b.total() > det->cap || cdiv(ldz, 64) > kDetTiles)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bn_sums, dim3(cdiv(ldz, 64), b.total()), dim3(1024), 0, s, Z, ldz, n, t, fsum,
                     det ? *det : DetAcc{});
  return hipGetLastError();
}

template <typename TO>
static hipError_t apply_fused(const float* Z, const float* dA, const BnSide& b, TO* dZ, hipStream_t s,
                              const float* loss_part, int loss_blocks, float* loss_out,
                              const typename ApplyDw<TO>::P* dw, int max_kps,
                              const typename ApplyDw<TO>::P* dw2 = nullptr) {
  if (b.ld > kApplyMaxLd || (b.ld % 4) || (dw2 && !dw)) return hipErrorInvalidValue;
  // element workgroups: fewer beside hosted dW tiles, which share the CUs
#ifndef DSSM_APPLY_GRID_DW
#define DSSM_APPLY_GRID_DW 512
#endif
  const int grid = std::min(ew_grid((size_t)(b.rows_q + b.rows_d) * (b.ld / 4)), dw ? DSSM_APPLY_GRID_DW : 1024);
  if ((dw && dw->k_per_split > max_kps) || (dw2 && dw2->k_per_split > max_kps)) return hipErrorInvalidValue;
  const typename ApplyDw<TO>::P p = dw ? *dw : typename ApplyDw<TO>::P{};
  const typename ApplyDw<TO>::P p2 = dw2 ? *dw2 : typename ApplyDw<TO>::P{};
  const int dw_x = dw ? cdiv(p.N, 64) : 1, dw_y = dw ? cdiv(p.M, 64) : 1;
  const int dw_blocks = dw ? dw_x * dw_y * cdiv(p.K, p.k_per_split) : 0;
  const int dw2_x = dw2 ? cdiv(p2.N, 64) : 1, dw2_y = dw2 ? cdiv(p2.M, 64) : 1;
  const int dw2_blocks = dw2 ? dw2_x * dw2_y * cdiv(p2.K, p2.k_per_split) : 0;
  hipLaunchKernelGGL(k_bn_bwd_apply_fs<TO>, dim3(dw_blocks + dw2_blocks + grid + 1), dim3(256), 0, s, Z, dA, b,
                     dZ, loss_part, loss_blocks, loss_out, grid, p, dw_x, dw_y, dw_blocks, p2, dw2_x, dw2_y,
                     dw2_blocks);
  return hipGetLastError();
}

hipError_t launch_bn_bwd_apply_fused(const float* Z, const float* dA, const BnSide& b, uint16_t* dZ,
                                     hipStream_t s, const float* loss_part, int loss_blocks,
                                     float* loss_out, const TnParams* dw, const TnParams* dw2) {
  return apply_fused<u16>(Z, dA, b, (u16*)dZ, s, loss_part, loss_blocks, loss_out, dw, 3 * 128, dw2);  // tn_chunk_body<3>
}

hipError_t launch_bn_bwd_apply_fused32(const float* Z, const float* dA, const BnSide& b, float* dZ,
                                       hipStream_t s, const float* loss_part, int loss_blocks,
                                       float* loss_out, const G32Params* dw) {
  return apply_fused<float>(Z, dA, b, dZ, s, loss_part, loss_blocks, loss_out, dw, kG32DwSplit);
}

}  // namespace dssm

#ifdef DSSM_WG_TL
extern "C" int dssm_debug_apply_timeline(int slot, unsigned long long* out, int n) {
  if (slot < 0 || slot >= 2 || n > 2048) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dssm::g_apply_tl), sizeof(unsigned long long) * 4 * n,
                             sizeof(unsigned long long) * 4 * 2048 * slot) == hipSuccess ? 0 : -2;
}
#endif
