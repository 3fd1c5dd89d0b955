// batch_normalization + ReLU (new_dssm.py:62-88, :128-136, :150-158) and its backward on gfx950.
//
// Towers: rows [0, row_split) are the query tower, [row_split, rows) the doc tower
// (concat[pos; neg], new_dssm.py:130) — each gets its own moments / gamma / beta / EMA.
// Statistics are deterministic two-level reductions: 64-row blocks (never straddling a tower)
// produce per-column Welford partials (mean, M2), a finalize kernel merges them in a fixed
// order (Chan et al.), so results do not depend on scheduling.  Thread <-> column keeps every
// Z access a coalesced 256-B row segment per wave.
#include "common.h"
#include "launch.h"

namespace dssm {
namespace {

constexpr int RB = 64;  // rows per statistics block

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

__device__ __forceinline__ void chan_merge(float& na, float& ma, float& m2a, float nb, float mb,
                                           float m2b) {
  const float n = na + nb;
  if (nb == 0.f) return;
  const float delta = mb - ma;
  const float f = nb / n;
  ma = ma + delta * f;
  m2a = m2a + m2b + delta * delta * na * f;
  na = n;
}

__global__ __launch_bounds__(256) void k_bn_stats_partial(const float* __restrict__ Z, int ldz,
                                                          BnTowers tw, float* __restrict__ part) {
  __shared__ float sn[4][64], smu[4][64], sm2[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int rb = blockIdx.y;
  RowBlocks blk(tw);
  int r0, r1, tower;
  blk.range(tw, rb, r0, r1, tower);
  float n = 0.f, mean = 0.f, m2 = 0.f;
  if (c < ldz) {
    for (int r = r0 + g; r < r1; r += 4) {
      const float x = Z[(size_t)r * ldz + c];
      n += 1.f;
      const float d = x - mean;
      mean += d / n;
      m2 = __fmaf_rn(d, x - mean, m2);
    }
  }
  sn[g][lane] = n; smu[g][lane] = mean; sm2[g][lane] = m2;
  __syncthreads();
  if (g == 0 && c < ldz) {
    for (int k = 1; k < 4; ++k) chan_merge(n, mean, m2, sn[k][lane], smu[k][lane], sm2[k][lane]);
    part[((size_t)rb * 2 + 0) * ldz + c] = mean;
    part[((size_t)rb * 2 + 1) * ldz + c] = m2;
  }
}

struct BnParams {
  const float* gamma[2];
  const float* beta[2];
  float* ema_mean[2];
  float* ema_var[2];
};

__global__ __launch_bounds__(256) void k_bn_stats_finalize(const float* __restrict__ part, int ldz,
                                                           int ncol, BnTowers tw, BnParams P,
                                                           float eps, float decay, int train,
                                                           float* __restrict__ batch_mean,
                                                           float* __restrict__ batch_var,
                                                           float* __restrict__ coef) {
  __shared__ float sn[4][64], smu[4][64], sm2[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int tower = blockIdx.y;
  RowBlocks blk(tw);
  const int first = tower == 0 ? 0 : blk.nq;
  const int count = tower == 0 ? blk.nq : blk.nd;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  if (train && c < ncol) {
    for (int k = g; k < count; k += 4) {
      const int rb = first + k;
      int r0, r1, tw_;
      blk.range(tw, rb, r0, r1, tw_);
      chan_merge(n, mean, m2, (float)(r1 - r0), part[((size_t)rb * 2) * ldz + c],
                 part[((size_t)rb * 2 + 1) * ldz + c]);
    }
  }
  sn[g][lane] = n; smu[g][lane] = mean; sm2[g][lane] = m2;
  __syncthreads();
  if (g != 0 || c >= ldz) return;
  float* co = coef;  // [4][2][ldz]
  const size_t o = (size_t)tower * ldz + c;
  const size_t plane = (size_t)2 * ldz;
  if (c >= ncol) {
    co[o] = 0.f; co[plane + o] = 0.f; co[2 * plane + o] = 0.f; co[3 * plane + o] = 0.f;
    return;
  }
  float mu, var;
  if (train) {
    for (int k = 1; k < 4; ++k) chan_merge(n, mean, m2, sn[k][lane], smu[k][lane], sm2[k][lane]);
    mu = mean;
    var = m2 / n;  // biased (tf.nn.moments)
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
  const float inv = rstd * P.gamma[tower][c];
  co[o] = mu;
  co[plane + o] = rstd;
  co[2 * plane + o] = inv;
  co[3 * plane + o] = P.beta[tower][c] - mu * inv;
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
      p.x = (unsigned)f2bf(y[0]) | ((unsigned)f2bf(y[1]) << 16);
      p.y = (unsigned)f2bf(y[2]) | ((unsigned)f2bf(y[3]) << 16);
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

__global__ __launch_bounds__(256) void k_bn_bwd_partial(const float* __restrict__ Z,
                                                        const float* __restrict__ dA, int ldz,
                                                        BnTowers tw, const float* __restrict__ coef,
                                                        float* __restrict__ part) {
  __shared__ float s1s[4][64], s2s[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int rb = blockIdx.y;
  RowBlocks blk(tw);
  int r0, r1, tower;
  blk.range(tw, rb, r0, r1, tower);
  float s1 = 0.f, s2 = 0.f;
  if (c < ldz) {
    const size_t plane = (size_t)2 * ldz, o = (size_t)tower * ldz + c;
    const float mu = coef[o], rstd = coef[plane + o], inv = coef[2 * plane + o],
                sh = coef[3 * plane + o];
    for (int r = r0 + g; r < r1; r += 4) {
      float dy, xh;
      bwd_terms(Z[(size_t)r * ldz + c], dA[(size_t)r * ldz + c], mu, rstd, inv, sh, dy, xh);
      s1 += dy;
      s2 = __fmaf_rn(dy, xh, s2);
    }
  }
  s1s[g][lane] = s1; s2s[g][lane] = s2;
  __syncthreads();
  if (g == 0 && c < ldz) {
    for (int k = 1; k < 4; ++k) { s1 += s1s[k][lane]; s2 += s2s[k][lane]; }
    part[((size_t)rb * 2 + 0) * ldz + c] = s1;
    part[((size_t)rb * 2 + 1) * ldz + c] = s2;
  }
}

struct BnGrads {
  float* dgamma[2];
  float* dbeta[2];
};

__global__ __launch_bounds__(256) void k_bn_bwd_finalize(const float* __restrict__ part, int ldz,
                                                         int ncol, BnTowers tw, BnGrads G,
                                                         float* __restrict__ bcoef) {
  __shared__ float s1s[4][64], s2s[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int tower = blockIdx.y;
  RowBlocks blk(tw);
  const int first = tower == 0 ? 0 : blk.nq;
  const int count = tower == 0 ? blk.nq : blk.nd;
  float s1 = 0.f, s2 = 0.f;
  if (c < ldz) {
    for (int k = g; k < count; k += 4) {
      s1 += part[((size_t)(first + k) * 2) * ldz + c];
      s2 += part[((size_t)(first + k) * 2 + 1) * ldz + c];
    }
  }
  s1s[g][lane] = s1; s2s[g][lane] = s2;
  __syncthreads();
  if (g != 0 || c >= ldz) return;
  for (int k = 1; k < 4; ++k) { s1 += s1s[k][lane]; s2 += s2s[k][lane]; }
  const float nrows = (float)(tower == 0 ? tw.row_split : tw.rows - tw.row_split);
  const size_t o = (size_t)tower * ldz + c;
  if (c < ncol) {
    G.dbeta[tower][c] = s1;
    G.dgamma[tower][c] = s2;
    bcoef[o] = s1 / nrows;
    bcoef[(size_t)2 * ldz + o] = s2 / nrows;
  } else {
    bcoef[o] = 0.f;
    bcoef[(size_t)2 * ldz + o] = 0.f;
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
      float dy, xh;
      bwd_terms(zz[k], dd[k], mm[k], rr[k], ii[k], ss[k], dy, xh);
      out[k] = ii[k] * (dy - a1[k] - xh * a2[k]);
    }
    if constexpr (sizeof(TO) == 4) {
      *reinterpret_cast<float4*>((float*)dZ + (size_t)r * ldz + c) = make_float4(out[0], out[1], out[2], out[3]);
    } else {
      uint2 p;
      p.x = (unsigned)f2bf(out[0]) | ((unsigned)f2bf(out[1]) << 16);
      p.y = (unsigned)f2bf(out[2]) | ((unsigned)f2bf(out[3]) << 16);
      *reinterpret_cast<uint2*>((u16*)dZ + (size_t)r * ldz + c) = p;
    }
  }
}

int ew_grid(size_t total) {
  size_t g = (total + 255) / 256;
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

}  // namespace

size_t bn_partial_floats(int rows, int ldz, int row_split) {
  BnTowers t{row_split, rows};
  RowBlocks b(t);
  return (size_t)b.total() * 2 * ldz;
}

hipError_t launch_bn_fwd_stats(const float* Z, int ldz, int n, BnTowers t, const float* gamma_q,
                               const float* beta_q, const float* gamma_d, const float* beta_d,
                               float* ema_q_mean, float* ema_q_var, float* ema_d_mean,
                               float* ema_d_var, float eps, float decay, bool train,
                               float* batch_mean, float* batch_var, float* partial, float* coef,
                               hipStream_t s) {
  RowBlocks b(t);
  if (train)
    hipLaunchKernelGGL(k_bn_stats_partial, dim3(cdiv(ldz, 64), b.total()), dim3(256), 0, s, Z,
                       ldz, t, partial);
  BnParams P;
  P.gamma[0] = gamma_q; P.gamma[1] = gamma_d;
  P.beta[0] = beta_q; P.beta[1] = beta_d;
  P.ema_mean[0] = ema_q_mean; P.ema_mean[1] = ema_d_mean;
  P.ema_var[0] = ema_q_var; P.ema_var[1] = ema_d_var;
  const int ntowers = t.row_split < t.rows ? 2 : 1;
  hipLaunchKernelGGL(k_bn_stats_finalize, dim3(cdiv(ldz, 64), ntowers), dim3(256), 0, s, partial, ldz,
                     n, t, P, eps, decay, train ? 1 : 0, batch_mean, batch_var, coef);
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
                         float* dbeta_d, float* partial, float* bcoef, void* dZ, bool dz_bf16,
                         hipStream_t s) {
  RowBlocks b(t);
  hipLaunchKernelGGL(k_bn_bwd_partial, dim3(cdiv(ldz, 64), b.total()), dim3(256), 0, s, Z, dA,
                     ldz, t, coef, partial);
  BnGrads G;
  G.dgamma[0] = dgamma_q; G.dgamma[1] = dgamma_d;
  G.dbeta[0] = dbeta_q; G.dbeta[1] = dbeta_d;
  const int ntowers = t.row_split < t.rows ? 2 : 1;
  hipLaunchKernelGGL(k_bn_bwd_finalize, dim3(cdiv(ldz, 64), ntowers), dim3(256), 0, s, partial, ldz, n,
                     t, G, bcoef);
  const int grid = ew_grid((size_t)t.rows * (ldz / 4));
  if (dz_bf16)
    hipLaunchKernelGGL(k_bn_bwd_apply<u16>, dim3(grid), dim3(256), 0, s, Z, dA, ldz, t, coef,
                       bcoef, (u16*)dZ);
  else
    hipLaunchKernelGGL(k_bn_bwd_apply<float>, dim3(grid), dim3(256), 0, s, Z, dA, ldz, t, coef,
                       bcoef, (float*)dZ);
  return hipGetLastError();
}

}  // namespace dssm
