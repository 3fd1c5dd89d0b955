// Merge_Negative_Doc + Cosine_Similarity + softmax Loss (new_dssm.py:160-213) fused with their
// backward, one wave per query on gfx950.
//
// The reference builds the merged doc matrix with BS*NEG tf.concat ops (new_dssm.py:169-179);
// here the merge is index arithmetic: doc (j, k) is row BS+j for k = 0 and row
// 2*BS + j*NEG + k-1 otherwise.  A wave loads its query row and all NEG+1 doc rows at once
// (lane owns columns lane, lane+64, ...; EPL per lane, register resident), applies the last
// layer's BN+ReLU on the fly when given the pre-BN activations (and writes the embeddings out),
// computes norms/dots by wave reductions, softmax/loss redundantly in every lane, and writes the
// gradient of every embedding row it owns (each doc row belongs to exactly one query: no
// atomics).  The per-block loss/accuracy partials are summed in fixed order by a later launch
// (the backward's first, or k_loss_finalize).
#include <algorithm>
#include <type_traits>

#include "bnfuse.h"

#include "common.h"
#include "launch.h"
#include "csc.h"

namespace dssm {
namespace {

constexpr int MAXK = 16;  // NEG + 1 <= 16

__device__ __forceinline__ int doc_row(int j, int k, int bs, int neg) {
  return k == 0 ? bs + j : 2 * bs + j * neg + (k - 1);
}

__device__ __forceinline__ void loss_finalize(const float* part, int nblk, int bs, float* out) {
  loss_reduce(part, nblk, bs, out);
}

// KM: register rows per query (NEG + 1 <= KM).  FSC (fused statistics, bnfuse.h): the last
// layer's coefficients come from its forward sums (workgroup 0 materialises them, the batch
// moments and the EMA update) and the workgroup adds its rows' backward sums (sum dy,
// sum dy*xhat per tower, ReLU mask applied) to fs.bsum.
constexpr int kCosMaxN = 512;
#ifndef DSSM_COS_LANEPAR  // the per-doc scalar math one doc per lane (0: every lane computes every doc's)
#define DSSM_COS_LANEPAR 1
#endif
#ifndef DSSM_COS_DPP  // the rows' norm / dot butterflies on DPP and row swaps (0: ds_bpermute shuffles)
#define DSSM_COS_DPP 1
#endif
// NW: waves (queries) per workgroup.  The fused kernel uses 16: each workgroup adds its backward
// sums with one fp64 atomic per (statistic, column), and the 64-deep same-address chains (instead
// of 256-deep at 4 waves) no longer trail the launch.
#ifdef DSSM_WG_TL
// Diagnostics build only: per-workgroup start / end stamps of the fused cosine launch (its query
// blocks, the materialising block, the CSC scatter blocks), read by dssm_debug_cos_timeline
__device__ unsigned long long g_cos_tl[1024][8];  // 0 start 1 end, 2..6 phases (query blocks)
#define COS_TL(idx)                                                                               \
  do {                                                                                            \
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_cos_tl[blockIdx.x][idx] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define COS_TL(idx) \
  do {              \
  } while (0)
#endif
// MAP: the merged row r of [q; pos; neg] is read from z row rmap[r] (the multi-view model's in-batch
// rotation as an index map instead of a gathered copy); dy stays in the merged layout.
__device__ __forceinline__ bool drop_kept(const CosDrop& d, int r, int c) {
  return d.all || dropout_hash((unsigned)(r * d.cols + c), d.seed, d.step) < d.thr;
}

// DROP: inverted dropout on the rows (CosDrop), fused (the unfused, unmapped form only).
template <int EPL, int KM, bool FSC, int NW, bool MAP = false, bool DROP = false>
__global__ __launch_bounds__(64 * NW) void k_cosine_loss(
    const float* __restrict__ z, int ld, int n, int bs, int neg, float gamma,
    const float* __restrict__ coef, float* __restrict__ y_out, float* __restrict__ cos_raw,
    float* __restrict__ cos_sim, float* __restrict__ prob, float* __restrict__ qnorm,
    float* __restrict__ part, float* __restrict__ dy, BnSide fs, CscScatter scat,
    const int* __restrict__ rmap, float* __restrict__ loss_out, CosDrop drop) {
  constexpr int NT = 64 * NW;
  COS_TL(0);
  __shared__ float s_part[2][NW];
  __shared__ float s_co[FSC ? 2 * 4 * kCosMaxN : 1];     // [tower][mu|rstd|inv|shift][c]
  __shared__ float s_bs[FSC ? NW * 4 * EPL * 64 : 1];    // [wave][sq1|sq2|sd1|sd2][c]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = blockIdx.x * NW + wv;
  const int K = neg + 1;
  const size_t plane = (size_t)2 * ld;
  const int nrow_blocks = (bs + NW - 1) / NW;
  // ---- the rows' raw loads go out first, ahead of the coefficient prologue (they need no
  // coefficient): query row + K doc rows
  float q[EPL], d[KM][EPL], zq[EPL], zd[FSC ? KM : 1][EPL];
  if (j < bs && (int)blockIdx.x < nrow_blocks) {
    int src[1 + KM];  // the source rows (MAP: wave-uniform map reads)
    src[0] = MAP ? rmap[j] : j;
#pragma unroll
    for (int k = 0; k < KM; ++k) src[1 + k] = k < K ? (MAP ? rmap[doc_row(j, k, bs, neg)] : doc_row(j, k, bs, neg)) : 0;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int c = lane + 64 * e;
      q[e] = (c < n) ? z[(size_t)src[0] * ld + c] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < KM; ++k)
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int c = lane + 64 * e;
        d[k][e] = (k < K && c < n) ? z[(size_t)src[1 + k] * ld + c] : 0.f;
      }
  }
  if constexpr (!FSC) {
    if ((int)blockIdx.x >= nrow_blocks) {  // fp32 parity mode: the CSC transpose's scatter (csc.h)
      csc_scatter_role(scat, (int)blockIdx.x - nrow_blocks);
      return;
    }
  }
  if constexpr (FSC) {
    if ((int)blockIdx.x >= nrow_blocks) {  // the extra block: BN_L's coefficients, moments, EMA
      const int xb = (int)blockIdx.x - nrow_blocks - 1;
      if (xb < 0) fs_materialize_fwd(fs);
      else csc_scatter_role(scat, xb);  // the CSC transpose's scatter (csc.h)
#ifdef DSSM_WG_TL
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      COS_TL(1);
#endif
      return;
    }
#ifdef DSSM_WG_TL
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    COS_TL(2);
#endif
    fs_coef_stage<(2 * kCosMaxN + NT - 1) / NT>(fs, threadIdx.x, NT,
                                          [&](int t, int c, float mu, float rs, float inv, float sh) {
      s_co[(t * 4 + 0) * kCosMaxN + c] = mu;
      s_co[(t * 4 + 1) * kCosMaxN + c] = rs;
      s_co[(t * 4 + 2) * kCosMaxN + c] = inv;
      s_co[(t * 4 + 3) * kCosMaxN + c] = sh;
    });
    __syncthreads();
  }
  COS_TL(3);
  float lj = 0.f, cj = 0.f;
  float bq1[EPL], bq2[EPL], bd1[EPL], bd2[EPL];  // FSC: this wave's backward sums per column
#pragma unroll
  for (int e = 0; e < EPL; ++e) bq1[e] = bq2[e] = bd1[e] = bd2[e] = 0.f;
  if (j < bs) {
    if constexpr (FSC) {
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        zq[e] = q[e];
#pragma unroll
        for (int k = 0; k < KM; ++k) zd[k][e] = d[k][e];
      }
    }
    if constexpr (DROP) {  // x * m / keep (k_dropout's arithmetic)
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int c = lane + 64 * e;
        if (c < n) {
          q[e] = drop_kept(drop, j, c) ? q[e] * drop.fwd : 0.f;
#pragma unroll
          for (int k = 0; k < KM; ++k)
            if (k < K) d[k][e] = drop_kept(drop, doc_row(j, k, bs, neg), c) ? d[k][e] * drop.fwd : 0.f;
        }
      }
    }
    if (coef || FSC) {  // last layer's BN + ReLU (query tower for q, doc tower for the docs)
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int c = lane + 64 * e;
        if (c < n) {
          const float iq = FSC ? s_co[2 * kCosMaxN + c] : coef[2 * plane + c];
          const float sq = FSC ? s_co[3 * kCosMaxN + c] : coef[3 * plane + c];
          q[e] = fmaxf(bn_affine(q[e], iq, sq), 0.f);
          const float inv = FSC ? s_co[6 * kCosMaxN + c] : coef[2 * plane + ld + c];
          const float sh = FSC ? s_co[7 * kCosMaxN + c] : coef[3 * plane + ld + c];
#pragma unroll
          for (int k = 0; k < KM; ++k)
            if (k < K) d[k][e] = fmaxf(bn_affine(d[k][e], inv, sh), 0.f);
        }
      }
    }
    if (y_out) {
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int c = lane + 64 * e;
        if (c < ld) {
          y_out[(size_t)j * ld + c] = q[e];
#pragma unroll
          for (int k = 0; k < KM; ++k)
            if (k < K) y_out[(size_t)doc_row(j, k, bs, neg) * ld + c] = d[k][e];
        }
      }
    }
    // all 1 + 2*KM lane partials first, then one interleaved butterfly (same order per value as
    // wave_sum: the shuffles of the independent sums overlap instead of chaining)
    float red[1 + 2 * KM];
    red[0] = 0.f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) red[0] = __fmaf_rn(q[e], q[e], red[0]);
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      float dd = 0.f, qd = 0.f;
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        dd = __fmaf_rn(d[k][e], d[k][e], dd);
        qd = __fmaf_rn(q[e], d[k][e], qd);
      }
      red[1 + 2 * k] = dd;
      red[2 + 2 * k] = qd;
    }
#if DSSM_COS_DPP
    auto stage = [&](auto st) {
#pragma unroll
      for (int i = 0; i < 1 + 2 * KM; ++i) red[i] = wave_allsum_step<decltype(st)::value>(red[i]);
    };
    stage(std::integral_constant<int, 0>{});
    stage(std::integral_constant<int, 1>{});
    stage(std::integral_constant<int, 2>{});
    stage(std::integral_constant<int, 3>{});
    stage(std::integral_constant<int, 4>{});
    stage(std::integral_constant<int, 5>{});
#else
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
      for (int i = 0; i < 1 + 2 * KM; ++i) red[i] += __shfl_xor(red[i], o);
#endif
    const float qn = sqrtf(red[0]);
    float cs[KM], dn[KM], p[KM];
    int amax = 0;
    float pbest = -1.f;
#if DSSM_COS_LANEPAR
    // The per-doc scalars (norms, cosines, softmax, gradient coefficients) are wave-uniform: lane k
    // computes doc k's, each an IEEE sqrt / exp / division of the same operands as the serial form,
    // and v_readlane hands them to the wave (one division sequence per stage instead of one per doc)
    auto bcast = [](float v, int k) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k)); };
    float my_dn = 1.f, my_cs = 0.f;
    {
      float dd = 0.f, qd = 0.f;
#pragma unroll
      for (int k = 0; k < KM; ++k)
        if (lane == k) {
          dd = red[1 + 2 * k];
          qd = red[2 + 2 * k];
        }
      if (lane < K) {
        my_dn = sqrtf(dd);
        my_cs = qd / (qn * my_dn);  // truediv(prod, query_norm*doc_norm); NaN on a zero row, as TF
      }
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      cs[k] = k < K ? bcast(my_cs, k) : 0.f;
      dn[k] = k < K ? bcast(my_dn, k) : 1.f;
    }
    // softmax over the K scaled scores (tf.nn.softmax: exp(x - max) / sum)
    float mx = gamma * cs[0];
#pragma unroll
    for (int k = 1; k < KM; ++k)
      if (k < K) mx = fmaxf(mx, gamma * cs[k]);
    const float my_ex = lane < K ? expf(gamma * my_cs - mx) : 0.f;
    float ex[KM], sum = 0.f;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      ex[k] = k < K ? bcast(my_ex, k) : 0.f;
      sum += ex[k];
    }
    const float my_p = my_ex / sum;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      p[k] = bcast(my_p, k);
      if (k < K && p[k] > pbest) { pbest = p[k]; amax = k; }
    }
#else
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      cs[k] = 0.f;
      dn[k] = 1.f;
      if (k < K) {
        dn[k] = sqrtf(red[1 + 2 * k]);
        cs[k] = red[2 + 2 * k] / (qn * dn[k]);  // truediv(prod, query_norm*doc_norm); NaN on a zero row, as TF
      }
    }
    // softmax over the K scaled scores (tf.nn.softmax: exp(x - max) / sum)
    float mx = gamma * cs[0];
#pragma unroll
    for (int k = 1; k < KM; ++k)
      if (k < K) mx = fmaxf(mx, gamma * cs[k]);
    float ex[KM], sum = 0.f;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      ex[k] = (k < K) ? expf(gamma * cs[k] - mx) : 0.f;
      sum += ex[k];
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      p[k] = ex[k] / sum;
      if (k < K && p[k] > pbest) { pbest = p[k]; amax = k; }
    }
#endif
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (k < K && k == lane) {
        cos_raw[(size_t)k * bs + j] = cs[k];
        cos_sim[(size_t)j * K + k] = gamma * cs[k];
        prob[(size_t)j * K + k] = p[k];
      }
    if (lane == 0) qnorm[j] = qn;
    lj = -logf(p[0]);
    cj = (amax == 0) ? 1.f : 0.f;
    COS_TL(4);
    // ---- backward: d loss / d cos_sim[j,k] = (p_k - [k==0]) / BS (skipped without dy: eval)
    if (FSC || dy != nullptr) {
    float dq[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) dq[e] = 0.f;
#if DSSM_COS_LANEPAR
    float my_a = 0.f, my_bq = 0.f, my_bd = 0.f;
    if (lane < K) {
      const float g = gamma * (my_p - (lane == 0 ? 1.f : 0.f)) / (float)bs;
      my_a = g / (qn * my_dn);
      my_bq = g * my_cs / (qn * qn);
      my_bd = g * my_cs / (my_dn * my_dn);
    }
#endif
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k < K) {
#if DSSM_COS_LANEPAR
        const float a = bcast(my_a, k), bq = bcast(my_bq, k), bd = bcast(my_bd, k);
#else
        const float g = gamma * (p[k] - (k == 0 ? 1.f : 0.f)) / (float)bs;
        const float a = g / (qn * dn[k]);
        const float bq = g * cs[k] / (qn * qn);
        const float bd = g * cs[k] / (dn[k] * dn[k]);
#endif
        const size_t row = (size_t)doc_row(j, k, bs, neg) * ld;
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const int c = lane + 64 * e;
          // explicit FMAs: one rounding sequence in every instantiation (the contraction the
          // compiler picks otherwise differs between them)
          dq[e] += __fmaf_rn(a, d[k][e], -(bq * q[e]));
          const float gd = (c < n) ? __fmaf_rn(a, q[e], -(bd * d[k][e])) : 0.f;
          if constexpr (DROP) {  // d loss / d x through the same mask
            if (c < ld) dy[row + c] = (c < n && drop_kept(drop, doc_row(j, k, bs, neg), c)) ? gd * drop.bwd : 0.f;
          } else {
            if (c < ld) dy[row + c] = gd;
          }
          if constexpr (FSC) {
            if (c < n) {
              const float m = d[k][e] > 0.f ? gd : 0.f;  // ReluGrad on the doc row
              bd1[e] += m;
              bd2[e] = __fmaf_rn(m, (zd[k][e] - s_co[4 * kCosMaxN + c]) * s_co[5 * kCosMaxN + c], bd2[e]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int c = lane + 64 * e;
      if constexpr (DROP) {
        if (c < ld) dy[(size_t)j * ld + c] = (c < n && drop_kept(drop, j, c)) ? dq[e] * drop.bwd : 0.f;
      } else {
        if (c < ld) dy[(size_t)j * ld + c] = (c < n) ? dq[e] : 0.f;
      }
      if constexpr (FSC) {
        if (c < n) {
          const float m = q[e] > 0.f ? dq[e] : 0.f;
          bq1[e] = m;
          bq2[e] = m * ((zq[e] - s_co[c]) * s_co[kCosMaxN + c]);
        }
      }
    }
    }  // backward
  }
  COS_TL(5);
  if constexpr (FSC) {
    // workgroup sums of the NW waves (fp64) -> the layer's backward accumulators
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int c = lane + 64 * e;
      s_bs[(wv * 4 + 0) * EPL * 64 + c] = bq1[e];
      s_bs[(wv * 4 + 1) * EPL * 64 + c] = bq2[e];
      s_bs[(wv * 4 + 2) * EPL * 64 + c] = bd1[e];
      s_bs[(wv * 4 + 3) * EPL * 64 + c] = bd2[e];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * n; i += NT) {
      const int st = i / n, c = i - st * n;  // st: q-sum, q-sum*xhat, d-sum, d-sum*xhat
      double acc = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) acc += s_bs[(w * 4 + st) * EPL * 64 + c];
      if (fs.bdet.slab)  // deterministic: this workgroup's slab row (both towers: [tower * 2 + stat])
        det_st(fs.bdet.slab + ((size_t)blockIdx.x * 4 + st) * ld + c, acc);
      else
        atomic_add_f64(fs.bsum + (size_t)st * ld + c, acc);
    }
    if (fs.bdet.slab) {
      __shared__ int s_last;
      det_publish(fs.bdet, 0, blockIdx.x, nrow_blocks, ld, 0, n, fs.bsum, &s_last);
    }
  }
  COS_TL(6);
  // ---- loss / accuracy: per-block partials, fixed-order sum by the last block
  if (lane == 0) {
    s_part[0][wv] = lj;
    s_part[1][wv] = cj;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      a += s_part[0][w];
      b += s_part[1][w];
    }
    // (an in-kernel finalize by the last workgroup behind a ticket measured slower on the multi-view
    // and RNN steps in round 4 and was removed; the partials are summed by a later launch)
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = b;
  }
#ifdef DSSM_WG_TL
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  COS_TL(1);
#endif
}

__global__ __launch_bounds__(64) void k_loss_finalize(const float* __restrict__ part, int nblk,
                                                      int bs, float* __restrict__ loss_out) {
  loss_finalize(part, nblk, bs, loss_out);
}

}  // namespace

size_t cosine_ws_floats(int bs) { return (size_t)2 * cdiv(bs, 4) + 64; }

hipError_t launch_cosine_loss(const float* z, int ld, int n, int bs, int neg, float gamma,
                              const float* coef, float* y_out, float* cos_raw, float* cos_sim,
                              float* prob, float* qnorm, float* ws, float* loss_out, float* dy,
                              hipStream_t s, const BnSide* fused, bool defer_finalize,
                              const CscScatter* scatter, const int* rmap, const CosDrop* drop) {
  if (neg + 1 > MAXK || n > kCosMaxN || (rmap && (fused || coef || y_out))) return hipErrorInvalidValue;
  const CosDrop dr = drop ? *drop : CosDrop{};
  if (dr.on && (fused || rmap || coef || scatter)) return hipErrorInvalidValue;  // the plain form only
  // ws: the per-workgroup loss / accuracy partials (2 floats each)
  const int nw = cosine_waves(n, fused != nullptr);
  const int blocks = cosine_blocks(bs, n, fused != nullptr);
  CscScatter sc = scatter ? *scatter : CscScatter{};
  if (sc.nblocks) sc.nblocks = std::max(1, sc.nblocks * 4 / nw);  // sized in 4-wave workgroups
  if (scatter && rmap) return hipErrorInvalidValue;  // the mapped form
  // fused: + materialising and scatter blocks
  dim3 grid(blocks + (fused ? 1 : 0) + sc.nblocks), block(64 * nw);
  const int epl = cdiv(n, 64);
  const BnSide fs = fused ? *fused : BnSide{};
  if (fs.bdet.slab && (cdiv(bs, nw) > fs.bdet.cap || ld > 64 * kDetTiles)) return hipErrorInvalidValue;
  // The loss partials are summed by a later launch (deferred: the caller's next one; else a tiny
  // launch here).
#define DSSM_COS3(E, KM, F)                                                                     \
  if (nw == kCosFusedWaves)                                                                     \
    hipLaunchKernelGGL((k_cosine_loss<E, KM, F, kCosFusedWaves>), grid, block, 0, s, z, ld, n, bs, neg, \
                       gamma, coef, y_out, cos_raw, cos_sim, prob, qnorm, ws, dy, fs, sc, nullptr, loss_out, dr); \
  else if (rmap)                                                                                \
    hipLaunchKernelGGL((k_cosine_loss<E, KM, false, 4, true>), grid, block, 0, s, z, ld, n, bs, neg, gamma, \
                       coef, y_out, cos_raw, cos_sim, prob, qnorm, ws, dy, fs, sc, rmap, loss_out, dr); \
  else if (dr.on)                                                                               \
    hipLaunchKernelGGL((k_cosine_loss<E, KM, false, 4, false, true>), grid, block, 0, s, z, ld, n, bs, neg, \
                       gamma, coef, y_out, cos_raw, cos_sim, prob, qnorm, ws, dy, fs, sc, nullptr, loss_out, \
                       dr);                                                                \
  else                                                                                          \
    hipLaunchKernelGGL((k_cosine_loss<E, KM, F, 4>), grid, block, 0, s, z, ld, n, bs, neg, gamma,    \
                       coef, y_out, cos_raw, cos_sim, prob, qnorm, ws, dy, fs, sc, nullptr, loss_out, dr)
#define DSSM_COS2(E, KM) \
  if (fused) DSSM_COS3(E, KM, true); else DSSM_COS3(E, KM, false)
#define DSSM_COS(E) \
  if (neg + 1 == 5) { DSSM_COS2(E, 5); } else if (neg + 1 <= 8) { DSSM_COS2(E, 8); } else { DSSM_COS2(E, 16); }
  if (epl <= 1) { DSSM_COS(1) }
  else if (epl <= 2) { DSSM_COS(2) }
  else if (epl <= 4) { DSSM_COS(4) }
  else { DSSM_COS(8) }
#undef DSSM_COS
#undef DSSM_COS2
#undef DSSM_COS3
  if (!defer_finalize)
    hipLaunchKernelGGL(k_loss_finalize, dim3(1), dim3(64), 0, s, ws, blocks, bs, loss_out);
  return hipGetLastError();
}

hipError_t launch_loss_finalize(const float* ws, int bs, int n, float* loss_out, hipStream_t s, bool fused) {
  // only after a forward that deferred its loss (the partials of a fused / unfused cosine launch)
  hipLaunchKernelGGL(k_loss_finalize, dim3(1), dim3(64), 0, s, ws, cosine_blocks(bs, n, fused), bs, loss_out);
  return hipGetLastError();
}

}  // namespace dssm

#ifdef DSSM_WG_TL
extern "C" int dssm_debug_cos_timeline(unsigned long long* out, int n) {
  if (n > 1024) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dssm::g_cos_tl), sizeof(unsigned long long) * 8 * n, 0) == hipSuccess
             ? 0 : -2;
}
#endif
