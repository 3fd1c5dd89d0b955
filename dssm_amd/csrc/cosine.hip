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
// atomics).  The per-block loss/accuracy partials are summed by the last block to finish
// (agent-scope ticket), in fixed order.
#include "common.h"
#include "launch.h"

namespace dssm {
namespace {

constexpr int MAXK = 16;  // NEG + 1 <= 16

__device__ __forceinline__ int doc_row(int j, int k, int bs, int neg) {
  return k == 0 ? bs + j : 2 * bs + j * neg + (k - 1);
}

__device__ void loss_finalize_impl(const float* __restrict__ part, int nblk, int bs,
                                   float* __restrict__ loss_out);
__device__ __forceinline__ void loss_finalize(const float* part, int nblk, int bs, float* out) {
  loss_finalize_impl(part, nblk, bs, out);
}

template <int EPL>
__global__ __launch_bounds__(256) void k_cosine_loss(
    const float* __restrict__ z, int ld, int n, int bs, int neg, float gamma,
    const float* __restrict__ coef, float* __restrict__ y_out, float* __restrict__ cos_raw,
    float* __restrict__ cos_sim, float* __restrict__ prob, float* __restrict__ qnorm,
    float* __restrict__ part, unsigned* __restrict__ ticket, float* __restrict__ loss_out,
    float* __restrict__ dy, int split) {
  __shared__ float s_part[2][4];
  __shared__ int s_flag;
  (void)s_flag;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = blockIdx.x * 4 + wv;
  const int K = neg + 1;
  const size_t plane = (size_t)2 * ld;
  float lj = 0.f, cj = 0.f;
  if (j < bs) {
    // ---- all loads first: query row + K doc rows
    float q[EPL], d[MAXK][EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int c = lane + 64 * e;
      q[e] = (c < n) ? z[(size_t)j * ld + c] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < MAXK; ++k)
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int c = lane + 64 * e;
        d[k][e] = (k < K && c < n) ? z[(size_t)doc_row(j, k, bs, neg) * ld + c] : 0.f;
      }
    if (coef) {  // last layer's BN + ReLU (query tower for q, doc tower for the docs)
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int c = lane + 64 * e;
        if (c < n) {
          q[e] = fmaxf(bn_affine(q[e], coef[2 * plane + c], coef[3 * plane + c]), 0.f);
          const float inv = coef[2 * plane + ld + c], sh = coef[3 * plane + ld + c];
#pragma unroll
          for (int k = 0; k < MAXK; ++k)
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
          for (int k = 0; k < MAXK; ++k)
            if (k < K) y_out[(size_t)doc_row(j, k, bs, neg) * ld + c] = d[k][e];
        }
      }
    }
    float qq = 0.f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) qq = __fmaf_rn(q[e], q[e], qq);
    qq = wave_sum(qq);
    const float qn = sqrtf(qq);
    float cs[MAXK], dn[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
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
        cs[k] = qd / (qn * dn[k]);  // truediv(prod, query_norm*doc_norm); NaN on a zero row, as TF
      }
    }
    // softmax over the K scaled scores (tf.nn.softmax: exp(x - max) / sum)
    float mx = gamma * cs[0];
#pragma unroll
    for (int k = 1; k < MAXK; ++k)
      if (k < K) mx = fmaxf(mx, gamma * cs[k]);
    float ex[MAXK], sum = 0.f;
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
      ex[k] = (k < K) ? expf(gamma * cs[k] - mx) : 0.f;
      sum += ex[k];
    }
    float p[MAXK];
    int amax = 0;
    float pbest = -1.f;
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
      p[k] = ex[k] / sum;
      if (k < K && p[k] > pbest) { pbest = p[k]; amax = k; }
    }
#pragma unroll
    for (int k = 0; k < MAXK; ++k)
      if (k < K && k == lane) {
        cos_raw[(size_t)k * bs + j] = cs[k];
        cos_sim[(size_t)j * K + k] = gamma * cs[k];
        prob[(size_t)j * K + k] = p[k];
      }
    if (lane == 0) qnorm[j] = qn;
    lj = -logf(p[0]);
    cj = (amax == 0) ? 1.f : 0.f;
    // ---- backward: d loss / d cos_sim[j,k] = (p_k - [k==0]) / BS
    float dq[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) dq[e] = 0.f;
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
      if (k < K) {
        const float g = gamma * (p[k] - (k == 0 ? 1.f : 0.f)) / (float)bs;
        const float a = g / (qn * dn[k]);
        const float bq = g * cs[k] / (qn * qn);
        const float bd = g * cs[k] / (dn[k] * dn[k]);
        const size_t row = (size_t)doc_row(j, k, bs, neg) * ld;
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const int c = lane + 64 * e;
          dq[e] += a * d[k][e] - bq * q[e];
          if (c < ld) dy[row + c] = (c < n) ? a * q[e] - bd * d[k][e] : 0.f;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int c = lane + 64 * e;
      if (c < ld) dy[(size_t)j * ld + c] = (c < n) ? dq[e] : 0.f;
    }
  }
  // ---- loss / accuracy: per-block partials, fixed-order sum by the last block
  if (lane == 0) {
    s_part[0][wv] = lj;
    s_part[1][wv] = cj;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s_part[0][0] + s_part[0][1] + s_part[0][2] + s_part[0][3];
    part[2 * blockIdx.x + 1] = s_part[1][0] + s_part[1][1] + s_part[1][2] + s_part[1][3];
  }
  if (split) return;  // k_loss_finalize sums the partials in its own launch
  if (!last_block_arrival(ticket, gridDim.x, &s_flag)) return;
  loss_finalize(part, (int)gridDim.x, bs, loss_out);
}

__global__ __launch_bounds__(64) void k_loss_finalize(const float* __restrict__ part, int nblk,
                                                      int bs, float* __restrict__ loss_out) {
  loss_finalize(part, nblk, bs, loss_out);
}

__device__ void loss_finalize_impl(const float* __restrict__ part, int nblk, int bs,
                                   float* __restrict__ loss_out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (wv == 0) {
    float a = 0.f, b = 0.f;
    for (int i = lane; i < nblk; i += 64) {
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

}  // namespace

size_t cosine_ws_floats(int bs) { return (size_t)2 * cdiv(bs, 4) + 64; }

hipError_t launch_cosine_loss(const float* z, int ld, int n, int bs, int neg, float gamma,
                              const float* coef, float* y_out, float* cos_raw, float* cos_sim,
                              float* prob, float* qnorm, float* ws, float* loss_out, float* dy,
                              bool split, hipStream_t s) {
  if (neg + 1 > MAXK || n > 512) return hipErrorInvalidValue;
  // ws: [partials 2*blocks floats][ticket] (ticket zero on first use; re-armed by the kernel)
  const int blocks = cdiv(bs, 4);
  unsigned* ticket = reinterpret_cast<unsigned*>(ws + 2 * blocks + 32);
  dim3 grid(blocks), block(256);
  const int epl = cdiv(n, 64);
#define DSSM_COS(E)                                                                           \
  hipLaunchKernelGGL(k_cosine_loss<E>, grid, block, 0, s, z, ld, n, bs, neg, gamma, coef, y_out, \
                     cos_raw, cos_sim, prob, qnorm, ws, ticket, loss_out, dy, split ? 1 : 0)
  if (epl <= 1) DSSM_COS(1);
  else if (epl <= 2) DSSM_COS(2);
  else if (epl <= 4) DSSM_COS(4);
  else DSSM_COS(8);
#undef DSSM_COS
  if (split)
    hipLaunchKernelGGL(k_loss_finalize, dim3(1), dim3(64), 0, s, ws, blocks, bs, loss_out);
  return hipGetLastError();
}

}  // namespace dssm
