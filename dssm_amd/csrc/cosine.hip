// Merge_Negative_Doc + Cosine_Similarity + softmax Loss (new_dssm.py:160-213) fused with their
// backward, one wave per query on gfx950.
//
// The reference builds the merged doc matrix with BS*NEG tf.concat ops (new_dssm.py:169-179);
// here the merge is index arithmetic: doc (j, k) is row BS+j for k = 0 and row
// 2*BS + j*NEG + k-1 otherwise.  Norms and dots are wave reductions over the embedding width
// (lane owns columns lane, lane+64, ...), softmax/loss are computed redundantly by every lane,
// and the gradient w.r.t. every embedding row is written by the wave that owns its query (each
// doc row belongs to exactly one query, so no atomics).
#include "common.h"
#include "launch.h"

namespace dssm {
namespace {

constexpr int MAXK = 16;  // NEG + 1 <= 16
constexpr int MAXE = 8;   // embedding width <= 512

__device__ __forceinline__ int doc_row(int j, int k, int bs, int neg) {
  return k == 0 ? bs + j : 2 * bs + j * neg + (k - 1);
}

__global__ __launch_bounds__(256) void k_cosine_loss(const float* __restrict__ y, int ld, int n,
                                                     int bs, int neg, float gamma,
                                                     float* __restrict__ cos_raw,
                                                     float* __restrict__ cos_sim,
                                                     float* __restrict__ prob,
                                                     float* __restrict__ qnorm,
                                                     float* __restrict__ loss_j,
                                                     float* __restrict__ correct_j,
                                                     float* __restrict__ dy) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= bs) return;
  const int K = neg + 1;
  float q[MAXE];
  float qq = 0.f;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int c = lane + 64 * e;
    q[e] = (c < n) ? y[(size_t)j * ld + c] : 0.f;
    qq = __fmaf_rn(q[e], q[e], qq);
  }
  qq = wave_sum(qq);
  const float qn = sqrtf(qq);
  float cs[MAXK], dn[MAXK];
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    cs[k] = 0.f;
    dn[k] = 1.f;
    if (k < K) {
      const float* d = y + (size_t)doc_row(j, k, bs, neg) * ld;
      float dd = 0.f, qd = 0.f;
#pragma unroll
      for (int e = 0; e < MAXE; ++e) {
        const int c = lane + 64 * e;
        const float x = (c < n) ? d[c] : 0.f;
        dd = __fmaf_rn(x, x, dd);
        qd = __fmaf_rn(q[e], x, qd);
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
  if (lane < K) {
    // each of the first K lanes writes one k (registers indexed with a compile-time k)
#pragma unroll
    for (int k = 0; k < MAXK; ++k)
      if (k == lane) {
        cos_raw[(size_t)k * bs + j] = cs[k];
        cos_sim[(size_t)j * K + k] = gamma * cs[k];
        prob[(size_t)j * K + k] = p[k];
      }
  }
  if (lane == 0) {
    qnorm[j] = qn;
    loss_j[j] = -logf(p[0]);
    correct_j[j] = (amax == 0) ? 1.f : 0.f;
  }
  // ---- backward: d loss / d cos_sim[j,k] = (p_k - [k==0]) / BS
  float dq[MAXE];
#pragma unroll
  for (int e = 0; e < MAXE; ++e) dq[e] = 0.f;
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    if (k < K) {
      const float g = gamma * (p[k] - (k == 0 ? 1.f : 0.f)) / (float)bs;
      const float a = g / (qn * dn[k]);
      const float bq = g * cs[k] / (qn * qn);
      const float bd = g * cs[k] / (dn[k] * dn[k]);
      const size_t row = (size_t)doc_row(j, k, bs, neg) * ld;
#pragma unroll
      for (int e = 0; e < MAXE; ++e) {
        const int c = lane + 64 * e;
        if (c < ld) {
          const float x = (c < n) ? y[row + c] : 0.f;
          dq[e] += a * x - bq * q[e];
          dy[row + c] = (c < n) ? a * q[e] - bd * x : 0.f;
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int c = lane + 64 * e;
    if (c < ld) dy[(size_t)j * ld + c] = (c < n) ? dq[e] : 0.f;
  }
}

// Deterministic fixed-order reduction: loss = sum_j loss_j / BS, accuracy = mean(correct).
__global__ __launch_bounds__(256) void k_loss_reduce(const float* __restrict__ loss_j,
                                                     const float* __restrict__ correct_j, int bs,
                                                     float* __restrict__ out) {
  __shared__ float s1[256], s2[256];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < bs; i += 256) {
    a += loss_j[i];
    b += correct_j[i];
  }
  s1[threadIdx.x] = a;
  s2[threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      s1[threadIdx.x] += s1[threadIdx.x + s];
      s2[threadIdx.x] += s2[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = s1[0] / (float)bs;
    out[1] = s2[0] / (float)bs;
  }
}

}  // namespace

hipError_t launch_cosine_loss(const float* y, int ld, int n, int bs, int neg, float gamma,
                              float* cos_raw, float* cos_sim, float* prob, float* qnorm,
                              float* loss_j, float* correct_j, float* loss_out, float* dy,
                              hipStream_t s) {
  if (neg + 1 > MAXK || n > 64 * MAXE) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_cosine_loss, dim3(cdiv(bs, 4)), dim3(256), 0, s, y, ld, n, bs, neg, gamma,
                     cos_raw, cos_sim, prob, qnorm, loss_j, correct_j, dy);
  hipLaunchKernelGGL(k_loss_reduce, dim3(1), dim3(256), 0, s, loss_j, correct_j, bs, loss_out);
  return hipGetLastError();
}

}  // namespace dssm
