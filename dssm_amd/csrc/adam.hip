// AdamOptimizer(lr).minimize(loss) (new_dssm.py:215-217) as TF1.x ApplyAdam over the flat
// parameter arena, dense (every element decays m/v every step, as TF does), fused with the
// refresh of the bf16 weight shadows that the perf-mode SpMM/GEMMs read.
//
//   alpha = lr * sqrt(1 - beta2^t) / (1 - beta1^t)          (host, fp32, like the TF kernel)
//   m += (g - m) * (1 - beta1);  v += (g*g - v) * (1 - beta2)
//   p -= (m * alpha) / (sqrt(v) + eps)
//
// HBM-bound: 28 B/param (p, m, v read+write, g read) + 2 B/param of shadow; float4 per thread.
#include "common.h"
#include "launch.h"

namespace dssm {
namespace {

__device__ __forceinline__ void write_shadow(const ShadowList& sh, int64_t i, float4 v) {
#pragma unroll 1
  for (int s = 0; s < sh.count; ++s) {
    const ShadowSeg& g = sh.seg[s];
    const int64_t rel = i - g.offset;
    if (rel >= 0 && rel < g.rows * g.cols) {
      const int64_t r = rel / g.cols;
      const int c = (int)(rel - r * g.cols);
      uint2 p;
      p.x = (unsigned)f2bf(v.x) | ((unsigned)f2bf(v.y) << 16);
      p.y = (unsigned)f2bf(v.z) | ((unsigned)f2bf(v.w) << 16);
      *reinterpret_cast<uint2*>(g.ptr + r * g.ld + c) = p;
      return;
    }
  }
}

__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, const float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v,
                                              int64_t n4, float alpha, float b1c, float b2c,
                                              float eps, float gs, ShadowList sh) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* P = &pp.x; float* G = &gg.x; float* M = &mm.x; float* V = &vv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = G[k] * gs;
      M[k] += (gk - M[k]) * b1c;
      V[k] += (gk * gk - V[k]) * b2c;
      P[k] -= (M[k] * alpha) / (sqrtf(V[k]) + eps);
    }
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (sh.count) write_shadow(sh, i * 4, pp);
  }
}

__global__ __launch_bounds__(256) void k_shadow_sync(const float* __restrict__ p, ShadowSeg g) {
  const int64_t n4 = g.rows * g.cols / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t rel = i * 4;
    const int64_t r = rel / g.cols;
    const int c = (int)(rel - r * g.cols);
    const float4 v = *reinterpret_cast<const float4*>(p + g.offset + rel);
    uint2 q;
    q.x = (unsigned)f2bf(v.x) | ((unsigned)f2bf(v.y) << 16);
    q.y = (unsigned)f2bf(v.z) | ((unsigned)f2bf(v.w) << 16);
    *reinterpret_cast<uint2*>(g.ptr + r * g.ld + c) = q;
  }
}

}  // namespace

hipError_t launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float alpha,
                       float beta1, float beta2, float eps, float grad_scale, ShadowList sh,
                       hipStream_t s) {
  if (n % 4) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 8192);
  hipLaunchKernelGGL(k_adam, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, p, g, m, v, n4, alpha,
                     1.0f - beta1, 1.0f - beta2, eps, grad_scale, sh);
  return hipGetLastError();
}

hipError_t launch_shadow_sync(const float* p, ShadowList sh, hipStream_t s) {
  for (int i = 0; i < sh.count; ++i) {
    const int64_t n4 = sh.seg[i].rows * sh.seg[i].cols / 4;
    const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 8192);
    hipLaunchKernelGGL(k_shadow_sync, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, p, sh.seg[i]);
  }
  return hipGetLastError();
}

}  // namespace dssm
