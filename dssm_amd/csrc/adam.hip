// AdamOptimizer(lr).minimize(loss) (new_dssm.py:215-217) as TF1.x ApplyAdam over the flat
// parameter arena, dense (every element decays m/v every step, as TF does), fused with the
// refresh of the bf16 weight shadows that the perf-mode SpMM/GEMMs read.
//
//   alpha = lr * sqrt(1 - beta2^t) / (1 - beta1^t)   (fp32, like the TF kernel; the beta powers
//   live on the device and k_adam_advance multiplies them after each step, so a captured step
//   graph needs no per-step host scalars)
//   m += (g - m) * (1 - beta1);  v += (g*g - v) * (1 - beta2)
//   p -= (m * alpha) / (sqrt(v) + eps)
//
// HBM-bound: 28 B/param (p, m, v read+write, g read) + 2 B/param of shadow.
//
// Two kernels:
//  * k_adam — float4 per thread over an arena range; gradients at index >= clear_from are
//    zeroed after use ("consume and clear"), so the atomically accumulated gradient blocks
//    start the next step at zero without a memset.
//  * k_adam_w1_fused — single-GPU path: one wave per row of the [W1; b1] block computes the
//    light rows' gradient inline from the CSC transpose and dZ1 (gather.h) and applies Adam in
//    the same pass, so a dense dW1 is never written or re-read; heavy rows (summed by
//    k_dw1_heavy into the gradient arena) are read and cleared.
#include "common.h"
#include "gather.h"
#include "launch.h"

namespace dssm {
namespace {

__device__ __forceinline__ void write_shadow4(const ShadowList& sh, int64_t i, float4 v) {
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
      if (g.tptr) {
        g.tptr[(int64_t)(c + 0) * g.tld + r] = f2bf(v.x);
        g.tptr[(int64_t)(c + 1) * g.tld + r] = f2bf(v.y);
        g.tptr[(int64_t)(c + 2) * g.tld + r] = f2bf(v.z);
        g.tptr[(int64_t)(c + 3) * g.tld + r] = f2bf(v.w);
      }
      return;
    }
  }
}

__device__ __forceinline__ void adam1(float& p, float& m, float& v, float g, float alpha,
                                      float b1c, float b2c, float eps) {
  m += (g - m) * b1c;
  v += (g * g - v) * b2c;
  p -= (m * alpha) / (sqrtf(v) + eps);
}

__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v,
                                              int64_t i4_begin, int64_t i4_end, int64_t clear_from,
                                              const float* __restrict__ st, float lr, float b1c,
                                              float b2c, float eps, float gs, ShadowList sh) {
  const float alpha = lr * sqrtf(1.0f - st[1]) / (1.0f - st[0]);
  for (int64_t i = i4_begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < i4_end;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    adam1(pp.x, mm.x, vv.x, gg.x * gs, alpha, b1c, b2c, eps);
    adam1(pp.y, mm.y, vv.y, gg.y * gs, alpha, b1c, b2c, eps);
    adam1(pp.z, mm.z, vv.z, gg.z * gs, alpha, b1c, b2c, eps);
    adam1(pp.w, mm.w, vv.w, gg.w * gs, alpha, b1c, b2c, eps);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (i * 4 >= clear_from) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (sh.count) write_shadow4(sh, i * 4, pp);
  }
}

template <typename TZ>
__global__ __launch_bounds__(256) void k_adam_w1_fused(
    float* __restrict__ p, float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    int D, int n, const int* __restrict__ col_ptr, const int* __restrict__ csc_row,
    const float* __restrict__ csc_val, const TZ* __restrict__ dZ, int lddz,
    const float* __restrict__ st, float lr, float b1c, float b2c, float eps, float gs,
    u16* __restrict__ shadow, int ldsh) {
  const float alpha = lr * sqrtf(1.0f - st[1]) / (1.0f - st[0]);
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);  // row of [W1; b1] == CSC column
  if (c > D) return;
  const int lane = lane_id();
  const int s = col_ptr[c], e = col_ptr[c + 1];
  const bool heavy = e - s > kLightEntries;
  for (int c0 = 0; c0 < n; c0 += 512) {
    const int cc = c0 + lane * 8;
    const int nvalid = n - cc;
    const size_t o = (size_t)c * n + cc;
    float P[8], M[8], V[8], G[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (nvalid > 0) {  // stream loads first: independent of the gather chain below
      load8(p + o, nvalid, P);
      load8(m + o, nvalid, M);
      load8(v + o, nvalid, V);
    }
    if (heavy) {
      if (nvalid > 0) {
        load8(g + o, nvalid, G);
        *reinterpret_cast<float4*>(g + o) = make_float4(0.f, 0.f, 0.f, 0.f);
        if (nvalid > 4) *reinterpret_cast<float4*>(g + o + 4) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {
      gather_accumulate(csc_row, csc_val, s, e, dZ, lddz, cc, nvalid, G);
    }
    if (nvalid > 0) {
      const int k = nvalid >= 8 ? 8 : 4;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (i < k) adam1(P[i], M[i], V[i], G[i] * gs, alpha, b1c, b2c, eps);
      *reinterpret_cast<float4*>(p + o) = make_float4(P[0], P[1], P[2], P[3]);
      *reinterpret_cast<float4*>(m + o) = make_float4(M[0], M[1], M[2], M[3]);
      *reinterpret_cast<float4*>(v + o) = make_float4(V[0], V[1], V[2], V[3]);
      if (k == 8) {
        *reinterpret_cast<float4*>(p + o + 4) = make_float4(P[4], P[5], P[6], P[7]);
        *reinterpret_cast<float4*>(m + o + 4) = make_float4(M[4], M[5], M[6], M[7]);
        *reinterpret_cast<float4*>(v + o + 4) = make_float4(V[4], V[5], V[6], V[7]);
      }
      if (shadow && c < D) {
        u16* q = shadow + (size_t)c * ldsh + cc;
        uint2 lo;
        lo.x = pack2bf(P[0], P[1]);
        lo.y = pack2bf(P[2], P[3]);
        *reinterpret_cast<uint2*>(q) = lo;
        if (k == 8) {
          uint2 hi;
          hi.x = pack2bf(P[4], P[5]);
          hi.y = pack2bf(P[6], P[7]);
          *reinterpret_cast<uint2*>(q + 4) = hi;
        }
      }
    }
  }
}

// beta1_power *= beta1; beta2_power *= beta2 (TF1.x AdamOptimizer._finish, fp32)
__global__ void k_adam_advance(float* __restrict__ st, float beta1, float beta2) {
  if (threadIdx.x == 0) {
    st[0] = st[0] * beta1;
    st[1] = st[1] * beta2;
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
    if (g.tptr) {
      g.tptr[(int64_t)(c + 0) * g.tld + r] = f2bf(v.x);
      g.tptr[(int64_t)(c + 1) * g.tld + r] = f2bf(v.y);
      g.tptr[(int64_t)(c + 2) * g.tld + r] = f2bf(v.z);
      g.tptr[(int64_t)(c + 3) * g.tld + r] = f2bf(v.w);
    }
  }
}

int grid_for(int64_t n4) {
  const int64_t g = (n4 + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

hipError_t launch_adam(float* p, float* g, float* m, float* v, int64_t begin, int64_t end,
                       int64_t clear_from, const float* st, float lr, float beta1, float beta2,
                       float eps, float grad_scale, ShadowList sh, hipStream_t s) {
  if ((begin % 4) || (end % 4)) return hipErrorInvalidValue;
  if (end <= begin) return hipSuccess;
  const int64_t b4 = begin / 4, e4 = end / 4;
  hipLaunchKernelGGL(k_adam, dim3(grid_for(e4 - b4)), dim3(256), 0, s, p, g, m, v, b4, e4,
                     clear_from, st, lr, 1.0f - beta1, 1.0f - beta2, eps, grad_scale, sh);
  return hipGetLastError();
}

hipError_t launch_adam_w1_fused(float* p, float* g, float* m, float* v, int D, int n,
                                const int* col_ptr, const int* csc_row, const float* csc_val,
                                const void* dZ, bool dz_bf16, int lddz, const float* st, float lr,
                                float beta1, float beta2, float eps, float grad_scale,
                                uint16_t* shadow, int ldsh, hipStream_t s) {
  dim3 grid(cdiv(D + 1, 4)), block(256);
  if (dz_bf16)
    hipLaunchKernelGGL(k_adam_w1_fused<u16>, grid, block, 0, s, p, g, m, v, D, n, col_ptr, csc_row,
                       csc_val, (const u16*)dZ, lddz, st, lr, 1.0f - beta1, 1.0f - beta2, eps,
                       grad_scale, shadow, ldsh);
  else
    hipLaunchKernelGGL(k_adam_w1_fused<float>, grid, block, 0, s, p, g, m, v, D, n, col_ptr,
                       csc_row, csc_val, (const float*)dZ, lddz, st, lr, 1.0f - beta1,
                       1.0f - beta2, eps, grad_scale, shadow, ldsh);
  return hipGetLastError();
}

hipError_t launch_adam_advance(float* st, float beta1, float beta2, hipStream_t s) {
  hipLaunchKernelGGL(k_adam_advance, dim3(1), dim3(64), 0, s, st, beta1, beta2);
  return hipGetLastError();
}

hipError_t launch_shadow_sync(const float* p, ShadowList sh, hipStream_t s) {
  for (int i = 0; i < sh.count; ++i) {
    const int64_t n4 = sh.seg[i].rows * sh.seg[i].cols / 4;
    hipLaunchKernelGGL(k_shadow_sync, dim3(grid_for(n4)), dim3(256), 0, s, p, sh.seg[i]);
  }
  return hipGetLastError();
}

}  // namespace dssm
