// Diagnostics prototype (not product): the FC1 SpMM over a column-sliced bf16 W1, one 40-column slice
// per XCD (blocks b and b + 8 share an XCD under round-robin dispatch), so each XCD gathers from a
// 2.4 MB slice that its 4 MB L2 can hold instead of the whole 18 MB shadow from the Infinity Cache.
// A wave holds 12 row groups of 5 lanes (8 columns per lane); each group walks one CSR row.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/proto/spmm_slice.hip -o tools/proto/libspmm_slice.so
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int SW = 40, NS = 8, LPG = 5, GPW = 12;

__device__ __forceinline__ void fma8(float v, uint4 a, float (&acc)[8]) {
  acc[0] = __fmaf_rn(v, __uint_as_float(a.x << 16), acc[0]);
  acc[1] = __fmaf_rn(v, __uint_as_float(a.x & 0xffff0000u), acc[1]);
  acc[2] = __fmaf_rn(v, __uint_as_float(a.y << 16), acc[2]);
  acc[3] = __fmaf_rn(v, __uint_as_float(a.y & 0xffff0000u), acc[3]);
  acc[4] = __fmaf_rn(v, __uint_as_float(a.z << 16), acc[4]);
  acc[5] = __fmaf_rn(v, __uint_as_float(a.z & 0xffff0000u), acc[5]);
  acc[6] = __fmaf_rn(v, __uint_as_float(a.w << 16), acc[6]);
  acc[7] = __fmaf_rn(v, __uint_as_float(a.w & 0xffff0000u), acc[7]);
}

template <int U>
__global__ __launch_bounds__(256) void k_spmm_sliced(const int* __restrict__ indptr, const int* __restrict__ indices,
                                                     const float* __restrict__ values, int rows,
                                                     const uint16_t* __restrict__ Ws, int D, int n,
                                                     const float* __restrict__ bias, float* __restrict__ Z, int ldz,
                                                     int xsel) {
  // xsel 0: slice = the block's XCD; 1 (control): slices spread over every XCD
  const int b = blockIdx.x;
  const int x = xsel == 0 ? b % NS : (b / NS) % NS;
  const int rb = xsel == 0 ? b / NS : (b / (NS * NS)) * NS + b % NS;
  if (rb * 4 * GPW >= rows) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane / LPG, k = lane - g * LPG;
  if (g >= GPW) return;
  const int row = (rb * 4 + wave) * GPW + g;
  if (row >= rows) return;
  const int c = x * SW + k * 8;
  if (c >= ldz) return;
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = (c + i < n) ? bias[c + i] : 0.f;
  const int s = indptr[row], e = indptr[row + 1];
  const uint16_t* base = Ws + (size_t)x * D * SW + k * 8;
  int j = s;
  for (; j + U <= e; j += U) {
    int idx[U];
    float val[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      idx[u] = indices[j + u];
      val[u] = values[j + u];
    }
    uint4 raw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) raw[u] = *reinterpret_cast<const uint4*>(base + (size_t)idx[u] * SW);
#pragma unroll
    for (int u = 0; u < U; ++u) fma8(val[u], raw[u], acc);
  }
  for (; j < e; ++j) {
    const int i0 = indices[j];
    const float v0 = values[j];
    fma8(v0, *reinterpret_cast<const uint4*>(base + (size_t)i0 * SW), acc);
  }
  float* zp = Z + (size_t)row * ldz + c;
  *reinterpret_cast<float4*>(zp) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  if (c + 4 < ldz) *reinterpret_cast<float4*>(zp + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
}
}  // namespace

extern "C" int proto_spmm_sliced(const int* indptr, const int* indices, const float* values, int rows,
                                 const uint16_t* Ws, int D, int n, const float* bias, float* Z, int ldz, int u,
                                 int xsel, void* stream) {
  const int rblocks = (rows + 4 * GPW - 1) / (4 * GPW);
  dim3 grid(xsel == 0 ? rblocks * NS : ((rblocks + NS - 1) / NS) * NS * NS);
  hipStream_t s = (hipStream_t)stream;
  if (u == 4)
    hipLaunchKernelGGL(k_spmm_sliced<4>, grid, dim3(256), 0, s, indptr, indices, values, rows, Ws, D, n, bias, Z, ldz, xsel);
  else
    hipLaunchKernelGGL(k_spmm_sliced<8>, grid, dim3(256), 0, s, indptr, indices, values, rows, Ws, D, n, bias, Z, ldz, xsel);
  return (int)hipGetLastError();
}
