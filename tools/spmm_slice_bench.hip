// Microbenchmark (diagnostics only): the FC1 SpMM's gather structure, one wave per CSR row over the
// whole 300-wide bf16 row (the shipping k_spmm_scan form) against XCD-sliced forms, where the
// workgroups sharing an XCD (blocks b, b + 8, ...) gather only one 40-column slice of W1, so each
// XCD's 4 MiB L2 holds its slice of the 30000-row table.
//   hipcc --offload-arch=gfx950 -O3 -o gpurun_out/ssb tools/spmm_slice_bench.hip
//   gpurun_out/ssb gpurun_out/csr.bin      (csr.bin: int32 rows, nnz, D; indptr; indices; f32 values)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

typedef unsigned short u16;
constexpr int N = 300, LDW = 304, LDZ = 304, SW = 40;  // slice width (5 groups of 8)

__device__ __forceinline__ void fma8(const uint4 a, float v, float (&acc)[8]) {
  acc[0] = __fmaf_rn(v, __uint_as_float(a.x << 16), acc[0]);
  acc[1] = __fmaf_rn(v, __uint_as_float(a.x & 0xffff0000u), acc[1]);
  acc[2] = __fmaf_rn(v, __uint_as_float(a.y << 16), acc[2]);
  acc[3] = __fmaf_rn(v, __uint_as_float(a.y & 0xffff0000u), acc[3]);
  acc[4] = __fmaf_rn(v, __uint_as_float(a.z << 16), acc[4]);
  acc[5] = __fmaf_rn(v, __uint_as_float(a.z & 0xffff0000u), acc[5]);
  acc[6] = __fmaf_rn(v, __uint_as_float(a.w << 16), acc[6]);
  acc[7] = __fmaf_rn(v, __uint_as_float(a.w & 0xffff0000u), acc[7]);
}

// A: the shipping structure (8-deep batches, the tail one at a time).  MODE 1: indices folded into
// 1024 rows (an L2-resident table); MODE 2: no arithmetic (the loads' bits xor-ed into acc);
// MODE 3 / 4: the entry's row replaced by a hash of its position, uniform over 1024 / 30000 rows
template <int MODE>
__global__ __launch_bounds__(256) void k_rows(const int* indptr, const int* idx, const float* val, int rows,
                                              const u16* W, const float* bias, float* Z) {
  const int row = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63, c = lane * 8;
  const bool ok = c < N;
  float acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (c + i < N) ? bias[c + i] : 0.f;
  const int s = indptr[row], e = indptr[row + 1];
  for (int base = s; base < e; base += 64) {
    const int cnt = min(64, e - base);
    int mi = 0;
    float mv = 0.f;
    if (lane < cnt) { mi = idx[base + lane]; mv = val[base + lane]; }
    if (MODE >= 3) {
      unsigned h = (unsigned)(base + lane) * 2654435761u;
      h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12;
      mi = MODE == 3 ? (int)(h & 1023) : (int)(h % 30000u);
    }
    int j = 0;
    for (; j + 8 <= cnt; j += 8) {
      uint4 x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        int r = __builtin_amdgcn_readlane(mi, j + u);
        if (MODE == 1) r &= 1023;
        if (ok) x[u] = *reinterpret_cast<const uint4*>(W + (size_t)r * LDW + c);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mv), j + u));
        if (ok) {
          if (MODE == 2) acc[u] = __uint_as_float(__float_as_uint(acc[u]) ^ x[u].x ^ x[u].w);
          else fma8(x[u], v, acc);
        }
      }
    }
    for (; j < cnt; ++j) {
      int r = __builtin_amdgcn_readlane(mi, j);
      if (MODE == 1) r &= 1023;
      const float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mv), j));
      if (ok) fma8(*reinterpret_cast<const uint4*>(W + (size_t)r * LDW + c), v, acc);
    }
  }
  if (ok) {
    float4* z = reinterpret_cast<float4*>(Z + (size_t)row * LDZ + c);
    z[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    z[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
}

// slice k of 8: groups [g0, g0 + ng) of the 38 8-column groups (5,5,5,5,5,5,4,4)
__device__ __forceinline__ int slice_g0(int k) { return k < 6 ? 5 * k : 30 + 4 * (k - 6); }
__device__ __forceinline__ int slice_ng(int k) { return k < 6 ? 5 : 4; }

// B / C: workgroups b, b + 8, ... gather slice b % 8.  Lanes: 12 slots x 5; slot q sums entries
// q, q + 12, ... of the row (U deep in one batch), the slots' partials are summed through LDS in
// slot order.  SLICED: W laid out [8][D][40] (B) or row-major LDW (C).  RPW rows per wave.
template <bool SLICED, int U, int RPW>
__global__ __launch_bounds__(256) void k_slices(const int* indptr, const int* idx, const float* val, int rows,
                                                int D, const u16* W, const float* bias, float* Z) {
  __shared__ float s_p[4][12][SW + 1];
  const int k = blockIdx.x & 7, grp = blockIdx.x >> 3;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int slot = lane / 5, j = lane - slot * 5;
  const int g0 = slice_g0(k), ng = slice_ng(k);
  const bool ok = slot < 12 && j < ng;
  const int c = (g0 + j) * 8;  // column of this lane's group
  const u16* Wk = SLICED ? W + (size_t)k * D * SW + j * 8 : W + c;
  const int ldw = SLICED ? SW : LDW;
  for (int rr = 0; rr < RPW; ++rr) {
    const int row = (grp * 4 + wave) * RPW + rr;
    if (row >= rows) return;
    const int s = indptr[row], e = indptr[row + 1];
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int base = s; base < e; base += 12 * U) {
      int ii[U];
      float vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = base + slot + 12 * u;
        const bool in = slot < 12 && t < e;
        ii[u] = in ? idx[t] : -1;
        vv[u] = in ? val[t] : 0.f;
      }
      uint4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (ok && ii[u] >= 0) x[u] = *reinterpret_cast<const uint4*>(Wk + (size_t)ii[u] * ldw);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (ok && ii[u] >= 0) fma8(x[u], vv[u], acc);
    }
    if (slot < 12 && j < 5) {
#pragma unroll
      for (int i = 0; i < 8; ++i) s_p[wave][slot][j * 8 + i] = acc[i];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own LDS writes (wave-private rows)
    __builtin_amdgcn_wave_barrier();
    if (lane < ng * 8) {
      float z = bias[g0 * 8 + lane];
#pragma unroll
      for (int q = 0; q < 12; ++q) z += s_p[wave][q][lane];
      if (g0 * 8 + lane < N) Z[(size_t)row * LDZ + g0 * 8 + lane] = z;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ __launch_bounds__(256) void k_empty(const int* indptr, float* Z) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (lane * 8 < N) Z[(size_t)row * LDZ + lane * 8] = (float)indptr[row];
}
__global__ __launch_bounds__(256) void k_nothing(float* Z) {
  if (threadIdx.x == 1000) Z[0] = 1.f;
}
__global__ void k_scrub(float4* p, size_t n, float v) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = make_float4(v, v, v, v);
}
// rewrite both W layouts (as the optimizer writes the bf16 shadow each step)
__global__ void k_rewrite(u16* Wr, u16* Ws, int D, unsigned salt) {
  const size_t n = (size_t)D * LDW;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const int r = i / LDW, c = i % LDW;
    unsigned h = (unsigned)(r * 2654435761u) ^ (unsigned)(c * 40503u) ^ salt;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    const float f = c < N ? ((int)(h & 1023) - 512) / 4096.f : 0.f;
    const u16 b = (u16)(__float_as_uint(f) >> 16);
    Wr[i] = b;
    if (c < 320) {
      const int g = c >> 3, k = g < 30 ? g / 5 : 6 + (g - 30) / 4, g0 = k < 6 ? 5 * k : 30 + 4 * (k - 6);
      if (g < 38) Ws[(size_t)k * D * SW + (size_t)r * SW + (c - g0 * 8)] = b;
    }
  }
}

int main(int argc, char** argv) {
  FILE* f = fopen(argc > 1 ? argv[1] : "gpurun_out/csr.bin", "rb");
  if (!f) { perror("csr"); return 1; }
  int hdr[3];
  if (fread(hdr, 4, 3, f) != 3) return 1;
  const int rows = hdr[0], nnz = hdr[1], D = hdr[2];
  std::vector<int> ip(rows + 1), ix(nnz);
  std::vector<float> vl(nnz);
  if (fread(ip.data(), 4, rows + 1, f) != (size_t)rows + 1 || fread(ix.data(), 4, nnz, f) != (size_t)nnz ||
      fread(vl.data(), 4, nnz, f) != (size_t)nnz) return 1;
  fclose(f);
  int max_row = 0;
  for (int r = 0; r < rows; ++r) max_row = std::max(max_row, ip[r + 1] - ip[r]);
  printf("rows %d nnz %d D %d max row %d\n", rows, nnz, D, max_row);
  int *d_ip, *d_ix;
  float *d_v, *d_b, *Z0, *Z1;
  u16 *Wr, *Ws;
  float4* scr;
  const size_t nscr = (size_t)320 << 20 >> 4;
  CK(hipMalloc(&d_ip, 4 * (rows + 1))); CK(hipMalloc(&d_ix, 4 * nnz)); CK(hipMalloc(&d_v, 4 * nnz));
  CK(hipMalloc(&d_b, 4 * LDZ)); CK(hipMalloc(&Z0, 4 * (size_t)rows * LDZ)); CK(hipMalloc(&Z1, 4 * (size_t)rows * LDZ));
  CK(hipMalloc(&Wr, 2 * (size_t)D * LDW + 64)); CK(hipMalloc(&Ws, 2 * (size_t)8 * D * SW + 64));
  CK(hipMalloc(&scr, 16 * nscr));
  CK(hipMemcpy(d_ip, ip.data(), 4 * (rows + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ix, ix.data(), 4 * nnz, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_v, vl.data(), 4 * nnz, hipMemcpyHostToDevice));
  std::vector<float> hb(LDZ);
  for (int i = 0; i < LDZ; ++i) hb[i] = i < N ? 0.01f * (i % 17) : 0.f;
  CK(hipMemcpy(d_b, hb.data(), 4 * LDZ, hipMemcpyHostToDevice));
  CK(hipMemset(Ws, 0, 2 * (size_t)8 * D * SW));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct V { const char* name; int kind; };
  const V vs[] = {{"rows (shipping)", 0}, {"slices row-major U8", 1}, {"slices sliced U8", 2},
                  {"slices sliced U4", 3}, {"slices sliced U8 RPW2", 4}, {"slices sliced U8 RPW4", 5},
                  {"rows, 1024-row table", 6}, {"rows, no arithmetic", 7}, {"indptr + store only", 8},
                  {"rows, uniform 1024 rows", 9}, {"rows, uniform 30000 rows", 10}, {"no memory", 11}};
  auto launch = [&](int kind, float* Z) {
    const int g1 = (rows + 3) / 4;
    switch (kind) {
      case 6: hipLaunchKernelGGL(k_rows<1>, dim3(g1), dim3(256), 0, 0, d_ip, d_ix, d_v, rows, Wr, d_b, Z); break;
      case 7: hipLaunchKernelGGL(k_rows<2>, dim3(g1), dim3(256), 0, 0, d_ip, d_ix, d_v, rows, Wr, d_b, Z); break;
      case 9: hipLaunchKernelGGL(k_rows<3>, dim3(g1), dim3(256), 0, 0, d_ip, d_ix, d_v, rows, Wr, d_b, Z); break;
      case 10: hipLaunchKernelGGL(k_rows<4>, dim3(g1), dim3(256), 0, 0, d_ip, d_ix, d_v, rows, Wr, d_b, Z); break;
      case 11: hipLaunchKernelGGL(k_nothing, dim3(g1), dim3(256), 0, 0, Z); break;
      case 8: hipLaunchKernelGGL(k_empty, dim3(g1), dim3(256), 0, 0, d_ip, Z); break;
      case 0: hipLaunchKernelGGL(k_rows<0>, dim3(g1), dim3(256), 0, 0, d_ip, d_ix, d_v, rows, Wr, d_b, Z); break;
      case 1: hipLaunchKernelGGL((k_slices<false, 8, 1>), dim3(8 * g1), dim3(256), 0, 0, d_ip, d_ix, d_v, rows, D, Wr, d_b, Z); break;
      case 2: hipLaunchKernelGGL((k_slices<true, 8, 1>), dim3(8 * g1), dim3(256), 0, 0, d_ip, d_ix, d_v, rows, D, Ws, d_b, Z); break;
      case 3: hipLaunchKernelGGL((k_slices<true, 4, 1>), dim3(8 * g1), dim3(256), 0, 0, d_ip, d_ix, d_v, rows, D, Ws, d_b, Z); break;
      case 4: hipLaunchKernelGGL((k_slices<true, 8, 2>), dim3(8 * ((rows + 7) / 8)), dim3(256), 0, 0, d_ip, d_ix, d_v, rows, D, Ws, d_b, Z); break;
      case 5: hipLaunchKernelGGL((k_slices<true, 8, 4>), dim3(8 * ((rows + 15) / 16)), dim3(256), 0, 0, d_ip, d_ix, d_v, rows, D, Ws, d_b, Z); break;
    }
  };
  hipLaunchKernelGGL(k_rewrite, dim3(2048), dim3(256), 0, 0, Wr, Ws, D, 1u);
  launch(0, Z0);
  CK(hipDeviceSynchronize());
  std::vector<float> h0((size_t)rows * LDZ), h1((size_t)rows * LDZ);
  CK(hipMemcpy(h0.data(), Z0, 4 * h0.size(), hipMemcpyDeviceToHost));
  for (const V& v : vs) {
    CK(hipMemset(Z1, 0, 4 * (size_t)rows * LDZ));
    launch(v.kind, Z1);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h1.data(), Z1, 4 * h1.size(), hipMemcpyDeviceToHost));
    double md = 0;
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < N; ++c)
        md = std::max(md, (double)fabsf(h0[(size_t)r * LDZ + c] - h1[(size_t)r * LDZ + c]));
    float tc = 0, th = 0;
    const int it = 40;
    for (int i = 0; i < it; ++i) {  // cold: a 320 MB stream and the table rewritten before each launch
      hipLaunchKernelGGL(k_scrub, dim3(4096), dim3(256), 0, 0, scr, nscr, (float)i);
      hipLaunchKernelGGL(k_rewrite, dim3(2048), dim3(256), 0, 0, Wr, Ws, D, 1u);
      CK(hipEventRecord(e0));
      launch(v.kind, Z1);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      tc += ms;
    }
    for (int i = 0; i < it; ++i) {  // warm: back to back
      CK(hipEventRecord(e0));
      launch(v.kind, Z1);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      th += ms;
    }
    printf("%-24s cold %7.2f us  warm %7.2f us  max|diff| %.3g\n", v.name, 1e3 * tc / it, 1e3 * th / it, md);
  }
  return 0;
}
