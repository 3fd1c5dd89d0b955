// Dispatch cost of a launch by workgroup size and LDS request (k_csc_rank's shape: 128
// workgroups of 1024 threads, ~136 KB LDS each) behind a trivial launch, in a captured graph.
// Build: hipcc --offload-arch=gfx950 -O3 dispatch_lds.hip -o dispatch_lds
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_triv(int* out) {
  if (threadIdx.x == 0 && out) out[blockIdx.x] = 1;
}
__global__ __launch_bounds__(1024) void k_lds(int* out, int D) {
  extern __shared__ int hist[];
  for (int c = threadIdx.x; c < D; c += blockDim.x) hist[c] = c;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = hist[(blockIdx.x * 7) % D];
}

static float run(int tb, size_t lds, int grid, int* buf, hipStream_t s, bool with_x) {
  hipGraph_t g;
  hipGraphExec_t ge;
  const int iters = 200;
  hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < iters; ++i) {
    hipLaunchKernelGGL(k_triv, dim3(256), dim3(256), 0, s, buf);
    if (with_x) hipLaunchKernelGGL(k_lds, dim3(grid), dim3(tb), lds, s, buf, (int)(lds / 4));
  }
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipGraphLaunch(ge, s);
  hipEventRecord(a, s);
  hipGraphLaunch(ge, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return ms * 1000.f / iters;
}

int main() {
  int* buf;
  hipMalloc(&buf, 1 << 20);
  hipStream_t s;
  hipStreamCreate(&s);
  hipFuncSetAttribute((const void*)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const float base = run(256, 0, 1, buf, s, false);
  printf("trivial alone: %.2f us per iteration\n", base);
  const int tbs[] = {256, 512, 1024};
  const size_t ldss[] = {4096, 65536, 120000, 136000, 150000};
  for (int tb : tbs)
    for (size_t l : ldss) {
      const float t = run(tb, l, 128, buf, s, true);
      printf("tb %4d lds %6zu grid 128: +%.2f us\n", tb, l, t - base);
    }
  const float t = run(1024, 120000, 256, buf, s, true);
  printf("tb 1024 lds 120000 grid 256: +%.2f us\n", t - base);
  return 0;
}
