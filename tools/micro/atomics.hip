// Micro-benchmark: throughput of device-scope fp64 atomic adds from many workgroups onto a small
// set of accumulators, contiguous vs one accumulator per 128-B line, vs replicated per XCD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_atom(double* acc, int naddr, int stride, int reps, int nrep_copies) {
  const int copy = blockIdx.x % nrep_copies;
  for (int r = 0; r < reps; ++r)
    for (int i = threadIdx.x; i < naddr; i += blockDim.x)
      __hip_atomic_fetch_add(acc + (size_t)copy * naddr * stride + (size_t)i * stride, 1.0,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int main() {
  double* acc;
  hipMalloc(&acc, 64 << 20);
  hipMemset(acc, 0, 64 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  struct Case { int blocks, naddr, stride, copies; };
  std::vector<Case> cases = {{384, 1200, 1, 1}, {384, 1200, 16, 1}, {384, 1200, 1, 8}, {384, 1200, 16, 8},
                             {480, 256, 1, 1}, {480, 256, 16, 1}, {1536, 1200, 1, 1}, {256, 512, 1, 1},
                             {256, 512, 16, 1}, {384, 1200, 2, 1}, {384, 1200, 4, 1}};
  for (auto c : cases) {
    for (int it = 0; it < 3; ++it) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k_atom, dim3(c.blocks), dim3(256), 0, 0, acc, c.naddr, c.stride, 1, c.copies);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (it == 2)
        printf("blocks %5d addrs %5d stride %2d copies %d: %8.2f us  (%ld atomics)\n", c.blocks, c.naddr,
               c.stride, c.copies, ms * 1e3, (long)c.blocks * c.naddr);
    }
  }
  // empty-kernel reference
  for (int it = 0; it < 3; ++it) {
    hipEventRecord(a);
    hipLaunchKernelGGL(k_atom, dim3(384), dim3(256), 0, 0, acc, 0, 1, 1, 1);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (it == 2) printf("empty: %.2f us\n", ms * 1e3);
  }
  return 0;
}
