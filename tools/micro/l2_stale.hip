// Do kernel boundaries on one stream make another XCD's writes visible to a reader whose XCD L2
// still holds an older copy of the line?  A: every block reads X (X's lines land in every XCD's
// L2).  B: one block rewrites X (plain stores, or memory-side atomic adds).  C: every block reads X
// again and counts elements that are not the new value.  Plain vector loads / stores only.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 16384;  // 64 KB of ints

__global__ void k_read(const int* __restrict__ x, int* __restrict__ sink) {
  int s = 0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) s += x[i];
  if (s == 0x7fffffff) sink[0] = s;  // keeps the loads
}
__global__ void k_write(int* x, int v, int atomic) {
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    if (atomic) atomicAdd(&x[i], 1);
    else x[i] = v;
  }
}
__global__ void k_check(const int* __restrict__ x, int v, int* __restrict__ bad) {
  int b = 0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) b += x[i] != v;
  if (b) atomicAdd(bad, b);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  int *x, *sink, *bad;
  hipMalloc(&x, N * 4);
  hipMalloc(&sink, 4);
  hipMalloc(&bad, 8);
  hipStream_t s;
  hipStreamCreate(&s);
  for (int atomic = 0; atomic < 2; ++atomic) {
    hipMemset(x, 0, N * 4);
    hipMemset(bad, 0, 8);
    hipDeviceSynchronize();
    for (int it = 1; it <= iters; ++it) {
      hipLaunchKernelGGL(k_read, dim3(1024), dim3(256), 0, s, x, sink);
      hipLaunchKernelGGL(k_write, dim3(1), dim3(256), 0, s, x, it, atomic);
      hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, s, x, it, bad);
    }
    hipStreamSynchronize(s);
    int h = 0;
    hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost);
    printf("%s writes: %d stale element reads over %d iterations x 1024 blocks x %d elements\n",
           atomic ? "atomic" : "plain", h, iters, N);
  }
  return 0;
}
