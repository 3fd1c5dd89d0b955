// Peer-store data-parallel exchange (include/dssm.h dssm_plan_set_dp_peers; DESIGN.md §6 "peer
// exchange").  The bf16-wire schedule's two collectives (the gradient all-to-all and the parameter
// all-gather, new_dssm.py:215-217's optimizer over a sharded batch) become stores into the peers'
// buffers, mapped into every rank through HIP IPC:
//   * the gradient pass (k_adam_step, gradient-pass mode) stores rank i's bf16 W1 gradient rows of
//     owner j's shard straight into owner j's stage at block i -- the layout the all-to-all delivers --
//     while it computes them, so the link traffic runs under the pass instead of after it;
//   * the fp32 tail (b1, W2.., BN: 0.5 MB) is pushed to every rank's tail stage (k_peer_tail_push),
//     whose last workgroup raises this step's GRAD flag on every rank;
//   * the push's last workgroup then waits for every rank's GRAD flag; the Adam shard sums the
//     world's tails in rank order (the replicated tail stays bit-identical on every rank) and the
//     stage's partials in rank order as the all-to-all schedule does, storing bf16(W1) of its shard
//     into EVERY rank's parameter wire;
//   * k_peer_signal raises this step's PARAM flag on every rank and its last workgroup waits for
//     every rank's; W1's bf16 shadow is then rebuilt from the parameter wire (k_peer_shadow).
// Per step: two launches of their own (push + wait, signal + wait) and the shadow rebuild; a wait
// is one wave of the launch's last workgroup, so it never holds more than one CU.
// No collective library runs on the data path.  Steps are numbered by a per-rank epoch (flags[SEQ],
// advanced by the tail push) and flags only grow, so nothing is re-armed between steps, graph
// replays or regions.  Reuse is ordered by the flags themselves: rank i overwrites owner j's stage
// (or tail slot) for step t+1 only after its PARAM wait of step t saw owner j's Adam of step t done,
// and owner j overwrites rank i's parameter wire for step t+1 only after its GRAD wait saw rank i's
// gradient pass of step t+1, which follows rank i's shadow rebuild of step t on rank i's stream.
//
// Memory: the stage, the parameter wire, the tail stage and the flags are fine-grained device
// allocations (hipDeviceMallocFinegrained: coherent across agents while kernels run), exported with
// hipIpcGetMemHandle.  Producers store plainly; a flag is raised only by a later launch whose
// workgroups (at least one per XCD) each issue a SYSTEM-scope release -- the write-back of that
// XCD's L2 -- and whose last workgroup then stores the flags (system-scope atomics).  The wait
// polls with system-scope atomic loads, and every consumer reads the payload with system-scope
// loads (launch.h ld_sys8; in the first design, plain loads behind a system-scope acquire read stale
// rows across two processes on one GPU).  Before the first step every rank runs the
// self-test below through the same path with synthetic patterns (dssm_plan_peer_selftest).
// Waits are bounded (a timeout sets flags[ERR]; later waits return at once; the host reads it with
// dssm_plan_peer_status), so a peer that never arrives cannot hang the GPU.
#include <cstring>
#include <string>

#include "../../include/dssm.h"
#include "common.h"
#include "launch.h"

namespace dssm {
int report_error(int code, const char* msg);  // plan.hip: sets dssm_last_error()

namespace {

__device__ __forceinline__ unsigned sys_poll(unsigned* p) {
  return __hip_atomic_fetch_add(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Lane k < world of the calling wave waits until flags[base + k] has reached epoch e (bounded by
// `ticks` of the 100 MHz counter; a timeout records 1 + base + k in flags[ERR]; after any timeout
// no wait waits again).
__device__ void wait_flags(unsigned* flags, int base, int world, unsigned e, unsigned long long ticks) {
  const int k = threadIdx.x;
  if (k >= world) return;
  if (__hip_atomic_load(flags + kPeerErr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((int)(sys_poll(flags + base + k) - e) < 0) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      __hip_atomic_store(flags + kPeerErr, (unsigned)(1 + base + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

// The tail's partial of this rank into slot `rank` of every rank's tail stage; every workgroup then
// writes back its XCD's L2 at system scope (at least kSignalBlocks workgroups: every XCD's, so the
// gradient pass's rows stored in the launch before leave too), and the last workgroup advances the
// epoch and raises this rank's GRAD flag on every rank.
__global__ __launch_bounds__(256) void k_peer_tail_push(PeerArgs a) {
  const int64_t n4 = a.tailn / 4;
  const float4* src = reinterpret_cast<const float4*>(a.tail_src);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = src[i];
    const uint2 lo = make_uint2(__float_as_uint(v.x), __float_as_uint(v.y));
    const uint2 hi = make_uint2(__float_as_uint(v.z), __float_as_uint(v.w));
    for (int k = 0; k < a.world; ++k) {
      float* d = a.rtail[k] + a.rank * a.tailn + 4 * i;
      st_sys8(d, lo);
      st_sys8(d + 2, hi);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ unsigned s_last;
  if (threadIdx.x == 0) {
    peer_release();
    const unsigned t = __hip_atomic_fetch_add(a.flags + kPeerTicket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == gridDim.x - 1;
    if (s_last) {
      __hip_atomic_store(a.flags + kPeerTicket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      peer_acquire();  // every workgroup's release (the ticket's RMW chain) before ...
      const unsigned e = __hip_atomic_load(a.flags + kPeerSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
      __hip_atomic_store(a.flags + kPeerSeq, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      peer_release();  // ... this workgroup's flags
      for (int k = 0; k < a.world; ++k)
        __hip_atomic_store(a.rflags[k] + kPeerGrad + a.rank, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      s_last = e;
    }
  }
  __syncthreads();
  // the last workgroup stays for every rank's gradient pass of this step (the next launch, Adam,
  // reads their rows)
  if (s_last && threadIdx.x < 64) wait_flags(a.flags, kPeerGrad, a.world, s_last, a.ticks);
}

// After this rank's Adam shard: every XCD's L2 written back at system scope (kSignalBlocks one-wave
// workgroups, dispatched round-robin over the 8 XCDs, each releasing its XCD's dirty lines -- the
// parameter-wire rows Adam stored there), then the last of them raises this step's PARAM flag on
// every rank.
constexpr int kSignalBlocks = 64;
__global__ __launch_bounds__(64) void k_peer_signal(PeerArgs a) {
  __shared__ unsigned s_e;
  if (threadIdx.x == 0) {
    peer_release();
    const unsigned t = __hip_atomic_fetch_add(a.flags + kPeerTicket2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_e = 0;
    if (t == gridDim.x - 1) {
      __hip_atomic_store(a.flags + kPeerTicket2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      peer_acquire();
      peer_release();
      const unsigned e = __hip_atomic_load(a.flags + kPeerSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int k = 0; k < a.world; ++k)
        __hip_atomic_store(a.rflags[k] + kPeerParam + a.rank, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      s_e = e;
    }
  }
  __syncthreads();
  // the last workgroup stays for every rank's Adam shard of this step (the next launch rebuilds the
  // shadow from the parameter wire they stored)
  if (s_e) wait_flags(a.flags, kPeerParam, a.world, s_e, a.ticks);
}

// ---- start-up self-test (dssm_plan_peer_selftest) -------------------------------------------------
// Synthetic patterns through the exchange's own store / release / flag / load path: every rank stores
// pattern(rank, j) plainly into its slot of every rank's tail stage and into its shard block of every
// rank's parameter wire; k_peer_signal writes back every XCD's L2, raises the flags and waits; then
// every rank reads all W slots and blocks back with system-scope loads and counts mismatches.
__device__ __forceinline__ float tail_pattern(int r, int64_t j) { return (float)((r + 1) * 4096 + (int)(j & 4095)); }
__device__ __forceinline__ unsigned short wire_pattern(int r, int64_t j) {
  return (unsigned short)((r * 40503u + (unsigned)j * 2654435761u) >> 16);
}
__global__ void k_peer_seq_bump(unsigned* flags) {
  const unsigned e = __hip_atomic_load(flags + kPeerSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(flags + kPeerSeq, e + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ __launch_bounds__(256) void k_peer_fill(PeerArgs a, uint16_t* const* pw, int64_t sub) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a.tailn; j += stride)
    for (int k = 0; k < a.world; ++k) a.rtail[k][a.rank * a.tailn + j] = tail_pattern(a.rank, j);
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < sub; j += stride)
    for (int k = 0; k < a.world; ++k) pw[k][a.rank * sub + j] = wire_pattern(a.rank, j);
}
__global__ __launch_bounds__(256) void k_peer_check(PeerArgs a, const uint16_t* pw, int64_t sub, unsigned* bad) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned nb = 0;
  const float* t = a.rtail[a.rank];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.world * a.tailn / 2; i += stride) {
    const int64_t e = 2 * i, r = e / a.tailn, j = e - r * a.tailn;  // tailn is even: a pair never straddles
    const uint2 q = ld_sys8(t + e);
    nb += (__uint_as_float(q.x) != tail_pattern((int)r, j)) + (__uint_as_float(q.y) != tail_pattern((int)r, j + 1));
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.world * sub / 4; i += stride) {
    const int64_t e = 4 * i, r = e / sub, j = e - r * sub;  // sub is a multiple of 4
    const uint2 q = ld_sys8(pw + e);
    nb += ((q.x & 0xffffu) != wire_pattern((int)r, j)) + ((q.x >> 16) != wire_pattern((int)r, j + 1)) +
          ((q.y & 0xffffu) != wire_pattern((int)r, j + 2)) + ((q.y >> 16) != wire_pattern((int)r, j + 3));
  }
  if (nb) atomicAdd(bad, nb);
}

// W1's bf16 shadow from the parameter wire (tight rows of stride geo.n, chunks == 1); system-scope loads.
__global__ __launch_bounds__(256) void k_peer_shadow(const u16* __restrict__ w, ShadowSeg g) {
  const int q = g.cols / 4;
  const int64_t n4 = g.rows * q;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / q;
    const int c = (int)(i - r * q) * 4;
    *reinterpret_cast<uint2*>(g.ptr + r * g.ld + c) = ld_sys8(w + r * g.cols + c);
  }
}

int grid_of(int64_t n4) {
  const int64_t b = (n4 + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

}  // namespace

hipError_t launch_peer_before_adam(const PeerArgs& a, hipStream_t s) {
  if (a.world < 1 || a.world > kPeerMax || a.tailn % 4) return hipErrorInvalidValue;
  const int g = grid_of(a.tailn / 4);
  hipLaunchKernelGGL(k_peer_tail_push, dim3(g < kSignalBlocks ? kSignalBlocks : g), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_peer_after_adam(const PeerArgs& a, hipStream_t s) {
  if (a.world < 1 || a.world > kPeerMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_peer_signal, dim3(kSignalBlocks), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_peer_selftest(const PeerArgs& a, uint16_t* const* pw_dev, const uint16_t* pw_local, int64_t sub,
                                unsigned* bad, hipStream_t s) {
  if (a.world < 1 || a.world > kPeerMax || (a.tailn % 2) || (sub % 4)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_peer_seq_bump, dim3(1), dim3(1), 0, s, a.flags);
  hipLaunchKernelGGL(k_peer_fill, dim3(512), dim3(256), 0, s, a, pw_dev, sub);
  hipLaunchKernelGGL(k_peer_signal, dim3(kSignalBlocks), dim3(64), 0, s, a);
  hipLaunchKernelGGL(k_peer_check, dim3(512), dim3(256), 0, s, a, pw_local, sub, bad);
  return hipGetLastError();
}

hipError_t launch_peer_shadow(const uint16_t* wire, ShadowSeg seg, hipStream_t s) {
  if (seg.cols % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_peer_shadow, dim3(grid_of(seg.rows * seg.cols / 4)), dim3(256), 0, s, wire, seg);
  return hipGetLastError();
}

}  // namespace dssm

// ---- C-ABI: fine-grained buffers and their IPC handles ------------------------------------------
namespace {
int perr(int code, const std::string& m) { return dssm::report_error(code, m.c_str()); }
}  // namespace

extern "C" {

int dssm_peer_alloc(int64_t bytes, void** out) {
  if (!out || bytes <= 0) return perr(DSSM_E_INVALID, "dssm_peer_alloc: bytes > 0 and an output pointer");
  *out = nullptr;
#ifdef DSSM_PEER_COARSE  // measurement: coarse-grained payload buffers (the flags buffer stays fine-grained)
  hipError_t e = bytes == DSSM_PEER_FLAG_BYTES ? hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocFinegrained)
                                               : hipMalloc(out, (size_t)bytes);
#else
  hipError_t e = hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocFinegrained);
#endif
  if (e != hipSuccess) return perr(DSSM_E_HIP, std::string("hipExtMallocWithFlags(fine-grained): ") + hipGetErrorString(e));
  e = hipMemset(*out, 0, (size_t)bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    (void)hipFree(*out);
    *out = nullptr;
    return perr(DSSM_E_HIP, std::string("hipMemset: ") + hipGetErrorString(e));
  }
  return DSSM_OK;
}

int dssm_peer_free(void* p) {
  if (!p) return DSSM_OK;
  hipError_t e = hipFree(p);
  return e == hipSuccess ? DSSM_OK : perr(DSSM_E_HIP, std::string("hipFree: ") + hipGetErrorString(e));
}

int dssm_peer_can_access(int peer_device, int* out) {
  if (!out) return perr(DSSM_E_INVALID, "dssm_peer_can_access: null output");
  int dev = -1;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess && dev == peer_device) {  // the same device (ranks sharing one GPU)
    *out = 1;
    return DSSM_OK;
  }
  if (e == hipSuccess) e = hipDeviceCanAccessPeer(out, dev, peer_device);
  if (e != hipSuccess) return perr(DSSM_E_HIP, std::string("hipDeviceCanAccessPeer: ") + hipGetErrorString(e));
  return DSSM_OK;
}

int dssm_ipc_handle(void* p, void* out64) {
  if (!p || !out64) return perr(DSSM_E_INVALID, "dssm_ipc_handle: null argument");
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle larger than 64 bytes");
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return perr(DSSM_E_HIP, std::string("hipIpcGetMemHandle: ") + hipGetErrorString(e));
  memset(out64, 0, 64);
  memcpy(out64, &h, sizeof(h));
  return DSSM_OK;
}

int dssm_ipc_open(const void* in64, void** out) {
  if (!in64 || !out) return perr(DSSM_E_INVALID, "dssm_ipc_open: null argument");
  hipIpcMemHandle_t h;
  memcpy(&h, in64, sizeof(h));
  *out = nullptr;
  hipError_t e = hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) return perr(DSSM_E_HIP, std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(e));
  return DSSM_OK;
}

int dssm_ipc_close(void* p) {
  if (!p) return DSSM_OK;
  hipError_t e = hipIpcCloseMemHandle(p);
  return e == hipSuccess ? DSSM_OK : perr(DSSM_E_HIP, std::string("hipIpcCloseMemHandle: ") + hipGetErrorString(e));
}

}  // extern "C"
