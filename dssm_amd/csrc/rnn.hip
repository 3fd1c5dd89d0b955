// RNN tower of the reference (semantic_matching/dssm_rnn/dssm_rnn.py:100-217):
// word-embedding lookup -> one bidirectional GRU (TF1 GRUCell, dynamic lengths) -> dropout ->
// the (NEG+1)-way cosine / softmax loss (summed over queries) -> Adam.  fp32 throughout.
//
// The recurrence is row-local: a sequence's state depends only on its own inputs, so one
// workgroup owns kRB sequences of one direction and walks all T steps inside ONE launch with its
// rows' states in LDS -- no grid-wide synchronisation between steps.  Per step it
//   stages z = [x_t, h] (x_t gathered from the embedding table: the lookup is fused),
//   gates = sigmoid(z Wg + bg) (thread o owns output column o; W rows stream from L2, coalesced
//   across threads; z is an LDS broadcast),
//   c = tanh([x_t, r*h] Wc + bc),  h' = u*h + (1-u)*c  (state carried past the row's length),
// and saves z, z2 = [x_t, r*h] and (r, u, c) for the backward.  The backward walks the steps in
// reverse the same way (transposed weight copies keep its W reads coalesced), writes the gate /
// candidate pre-activation gradients per step and scatter-adds dx into the embedding gradient;
// the weight gradients [W; b] are then ONE split-K GEMM per matrix over all T*R (step, row)
// pairs (gemm.hip's TN GEMM with its virtual ones row for the bias), not T small ones.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "../../include/dssm.h"
#include "common.h"
#include "launch.h"

namespace dssm {
int report_error(int code, const char* msg);
}

namespace dssm {
namespace {

constexpr int kRB = 8;        // sequences per workgroup
constexpr int kMaxK = 512;    // E + H
constexpr int kMaxH = 256;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

struct GruDims {
  int R, T, E, H;
};

// ---- forward -----------------------------------------------------------------------------------
// grid (ceil(R / kRB), 2 directions), 256 threads.  W: [Wg_b (K+1)x2H, Wc_b (K+1)xH] per direction
// (last row = bias).  Z, Z2: [dir][T][R][K]; G: [dir][T][R][3H] = (r, u, c); out: [R x 2H]
// (forward state in [0, H), backward in [H, 2H)).
__global__ __launch_bounds__(256) void k_gru_fwd(GruDims d, const int* __restrict__ ids,
                                                 const int* __restrict__ lens,
                                                 const float* __restrict__ emb,
                                                 const float* __restrict__ wg_fw,
                                                 const float* __restrict__ wc_fw,
                                                 const float* __restrict__ wg_bw,
                                                 const float* __restrict__ wc_bw, float* __restrict__ Z, float* __restrict__ Z2,
                                                 float* __restrict__ G, float* __restrict__ out, int ldo) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int dir = blockIdx.y;
  const float* Wg = dir ? wg_bw : wg_fw;
  const float* Wc = dir ? wc_bw : wc_fw;
  const int E = d.E, H = d.H, K = E + H, T = d.T, R = d.R;
  const int r0 = blockIdx.x * kRB, tid = threadIdx.x;
  float* z = lds;                  // [kRB][K]
  float* z2 = z + kRB * K;         // [kRB][K]
  float* h = z2 + kRB * K;         // [kRB][H]
  float* gate = h + kRB * H;       // [kRB][2H]
  float* part = gate + kRB * 2 * H;  // [2][kRB][H]
  int len[kRB];
#pragma unroll
  for (int i = 0; i < kRB; ++i) len[i] = r0 + i < R ? lens[r0 + i] : 0;
  for (int i = tid; i < kRB * H; i += 256) h[i] = 0.f;
  __syncthreads();
  const size_t plane = (size_t)T * R;
  for (int t = 0; t < T; ++t) {
    // z = [x_t, h]
    for (int i = tid; i < kRB * K; i += 256) {
      const int rr = i / K, k = i - rr * K, r = r0 + rr;
      float v = 0.f;
      if (r < R) {
        if (k < E) {
          const bool act = t < len[rr];
          const int idx = act ? (dir ? len[rr] - 1 - t : t) : 0;
          v = emb[(size_t)ids[(size_t)r * T + idx] * E + k];
        } else {
          v = h[(rr) * H + k - E];
        }
        Z[((size_t)dir * plane + (size_t)t * R + r) * K + k] = v;
      }
      z[(rr) * K + k] = v;
    }
    __syncthreads();
    // gates: sigmoid(z Wg + bg)
    for (int o = tid; o < 2 * H; o += 256) {
      float acc[kRB];
      const float b = Wg[(size_t)K * 2 * H + o];
#pragma unroll
      for (int i = 0; i < kRB; ++i) acc[i] = b;
      for (int k = 0; k < K; k += 4) {  // 4 k per LDS broadcast (ds_read_b128), W coalesced
        const float w0 = Wg[(size_t)k * 2 * H + o], w1 = Wg[(size_t)(k + 1) * 2 * H + o];
        const float w2 = Wg[(size_t)(k + 2) * 2 * H + o], w3 = Wg[(size_t)(k + 3) * 2 * H + o];
#pragma unroll
        for (int i = 0; i < kRB; ++i) {
          const float4 zz = *reinterpret_cast<const float4*>(&z[(i) * K + k]);
          acc[i] = fmaf(zz.x, w0, fmaf(zz.y, w1, fmaf(zz.z, w2, fmaf(zz.w, w3, acc[i]))));
        }
      }
#pragma unroll
      for (int i = 0; i < kRB; ++i) gate[(i) * 2 * H + o] = sigm(acc[i]);
    }
    __syncthreads();
    // z2 = [x_t, r * h]
    for (int i = tid; i < kRB * K; i += 256) {
      const int rr = i / K, k = i - rr * K, r = r0 + rr;
      const float v = k < E ? z[(rr) * K + k] : gate[(rr) * 2 * H + k - E] * h[(rr) * H + k - E];
      z2[(rr) * K + k] = v;
      if (r < R) Z2[((size_t)dir * plane + (size_t)t * R + r) * K + k] = v;
    }
    __syncthreads();
    // candidate: two halves of K per output column, summed through LDS
    for (int q = tid; q < 2 * H; q += 256) {
      const int o = q % H, half = q / H;
      const int kh = (K / 2) & ~3;
      const int k0 = half ? kh : 0, k1 = half ? K : kh;
      float acc[kRB];
#pragma unroll
      for (int i = 0; i < kRB; ++i) acc[i] = 0.f;
      for (int k = k0; k < k1; k += 4) {
        const float w0 = Wc[(size_t)k * H + o], w1 = Wc[(size_t)(k + 1) * H + o];
        const float w2 = Wc[(size_t)(k + 2) * H + o], w3 = Wc[(size_t)(k + 3) * H + o];
#pragma unroll
        for (int i = 0; i < kRB; ++i) {
          const float4 zz = *reinterpret_cast<const float4*>(&z2[(i) * K + k]);
          acc[i] = fmaf(zz.x, w0, fmaf(zz.y, w1, fmaf(zz.z, w2, fmaf(zz.w, w3, acc[i]))));
        }
      }
#pragma unroll
      for (int i = 0; i < kRB; ++i) part[(half * kRB + i) * H + o] = acc[i];
    }
    __syncthreads();
    for (int i = tid; i < kRB * H; i += 256) {
      const int rr = i / H, o = i - rr * H, r = r0 + rr;
      const float c = tanhf(part[rr * H + o] + part[(kRB + rr) * H + o] + Wc[(size_t)K * H + o]);
      const float u = gate[(rr) * 2 * H + H + o], hv = h[(rr) * H + o];
      if (r < R) {
        float* g = G + ((size_t)dir * plane + (size_t)t * R + r) * 3 * H;
        g[o] = gate[(rr) * 2 * H + o];
        g[H + o] = u;
        g[2 * H + o] = c;
        if (t < len[rr]) h[(rr) * H + o] = u * hv + (1.f - u) * c;
      }
    }
    __syncthreads();
  }
  for (int i = tid; i < kRB * H; i += 256) {
    const int rr = i / H, o = i - rr * H, r = r0 + rr;
    if (r < R) out[(size_t)r * ldo + dir * H + o] = h[(rr) * H + o];
  }
}

// ---- backward ----------------------------------------------------------------------------------
// WgT [2H x K], WcT [H x K] (transposed weights, bias rows dropped).  dout [R x ldo].  Writes
// dG [dir][T][R][2H] (gate pre-activation gradients), dC [dir][T][R][H] (candidate), zero at a
// row's inactive steps, and adds dx into demb (fp32 atomics).
__global__ __launch_bounds__(256) void k_gru_bwd(GruDims d, const int* __restrict__ ids,
                                                 const int* __restrict__ lens,
                                                 const float* __restrict__ wgT_fw,
                                                 const float* __restrict__ wcT_fw,
                                                 const float* __restrict__ wgT_bw,
                                                 const float* __restrict__ wcT_bw,
                                                 const float* __restrict__ dout, int ldo,
                                                 const float* __restrict__ Z,
                                                 const float* __restrict__ G, float* __restrict__ dG,
                                                 float* __restrict__ dC,
                                                 float* __restrict__ demb) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int dir = blockIdx.y;
  const float* WgT = dir ? wgT_bw : wgT_fw;
  const float* WcT = dir ? wcT_bw : wcT_fw;
  const int E = d.E, H = d.H, K = E + H, T = d.T, R = d.R;
  const int r0 = blockIdx.x * kRB, tid = threadIdx.x;
  float* dcand = lds;                // [kRB][H]  candidate pre-activation gradient
  float* dgate = dcand + kRB * H;    // [kRB][2H]
  float* dz2 = dgate + kRB * 2 * H;  // [kRB][K]  dcand Wc^T
  float* dh = dz2 + kRB * K;         // [kRB][H]  gradient reaching the state after step t
  float* dhp = dh + kRB * H;         // [kRB][H]  dh_prev without the gate path
  float* hold = dhp + kRB * H;       // [kRB][H]  state before step t
  float* rs = hold + kRB * H;        // [kRB][H]  reset gate
  float* dzs = rs + kRB * H;         // [kRB][H]  state part of dgate Wg^T
  int len[kRB];
#pragma unroll
  for (int i = 0; i < kRB; ++i) len[i] = r0 + i < R ? lens[r0 + i] : 0;
  for (int i = tid; i < kRB * H; i += 256) {
    const int rr = i / H, o = i - rr * H, r = r0 + rr;
    dh[(rr) * H + o] = r < R ? dout[(size_t)r * ldo + dir * H + o] : 0.f;
  }
  __syncthreads();
  const size_t plane = (size_t)T * R;
  for (int t = T - 1; t >= 0; --t) {
    // 1. new_h = u*h + (1-u)*c: candidate and update-gate pre-activation gradients
    for (int i = tid; i < kRB * H; i += 256) {
      const int rr = i / H, o = i - rr * H, r = r0 + rr;
      float dc_ = 0.f, du = 0.f, h0 = 0.f, rg = 0.f;
      if (r < R) {
        const size_t row = (size_t)dir * plane + (size_t)t * R + r;
        const float* g = G + row * 3 * H;
        rg = g[o];
        const float u = g[H + o], c = g[2 * H + o];
        h0 = Z[row * K + E + o];
        const float dhn = t < len[rr] ? dh[(rr) * H + o] : 0.f;
        dc_ = dhn * (1.f - u) * (1.f - c * c);
        du = dhn * (h0 - c) * u * (1.f - u);
        dC[row * H + o] = dc_;
        dhp[(rr) * H + o] = t < len[rr] ? dhn * u : dh[(rr) * H + o];  // carried past the row's length
      } else {
        dhp[(rr) * H + o] = 0.f;
      }
      hold[(rr) * H + o] = h0;
      rs[(rr) * H + o] = rg;
      dcand[(rr) * H + o] = dc_;
      dgate[(rr) * 2 * H + H + o] = du;
    }
    __syncthreads();
    // 2. dz2 = dcand Wc^T
    for (int k = tid; k < K; k += 256) {
      float acc[kRB];
#pragma unroll
      for (int i = 0; i < kRB; ++i) acc[i] = 0.f;
      for (int o = 0; o < H; o += 4) {
        const float w0 = WcT[(size_t)o * K + k], w1 = WcT[(size_t)(o + 1) * K + k];
        const float w2 = WcT[(size_t)(o + 2) * K + k], w3 = WcT[(size_t)(o + 3) * K + k];
#pragma unroll
        for (int i = 0; i < kRB; ++i) {
          const float4 q = *reinterpret_cast<const float4*>(&dcand[(i) * H + o]);
          acc[i] = fmaf(q.x, w0, fmaf(q.y, w1, fmaf(q.z, w2, fmaf(q.w, w3, acc[i]))));
        }
      }
#pragma unroll
      for (int i = 0; i < kRB; ++i) dz2[(i) * K + k] = acc[i];
    }
    __syncthreads();
    // 3. reset gate through r*h; the state gradient through r*h
    for (int i = tid; i < kRB * H; i += 256) {
      const int rr = i / H, o = i - rr * H, r = r0 + rr;
      const float rg = rs[(rr) * H + o], drh = dz2[(rr) * K + E + o];
      const float dr = drh * hold[(rr) * H + o] * rg * (1.f - rg);
      dgate[(rr) * 2 * H + o] = dr;
      if (r < R) {
        const size_t row = (size_t)dir * plane + (size_t)t * R + r;
        dG[row * 2 * H + o] = dr;
        dG[row * 2 * H + H + o] = dgate[(rr) * 2 * H + H + o];
        if (t < len[rr]) dhp[(rr) * H + o] += drh * rg;
      }
    }
    __syncthreads();
    // 4. dz = dgate Wg^T: input part + dz2's input part -> embedding gradient, state part kept
    for (int k = tid; k < K; k += 256) {
      float acc[kRB];
#pragma unroll
      for (int i = 0; i < kRB; ++i) acc[i] = 0.f;
      for (int o = 0; o < 2 * H; o += 4) {
        const float w0 = WgT[(size_t)o * K + k], w1 = WgT[(size_t)(o + 1) * K + k];
        const float w2 = WgT[(size_t)(o + 2) * K + k], w3 = WgT[(size_t)(o + 3) * K + k];
#pragma unroll
        for (int i = 0; i < kRB; ++i) {
          const float4 q = *reinterpret_cast<const float4*>(&dgate[(i) * 2 * H + o]);
          acc[i] = fmaf(q.x, w0, fmaf(q.y, w1, fmaf(q.z, w2, fmaf(q.w, w3, acc[i]))));
        }
      }
#pragma unroll
      for (int i = 0; i < kRB; ++i) {
        const int r = r0 + i;
        if (k >= E) {
          dzs[(i) * H + k - E] = acc[i];
        } else if (r < R && t < len[i]) {
          const int idx = dir ? len[i] - 1 - t : t;
          using gfloat = __attribute__((address_space(1))) float;
          __hip_atomic_fetch_add((gfloat*)(demb + (size_t)ids[(size_t)r * T + idx] * E + k),
                                 acc[i] + dz2[(i) * K + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    __syncthreads();
    // 5. gradient reaching the state before step t
    for (int i = tid; i < kRB * H; i += 256) {
      const int rr = i / H, o = i - rr * H;
      dh[(rr) * H + o] = t < len[rr] ? dhp[(rr) * H + o] + dzs[(rr) * H + o] : dhp[(rr) * H + o];
    }
    __syncthreads();
  }
}

// [rows x cols] -> [cols x ld] (the bias row is not transposed: pass rows = K)
__global__ void k_transpose(const float* __restrict__ src, int rows, int cols, float* __restrict__ dst,
                            int ld) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + threadIdx.x;
    tile[i][threadIdx.x] = (r < rows && c < cols) ? src[(size_t)r * cols + c] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + threadIdx.x;
    if (c < cols && r < rows) dst[(size_t)c * ld + r] = tile[threadIdx.x][i];
  }
}

// inverted dropout with the counter-based mask (oracle/rnn_oracle.py dropout_mask): y = x * m *
// scale / keep; the backward uses the same call on dy (scale folds the summed loss's BS).

__global__ void k_dropout(const float* __restrict__ x, float* __restrict__ y, int rows, int cols,
                          int ld, float keep, unsigned thr, unsigned seed, unsigned step, float scale) {
  const int n = rows * cols;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = i / cols, c = i - r * cols;
    const bool kept = keep >= 1.f || dropout_hash((unsigned)i, seed, step) < thr;
    y[(size_t)r * ld + c] = kept ? x[(size_t)r * ld + c] * (scale / (keep >= 1.f ? 1.f : keep)) : 0.f;
  }
}

// TF1.x Adam over the RNN arena: [0, n_sparse) is the embedding table (IndexedSlices gradient:
// _apply_sparse_shared's m*b1 + (1-b1) g form), the rest dense ApplyAdam.  st: device beta powers.
__global__ __launch_bounds__(256) void k_rnn_adam(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ m, float* __restrict__ v,
                                                  int64_t n_sparse, int64_t n, const float* st,
                                                  float lr, float b1, float b2, float eps, float gs,
                                                  uint16_t* __restrict__ shadow = nullptr) {
  const float alpha = lr * sqrtf(1.0f - st[1]) / (1.0f - st[0]);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * gs;
    float mi = m[i], vi = v[i];
    if (i < n_sparse) {
      mi = mi * b1 + gi * (1.0f - b1);
      vi = vi * b2 + (gi * gi) * (1.0f - b2);
    } else {
      mi += (gi - mi) * (1.0f - b1);
      vi += (gi * gi - vi) * (1.0f - b2);
    }
    m[i] = mi;
    v[i] = vi;
    const float pi = p[i] - (mi * alpha) / (sqrtf(vi) + eps);
    p[i] = pi;
    // the embedding table's bf16 copy the bf16 recurrences gather (no per-step conversion pass)
    if (shadow && i < n_sparse) shadow[i] = f2bf(pi);
  }
}

__global__ void k_rnn_adam_advance(float* st, float b1, float b2) {
  if (threadIdx.x == 0) {
    st[0] *= b1;
    st[1] *= b2;
  }
}

}  // namespace
}  // namespace dssm

// ---- C-ABI -------------------------------------------------------------------------------------
namespace {
int rerr(int code, const char* m) { return dssm::report_error(code, m); }
bool dims_ok(int R, int T, int E, int H) {
  return R > 0 && T > 0 && E > 0 && H > 0 && E + H <= dssm::kMaxK && H <= dssm::kMaxH && (E % 4) == 0 &&
         (H % 4) == 0;
}
// HIP-event probes around dssm_adam_step's optimizer launch (bench.py's multi-view roofline: the
// launch's duration measured on the stream it runs on; recorded inside a graph capture they become
// event-record nodes, which time each captured launch's latest replay)
struct AdamProbe {
  std::vector<hipEvent_t> ev;  // pairs
  int used = 0;
} g_adam_probe;
}  // namespace

namespace dssm {
// the optimizer-launch probe (dssm_adam_probe): an event before and after each probed launch on the
// stream it runs on; adam_probe_begin says whether this launch is probed
bool adam_probe_begin(hipStream_t s) {
  const bool probe = g_adam_probe.used < (int)g_adam_probe.ev.size() / 2;
  if (probe) record_probe_event(s, g_adam_probe.ev[2 * g_adam_probe.used]);
  return probe;
}
void adam_probe_end(hipStream_t s) { record_probe_event(s, g_adam_probe.ev[2 * g_adam_probe.used++ + 1]); }
}  // namespace dssm

extern "C" {

size_t dssm_rnn_ws_floats(int R, int T, int E, int H) {
  if (!dims_ok(R, T, E, H)) return 0;
  const size_t K = E + H, plane = (size_t)2 * T * R;
  size_t n = plane * K * 2            // Z, Z2
             + plane * 3 * H          // G
             + plane * 2 * H          // dG
             + plane * H              // dC
             + 2 * (size_t)(2 * H + H) * K;  // transposed weights
  const size_t slab = std::max(dssm::gemm_dw_slab_floats(K + 1, 2 * H, T * R, false),
                               dssm::gemm_dw_slab_floats(K + 1, H, T * R, false));
  return n + slab + 64;
}

int dssm_rnn_forward(const int32_t* ids, const int32_t* lens, int R, int T, const float* emb, int E,
                     int H, const float* const* w, float* ws, float* y, int ldy, void* stream) {
  if (!ids || !lens || !emb || !w || !ws || !y || !dims_ok(R, T, E, H) || ldy < 2 * H)
    return rerr(DSSM_E_INVALID, "rnn_forward: bad argument");
  const size_t K = E + H, plane = (size_t)2 * T * R;
  float* Z = ws;
  float* Z2 = Z + plane * K;
  float* G = Z2 + plane * K;
  const dssm::GruDims d{R, T, E, H};
  const size_t lds = sizeof(float) * dssm::kRB * (2 * K + 5 * (size_t)H);
  hipLaunchKernelGGL(dssm::k_gru_fwd, dim3((R + dssm::kRB - 1) / dssm::kRB, 2), dim3(256), lds,
                     (hipStream_t)stream, d, ids, lens, emb, w[0], w[1], w[2], w[3], Z, Z2, G, y, ldy);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DSSM_OK : rerr(DSSM_E_HIP, hipGetErrorString(e));
}

int dssm_rnn_dropout(const float* x, float* y, int rows, int cols, int ld, float keep, uint32_t seed,
                     uint32_t step, float scale, void* stream) {
  if (!x || !y || rows < 0 || cols < 0 || ld < cols || !(keep > 0.f))
    return rerr(DSSM_E_INVALID, "rnn_dropout: bad argument");
  const double t = (double)keep * 4294967296.0;
  const unsigned thr = t >= 4294967295.0 ? 0xFFFFFFFFu : (unsigned)t;
  const int n = rows * cols, grid = std::max(1, std::min((n + 255) / 256, 2048));
  hipLaunchKernelGGL(dssm::k_dropout, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, y, rows, cols,
                     ld, keep, thr, seed, step, scale);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DSSM_OK : rerr(DSSM_E_HIP, hipGetErrorString(e));
}

int dssm_rnn_backward(const int32_t* ids, const int32_t* lens, int R, int T, int E, int H,
                      const float* const* w, const float* dy, int lddy, float* ws, float* demb,
                      int64_t demb_elems, float* const* gw, void* stream) {
  if (!ids || !lens || !w || !dy || !ws || !demb || !gw || !dims_ok(R, T, E, H) || lddy < 2 * H ||
      demb_elems < 0)
    return rerr(DSSM_E_INVALID, "rnn_backward: bad argument");
  hipStream_t s = (hipStream_t)stream;
  if (zero_bytes_async(demb, sizeof(float) * (size_t)demb_elems, s) != hipSuccess)
    return rerr(DSSM_E_HIP, "rnn_backward: zero fill");
  const int K = E + H;
  const size_t plane = (size_t)2 * T * R;
  float* Z = ws;
  float* Z2 = Z + plane * K;
  float* G = Z2 + plane * K;
  float* dG = G + plane * 3 * H;
  float* dC = dG + plane * 2 * H;
  float* wT = dC + plane * H;  // [dir][WgT (2H x K) | WcT (H x K)]
  float* slab = wT + 2 * (size_t)(3 * H) * K;
  for (int dir = 0; dir < 2; ++dir) {
    float* gT = wT + (size_t)dir * 3 * H * K;
    hipLaunchKernelGGL(dssm::k_transpose, dim3((2 * H + 31) / 32, (K + 31) / 32), dim3(32, 8), 0, s,
                       w[2 * dir], K, 2 * H, gT, K);
    hipLaunchKernelGGL(dssm::k_transpose, dim3((H + 31) / 32, (K + 31) / 32), dim3(32, 8), 0, s,
                       w[2 * dir + 1], K, H, gT + (size_t)2 * H * K, K);
  }
  const dssm::GruDims d{R, T, E, H};
  const size_t lds = sizeof(float) * dssm::kRB * ((size_t)K + 8 * H);
  hipLaunchKernelGGL(dssm::k_gru_bwd, dim3((R + dssm::kRB - 1) / dssm::kRB, 2), dim3(256), lds, s, d,
                     ids, lens, wT, wT + (size_t)2 * H * K, wT + (size_t)3 * H * K,
                     wT + (size_t)5 * H * K, dy, lddy, Z, G, dG, dC, demb);
  // [W; b] gradients: one split-K TN GEMM per matrix over all (step, row) pairs, ones row = bias
  const size_t half = plane / 2;
  for (int dir = 0; dir < 2; ++dir) {
    hipError_t e = dssm::launch_gemm(dssm::GEMM_DW, false, K + 1, 2 * H, T * R, Z + half * dir * K, K,
                                     dG + half * dir * 2 * H, 2 * H, gw[2 * dir], 2 * H, nullptr, true,
                                     slab, s, nullptr);
    if (e == hipSuccess)
      e = dssm::launch_gemm(dssm::GEMM_DW, false, K + 1, H, T * R, Z2 + half * dir * K, K,
                            dC + half * dir * H, H, gw[2 * dir + 1], H, nullptr, true, slab, s, nullptr);
    if (e != hipSuccess) return rerr(DSSM_E_HIP, hipGetErrorString(e));
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DSSM_OK : rerr(DSSM_E_HIP, hipGetErrorString(e));
}

int dssm_rnn_adam_ex(float* p, const float* g, float* m, float* v, int64_t n_sparse, int64_t n,
                     float* state, float lr, float beta1, float beta2, float eps, uint16_t* shadow, void* stream) {
  if (!p || !g || !m || !v || !state || n_sparse < 0 || n < n_sparse)
    return rerr(DSSM_E_INVALID, "rnn_adam: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096));
  hipLaunchKernelGGL(dssm::k_rnn_adam, dim3(grid), dim3(256), 0, s, p, g, m, v, n_sparse, n, state, lr,
                     beta1, beta2, eps, 1.0f, shadow);
  hipLaunchKernelGGL(dssm::k_rnn_adam_advance, dim3(1), dim3(64), 0, s, state, beta1, beta2);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DSSM_OK : rerr(DSSM_E_HIP, hipGetErrorString(e));
}

int dssm_rnn_adam(float* p, const float* g, float* m, float* v, int64_t n_sparse, int64_t n,
                  float* state, float lr, float beta1, float beta2, float eps, void* stream) {
  return dssm_rnn_adam_ex(p, g, m, v, n_sparse, n, state, lr, beta1, beta2, eps, nullptr, stream);
}

}  // extern "C"

extern "C" int dssm_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                              float beta1, float beta2, float eps, float* state, float grad_scale,
                              int advance, void* stream) {
  if (!p || !g || !m || !v || !state || n < 0) return rerr(DSSM_E_INVALID, "adam_step: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096));
  const bool probe = dssm::adam_probe_begin(s);
  hipLaunchKernelGGL(dssm::k_rnn_adam, dim3(grid), dim3(256), 0, s, p, g, m, v, (int64_t)0, n, state, lr,
                     beta1, beta2, eps, grad_scale, nullptr);
  if (probe) dssm::adam_probe_end(s);
  if (advance) hipLaunchKernelGGL(dssm::k_rnn_adam_advance, dim3(1), dim3(64), 0, s, state, beta1, beta2);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DSSM_OK : rerr(DSSM_E_HIP, hipGetErrorString(e));
}

extern "C" int dssm_adam_step_shadow(float* p, const float* g, float* m, float* v, const int64_t* ranges, int nr,
                                     float lr, float beta1, float beta2, float eps, float* state, float grad_scale,
                                     int advance, const dssm_shadow_seg* segs, int nseg, void* stream) {
  if (!p || !g || !m || !v || !state || !ranges || nr < 1 || nr > 2 || nseg < 0 || nseg > 4 || (nseg && !segs))
    return rerr(DSSM_E_INVALID, "adam_step_shadow: bad argument");
  dssm::AdamRanges rg{};
  rg.nr = nr;
  for (int k = 0; k < nr; ++k) {
    const int64_t b = ranges[2 * k], e = ranges[2 * k + 1];
    if (b < 0 || e < b || b % 4 || e % 4) return rerr(DSSM_E_INVALID, "adam_step_shadow: ranges are 4-aligned");
    rg.b4[k] = b / 4;
    rg.n4[k] = (e - b) / 4;
  }
  dssm::ShadowList sh{};
  sh.count = nseg;
  for (int i = 0; i < nseg; ++i) {
    const dssm_shadow_seg& q = segs[i];
    if (!q.ptr || q.offset < 0 || q.rows < 0 || q.cols <= 0 || q.ld < q.cols)
      return rerr(DSSM_E_INVALID, "adam_step_shadow: bad shadow segment");
    sh.seg[i] = dssm::ShadowSeg{q.offset, q.rows, q.cols, q.ld, q.ptr, nullptr, 0};
  }
  hipStream_t s = (hipStream_t)stream;
  const bool probe = dssm::adam_probe_begin(s);
  hipError_t e = dssm::launch_adam_flat_shadow(p, g, m, v, rg, state, lr, beta1, beta2, eps, grad_scale, sh, s);
  if (e != hipSuccess) return rerr(DSSM_E_INVALID, "adam_step_shadow: 16-B alignment, segment offsets / widths");
  if (probe) dssm::adam_probe_end(s);
  if (advance) hipLaunchKernelGGL(dssm::k_rnn_adam_advance, dim3(1), dim3(64), 0, s, state, beta1, beta2);
  e = hipGetLastError();
  return e == hipSuccess ? DSSM_OK : rerr(DSSM_E_HIP, hipGetErrorString(e));
}

extern "C" int dssm_adam_advance(float* state, float beta1, float beta2, void* stream) {
  if (!state) return rerr(DSSM_E_INVALID, "adam_advance: bad argument");
  hipLaunchKernelGGL(dssm::k_rnn_adam_advance, dim3(1), dim3(64), 0, (hipStream_t)stream, state, beta1, beta2);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DSSM_OK : rerr(DSSM_E_HIP, hipGetErrorString(e));
}

extern "C" int dssm_adam_probe(int n_max) {
  for (hipEvent_t e : g_adam_probe.ev) (void)hipEventDestroy(e);
  g_adam_probe.ev.clear();
  g_adam_probe.used = 0;
  for (int i = 0; i < 2 * n_max; ++i) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return rerr(DSSM_E_HIP, "adam_probe: hipEventCreate");
    g_adam_probe.ev.push_back(e);
  }
  return DSSM_OK;
}

extern "C" int dssm_adam_probe_span(int first, int n, double* span_ms) {
  if (!span_ms || first < 0 || n < 1 || first + n > g_adam_probe.used)
    return rerr(DSSM_E_INVALID, "adam_probe_span: bad argument");
  // launches first .. first+n-1 (e.g. concurrent ones on several streams): latest end - earliest
  // start, both relative to the first launch's start event
  double lo = 0.0, hi = 0.0;
  for (int i = first; i < first + n; ++i) {
    float s = 0.f, e = 0.f;
    if (hipEventSynchronize(g_adam_probe.ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(&s, g_adam_probe.ev[2 * first], g_adam_probe.ev[2 * i]) != hipSuccess ||
        hipEventElapsedTime(&e, g_adam_probe.ev[2 * first], g_adam_probe.ev[2 * i + 1]) != hipSuccess)
      return rerr(DSSM_E_HIP, "adam_probe_span: event");
    lo = std::min(lo, (double)s);
    hi = std::max(hi, (double)e);
  }
  *span_ms = hi - lo;
  return DSSM_OK;
}

extern "C" int dssm_adam_probe_read(double* avg_ms, int* count) {
  if (!avg_ms || !count) return rerr(DSSM_E_INVALID, "adam_probe_read: bad argument");
  double tot = 0.0;
  for (int i = 0; i < g_adam_probe.used; ++i) {
    float ms = 0.f;
    if (hipEventSynchronize(g_adam_probe.ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(&ms, g_adam_probe.ev[2 * i], g_adam_probe.ev[2 * i + 1]) != hipSuccess)
      return rerr(DSSM_E_HIP, "adam_probe_read: event");
    tot += ms;
  }
  *count = g_adam_probe.used;
  *avg_ms = g_adam_probe.used ? tot / g_adam_probe.used : 0.0;
  return DSSM_OK;
}
