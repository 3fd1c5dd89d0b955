// bf16 perf mode of the RNN tower (semantic_matching/dssm_rnn/dssm_rnn.py:100-217, SURVEY §8(f)
// row 4): the bidirectional GRU's recurrences on the matrix cores.
//
// The fp32 kernels of rnn.hip stream every weight row from L2 for each 8 sequences and step
// (≈25 TFLOP/s).  Here a workgroup of H/16 waves owns M = 16·MT sequences of one direction for all
// T steps and keeps BOTH weight matrices of its direction resident in VGPRs as bf16 MFMA B
// fragments for the whole launch (wave w owns output columns 16w..16w+15 of every H-wide block:
// the r and u gate columns, the candidate column, 96 VGPRs at E = H = 128).  Only the A operands
// ([x_t | h], [x_t | r*h]) pass through LDS, and each lane keeps its 4·MT (row, column) states in
// fp32 registers in the MFMA accumulator layout (col = lane & 15, row = 4 (lane >> 4) + i), which
// is also the layout the gates come out in, so the elementwise GRU update never leaves the lane.
//
// Per step (v_mfma_f32_16x16x32_bf16, fp32 accumulation):
//   P1  [x_t | h] · [Wg | Wc_x]   -> r, u (sigmoid), the candidate's x part
//   P2  (r*h) · Wc_h              -> c = tanh(...), h' = u h + (1 - u) c (carried past the length)
// The BPTT kernel mirrors it with the transposed products (dc · Wc^T, [dr | du] · Wg^T), the
// lane-local gate derivatives and the embedding gradient as fp32 atomics from the x columns.
// Saved for the backward: [x_t | h_{t-1}] and r*h_{t-1} row-major (the weight-gradient GEMMs'
// A operands) and (r, u, c, h_{t-1}) in the accumulator layout (read back by the same lane of
// the BPTT kernel as two 16-B loads); BPTT writes [dr | du] and dc row-major for the GEMMs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/dssm.h"
#include "common.h"
#include "launch.h"

namespace dssm {
int report_error(int code, const char* msg);
}

namespace dssm {
namespace {

struct GruDimsB {
  int R, T;
};

template <int E, int H, int MT>
struct Geo {
  static constexpr int K = E + H, KC = K / 32, XC = E / 32, HC = H / 32, NW = H / 16, NT = NW * 64;
  static constexpr int M = 16 * MT;
  static constexpr int LDA = K + 8, LDR = H + 8, LDG = 2 * H + 8;  // LDS row strides (u16)
};

__device__ __forceinline__ float fsig(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ float ftanh(float x) { return 1.0f - 2.0f / (__expf(2.0f * x) + 1.0f); }

__device__ __forceinline__ unsigned pk2(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}
__device__ __forceinline__ float lo16(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float hi16(unsigned v) { return __uint_as_float(v & 0xffff0000u); }

// one bf16 B fragment from a row-major fp32 matrix: element j = W[(k0 + j) * ld + n] (stride) or
// W[n * ld + k0 + j] (contiguous, the transposed use)
__device__ __forceinline__ bf16x8 frag_strided(const float* W, int ld, int k0, int n) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)W[(size_t)(k0 + j) * ld + n];
  return f;
}
__device__ __forceinline__ bf16x8 frag_contig(const float* W, int ld, int k0, int n) {
  const float4 a = *reinterpret_cast<const float4*>(W + (size_t)n * ld + k0);
  const float4 b = *reinterpret_cast<const float4*>(W + (size_t)n * ld + k0 + 4);
  bf16x8 f;
  f[0] = (__bf16)a.x; f[1] = (__bf16)a.y; f[2] = (__bf16)a.z; f[3] = (__bf16)a.w;
  f[4] = (__bf16)b.x; f[5] = (__bf16)b.y; f[6] = (__bf16)b.z; f[7] = (__bf16)b.w;
  return f;
}

__device__ __forceinline__ bf16x8 lds_frag(const u16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// token of row `row` at step t of direction dir (reversed within the row's length; padding steps
// read token 0's slot, their results are masked)
__device__ __forceinline__ int tok(const int* sIds, const int* sLen, int row, int t, int T, int dir) {
  const int L = sLen[row];
  const int idx = t < L ? (dir ? L - 1 - t : t) : 0;
  return sIds[row * T + idx];
}

// ---- forward -----------------------------------------------------------------------------------
// grid (ceil(R / M), 2 directions), NT threads.  Wg: [(K+1) x 2H], Wc: [(K+1) x H] fp32 (last row
// bias).  XH [dir][t][R][K], RH [dir][t][R][H] (u16), GF [dir][t][NB][NW][64][16] (u16), out [R x ldo]
// fp32 final states (fw in [0, H), bw in [H, 2H)).
template <int E, int H, int MT>
__global__ __launch_bounds__(H / 16 * 64) void k_gru_fwd_mfma(
    GruDimsB d, const int* __restrict__ ids, const int* __restrict__ lens, const u16* __restrict__ emb16,
    const float* __restrict__ wg_fw, const float* __restrict__ wc_fw, const float* __restrict__ wg_bw,
    const float* __restrict__ wc_bw, u16* __restrict__ XH, u16* __restrict__ RH, u16* __restrict__ GF,
    float* __restrict__ out, int ldo) {
  using G = Geo<E, H, MT>;
  constexpr int K = G::K, KC = G::KC, XC = G::XC, HC = G::HC, NW = G::NW, NT = G::NT, M = G::M;
  constexpr int LDA = G::LDA, LDR = G::LDR;
  constexpr int EC8 = E / 8, HC8 = H / 8, NXQ = M * EC8, XPT = (NXQ + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) u16 sA[M * LDA];  // [x_t | h_{t-1}]
  __shared__ __attribute__((aligned(16))) u16 sR[M * LDR];  // r * h_{t-1}
  extern __shared__ int sDyn[];                              // lens [M], ids [M][T]
  int* sLen = sDyn;
  int* sIds = sDyn + M;

  const int T = d.T, R = d.R, dir = blockIdx.y;
  const float* Wg = dir ? wg_bw : wg_fw;
  const float* Wc = dir ? wc_bw : wc_fw;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lc = lane & 15, lg = lane >> 4;
  const int r0 = blockIdx.x * M, nrow = min(M, R - r0);
  for (int i = tid; i < M; i += NT) sLen[i] = i < nrow ? lens[r0 + i] : 0;
  for (int i = tid; i < M * T; i += NT) sIds[i] = i < nrow * T ? ids[(size_t)r0 * T + i] : 0;

  // this wave's weight columns as bf16 B fragments, resident for all T steps
  const int gcol = 16 * w + lc;
  bf16x8 bR[KC], bU[KC], bC[KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const int k0 = 32 * c + 8 * lg;
    bR[c] = frag_strided(Wg, 2 * H, k0, gcol);
    bU[c] = frag_strided(Wg, 2 * H, k0, H + gcol);
    bC[c] = frag_strided(Wc, H, k0, gcol);
  }
  const float biasR = Wg[(size_t)K * 2 * H + gcol], biasU = Wg[(size_t)K * 2 * H + H + gcol];
  const float biasC = Wc[(size_t)K * H + gcol];
  __syncthreads();

  int len_r[MT][4];
  float hs[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      len_r[m][i] = sLen[16 * m + 4 * lg + i];
      hs[m][i] = 0.f;
    }
  // x_0 and h_{-1} = 0
  uint4 xr[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int q = tid + i * NT;
    if (q < NXQ) {
      const int row = q / EC8, c8 = q - row * EC8;
      xr[i] = *reinterpret_cast<const uint4*>(emb16 + (size_t)tok(sIds, sLen, row, 0, T, dir) * E + c8 * 8);
      *reinterpret_cast<uint4*>(&sA[row * LDA + c8 * 8]) = xr[i];
    }
  }
  for (int i = tid; i < M * HC8; i += NT) {
    const int row = i / HC8, c8 = i - row * HC8;
    *reinterpret_cast<uint4*>(&sA[row * LDA + E + c8 * 8]) = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();

  const size_t plane = (size_t)T * R;
  const int NB = (R + 15) / 16;
  for (int t = 0; t < T; ++t) {
    // next step's input rows in flight during this step
    if (t + 1 < T) {
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int q = tid + i * NT;
        if (q < NXQ) {
          const int row = q / EC8, c8 = q - row * EC8;
          xr[i] = *reinterpret_cast<const uint4*>(emb16 + (size_t)tok(sIds, sLen, row, t + 1, T, dir) * E +
                                                  c8 * 8);
        }
      }
    }
    // P1: gates and the candidate's x part
    f32x4 ar[MT], au[MT], ac[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      ar[m] = f32x4{biasR, biasR, biasR, biasR};
      au[m] = f32x4{biasU, biasU, biasU, biasU};
      ac[m] = f32x4{biasC, biasC, biasC, biasC};
    }
#pragma unroll
    for (int c = 0; c < KC; ++c) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const bf16x8 a = lds_frag(&sA[(16 * m + lc) * LDA + 32 * c + 8 * lg]);
        ar[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bR[c], ar[m], 0, 0, 0);
        au[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bU[c], au[m], 0, 0, 0);
        if (c < XC) ac[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bC[c], ac[m], 0, 0, 0);
      }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float rv = fsig(ar[m][i]), uv = fsig(au[m][i]);
        ar[m][i] = rv;
        au[m][i] = uv;
        sR[(16 * m + 4 * lg + i) * LDR + gcol] = f2bf(rv * hs[m][i]);
      }
    __syncthreads();
    // save [x_t | h_{t-1}] and r*h_{t-1}; the x slots take x_{t+1} (same thread, same chunk)
    const size_t rowbase = (size_t)dir * plane + (size_t)t * R + r0;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int q = tid + i * NT;
      if (q < NXQ) {
        const int row = q / EC8, c8 = q - row * EC8;
        uint4* p = reinterpret_cast<uint4*>(&sA[row * LDA + c8 * 8]);
        if (row < nrow) *reinterpret_cast<uint4*>(XH + (rowbase + row) * K + c8 * 8) = *p;
        if (t + 1 < T) *p = xr[i];
      }
    }
    for (int i = tid; i < M * HC8; i += NT) {
      const int row = i / HC8, c8 = i - row * HC8;
      if (row < nrow) {
        *reinterpret_cast<uint4*>(XH + (rowbase + row) * K + E + c8 * 8) =
            *reinterpret_cast<const uint4*>(&sA[row * LDA + E + c8 * 8]);
        *reinterpret_cast<uint4*>(RH + (rowbase + row) * H + c8 * 8) =
            *reinterpret_cast<const uint4*>(&sR[row * LDR + c8 * 8]);
      }
    }
    // P2: the candidate's state part
#pragma unroll
    for (int c = 0; c < HC; ++c)
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const bf16x8 a = lds_frag(&sR[(16 * m + lc) * LDR + 32 * c + 8 * lg]);
        ac[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bC[XC + c], ac[m], 0, 0, 0);
      }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float cv[4], h0[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        cv[i] = ftanh(ac[m][i]);
        h0[i] = hs[m][i];
        const float uv = au[m][i];
        if (t < len_r[m][i]) hs[m][i] = uv * h0[i] + (1.0f - uv) * cv[i];
        sA[(16 * m + 4 * lg + i) * LDA + E + gcol] = f2bf(hs[m][i]);
      }
      const int blk = r0 / 16 + m;
      if (blk < NB) {
        uint4* g = reinterpret_cast<uint4*>(
            GF + ((((size_t)dir * T + t) * NB + blk) * NW + w) * 1024 + (size_t)lane * 16);
        g[0] = make_uint4(pk2(ar[m][0], ar[m][1]), pk2(ar[m][2], ar[m][3]), pk2(au[m][0], au[m][1]),
                          pk2(au[m][2], au[m][3]));
        g[1] = make_uint4(pk2(cv[0], cv[1]), pk2(cv[2], cv[3]), pk2(h0[0], h0[1]), pk2(h0[2], h0[3]));
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * m + 4 * lg + i;
      if (row < nrow) out[(size_t)(r0 + row) * ldo + dir * H + gcol] = hs[m][i];
    }
}

// ---- BPTT --------------------------------------------------------------------------------------
// Same grid.  dout [R x ldo] fp32.  Writes DG [dir][t][R][2H] = (dr, du) and DC [dir][t][R][H]
// (u16; zero at a row's padding steps) and adds dx into demb (fp32 atomics).
template <int E, int H, int MT>
__global__ __launch_bounds__(H / 16 * 64) void k_gru_bwd_mfma(
    GruDimsB d, const int* __restrict__ ids, const int* __restrict__ lens, const float* __restrict__ wg_fw,
    const float* __restrict__ wc_fw, const float* __restrict__ wg_bw, const float* __restrict__ wc_bw,
    const float* __restrict__ dout, int ldo, const u16* __restrict__ GF, u16* __restrict__ DG,
    u16* __restrict__ DC, float* __restrict__ demb) {
  using G = Geo<E, H, MT>;
  constexpr int HC = G::HC, NW = G::NW, NT = G::NT, M = G::M, LDR = G::LDR, LDG = G::LDG;
  constexpr int HC8 = H / 8;
  __shared__ __attribute__((aligned(16))) u16 sC[M * LDR];  // dc
  __shared__ __attribute__((aligned(16))) u16 sG[M * LDG];  // [dr | du]
  extern __shared__ int sDyn[];
  int* sLen = sDyn;
  int* sIds = sDyn + M;

  const int T = d.T, R = d.R, dir = blockIdx.y;
  const float* Wg = dir ? wg_bw : wg_fw;
  const float* Wc = dir ? wc_bw : wc_fw;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lc = lane & 15, lg = lane >> 4;
  const int r0 = blockIdx.x * M, nrow = min(M, R - r0);
  for (int i = tid; i < M; i += NT) sLen[i] = i < nrow ? lens[r0 + i] : 0;
  for (int i = tid; i < M * T; i += NT) sIds[i] = i < nrow * T ? ids[(size_t)r0 * T + i] : 0;

  // transposed products: B[k = gate/candidate column][n = input column] = W[n][k] (contiguous)
  const int gcol = 16 * w + lc;
  const bool hasx = 16 * w < E;  // wave-uniform: this wave also owns x columns 16w..16w+15
  const int kh = E + gcol, kx = hasx ? gcol : 0;
  bf16x8 c1h[HC], c1x[HC], c2h[2 * HC], c2x[2 * HC];
#pragma unroll
  for (int c = 0; c < HC; ++c) {
    c1h[c] = frag_contig(Wc, H, 32 * c + 8 * lg, kh);
    c1x[c] = frag_contig(Wc, H, 32 * c + 8 * lg, kx);
  }
#pragma unroll
  for (int c = 0; c < 2 * HC; ++c) {
    c2h[c] = frag_contig(Wg, 2 * H, 32 * c + 8 * lg, kh);
    c2x[c] = frag_contig(Wg, 2 * H, 32 * c + 8 * lg, kx);
  }
  __syncthreads();

  float dh[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * m + 4 * lg + i;
      dh[m][i] = row < nrow ? dout[(size_t)(r0 + row) * ldo + dir * H + gcol] : 0.f;
    }
  const size_t plane = (size_t)T * R;
  const int NB = (R + 15) / 16;
  auto gf_ptr = [&](int t, int m) {
    const int blk = min(r0 / 16 + m, NB - 1);
    return reinterpret_cast<const uint4*>(GF + ((((size_t)dir * T + t) * NB + blk) * NW + w) * 1024 +
                                          (size_t)lane * 16);
  };
  // (r, u, c, h_{t-1}) of the current step, packed; the previous step's are loaded into the same
  // registers once P1's epilogue has used them, and stay in flight across P2 and the stores
  uint4 gf[MT][2];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    gf[m][0] = gf_ptr(T - 1, m)[0];
    gf[m][1] = gf_ptr(T - 1, m)[1];
  }
  for (int t = T - 1; t >= 0; --t) {
    float dhp[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const uint4 g0 = gf[m][0], g1 = gf[m][1];
      const float uv[4] = {lo16(g0.z), hi16(g0.z), lo16(g0.w), hi16(g0.w)};
      const float cv[4] = {lo16(g1.x), hi16(g1.x), lo16(g1.y), hi16(g1.y)};
      const float h0[4] = {lo16(g1.z), hi16(g1.z), lo16(g1.w), hi16(g1.w)};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 16 * m + 4 * lg + i;
        const bool act = t < sLen[row];
        const float dhn = act ? dh[m][i] : 0.f;
        const float dcv = dhn * (1.0f - uv[i]) * (1.0f - cv[i] * cv[i]);
        const float duv = dhn * (h0[i] - cv[i]) * uv[i] * (1.0f - uv[i]);
        dhp[m][i] = act ? dhn * uv[i] : dh[m][i];
        sC[row * LDR + gcol] = f2bf(dcv);
        sG[row * LDG + H + gcol] = f2bf(duv);
      }
    }
    __syncthreads();
    // P1: dc · Wc^T -> state part (the reset gate's and the state's gradient through r*h) and x part
    f32x4 ah[MT], ax[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      ah[m] = f32x4{0.f, 0.f, 0.f, 0.f};
      ax[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int c = 0; c < HC; ++c)
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const bf16x8 a = lds_frag(&sC[(16 * m + lc) * LDR + 32 * c + 8 * lg]);
        ah[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, c1h[c], ah[m], 0, 0, 0);
        if (hasx) ax[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, c1x[c], ax[m], 0, 0, 0);
      }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const uint4 g0 = gf[m][0], g1 = gf[m][1];
      const float rv[4] = {lo16(g0.x), hi16(g0.x), lo16(g0.y), hi16(g0.y)};
      const float h0[4] = {lo16(g1.z), hi16(g1.z), lo16(g1.w), hi16(g1.w)};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float drh = ah[m][i];
        sG[(16 * m + 4 * lg + i) * LDG + gcol] = f2bf(drh * h0[i] * rv[i] * (1.0f - rv[i]));
        dhp[m][i] += drh * rv[i];
      }
    }
    if (t > 0) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        gf[m][0] = gf_ptr(t - 1, m)[0];
        gf[m][1] = gf_ptr(t - 1, m)[1];
      }
    }
    __syncthreads();
    // save dc and [dr | du] for the weight-gradient GEMMs
    const size_t rowbase = (size_t)dir * plane + (size_t)t * R + r0;
    for (int i = tid; i < M * HC8; i += NT) {
      const int row = i / HC8, c8 = i - row * HC8;
      if (row < nrow)
        *reinterpret_cast<uint4*>(DC + (rowbase + row) * H + c8 * 8) =
            *reinterpret_cast<const uint4*>(&sC[row * LDR + c8 * 8]);
    }
    for (int i = tid; i < M * 2 * HC8; i += NT) {
      const int row = i / (2 * HC8), c8 = i - row * 2 * HC8;
      if (row < nrow)
        *reinterpret_cast<uint4*>(DG + (rowbase + row) * 2 * H + c8 * 8) =
            *reinterpret_cast<const uint4*>(&sG[row * LDG + c8 * 8]);
    }
    // P2: [dr | du] · Wg^T -> state part (+ dhp = the gradient before step t) and x part
    f32x4 a2[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) a2[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 2 * HC; ++c)
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const bf16x8 a = lds_frag(&sG[(16 * m + lc) * LDG + 32 * c + 8 * lg]);
        a2[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, c2h[c], a2[m], 0, 0, 0);
        if (hasx) ax[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, c2x[c], ax[m], 0, 0, 0);
      }
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) dh[m][i] = dhp[m][i] + a2[m][i];
    if (hasx) {
      using gfloat = __attribute__((address_space(1))) float;
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 16 * m + 4 * lg + i;
          if (t < sLen[row])
            __hip_atomic_fetch_add((gfloat*)(demb + (size_t)tok(sIds, sLen, row, t, T, dir) * E + gcol),
                                   ax[m][i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
  }
}

__global__ void k_to_bf16(const float* __restrict__ x, u16* __restrict__ y, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 a = *reinterpret_cast<const float4*>(x + 8 * i);
    const float4 b = *reinterpret_cast<const float4*>(x + 8 * i + 4);
    *reinterpret_cast<uint4*>(y + 8 * i) = make_uint4(pk2(a.x, a.y), pk2(a.z, a.w), pk2(b.x, b.y), pk2(b.z, b.w));
  }
}

// ---- workspace and dispatch -------------------------------------------------------------------
struct WsB {
  u16 *XH, *RH, *GF, *DG, *DC, *emb16;
  float* slab;
  size_t bytes;
};

size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

WsB ws_layout(char* base, int R, int T, int E, int H, int V) {
  const size_t TR = (size_t)T * R, K = (size_t)E + H, NB = (R + 15) / 16;
  WsB w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += al256(bytes);
    return p;
  };
  w.XH = (u16*)take(2 * TR * K * 2);
  w.RH = (u16*)take(2 * TR * H * 2);
  w.GF = (u16*)take(2 * (size_t)T * NB * 16 * H * 4 * 2);
  w.DG = (u16*)take(2 * TR * 2 * H * 2);
  w.DC = (u16*)take(2 * TR * H * 2);
  w.emb16 = (u16*)take((size_t)V * E * 2);
  const size_t slab = std::max({gemm_dw_slab_floats((int)K + 1, 2 * H, (int)TR, true),
                                gemm_dw_slab_floats(E, H, (int)TR, true),
                                gemm_dw_slab_floats(H + 1, H, (int)TR, true)});
  w.slab = (float*)take(slab * 4 + 64);
  w.bytes = off;
  return w;
}

bool shape_ok(int E, int H) { return (E == 128 && H == 128) || (E == 64 && H == 128) || (E == 32 && H == 32); }

// sequences per workgroup: fewest rounds of the 256 CUs (one workgroup per CU), then the fewest
// MFMA tiles per step
int pick_mt(int R) {
  int best = 1;
  double best_cost = 1e30;
  for (int mt = 1; mt <= 4; ++mt) {
    const int wgs = 2 * ((R + 16 * mt - 1) / (16 * mt));
    const double cost = (double)((wgs + 255) / 256) * (mt + 1.5);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = mt;
    }
  }
  return best;
}

template <int E, int H, int MT>
void launch_fwd_t(const GruDimsB& d, const int* ids, const int* lens, const u16* emb16, const float* const* w,
                  const WsB& ws, float* y, int ldy, hipStream_t s) {
  constexpr int M = 16 * MT;
  const size_t dyn = sizeof(int) * (size_t)M * (1 + d.T);
  hipLaunchKernelGGL((k_gru_fwd_mfma<E, H, MT>), dim3((d.R + M - 1) / M, 2), dim3(Geo<E, H, MT>::NT), dyn, s, d,
                     ids, lens, emb16, w[0], w[1], w[2], w[3], ws.XH, ws.RH, ws.GF, y, ldy);
}

template <int E, int H, int MT>
void launch_bwd_t(const GruDimsB& d, const int* ids, const int* lens, const float* const* w, const float* dy,
                  int lddy, const WsB& ws, float* demb, hipStream_t s) {
  constexpr int M = 16 * MT;
  const size_t dyn = sizeof(int) * (size_t)M * (1 + d.T);
  hipLaunchKernelGGL((k_gru_bwd_mfma<E, H, MT>), dim3((d.R + M - 1) / M, 2), dim3(Geo<E, H, MT>::NT), dyn, s, d,
                     ids, lens, w[0], w[1], w[2], w[3], dy, lddy, ws.GF, ws.DG, ws.DC, demb);
}

template <int E, int H>
void dispatch_fwd(int mt, const GruDimsB& d, const int* ids, const int* lens, const u16* emb16,
                  const float* const* w, const WsB& ws, float* y, int ldy, hipStream_t s) {
  switch (mt) {
    case 1: launch_fwd_t<E, H, 1>(d, ids, lens, emb16, w, ws, y, ldy, s); break;
    case 2: launch_fwd_t<E, H, 2>(d, ids, lens, emb16, w, ws, y, ldy, s); break;
    case 3: launch_fwd_t<E, H, 3>(d, ids, lens, emb16, w, ws, y, ldy, s); break;
    default: launch_fwd_t<E, H, 4>(d, ids, lens, emb16, w, ws, y, ldy, s); break;
  }
}

template <int E, int H>
void dispatch_bwd(int mt, const GruDimsB& d, const int* ids, const int* lens, const float* const* w,
                  const float* dy, int lddy, const WsB& ws, float* demb, hipStream_t s) {
  switch (mt) {
    case 1: launch_bwd_t<E, H, 1>(d, ids, lens, w, dy, lddy, ws, demb, s); break;
    case 2: launch_bwd_t<E, H, 2>(d, ids, lens, w, dy, lddy, ws, demb, s); break;
    case 3: launch_bwd_t<E, H, 3>(d, ids, lens, w, dy, lddy, ws, demb, s); break;
    default: launch_bwd_t<E, H, 4>(d, ids, lens, w, dy, lddy, ws, demb, s); break;
  }
}

}  // namespace
}  // namespace dssm

// ---- C-ABI -------------------------------------------------------------------------------------
namespace {
int rerr_b(int code, const char* m) { return dssm::report_error(code, m); }
}

extern "C" {

int dssm_rnn_bf16_supported(int E, int H) { return dssm::shape_ok(E, H) ? 1 : 0; }

size_t dssm_rnn_bf16_ws_bytes(int R, int T, int E, int H, int V) {
  if (R <= 0 || T <= 0 || V <= 0 || !dssm::shape_ok(E, H)) return 0;
  return dssm::ws_layout(nullptr, R, T, E, H, V).bytes;
}

int dssm_rnn_bf16_forward(const int32_t* ids, const int32_t* lens, int R, int T, const float* emb, int V,
                          int E, int H, const float* const* w, void* ws, float* y, int ldy, void* stream) {
  if (!ids || !lens || !emb || !w || !ws || !y || R <= 0 || T <= 0 || V <= 0 || !dssm::shape_ok(E, H) ||
      ldy < 2 * H)
    return rerr_b(DSSM_E_INVALID, "rnn_bf16_forward: bad argument or unsupported (E, H)");
  hipStream_t s = (hipStream_t)stream;
  const dssm::WsB L = dssm::ws_layout((char*)ws, R, T, E, H, V);
  const int64_t n8 = (int64_t)V * E / 8;
  hipLaunchKernelGGL(dssm::k_to_bf16, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((n8 + 255) / 256, 2048))),
                     dim3(256), 0, s, emb, L.emb16, n8);
  const dssm::GruDimsB d{R, T};
  const int mt = dssm::pick_mt(R);
  if (E == 128)
    dssm::dispatch_fwd<128, 128>(mt, d, ids, lens, L.emb16, w, L, y, ldy, s);
  else if (E == 64)
    dssm::dispatch_fwd<64, 128>(mt, d, ids, lens, L.emb16, w, L, y, ldy, s);
  else
    dssm::dispatch_fwd<32, 32>(mt, d, ids, lens, L.emb16, w, L, y, ldy, s);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DSSM_OK : rerr_b(DSSM_E_HIP, hipGetErrorString(e));
}

int dssm_rnn_bf16_backward(const int32_t* ids, const int32_t* lens, int R, int T, int V, int E, int H,
                           const float* const* w, const float* dy, int lddy, void* ws, float* demb,
                           float* const* gw, void* stream) {
  if (!ids || !lens || !w || !dy || !ws || !demb || !gw || R <= 0 || T <= 0 || V <= 0 ||
      !dssm::shape_ok(E, H) || lddy < 2 * H)
    return rerr_b(DSSM_E_INVALID, "rnn_bf16_backward: bad argument or unsupported (E, H)");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(demb, 0, sizeof(float) * (size_t)V * E, s) != hipSuccess)
    return rerr_b(DSSM_E_HIP, "rnn_bf16_backward: hipMemsetAsync");
  const dssm::WsB L = dssm::ws_layout((char*)ws, R, T, E, H, V);
  const dssm::GruDimsB d{R, T};
  const int mt = dssm::pick_mt(R);
  if (E == 128)
    dssm::dispatch_bwd<128, 128>(mt, d, ids, lens, w, dy, lddy, L, demb, s);
  else if (E == 64)
    dssm::dispatch_bwd<64, 128>(mt, d, ids, lens, w, dy, lddy, L, demb, s);
  else
    dssm::dispatch_bwd<32, 32>(mt, d, ids, lens, w, dy, lddy, L, demb, s);
  // [W; b] gradients: split-K bf16 TN GEMMs over all T*R (step, row) pairs; the ones row = bias.
  //   dWg = [x | h]^T [dr | du];  dWc = [x ; r*h]^T dc in two row blocks (x rows, then state rows + bias)
  const int K = E + H, TR = T * R;
  const size_t half = (size_t)TR;
  for (int dir = 0; dir < 2; ++dir) {
    const u16* XH = L.XH + half * dir * K;
    hipError_t e = dssm::launch_gemm(dssm::GEMM_DW, true, K + 1, 2 * H, TR, XH, K, L.DG + half * dir * 2 * H,
                                     2 * H, gw[2 * dir], 2 * H, nullptr, true, L.slab, s, nullptr);
    if (e == hipSuccess)
      e = dssm::launch_gemm(dssm::GEMM_DW, true, E, H, TR, XH, K, L.DC + half * dir * H, H, gw[2 * dir + 1], H,
                            nullptr, false, L.slab, s, nullptr);
    if (e == hipSuccess)
      e = dssm::launch_gemm(dssm::GEMM_DW, true, H + 1, H, TR, L.RH + half * dir * H, H, L.DC + half * dir * H,
                            H, gw[2 * dir + 1] + (size_t)E * H, H, nullptr, true, L.slab, s, nullptr);
    if (e != hipSuccess) return rerr_b(DSSM_E_HIP, hipGetErrorString(e));
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DSSM_OK : rerr_b(DSSM_E_HIP, hipGetErrorString(e));
}

}  // extern "C"
