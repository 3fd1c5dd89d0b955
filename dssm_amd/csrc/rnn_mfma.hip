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
// Saved for the backward: h_{t-1} and r*h_{t-1} row-major and the step's token per row (the
// weight-gradient kernel's A operands; x_t is re-gathered from the bf16 embedding copy by token), and
// (r, u, c, h_{t-1}) in the accumulator layout (read back by the same lane of the BPTT kernel as two
// 16-B loads); BPTT writes [dr | du], dc and dx row-major.
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

// v_exp_f32 + v_rcp_f32 (1 ulp): the IEEE division sequence was half of the forward's VALU work
__device__ __forceinline__ float fsig(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float ftanh(float x) {
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(__expf(2.0f * x) + 1.0f);
}

__device__ __forceinline__ unsigned pk2(float a, float b) { return pack2bf(a, b); }
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
// bias).  HS, RH [dir][t][R][H] (u16: h_{t-1}, r*h_{t-1}), TOK [dir][t][R] (int: the token of x_t),
// GA [dir][t][NB][NW][64][8] (u16: r, u), GC [dir][t][NB][NW][64][8] (u16: c, h_{t-1}), out [R x ldo] fp32 final
// states (fw in [0, H), bw in [H, 2H)).
template <int E, int H, int MT>
__global__ __launch_bounds__(H / 16 * 64) void k_gru_fwd_mfma(
    GruDimsB d, const int* __restrict__ ids, const int* __restrict__ lens, const u16* __restrict__ emb16,
    const float* __restrict__ wg_fw, const float* __restrict__ wc_fw, const float* __restrict__ wg_bw,
    const float* __restrict__ wc_bw, u16* __restrict__ HS, u16* __restrict__ RH, int* __restrict__ TOK,
    u16* __restrict__ GA, u16* __restrict__ GC, float* __restrict__ out, int ldo) {
  using G = Geo<E, H, MT>;
  constexpr int K = G::K, KC = G::KC, XC = G::XC, HC = G::HC, NW = G::NW, NT = G::NT, M = G::M;
  constexpr int LDA = G::LDA, LDR = G::LDR;
  constexpr int EC8 = E / 8, HC8 = H / 8, NXQ = M * EC8, XPT = (NXQ + NT - 1) / NT;
  // [x_t | h_{t-1}], double-buffered by step parity: step t reads sA[t & 1] and fills sA[(t+1) & 1],
  // so the step needs two barriers (after the gates' r*h, after the state update), not three
  __shared__ __attribute__((aligned(16))) u16 sA[2][M * LDA];
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
  // x_0 and h_{-1} = 0.  A thread stages at most two 16-B chunks of x per step (x0, x1: named
  // registers, not an array, so nothing is indexed at run time)
  static_assert(XPT <= 2, "x staging: at most two chunks per thread");
  auto xsrc = [&](int q, int t) {
    const int row = q / EC8, c8 = q - row * EC8;
    return reinterpret_cast<const uint4*>(emb16 + (size_t)tok(sIds, sLen, row, t, T, dir) * E + c8 * 8);
  };
  auto xdst = [&](u16* A, int q) {
    const int row = q / EC8, c8 = q - row * EC8;
    return reinterpret_cast<uint4*>(&A[row * LDA + c8 * 8]);
  };
  const int q0 = tid, q1 = tid + NT;
  const bool has0 = q0 < NXQ, has1 = XPT > 1 && q1 < NXQ;
  uint4 x0 = make_uint4(0, 0, 0, 0), x1 = x0;
  if (has0) *xdst(sA[0], q0) = *xsrc(q0, 0);
  if (has1) *xdst(sA[0], q1) = *xsrc(q1, 0);
  for (int i = tid; i < M * HC8; i += NT) {
    const int row = i / HC8, c8 = i - row * HC8;
    *reinterpret_cast<uint4*>(&sA[0][row * LDA + E + c8 * 8]) = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();

  const size_t plane = (size_t)T * R;
  const int NB = (R + 15) / 16;
  for (int t = 0; t < T; ++t) {
    u16* A = sA[t & 1];
    u16* An = sA[(t + 1) & 1];
    // next step's input rows in flight during this step
    if (t + 1 < T) {
      if (has0) x0 = *xsrc(q0, t + 1);
      if (has1) x1 = *xsrc(q1, t + 1);
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
        const bf16x8 a = lds_frag(&A[(16 * m + lc) * LDA + 32 * c + 8 * lg]);
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
    // save x_t's token, h_{t-1} and r*h_{t-1}
    const size_t rowbase = (size_t)dir * plane + (size_t)t * R + r0;
    for (int row = tid; row < nrow; row += NT) TOK[rowbase + row] = tok(sIds, sLen, row, t, T, dir);
    for (int i = tid; i < M * HC8; i += NT) {
      const int row = i / HC8, c8 = i - row * HC8;
      if (row < nrow) {
        *reinterpret_cast<uint4*>(HS + (rowbase + row) * H + c8 * 8) =
            *reinterpret_cast<const uint4*>(&A[row * LDA + E + c8 * 8]);
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
    // x_{t+1} and h_t into the other buffer (last read by step t-1, before the previous barrier);
    // the x loads had the whole step to land
    if (t + 1 < T) {
      if (has0) *xdst(An, q0) = x0;
      if (has1) *xdst(An, q1) = x1;
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float cv[4], h0[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        cv[i] = ftanh(ac[m][i]);
        h0[i] = hs[m][i];
        const float uv = au[m][i];
        if (t < len_r[m][i]) hs[m][i] = uv * h0[i] + (1.0f - uv) * cv[i];
        An[(16 * m + 4 * lg + i) * LDA + E + gcol] = f2bf(hs[m][i]);
      }
      const int blk = r0 / 16 + m;
      if (blk < NB) {
        const size_t f = (((size_t)dir * T + t) * NB + blk) * NW + w;
        *reinterpret_cast<uint4*>(GA + f * 512 + (size_t)lane * 8) =
            make_uint4(pk2(ar[m][0], ar[m][1]), pk2(ar[m][2], ar[m][3]), pk2(au[m][0], au[m][1]),
                       pk2(au[m][2], au[m][3]));
        *reinterpret_cast<uint4*>(GC + f * 512 + (size_t)lane * 8) =
            make_uint4(pk2(cv[0], cv[1]), pk2(cv[2], cv[3]), pk2(h0[0], h0[1]), pk2(h0[2], h0[3]));
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
// Same grid.  dout [R x ldo] fp32.  Writes DG [dir][t][R][2H] = (dr, du), DC [dir][t][R][H] and the
// input gradient DX [dir][t][R][E] (u16; zero at a row's padding steps).  The embedding gradient is
// DX summed per token afterwards (k_emb_grad), not scattered with atomics here: 50M fp32 atomic adds
// per config-4 step would run at the chip's ~1.3 TB/s atomic rate (MI355X_MICROARCH.md).
template <int E, int H, int MT>
__global__ __launch_bounds__(H / 16 * 64) void k_gru_bwd_mfma(
    GruDimsB d, const int* __restrict__ ids, const int* __restrict__ lens, const float* __restrict__ wg_fw,
    const float* __restrict__ wc_fw, const float* __restrict__ wg_bw, const float* __restrict__ wc_bw,
    const float* __restrict__ dout, int ldo, const u16* __restrict__ GA, const u16* __restrict__ GC,
    u16* __restrict__ DG, u16* __restrict__ DC, u16* __restrict__ DX) {
  using G = Geo<E, H, MT>;
  constexpr int HC = G::HC, NW = G::NW, NT = G::NT, M = G::M, LDR = G::LDR, LDG = G::LDG;
  constexpr int HC8 = H / 8, EC8 = E / 8, LDX = E + 8;
  // dc, [dr | du] and dx tiles, double-buffered by step parity: two barriers per step (the next
  // step writes the other buffers), dx rows of step t stored after the first barrier of step t-1
  __shared__ __attribute__((aligned(16))) u16 sCb[2][M * LDR];
  __shared__ __attribute__((aligned(16))) u16 sGb[2][M * LDG];
  __shared__ __attribute__((aligned(16))) u16 sXb[2][M * LDX];
  extern __shared__ int sDyn[];
  int* sLen = sDyn;

  const int T = d.T, R = d.R, dir = blockIdx.y;
  const float* Wg = dir ? wg_bw : wg_fw;
  const float* Wc = dir ? wc_bw : wc_fw;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lc = lane & 15, lg = lane >> 4;
  const int r0 = blockIdx.x * M, nrow = min(M, R - r0);
  for (int i = tid; i < M; i += NT) sLen[i] = i < nrow ? lens[r0 + i] : 0;

  // transposed products: B[k = gate/candidate column][n = input column] = W[n][k] (contiguous)
  const int gcol = 16 * w + lc;
  // wave-uniform: this wave also owns x columns 16w..16w+15 (every wave when E >= H: a constant, so
  // the conditional MFMAs on ax compile without accumulator copies)
  const bool hasx = (E >= H) || 16 * w < E;
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
  // (r, u), (c) and h_{t-1} of the current step, packed; the previous step's are loaded into the same
  // registers once P1's epilogue has used them, and stay in flight across P2 and the stores
  struct Cache {
    uint4 ru, ch;  // (r, u), (c, h_{t-1})
  };
  auto load_cache = [&](int t, int m) {
    const int blk = min(r0 / 16 + m, NB - 1);
    const size_t f = (((size_t)dir * T + t) * NB + blk) * NW + w;
    Cache x;
    x.ru = *reinterpret_cast<const uint4*>(GA + f * 512 + (size_t)lane * 8);
    x.ch = *reinterpret_cast<const uint4*>(GC + f * 512 + (size_t)lane * 8);
    return x;
  };
  Cache gf[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) gf[m] = load_cache(T - 1, m);
  auto store_dx = [&](int t) {
    const u16* sX = sXb[t & 1];
    const size_t rb = (size_t)dir * plane + (size_t)t * R + r0;
    for (int i = tid; i < M * EC8; i += NT) {
      const int row = i / EC8, c8 = i - row * EC8;
      if (row < nrow)
        *reinterpret_cast<uint4*>(DX + (rb + row) * E + c8 * 8) =
            *reinterpret_cast<const uint4*>(&sX[row * LDX + c8 * 8]);
    }
  };
  for (int t = T - 1; t >= 0; --t) {
    u16* sC = sCb[t & 1];
    u16* sG = sGb[t & 1];
    u16* sX = sXb[t & 1];
    float dhp[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const uint4 g0 = gf[m].ru, g1 = gf[m].ch;
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
    if (t + 1 < T) store_dx(t + 1);  // written before this barrier, rewritten after the next one
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
      const uint4 g0 = gf[m].ru, g1 = gf[m].ch;
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
      for (int m = 0; m < MT; ++m) gf[m] = load_cache(t - 1, m);
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
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) sX[(16 * m + 4 * lg + i) * LDX + kx] = f2bf(ax[m][i]);
    }
  }
  __syncthreads();
  store_dx(0);
}

// ---- embedding gradient: dx summed per token -------------------------------------------------
// The batch's active (row, position) pairs bucketed by token (count, one-workgroup scan, fill), then
// one wave per token sums its positions' dx rows of both directions (fw at step s, bw at step
// len - 1 - s) in fp32 and writes the token's whole gradient row (zero for absent tokens).
// the batch's active positions bucketed by token: count (each position keeps its rank within its
// token: the returning atomic's value), exclusive scan (which re-zeroes the counts for the next
// step), fill pos[start[token] + rank] = position (plain stores)
__global__ void k_tok_count(const int* __restrict__ ids, const int* __restrict__ lens, int R, int T,
                            int* __restrict__ cnt, int* __restrict__ rank) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < R * T; i += gridDim.x * blockDim.x) {
    const int r = i / T, p = i - r * T;
    if (p < lens[r]) rank[i] = atomicAdd(&cnt[ids[i]], 1);
  }
}

// exclusive scan of cnt[0, V) (V <= 32768) by one workgroup: the counts are loaded coalesced into
// LDS (dynamic, V ints), each thread scans its contiguous slice, a shuffle scan per wave and a scan
// of the 16 wave totals join the slices
__global__ __launch_bounds__(1024) void k_tok_scan(int* __restrict__ cnt, int V, int* __restrict__ start) {
  extern __shared__ int sc[];
  __shared__ int wsum[16];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, per = (V + 1023) / 1024, b = min(V, t * per),
            e = min(V, b + per);
  for (int i = t; i < V; i += 1024) {
    sc[i] = cnt[i];
    cnt[i] = 0;  // zero for the next step's count
  }
  __syncthreads();
  int s = 0;
  for (int i = b; i < e; ++i) s += sc[i];
  int x = s;  // inclusive scan over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  int off = 0;
  for (int i = 0; i < wv; ++i) off += wsum[i];
  int run = off + x - s;
  for (int i = b; i < e; ++i) {
    const int c = sc[i];
    sc[i] = run;
    run += c;
  }
  __syncthreads();
  for (int i = t; i < V; i += 1024) {
    start[i] = sc[i];
  }
  if (t == 1023) start[V] = off + x;
}

__global__ void k_tok_fill(const int* __restrict__ ids, const int* __restrict__ lens, int R, int T,
                           const int* __restrict__ start, const int* __restrict__ rank, int* __restrict__ pos) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < R * T; i += gridDim.x * blockDim.x) {
    const int r = i / T, p = i - r * T;
    if (p < lens[r]) pos[start[ids[i]] + rank[i]] = i;
  }
}

template <int E>
__global__ __launch_bounds__(256) void k_emb_grad(const int* __restrict__ start, const int* __restrict__ pos,
                                                  const int* __restrict__ lens, int R, int T, int V,
                                                  const u16* __restrict__ DX, float* __restrict__ demb) {
  constexpr int CPL = E >= 128 ? E / 64 : 1;  // columns per lane
  static_assert(CPL <= 2, "E <= 128");
  const int lane = threadIdx.x & 63;
  const int v = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (v >= V) return;
  const bool on = lane * CPL < E;
  const int c = on ? lane * CPL : 0;  // idle lanes (E = 32) read column 0 and write nothing
  const size_t plane = (size_t)T * R;
  float a0 = 0.f, a1 = 0.f;
  const int b = start[v], n = start[v + 1] - b;
  // 64 entries at a time: lane l resolves entry l's two row offsets, then every lane walks the
  // entries with the offsets broadcast, the row loads of different entries independent
  for (int j0 = 0; j0 < n; j0 += 64) {
    const int cnt = min(64, n - j0);
    int ofw = 0, obw = 0;  // element offsets / E (rows of DX)
    if (lane < cnt) {
      const int i = pos[b + j0 + lane], r = i / T, p = i - r * T, L = lens[r];
      ofw = p * R + r;
      obw = (int)plane + (L - 1 - p) * R + r;
    }
    auto add = [&](int k) {
      const u16* fw = DX + (size_t)__shfl(ofw, k) * E + c;
      const u16* bw = DX + (size_t)__shfl(obw, k) * E + c;
      if constexpr (CPL == 2) {
        const unsigned x = *reinterpret_cast<const unsigned*>(fw), y = *reinterpret_cast<const unsigned*>(bw);
        a0 += lo16(x) + lo16(y);
        a1 += hi16(x) + hi16(y);
      } else {
        a0 += bf2f(*fw) + bf2f(*bw);
      }
    };
    int k = 0;
    for (; k + 4 <= cnt; k += 4) {  // four entries' loads in flight together
      add(k);
      add(k + 1);
      add(k + 2);
      add(k + 3);
    }
    for (; k < cnt; ++k) add(k);
  }
  if (on) {
    demb[(size_t)v * E + c] = a0;
    if constexpr (CPL == 2) demb[(size_t)v * E + c + 1] = a1;
  }
}

// ---- weight gradients ---------------------------------------------------------------------------
// dW = Z^T dP over all T*R (step, row) pairs of a direction, with Z, dP the row-major bf16 step caches
// ([x | h] or r*h, and [dr | du] or dc): a reduction over ~2e5 rows into a few 128 x 128 tiles.
// One launch covers every output tile of both directions x S row splits.  A workgroup (8 waves, 2 x 4
// of 64 x 32) streams its split's 64-row slabs of the two 128-column panels into LDS as plain
// 16-B row chunks (XOR-swizzled chunk order) and takes BOTH MFMA operands k-contiguous with
// ds_read_b64_tr_b16 (two per 16x16x32 fragment) -- the transpose the row-major caches need happens in
// the LDS read, conflict-free.  The bias gradient (column sums of dP) rides on the B fragments of the
// first row of waves.  Partials go to a [split][tile][129][128] slab; a second launch sums the splits
// in fixed order into the arena.
// A's columns [0, ex) are x: gathered as rows tok[k] of the bf16 embedding copy emb ([V x ex]);
// columns [ex, ...) are column (c - ex) of the row-major A (ex = 0: a plain A).
struct DwTile {
  const u16* A;
  const u16* B;
  float* dest;  // row drow0 of the destination block, ld ldd
  float* bias;  // null: no bias row from this tile
  const int* tok;
  const u16* emb;
  int lda, ldb, m0, mlen, n0, nlen, ldd, drow0, ex;
};
constexpr int kDwMaxTiles = 16, kDwSlabRows = 129;
struct DwArgs {
  DwTile t[kDwMaxTiles];
  int ntiles, TR, splits, kps;
  float* slab;
};

typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef short v8s_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;

__device__ __forceinline__ int dw_sw(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int dw_off(int row, int ch) { return row * 128 + 8 * (ch ^ dw_sw(row)); }

// fragment of a [64 k][128 col] swizzled image: lane (g, i) gets col c0 + i, rows kk0 + 8g + 0..7
__device__ __forceinline__ bf16x8 dw_frag(const u16* S, int kk0, int c0, int g, int q, int p) {
  const int r0 = kk0 + 8 * g + q, ch = (c0 >> 3) + (p >> 1), sub = 4 * (p & 1);
  const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(S + dw_off(r0, ch) + sub));
  const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(S + dw_off(r0 + 4, ch) + sub));
  const v8s_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

__global__ __launch_bounds__(512) void k_rnn_dw(DwArgs a) {
  __shared__ __attribute__((aligned(16))) u16 sA[2][64 * 128];
  __shared__ __attribute__((aligned(16))) u16 sB[2][64 * 128];
  const int W = a.splits * a.ntiles;
  // the tiles of one row split on one XCD (round-robin dispatch): they share the split's panels in L2
  const int L = (W % 8 == 0) ? (int)(blockIdx.x % 8) * (W / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const int ti = L % a.ntiles, split = L / a.ntiles;
  // the tile record read in place from the kernarg segment (a dynamic index into the by-value
  // argument would copy it to scratch)
  const DwTile& T = ((const DwArgs*)__builtin_amdgcn_kernarg_segment_ptr())->t[ti];
  const int kbeg = split * a.kps, kend = min(a.TR, kbeg + a.kps);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 2, wn = w & 3;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;

  // two register sets: the global loads of slab s + 2 are issued while slab s is multiplied, so each
  // has a whole iteration to land before its LDS store at the end of iteration s + 1
  struct Set {
    uint4 a0, a1, b0, b1;
  };
  const int ch = tid & 15, row0 = tid >> 4;  // chunk e = tid + 512 s: row row0 + 32 s, chunk ch
  const bool okm = ch * 8 < T.mlen, okn = ch * 8 < T.nlen;
  const int col = T.m0 + ch * 8;
  const bool xcol = col < T.ex;  // this thread's A chunk is a gathered embedding chunk
  const u16* pa = xcol ? T.emb + col : T.A + (col - T.ex);
  const u16* pb = T.B + T.n0 + ch * 8;
  const int lda = xcol ? T.ex : T.lda, ldb = T.ldb;
  const int* tok = T.tok;
  auto ld1 = [&](const u16* base, int ld, bool okc, int k) {
    // a value select, not a select of addresses (that would put the zero vector on scratch)
    uint4 v = make_uint4(0, 0, 0, 0);
    if (okc && k < kend) v = *reinterpret_cast<const uint4*>(base + (size_t)k * ld);
    return v;
  };
  // gathered chunks: the tokens of a load's rows were fetched by the previous load (loads are issued
  // in increasing k0, 64 rows apart), so the embedding gather waits on no dependent load
  auto tok1 = [&](int k) { return (xcol && okm && k < kend) ? tok[k] : 0; };
  int tk0 = tok1(kbeg + row0), tk1 = tok1(kbeg + row0 + 32);
  auto lda1 = [&](int k, int tk) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (okm && k < kend) v = *reinterpret_cast<const uint4*>(pa + (size_t)(xcol ? tk : k) * lda);
    return v;
  };
  auto load = [&](int k0) {
    Set r;
    r.a0 = lda1(k0 + row0, tk0);
    r.a1 = lda1(k0 + row0 + 32, tk1);
    tk0 = tok1(k0 + 64 + row0);
    tk1 = tok1(k0 + 64 + row0 + 32);
    r.b0 = ld1(pb, ldb, okn, k0 + row0);
    r.b1 = ld1(pb, ldb, okn, k0 + row0 + 32);
    return r;
  };
  const int o0 = dw_off(row0, ch), o1 = dw_off(row0 + 32, ch);
  auto store = [&](int buf, const Set& r) {
    *reinterpret_cast<uint4*>(&sA[buf][o0]) = r.a0;
    *reinterpret_cast<uint4*>(&sA[buf][o1]) = r.a1;
    *reinterpret_cast<uint4*>(&sB[buf][o0]) = r.b0;
    *reinterpret_cast<uint4*>(&sB[buf][o1]) = r.b1;
  };

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum[2] = {0.f, 0.f};
  const bool dobias = T.bias != nullptr && wm == 0;  // wave-uniform

  auto compute = [&](int buf) {
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      bf16x8 af[4], bfr[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = dw_frag(sA[buf], 32 * kc, wm * 64 + 16 * i, g, q, p);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = dw_frag(sB[buf], 32 * kc, wn * 32 + 16 * j, g, q, p);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if (dobias) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) bsum[j] += (float)bfr[j][e];
      }
    }
  };
  const int nst = kbeg < kend ? (kend - kbeg + 63) / 64 : 0;
  Set r0{}, r1{};
  if (nst > 0) r0 = load(kbeg);
  if (nst > 1) r1 = load(kbeg + 64);
  if (nst > 0) store(0, r0);
  __syncthreads();
  // iteration s: multiply slab s (LDS buffer s & 1), load slab s + 2 into set s & 1, store slab s + 1
  // (set (s + 1) & 1) into the other buffer; unrolled by two so the sets stay in registers
  for (int s = 0; s < nst; s += 2) {
    if (s + 2 < nst) r0 = load(kbeg + 64 * (s + 2));
    compute(0);
    if (s + 1 < nst) store(1, r1);
    __syncthreads();
    if (s + 1 >= nst) break;
    if (s + 3 < nst) r1 = load(kbeg + 64 * (s + 3));
    compute(1);
    if (s + 2 < nst) store(0, r0);
    __syncthreads();
  }
  float* out = a.slab + ((size_t)split * a.ntiles + ti) * kDwSlabRows * 128;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(size_t)(wm * 64 + 16 * i + 4 * g + r) * 128 + wn * 32 + 16 * j + li] = acc[i][j][r];
  if (dobias) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float v = bsum[j];
      v = sum_xor32(sum_xor16(v));
      if (g == 0) out[(size_t)128 * 128 + wn * 32 + 16 * j + li] = v;
    }
  }
}

// sum the splits in fixed order into the destinations (rows < mlen, columns < nlen; row 128 = bias)
__global__ __launch_bounds__(256) void k_rnn_dw_reduce(DwArgs a) {
  const int per_tile = kDwSlabRows * 32;  // float4 groups
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < a.ntiles * per_tile; e += gridDim.x * blockDim.x) {
    const int ti = e / per_tile, rem = e - ti * per_tile, row = rem >> 5, c4 = (rem & 31) * 4;
    const DwTile& T = ((const DwArgs*)__builtin_amdgcn_kernarg_segment_ptr())->t[ti];
    if (c4 >= T.nlen) continue;
    if (row < 128 ? row >= T.mlen : T.bias == nullptr) continue;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* src = a.slab + ((size_t)ti * kDwSlabRows + row) * 128 + c4;
    const size_t stride = (size_t)a.ntiles * kDwSlabRows * 128;  // one split
    int sp = 0;
    for (; sp + 8 <= a.splits; sp += 8) {  // eight loads in flight, added in split order
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(src + (size_t)(sp + u) * stride);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w;
      }
    }
    for (; sp < a.splits; ++sp) {
      const float4 v = *reinterpret_cast<const float4*>(src + (size_t)sp * stride);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    float* d = row < 128 ? T.dest + (size_t)(T.drow0 + row) * T.ldd + T.n0 + c4 : T.bias + T.n0 + c4;
    *reinterpret_cast<float4*>(d) = s;
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
#ifndef DSSM_RNN_DW_WGS  // workgroups of one k_rnn_dw launch (tiles x row splits): 2 per CU
#define DSSM_RNN_DW_WGS 512
#endif
constexpr int kDwMaxSplits = 64;

struct WsB {
  u16 *HS, *RH, *GA, *GC, *DG, *DC, *DX, *emb16;
  int *TOK, *cnt, *start, *rank, *pos;
  float* slab;
  size_t bytes, emb16_off;
};

size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

WsB ws_layout(char* base, int R, int T, int E, int H, int V) {
  const size_t TR = (size_t)T * R, NB = (R + 15) / 16;
  WsB w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += al256(bytes);
    return p;
  };
  w.HS = (u16*)take(2 * TR * H * 2);
  w.RH = (u16*)take(2 * TR * H * 2);
  w.TOK = (int*)take(2 * TR * 4);
  w.GA = (u16*)take(2 * (size_t)T * NB * 16 * H * 2 * 2);
  w.GC = (u16*)take(2 * (size_t)T * NB * 16 * H * 2 * 2);
  w.DG = (u16*)take(2 * TR * 2 * H * 2);
  w.DC = (u16*)take(2 * TR * H * 2);
  w.DX = (u16*)take(2 * TR * E * 2);
  w.emb16_off = off;
  w.emb16 = (u16*)take((size_t)V * E * 2);
  w.cnt = (int*)take(((size_t)V + 1) * 4);
  w.start = (int*)take(((size_t)V + 1) * 4);
  w.rank = (int*)take(TR * 4);
  w.pos = (int*)take(TR * 4);
  w.slab = (float*)take((size_t)kDwMaxSplits * kDwMaxTiles * kDwSlabRows * 128 * 4);
  w.bytes = off;
  return w;
}

// (the vocabulary is bounded separately: V <= 32768 for k_tok_scan)
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
                     ids, lens, emb16, w[0], w[1], w[2], w[3], ws.HS, ws.RH, ws.TOK, ws.GA, ws.GC, y, ldy);
}

template <int E, int H, int MT>
void launch_bwd_t(const GruDimsB& d, const int* ids, const int* lens, const float* const* w, const float* dy,
                  int lddy, const WsB& ws, float* demb, hipStream_t s) {
  constexpr int M = 16 * MT;
  const size_t dyn = sizeof(int) * (size_t)M;
  hipLaunchKernelGGL((k_gru_bwd_mfma<E, H, MT>), dim3((d.R + M - 1) / M, 2), dim3(Geo<E, H, MT>::NT), dyn, s, d,
                     ids, lens, w[0], w[1], w[2], w[3], dy, lddy, ws.GA, ws.GC, ws.DG, ws.DC, ws.DX);
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
#include <vector>
namespace {
int rerr_b(int code, const char* m) { return dssm::report_error(code, m); }
// HIP-event probes around the BPTT launch (bench.py's roofline: the launch's duration measured on
// the stream it runs on, inside the timed region)
struct BpttProbe {
  std::vector<hipEvent_t> ev;  // pairs
  int used = 0;
} g_probe;
}

extern "C" {

int dssm_rnn_bf16_supported(int E, int H) { return dssm::shape_ok(E, H) ? 1 : 0; }

size_t dssm_rnn_bf16_ws_bytes(int R, int T, int E, int H, int V) {
  if (R <= 0 || T <= 0 || V <= 0 || V > 32768 || !dssm::shape_ok(E, H)) return 0;
  return dssm::ws_layout(nullptr, R, T, E, H, V).bytes;
}

size_t dssm_rnn_bf16_emb16_offset(int R, int T, int E, int H, int V) {
  if (R <= 0 || T <= 0 || V <= 0 || V > 32768 || !dssm::shape_ok(E, H)) return 0;
  return dssm::ws_layout(nullptr, R, T, E, H, V).emb16_off;
}

int dssm_rnn_bf16_forward_ex(const int32_t* ids, const int32_t* lens, int R, int T, const float* emb, int V,
                             int E, int H, const float* const* w, void* ws, float* y, int ldy, int emb16_current,
                             void* stream) {
  if (!ids || !lens || !emb || !w || !ws || !y || R <= 0 || T <= 0 || V <= 0 || V > 32768 || !dssm::shape_ok(E, H) ||
      ldy < 2 * H)
    return rerr_b(DSSM_E_INVALID, "rnn_bf16_forward: bad argument or unsupported (E, H)");
  hipStream_t s = (hipStream_t)stream;
  const dssm::WsB L = dssm::ws_layout((char*)ws, R, T, E, H, V);
  const int64_t n8 = (int64_t)V * E / 8;
  if (!emb16_current)
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

int dssm_rnn_bf16_forward(const int32_t* ids, const int32_t* lens, int R, int T, const float* emb, int V,
                          int E, int H, const float* const* w, void* ws, float* y, int ldy, void* stream) {
  return dssm_rnn_bf16_forward_ex(ids, lens, R, T, emb, V, E, H, w, ws, y, ldy, 0, stream);
}

int dssm_rnn_bf16_backward(const int32_t* ids, const int32_t* lens, int R, int T, int V, int E, int H,
                           const float* const* w, const float* dy, int lddy, void* ws, float* demb,
                           float* const* gw, void* stream) {
  if (!ids || !lens || !w || !dy || !ws || !demb || !gw || R <= 0 || T <= 0 || V <= 0 || V > 32768 ||
      !dssm::shape_ok(E, H) || lddy < 2 * H)
    return rerr_b(DSSM_E_INVALID, "rnn_bf16_backward: bad argument or unsupported (E, H)");
  hipStream_t s = (hipStream_t)stream;
  const dssm::WsB L = dssm::ws_layout((char*)ws, R, T, E, H, V);
  // the batch's positions bucketed by token (for the embedding gradient after the BPTT)
  // (the counts start zero: the workspace is zero-filled once, and each scan re-zeroes them)
  const int gpos = std::max(1, std::min((R * T + 255) / 256, 2048));
  hipLaunchKernelGGL(dssm::k_tok_count, dim3(gpos), dim3(256), 0, s, ids, lens, R, T, L.cnt, L.rank);
  hipLaunchKernelGGL(dssm::k_tok_scan, dim3(1), dim3(1024), sizeof(int) * (size_t)V, s, L.cnt, V, L.start);
  hipLaunchKernelGGL(dssm::k_tok_fill, dim3(gpos), dim3(256), 0, s, ids, lens, R, T, L.start, L.rank, L.pos);
  const dssm::GruDimsB d{R, T};
  const int mt = dssm::pick_mt(R);
  const bool probe = g_probe.used < (int)g_probe.ev.size() / 2;
  if (probe) dssm::record_probe_event(s, g_probe.ev[2 * g_probe.used]);
  if (E == 128)
    dssm::dispatch_bwd<128, 128>(mt, d, ids, lens, w, dy, lddy, L, demb, s);
  else if (E == 64)
    dssm::dispatch_bwd<64, 128>(mt, d, ids, lens, w, dy, lddy, L, demb, s);
  else
    dssm::dispatch_bwd<32, 32>(mt, d, ids, lens, w, dy, lddy, L, demb, s);
  if (probe) dssm::record_probe_event(s, g_probe.ev[2 * g_probe.used++ + 1]);
  const dim3 gemb((V + 3) / 4);
  if (E == 128)
    hipLaunchKernelGGL(dssm::k_emb_grad<128>, gemb, dim3(256), 0, s, L.start, L.pos, lens, R, T, V, L.DX, demb);
  else if (E == 64)
    hipLaunchKernelGGL(dssm::k_emb_grad<64>, gemb, dim3(256), 0, s, L.start, L.pos, lens, R, T, V, L.DX, demb);
  else
    hipLaunchKernelGGL(dssm::k_emb_grad<32>, gemb, dim3(256), 0, s, L.start, L.pos, lens, R, T, V, L.DX, demb);
  // [W; b] gradients, both directions in one launch (k_rnn_dw) + a fixed-order split reduce:
  //   dWg = [x | h]^T [dr | du] (+ bias = column sums),  dWc rows [0, E) = x^T dc (+ bias),
  //   dWc rows [E, E+H) = (r*h)^T dc
  const int K = E + H, TR = T * R;
  dssm::DwArgs A{};
  int n = 0;
  for (int dir = 0; dir < 2; ++dir) {
    const size_t half = (size_t)TR * dir;
    const u16* HS = L.HS + half * H;
    const int* TK = L.TOK + half;
    const u16* RH = L.RH + half * H;
    const u16* DG = L.DG + half * 2 * H;
    const u16* DC = L.DC + half * H;
    float* gg = gw[2 * dir];
    float* gc = gw[2 * dir + 1];
    // [x | h] = embedding rows by token (columns < E) and the h_{t-1} cache
    for (int mb = 0; mb < K; mb += 128)
      for (int nb = 0; nb < 2 * H; nb += 128)
        A.t[n++] = dssm::DwTile{HS, DG, gg, mb == 0 ? gg + (size_t)K * 2 * H : nullptr, TK, L.emb16, H, 2 * H, mb,
                                std::min(128, K - mb), nb, std::min(128, 2 * H - nb), 2 * H, mb, E};
    for (int mb = 0; mb < E; mb += 128)
      for (int nb = 0; nb < H; nb += 128)
        A.t[n++] = dssm::DwTile{HS, DC, gc, mb == 0 ? gc + (size_t)K * H : nullptr, TK, L.emb16, H, H, mb,
                                std::min(128, E - mb), nb, std::min(128, H - nb), H, mb, E};
    for (int mb = 0; mb < H; mb += 128)
      for (int nb = 0; nb < H; nb += 128)
        A.t[n++] = dssm::DwTile{RH, DC, gc, nullptr, nullptr, nullptr, H, H, mb, std::min(128, H - mb), nb,
                                std::min(128, H - nb), H, E + mb, 0};
  }
  A.ntiles = n;
  A.TR = TR;
  // about two workgroups per CU (64 KB of LDS each) in one round
  A.splits = std::max(1, std::min({dssm::kDwMaxSplits, DSSM_RNN_DW_WGS / n, (TR + 63) / 64}));
  A.splits -= A.splits & 1;  // even: with 12 tiles (E = H = 128) the XCD grouping needs splits * ntiles % 8 == 0
  A.splits = std::max(A.splits, 1);
  A.splits = std::min(A.splits, dssm::kDwMaxSplits);
  A.kps = ((TR + A.splits - 1) / A.splits + 63) / 64 * 64;
  A.slab = L.slab;
  hipLaunchKernelGGL(dssm::k_rnn_dw, dim3(A.splits * n), dim3(512), 0, s, A);
  hipLaunchKernelGGL(dssm::k_rnn_dw_reduce, dim3((n * dssm::kDwSlabRows * 32 + 255) / 256), dim3(256), 0, s, A);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DSSM_OK : rerr_b(DSSM_E_HIP, hipGetErrorString(e));
}

int dssm_rnn_bf16_probe(int n_max) {
  for (hipEvent_t e : g_probe.ev) (void)hipEventDestroy(e);
  g_probe.ev.clear();
  g_probe.used = 0;
  for (int i = 0; i < 2 * n_max; ++i) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return rerr_b(DSSM_E_HIP, "rnn_bf16_probe: hipEventCreate");
    g_probe.ev.push_back(e);
  }
  return DSSM_OK;
}

int dssm_rnn_bf16_probe_read(double* avg_ms, int* count) {
  if (!avg_ms || !count) return rerr_b(DSSM_E_INVALID, "rnn_bf16_probe_read: bad argument");
  double tot = 0.0;
  for (int i = 0; i < g_probe.used; ++i) {
    float ms = 0.f;
    if (hipEventSynchronize(g_probe.ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(&ms, g_probe.ev[2 * i], g_probe.ev[2 * i + 1]) != hipSuccess)
      return rerr_b(DSSM_E_HIP, "rnn_bf16_probe_read: event");
    tot += ms;
  }
  *count = g_probe.used;
  *avg_ms = g_probe.used ? tot / g_probe.used : 0.0;
  return DSSM_OK;
}

}  // extern "C"
