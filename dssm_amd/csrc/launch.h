// Host-side launchers for the DSSM kernels (one per .hip translation unit).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csc.h"


namespace dssm {

struct BnSide;    // bnfuse.h
struct DetAcc;    // bnfuse.h
struct TnParams;  // tn.h
struct G32Params;  // g32.h

// Eval-mode (on_train=False) BN coefficients of every layer from the EMA shadows
// (new_dssm.py:85-86): they depend on the parameters only, not on the batch, so the forward
// computes all of them up front, in extra workgroups of the SpMM launch.
struct EvalCoef {
  int L;
  int n[8], ld[8];
  const float* gamma[8][2];
  const float* beta[8][2];
  const float* ema_mean[8][2];
  const float* ema_var[8][2];
  float* coef[8];  // [4][2][ld]: mean, rstd, inv, shift (as k_bn_stats writes them)
  float eps;
};
int eval_coef_blocks(const EvalCoef& e);

// ---- sparse (spmm.hip) ----
// FC1 forward: Z = X*W + b, one wave per CSR row, lane owns 8 output columns; with ec, its
// eval_coef_blocks(*ec) extra workgroups write the eval BN coefficients.
hipError_t launch_spmm_fwd(const int* indptr, const int* indices, const float* values, int rows,
                           const void* W, bool w_bf16, int ldw, int n, const float* bias, float* Z,
                           int ldz, hipStream_t s, const EvalCoef* ec = nullptr, bool relu = false,
                           bool z_bf16 = false);
// CSR -> CSC transpose of X with a virtual all-ones column D appended (its dW row = db1).
// scratch: csc_scratch_ints() ints, zero on first use (kept zero between calls);
// col_ptr: int[D+2]; csc_*: capacity max_nnz + rows.
size_t csc_scratch_ints(int D, int rows, int max_nnz);
// the rank transpose (default) fits: D-bin LDS histogram; it also lists the heavy columns
bool csc_rank_supported(int D);
// heavy-column work list of the rank transpose inside its scratch: item count, items {column,
// item} (kHeavyItem entries each), per-column tickets (D+1, zero-initialised)
int* csc_heavy_count(int* scratch, int D, int max_nnz);
unsigned* csc_heavy_tickets(int* scratch, int D, int rows, int max_nnz);
constexpr int kHeavyItem = 256;
hipError_t launch_csc_build(const int* indptr, const int* indices, const float* values, int rows,
                            int D, int max_nnz, int* scratch, int* col_ptr, int* csc_row,
                            float* csc_val, int* csc_col, hipStream_t s, double* zero = nullptr,
                            int nzero = 0, bool rank_path = true, bool rank_only = false,
                            int* sort_row = nullptr, float* sort_val = nullptr);
// sort_row / sort_val (deterministic mode; capacity as csc_row / csc_val, not with rank_only):
// scratch for the scatter, whose output every column then gets in row order.
// Every column [col_ptr[c], col_ptr[c+1]) of (row_in, val_in) into (row_out, val_out) in row order
// (deterministic mode of the merged transpose, after its scatter).
// scratch / max_nnz (optional): the rank transpose's scratch, whose heavy-column list sends the long
// columns to their own workgroups.
hipError_t launch_csc_sort(const int* col_ptr, int rows, int D, const int* row_in, const float* val_in,
                           int* row_out, float* val_out, hipStream_t s, int* scratch = nullptr, int max_nnz = 0);
// The rank transpose split across the fused-statistics forward (rank_only above first):
// FC1 SpMM rows + the column scan in one launch; BN1 sums + the scatter in one launch.
hipError_t launch_spmm_scan(const int* indptr, const int* indices, const float* values, int rows,
                            const void* W, bool w_bf16, int ldw, int n, const float* bias, float* Z, int ldz,
                            int D, int max_nnz, int* scratch, int* col_ptr, hipStream_t s);
// The scatter as a role of a later launch (launch_cosine_loss), on the rank transpose's scratch.
CscScatter csc_scatter_args(const int* indptr, const int* indices, const float* values, int rows, int D,
                            int* scratch, const int* col_ptr, int* csc_row, float* csc_val, int* csc_col);
hipError_t launch_sums_scatter(const float* Z, int ldz, int n, int row_split, double* fsum,
                               const int* indptr, const int* indices, const float* values, int rows,
                               int D, int max_nnz, int* scratch, const int* col_ptr, int* csc_row,
                               float* csc_val, int* csc_col, hipStream_t s,
                               CscScatter* scatter_out = nullptr, const DetAcc* det = nullptr);
// scatter_out: the launch runs the BN1 sums alone and hands the scatter to *scatter_out (a role of
// a later launch: launch_cosine_loss).
// dW1 (+ db1 as row D) = [X | 1]^T * dZ1 into G [(D+1) x n] fp32 (ld n).  light=true: every row
// is written (light rows summed, heavy rows zeroed) then heavy rows accumulated with atomics;
// light=false: only the heavy rows are accumulated (into rows that must already be zero).
hipError_t launch_dw1(const int* col_ptr, const int* csc_row, const float* csc_val,
                      const int* csc_col, int D, int rows, int max_nnz, const void* dZ,
                      bool dz_bf16, int lddz, int n, float* G, bool light, hipStream_t s,
                      int* csc_scratch = nullptr,   // non-null: heavy items of the rank transpose
                      float* heavy_slab = nullptr);  // deterministic: [items][n] partial rows
size_t csc_heavy_cap(int rows, int max_nnz);  // heavy work items one step can list
// the rank pass of launch_csc_build (rank_path) as a role of another launch (csc.h), same outputs
CscRankRole csc_rank_role_args(const int* indptr, const int* indices, int rows, int D, int* scratch,
                               double* zero, int nzero);

// ---- dense GEMM (gemm.hip) ----
enum GemmMode { GEMM_FWD = 0, GEMM_DA = 1, GEMM_DW = 2 };
constexpr int kMaxDwSplits = 32;
// Workspace floats the DW split-K partial slabs need for an (M x N) output over K rows.
size_t gemm_dw_slab_floats(int M, int N, int K, bool bf16);
// FWD: C[M x ldc] = A[M x K] * B[K x N] + bias (cols >= N written 0), then ReLU when relu != 0
// DA : C[M x ldc] = A[M x K] * B^T where B is [N x K] (ld ldb); with mask [M x ldmask], elements
//      where mask <= 0 are written 0 (ReluGrad through the layer input)
// DW : C[M x N] = A^T * B, A is [K x M] (ld lda) with a virtual ones row at m == M-1 when
//      ones_row != 0; B is [K x N]; split-K over the K (rows) dimension into `slab`
//      (gemm_dw_slab_floats) then a fixed-order reduce into C (ldc must equal N).
// flags (FWD / DA): kGemmOutBf16 = C stored as bf16, kGemmMaskBf16 = the DA mask is bf16
constexpr int kGemmOutBf16 = 1, kGemmMaskBf16 = 2;
hipError_t launch_gemm(GemmMode mode, bool bf16, int M, int N, int K, const void* A, int lda,
                       const void* B, int ldb, void* C, int ldc, const float* bias, bool ones_row,
                       float* slab, hipStream_t s,
                       int* deferred_splits = nullptr, int relu = 0, const void* mask = nullptr,
                       int ldmask = 0, int flags = 0);

// bf16 "NT" GEMM: C[M x ldc] = A . B + bias, B given k-contiguous as BT [N x ldb]
// (BT[n][k] = B[k][n]).  bn_a: A = relu(Z*inv + shift) from fp32 Z [M x lda] with BN coefficients
// coef ([4][2][lda], tower by row < row_split), also written once to a_out (bf16, ld lda) when
// a_out != null; otherwise A is bf16 [M x lda].  bias may be null (dA).
hipError_t launch_gemm_nt(int M, int N, int K, const void* A, int lda, bool bn_a,
                          const float* coef, int row_split, const uint16_t* BT, int ldb, float* C,
                          int ldc, const float* bias, uint16_t* a_out, hipStream_t s);

// Fused-statistics variants (bnfuse.h; bf16, row_split % 64 == 0):
// forward NT GEMM of layer l with BN_{l-1}+ReLU staged on the A operand, whose coefficients come
// from `coef` or, when in_from_sums != null, from that layer's sums (and are materialised by
// one workgroup); the output's per-tower column sums (with bias) are added to out_sum.
hipError_t launch_gemm_nt_fwd_fused(int M, int N, int K, const float* Z, int lda, const float* coef,
                                    const BnSide* in_from_sums, int row_split, const uint16_t* BT,
                                    int ldb, float* C, int ldc, const float* bias, uint16_t* a_out,
                                    double* out_sum, hipStream_t s, const DetAcc* det = nullptr);
// Backward of layer l in one launch: dA_{l-1} = dZ_l . W_l^T (+ BN_{l-1} backward sums from
// z_prev / coef_prev into bsum_prev) and dW_l = [A_{l-1}; 1]^T . dZ_l (split-K into slab;
// defer: the splits are left for the Adam step, *deferred_splits = count; else reduced into gw).
hipError_t launch_bwd_pair(int M, int kin, int n, const uint16_t* dZ, int lddz, const uint16_t* W,
                           int ldw, float* dA, int ldda, const float* z_prev, const float* coef_prev,
                           double* bsum_prev, int row_split, const uint16_t* A_prev, int lda_prev,
                           float* slab, float* gw, bool defer, hipStream_t s, int* deferred_splits,
                           TnParams* dw_out = nullptr, const DetAcc* det = nullptr);
// dw_out (whole-K path): the launch runs the dA tiles only and hands dW_l's split-K tiles (64 x 64,
// 384-row splits, same slabs) to *dw_out for the next BN-backward apply launch; without defer the
// caller then sums the slabs into gw with launch_splitk_reduce.
// The same for layer l (n <= 128) with BN_l's backward folded into the A staging: dZ_l
// formed from dA_l / Z_l / b's coefficients and backward sums, written bf16 to dZ_out (stride lddz
// = b.ld); one extra workgroup writes dgamma / dbeta and reduces the deferred loss (loss_part).
hipError_t launch_bwd_pair_bnb(int M, int kin, int n, const float* dA_l, const float* Z_l, const BnSide& b,
                               uint16_t* dZ_out, int lddz, const uint16_t* W, int ldw, float* dA, int ldda,
                               const float* z_prev, const float* coef_prev, double* bsum_prev, int row_split,
                               const uint16_t* A_prev, int lda_prev, float* slab, float* gw, bool defer,
                               hipStream_t s, int* deferred_splits, TnParams* dw_out, const DetAcc* det,
                               const float* loss_part, int loss_blocks, float* loss_out);
hipError_t launch_splitk_reduce(const float* slab, int splits, int64_t n, float* dst, hipStream_t s);

// ---- fp32 parity mode's fused dense layers (gemm32.hip, g32.h: f32-input MFMA 16x16x4) ----
// Forward of layer l: C = relu(BN_{l-1}(Z)) . W + bias with W [K x ldw] row-major (the arena's
// block), the activation written to a_out (fp32, ld lda), BN coefficients from in_from_sums (then
// materialised by one extra workgroup) or coef; Z_l's per-tower column sums into out_sum.
// K <= 320, widths multiples of 4, row_split % 64 == 0.
hipError_t launch_g32_fwd(int M, int N, int K, const float* Z, int lda, const float* coef,
                          const BnSide* in_from_sums, int row_split, const float* W, int ldw, float* C,
                          int ldc, const float* bias, float* a_out, double* out_sum, hipStream_t s,
                          const DetAcc* det = nullptr, uint16_t* a_out16 = nullptr);
// Backward of layer l: dA_{l-1} = dZ_l . W_l^T (BN_{l-1}'s backward sums from z_prev / coef_prev
// into bsum_prev); dW_l = [A_{l-1}; 1]^T . dZ_l in kG32DwSplit-row split-K slabs, handed to
// *dw_out for the next BN-backward apply launch or launched here (then reduced into gw unless
// defer: *deferred_splits = count for the Adam step).
hipError_t launch_g32_pair(int M, int kin, int n, const float* dZ, int lddz, const float* W, int ldw,
                           float* dA, int ldda, const float* z_prev, const float* coef_prev, double* bsum_prev,
                           int row_split, const float* A_prev, int lda_prev, float* slab, float* gw, bool defer,
                           hipStream_t s, int* deferred_splits, G32Params* dw_out = nullptr,
                           const DetAcc* det = nullptr);
hipError_t launch_g32_dw(const G32Params& dw, hipStream_t s);
int g32_dw_splits(int rows);

// ---- batch norm (bn.hip) ----
struct BnTowers {
  int row_split;   // rows [0,row_split) tower 0 (query), [row_split, rows) tower 1 (doc)
  int rows;
};
size_t bn_partial_floats(int rows, int ldz, int row_split);
// Ticket words one statistics launch needs (zero-initialised once; re-armed by the kernel).
size_t bn_ticket_count(int ldz);
// Forward statistics + EMA + affine coefficients for both towers, one launch.
// coef layout (floats): [4][2][ldz] = mean_used, rstd, inv, shift per tower.
hipError_t launch_bn_fwd_stats(const float* Z, int ldz, int n, BnTowers t, const float* gamma_q,
                               const float* beta_q, const float* gamma_d, const float* beta_d,
                               float* ema_q_mean, float* ema_q_var, float* ema_d_mean,
                               float* ema_d_var, float eps, float decay, bool train,
                               float* batch_mean /*[2*n] or null*/, float* batch_var,
                               float* partial, unsigned* tickets, float* coef, hipStream_t s,
                               double* zero = nullptr, int nzero = 0);
// Fused-statistics forward sums of one layer (bnfuse.h): fsum [2 towers][2][ldz] += sum z, z^2.
hipError_t launch_bn_sums(const float* Z, int ldz, int n, BnTowers t, double* fsum, hipStream_t s,
                          const DetAcc* det = nullptr);
// Fused-statistics backward apply: dZ (bf16) of layer b from Z, dA and b's backward sums;
// also writes b.dgamma / b.dbeta.
hipError_t launch_bn_bwd_apply_fused(const float* Z, const float* dA, const BnSide& b, uint16_t* dZ,
                                     hipStream_t s, const float* loss_part = nullptr,
                                     int loss_blocks = 0, float* loss_out = nullptr,
                                     const TnParams* dw = nullptr, const TnParams* dw2 = nullptr);
// fp32 parity mode: dZ stored fp32; the hosted dW tiles are the fp32 ones (g32.h)
hipError_t launch_bn_bwd_apply_fused32(const float* Z, const float* dA, const BnSide& b, float* dZ,
                                       hipStream_t s, const float* loss_part = nullptr,
                                       int loss_blocks = 0, float* loss_out = nullptr,
                                       const G32Params* dw = nullptr);
// out = relu?(Z*inv + shift) in out dtype; pads zero.
hipError_t launch_bn_apply(const float* Z, int ldz, int n, BnTowers t, const float* coef,
                           bool relu, void* out, bool out_bf16, hipStream_t s);
// Backward: dY = dA*(y>0); dgamma/dbeta per tower into grad slots; dZ (out dtype).
// bcoef layout: [2][2][ldz] = (mean dy, mean dy*xhat) per tower.
hipError_t launch_bn_bwd(const float* Z, const float* dA, int ldz, int n, BnTowers t,
                         const float* coef, float* dgamma_q, float* dbeta_q, float* dgamma_d,
                         float* dbeta_d, float* partial, unsigned* tickets, float* bcoef,
                         void* dZ, bool dz_bf16, hipStream_t s, const float* loss_part = nullptr,
                         int loss_nblk = 0, float* loss_out = nullptr);
// loss_part: the forward's deferred loss partials (loss_nblk cosine workgroups), reduced into
// loss_out by one extra workgroup of the statistics launch

// ---- cosine / loss (cosine.hip) ----
// z: last-layer activations [R x ld] fp32: pre-BN when coef != null (BN+ReLU applied on the
// fly, embeddings written to y_out if non-null), else the embeddings themselves.
// ws: cosine_ws_floats(bs) floats, zero-filled before first use (holds a re-armed ticket).
size_t cosine_ws_floats(int bs);
// Inverted dropout on the cosine's input rows (the RNN tower: dropout(keep) on the final states,
// dssm_rnn.py), fused: rows read as x * m / keep, dy stored as dy * m * bwd (bwd = scale / keep).
struct CosDrop {
  int on;
  unsigned thr, seed, step;  // mask: dropout_hash(r * cols + c, seed, step) < thr (all kept: thr unused)
  int all, cols;
  float fwd, bwd;
};
hipError_t launch_cosine_loss(const float* z, int ld, int n, int bs, int neg, float gamma,
                              const float* coef, float* y_out, float* cos_raw, float* cos_sim,
                              float* prob, float* qnorm, float* ws, float* loss_out, float* dy,
                              hipStream_t s, const BnSide* fused = nullptr,
                              bool defer_finalize = false, const CscScatter* scatter = nullptr,
                              const int* rmap = nullptr, const CosDrop* drop = nullptr);
// rmap (unfused, no coef / y_out): merged row r read from z row rmap[r]
// the cosine workspace's per-workgroup loss partials (finalized by a later launch when deferred)
// (queries per workgroup: kCosFusedWaves for the fused-statistics kernel at widths <= 128,
// whose per-wave LDS slots then stay small; otherwise 4)
#ifndef DSSM_COS_FUSED_WAVES
#define DSSM_COS_FUSED_WAVES 16
#endif
constexpr int kCosFusedWaves = DSSM_COS_FUSED_WAVES;
inline int cosine_waves(int n, bool fused) { return (fused && n <= 128) ? kCosFusedWaves : 4; }
inline int cosine_blocks(int bs, int n = 0, bool fused = false) {
  const int w = cosine_waves(n, fused);
  return (bs + w - 1) / w;
}
hipError_t launch_loss_finalize(const float* ws, int bs, int n, float* loss_out, hipStream_t s, bool fused = true);

// ---- optimizer (adam.hip) ----
struct ShadowSeg {
  int64_t offset;  // arena element offset of the weight block
  int64_t rows;    // weight rows (bias row excluded)
  int cols;        // == arena row length
  int ld;          // shadow leading dimension
  uint16_t* ptr;   // bf16 shadow [rows x ld]
  uint16_t* tptr;  // optional transposed bf16 shadow [cols x tld] (null: none)
  int tld;
};
struct ShadowList {
  int count;
  ShadowSeg seg[8];
};
// Adam over arena elements [begin, end) (multiples of 4); gradients at index >= clear_from are
// zeroed after use.
// One optimizer step over the arena (adam.hip).  st: device {beta1_power, beta2_power} of this
// step, advanced by the kernel; ticket: kAdamTicketUints zero-initialised counters, re-armed by
// the kernel.
#ifndef DSSM_ADAM_W1B
#define DSSM_ADAM_W1B 2048
#endif
#ifndef DSSM_ADAM_ITEMS
#define DSSM_ADAM_ITEMS 512
#endif
constexpr int kAdamW1Blocks = DSSM_ADAM_W1B;
constexpr int kAdamDenseBlocks = 2048;
constexpr int kAdamSubTickets = 64;
// ticket area: top counter + kAdamSubTickets counters, each on its own 256-B line
constexpr int kAdamTicketUints = 64 * (kAdamSubTickets + 1);
// A gradient block left as split-K partial slabs [splits][count] (plan fused mode): the Adam step
// sums them in fixed split order instead of a separate reduce launch.
struct SlabSeg {
  int64_t offset, count;
  int splits;
  const float* slab;
};
struct SlabList {
  int count;
  SlabSeg seg[8];
};
// Data-parallel wire layout (dssm_plan_set_dp_wire): W1's rows [0, D) in sub-chunks of s rows;
// rank j's optimizer shard is rows [j*chunks*s, (j+1)*chunks*s) and its sub-chunk p holds rows
// (j*chunks + p)*s + [0, s).  The wire stores sub-chunk (p, j) at ((p*world + j)*s)*n, so the
// collectives of chunk p (all-to-all of the gradient, all-gather of the parameters) each move one
// contiguous block of world * s * n elements.  chunks == 1: the wire is the arena's own layout.
struct WireGeo {
  int ww, wp, ws;  // world, chunks, rows per sub-chunk (ww == 0: identity)
  int n;           // row length (W1's width)
};
__host__ __device__ inline int64_t wire_row_off(const WireGeo& g, int row) {
  if (!g.ww) return (int64_t)row * g.n;
  const int j = row / (g.ws * g.wp), p = (row / g.ws) % g.wp, s = row % g.ws;
  return ((int64_t)(p * g.ww + j) * g.ws + s) * g.n;
}
// row of chunk `chunk`'s v-th row slot (v < ww * ws), -1 past W1's rows
__host__ __device__ inline int wire_chunk_row(const WireGeo& g, int chunk, int v, int D) {
  const int c = ((v / g.ws) * g.wp + chunk) * g.ws + v % g.ws;
  return c < D ? c : -1;
}

// Peer-store exchange (peer.hip): flag words of each rank's flags buffer (one 256-B line each group)
constexpr int kPeerMax = 8;  // ranks
constexpr int kPeerGrad = 0, kPeerParam = 64, kPeerSeq = 128, kPeerTicket = 192, kPeerTicket2 = 224, kPeerErr = 256;
constexpr int kPeerFlagWords = 320;
// SYSTEM-scope release / acquire (fine-grained buffers shared with other agents); the explicit wait
// keeps the compiler from dropping the drain after the write-back (MI355X_MICROARCH.md, compiler hazard)
__device__ __forceinline__ void peer_release() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void peer_acquire() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// payload accesses of the peer exchange, 8-B aligned.  Loads: system-scope relaxed atomic loads
// (global_load ... sc0 sc1, as the flag polls) -- coherent whatever the reader's L2 holds; in the
// exchange's first design, plain loads behind a system-scope acquire read stale stage rows in the
// second of two processes sharing IPC buffers.  Stores: plain (the signalling launches
// write back every XCD's L2 at system scope before the flag).  Build knobs (measurement): DSSM_PEER_ST 1 makes the stores
// system-scope atomics too, DSSM_PEER_LD 0 makes the loads plain.
#ifndef DSSM_PEER_ST
#define DSSM_PEER_ST 0
#endif
#ifndef DSSM_PEER_LD
#define DSSM_PEER_LD 1
#endif
__device__ __forceinline__ void st_sys8(void* p, uint2 v) {
#if DSSM_PEER_ST
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     (unsigned long long)v.x | ((unsigned long long)v.y << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
#else
  *reinterpret_cast<uint2*>(p) = v;
#endif
}
__device__ __forceinline__ void st_sys4(void* p, unsigned v) {
#if DSSM_PEER_ST
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
  *reinterpret_cast<unsigned*>(p) = v;
#endif
}
__device__ __forceinline__ uint2 ld_sys8(const void* p) {
#if DSSM_PEER_LD
  const unsigned long long u = __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<void*>(p)),
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return make_uint2((unsigned)u, (unsigned)(u >> 32));
#else
  return *reinterpret_cast<const uint2*>(p);
#endif
}
struct PeerArgs {
  int world, rank;
  unsigned* flags;            // this rank's flags
  unsigned* rflags[kPeerMax]; // every rank's flags (rflags[rank] == flags)
  float* rtail[kPeerMax];     // every rank's tail stage ([world][tailn] fp32)
  const float* tail_src;      // this rank's tail gradient (the arena's [extent, param_count))
  int64_t tailn;
  unsigned long long ticks;   // wait bound (100 MHz counter)
};
hipError_t launch_peer_before_adam(const PeerArgs& a, hipStream_t s);
hipError_t launch_peer_after_adam(const PeerArgs& a, hipStream_t s);
// start-up self-test: patterns into every rank's tail slot / parameter-wire shard block, released,
// flagged and read back with system-scope loads; mismatches added to *bad (pw_dev: a device array of
// the world's parameter-wire pointers)
hipError_t launch_peer_selftest(const PeerArgs& a, uint16_t* const* pw_dev, const uint16_t* pw_local, int64_t sub,
                                unsigned* bad, hipStream_t s);

struct AdamStep {
  float* p;
  float* g;
  float* m;
  float* v;
  // fused W1 rows (w1_blocks > 0): rows [0, D] of the [W1; b1] block at arena offset 0
  int w1_blocks;
  int D, n;
  const int* col_ptr;
  const int* csc_row;
  const float* csc_val;
  const void* dZ;
  int lddz;
  uint16_t* shadow;
  int ldsh;
  // dense float4 range [d4_begin, d4_end); gradients at element index >= clear_from are zeroed
  int64_t d4_begin, d4_end, clear_from;
  int dense_blocks;
  float* st;
  unsigned* ticket;
  float lr, beta1, beta2, b1c, b2c, eps, gs;
  ShadowList sh;
  SlabList slabs;
  // heavy W1 columns computed inside the step (item_blocks > 0): work items of the CSC scan
  // (k_csc_scan_multi), per-column arrival tickets (zero-initialised, re-armed)
  int item_blocks;
  // W1 rows with no entry this step (g = 0: pure decay) by the flat streaming role instead of a
  // wave per row (full lanes, no gather); set with item_blocks
  int w1_flat;
  const int* heavy_n;
  const int2* heavy_items;
  unsigned* heavy_ticket;
  // data-parallel bf16 wire (dssm_plan_set_dp_wire): float4 index i < wire4 takes its gradient from
  // the reduce-scattered bf16 gradient wire and writes bf16(p) to the parameter wire (the
  // all-gather's input) instead of the shadows; a second dense range [t4_begin, t4_end) (the
  // replicated fp32 tail) follows [d4_begin, d4_end)
  const uint16_t* gwire;
  uint16_t* pwire;
  int64_t wire4;
  // all-to-all wire: the W1 gradient of float4 i (< wire4) is the fp32 sum of gparts bf16 partials
  // gstage[k * gstride + 4 * (i - gbase4)] (k = 0, 1, ...: fixed order), instead of gwire[i]
  const uint16_t* gstage;
  int gparts;
  int64_t gstride, gbase4;
  int64_t t4_begin, t4_end;
  // deterministic mode: a multi-item heavy column's items store their partial rows here ([item][n],
  // write-through) and its last arrival sums them in item order (no fp32 atomics)
  float* heavy_slab;
  // the NEXT step's CSC rank pass as extra workgroups (csc.h; rank.nblocks == 0: none), LAST in
  // dispatch order by default (build knob DSSM_RANK_POS in adam.hip: 0 first, 2 after the heavy items),
  // with heavy_reset: the heavy-item count this step's scan filled, zeroed by the last block once
  // every block has read it (the next step's rank launch, which would zero it, is skipped)
  CscRankRole rank;
  int* heavy_reset;
  // gradient pass (data parallel, bf16 wire): the W1 roles compute dW1 rows (inline gather, heavy
  // items, zero for untouched rows) and write them as bf16 to gout (wire layout below; the bias row
  // as fp32 into g) instead of updating parameters; no dense range, no beta-power advance
  uint16_t* gout;
  // chunked wire geometry (WireGeo; ww == 0: the wire is laid out as the arena)
  WireGeo geo;
  int wchunk = -1;     // gradient pass: only the rows of this chunk (-1: every row)
  int64_t pwire_off4;  // the dense range's parameter-wire float4 index = i + pwire_off4
  int no_advance;      // a chunk of a chunked Adam step other than the last: no beta-power advance
  // one of group_n launches of the same step (each with its own ticket): the last to finish advances
  unsigned* group_ticket;
  int group_n;
  // gradient pass: the dense role sums the deferred split-K slabs (slabs) of [t4_begin, t4_end) into
  // the gradient arena instead of updating parameters (the tail's all-reduce then sends the sums)
  int slab_to_g;
  // peer-store exchange (peer.hip; wire chunks == 1): npeer ranks.  Gradient pass: row c's bf16
  // gradient goes to gpeer[c / geo.ws] + wire_row_off(geo, c) (owner j's stage, block of this rank)
  // instead of gout.  Adam: bf16(p) of the shard goes to every ppeer[k] at the wire offset instead of
  // pwire; the stage is read with system-scope loads.  (The stores are plain: the signalling
  // launches after this one write back every XCD's L2 at system scope before raising a flag.)
  int npeer;
  uint16_t* gpeer[kPeerMax];
  uint16_t* ppeer[kPeerMax];
  // Adam: the tail's gradient (float4 i in [t4_begin, t4_end)) is the rank-order sum of the npeer fp32
  // partials ptail[k * tailn + 4 * i - tail0] (system-scope loads) instead of g
  const float* ptail;
  int64_t tailn, tail0;
};
constexpr int kAdamItemBlocks = DSSM_ADAM_ITEMS;  // persistent workgroups for the heavy W1 columns
hipError_t launch_adam_step(AdamStep a, bool dz_bf16, hipStream_t s);
// a timing probe's event (plan.hip): hipEventRecord, or an event-record node while s is capturing
void record_probe_event(hipStream_t s, hipEvent_t e);
hipError_t launch_shadow_sync(const float* p, ShadowList sh, hipStream_t s);
// ApplyAdam over one or two float4 ranges [b4, b4 + n4) of p (16-B aligned; element indices < 2^31)
// in one launch, each updated weight of a shadow segment (<= 4; offsets in p, no transposed shadows)
// also written as bf16 to its shadow
struct AdamRanges {
  int64_t b4[2], n4[2];
  int nr;
};
hipError_t launch_adam_flat_shadow(float* p, const float* g, float* m, float* v, AdamRanges rg, const float* st,
                                  float lr, float beta1, float beta2, float eps, float gs, ShadowList sh,
                                  hipStream_t s);
// bf16 wire helpers (data parallel): the wire's W1 rows = bf16(g) (rows [0, D) of row length
// geo.n); the W1 shadow rows from the all-gathered bf16 parameter wire (chunk: that chunk's rows
// only, -1: all)
hipError_t launch_wire_pack(const float* g, uint16_t* wire, int D, WireGeo geo, hipStream_t s);
hipError_t launch_wire_shadow(const uint16_t* wire, ShadowSeg seg, WireGeo geo, int chunk, hipStream_t s);
// the peer exchange's shadow rebuild (tight rows, chunks == 1) behind a system-scope acquire per workgroup
hipError_t launch_peer_shadow(const uint16_t* wire, ShadowSeg seg, hipStream_t s);
// one workgroup spinning for `ns` nanoseconds (the data-parallel rehearsal's modelled collective)
hipError_t launch_spin(double ns, hipStream_t s);
// device-to-device copy as a kernel (captured graphs: ordered like the neighbouring kernel nodes)
hipError_t launch_copy_bytes(void* dst, const void* src, size_t bytes, hipStream_t s);

}  // namespace dssm
