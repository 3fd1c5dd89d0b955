// Persistent dense-stack kernels (dense.hip): argument block, shared by the plan (host) and the
// kernels (device).  The plan writes one DenseArgs into the workspace at creation; the kernels
// read it through a pointer (its buffers never move).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

// Device code (dense.hip) sees every buffer pointer as a global-address-space pointer, so its
// loads/stores compile to global_* instructions (generic pointers read from this struct would
// become flat_* instructions, which also count against lgkmcnt and make every LDS wait stall on
// outstanding global loads).  Host code sees plain pointers; the layout is identical.
#ifndef DSSM_GAS
#define DSSM_GAS
#endif

namespace dssm {

constexpr int kDenseMaxLayers = 8;

struct DenseLayer {
  int n, ld;                 // width, padded row stride (multiple of 8)
  float DSSM_GAS* Z;                  // [R x ld] fp32 pre-BN
  uint16_t DSSM_GAS* A;               // [R x ld] bf16 post-BN+ReLU (layers < L-1)
  float DSSM_GAS* Y;                  // [R x ld] fp32 embeddings (last layer)
  float DSSM_GAS* dy;                 // [R x ld] fp32 ReLU-masked d loss / d A
  uint16_t DSSM_GAS* dZ;              // [R x ld] bf16
  const uint16_t DSSM_GAS* W;         // [in x ld] bf16 weight shadow (layers >= 1)
  const uint16_t DSSM_GAS* WT;        // [n x ld_in] bf16 transposed shadow (layers >= 1)
  const float DSSM_GAS* bias;         // [n]
  const float DSSM_GAS* gamma[2];
  const float DSSM_GAS* beta[2];
  float DSSM_GAS* ema_mean[2];
  float DSSM_GAS* ema_var[2];
  float DSSM_GAS* dgamma[2];
  float DSSM_GAS* dbeta[2];
  float DSSM_GAS* coef;               // [4][2][ld]: mu, rstd, inv, shift (materialized for the backward)
  double DSSM_GAS* fsum;              // [2 towers][2][ld]: sum z, sum z^2 of the step (zero between uses)
  double DSSM_GAS* bsum;              // [2 towers][2][ld]: sum dy, sum dy*xhat (zero between uses)
  float DSSM_GAS* bmean;              // [2][n]
  float DSSM_GAS* bvar;               // [2][n]
  float DSSM_GAS* gW;                 // [(in+1) x n] gradient block of [W; b] (layers >= 1)
  float DSSM_GAS* slab;               // [splits][(in+1) x n] split-K partials (layers >= 1)
  int splits;
};

struct DenseArgs {
  int L, R, BS, NEG;
  float gamma_cos, eps, decay;
  DenseLayer ly[kDenseMaxLayers];
  float DSSM_GAS* cos_raw;            // [(NEG+1)*BS]
  float DSSM_GAS* cos_sim;            // [BS][NEG+1]
  float DSSM_GAS* prob;               // [BS][NEG+1]
  float DSSM_GAS* qnorm;              // [BS]
  float DSSM_GAS* loss;               // [2] loss, accuracy
  float DSSM_GAS* loss_part;          // [grid][2]
  unsigned DSSM_GAS* tickets;         // [0] forward end, [64] backward end (zero-initialised, re-armed)
  unsigned DSSM_GAS* bar;             // grid barrier words: [0] count, [64] generation, [128] error
  unsigned long long DSSM_GAS* timing;  // optional [2][64] s_memrealtime stamps (fwd, bwd) of block 0
  int exp;                   // experiment bits (DSSM_DENSE_EXP; 0 in production)
};
int dense_dw_splits(int R);
size_t dense_smem_bytes(const int* ld, int L);
bool dense_supported(int L, const int* n, const int* ld, int BS, int NEG);
hipError_t dense_prepare(size_t smem);
int dense_max_grid(size_t smem);
// kmax: the largest padded width (ld) of the stack
hipError_t launch_dense_fwd(const DenseArgs* dev_args, int last_ld, int kmax, int neg, int train,
                            int grid, size_t smem, hipStream_t s);
hipError_t launch_dense_bwd(const DenseArgs* dev_args, int kmax, int defer, int grid, size_t smem,
                            hipStream_t s);

}  // namespace dssm
