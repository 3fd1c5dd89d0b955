/* CPU restatement of the DSSM training step, fp32 + OpenMP (TEST INFRASTRUCTURE / CPU BASELINE).
 *
 * This is the CPU baseline of SURVEY §8d: the reference's TF1.x CPU path cannot run here (TF is absent),
 * so this restates the same step in C.  It follows new_dssm.py exactly like oracle/dssm_oracle.py does:
 *   - forward: FC1 sparse x W1 + b1 (:124-126); per-tower batch-stat BN, EMA decay 0.5,
 *     eps 1e-3 (:62-88); ReLU (:134-136); FC_l (:146-148); merge as index arithmetic
 *     (:169-179); cosine x 20 (:182-199); softmax loss / BS (:203-209);
 *   - backward: TF autodiff of the above;
 *   - update: TF1.x ApplyAdam with fp32 beta powers (:215-217).
 * It omits the reference's O(n^2) concat chain, which would only make TF slower.
 *
 * Only tests/ and bench.py's cpu_baseline leg load it (through oracle/cpu_port.py).  It is never
 * part of the product path.  Validated against the NumPy oracle in tests/test_cpu_c.py.
 *
 * Layout: W_l row-major [in_l x n_l]; b_l [n_l]; gamma/beta [2 towers][n_l]; EMA [2][2][n_l]
 * (tower, {mean, var}).  Batch rows are [q(BS); pos(BS); neg(BS*NEG)].
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MAXL 8

typedef struct {
  int D, L, BS, NEG;
  int widths[MAXL];
  float lr, beta1, beta2, adam_eps, bn_eps, ema_decay, gamma;
} cpu_cfg;

typedef struct {
  float* W[MAXL];
  float* b[MAXL];
  float* bn_g[MAXL];   /* [2][n] */
  float* bn_b[MAXL];   /* [2][n] */
} cpu_params;          /* the same struct type holds gradients, Adam m and Adam v */

static int in_dim(const cpu_cfg* c, int l) { return l == 0 ? c->D : c->widths[l - 1]; }

/* workspace: per-layer Z, A (post BN+ReLU), xhat, per-tower inv; cosine temporaries. */
typedef struct {
  float *Z[MAXL], *A[MAXL], *xh[MAXL], *inv[MAXL], *dA, *dZ, *dAprev;
  float *qn, *dn, *cs, *prob;
  int* csc_ptr;
  int* csc_row;
  float* csc_val;
  float loss, acc;
} cpu_ws;

static void* xalloc(size_t n) {
  void* p = NULL;
  if (posix_memalign(&p, 64, n ? n : 64)) return NULL;
  memset(p, 0, n ? n : 64);
  return p;
}

void* dssm_cpu_ws_create(const cpu_cfg* c, int max_nnz) {
  cpu_ws* w = (cpu_ws*)xalloc(sizeof(cpu_ws));
  const size_t R = (size_t)c->BS * (2 + c->NEG);
  int nmax = 0;
  for (int l = 0; l < c->L; ++l) {
    const int n = c->widths[l];
    if (n > nmax) nmax = n;
    w->Z[l] = (float*)xalloc(R * n * 4);
    w->A[l] = (float*)xalloc(R * n * 4);
    w->xh[l] = (float*)xalloc(R * n * 4);
    w->inv[l] = (float*)xalloc(2 * n * 4);
  }
  w->dA = (float*)xalloc(R * nmax * 4);
  w->dZ = (float*)xalloc(R * nmax * 4);
  w->dAprev = (float*)xalloc(R * nmax * 4);
  const int K = c->NEG + 1;
  w->qn = (float*)xalloc(c->BS * 4);
  w->dn = (float*)xalloc((size_t)c->BS * K * 4);
  w->cs = (float*)xalloc((size_t)c->BS * K * 4);
  w->prob = (float*)xalloc((size_t)c->BS * K * 4);
  w->csc_ptr = (int*)xalloc((size_t)(c->D + 1) * 4);
  w->csc_row = (int*)xalloc((size_t)max_nnz * 4);
  w->csc_val = (float*)xalloc((size_t)max_nnz * 4);
  return w;
}

void dssm_cpu_ws_destroy(void* p, const cpu_cfg* c) {
  cpu_ws* w = (cpu_ws*)p;
  if (!w) return;
  for (int l = 0; l < c->L; ++l) {
    free(w->Z[l]);
    free(w->A[l]);
    free(w->xh[l]);
    free(w->inv[l]);
  }
  free(w->dA);
  free(w->dZ);
  free(w->dAprev);
  free(w->qn);
  free(w->dn);
  free(w->cs);
  free(w->prob);
  free(w->csc_ptr);
  free(w->csc_row);
  free(w->csc_val);
  free(w);
}

static int doc_row(int j, int k, int BS, int NEG) { return k == 0 ? BS + j : 2 * BS + j * NEG + k - 1; }

/* one training (train=1) or eval (train=0) forward; returns loss in w->loss */
static void forward(const cpu_cfg* c, const cpu_params* P, float* ema, cpu_ws* w, const int* indptr,
                    const int* indices, const float* values, int train) {
  const int BS = c->BS, NEG = c->NEG, R = BS * (2 + NEG);
  float* ema_l = ema;
  for (int l = 0; l < c->L; ++l) {
    const int n = c->widths[l], K = in_dim(c, l);
    float* Z = w->Z[l];
    const float* W = P->W[l];
    const float* b = P->b[l];
    if (l == 0) {
#pragma omp parallel for schedule(static)
      for (int r = 0; r < R; ++r) {
        float* z = Z + (size_t)r * n;
        for (int j = 0; j < n; ++j) z[j] = 0.f;
        for (int e = indptr[r]; e < indptr[r + 1]; ++e) {
          const float v = values[e];
          const float* wr = W + (size_t)indices[e] * n;
          for (int j = 0; j < n; ++j) z[j] += v * wr[j];
        }
        for (int j = 0; j < n; ++j) z[j] += b[j];
      }
    } else {
      const float* A = w->A[l - 1];
#pragma omp parallel for schedule(static)
      for (int r = 0; r < R; ++r) {
        float* z = Z + (size_t)r * n;
        for (int j = 0; j < n; ++j) z[j] = 0.f;
        const float* a = A + (size_t)r * K;
        for (int k = 0; k < K; ++k) {
          const float av = a[k];
          if (av == 0.f) continue;
          const float* wr = W + (size_t)k * n;
          for (int j = 0; j < n; ++j) z[j] += av * wr[j];
        }
        for (int j = 0; j < n; ++j) z[j] += b[j];
      }
    }
    /* per-tower BN (two-pass moments in double per column), EMA, affine, ReLU */
    for (int t = 0; t < 2; ++t) {
      const int r0 = t == 0 ? 0 : BS, r1 = t == 0 ? BS : R, rows = r1 - r0;
      float* em = ema_l + (size_t)t * 2 * n;  /* [mean n][var n] */
#pragma omp parallel for schedule(static)
      for (int j = 0; j < n; ++j) {
        double s = 0.0;
        for (int r = r0; r < r1; ++r) s += Z[(size_t)r * n + j];
        const double mu = s / rows;
        double q = 0.0;
        for (int r = r0; r < r1; ++r) {
          const double d = Z[(size_t)r * n + j] - mu;
          q += d * d;
        }
        const double var = q / rows;
        double m_use = mu, v_use = var;
        if (train) {
          em[j] = (float)(em[j] - (em[j] - mu) * (1.0 - c->ema_decay));
          em[n + j] = (float)(em[n + j] - (em[n + j] - var) * (1.0 - c->ema_decay));
        } else {
          m_use = em[j];
          v_use = em[n + j];
        }
        const float rs = (float)(1.0 / sqrt(v_use + c->bn_eps));
        const float inv = rs * P->bn_g[l][t * n + j];
        const float shift = P->bn_b[l][t * n + j] - (float)m_use * inv;
        w->inv[l][t * n + j] = inv;
        for (int r = r0; r < r1; ++r) {
          const float z = Z[(size_t)r * n + j];
          w->xh[l][(size_t)r * n + j] = (float)((z - m_use) * rs);
          const float y = z * inv + shift;
          w->A[l][(size_t)r * n + j] = y > 0.f ? y : 0.f;
        }
      }
    }
    ema_l += 4 * (size_t)n;
  }
  /* merge + cosine + softmax + loss (+ dy into w->dA) */
  const int n = c->widths[c->L - 1], K = NEG + 1;
  const float* Y = w->A[c->L - 1];
  double loss = 0.0, acc = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : loss, acc)
  for (int j = 0; j < BS; ++j) {
    const float* q = Y + (size_t)j * n;
    double qq = 0.0;
    for (int e = 0; e < n; ++e) qq += (double)q[e] * q[e];
    const float qn = (float)sqrt(qq);
    w->qn[j] = qn;
    float mx = -INFINITY;
    for (int k = 0; k < K; ++k) {
      const float* d = Y + (size_t)doc_row(j, k, BS, NEG) * n;
      double dd = 0.0, qd = 0.0;
      for (int e = 0; e < n; ++e) {
        dd += (double)d[e] * d[e];
        qd += (double)q[e] * d[e];
      }
      const float dn = (float)sqrt(dd);
      const float cs = (float)(qd / ((double)qn * dn));
      w->dn[j * K + k] = dn;
      w->cs[j * K + k] = cs;
      if (c->gamma * cs > mx) mx = c->gamma * cs;
    }
    double sum = 0.0;
    for (int k = 0; k < K; ++k) sum += exp((double)(c->gamma * w->cs[j * K + k] - mx));
    int amax = 0;
    for (int k = 0; k < K; ++k) {
      w->prob[j * K + k] = (float)(exp((double)(c->gamma * w->cs[j * K + k] - mx)) / sum);
      if (w->prob[j * K + k] > w->prob[j * K + amax]) amax = k;
    }
    loss += -log((double)w->prob[j * K]);
    acc += amax == 0 ? 1.0 : 0.0;
  }
  w->loss = (float)(loss / BS);
  w->acc = (float)(acc / BS);
}

/* d loss / d y for every embedding row (each doc row belongs to exactly one query) */
static void cosine_backward(const cpu_cfg* c, cpu_ws* w) {
  const int BS = c->BS, NEG = c->NEG, K = NEG + 1, n = c->widths[c->L - 1];
  const float* Y = w->A[c->L - 1];
  float* dY = w->dA;
#pragma omp parallel for schedule(static)
  for (int j = 0; j < BS; ++j) {
    const float* q = Y + (size_t)j * n;
    float* dq = dY + (size_t)j * n;
    for (int e = 0; e < n; ++e) dq[e] = 0.f;
    const float qn = w->qn[j];
    for (int k = 0; k < K; ++k) {
      const int dr = doc_row(j, k, BS, NEG);
      const float* d = Y + (size_t)dr * n;
      float* dd = dY + (size_t)dr * n;
      const float g = c->gamma * (w->prob[j * K + k] - (k == 0 ? 1.f : 0.f)) / BS;
      const float dn = w->dn[j * K + k], cs = w->cs[j * K + k];
      const float a = g / (qn * dn), bq = g * cs / (qn * qn), bd = g * cs / (dn * dn);
      for (int e = 0; e < n; ++e) {
        dq[e] += a * d[e] - bq * q[e];
        dd[e] = a * q[e] - bd * d[e];
      }
    }
  }
}

static void backward(const cpu_cfg* c, const cpu_params* P, cpu_params* G, cpu_ws* w,
                     const int* indptr, const int* indices, const float* values) {
  const int BS = c->BS, R = BS * (2 + c->NEG);
  cosine_backward(c, w);
  for (int l = c->L - 1; l >= 0; --l) {
    const int n = c->widths[l], Kin = in_dim(c, l);
    float* dA = w->dA;  /* d loss / d A_l  [R x n] */
    float* dZ = w->dZ;
    /* ReLU mask + BN backward per tower and column */
    for (int t = 0; t < 2; ++t) {
      const int r0 = t == 0 ? 0 : BS, r1 = t == 0 ? BS : R, rows = r1 - r0;
#pragma omp parallel for schedule(static)
      for (int j = 0; j < n; ++j) {
        double s1 = 0.0, s2 = 0.0;
        for (int r = r0; r < r1; ++r) {
          const size_t o = (size_t)r * n + j;
          const float dy = w->A[l][o] > 0.f ? dA[o] : 0.f;
          s1 += dy;
          s2 += (double)dy * w->xh[l][o];
        }
        G->bn_b[l][t * n + j] = (float)s1;
        G->bn_g[l][t * n + j] = (float)s2;
        const float m1 = (float)(s1 / rows), m2 = (float)(s2 / rows), inv = w->inv[l][t * n + j];
        for (int r = r0; r < r1; ++r) {
          const size_t o = (size_t)r * n + j;
          const float dy = w->A[l][o] > 0.f ? dA[o] : 0.f;
          dZ[o] = inv * (dy - m1 - w->xh[l][o] * m2);
        }
      }
    }
    /* db = sum_r dZ */
#pragma omp parallel for schedule(static)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int r = 0; r < R; ++r) s += dZ[(size_t)r * n + j];
      G->b[l][j] = (float)s;
    }
    if (l > 0) {
      const float* A = w->A[l - 1];
      float* dW = G->W[l];
      /* dW[k, :] = sum_r A[r, k] dZ[r, :]  (threads own rows k of dW) */
#pragma omp parallel for schedule(static)
      for (int k = 0; k < Kin; ++k) {
        float* g = dW + (size_t)k * n;
        for (int j = 0; j < n; ++j) g[j] = 0.f;
        for (int r = 0; r < R; ++r) {
          const float a = A[(size_t)r * Kin + k];
          if (a == 0.f) continue;
          const float* dz = dZ + (size_t)r * n;
          for (int j = 0; j < n; ++j) g[j] += a * dz[j];
        }
      }
      /* dA_{l-1} = dZ W^T */
      const float* W = P->W[l];
      float* dAp = w->dAprev;
#pragma omp parallel for schedule(static)
      for (int r = 0; r < R; ++r) {
        const float* dz = dZ + (size_t)r * n;
        float* o = dAp + (size_t)r * Kin;
        for (int k = 0; k < Kin; ++k) {
          const float* wr = W + (size_t)k * n;
          float s = 0.f;
          for (int j = 0; j < n; ++j) s += dz[j] * wr[j];
          o[k] = s;
        }
      }
      float* tmp = w->dA;
      w->dA = w->dAprev;
      w->dAprev = tmp;
    } else {
      /* dW1 = X^T dZ1 (dense [D x n]) through a CSC transpose (counting sort) */
      const int D = c->D;
      int* cp = w->csc_ptr;
      memset(cp, 0, (size_t)(D + 1) * 4);
      const int nnz = indptr[R];
      for (int e = 0; e < nnz; ++e) cp[indices[e] + 1]++;
      for (int k = 0; k < D; ++k) cp[k + 1] += cp[k];
      int* cur = (int*)malloc((size_t)D * 4);
      memcpy(cur, cp, (size_t)D * 4);
      for (int r = 0; r < R; ++r)
        for (int e = indptr[r]; e < indptr[r + 1]; ++e) {
          const int p = cur[indices[e]]++;
          w->csc_row[p] = r;
          w->csc_val[p] = values[e];
        }
      free(cur);
      float* dW = G->W[0];
#pragma omp parallel for schedule(dynamic, 64)
      for (int k = 0; k < D; ++k) {
        float* g = dW + (size_t)k * n;
        for (int j = 0; j < n; ++j) g[j] = 0.f;
        for (int p = cp[k]; p < cp[k + 1]; ++p) {
          const float v = w->csc_val[p];
          const float* dz = dZ + (size_t)w->csc_row[p] * n;
          for (int j = 0; j < n; ++j) g[j] += v * dz[j];
        }
      }
    }
  }
}

static void adam_range(float* p, const float* g, float* m, float* v, size_t n, float alpha,
                       float b1c, float b2c, float eps, float gs) {
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < n; ++i) {
    const float gi = g[i] * gs;
    m[i] += (gi - m[i]) * b1c;
    v[i] += (gi * gi - v[i]) * b2c;
    p[i] -= (m[i] * alpha) / (sqrtf(v[i]) + eps);
  }
}

/* ApplyAdam over every variable with gradients scaled by grad_scale (1/world for the
 * data-parallel mean); advances beta_powers. */
void dssm_cpu_adam(const cpu_cfg* c, cpu_params* P, cpu_params* G, cpu_params* M, cpu_params* V,
                   float* beta_powers, float gs) {
  const float alpha = c->lr * sqrtf(1.0f - beta_powers[1]) / (1.0f - beta_powers[0]);
  const float b1c = 1.0f - c->beta1, b2c = 1.0f - c->beta2;
  for (int l = 0; l < c->L; ++l) {
    const int n = c->widths[l];
    adam_range(P->W[l], G->W[l], M->W[l], V->W[l], (size_t)in_dim(c, l) * n, alpha, b1c, b2c, c->adam_eps, gs);
    adam_range(P->b[l], G->b[l], M->b[l], V->b[l], n, alpha, b1c, b2c, c->adam_eps, gs);
    adam_range(P->bn_g[l], G->bn_g[l], M->bn_g[l], V->bn_g[l], 2 * (size_t)n, alpha, b1c, b2c, c->adam_eps, gs);
    adam_range(P->bn_b[l], G->bn_b[l], M->bn_b[l], V->bn_b[l], 2 * (size_t)n, alpha, b1c, b2c, c->adam_eps, gs);
  }
  beta_powers[0] *= c->beta1;
  beta_powers[1] *= c->beta2;
}

/* One sess.run(train_step): forward(train) + backward + ApplyAdam.  beta_powers[2] are TF's
 * beta1_power/beta2_power for this step (advanced on return).  Returns the step's loss. */
float dssm_cpu_train_step(const cpu_cfg* c, cpu_params* P, cpu_params* G, cpu_params* M,
                          cpu_params* V, float* ema, void* ws, const int* indptr,
                          const int* indices, const float* values, float* beta_powers) {
  cpu_ws* w = (cpu_ws*)ws;
  forward(c, P, ema, w, indptr, indices, values, 1);
  backward(c, P, G, w, indptr, indices, values);
  dssm_cpu_adam(c, P, G, M, V, beta_powers, 1.0f);
  return w->loss;
}

/* forward only (train=0: EMA BN) + backward without update, for validation. */
float dssm_cpu_forward_backward(const cpu_cfg* c, cpu_params* P, cpu_params* G, float* ema,
                                void* ws, const int* indptr, const int* indices,
                                const float* values, int train, int with_backward) {
  cpu_ws* w = (cpu_ws*)ws;
  forward(c, P, ema, w, indptr, indices, values, train);
  if (with_backward) backward(c, P, G, w, indptr, indices, values);
  return w->loss;
}

float dssm_cpu_accuracy(void* ws) { return ((cpu_ws*)ws)->acc; }

/* OpenMP team size of the following steps (bench.py's cpu_baseline.scaling: 1..16 threads inside the
 * box's CPU share); n <= 0 leaves it as OMP_NUM_THREADS set it.  Returns the team size now in effect. */
#include <omp.h>
int dssm_cpu_set_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
  return omp_get_max_threads();
}
