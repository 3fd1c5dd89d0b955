/* CPU restatement of the RNN-tower DSSM training step, fp32 + OpenMP (TEST INFRASTRUCTURE / CPU
 * BASELINE of BASELINE.json config 4).
 *
 * The reference's TF1.x CPU path cannot run here (TF is absent), so this restates the step of
 * semantic_matching/dssm_rnn/dssm_rnn.py:100-218 the way oracle/rnn_oracle.py does (the checker it
 * is validated against in tests/test_cpu_c.py):
 *   - forward: embedding lookup; one bidirectional GRU (TF1 GRUCell: gates = sigmoid([x, h] Wg + bg),
 *     c = tanh([x, r*h] Wc + bc), h' = u*h + (1-u)*c; dynamic lengths: the state is carried past a
 *     row's length and the backward direction reads ids len-1-t); dropout with a given mask / keep;
 *     Merge_Negative_Doc as index arithmetic; x gamma cosine; softmax; loss = -sum_j log p[j, 0];
 *   - backward: BPTT; weight gradients [W; b] summed over steps and rows; the embedding gradient
 *     summed per token in (direction, step, row) order (deterministic);
 *   - update: TF1.x Adam, dense for the GRU, the IndexedSlices form for the embedding table.
 * Rows run in parallel (OpenMP); per-thread weight-gradient accumulators are reduced in thread
 * order.  Only tests/ and bench.py's cpu_baseline leg load it (oracle/cpu_c/__init__.py).
 *
 * Parameter layout (the GPU arena's, dssm_amd/rnn.py): emb [V x E]; per direction Wg_b
 * [(K+1) x 2H] and Wc_b [(K+1) x H] (last row = bias), K = E + H.  ids [R x T], rows [q; pos; neg].
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int V, E, H, T, BS, NEG;
  float lr, beta1, beta2, eps, gamma;
} rnn_cfg;

typedef struct {
  float* emb;
  float* w[4]; /* fw_g, fw_c, bw_g, bw_c */
} rnn_params; /* the same type holds gradients and Adam m / v */

typedef struct {
  int R, nthr;
  float *hp, *rg, *ug, *cg; /* [2][T][R][H]: state before the step, r, u, c */
  float *y0, *y, *dy, *qn, *dn, *cs, *prob;
  float *dx;                /* [2][T][R][E] embedding-input gradient per (dir, step, row) */
  int *tok_ptr, *tok_ent;   /* per token: its (dir, step, row) entries in order */
  float *acc;               /* per-thread weight-gradient accumulators */
  float *wgT, *wcT;         /* transposed weights of the direction being back-propagated */
  float loss;
} rnn_ws;

static void* xalloc(size_t n) {
  void* p = NULL;
  if (posix_memalign(&p, 64, n ? n : 64)) return NULL;
  memset(p, 0, n ? n : 64);
  return p;
}

static size_t wsize(const rnn_cfg* c, int m) { /* elements of w[m] */
  const size_t K1 = (size_t)c->E + c->H + 1;
  return K1 * (size_t)((m & 1) ? c->H : 2 * c->H);
}

void* rnn_cpu_ws_create(const rnn_cfg* c) {
  rnn_ws* w = (rnn_ws*)xalloc(sizeof(rnn_ws));
  const size_t R = (size_t)c->BS * (2 + c->NEG), T = c->T, H = c->H, E = c->E, K = E + H;
  w->R = (int)R;
  w->nthr = omp_get_max_threads();
  const size_t plane = 2 * T * R * H;
  w->hp = (float*)xalloc(plane * 4);
  w->rg = (float*)xalloc(plane * 4);
  w->ug = (float*)xalloc(plane * 4);
  w->cg = (float*)xalloc(plane * 4);
  w->y0 = (float*)xalloc(R * 2 * H * 4);
  w->y = (float*)xalloc(R * 2 * H * 4);
  w->dy = (float*)xalloc(R * 2 * H * 4);
  w->qn = (float*)xalloc((size_t)c->BS * 4);
  w->dn = (float*)xalloc((size_t)c->BS * (c->NEG + 1) * 4);
  w->cs = (float*)xalloc((size_t)c->BS * (c->NEG + 1) * 4);
  w->prob = (float*)xalloc((size_t)c->BS * (c->NEG + 1) * 4);
  w->dx = (float*)xalloc(2 * T * R * E * 4);
  w->tok_ptr = (int*)xalloc(((size_t)c->V + 1) * 4);
  w->tok_ent = (int*)xalloc(2 * T * R * 4);
  w->acc = (float*)xalloc((size_t)w->nthr * (K + 1) * 3 * H * 4);
  w->wgT = (float*)xalloc(2 * H * K * 4);
  w->wcT = (float*)xalloc(H * K * 4);
  return w;
}

void rnn_cpu_ws_destroy(void* p) {
  rnn_ws* w = (rnn_ws*)p;
  if (!w) return;
  free(w->hp); free(w->rg); free(w->ug); free(w->cg);
  free(w->y0); free(w->y); free(w->dy); free(w->qn); free(w->dn); free(w->cs); free(w->prob);
  free(w->dx); free(w->tok_ptr); free(w->tok_ent); free(w->acc); free(w->wgT); free(w->wcT);
  free(w);
}

static float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }
static int doc_row(int j, int k, int BS, int NEG) { return k == 0 ? BS + j : 2 * BS + j * NEG + k - 1; }
static int step_idx(int t, int len, int dir) { return t < len ? (dir ? len - 1 - t : t) : 0; }

#define RB 16 /* rows per block: a weight row is reused across the block's rows from L1 */

/* out[i][o] = b[o] + sum_k z[i][k] W[k][o] for the block's nr rows (W row-major [K x n]) */
static void block_mm(const float* z, int K, int nr, const float* W, const float* b, int n, float* out) {
  for (int i = 0; i < nr; ++i)
    for (int o = 0; o < n; ++o) out[i * n + o] = b[o];
  for (int k = 0; k < K; ++k) {
    const float* wr = W + (size_t)k * n;
    for (int i = 0; i < nr; ++i) {
      const float zk = z[i * K + k];
      float* oi = out + i * n;
      for (int o = 0; o < n; ++o) oi[o] += zk * wr[o];
    }
  }
}

/* out[i][k] = sum_o d[i][o] W[k][o], from Wt = W^T row-major [n x K] (k innermost: vectorised) */
static void block_mmT(const float* d, int n, int nr, const float* Wt, int K, float* out) {
  for (int i = 0; i < nr * K; ++i) out[i] = 0.f;
  for (int o = 0; o < n; ++o) {
    const float* wr = Wt + (size_t)o * K;
    for (int i = 0; i < nr; ++i) {
      const float dio = d[i * n + o];
      float* oi = out + i * K;
      for (int k = 0; k < K; ++k) oi[k] += dio * wr[k];
    }
  }
}

/* Wt[o][k] = W[k][o] for k < K (the bias row is not transposed) */
static void transpose(const float* W, int K, int n, float* Wt) {
#pragma omp parallel for schedule(static)
  for (int o = 0; o < n; ++o)
    for (int k = 0; k < K; ++k) Wt[(size_t)o * K + k] = W[(size_t)k * n + o];
}

/* acc[k][o] += sum_i z[i][k] d[i][o], k < K, plus the ones row k = K (bias) */
static void block_outer(const float* z, int K, int nr, const float* d, int n, float* acc) {
  for (int k = 0; k <= K; ++k) {
    float* ar = acc + (size_t)k * n;
    for (int i = 0; i < nr; ++i) {
      const float zk = k < K ? z[i * K + k] : 1.f;
      const float* di = d + i * n;
      for (int o = 0; o < n; ++o) ar[o] += zk * di[o];
    }
  }
}

static void forward(const rnn_cfg* c, const rnn_params* P, rnn_ws* w, const int* ids, const int* lens,
                    const float* mask, float keep) {
  const int R = w->R, T = c->T, H = c->H, E = c->E, K = E + H;
  const int nblk = (R + RB - 1) / RB;
  for (int dir = 0; dir < 2; ++dir) {
    const float* Wg = P->w[2 * dir];
    const float* Wc = P->w[2 * dir + 1];
#pragma omp parallel
    {
      float* z = (float*)malloc(sizeof(float) * RB * (K + 4 * H));
      float* g = z + RB * K;    /* [RB][2H] */
      float* cc = g + RB * 2 * H; /* [RB][H] */
      float* h = cc + RB * H;   /* [RB][H] */
#pragma omp for schedule(static)
      for (int blk = 0; blk < nblk; ++blk) {
        const int r0 = blk * RB, nr = R - r0 < RB ? R - r0 : RB;
        memset(h, 0, sizeof(float) * RB * H);
        for (int t = 0; t < T; ++t) {
          for (int i = 0; i < nr; ++i) {
            const int r = r0 + i;
            const float* x = P->emb + (size_t)ids[(size_t)r * T + step_idx(t, lens[r], dir)] * E;
            memcpy(z + i * K, x, sizeof(float) * E);
            memcpy(z + i * K + E, h + i * H, sizeof(float) * H);
          }
          block_mm(z, K, nr, Wg, Wg + (size_t)K * 2 * H, 2 * H, g);
          for (int i = 0; i < nr * 2 * H; ++i) g[i] = sigm(g[i]);
          for (int i = 0; i < nr; ++i)
            for (int q = 0; q < H; ++q) z[i * K + E + q] = g[i * 2 * H + q] * h[i * H + q];
          block_mm(z, K, nr, Wc, Wc + (size_t)K * H, H, cc);
          for (int i = 0; i < nr; ++i) {
            const int r = r0 + i;
            const size_t o = (((size_t)dir * T + t) * R + r) * H;
            float* hi = h + i * H;
            for (int q = 0; q < H; ++q) {
              const float cv = tanhf(cc[i * H + q]), u = g[i * 2 * H + H + q];
              w->hp[o + q] = hi[q];
              w->rg[o + q] = g[i * 2 * H + q];
              w->ug[o + q] = u;
              w->cg[o + q] = cv;
              if (t < lens[r]) hi[q] = u * hi[q] + (1.f - u) * cv;
            }
          }
        }
        for (int i = 0; i < nr; ++i)
          for (int q = 0; q < H; ++q) w->y0[(size_t)(r0 + i) * 2 * H + dir * H + q] = h[i * H + q];
      }
      free(z);
    }
  }
  const size_t n2 = (size_t)R * 2 * H;
  for (size_t i = 0; i < n2; ++i) w->y[i] = mask ? w->y0[i] * mask[i] / keep : w->y0[i];
  /* merge + cosine x gamma + softmax + summed loss */
  const int BS = c->BS, NEG = c->NEG, Kc = NEG + 1, n = 2 * H;
  double loss = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : loss)
  for (int j = 0; j < BS; ++j) {
    const float* q = w->y + (size_t)j * n;
    double qq = 0.0;
    for (int e = 0; e < n; ++e) qq += (double)q[e] * q[e];
    const float qn = (float)sqrt(qq);
    w->qn[j] = qn;
    float mx = -INFINITY;
    for (int k = 0; k < Kc; ++k) {
      const float* d = w->y + (size_t)doc_row(j, k, BS, NEG) * n;
      double dd = 0.0, qd = 0.0;
      for (int e = 0; e < n; ++e) {
        dd += (double)d[e] * d[e];
        qd += (double)q[e] * d[e];
      }
      const float dn = (float)sqrt(dd), cs = (float)(qd / ((double)qn * dn));
      w->dn[j * Kc + k] = dn;
      w->cs[j * Kc + k] = cs;
      if (c->gamma * cs > mx) mx = c->gamma * cs;
    }
    double sum = 0.0;
    for (int k = 0; k < Kc; ++k) sum += exp((double)(c->gamma * w->cs[j * Kc + k] - mx));
    for (int k = 0; k < Kc; ++k)
      w->prob[j * Kc + k] = (float)(exp((double)(c->gamma * w->cs[j * Kc + k] - mx)) / sum);
    loss += -log((double)w->prob[j * Kc]);
  }
  w->loss = (float)loss;
}

static void backward(const rnn_cfg* c, const rnn_params* P, rnn_params* G, rnn_ws* w, const int* ids,
                     const int* lens, const float* mask, float keep) {
  const int R = w->R, T = c->T, H = c->H, E = c->E, K = E + H, BS = c->BS, NEG = c->NEG, Kc = NEG + 1;
  const int n = 2 * H, nblk = (R + RB - 1) / RB;
  /* d(sum loss) / dy, then through the dropout mask */
#pragma omp parallel for schedule(static)
  for (int j = 0; j < BS; ++j) {
    const float* q = w->y + (size_t)j * n;
    float* dq = w->dy + (size_t)j * n;
    for (int e = 0; e < n; ++e) dq[e] = 0.f;
    const float qn = w->qn[j];
    for (int k = 0; k < Kc; ++k) {
      const int dr = doc_row(j, k, BS, NEG);
      const float* d = w->y + (size_t)dr * n;
      float* dd = w->dy + (size_t)dr * n;
      const float g = c->gamma * (w->prob[j * Kc + k] - (k == 0 ? 1.f : 0.f));
      const float dn = w->dn[j * Kc + k], cs = w->cs[j * Kc + k];
      const float a = g / (qn * dn), bq = g * cs / (qn * qn), bd = g * cs / (dn * dn);
      for (int e = 0; e < n; ++e) {
        dq[e] += a * d[e] - bq * q[e];
        dd[e] = a * q[e] - bd * d[e];
      }
    }
  }
  if (mask)
    for (size_t i = 0; i < (size_t)R * n; ++i) w->dy[i] *= mask[i] / keep;
  const size_t wg = (size_t)(K + 1) * 2 * H, wc = (size_t)(K + 1) * H;
  for (int dir = 0; dir < 2; ++dir) {
    const float* Wg = P->w[2 * dir];
    const float* Wc = P->w[2 * dir + 1];
    memset(w->acc, 0, sizeof(float) * (size_t)w->nthr * (wg + wc));
    transpose(Wg, K, 2 * H, w->wgT);
    transpose(Wc, K, H, w->wcT);
#pragma omp parallel
    {
      const int tid = omp_get_thread_num();
      float* aG = w->acc + (size_t)tid * (wg + wc);
      float* aC = aG + wg;
      float* buf = (float*)malloc(sizeof(float) * RB * (6 * H + 3 * K));
      float* dh = buf;                 /* [RB][H] */
      float* dcand = dh + RB * H;      /* [RB][H] */
      float* dgate = dcand + RB * H;   /* [RB][2H] */
      float* dhp = dgate + RB * 2 * H; /* [RB][H] */
      float* dz2 = dhp + RB * H;       /* [RB][K] */
      float* dz = dz2 + RB * K;        /* [RB][K] */
      float* z = dz + RB * K;          /* [RB][K] */
#pragma omp for schedule(static)
      for (int blk = 0; blk < nblk; ++blk) {
        const int r0 = blk * RB, nr = R - r0 < RB ? R - r0 : RB;
        for (int i = 0; i < nr; ++i)
          for (int q = 0; q < H; ++q) dh[i * H + q] = w->dy[(size_t)(r0 + i) * n + dir * H + q];
        for (int t = T - 1; t >= 0; --t) {
          /* inactive rows (t >= len) contribute zeros and carry dh unchanged */
          for (int i = 0; i < nr; ++i) {
            const int r = r0 + i, act = t < lens[r];
            const size_t o = (((size_t)dir * T + t) * R + r) * H;
            const float *hp = w->hp + o, *ug = w->ug + o, *cg = w->cg + o;
            for (int q = 0; q < H; ++q) {
              const float dhn = act ? dh[i * H + q] : 0.f, u = ug[q], cv = cg[q];
              dcand[i * H + q] = dhn * (1.f - u) * (1.f - cv * cv);
              dgate[i * 2 * H + H + q] = dhn * (hp[q] - cv) * u * (1.f - u);
              dhp[i * H + q] = act ? dhn * u : dh[i * H + q];
            }
          }
          block_mmT(dcand, H, nr, w->wcT, K, dz2);
          for (int i = 0; i < nr; ++i) {
            const int r = r0 + i, act = t < lens[r];
            const size_t o = (((size_t)dir * T + t) * R + r) * H;
            const float *hp = w->hp + o, *rg = w->rg + o;
            for (int q = 0; q < H; ++q) {
              const float drh = dz2[i * K + E + q], rr = rg[q];
              dgate[i * 2 * H + q] = drh * hp[q] * rr * (1.f - rr);
              if (act) dhp[i * H + q] += drh * rr;
            }
          }
          block_mmT(dgate, 2 * H, nr, w->wgT, K, dz);
          /* weight gradients: z = [x, h], z2 = [x, r*h], bias = the ones row */
          for (int i = 0; i < nr; ++i) {
            const int r = r0 + i;
            const size_t o = (((size_t)dir * T + t) * R + r) * H;
            const float* x = P->emb + (size_t)ids[(size_t)r * T + step_idx(t, lens[r], dir)] * E;
            memcpy(z + i * K, x, sizeof(float) * E);
            memcpy(z + i * K + E, w->hp + o, sizeof(float) * H);
          }
          block_outer(z, K, nr, dgate, 2 * H, aG);
          for (int i = 0; i < nr; ++i) {
            const size_t o = (((size_t)dir * T + t) * R + r0 + i) * H;
            for (int q = 0; q < H; ++q) z[i * K + E + q] = w->rg[o + q] * w->hp[o + q];
          }
          block_outer(z, K, nr, dcand, H, aC);
          for (int i = 0; i < nr; ++i) {
            const int r = r0 + i, act = t < lens[r];
            float* dx = w->dx + (((size_t)dir * T + t) * R + r) * E;
            for (int e = 0; e < E; ++e) dx[e] = act ? dz[i * K + e] + dz2[i * K + e] : 0.f;
            for (int q = 0; q < H; ++q) dh[i * H + q] = act ? dhp[i * H + q] + dz[i * K + E + q] : dhp[i * H + q];
          }
        }
      }
      free(buf);
    }
    /* reduce the per-thread accumulators in thread order */
    float* gG = G->w[2 * dir];
    float* gC = G->w[2 * dir + 1];
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < wg + wc; ++i) {
      float s = 0.f;
      for (int q = 0; q < w->nthr; ++q) s += w->acc[(size_t)q * (wg + wc) + i];
      if (i < wg) gG[i] = s;
      else gC[i - wg] = s;
    }
  }
  /* embedding gradient: per token, its entries' dx in (dir, step, row) order */
  memset(w->tok_ptr, 0, sizeof(int) * ((size_t)c->V + 1));
  for (int dir = 0; dir < 2; ++dir)
    for (int t = 0; t < T; ++t)
      for (int r = 0; r < R; ++r)
        if (t < lens[r]) w->tok_ptr[ids[(size_t)r * T + step_idx(t, lens[r], dir)] + 1]++;
  for (int v = 0; v < c->V; ++v) w->tok_ptr[v + 1] += w->tok_ptr[v];
  int* fill = (int*)malloc(sizeof(int) * (size_t)c->V);
  memcpy(fill, w->tok_ptr, sizeof(int) * (size_t)c->V);
  for (int dir = 0; dir < 2; ++dir)
    for (int t = 0; t < T; ++t)
      for (int r = 0; r < R; ++r)
        if (t < lens[r])
          w->tok_ent[fill[ids[(size_t)r * T + step_idx(t, lens[r], dir)]]++] = (dir * T + t) * R + r;
  free(fill);
#pragma omp parallel for schedule(dynamic, 64)
  for (int v = 0; v < c->V; ++v) {
    float* ge = G->emb + (size_t)v * E;
    for (int e = 0; e < E; ++e) ge[e] = 0.f;
    for (int p = w->tok_ptr[v]; p < w->tok_ptr[v + 1]; ++p) {
      const float* dx = w->dx + (size_t)w->tok_ent[p] * E;
      for (int e = 0; e < E; ++e) ge[e] += dx[e];
    }
  }
}

/* TF1.x Adam: emb in the IndexedSlices form (m = m b1 + g (1 - b1)), the GRU blocks dense. */
void rnn_cpu_adam(const rnn_cfg* c, rnn_params* P, const rnn_params* G, rnn_params* M, rnn_params* Vv,
                  float* beta_powers) {
  const float alpha = c->lr * sqrtf(1.0f - beta_powers[1]) / (1.0f - beta_powers[0]);
  const float b1 = c->beta1, b2 = c->beta2;
  const size_t ne = (size_t)c->V * c->E;
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < ne; ++i) {
    const float g = G->emb[i];
    M->emb[i] = M->emb[i] * b1 + g * (1.f - b1);
    Vv->emb[i] = Vv->emb[i] * b2 + (g * g) * (1.f - b2);
    P->emb[i] -= (M->emb[i] * alpha) / (sqrtf(Vv->emb[i]) + c->eps);
  }
  for (int m = 0; m < 4; ++m) {
    const size_t n = wsize(c, m);
    float *p = P->w[m], *mm = M->w[m], *vv = Vv->w[m];
    const float* g = G->w[m];
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; ++i) {
      mm[i] += (g[i] - mm[i]) * (1.f - b1);
      vv[i] += (g[i] * g[i] - vv[i]) * (1.f - b2);
      p[i] -= (mm[i] * alpha) / (sqrtf(vv[i]) + c->eps);
    }
  }
  beta_powers[0] *= b1;
  beta_powers[1] *= b2;
}

/* forward (+ backward when G) of one step; returns the summed loss.  mask [R x 2H] or NULL. */
float rnn_cpu_forward_backward(const rnn_cfg* c, const rnn_params* P, rnn_params* G, void* ws,
                               const int* ids, const int* lens, const float* mask, float keep) {
  rnn_ws* w = (rnn_ws*)ws;
  forward(c, P, w, ids, lens, mask, keep);
  if (G) backward(c, P, G, w, ids, lens, mask, keep);
  return w->loss;
}

const float* rnn_cpu_output(void* ws) { return ((rnn_ws*)ws)->y0; }

float rnn_cpu_train_step(const rnn_cfg* c, rnn_params* P, rnn_params* G, rnn_params* M, rnn_params* V,
                         void* ws, const int* ids, const int* lens, const float* mask, float keep,
                         float* beta_powers) {
  const float loss = rnn_cpu_forward_backward(c, P, G, ws, ids, lens, mask, keep);
  rnn_cpu_adam(c, P, G, M, V, beta_powers);
  return loss;
}
