// C-ABI of libdssm.so (include/dssm.h): layout of the parameter arena and the workspace, the
// training-step plan that sequences the HIP kernels on one stream, the functional entry points
// behind the Python add_layer / batch_normalization / cosine API, and the RCCL communicator.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/dssm.h"
#include "common.h"
#include "bnfuse.h"
#include "launch.h"
#include "tn.h"
#include "g32.h"
#include "csc.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(DSSM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
  } while (0)

inline int64_t align64(int64_t x) { return (x + 63) & ~int64_t(63); }
inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

struct Layout {
  int L = 0, D = 0, BS = 0, NEG = 0, R = 0;
  bool bf16 = false;
  int n[DSSM_MAX_LAYERS] = {}, ldp[DSSM_MAX_LAYERS] = {}, in_dim[DSSM_MAX_LAYERS] = {};
  // parameter arena (fp32 elements)
  int64_t fc_off[DSSM_MAX_LAYERS] = {};      // [W_l; b_l] as (in+1) x n
  int64_t bn_off[DSSM_MAX_LAYERS][4] = {};  // q_gamma, q_beta, d_gamma, d_beta
  int64_t total = 0;
  int64_t ema_off[DSSM_MAX_LAYERS] = {};     // q_mean, q_var, d_mean, d_var (each n)
  int64_t ema_total = 0;
  // workspace (bytes)
  size_t Z[DSSM_MAX_LAYERS], A[DSSM_MAX_LAYERS], dA[DSSM_MAX_LAYERS], dZ[DSSM_MAX_LAYERS];
  size_t tickets[DSSM_MAX_LAYERS][2];
  size_t coef[DSSM_MAX_LAYERS], bcoef[DSSM_MAX_LAYERS], bmean[DSSM_MAX_LAYERS],
      bvar[DSSM_MAX_LAYERS], shadow[DSSM_MAX_LAYERS], shadowT[DSSM_MAX_LAYERS];
  size_t dw_slab[DSSM_MAX_LAYERS] = {}, partial, cos_raw, cos_sim, prob, qnorm, loss_j, loss;
  size_t csc_scratch, col_ptr, csc_row, csc_val, csc_col, adam_state;
  size_t sort_row, sort_val, heavy_slab;  // deterministic mode: transpose scratch, heavy partial rows
  // fp64 accumulators of the fused BN statistics (bnfuse.h), one zeroed region
  size_t sums = 0, sums_bytes = 0;
  size_t fsum[DSSM_MAX_LAYERS] = {}, bsum[DSSM_MAX_LAYERS] = {};
  // deterministic mode of the fused statistics (bnfuse.h DetAcc): producer slabs and tickets
  size_t fslab[DSSM_MAX_LAYERS] = {}, bslab[DSSM_MAX_LAYERS] = {}, det_ticket[DSSM_MAX_LAYERS] = {};
  int det_rows = 0;
  size_t ws = 0;
  int max_nnz = 0;
};

int check_cfg(const dssm_config* c) {
  if (!c) return fail(DSSM_E_INVALID, "null config");
  if (c->abi_version != DSSM_ABI_VERSION) return fail(DSSM_E_INVALID, "abi_version mismatch");
  if (c->trigram_d < 1) return fail(DSSM_E_INVALID, "trigram_d must be >= 1");
  if (c->n_layers < 1 || c->n_layers > DSSM_MAX_LAYERS)
    return fail(DSSM_E_INVALID, "n_layers must be in [1, 8]");
  for (int l = 0; l < c->n_layers; ++l) {
    const int w = c->widths[l];
    if (w < 4 || w > 4096 || (w % 4))
      return fail(DSSM_E_UNSUPPORTED, "layer widths must be multiples of 4 in [4, 4096]");
  }
  if (c->widths[c->n_layers - 1] > 512)
    return fail(DSSM_E_UNSUPPORTED, "embedding (last) width must be <= 512");
  if (c->query_bs < 1) return fail(DSSM_E_INVALID, "query_bs must be >= 1");
  if (c->neg < 1 || c->neg > 15) return fail(DSSM_E_UNSUPPORTED, "NEG must be in [1, 15]");
  if (c->max_nnz < 0) return fail(DSSM_E_INVALID, "max_nnz must be >= 0");
  if ((int64_t)c->query_bs * (2 + c->neg) > (1 << 26)) return fail(DSSM_E_UNSUPPORTED, "too many rows");
  if (c->compute_dtype != DSSM_F32 && c->compute_dtype != DSSM_BF16)
    return fail(DSSM_E_INVALID, "compute_dtype must be DSSM_F32 or DSSM_BF16");
  return DSSM_OK;
}

void make_layout(const dssm_config* c, Layout& Lt) {
  Lt.L = c->n_layers;
  Lt.D = c->trigram_d;
  Lt.BS = c->query_bs;
  Lt.NEG = c->neg;
  Lt.R = c->query_bs * (2 + c->neg);
  Lt.bf16 = c->compute_dtype == DSSM_BF16;
  Lt.max_nnz = c->max_nnz;
  int64_t off = 0;
  for (int l = 0; l < Lt.L; ++l) {
    Lt.n[l] = c->widths[l];
    Lt.ldp[l] = ldp8(c->widths[l]);
    Lt.in_dim[l] = l == 0 ? c->trigram_d : c->widths[l - 1];
    Lt.fc_off[l] = off;
    off = align64(off + (int64_t)(Lt.in_dim[l] + 1) * Lt.n[l]);
  }
  for (int l = 0; l < Lt.L; ++l)
    for (int k = 0; k < 4; ++k) {
      Lt.bn_off[l][k] = off;
      off = align64(off + Lt.n[l]);
    }
  Lt.total = off;
  int64_t e = 0;
  for (int l = 0; l < Lt.L; ++l) {
    Lt.ema_off[l] = e;
    e += 4 * (int64_t)Lt.n[l];
  }
  Lt.ema_total = e;

  size_t w = 0;
  auto take = [&](size_t bytes) {
    size_t o = w;
    w = align256(w + bytes);
    return o;
  };
  const size_t R = Lt.R;
  const size_t act = Lt.bf16 ? 2 : 4;
  size_t max_part = 0;
  for (int l = 0; l < Lt.L; ++l) {
    const size_t ld = Lt.ldp[l];
    Lt.Z[l] = take(R * ld * 4);
    Lt.A[l] = take(R * ld * (l == Lt.L - 1 ? 4 : act));
    Lt.dA[l] = take(R * ld * 4);
    Lt.dZ[l] = take(R * ld * act);
    Lt.coef[l] = take(4 * 2 * ld * 4);
    Lt.tickets[l][0] = take(dssm::bn_ticket_count(Lt.ldp[l]) * 4);
    Lt.tickets[l][1] = take(dssm::bn_ticket_count(Lt.ldp[l]) * 4);
    Lt.bcoef[l] = take(2 * 2 * ld * 4);
    Lt.bmean[l] = take(2 * Lt.n[l] * 4);
    Lt.bvar[l] = take(2 * Lt.n[l] * 4);
    Lt.shadow[l] = Lt.bf16 ? take((size_t)Lt.in_dim[l] * ld * 2) : 0;
    // transposed bf16 weights [n_l x ldp(in)] for the whole-K forward GEMM (layers >= 2)
    Lt.shadowT[l] = (Lt.bf16 && l > 0) ? take((size_t)Lt.n[l] * Lt.ldp[l - 1] * 2) : 0;
    max_part = std::max(max_part, dssm::bn_partial_floats(Lt.R, Lt.ldp[l], Lt.BS));
  }
  Lt.partial = take(max_part * 4);
  // split-K slabs of dW_l (l >= 2), one per layer: in fused mode the Adam step sums them
  for (int l = 1; l < Lt.L; ++l)
    Lt.dw_slab[l] = take(
        std::max<size_t>(dssm::gemm_dw_slab_floats(Lt.in_dim[l] + 1, Lt.n[l], Lt.R, Lt.bf16), 1) * 4);
  const size_t K = Lt.NEG + 1;
  Lt.cos_raw = take(K * Lt.BS * 4);
  Lt.cos_sim = take(K * Lt.BS * 4);
  Lt.prob = take(K * Lt.BS * 4);
  Lt.qnorm = take(Lt.BS * 4);
  Lt.loss_j = take(dssm::cosine_ws_floats(Lt.BS) * 4);
  Lt.loss = take(2 * 4);
  Lt.csc_scratch = take(dssm::csc_scratch_ints(Lt.D, Lt.R, Lt.max_nnz) * 4);
  Lt.col_ptr = take((size_t)(Lt.D + 2) * 4);
  const size_t ent = (size_t)Lt.max_nnz + R;
  Lt.csc_row = take(ent * 4);
  Lt.csc_val = take(ent * 4);
  Lt.csc_col = take(ent * 4);
  Lt.sort_row = take(ent * 4);
  Lt.sort_val = take(ent * 4);
  Lt.heavy_slab = take(dssm::csc_heavy_cap(Lt.R, Lt.max_nnz) * Lt.n[0] * 4);
  // {beta1_power, beta2_power} (device-side Adam step state), then the Adam kernel's tickets
  Lt.adam_state = take(4 * (64 + dssm::kAdamTicketUints));
  {
    // fp64 [2 towers][2][ld] forward and backward accumulators per layer (fused statistics, both
    // dtypes), one contiguous region zeroed as a whole by the step's first launch
    size_t sums = 0;
    for (int l = 0; l < Lt.L; ++l) sums += 2 * (size_t)4 * Lt.ldp[l] * 8;
    Lt.sums = take(sums);
    Lt.sums_bytes = sums;
    // producer rows of any fused-statistics launch: 64-row tiles bound them all (the launchers
    // check), plus the reduction tree's level-2 rows (bnfuse.h det_publish)
    Lt.det_rows = (int)((R + 63) / 64) + 2;
    for (int l = 0; l < Lt.L; ++l) {
      const size_t slab = dssm::det_slab_rows(Lt.det_rows) * 4 * Lt.ldp[l] * 8;
      Lt.fslab[l] = take(slab);
      Lt.bslab[l] = take(slab);
      Lt.det_ticket[l] = take(2 * dssm::kDetTiles * dssm::kDetTickets * 4);  // [fwd | bwd][tile][ticket]
    }
    size_t o = Lt.sums;
    for (int l = 0; l < Lt.L; ++l) {
      Lt.fsum[l] = o;
      o += (size_t)4 * Lt.ldp[l] * 8;
      Lt.bsum[l] = o;
      o += (size_t)4 * Lt.ldp[l] * 8;
    }
  }
  Lt.ws = w;
}

}  // namespace

struct dssm_plan {
  dssm_config cfg;
  Layout Lt;
  char* ws;
  float *p, *g, *m, *v, *ema;
  const int32_t* indptr = nullptr;
  const int32_t* indices = nullptr;
  const float* values = nullptr;
  bool fwd_train_done = false;
  int64_t adam_begin = 0, adam_end = -1;  // sharded optimizer range (dssm_plan_set_adam_range)
  // data-parallel bf16 wire (dssm_plan_set_dp_wire, layout dssm::WireGeo): the gradient pass
  // writes every rank's W1 rows into gwire, the all-to-all delivers this rank's shard from every
  // rank into gstage (summed in fp32, rank order, by the Adam launch), Adam writes bf16(W1) of the
  // shard into pwire, which the all-gather completes; arena elements [0, wire_end) are W1's rows
  uint16_t* gwire = nullptr;
  uint16_t* pwire = nullptr;
  const uint16_t* gstage = nullptr;
  // the captured data-parallel graph's steps after the first (one wire chunk): the forward's SpMM
  // reads W1 straight from the all-gathered parameter wire (row stride geo.n) instead of the shadow
  // the k_wire_shadow launch would rebuild from it; the region's last step still rebuilds the shadow
  const uint16_t* w1_wire = nullptr;
  dssm::WireGeo geo{};
  int dp_rank = 0;
  // peer-store exchange (dssm_plan_set_dp_peers, peer.hip): every rank's stage / parameter wire /
  // tail stage / flags mapped into this process; world 0: off
  struct PeerSet {
    int world = 0;
    uint16_t* stage[dssm::kPeerMax] = {};
    uint16_t* pwire[dssm::kPeerMax] = {};
    float* tail[dssm::kPeerMax] = {};
    unsigned* flags[dssm::kPeerMax] = {};
    unsigned long long wait_ticks = 2000000000ull;  // 20 s of the 100 MHz counter
  } peer;
  // the peer self-test's device scratch ([kPeerMax] parameter-wire pointers + a counter), allocated
  // once by dssm_plan_set_dp_peers (no allocation, hence no device-wide synchronisation, inside the
  // self-test: ranks sharing a GPU run theirs concurrently)
  void* peer_scratch = nullptr;
  bool peer_on() const { return peer.world > 0 && pwire != nullptr; }
  bool dp_defer_gradpass = false;  // the data-parallel graph builder launches the chunks itself
  // the data-parallel graph builder's hook after each Adam chunk launch (that chunk's all-gather)
  std::function<int(int)> dp_hook;
  int64_t wire_end() const { return Lt.fc_off[0] + (int64_t)Lt.in_dim[0] * Lt.n[0]; }
  int64_t sub_elems() const { return (int64_t)geo.ws * geo.n; }
  // rows [r0, r1) of this rank's sub-chunk p (r1 <= r0: none past W1's rows)
  void dp_chunk_rows(int p, int& r0, int& r1) const {
    r0 = std::min((dp_rank * geo.wp + p) * geo.ws, Lt.D);
    r1 = std::min(r0 + geo.ws, Lt.D);
  }
  bool fwd_fused = false;  // the last train forward ran the fused-statistics schedule
  bool loss_pending = false;  // its loss partials await the backward's first launch
  bool grads_clean = true;     // atomic-target gradient blocks are zero (Adam clears them)
  int dw_deferred[DSSM_MAX_LAYERS] = {};  // split count of dW_l left in its slab (fused mode)
  // Multi-step graphs: the Adam launch of step i hosts step i+1's CSC rank pass (csc.h) when the
  // next batch is known (host_rank_*); rank_done_for = that batch, whose forward then skips the
  // transpose's first launch (the rank launch, 11 us at C2).
  const int32_t* host_rank_indptr = nullptr;
  const int32_t* host_rank_indices = nullptr;
  const int32_t* rank_done_for = nullptr;
  // Schedule options (dssm_plan_set_option; never read from the environment).  Each names a
  // measured-faster default and the alternative it replaced, kept for parity tests and shapes the
  // default does not support.  Graphs captured earlier keep the schedule they were captured with.
  int opt[DSSM_OPT_COUNT] = {
      1,  // FUSED_STATS: BN statistics fused into producers / consumers (where supported)
      1,  // MERGED_CSC: the rank transpose's scan / scatter ride in the forward's launches
      1,  // HEAVY_IN_ADAM: dW1's heavy columns as work items of the Adam launch
      1,  // SCATTER_IN_COS: the transpose's scatter as workgroups of the cosine launch
      1,  // DW_IN_APPLY: dW_l split-K tiles inside the next BN-backward apply launch
      1,  // WIRE_GRAD_PASS: data parallel bf16 wire: dW1 written straight into the wire
      1,  // CSC_RANK: rank / scan / scatter transpose (0: histogram / fill launches)
      0,  // DETERMINISTIC: fixed-order reductions, bit-identical repeated runs
      1,  // FUSED_W1_ADAM: dW1 light rows and the dW_l slabs consumed inside Adam
      1,  // RANK_IN_ADAM: multi-step graphs: the next step's CSC rank pass inside this Adam launch
      0,  // MEMCPY_NODES: diagnostics: data-parallel device copies as hipMemcpyAsync nodes
      1,  // BNB_IN_PAIR: the last layer's BN backward formed in the dA pair's A staging
      0,  // TAIL_IN_A2A: data-parallel graph: the tail's all-reduce in the last all-to-all's RCCL group
      0,  // FWD32: bf16 plan: the forward on fp32 weights / tiles (fp32-accurate loss, cosine), bf16 backward
  };
  bool on(int o) const { return opt[o] != 0; }
  // Captured train steps (hipGraph) and, while capturing, the slot whose probe events to record.
  struct GraphSlot {
    hipGraphExec_t exec = nullptr;
    hipEvent_t ev[DSSM_PROBE_COUNT][2] = {};
    bool probes = false;
    unsigned probe_mask = ~0u;  // while capturing: which probe ids record event nodes
    int64_t topo[8] = {};  // the captured graph's shape (graph_topology)
  };
  std::vector<GraphSlot*> graphs;
  GraphSlot* capturing = nullptr;
  // hipEventRecord on a capturing stream only marks a fork/join point; a timing record needs an
  // explicit event-record node appended after the stream's current capture frontier.
  static void graph_event_node(hipStream_t s, hipEvent_t e) {
    hipStreamCaptureStatus st;
    unsigned long long id;
    hipGraph_t g;
    const hipGraphNode_t* deps;
    size_t nd;
    if (hipStreamGetCaptureInfo_v2(s, &st, &id, &g, &deps, &nd) != hipSuccess ||
        st != hipStreamCaptureStatusActive)
      return;
    hipGraphNode_t node;
    if (hipGraphAddEventRecordNode(&node, g, deps, nd, e) != hipSuccess) return;
    hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies);
  }
  // Kernel timing probes: HIP events recorded on the launch stream around one kernel family.
  struct Probe {
    bool on = false;
    std::vector<hipEvent_t> ev;  // start/stop pairs
    int next = 0;
  } probe[DSSM_PROBE_COUNT];

  void probe_begin(int id, hipStream_t s) {
    if (capturing) {
      if (capturing->probes && (capturing->probe_mask >> id & 1)) graph_event_node(s, capturing->ev[id][0]);
      return;
    }
    Probe& p = probe[id];
    if (p.on && p.next + 1 < (int)p.ev.size()) hipEventRecord(p.ev[p.next], s);
  }
  void probe_end(int id, hipStream_t s) {
    if (capturing) {
      if (capturing->probes && (capturing->probe_mask >> id & 1)) graph_event_node(s, capturing->ev[id][1]);
      return;
    }
    Probe& p = probe[id];
    if (p.on && p.next + 1 < (int)p.ev.size()) {
      hipEventRecord(p.ev[p.next + 1], s);
      p.next += 2;
    }
  }

  template <typename T> T* at(size_t off) const { return reinterpret_cast<T*>(ws + off); }
  const void* weight(int l) const {  // what the kernels read for W_l
    if (l == 0 && w1_wire) return w1_wire;
    return Lt.bf16 ? (const void*)at<u16>(Lt.shadow[l]) : (const void*)(p + Lt.fc_off[l]);
  }
  int weight_ld(int l) const {
    if (l == 0 && w1_wire) return geo.n;
    return Lt.bf16 ? Lt.ldp[l] : Lt.n[l];
  }
  // Layer l (>= 1) runs its forward/dA GEMMs on the bf16 NT kernel (fused BN staging).
  bool wholek(int l) const { return Lt.bf16 && l > 0 && Lt.ldp[l - 1] <= 512; }
  // fp32 parity mode: layer l (>= 1) on the fused fp32 MFMA tiles (g32.h: K <= 320 both ways)
  bool g32_fits(int l) const { return l > 0 && Lt.in_dim[l] <= 320 && Lt.n[l] <= 320; }
  bool nt32(int l) const { return !Lt.bf16 && g32_fits(l); }
  // bf16 plan with the fp32-accurate forward (DSSM_OPT_FWD32): the SpMM on the fp32 W1 masters, the
  // layers >= 2 forward on the g32 tiles and fp32 W_l; not with the data-parallel bf16 wire (W1's fp32
  // rows outside a rank's shard are stale there)
  bool fwd32() const { return Lt.bf16 && on(DSSM_OPT_FWD32) && !pwire; }
  const void* fwd_weight0() const { return fwd32() ? (const void*)(p + Lt.fc_off[0]) : weight(0); }
  bool fwd_weight0_bf16() const { return fwd32() ? false : Lt.bf16; }
  int fwd_weight0_ld() const { return fwd32() ? Lt.n[0] : weight_ld(0); }
  const float* bias(int l) const { return p + Lt.fc_off[l] + (int64_t)Lt.in_dim[l] * Lt.n[l]; }
  dssm::BnSide bn_side(int l) const {
    dssm::BnSide b{};
    const int n = Lt.n[l];
    b.n = n;
    b.ld = Lt.ldp[l];
    b.rows_q = Lt.BS;
    b.rows_d = Lt.R - Lt.BS;
    b.eps = cfg.bn_eps;
    b.decay = cfg.ema_decay;
    for (int t = 0; t < 2; ++t) {
      b.gamma[t] = p + Lt.bn_off[l][2 * t];
      b.beta[t] = p + Lt.bn_off[l][2 * t + 1];
      b.dgamma[t] = g + Lt.bn_off[l][2 * t];
      b.dbeta[t] = g + Lt.bn_off[l][2 * t + 1];
      b.ema_mean[t] = ema + Lt.ema_off[l] + (int64_t)(2 * t) * n;
      b.ema_var[t] = ema + Lt.ema_off[l] + (int64_t)(2 * t + 1) * n;
    }
    b.coef = at<float>(Lt.coef[l]);
    b.bmean = at<float>(Lt.bmean[l]);
    b.bvar = at<float>(Lt.bvar[l]);
    b.fsum = at<double>(Lt.fsum[l]);
    b.bsum = at<double>(Lt.bsum[l]);
    if (deterministic() && Lt.det_rows) {
      unsigned* tk = at<unsigned>(Lt.det_ticket[l]);
      b.fdet = dssm::DetAcc{at<double>(Lt.fslab[l]), tk, Lt.det_rows};
      b.bdet = dssm::DetAcc{at<double>(Lt.bslab[l]), tk + dssm::kDetTiles * dssm::kDetTickets, Lt.det_rows};
    }
    return b;
  }
  bool csc_rank_path() const { return on(DSSM_OPT_CSC_RANK) && dssm::csc_rank_supported(Lt.D); }
  bool fused_w1_adam() const { return on(DSSM_OPT_FUSED_W1_ADAM); }
  // deterministic mode: fused statistics summed in a fixed order (bnfuse.h DetAcc slabs instead of
  // fp64 atomics), every CSC column in row order, heavy dW1 rows through per-item slabs
  bool deterministic() const { return on(DSSM_OPT_DETERMINISTIC); }
  bool fused_stats() const { return on(DSSM_OPT_FUSED_STATS) && fused_stats_ok(); }
  // the rank transpose's launches merged into the step's: the scan beside the SpMM rows, the scatter
  // beside the cosine (or BN1 sums), the rank in the previous Adam.  fp32 parity mode (no fused
  // statistics): the scatter always rides in the cosine launch, and not in deterministic mode
  bool merged_csc() const {
    if (!on(DSSM_OPT_MERGED_CSC) || !csc_rank_path() || (Lt.BS % 128)) return false;
    if (fused_stats()) return true;
    return !Lt.bf16 && on(DSSM_OPT_SCATTER_IN_COS) && !deterministic();
  }
  bool heavy_in_adam() const { return on(DSSM_OPT_HEAVY_IN_ADAM) && csc_rank_path(); }
  // bf16 fused schedule: the last layer's BN backward inside its dA pair launch (gemm.hip
  // launch_bwd_pair_bnb: whole-K 128-row tiles, K <= 128, the dW tiles handed to the next apply)
  // launch_bwd_pair_bnb: whole-K 128-row tiles, K <= 128, the dW tiles handed to the next apply.
  // Of the last two layers (>= 1) those <= 128 wide fold, so the apply launch after them hosts at
  // most two dW tile sets (C2: the last layer; the 300-wide fold measured slower, gemm.hip kBnbMaxK).
  bool bnb_fold(int l) const {
    return on(DSSM_OPT_BNB_IN_PAIR) && on(DSSM_OPT_DW_IN_APPLY) && Lt.bf16 && l >= 1 && l >= Lt.L - 2 &&
           fused_stats() && wholek(l) && Lt.n[l] <= 128 && (Lt.BS % 128) == 0 && ((Lt.R - Lt.BS) % 128) == 0;
  }
  bool bnb_in_pair() const { return Lt.L >= 2 && bnb_fold(Lt.L - 1); }
  bool fused_stats_ok() const {
    if (Lt.L < 2 || (Lt.BS % 64) || !Lt.sums_bytes) return false;
    for (int l = 0; l < Lt.L; ++l)
      if (Lt.ldp[l] > 512) return false;
    for (int l = 1; l < Lt.L; ++l)
      if (!(Lt.bf16 ? wholek(l) && (!fwd32() || g32_fits(l)) : nt32(l))) return false;
    return true;
  }
  dssm::ShadowList shadows() {
    dssm::ShadowList s;
    s.count = 0;
    if (!Lt.bf16) return s;
    for (int l = 0; l < Lt.L; ++l) {
      dssm::ShadowSeg& g = s.seg[s.count++];
      g.offset = Lt.fc_off[l];
      g.rows = Lt.in_dim[l];
      g.cols = Lt.n[l];
      g.ld = Lt.ldp[l];
      g.ptr = at<uint16_t>(Lt.shadow[l]);
      g.tptr = l > 0 ? at<uint16_t>(Lt.shadowT[l]) : nullptr;
      g.tld = Lt.ldp[l - (l > 0 ? 1 : 0)];
    }
    return s;
  }
};

#ifndef DSSM_GRAPH_UPLOAD
#define DSSM_GRAPH_UPLOAD 1
#endif

namespace dssm {
// A timing probe's event on stream s: a plain record, or while s is capturing, an explicit
// event-record node after the capture frontier (hipEventRecord on a capturing stream only marks a
// fork / join point).  Shared by the functional API's probes (rnn.hip, rnn_mfma.hip).
void record_probe_event(hipStream_t s, hipEvent_t e) {
  hipStreamCaptureStatus st;
  if (hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusActive) {
    unsigned long long id;
    hipGraph_t g;
    const hipGraphNode_t* deps;
    size_t nd;
    if (hipStreamGetCaptureInfo_v2(s, &st, &id, &g, &deps, &nd) != hipSuccess) return;
    hipGraphNode_t node;
    if (hipGraphAddEventRecordNode(&node, g, deps, nd, e) != hipSuccess) return;
    hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies);
    return;
  }
  (void)hipEventRecord(e, s);
}
}  // namespace dssm

namespace dssm {
int report_error(int code, const char* msg) { return fail(code, msg ? msg : ""); }
}  // namespace dssm

extern "C" {

int dssm_abi_version(void) { return DSSM_ABI_VERSION; }
const char* dssm_last_error(void) { return g_err.c_str(); }

int dssm_config_check(const dssm_config* cfg) { return check_cfg(cfg); }

int64_t dssm_param_count(const dssm_config* cfg) {
  if (check_cfg(cfg)) return -1;
  Layout Lt;
  make_layout(cfg, Lt);
  return Lt.total;
}

int64_t dssm_ema_count(const dssm_config* cfg) {
  if (check_cfg(cfg)) return -1;
  Layout Lt;
  make_layout(cfg, Lt);
  return Lt.ema_total;
}

int dssm_param_layout(const dssm_config* cfg, dssm_segment* segs, int max_segs) {
  if (int rc = check_cfg(cfg)) return rc;
  Layout Lt;
  make_layout(cfg, Lt);
  int k = 0;
  auto put = [&](const char* name, int64_t off, int64_t rows, int64_t cols) {
    if (segs && k < max_segs) {
      std::snprintf(segs[k].name, sizeof(segs[k].name), "%s", name);
      segs[k].offset = off;
      segs[k].rows = rows;
      segs[k].cols = cols;
    }
    ++k;
  };
  char nm[32];
  for (int l = 0; l < Lt.L; ++l) {
    std::snprintf(nm, sizeof nm, "fc%d", l + 1);
    put(nm, Lt.fc_off[l], Lt.in_dim[l] + 1, Lt.n[l]);
  }
  static const char* bnn[4] = {"q_gamma", "q_beta", "d_gamma", "d_beta"};
  for (int l = 0; l < Lt.L; ++l)
    for (int j = 0; j < 4; ++j) {
      std::snprintf(nm, sizeof nm, "bn%d_%s", l + 1, bnn[j]);
      put(nm, Lt.bn_off[l][j], 1, Lt.n[l]);
    }
  return k;
}

size_t dssm_workspace_bytes(const dssm_config* cfg) {
  if (check_cfg(cfg)) return 0;
  Layout Lt;
  make_layout(cfg, Lt);
  return Lt.ws;
}

int dssm_plan_create(const dssm_config* cfg, void* workspace, size_t workspace_bytes, float* params,
                     float* grads, float* adam_m, float* adam_v, float* ema, dssm_plan** out) {
  if (int rc = check_cfg(cfg)) return rc;
  if (!out || !workspace || !params || !grads || !adam_m || !adam_v || !ema)
    return fail(DSSM_E_INVALID, "null buffer passed to dssm_plan_create");
  dssm_plan* P = new dssm_plan();
  P->cfg = *cfg;
  make_layout(cfg, P->Lt);
  if (workspace_bytes < P->Lt.ws) {
    delete P;
    return fail(DSSM_E_INVALID, "workspace too small");
  }
  if ((reinterpret_cast<uintptr_t>(workspace) & 255) || (reinterpret_cast<uintptr_t>(params) & 15)) {
    delete P;
    return fail(DSSM_E_INVALID, "workspace must be 256-B aligned and arenas 16-B aligned");
  }
  P->ws = static_cast<char*>(workspace);
  P->p = params;
  P->g = grads;
  P->m = adam_m;
  P->v = adam_v;
  P->ema = ema;
  const float st[4] = {cfg->beta1, cfg->beta2, 0.f, 0.f};  // TF: beta*_power start at beta*
  if (hipMemcpy(P->ws + P->Lt.adam_state, st, sizeof st, hipMemcpyHostToDevice) != hipSuccess) {
    delete P;
    return fail(DSSM_E_HIP, "failed to initialise the device Adam state");
  }
  *out = P;
  return DSSM_OK;
}

int dssm_plan_destroy(dssm_plan* plan) {
  if (plan) {
    if (plan->peer_scratch) (void)hipFree(plan->peer_scratch);
    for (auto& p : plan->probe)
      for (hipEvent_t e : p.ev) hipEventDestroy(e);
    for (auto* g : plan->graphs) {
      if (g->exec) hipGraphExecDestroy(g->exec);
      for (auto& pr : g->ev)
        for (hipEvent_t e : pr)
          if (e) hipEventDestroy(e);
      delete g;
    }
  }
  delete plan;
  return DSSM_OK;
}

int dssm_plan_set_option(dssm_plan* P, int option, int value) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  if (option < 0 || option >= DSSM_OPT_COUNT) return fail(DSSM_E_INVALID, "unknown plan option");
  if (P->capturing) return fail(DSSM_E_INVALID, "options cannot change during a graph capture");
  P->opt[option] = value != 0;
  return DSSM_OK;
}

int dssm_plan_get_option(const dssm_plan* P, int option) {
  if (!P || option < 0 || option >= DSSM_OPT_COUNT) return -1;
  return P->opt[option];
}

int dssm_plan_probe_enable(dssm_plan* P, int id, int max_samples) {
  if (!P || id < 0 || id >= DSSM_PROBE_COUNT || max_samples < 0)
    return fail(DSSM_E_INVALID, "bad probe arguments");
  auto& p = P->probe[id];
  for (hipEvent_t e : p.ev) hipEventDestroy(e);
  p.ev.clear();
  p.next = 0;
  p.on = max_samples > 0;
  for (int i = 0; i < 2 * max_samples; ++i) {
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    p.ev.push_back(e);
  }
  return DSSM_OK;
}

int dssm_plan_probe_read(dssm_plan* P, int id, float* total_ms, int* count) {
  if (!P || id < 0 || id >= DSSM_PROBE_COUNT || !total_ms || !count)
    return fail(DSSM_E_INVALID, "bad probe arguments");
  auto& p = P->probe[id];
  float tot = 0.f;
  int n = 0;
  for (int i = 0; i + 1 < p.next; i += 2) {
    HIP_TRY(hipEventSynchronize(p.ev[i + 1]));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, p.ev[i], p.ev[i + 1]));
    tot += ms;
    ++n;
  }
  *total_ms = tot;
  *count = n;
  return DSSM_OK;
}

int dssm_plan_buffer(const dssm_plan* P, int id, int layer, void** ptr, size_t* bytes) {
  if (!P || !ptr) return fail(DSSM_E_INVALID, "null plan/ptr");
  const Layout& Lt = P->Lt;
  const int K = Lt.NEG + 1;
  if (layer < 0 || layer >= Lt.L) layer = Lt.L - 1;
  size_t off = 0, n = 0;
  switch (id) {
    case DSSM_BUF_LOSS: off = Lt.loss; n = 8; break;
    case DSSM_BUF_COS_SIM_RAW: off = Lt.cos_raw; n = (size_t)K * Lt.BS * 4; break;
    case DSSM_BUF_COS_SIM: off = Lt.cos_sim; n = (size_t)K * Lt.BS * 4; break;
    case DSSM_BUF_PROB: off = Lt.prob; n = (size_t)K * Lt.BS * 4; break;
    case DSSM_BUF_QUERY_NORM: off = Lt.qnorm; n = (size_t)Lt.BS * 4; break;
    case DSSM_BUF_EMBED: off = Lt.A[Lt.L - 1]; n = (size_t)Lt.R * Lt.ldp[Lt.L - 1] * 4; break;
    case DSSM_BUF_Z: off = Lt.Z[layer]; n = (size_t)Lt.R * Lt.ldp[layer] * 4; break;
    case DSSM_BUF_BATCH_MEAN: off = Lt.bmean[layer]; n = (size_t)2 * Lt.n[layer] * 4; break;
    case DSSM_BUF_BATCH_VAR: off = Lt.bvar[layer]; n = (size_t)2 * Lt.n[layer] * 4; break;
    case DSSM_BUF_DZ: off = Lt.dZ[layer]; n = (size_t)Lt.R * Lt.ldp[layer] * (Lt.bf16 ? 2 : 4); break;
    case DSSM_BUF_A:
      off = Lt.A[layer];
      n = (size_t)Lt.R * Lt.ldp[layer] * (Lt.bf16 && layer < Lt.L - 1 ? 2 : 4);
      break;
    case DSSM_BUF_DA: off = Lt.dA[layer]; n = (size_t)Lt.R * Lt.ldp[layer] * 4; break;
    default: return fail(DSSM_E_INVALID, "unknown buffer id");
  }
  *ptr = P->ws + off;
  if (bytes) *bytes = n;
  return DSSM_OK;
}

int dssm_plan_set_batch(dssm_plan* P, const int32_t* indptr, const int32_t* indices,
                        const float* values) {
  if (!P || !indptr || (!indices && P->Lt.max_nnz) || (!values && P->Lt.max_nnz))
    return fail(DSSM_E_INVALID, "null batch pointer");
  P->indptr = indptr;
  P->indices = indices;
  P->values = values;
  return DSSM_OK;
}

int dssm_plan_sync_shadows(dssm_plan* P, void* stream) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  if (!P->Lt.bf16) return DSSM_OK;
  HIP_TRY(dssm::launch_shadow_sync(P->p, P->shadows(), (hipStream_t)stream));
  return DSSM_OK;
}

int dssm_plan_forward(dssm_plan* P, int train, void* stream) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  if (!P->indptr) return fail(DSSM_E_INVALID, "no batch set (dssm_plan_set_batch)");
  hipStream_t s = (hipStream_t)stream;
  const Layout& Lt = P->Lt;
  const dssm_config& c = P->cfg;
  const dssm::BnTowers tw{Lt.BS, Lt.R};
  const bool fused = train && P->fused_stats();
  const bool merged = train && P->merged_csc();
  if (train && P->fwd32() && !fused)
    return fail(DSSM_E_UNSUPPORTED, "FWD32 trains on the fused-statistics schedule only");
  if (train) {
    // The CSC transpose of the batch (dW1's operand).  Fused-statistics steps: its first launch
    // also clears the step's BN sums; merged: its scan / scatter ride in later launches.
    P->probe_begin(DSSM_PROBE_CSC, s);
    const bool hosted = merged && P->rank_done_for == P->indptr;  // done by the last Adam launch
    P->rank_done_for = nullptr;
    if (!hosted)
    HIP_TRY(dssm::launch_csc_build(P->indptr, P->indices, P->values, Lt.R, Lt.D, Lt.max_nnz,
                                   P->at<int>(Lt.csc_scratch), P->at<int>(Lt.col_ptr),
                                   P->at<int>(Lt.csc_row), P->at<float>(Lt.csc_val),
                                   P->csc_rank_path() ? nullptr : P->at<int>(Lt.csc_col), s,
                                   fused ? P->at<double>(Lt.sums) : nullptr,
                                   fused ? (int)(Lt.sums_bytes / 8) : 0, P->csc_rank_path(), merged,
                                   P->deterministic() && !merged ? P->at<int>(Lt.sort_row) : nullptr,
                                   P->deterministic() && !merged ? P->at<float>(Lt.sort_val) : nullptr));
    P->probe_end(DSSM_PROBE_CSC, s);
  }
  P->probe_begin(DSSM_PROBE_SPMM_FWD, s);
  if (merged) {  // the SpMM rows share their launch with the column scan
    HIP_TRY(dssm::launch_spmm_scan(P->indptr, P->indices, P->values, Lt.R,
                                   P->fwd_weight0(), P->fwd_weight0_bf16(), P->fwd_weight0_ld(), Lt.n[0], P->bias(0),
                                   P->at<float>(Lt.Z[0]), Lt.ldp[0], Lt.D, Lt.max_nnz,
                                   P->at<int>(Lt.csc_scratch), P->at<int>(Lt.col_ptr), s));
  } else {
    // eval: every layer's BN coefficients from the EMA, in the SpMM launch's extra workgroups
    dssm::EvalCoef ec{};
    if (!train) {
      static_assert(DSSM_MAX_LAYERS <= 8, "EvalCoef holds 8 layers");
      ec.L = Lt.L;
      ec.eps = c.bn_eps;
      for (int l = 0; l < Lt.L; ++l) {
        const float* ema = P->ema + Lt.ema_off[l];
        ec.n[l] = Lt.n[l];
        ec.ld[l] = Lt.ldp[l];
        ec.coef[l] = P->at<float>(Lt.coef[l]);
        for (int t = 0; t < 2; ++t) {
          ec.gamma[l][t] = P->p + Lt.bn_off[l][2 * t];
          ec.beta[l][t] = P->p + Lt.bn_off[l][2 * t + 1];
          ec.ema_mean[l][t] = ema + 2 * t * Lt.n[l];
          ec.ema_var[l][t] = ema + (2 * t + 1) * Lt.n[l];
        }
      }
    }
    HIP_TRY(dssm::launch_spmm_fwd(P->indptr, P->indices, P->values, Lt.R, P->fwd_weight0(),
                                P->fwd_weight0_bf16(), P->fwd_weight0_ld(), Lt.n[0], P->bias(0),
                                P->at<float>(Lt.Z[0]), Lt.ldp[0], s, train ? nullptr : &ec));
  }
  P->probe_end(DSSM_PROBE_SPMM_FWD, s);
  if (fused) {
    // BN1 sums by their own launch; each NT GEMM stages the previous layer's BN+ReLU and
    // accumulates its own output's sums, the cosine kernel the last layer's backward sums
    // (bnfuse.h).  Merged: the transpose's scatter rides beside the BN1 sums or, by default,
    // in the cosine launch (csc.h).
    dssm::CscScatter scat{};
    const bool scat_cos = merged && P->on(DSSM_OPT_SCATTER_IN_COS);
    const bool det = P->deterministic();
    // deterministic: the scatter writes the sort scratch, then every column is put in row order
    int* scat_row = det ? P->at<int>(Lt.sort_row) : P->at<int>(Lt.csc_row);
    float* scat_val = det ? P->at<float>(Lt.sort_val) : P->at<float>(Lt.csc_val);
    const dssm::BnSide b0 = P->bn_side(0);
    if (merged)
      HIP_TRY(dssm::launch_sums_scatter(P->at<float>(Lt.Z[0]), Lt.ldp[0], Lt.n[0], Lt.BS,
                                        P->at<double>(Lt.fsum[0]), P->indptr, P->indices, P->values,
                                        Lt.R, Lt.D, Lt.max_nnz, P->at<int>(Lt.csc_scratch),
                                        P->at<int>(Lt.col_ptr), scat_row, scat_val,
                                        nullptr, s, scat_cos ? &scat : nullptr,  // csc_col: unread on the rank path
                                        det ? &b0.fdet : nullptr));
    else
      HIP_TRY(dssm::launch_bn_sums(P->at<float>(Lt.Z[0]), Lt.ldp[0], Lt.n[0], tw,
                                   P->at<double>(Lt.fsum[0]), s, det ? &b0.fdet : nullptr));
    for (int l = 1; l < Lt.L; ++l) {
      const dssm::BnSide in = P->bn_side(l - 1);
      const dssm::BnSide out = P->bn_side(l);
      if (!Lt.bf16 || P->fwd32()) {  // fp32 parity mode / FWD32: W_l straight from the arena ([in x n])
        // FWD32: the activation the bf16 backward reads is written bf16 (the bf16 mode's rounding)
        HIP_TRY(dssm::launch_g32_fwd(Lt.R, Lt.n[l], Lt.n[l - 1], P->at<float>(Lt.Z[l - 1]), Lt.ldp[l - 1],
                                     P->at<float>(Lt.coef[l - 1]), &in, Lt.BS, P->p + Lt.fc_off[l], Lt.n[l],
                                     P->at<float>(Lt.Z[l]), Lt.ldp[l], P->bias(l),
                                     Lt.bf16 ? nullptr : P->at<float>(Lt.A[l - 1]),
                                     P->at<double>(Lt.fsum[l]), s, det ? &out.fdet : nullptr,
                                     Lt.bf16 ? P->at<uint16_t>(Lt.A[l - 1]) : nullptr));
        continue;
      }
      HIP_TRY(dssm::launch_gemm_nt_fwd_fused(
          Lt.R, Lt.n[l], Lt.n[l - 1], P->at<float>(Lt.Z[l - 1]), Lt.ldp[l - 1],
          P->at<float>(Lt.coef[l - 1]), &in, Lt.BS, P->at<uint16_t>(Lt.shadowT[l]), Lt.ldp[l - 1],
          P->at<float>(Lt.Z[l]), Lt.ldp[l], P->bias(l), P->at<uint16_t>(Lt.A[l - 1]),
          P->at<double>(Lt.fsum[l]), s, det ? &out.fdet : nullptr));
    }
    const int lL = Lt.L - 1;
    const dssm::BnSide last = P->bn_side(lL);
    HIP_TRY(dssm::launch_cosine_loss(
        P->at<float>(Lt.Z[lL]), Lt.ldp[lL], Lt.n[lL], Lt.BS, Lt.NEG, c.gamma,
        P->at<float>(Lt.coef[lL]), P->at<float>(Lt.A[lL]), P->at<float>(Lt.cos_raw),
        P->at<float>(Lt.cos_sim), P->at<float>(Lt.prob), P->at<float>(Lt.qnorm),
        P->at<float>(Lt.loss_j), P->at<float>(Lt.loss), P->at<float>(Lt.dA[lL]), s, &last,
        /*defer_finalize=*/true, scat_cos ? &scat : nullptr));
    if (merged && det)
      HIP_TRY(dssm::launch_csc_sort(P->at<int>(Lt.col_ptr), Lt.R, Lt.D, P->at<int>(Lt.sort_row),
                                    P->at<float>(Lt.sort_val), P->at<int>(Lt.csc_row),
                                    P->at<float>(Lt.csc_val), s, P->at<int>(Lt.csc_scratch), Lt.max_nnz));
    P->fwd_train_done = true;
    P->fwd_fused = true;
    P->loss_pending = true;
    return DSSM_OK;
  }
  P->fwd_fused = false;
  for (int l = 0; l < Lt.L; ++l) {
    float* ema = P->ema + Lt.ema_off[l];
    const int n = Lt.n[l];
    if (train)  // eval coefficients: written by the SpMM launch above
      HIP_TRY(dssm::launch_bn_fwd_stats(
          P->at<float>(Lt.Z[l]), Lt.ldp[l], n, tw, P->p + Lt.bn_off[l][0], P->p + Lt.bn_off[l][1],
          P->p + Lt.bn_off[l][2], P->p + Lt.bn_off[l][3], ema, ema + n, ema + 2 * n, ema + 3 * n,
          c.bn_eps, c.ema_decay, true, P->at<float>(Lt.bmean[l]), P->at<float>(Lt.bvar[l]),
          P->at<float>(Lt.partial), P->at<unsigned>(Lt.tickets[l][0]), P->at<float>(Lt.coef[l]), s));
    const bool last = l == Lt.L - 1;
    if (last) break;  // the cosine kernel applies the last BN+ReLU itself (and writes the embeddings)
    if (P->fwd32()) {
      // FWD32 eval: the fp32 parity mode's path -- BN + ReLU into an fp32 scratch (dA_l: free in a
      // forward; the backward rewrites it before reading) and the fp32 GEMM on the fp32 W_{l+1}
      HIP_TRY(dssm::launch_bn_apply(P->at<float>(Lt.Z[l]), Lt.ldp[l], n, tw, P->at<float>(Lt.coef[l]), true,
                                    P->ws + Lt.dA[l], false, s));
      HIP_TRY(dssm::launch_gemm(dssm::GEMM_FWD, false, Lt.R, Lt.n[l + 1], n, P->ws + Lt.dA[l], Lt.ldp[l],
                                P->p + Lt.fc_off[l + 1], Lt.n[l + 1], P->at<float>(Lt.Z[l + 1]), Lt.ldp[l + 1],
                                P->bias(l + 1), false, nullptr, s));
      continue;
    }
    if (!last && P->wholek(l + 1)) {
      // BN+ReLU of layer l applied while staging the next GEMM's A operand; the bf16 activation
      // is written once (for the dW GEMM) by the first column tile.
      HIP_TRY(dssm::launch_gemm_nt(Lt.R, Lt.n[l + 1], n, P->ws + Lt.Z[l], Lt.ldp[l], true,
                                   P->at<float>(Lt.coef[l]), Lt.BS,
                                   P->at<uint16_t>(Lt.shadowT[l + 1]), Lt.ldp[l],
                                   P->at<float>(Lt.Z[l + 1]), Lt.ldp[l + 1], P->bias(l + 1),
                                   P->at<uint16_t>(Lt.A[l]), s));
      continue;
    }
    HIP_TRY(dssm::launch_bn_apply(P->at<float>(Lt.Z[l]), Lt.ldp[l], n, tw,
                                  P->at<float>(Lt.coef[l]), true, P->ws + Lt.A[l],
                                  Lt.bf16 && !last, s));
    if (!last)
      HIP_TRY(dssm::launch_gemm(dssm::GEMM_FWD, Lt.bf16, Lt.R, Lt.n[l + 1], n, P->ws + Lt.A[l],
                                Lt.ldp[l], P->weight(l + 1), P->weight_ld(l + 1),
                                P->at<float>(Lt.Z[l + 1]), Lt.ldp[l + 1], P->bias(l + 1), false,
                                nullptr, s));
  }
  const int lL = Lt.L - 1;
  dssm::CscScatter scat{};  // merged (fp32 parity mode): the transpose's scatter rides in the cosine launch
  if (merged)
    scat = dssm::csc_scatter_args(P->indptr, P->indices, P->values, Lt.R, Lt.D, P->at<int>(Lt.csc_scratch),
                                  P->at<int>(Lt.col_ptr), P->at<int>(Lt.csc_row), P->at<float>(Lt.csc_val),
                                  nullptr);  // csc_col: unread on the rank path
  HIP_TRY(dssm::launch_cosine_loss(
      P->at<float>(Lt.Z[lL]), Lt.ldp[lL], Lt.n[lL], Lt.BS, Lt.NEG,
      c.gamma, P->at<float>(Lt.coef[lL]),
      P->at<float>(Lt.A[lL]), P->at<float>(Lt.cos_raw),
      P->at<float>(Lt.cos_sim), P->at<float>(Lt.prob), P->at<float>(Lt.qnorm),
      P->at<float>(Lt.loss_j), P->at<float>(Lt.loss),
      train ? P->at<float>(Lt.dA[lL]) : nullptr,  // eval: no gradient
      s, nullptr, /*defer_finalize=*/train != 0, merged ? &scat : nullptr));
  // train: the loss partials are reduced by the backward's first launch (or finalize_loss)
  P->loss_pending = train != 0;
  P->fwd_train_done = train != 0;
  return DSSM_OK;
}

static bool wire_gradient_pass(const dssm_plan* P);
static int launch_wire_gradient_pass(dssm_plan* P, hipStream_t s, int chunk);

// dW1 = X^T dZ1 from the batch's CSC transpose: heavy columns here, light columns either here
// (unfused) or inside the Adam step (fused).
static int dw1_backward(dssm_plan* P, hipStream_t s) {
  const Layout& Lt = P->Lt;
  P->probe_begin(DSSM_PROBE_DW1, s);
  // fused single-GPU step with the rank transpose: the heavy columns are computed inside Adam
  // (the DW1 probe then brackets no kernel)
  if (P->fused_w1_adam() && P->heavy_in_adam()) {
    P->probe_end(DSSM_PROBE_DW1, s);
    return DSSM_OK;
  }
  if (wire_gradient_pass(P)) {
    if (!P->dp_defer_gradpass)
      for (int c = 0; c < P->geo.wp; ++c)
        if (int rc = launch_wire_gradient_pass(P, s, c)) return rc;
    P->probe_end(DSSM_PROBE_DW1, s);
    return DSSM_OK;
  }
  HIP_TRY(dssm::launch_dw1(P->at<int>(Lt.col_ptr), P->at<int>(Lt.csc_row), P->at<float>(Lt.csc_val),
                           P->at<int>(Lt.csc_col), Lt.D, Lt.R, Lt.max_nnz, P->ws + Lt.dZ[0],
                           Lt.bf16, Lt.ldp[0], Lt.n[0], P->g + Lt.fc_off[0], !P->fused_w1_adam(), s,
                           P->csc_rank_path() ? P->at<int>(Lt.csc_scratch) : nullptr,
                           P->deterministic() ? P->at<float>(Lt.heavy_slab) : nullptr));
  P->probe_end(DSSM_PROBE_DW1, s);
  return DSSM_OK;
}

static int backward_impl(dssm_plan* P, void* stream);

int dssm_plan_backward(dssm_plan* P, void* stream) {
  if (int rc = backward_impl(P, stream)) return rc;
  if (P->gwire && !wire_gradient_pass(P))  // data parallel: the W1 gradient rows leave as bf16
    HIP_TRY(dssm::launch_wire_pack(P->g, P->gwire, P->Lt.D, P->geo, (hipStream_t)stream));
  return DSSM_OK;
}

static int backward_impl(dssm_plan* P, void* stream) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  if (!P->fwd_train_done) return fail(DSSM_E_INVALID, "backward needs a train-mode forward first");
  hipStream_t s = (hipStream_t)stream;
  const Layout& Lt = P->Lt;
  const dssm::BnTowers tw{Lt.BS, Lt.R};
  if (!P->grads_clean && P->fused_w1_adam()) {
    // backward() twice without an Adam step in between: re-zero the atomic-target blocks (only
    // the fused path leaves dW1's heavy rows to be cleared by Adam; otherwise dw1-light
    // overwrites every row before the heavy atomics).
    HIP_TRY(zero_bytes_async(P->g, sizeof(float) * (size_t)Lt.total, s));
  }
  P->grads_clean = false;
  if (P->fwd_fused) {
    // BN_L apply from the cosine kernel's sums, then per layer one launch for dA_{l-1} (with
    // BN_{l-1}'s backward sums) + dW_l, and BN_{l-1}'s apply.
    // DW_IN_APPLY: the pair launches run their dA tiles only (one round) and each dW_l's tiles
    // ride in the following apply launch (BN_{l-1}'s), whose element blocks leave CUs idle
    // bf16: the dW split-K tile sets handed from the pairs to the next apply (two when the pair in
    // between folded its BN backward, BNB_IN_PAIR), each with the gradient its slabs are summed into
    // when not deferred
    dssm::TnParams dwq[2] = {};
    float* dwq_reduce[2] = {nullptr, nullptr};
    int nq = 0;
    dssm::TnParams dw{};
    dssm::G32Params dw32{};   // fp32: the same for the g32.h tiles (one set)
    bool dw_pending = false;
    float* dw_reduce_to = nullptr;
    // dW_l's split-K slabs summed later: by the fused Adam step, or by the wire gradient pass
    const bool defer_slabs = P->fused_w1_adam() || wire_gradient_pass(P);
    for (int l = Lt.L - 1; l >= 0; --l) {
      const dssm::BnSide b = P->bn_side(l);
      const bool fin = l == Lt.L - 1;  // the forward's loss, deferred to this launch
      const float* lp = fin ? P->at<float>(Lt.loss_j) : nullptr;
      const int lb = dssm::cosine_blocks(Lt.BS, Lt.n[Lt.L - 1], true);
      const bool folded = P->bnb_fold(l);  // BN_l's backward rides in the pair launch below
      if (folded) {
        // nothing here: the pending dW tile sets wait for the next apply
      } else if (Lt.bf16) {
        HIP_TRY(dssm::launch_bn_bwd_apply_fused(P->at<float>(Lt.Z[l]), P->at<float>(Lt.dA[l]), b,
                                                P->at<uint16_t>(Lt.dZ[l]), s, lp, lb, P->at<float>(Lt.loss),
                                                nq > 0 ? &dwq[0] : nullptr, nq > 1 ? &dwq[1] : nullptr));
        for (int q = 0; q < nq; ++q)
          if (dwq_reduce[q])  // not deferred to Adam: the slabs summed right after
            HIP_TRY(dssm::launch_splitk_reduce(dwq[q].C, (dwq[q].K + dwq[q].k_per_split - 1) / dwq[q].k_per_split,
                                               (int64_t)dwq[q].M * dwq[q].N, dwq_reduce[q], s));
        nq = 0;
      } else {
        HIP_TRY(dssm::launch_bn_bwd_apply_fused32(P->at<float>(Lt.Z[l]), P->at<float>(Lt.dA[l]), b,
                                                  P->at<float>(Lt.dZ[l]), s, lp, lb, P->at<float>(Lt.loss),
                                                  dw_pending ? &dw32 : nullptr));
        if (dw_pending && dw_reduce_to)  // not deferred to Adam: the slabs summed right after
          HIP_TRY(dssm::launch_splitk_reduce(dw32.C, (dw32.K + dw32.k_per_split - 1) / dw32.k_per_split,
                                             (int64_t)dw32.M * dw32.N, dw_reduce_to, s));
      }
      dw_pending = false;
      dw_reduce_to = nullptr;
      if (fin) P->loss_pending = false;
      if (l == 0) break;
      const bool host_dw = P->on(DSSM_OPT_DW_IN_APPLY);
      const dssm::BnSide bprev = P->bn_side(l - 1);
      dw = dssm::TnParams{};  // filled by the pair launch when it hands its dW tiles over
      dw32 = dssm::G32Params{};
      float* gw = P->g + Lt.fc_off[l];
      if (folded)
        HIP_TRY(dssm::launch_bwd_pair_bnb(
            Lt.R, Lt.in_dim[l], Lt.n[l], P->at<float>(Lt.dA[l]), P->at<float>(Lt.Z[l]), b,
            P->at<uint16_t>(Lt.dZ[l]), Lt.ldp[l], P->at<uint16_t>(Lt.shadow[l]), Lt.ldp[l],
            P->at<float>(Lt.dA[l - 1]), Lt.ldp[l - 1], P->at<float>(Lt.Z[l - 1]), P->at<float>(Lt.coef[l - 1]),
            P->at<double>(Lt.bsum[l - 1]), Lt.BS, P->at<uint16_t>(Lt.A[l - 1]), Lt.ldp[l - 1],
            P->at<float>(Lt.dw_slab[l]), gw, defer_slabs, s, &P->dw_deferred[l], &dw,
            P->deterministic() ? &bprev.bdet : nullptr, lp, lb, P->at<float>(Lt.loss)));
      else if (Lt.bf16)
        HIP_TRY(dssm::launch_bwd_pair(
            Lt.R, Lt.in_dim[l], Lt.n[l], P->at<uint16_t>(Lt.dZ[l]), Lt.ldp[l],
            P->at<uint16_t>(Lt.shadow[l]), Lt.ldp[l], P->at<float>(Lt.dA[l - 1]), Lt.ldp[l - 1],
            P->at<float>(Lt.Z[l - 1]), P->at<float>(Lt.coef[l - 1]), P->at<double>(Lt.bsum[l - 1]),
            Lt.BS, P->at<uint16_t>(Lt.A[l - 1]), Lt.ldp[l - 1], P->at<float>(Lt.dw_slab[l]),
            gw, defer_slabs, s, &P->dw_deferred[l], host_dw ? &dw : nullptr,
            P->deterministic() ? &bprev.bdet : nullptr));
      else  // fp32: W_l [in x n] from the arena is dA's B^T as it lies
        HIP_TRY(dssm::launch_g32_pair(
            Lt.R, Lt.in_dim[l], Lt.n[l], P->at<float>(Lt.dZ[l]), Lt.ldp[l], P->p + Lt.fc_off[l], Lt.n[l],
            P->at<float>(Lt.dA[l - 1]), Lt.ldp[l - 1], P->at<float>(Lt.Z[l - 1]), P->at<float>(Lt.coef[l - 1]),
            P->at<double>(Lt.bsum[l - 1]), Lt.BS, P->at<float>(Lt.A[l - 1]), Lt.ldp[l - 1],
            P->at<float>(Lt.dw_slab[l]), gw, defer_slabs, s, &P->dw_deferred[l], host_dw ? &dw32 : nullptr,
            P->deterministic() ? &bprev.bdet : nullptr));
      const float* handed = Lt.bf16 ? dw.C : dw32.C;
      dw_pending = host_dw && handed != nullptr;
      if (dw_pending && !defer_slabs && handed != gw) dw_reduce_to = gw;
      if (Lt.bf16 && dw_pending) {  // queued for the next apply
        if (nq == 2) return fail(DSSM_E_INVALID, "internal: more than two pending dW tile sets");
        dwq[nq] = dw;
        dwq_reduce[nq++] = dw_reduce_to;
      }
    }
    return dw1_backward(P, s);
  }
  for (int l = Lt.L - 1; l >= 0; --l) {
    const int n = Lt.n[l];
    const bool fin = l == Lt.L - 1 && P->loss_pending;  // the forward's loss, deferred to this launch
    HIP_TRY(dssm::launch_bn_bwd(P->at<float>(Lt.Z[l]), P->at<float>(Lt.dA[l]), Lt.ldp[l], n, tw,
                                P->at<float>(Lt.coef[l]), P->g + Lt.bn_off[l][0],
                                P->g + Lt.bn_off[l][1], P->g + Lt.bn_off[l][2],
                                P->g + Lt.bn_off[l][3], P->at<float>(Lt.partial),
                                P->at<unsigned>(Lt.tickets[l][1]), P->at<float>(Lt.bcoef[l]),
                                P->ws + Lt.dZ[l], Lt.bf16, s, fin ? P->at<float>(Lt.loss_j) : nullptr,
                                dssm::cosine_blocks(Lt.BS, Lt.n[Lt.L - 1], false), P->at<float>(Lt.loss)));
    if (fin) P->loss_pending = false;
    if (l > 0) {
      const int kin = Lt.in_dim[l];
      float* gw = P->g + Lt.fc_off[l];
      HIP_TRY(dssm::launch_gemm(dssm::GEMM_DW, Lt.bf16, kin + 1, n, Lt.R, P->ws + Lt.A[l - 1],
                                Lt.ldp[l - 1], P->ws + Lt.dZ[l], Lt.ldp[l], gw, n, nullptr, true,
                                P->at<float>(Lt.dw_slab[l]), s,
                                P->fused_w1_adam() ? &P->dw_deferred[l] : nullptr));
      if (!P->fused_w1_adam()) P->dw_deferred[l] = 0;
      if (P->wholek(l))  // dA = dZ . W^T: the weight shadow rows are already k-contiguous
        HIP_TRY(dssm::launch_gemm_nt(Lt.R, kin, n, P->ws + Lt.dZ[l], Lt.ldp[l], false, nullptr,
                                     Lt.BS, P->at<uint16_t>(Lt.shadow[l]), Lt.ldp[l],
                                     P->at<float>(Lt.dA[l - 1]), Lt.ldp[l - 1], nullptr, nullptr, s));
      else
        HIP_TRY(dssm::launch_gemm(dssm::GEMM_DA, Lt.bf16, Lt.R, kin, n, P->ws + Lt.dZ[l],
                                  Lt.ldp[l], P->weight(l), P->weight_ld(l),
                                  P->at<float>(Lt.dA[l - 1]), Lt.ldp[l - 1], nullptr, false,
                                  nullptr, s));
    } else {
      return dw1_backward(P, s);
    }
  }
  return DSSM_OK;
}

// The W1 roles of k_adam_step (inline gather of the light rows from the CSC transpose, heavy
// columns as work items): shared by the fused single-GPU Adam and the data-parallel gradient pass.
static void fill_w1_roles(dssm_plan* P, dssm::AdamStep& a) {
  const Layout& Lt = P->Lt;
  a.w1_blocks = 1;  // sized by the launcher
  a.D = Lt.D;
  a.n = Lt.n[0];
  a.col_ptr = P->at<int>(Lt.col_ptr);
  a.csc_row = P->at<int>(Lt.csc_row);
  a.csc_val = P->at<float>(Lt.csc_val);
  a.dZ = P->ws + Lt.dZ[0];
  a.lddz = Lt.ldp[0];
  a.shadow = Lt.bf16 ? P->at<uint16_t>(Lt.shadow[0]) : nullptr;
  a.ldsh = Lt.ldp[0];
  if (P->heavy_in_adam()) {
    int* scr = P->at<int>(Lt.csc_scratch);
    a.item_blocks = dssm::kAdamItemBlocks;
    a.heavy_n = dssm::csc_heavy_count(scr, Lt.D, Lt.max_nnz);
    a.heavy_items = reinterpret_cast<const int2*>(a.heavy_n + 64);
    a.heavy_ticket = dssm::csc_heavy_tickets(scr, Lt.D, Lt.R, Lt.max_nnz);
    a.heavy_slab = P->deterministic() ? P->at<float>(Lt.heavy_slab) : nullptr;
  }
}

// Data parallel with the bf16 wire: dW1 straight into the gradient wire (bf16 rows, b1's row fp32
// into the gradient arena) by k_adam_step's W1 roles in gradient-pass mode, instead of the
// materialising dW1 launches + the wire pack.
static bool wire_gradient_pass(const dssm_plan* P) {
  return P->gwire && !P->fused_w1_adam() && P->heavy_in_adam() && P->on(DSSM_OPT_WIRE_GRAD_PASS);
}

static int launch_wire_gradient_pass(dssm_plan* P, hipStream_t s, int chunk) {
  dssm::AdamStep a{};
  a.p = P->p;
  a.g = P->g;
  a.m = P->m;
  a.v = P->v;
  a.st = P->at<float>(P->Lt.adam_state);
  a.lr = P->cfg.lr;
  a.beta1 = P->cfg.beta1;
  a.beta2 = P->cfg.beta2;
  a.eps = P->cfg.adam_eps;
  a.gs = 1.0f;
  a.clear_from = P->Lt.total;
  fill_w1_roles(P, a);
  a.shadow = nullptr;
  a.gout = P->gwire;
  a.geo = P->geo;
  a.wchunk = P->geo.wp > 1 ? chunk : -1;
  if (P->peer_on()) {  // rank i's rows of owner j: block i of j's stage (the all-to-all's layout)
    const int64_t sub = P->sub_elems();
    a.npeer = P->peer.world;
    for (int j = 0; j < a.npeer; ++j)
      a.gpeer[j] = reinterpret_cast<uint16_t*>(reinterpret_cast<intptr_t>(P->peer.stage[j]) +
                                               (intptr_t)((int64_t)(P->dp_rank - j) * sub * 2));
  }
  // the pass of b1's row (the last chunk) also sums the deferred dW_l split-K slabs into the
  // gradient arena (no separate reduce launches; the tail's all-reduce follows this launch)
  if (chunk < 0 || chunk == P->geo.wp - 1) {
    const Layout& Lt = P->Lt;
    int64_t lo = Lt.total, hi = 0;
    for (int l = 1; l < Lt.L; ++l)
      if (P->dw_deferred[l] > 0) {
        dssm::SlabSeg& sg = a.slabs.seg[a.slabs.count++];
        sg.offset = Lt.fc_off[l];
        sg.count = (int64_t)(Lt.in_dim[l] + 1) * Lt.n[l];
        sg.splits = P->dw_deferred[l];
        sg.slab = P->at<float>(Lt.dw_slab[l]);
        lo = std::min(lo, sg.offset);
        hi = std::max(hi, sg.offset + sg.count);
      }
    if (a.slabs.count) {
      if ((lo % 4) || (hi % 4)) return fail(DSSM_E_INVALID, "dW slab segments must be 4-aligned");
      a.slab_to_g = 1;
      a.t4_begin = lo / 4;
      a.t4_end = hi / 4;
    }
  }
  HIP_TRY(dssm::launch_adam_step(a, P->Lt.bf16, s));
  if (a.slab_to_g)
    for (int l = 1; l < P->Lt.L; ++l) P->dw_deferred[l] = 0;  // the arena holds dW_l now
  return DSSM_OK;
}

// One launch of the data-parallel Adam step: this rank's W1 sub-chunk c (its gradient the fp32
// sum of the world's bf16 partials in the stage, its bf16 parameters into the wire); the last
// chunk also updates the replicated tail, hosts any rank role and advances the beta powers.
static int dp_adam_chunk(dssm_plan* P, const dssm::AdamStep& base, int c, hipStream_t s) {
  dssm::AdamStep a = base;
  const bool last = c == P->geo.wp - 1;
  int r0, r1;
  P->dp_chunk_rows(c, r0, r1);
  const int n = P->geo.n;
  a.d4_begin = (int64_t)r0 * n / 4;
  a.d4_end = (int64_t)std::max(r0, r1) * n / 4;
  const int64_t sub = P->sub_elems();
  a.gstage = P->gstage + (int64_t)c * P->geo.ww * sub;
  a.gbase4 = a.d4_begin;
  a.pwire_off4 = ((int64_t)c * P->geo.ww + P->dp_rank) * sub / 4 - a.d4_begin;
  if (P->peer_on()) {  // bf16(W1) of the shard into every rank's parameter wire
    a.npeer = P->peer.world;
    for (int k = 0; k < a.npeer; ++k) a.ppeer[k] = P->peer.pwire[k];
    if (last) {  // the replicated tail's gradient: the world's pushed partials, summed in rank order
      a.ptail = P->peer.tail[P->dp_rank];
      a.tailn = P->Lt.total - P->wire_end();
      a.tail0 = P->wire_end();
    }
  }
  if (!last) {
    a.t4_begin = a.t4_end = 0;
    a.no_advance = 1;
    a.clear_from = P->Lt.total;
    a.sh.count = 0;
    a.slabs.count = 0;
    a.rank = dssm::CscRankRole{};
    a.heavy_reset = nullptr;
  }
  HIP_TRY(dssm::launch_adam_step(a, P->Lt.bf16, s));
  return DSSM_OK;
}

int dssm_plan_adam(dssm_plan* P, float grad_scale, void* stream) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  const dssm_config& c = P->cfg;
  const Layout& Lt = P->Lt;
  float* st = P->at<float>(Lt.adam_state);
  hipStream_t s = (hipStream_t)stream;
  const int64_t rest = Lt.L > 1 ? Lt.fc_off[1] : Lt.bn_off[0][0];
  dssm::ShadowList sh = P->shadows();
  dssm::AdamStep a{};
  a.p = P->p;
  a.g = P->g;
  a.m = P->m;
  a.v = P->v;
  a.st = st;
  a.ticket = reinterpret_cast<unsigned*>(st + 64);
  a.lr = c.lr;
  a.beta1 = c.beta1;
  a.beta2 = c.beta2;
  a.eps = c.adam_eps;
  a.gs = grad_scale;
  a.clear_from = Lt.total;
  a.d4_begin = P->adam_begin / 4;
  a.d4_end = (P->adam_end >= 0 ? P->adam_end : Lt.total) / 4;
  if (P->fused_w1_adam() && (P->adam_begin != 0 || (P->adam_end >= 0 && P->adam_end != Lt.total)))
    return fail(DSSM_E_INVALID, "a sharded Adam range needs the fused W1 Adam off");
  if (P->pwire && P->fused_w1_adam()) return fail(DSSM_E_INVALID, "the bf16 wire needs the fused W1 Adam off");
  if (P->pwire) {
    // bf16 wire: the rank's W1 shard, sub-chunk by sub-chunk, from the all-to-all's stage (writing
    // the parameter wire); the last launch also takes the replicated fp32 tail [wire_end, total)
    // with its shadows and advances the beta powers
    const int64_t we = P->wire_end();
    a.t4_begin = we / 4;
    a.t4_end = Lt.total / 4;
    a.gwire = P->gwire;
    a.pwire = P->pwire;
    a.wire4 = we / 4;
    a.gstage = P->gstage;
    a.gparts = P->geo.ww;
    a.gstride = P->sub_elems();
    // the tail's gradient is consumed here; clear it (b1's row is the gradient pass's atomic target)
    if (wire_gradient_pass(P)) a.clear_from = we;
    for (int i = 1; i < sh.count; ++i) sh.seg[i - 1] = sh.seg[i];  // W1's shadow: from the wire
    if (sh.count) sh.count -= 1;
  }
  if (P->fused_w1_adam()) {
    if (P->grads_clean) return fail(DSSM_E_INVALID, "fused W1 Adam needs backward() of this step first");
    fill_w1_roles(P, a);
    a.d4_begin = rest / 4;
    if (sh.count) {  // W1's shadow is written by the fused rows
      for (int i = 1; i < sh.count; ++i) sh.seg[i - 1] = sh.seg[i];
      sh.count -= 1;
    }
  }
  // the next step's rank pass as workgroups of this step's (last) launch (multi-step graphs); the
  // heavy-item count it re-arms was consumed by this launch's W1 roles (fused) or the backward's
  // gradient pass (data parallel)
  int* heavy_n = P->heavy_in_adam() ? dssm::csc_heavy_count(P->at<int>(Lt.csc_scratch), Lt.D, Lt.max_nnz) : nullptr;
  if (P->host_rank_indptr && (P->fused_w1_adam() || wire_gradient_pass(P)) && heavy_n && P->merged_csc() &&
      Lt.D <= dssm::kRankMaxD) {
    a.rank = dssm::csc_rank_role_args(P->host_rank_indptr, P->host_rank_indices, Lt.R, Lt.D,
                                      P->at<int>(Lt.csc_scratch), P->at<double>(Lt.sums),
                                      (int)(Lt.sums_bytes / 8));
    a.heavy_reset = heavy_n;
    P->rank_done_for = P->host_rank_indptr;
  }
  P->host_rank_indptr = nullptr;
  P->host_rank_indices = nullptr;
  for (int l = 1; l < Lt.L; ++l)
    if (P->dw_deferred[l] > 0) {  // dW_l still in its split-K slab: summed inside the step
      dssm::SlabSeg& sg = a.slabs.seg[a.slabs.count++];
      sg.offset = Lt.fc_off[l];
      sg.count = (int64_t)(Lt.in_dim[l] + 1) * Lt.n[l];
      sg.splits = P->dw_deferred[l];
      sg.slab = P->at<float>(Lt.dw_slab[l]);
    }
  a.sh = sh;
  P->probe_begin(DSSM_PROBE_ADAM, s);
  if (P->pwire) {
    // the Adam probe ends with the last chunk's Adam launch; the all-gather behind it (the data-
    // parallel graph's hook) has its own probe
    for (int c = 0; c < P->geo.wp; ++c) {
      const bool last = c == P->geo.wp - 1;
      if (int rc = dp_adam_chunk(P, a, c, s)) return rc;
      if (last) P->probe_end(DSSM_PROBE_ADAM, s);
      if (P->dp_hook) {
        if (last) P->probe_begin(DSSM_PROBE_DP_ALL_GATHER, s);
        if (int rc = P->dp_hook(c)) return rc;
        if (last) P->probe_end(DSSM_PROBE_DP_ALL_GATHER, s);
      }
    }
  } else {
    HIP_TRY(dssm::launch_adam_step(a, Lt.bf16, s));
    P->probe_end(DSSM_PROBE_ADAM, s);
  }
  P->grads_clean = true;
  return DSSM_OK;
}

int dssm_plan_set_adam_range(dssm_plan* P, int64_t begin, int64_t end) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  const int64_t total = P->Lt.total;
  if (begin < 0 || end < begin || end > total || (begin % 4) || (end % 4 && end != total))
    return fail(DSSM_E_INVALID, "adam range must be 4-aligned within [0, param_count]");
  if ((end % 4) && end == total) return fail(DSSM_E_INVALID, "param_count is a multiple of 64");
  P->adam_begin = begin;
  P->adam_end = end;
  return DSSM_OK;
}

int64_t dssm_plan_wire_extent(const dssm_plan* P) { return P ? P->wire_end() : -1; }

static dssm::WireGeo dp_geo(const dssm_plan* P, int world, int chunks) {
  dssm::WireGeo g{};
  g.ww = world;
  g.wp = chunks;
  g.ws = (P->Lt.D + world * chunks - 1) / (world * chunks);
  g.n = P->Lt.n[0];
  return g;
}

int64_t dssm_plan_dp_wire_size(const dssm_plan* P, int world, int chunks) {
  if (!P || world < 1 || chunks < 1) return -1;
  const dssm::WireGeo g = dp_geo(P, world, chunks);
  // + 8 elements of slack: the SpMM's tight-row reads of the parameter wire load up to 8 B past the
  // last row (RawRow8<u16t>, masked)
  return (int64_t)g.ww * g.wp * g.ws * g.n + 8;
}

int dssm_plan_set_dp_wire(dssm_plan* P, int world, int rank, int chunks, uint16_t* grad_wire,
                          const uint16_t* stage, uint16_t* param_wire, int64_t count) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  if (P->capturing) return fail(DSSM_E_INVALID, "the wire cannot change during a graph capture");
  {  // a new wire drops the peer set (dssm_plan_set_dp_peers maps the new buffers)
    const unsigned long long t = P->peer.wait_ticks;
    P->peer = dssm_plan::PeerSet{};
    P->peer.wait_ticks = t;
  }
  if (!grad_wire && !param_wire && !stage) {
    P->gwire = P->pwire = nullptr;
    P->gstage = nullptr;
    P->geo = dssm::WireGeo{};
    return DSSM_OK;
  }
  if (!grad_wire || !param_wire || !stage) return fail(DSSM_E_INVALID, "grad_wire, stage and param_wire, or none");
  if (!P->Lt.bf16) return fail(DSSM_E_UNSUPPORTED, "the bf16 wire is a bf16-mode (perf) option");
  if (P->fused_w1_adam()) return fail(DSSM_E_INVALID, "the bf16 wire needs the fused W1 Adam off");
  if (world < 1 || rank < 0 || rank >= world || chunks < 1 || chunks > 64)
    return fail(DSSM_E_INVALID, "dp wire: 0 <= rank < world, 1 <= chunks <= 64");
  if (world > 1 && stage == grad_wire) return fail(DSSM_E_INVALID, "the stage is the all-to-all's output");
  if (P->Lt.fc_off[0] != 0 || (P->Lt.n[0] % 4))
    return fail(DSSM_E_UNSUPPORTED, "the wire needs W1 at arena offset 0 and a width multiple of 4");
  if (count < dssm_plan_dp_wire_size(P, world, chunks))
    return fail(DSSM_E_INVALID, "wire buffers must hold dssm_plan_dp_wire_size() elements");
  if ((reinterpret_cast<uintptr_t>(grad_wire) | reinterpret_cast<uintptr_t>(param_wire) |
       reinterpret_cast<uintptr_t>(stage)) & 7)
    return fail(DSSM_E_INVALID, "wire buffers must be 8-byte aligned");
  P->gwire = grad_wire;
  P->pwire = param_wire;
  P->gstage = stage;
  P->geo = dp_geo(P, world, chunks);
  P->dp_rank = rank;
  return DSSM_OK;
}

int dssm_plan_dp_geometry(const dssm_plan* P, int64_t* out) {
  if (!P || !out) return fail(DSSM_E_INVALID, "null argument");
  if (!P->pwire) return fail(DSSM_E_INVALID, "no wire set (dssm_plan_set_dp_wire)");
  const dssm::WireGeo& g = P->geo;
  const int64_t r0 = std::min<int64_t>((int64_t)P->dp_rank * g.wp * g.ws, P->Lt.D);
  const int64_t r1 = std::min<int64_t>(r0 + (int64_t)g.wp * g.ws, P->Lt.D);
  out[0] = g.ww;
  out[1] = g.wp;
  out[2] = g.ws;
  out[3] = P->sub_elems();
  out[4] = r0 * g.n;  // this rank's W1 shard in the arena: [out[4], out[5])
  out[5] = r1 * g.n;
  out[6] = P->wire_end();
  out[7] = P->Lt.total;
  return DSSM_OK;
}

int dssm_plan_wire_shadows(dssm_plan* P, void* stream) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  if (!P->pwire) return fail(DSSM_E_INVALID, "no wire set (dssm_plan_set_dp_wire)");
  if (P->peer_on()) HIP_TRY(dssm::launch_peer_shadow(P->pwire, P->shadows().seg[0], (hipStream_t)stream));
  else HIP_TRY(dssm::launch_wire_shadow(P->pwire, P->shadows().seg[0], P->geo, -1, (hipStream_t)stream));
  return DSSM_OK;
}

static dssm::PeerArgs peer_args(const dssm_plan* P) {
  dssm::PeerArgs a{};
  a.world = P->peer.world;
  a.rank = P->dp_rank;
  a.flags = P->peer.flags[P->dp_rank];
  for (int k = 0; k < a.world; ++k) {
    a.rflags[k] = P->peer.flags[k];
    a.rtail[k] = P->peer.tail[k];
  }
  const int64_t we = P->wire_end();
  a.tail_src = P->g + we;
  a.tailn = P->Lt.total - we;
  a.ticks = P->peer.wait_ticks;
  return a;
}

int dssm_plan_set_dp_peers(dssm_plan* P, int world, uint16_t* const* stages, uint16_t* const* param_wires,
                           float* const* tails, unsigned* const* flags) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  if (P->capturing) return fail(DSSM_E_INVALID, "the peers cannot change during a graph capture");
  if (!stages && !param_wires && !tails && !flags) {
    P->peer = dssm_plan::PeerSet{};
    return DSSM_OK;
  }
  if (!stages || !param_wires || !tails || !flags) return fail(DSSM_E_INVALID, "stages, param_wires, tails and flags, or none");
  if (!P->pwire) return fail(DSSM_E_INVALID, "set the bf16 wire first (dssm_plan_set_dp_wire)");
  if (world < 1 || world > dssm::kPeerMax || world != P->geo.ww)
    return fail(DSSM_E_INVALID, "peer exchange: world must be the wire's world size, at most 8");
  if (P->geo.wp != 1) return fail(DSSM_E_UNSUPPORTED, "peer exchange: one wire chunk");
  if (!wire_gradient_pass(P)) return fail(DSSM_E_UNSUPPORTED, "peer exchange: needs the wire gradient pass");
  if ((P->Lt.total - P->wire_end()) % 4) return fail(DSSM_E_UNSUPPORTED, "peer exchange: tail not a multiple of 4");
  for (int k = 0; k < world; ++k)
    if (!stages[k] || !param_wires[k] || !tails[k] || !flags[k]) return fail(DSSM_E_INVALID, "null peer buffer");
  if (stages[P->dp_rank] != P->gstage || param_wires[P->dp_rank] != P->pwire)
    return fail(DSSM_E_INVALID, "this rank's stage and parameter wire must be the wire's (dssm_plan_set_dp_wire)");
  if (!P->peer_scratch) HIP_TRY(hipMalloc(&P->peer_scratch, sizeof(uint16_t*) * dssm::kPeerMax + 64));
  dssm_plan::PeerSet ps;
  ps.world = world;
  ps.wait_ticks = P->peer.wait_ticks;
  for (int k = 0; k < world; ++k) {
    ps.stage[k] = stages[k];
    ps.pwire[k] = param_wires[k];
    ps.tail[k] = tails[k];
    ps.flags[k] = flags[k];
  }
  P->peer = ps;
  return DSSM_OK;
}

int dssm_plan_set_peer_timeout(dssm_plan* P, double ms) {
  if (!P || !(ms > 0.0)) return fail(DSSM_E_INVALID, "null plan or timeout <= 0");
  P->peer.wait_ticks = (unsigned long long)(ms * 1e5);  // 100 MHz counter
  return DSSM_OK;
}

int dssm_plan_peer_exchange(dssm_plan* P, int phase, void* stream) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  if (!P->peer_on()) return fail(DSSM_E_INVALID, "no peer exchange set (dssm_plan_set_dp_peers)");
  hipStream_t s = (hipStream_t)stream;
  const dssm::PeerArgs a = peer_args(P);
  if (phase == 0) HIP_TRY(dssm::launch_peer_before_adam(a, s));
  else if (phase == 1) HIP_TRY(dssm::launch_peer_after_adam(a, s));
  else return fail(DSSM_E_INVALID, "phase: 0 (before Adam) or 1 (after Adam)");
  return DSSM_OK;
}

int dssm_plan_peer_selftest(dssm_plan* P, int64_t* mismatches, void* stream) {
  if (!P || !mismatches) return fail(DSSM_E_INVALID, "null argument");
  if (!P->peer_on()) return fail(DSSM_E_INVALID, "no peer exchange set (dssm_plan_set_dp_peers)");
  if (P->capturing) return fail(DSSM_E_INVALID, "the self-test cannot be captured");
  hipStream_t s = (hipStream_t)stream;
  const dssm::PeerArgs a = peer_args(P);
  const int W = P->peer.world;
  void* dev = P->peer_scratch;  // [W] parameter-wire pointers + the mismatch counter
  uint16_t** pw = static_cast<uint16_t**>(dev);
  unsigned* bad = reinterpret_cast<unsigned*>(static_cast<char*>(dev) + sizeof(uint16_t*) * dssm::kPeerMax);
  hipError_t e = hipMemcpyAsync(pw, P->peer.pwire, sizeof(uint16_t*) * W, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemsetAsync(bad, 0, sizeof(unsigned), s);
  if (e == hipSuccess) e = dssm::launch_peer_selftest(a, pw, P->pwire, P->sub_elems(), bad, s);
  unsigned nb = 0, err = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&nb, bad, sizeof(unsigned), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(&err, a.flags + dssm::kPeerErr, sizeof(unsigned), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return fail(DSSM_E_HIP, std::string("peer self-test: ") + hipGetErrorString(e));
  *mismatches = err ? -1 : (int64_t)nb;  // -1: a wait timed out
  return DSSM_OK;
}

int dssm_plan_peer_status(const dssm_plan* P, unsigned* out2) {
  if (!P || !out2) return fail(DSSM_E_INVALID, "null argument");
  if (!P->peer_on()) return fail(DSSM_E_INVALID, "no peer exchange set (dssm_plan_set_dp_peers)");
  unsigned* f = P->peer.flags[P->dp_rank];
  HIP_TRY(hipMemcpy(&out2[0], f + dssm::kPeerErr, sizeof(unsigned), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&out2[1], f + dssm::kPeerSeq, sizeof(unsigned), hipMemcpyDeviceToHost));
  return DSSM_OK;
}

int dssm_plan_set_fused_w1_adam(dssm_plan* P, int on) {
  return dssm_plan_set_option(P, DSSM_OPT_FUSED_W1_ADAM, on);
}

int dssm_plan_train_step(dssm_plan* P, void* stream) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  int rc = dssm_plan_forward(P, 1, stream);
  if (!rc) rc = dssm_plan_backward(P, stream);
  if (!rc) rc = dssm_plan_adam(P, 1.0f, stream);
  return rc;
}

int dssm_plan_finalize_loss(dssm_plan* P, void* stream) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  if (P->loss_pending) {
    HIP_TRY(dssm::launch_loss_finalize(P->at<float>(P->Lt.loss_j), P->Lt.BS, P->Lt.n[P->Lt.L - 1],
                                       P->at<float>(P->Lt.loss), (hipStream_t)stream, P->fwd_fused));
    P->loss_pending = false;
  }
  return DSSM_OK;
}

int dssm_plan_schedule(const dssm_plan* P) {
  if (!P) return 0;
  int f = 0;
  const bool fs = P->fused_stats();
  if (fs) f |= DSSM_SCHED_FUSED_STATS;
  if (P->merged_csc()) f |= DSSM_SCHED_MERGED_CSC;
  if (P->heavy_in_adam()) f |= DSSM_SCHED_HEAVY_IN_ADAM;
  if (P->fused_w1_adam()) f |= DSSM_SCHED_FUSED_W1_ADAM;
  bool wk = P->Lt.L > 1, w32 = P->Lt.L > 1;
  for (int l = 1; l < P->Lt.L; ++l) {
    wk = wk && P->wholek(l);
    w32 = w32 && P->nt32(l);
  }
  if (wk) f |= DSSM_SCHED_WHOLEK;
  if (fs && w32) f |= DSSM_SCHED_NT32;
  if (fs && P->on(DSSM_OPT_DW_IN_APPLY)) f |= DSSM_SCHED_DW_IN_APPLY;
  if (P->merged_csc() && P->on(DSSM_OPT_SCATTER_IN_COS)) f |= DSSM_SCHED_SCATTER_IN_COS;
  if (P->deterministic()) f |= DSSM_SCHED_DETERMINISTIC;
  if (P->bnb_in_pair()) f |= DSSM_SCHED_BNB_IN_PAIR;
  if (P->fwd32()) f |= DSSM_SCHED_FWD32;
  return f;
}

int dssm_plan_fused_stats(dssm_plan* P) { return P && P->fused_stats() ? 1 : 0; }

int dssm_plan_set_adam_state(dssm_plan* P, float beta1_power, float beta2_power, void* stream) {
  if (!P) return fail(DSSM_E_INVALID, "null plan");
  const float st[2] = {beta1_power, beta2_power};
  HIP_TRY(hipMemcpyAsync(P->ws + P->Lt.adam_state, st, sizeof st, hipMemcpyHostToDevice,
                         (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return DSSM_OK;
}

int dssm_plan_get_adam_state(dssm_plan* P, float* beta1_power, float* beta2_power, void* stream) {
  if (!P || !beta1_power || !beta2_power) return fail(DSSM_E_INVALID, "null argument");
  float st[2];
  HIP_TRY(hipMemcpyAsync(st, P->ws + P->Lt.adam_state, sizeof st, hipMemcpyDeviceToHost,
                         (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  *beta1_power = st[0];
  *beta2_power = st[1];
  return DSSM_OK;
}

// The captured graph's shape, kept per graph for dssm_plan_graph_topology: {nodes, edges, roots,
// kernel nodes, memcpy nodes, memset nodes, other nodes, chain}.  chain = 1 when the graph is ONE
// path through every node (nodes == edges + 1, in- and out-degree <= 1, one root): then every node,
// whatever its type, runs after every node captured before it on the stream.
static void graph_topology(hipGraph_t graph, int64_t* out) {
  for (int i = 0; i < 8; ++i) out[i] = -1;
  size_t nn = 0, ne = 0;
  if (hipGraphGetNodes(graph, nullptr, &nn) != hipSuccess || hipGraphGetEdges(graph, nullptr, nullptr, &ne) != hipSuccess)
    return;
  std::vector<hipGraphNode_t> nodes(nn), from(ne), to(ne);
  if ((nn && hipGraphGetNodes(graph, nodes.data(), &nn) != hipSuccess) ||
      (ne && hipGraphGetEdges(graph, from.data(), to.data(), &ne) != hipSuccess))
    return;
  int64_t kern = 0, cpy = 0, set = 0, other = 0;
  for (hipGraphNode_t n : nodes) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(n, &t) != hipSuccess) return;
    if (t == hipGraphNodeTypeKernel) ++kern;
    else if (t == hipGraphNodeTypeMemcpy) ++cpy;
    else if (t == hipGraphNodeTypeMemset) ++set;
    else ++other;
  }
  std::vector<int> indeg(nn, 0), outdeg(nn, 0);
  auto idx = [&](hipGraphNode_t n) {
    return (int)(std::find(nodes.begin(), nodes.end(), n) - nodes.begin());
  };
  for (size_t i = 0; i < ne; ++i) {
    const int a = idx(from[i]), b = idx(to[i]);
    if (a >= (int)nn || b >= (int)nn) return;
    ++outdeg[a];
    ++indeg[b];
  }
  int64_t roots = 0;
  bool chain = nn == ne + 1;
  for (size_t i = 0; i < nn; ++i) {
    roots += indeg[i] == 0;
    chain = chain && indeg[i] <= 1 && outdeg[i] <= 1;
  }
  chain = chain && roots == 1;
  const int64_t v[8] = {(int64_t)nn, (int64_t)ne, roots, kern, cpy, set, other, chain ? 1 : 0};
  for (int i = 0; i < 8; ++i) out[i] = v[i];
}

int dssm_plan_graph_topology(const dssm_plan* P, int graph_id, int64_t* out) {
  if (!P || !out || graph_id < 0 || graph_id >= (int)P->graphs.size())
    return fail(DSSM_E_INVALID, "dssm_plan_graph_topology: bad plan / graph id / output");
  for (int i = 0; i < 8; ++i) out[i] = P->graphs[graph_id]->topo[i];
  return DSSM_OK;
}

int dssm_plan_graph_build(dssm_plan* P, int parts, float grad_scale, int with_probes, void* stream,
                          int* graph_id) {
  if (!P || !graph_id) return fail(DSSM_E_INVALID, "null argument");
  if (!stream) return fail(DSSM_E_INVALID, "graph capture needs a non-default stream");
  const int all = DSSM_GRAPH_FWD_BWD | DSSM_GRAPH_ADAM | DSSM_GRAPH_SHADOWS | DSSM_GRAPH_WIRE_SHADOWS;
  if (!(parts & all) || (parts & ~all))
    return fail(DSSM_E_INVALID, "graph parts: DSSM_GRAPH_FWD_BWD | DSSM_GRAPH_ADAM | DSSM_GRAPH_SHADOWS"
                                " | DSSM_GRAPH_WIRE_SHADOWS");
  if (P->capturing) return fail(DSSM_E_INVALID, "already capturing");
  if (P->fused_w1_adam() && parts != (DSSM_GRAPH_FWD_BWD | DSSM_GRAPH_ADAM))
    return fail(DSSM_E_INVALID, "with the fused W1 Adam a graph must hold the whole step");
  hipStream_t s = (hipStream_t)stream;
  auto* g = new dssm_plan::GraphSlot();
  g->probes = with_probes != 0;
  if (g->probes)
    for (auto& pr : g->ev)
      for (hipEvent_t& e : pr)
        if (hipEventCreate(&e) != hipSuccess) {
          delete g;
          return fail(DSSM_E_HIP, "hipEventCreate failed");
        }
  const bool was_clean = P->grads_clean, was_fwd = P->fwd_train_done;
  // A replayed step starts from the state a previous step leaves: clean gradients.
  if (parts & DSSM_GRAPH_FWD_BWD) P->grads_clean = true;
  hipError_t e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    delete g;
    return fail(DSSM_E_HIP, std::string("hipStreamBeginCapture: ") + hipGetErrorString(e));
  }
  P->capturing = g;
  int rc = DSSM_OK;
  // a shadow part with FWD_BWD and no ADAM: the previous step's shadow refresh, then this step's
  // forward + backward (data parallel: one graph boundary fewer per step, the refresh and the next
  // forward have no collective between them)
  const bool shadows_first = (parts & DSSM_GRAPH_FWD_BWD) && !(parts & DSSM_GRAPH_ADAM) &&
                             (parts & (DSSM_GRAPH_SHADOWS | DSSM_GRAPH_WIRE_SHADOWS));
  auto shadow_parts = [&]() {
    if (!rc && (parts & DSSM_GRAPH_SHADOWS)) rc = dssm_plan_sync_shadows(P, stream);
    if (!rc && (parts & DSSM_GRAPH_WIRE_SHADOWS)) rc = dssm_plan_wire_shadows(P, stream);
  };
  if (shadows_first) shadow_parts();
  if (!rc && (parts & DSSM_GRAPH_FWD_BWD)) {
    rc = dssm_plan_forward(P, 1, stream);
    if (!rc) rc = dssm_plan_backward(P, stream);
  }
  if (!rc && (parts & DSSM_GRAPH_ADAM)) rc = dssm_plan_adam(P, grad_scale, stream);
  if (!shadows_first) shadow_parts();
  P->capturing = nullptr;
  std::string err = rc ? g_err : std::string();
  hipGraph_t graph = nullptr;
  e = hipStreamEndCapture(s, &graph);
  // capture only recorded work: restore the host-side step state it advanced
  P->grads_clean = (parts & DSSM_GRAPH_ADAM) ? true : (parts & DSSM_GRAPH_FWD_BWD ? false : was_clean);
  P->fwd_train_done = (parts & DSSM_GRAPH_FWD_BWD) ? true : was_fwd;
  if (rc || e != hipSuccess || !graph) {
    if (graph) hipGraphDestroy(graph);
    delete g;
    return fail(rc ? rc : DSSM_E_HIP, rc ? err : std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
  }
  graph_topology(graph, g->topo);
  e = hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0);
  hipGraphDestroy(graph);
  if (e != hipSuccess) {
    delete g;
    return fail(DSSM_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
  }
#if DSSM_GRAPH_UPLOAD
  // upload the executable graph now (without running it), so its first launch pays no upload
  (void)hipGraphUpload(g->exec, s);
#endif
  P->graphs.push_back(g);
  *graph_id = (int)P->graphs.size() - 1;
  return DSSM_OK;
}

int dssm_plan_graph_build_steps(dssm_plan* P, const int32_t* const* indptrs,
                                const int32_t* const* indices, const float* const* values,
                                int nsteps, int with_probes, void* stream, int* graph_id) {
  if (!P || !graph_id || !indptrs || !indices || !values || nsteps < 1)
    return fail(DSSM_E_INVALID, "null argument or nsteps < 1");
  if (!stream) return fail(DSSM_E_INVALID, "graph capture needs a non-default stream");
  if (P->capturing) return fail(DSSM_E_INVALID, "already capturing");
  for (int i = 0; i < nsteps; ++i)
    if (!indptrs[i] || (P->Lt.max_nnz && (!indices[i] || !values[i])))
      return fail(DSSM_E_INVALID, "null batch pointer");
  hipStream_t s = (hipStream_t)stream;
  auto* g = new dssm_plan::GraphSlot();
  g->probes = with_probes != 0;
  if (g->probes)
    for (auto& pr : g->ev)
      for (hipEvent_t& e : pr)
        if (hipEventCreate(&e) != hipSuccess) {
          delete g;
          return fail(DSSM_E_HIP, "hipEventCreate failed");
        }
  const int32_t* keep_ip = P->indptr;
  const int32_t* keep_ix = P->indices;
  const float* keep_v = P->values;
  const bool was_fwd = P->fwd_train_done;
  P->grads_clean = true;  // a replay starts from the state a completed step leaves
  hipError_t e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    delete g;
    return fail(DSSM_E_HIP, std::string("hipStreamBeginCapture: ") + hipGetErrorString(e));
  }
  P->capturing = g;
  int rc = DSSM_OK;
  P->rank_done_for = nullptr;
  for (int i = 0; i < nsteps && !rc; ++i) {
    // probes (event-record nodes): the transpose / SpMM / dW1 ones in the first step (the only one
    // with its own rank launch when the rank pass rides in Adam), the Adam one in the last step (the
    // only Adam launch hosting no rank pass: it times the optimizer alone)
    // (with_probes == 2: the Adam probe alone)
    g->probes = with_probes != 0 && ((i == 0 && with_probes != 2) || i == nsteps - 1);
    g->probe_mask = (i == 0 && with_probes != 2 ? ~(1u << DSSM_PROBE_ADAM) : 0u) |
                    (i == nsteps - 1 ? 1u << DSSM_PROBE_ADAM : 0u);
    P->indptr = indptrs[i];
    P->indices = indices[i];
    P->values = values[i];
    rc = dssm_plan_forward(P, 1, stream);
    if (!rc) rc = dssm_plan_backward(P, stream);
    if (!rc && i + 1 < nsteps && P->opt[DSSM_OPT_RANK_IN_ADAM]) {  // step i+1's rank pass rides in this Adam
      P->host_rank_indptr = indptrs[i + 1];
      P->host_rank_indices = indices[i + 1];
    }
    if (!rc) rc = dssm_plan_adam(P, 1.0f, stream);
  }
  P->host_rank_indptr = P->host_rank_indices = nullptr;
  P->rank_done_for = nullptr;
  g->probes = with_probes != 0;
  g->probe_mask = ~0u;
  P->capturing = nullptr;
  std::string err = rc ? g_err : std::string();
  hipGraph_t graph = nullptr;
  e = hipStreamEndCapture(s, &graph);
  P->indptr = keep_ip;
  P->indices = keep_ix;
  P->values = keep_v;
  P->grads_clean = true;
  P->fwd_train_done = was_fwd;
  if (rc || e != hipSuccess || !graph) {
    if (graph) hipGraphDestroy(graph);
    delete g;
    return fail(rc ? rc : DSSM_E_HIP, rc ? err : std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
  }
  graph_topology(graph, g->topo);
  e = hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0);
  hipGraphDestroy(graph);
  if (e != hipSuccess) {
    delete g;
    return fail(DSSM_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
  }
#if DSSM_GRAPH_UPLOAD
  // upload the executable graph now (without running it), so its first launch pays no upload
  (void)hipGraphUpload(g->exec, s);
#endif
  P->graphs.push_back(g);
  *graph_id = (int)P->graphs.size() - 1;
  return DSSM_OK;
}

int dssm_plan_graph_launch(dssm_plan* P, int graph_id, void* stream) {
  if (!P || graph_id < 0 || graph_id >= (int)P->graphs.size())
    return fail(DSSM_E_INVALID, "bad graph id");
  HIP_TRY(hipGraphLaunch(P->graphs[graph_id]->exec, (hipStream_t)stream));
  return DSSM_OK;
}

int dssm_plan_graph_probe_read(dssm_plan* P, int graph_id, int probe_id, float* ms) {
  if (!P || !ms || graph_id < 0 || graph_id >= (int)P->graphs.size() || probe_id < 0 ||
      probe_id >= DSSM_PROBE_COUNT)
    return fail(DSSM_E_INVALID, "bad argument");
  auto* g = P->graphs[graph_id];
  if (!g->probes) return fail(DSSM_E_INVALID, "graph built without probes");
  HIP_TRY(hipEventSynchronize(g->ev[probe_id][1]));
  HIP_TRY(hipEventElapsedTime(ms, g->ev[probe_id][0], g->ev[probe_id][1]));
  return DSSM_OK;
}

// ---- functional entry points ------------------------------------------------------------
int dssm_spmm_csr_fwd_act(const int32_t* indptr, const int32_t* indices, const float* values, int rows,
                          const void* W, int w_dtype, int ldw, int n, const float* bias, float* Z,
                          int ldz, int act, void* stream) {
  if (!indptr || !W || !bias || !Z || rows < 0 || n < 4 || (n % 4) || ldz < n || (ldz % 8) ||
      ldw < n || (ldw % 4) || (act != DSSM_ACT_NONE && act != DSSM_ACT_RELU))
    return fail(DSSM_E_INVALID, "dssm_spmm_csr_fwd: bad arguments (n%4==0, ldz%8==0, ldw>=n)");
  if (w_dtype == DSSM_BF16 && ldw < ldp8(n))
    return fail(DSSM_E_INVALID, "bf16 W needs ldw >= round_up(n, 8) with zero pads");
  HIP_TRY(dssm::launch_spmm_fwd(indptr, indices, values, rows, W, w_dtype == DSSM_BF16, ldw, n,
                                bias, Z, ldz, (hipStream_t)stream, nullptr, act == DSSM_ACT_RELU));
  return DSSM_OK;
}

int dssm_spmm_csr_fwd_ex(const int32_t* indptr, const int32_t* indices, const float* values, int rows,
                         const void* W, int w_dtype, int ldw, int n, const float* bias, void* Z, int z_dtype,
                         int ldz, int act, void* stream) {
  if (z_dtype == DSSM_F32)
    return dssm_spmm_csr_fwd_act(indptr, indices, values, rows, W, w_dtype, ldw, n, bias, static_cast<float*>(Z),
                                 ldz, act, stream);
  if (!indptr || !W || !bias || !Z || rows < 0 || n < 4 || (n % 4) || ldz < n || (ldz % 8) ||
      z_dtype != DSSM_BF16 || w_dtype != DSSM_BF16 || ldw < ldp8(n) || (ldw % 8) ||
      (act != DSSM_ACT_NONE && act != DSSM_ACT_RELU))
    return fail(DSSM_E_INVALID, "dssm_spmm_csr_fwd_ex: a bf16 output needs bf16 W (ldw >= round_up(n, 8), zero "
                                "pads) and ldz % 8 == 0");
  HIP_TRY(dssm::launch_spmm_fwd(indptr, indices, values, rows, W, true, ldw, n, bias, static_cast<float*>(Z), ldz,
                                (hipStream_t)stream, nullptr, act == DSSM_ACT_RELU, true));
  return DSSM_OK;
}

int dssm_spmm_csr_fwd(const int32_t* indptr, const int32_t* indices, const float* values, int rows,
                      const void* W, int w_dtype, int ldw, int n, const float* bias, float* Z,
                      int ldz, void* stream) {
  return dssm_spmm_csr_fwd_act(indptr, indices, values, rows, W, w_dtype, ldw, n, bias, Z, ldz,
                               DSSM_ACT_NONE, stream);
}

int dssm_dense_fwd_act(const void* A, int lda, const void* W, int ldw, int dtype, int M, int K, int N,
                       const float* bias, float* Z, int ldz, int act, void* stream) {
  if (!A || !W || !bias || !Z || M < 0 || K < 1 || N < 1 || lda < K || ldw < N || ldz < N ||
      (lda % 8) || (ldw % 4) || (ldz % 4) || (dtype == DSSM_BF16 && (ldw % 8)) ||
      (act != DSSM_ACT_NONE && act != DSSM_ACT_RELU))
    return fail(DSSM_E_INVALID, "dssm_dense_fwd: bad arguments");
  HIP_TRY(dssm::launch_gemm(dssm::GEMM_FWD, dtype == DSSM_BF16, M, N, K, A, lda, W, ldw, Z, ldz,
                            bias, false, nullptr, (hipStream_t)stream, nullptr,
                            act == DSSM_ACT_RELU ? 1 : 0));
  return DSSM_OK;
}

int dssm_dense_fwd(const void* A, int lda, const void* W, int ldw, int dtype, int M, int K, int N,
                   const float* bias, float* Z, int ldz, void* stream) {
  return dssm_dense_fwd_act(A, lda, W, ldw, dtype, M, K, N, bias, Z, ldz, DSSM_ACT_NONE, stream);
}

size_t dssm_bn_ws_bytes(int rows, int ldz) {
  return align256(dssm::bn_partial_floats(rows, ldz, rows) * 4) + align256(4 * 2 * (size_t)ldz * 4) +
         align256(dssm::bn_ticket_count(ldz) * 4);
}

int dssm_bn_relu_fwd(const float* Z, int ldz, int rows, int n, const float* gamma, const float* beta,
                     float* ema_mean, float* ema_var, float eps, float decay, int train, int relu,
                     void* out, int out_dtype, float* batch_mean, float* batch_var, void* ws,
                     void* stream) {
  if (!Z || !gamma || !beta || !ema_mean || !ema_var || !out || !ws || rows < 1 || n < 4 ||
      (n % 4) || ldz != ldp8(n))
    return fail(DSSM_E_INVALID, "dssm_bn_relu_fwd: bad arguments (ldz must be round_up(n,8))");
  hipStream_t s = (hipStream_t)stream;
  const dssm::BnTowers tw{rows, rows};
  // ws: [partials | coef | tickets]; the tickets must be zero on first use (caller zeroes ws
  // once) and are re-armed by the kernel.
  char* w = static_cast<char*>(ws);
  float* part = reinterpret_cast<float*>(w);
  const size_t o1 = align256(dssm::bn_partial_floats(rows, ldz, rows) * 4);
  float* coef = reinterpret_cast<float*>(w + o1);
  unsigned* tickets = reinterpret_cast<unsigned*>(w + o1 + align256(4 * 2 * (size_t)ldz * 4));
  HIP_TRY(dssm::launch_bn_fwd_stats(Z, ldz, n, tw, gamma, beta, gamma, beta, ema_mean, ema_var,
                                    ema_mean, ema_var, eps, decay, train != 0, batch_mean,
                                    batch_var, part, tickets, coef, s));
  HIP_TRY(dssm::launch_bn_apply(Z, ldz, n, tw, coef, relu != 0, out, out_dtype == DSSM_BF16, s));
  return DSSM_OK;
}

// (round 4: the last workgroup summing the functional cosine's loss partials in-kernel, behind a
// ticket, measured slower on the multi-view step -- 0.2554-0.2591 against 0.2424 ms/step -- and
// neutral on the RNN step; removed: the finalize is a separate one-wave launch)
int dssm_cosine_softmax_loss_mapped(const float* y, int ld, const int32_t* row_map, int n, int query_bs, int neg,
                                    float gamma, float* cos_sim_raw, float* cos_sim, float* prob,
                                    float* query_norm, float* loss, float* dy, float* ws, void* stream) {
  if (!y || !row_map || !cos_sim_raw || !cos_sim || !prob || !query_norm || !loss || !dy || !ws ||
      query_bs < 1 || neg < 1 || neg > 15 || n < 1 || n > 512 || ld < n)
    return fail(DSSM_E_INVALID, "dssm_cosine_softmax_loss_mapped: bad arguments");
  HIP_TRY(dssm::launch_cosine_loss(y, ld, n, query_bs, neg, gamma, nullptr, nullptr, cos_sim_raw,
                                   cos_sim, prob, query_norm, ws, loss, dy, (hipStream_t)stream, nullptr,
                                   false, nullptr, row_map));
  return DSSM_OK;
}

int dssm_cosine_softmax_loss(const float* y, int ld, int n, int query_bs, int neg, float gamma,
                             float* cos_sim_raw, float* cos_sim, float* prob, float* query_norm,
                             float* loss, float* dy, float* ws, void* stream) {
  if (!y || !cos_sim_raw || !cos_sim || !prob || !query_norm || !loss || !dy || !ws ||
      query_bs < 1 || neg < 1 || neg > 15 || n < 1 || n > 512 || ld < n)
    return fail(DSSM_E_INVALID, "dssm_cosine_softmax_loss: bad arguments");
  HIP_TRY(dssm::launch_cosine_loss(y, ld, n, query_bs, neg, gamma, nullptr, nullptr, cos_sim_raw,
                                   cos_sim, prob, query_norm, ws, loss, dy, (hipStream_t)stream, nullptr,
                                   false, nullptr, nullptr));
  return DSSM_OK;
}

int dssm_cosine_softmax_loss_dropout(const float* x, int ld, int n, int query_bs, int neg, float gamma, float keep,
                                     uint32_t seed, uint32_t step, float bwd_scale, float* y, float* cos_sim_raw,
                                     float* cos_sim, float* prob, float* query_norm, float* loss, float* dy,
                                     float* ws, void* stream) {
  if (!x || !cos_sim_raw || !cos_sim || !prob || !query_norm || !loss || !dy || !ws || query_bs < 1 || neg < 1 ||
      neg > 15 || n < 1 || n > 512 || ld < n || !(keep > 0.f) || (int64_t)query_bs * (2 + neg) * n >= (1ll << 31))
    return fail(DSSM_E_INVALID, "dssm_cosine_softmax_loss_dropout: bad arguments");
  // dssm_rnn_dropout's mask and arithmetic: thr = keep * 2^32, x * (1 / keep), dy * (scale / keep)
  const double t = (double)keep * 4294967296.0;
  dssm::CosDrop d{};
  d.on = 1;
  d.all = keep >= 1.f ? 1 : 0;
  d.thr = t >= 4294967295.0 ? 0xFFFFFFFFu : (unsigned)t;
  d.seed = seed;
  d.step = step;
  d.cols = n;
  const float kd = keep >= 1.f ? 1.f : keep;
  d.fwd = 1.0f / kd;
  d.bwd = bwd_scale / kd;
  HIP_TRY(dssm::launch_cosine_loss(x, ld, n, query_bs, neg, gamma, nullptr, y, cos_sim_raw, cos_sim, prob,
                                   query_norm, ws, loss, dy, (hipStream_t)stream, nullptr, false, nullptr, nullptr,
                                   &d));
  return DSSM_OK;
}

// ---- RCCL ---------------------------------------------------------------------------------
// The library's own communicator (one per process: one process per GPU).  Collectives are
// enqueued on the caller's stream, between the step's graphs.
static ncclComm_t g_comm = nullptr;
static int g_rank = 0, g_world = 0;

static bool nccl_type(int dtype, ncclDataType_t* t, size_t* es) {
  if (dtype == DSSM_F32) { *t = ncclFloat32; *es = 4; return true; }
  if (dtype == DSSM_BF16) { *t = ncclBfloat16; *es = 2; return true; }
  if (dtype == DSSM_I32) { *t = ncclInt32; *es = 4; return true; }
  return false;
}

#define RCCL_TRY(expr)                                                                    \
  do {                                                                                  \
    ncclResult_t r_ = (expr);                                                           \
    if (r_ != ncclSuccess) return fail(DSSM_E_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

int dssm_comm_unique_id(void* out128) {
  if (!out128) return fail(DSSM_E_INVALID, "null id buffer");
  ncclUniqueId id;
  RCCL_TRY(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(out128, &id, 128);
  return DSSM_OK;
}

int dssm_comm_init(int rank, int world, const void* unique_id128) {
  if (!unique_id128 || world < 1 || rank < 0 || rank >= world)
    return fail(DSSM_E_INVALID, "dssm_comm_init: bad arguments");
  if (g_comm) return fail(DSSM_E_INVALID, "communicator already initialised");
  ncclUniqueId id;
  std::memcpy(&id, unique_id128, 128);
  ncclResult_t r = ncclCommInitRank(&g_comm, world, id, rank);
  if (r != ncclSuccess) {
    g_comm = nullptr;
    return fail(DSSM_E_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  g_rank = rank;
  g_world = world;
  return DSSM_OK;
}

int dssm_comm_world(void) { return g_comm ? g_world : 0; }

int dssm_comm_info(int* rccl_world, int* rccl_rank, int* rccl_version) {
  if (!rccl_world || !rccl_rank || !rccl_version) return fail(DSSM_E_INVALID, "null argument");
  *rccl_world = *rccl_rank = -1;
  RCCL_TRY(ncclGetVersion(rccl_version));
  if (g_comm) {
    RCCL_TRY(ncclCommCount(g_comm, rccl_world));
    RCCL_TRY(ncclCommUserRank(g_comm, rccl_rank));
  }
  return DSSM_OK;
}

int dssm_allreduce_sum(void* buf, int64_t count, int dtype, void* stream) {
  if (!g_comm) return fail(DSSM_E_INVALID, "communicator not initialised");
  ncclDataType_t t;
  size_t es;
  if (!buf || count < 0 || !nccl_type(dtype, &t, &es)) return fail(DSSM_E_INVALID, "dssm_allreduce_sum: bad arguments");
  RCCL_TRY(ncclAllReduce(buf, buf, (size_t)count, t, ncclSum, g_comm, (hipStream_t)stream));
  return DSSM_OK;
}

int dssm_allreduce_sum_f32(float* buf, int64_t count, void* stream) {
  return dssm_allreduce_sum(buf, count, DSSM_F32, stream);
}

int dssm_reduce_scatter_sum(const void* send, void* recv, int64_t count, int dtype, void* stream) {
  if (!g_comm) return fail(DSSM_E_INVALID, "communicator not initialised");
  ncclDataType_t t;
  size_t es;
  if (!send || !recv || count < 0 || !nccl_type(dtype, &t, &es))
    return fail(DSSM_E_INVALID, "dssm_reduce_scatter_sum: bad arguments");
  RCCL_TRY(ncclReduceScatter(send, recv, (size_t)count, t, ncclSum, g_comm, (hipStream_t)stream));
  return DSSM_OK;
}

int dssm_all_gather(const void* send, void* recv, int64_t count, int dtype, void* stream) {
  if (!g_comm) return fail(DSSM_E_INVALID, "communicator not initialised");
  ncclDataType_t t;
  size_t es;
  if (!send || !recv || count < 0 || !nccl_type(dtype, &t, &es))
    return fail(DSSM_E_INVALID, "dssm_all_gather: bad arguments");
  RCCL_TRY(ncclAllGather(send, recv, (size_t)count, t, g_comm, (hipStream_t)stream));
  return DSSM_OK;
}

// all-to-all as the rank's own chunk by a device copy plus one grouped send / recv per peer (all
// xGMI links busy at once on a fully connected node: one step, not world - 1 ring steps).  (RCCL's
// ncclAllToAll crashed in hipGraph capture at world 1 on this image; the grouped form captures.)
// A device copy on the stream: a copy kernel, or (plan option MEMCPY_NODES, diagnostics: the round-3
// form) a hipMemcpyAsync, which a capture records as a memcpy node.
static hipError_t device_copy(void* dst, const void* src, size_t bytes, hipStream_t s, bool memcpy_node) {
  if (memcpy_node) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s);
  return dssm::launch_copy_bytes(dst, src, bytes, s);
}

static int all_to_all_impl(const void* send, void* recv, int64_t count, ncclDataType_t t, size_t es,
                           hipStream_t s, bool memcpy_node = false, float* tail = nullptr, size_t tail_n = 0) {
  const char* sp = static_cast<const char*>(send);
  char* rp = static_cast<char*>(recv);
  const size_t chunk = (size_t)count * es;
  HIP_TRY(device_copy(rp + (size_t)g_rank * chunk, sp + (size_t)g_rank * chunk, chunk, s, memcpy_node));
  if (g_world == 1 && !tail) return DSSM_OK;
  RCCL_TRY(ncclGroupStart());
  for (int j = 0; j < g_world; ++j) {
    if (j == g_rank) continue;
    ncclResult_t r = ncclSend(sp + (size_t)j * chunk, (size_t)count, t, j, g_comm, s);
    if (r == ncclSuccess) r = ncclRecv(rp + (size_t)j * chunk, (size_t)count, t, j, g_comm, s);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return fail(DSSM_E_RCCL, std::string("ncclSend/ncclRecv: ") + ncclGetErrorString(r));
    }
  }
  if (tail && tail_n) {  // the fp32 tail's sum in the same group (plan option TAIL_IN_A2A)
    ncclResult_t r = ncclAllReduce(tail, tail, tail_n, ncclFloat32, ncclSum, g_comm, s);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return fail(DSSM_E_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    }
  }
  RCCL_TRY(ncclGroupEnd());
  return DSSM_OK;
}

int dssm_all_to_all(const void* send, void* recv, int64_t count, int dtype, void* stream) {
  if (!g_comm) return fail(DSSM_E_INVALID, "communicator not initialised");
  ncclDataType_t t;
  size_t es;
  if (!send || !recv || count < 0 || !nccl_type(dtype, &t, &es) || send == recv)
    return fail(DSSM_E_INVALID, "dssm_all_to_all: bad arguments (distinct send / recv)");
  return all_to_all_impl(send, recv, count, t, es, (hipStream_t)stream);
}

int dssm_all_to_all_tail(const void* send, void* recv, int64_t count, int dtype, float* tail, int64_t tail_count,
                         void* stream) {
  if (!g_comm) return fail(DSSM_E_INVALID, "communicator not initialised");
  ncclDataType_t t;
  size_t es;
  if (!send || !recv || count < 0 || !nccl_type(dtype, &t, &es) || send == recv || !tail || tail_count <= 0)
    return fail(DSSM_E_INVALID, "dssm_all_to_all_tail: bad arguments (distinct send / recv, a tail)");
  return all_to_all_impl(send, recv, count, t, es, (hipStream_t)stream, false, tail, (size_t)tail_count);
}

// Variable-count all-to-all of the touched-row sparse exchange, with the replicated tail's sum in the
// same RCCL group (one launch of the group for both).  The rank's own part is a device copy.
int dssm_all_to_allv(const void* send, const int64_t* send_counts, void* recv, const int64_t* recv_counts,
                     int dtype, void* tail, int64_t tail_count, int tail_dtype, void* stream) {
  if (!g_comm) return fail(DSSM_E_INVALID, "communicator not initialised");
  ncclDataType_t t, tt = ncclFloat32;
  size_t es, tes = 4;
  if (!send_counts || !recv_counts || !nccl_type(dtype, &t, &es) || send == recv ||
      (tail && (tail_count < 0 || !nccl_type(tail_dtype, &tt, &tes))))
    return fail(DSSM_E_INVALID, "dssm_all_to_allv: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const char* sp = static_cast<const char*>(send);
  char* rp = static_cast<char*>(recv);
  int64_t so = 0, ro = 0;
  std::vector<int64_t> soff(g_world), roff(g_world);
  for (int j = 0; j < g_world; ++j) {
    if (send_counts[j] < 0 || recv_counts[j] < 0) return fail(DSSM_E_INVALID, "dssm_all_to_allv: negative count");
    soff[j] = so;
    roff[j] = ro;
    so += send_counts[j];
    ro += recv_counts[j];
  }
  if (send_counts[g_rank] != recv_counts[g_rank]) return fail(DSSM_E_INVALID, "dssm_all_to_allv: own counts differ");
  if (send_counts[g_rank])
    HIP_TRY(device_copy(rp + (size_t)roff[g_rank] * es, sp + (size_t)soff[g_rank] * es,
                        (size_t)send_counts[g_rank] * es, s, false));
  RCCL_TRY(ncclGroupStart());
  for (int j = 0; j < g_world; ++j) {
    if (j == g_rank) continue;
    ncclResult_t r = ncclSuccess;
    if (send_counts[j]) r = ncclSend(sp + (size_t)soff[j] * es, (size_t)send_counts[j], t, j, g_comm, s);
    if (r == ncclSuccess && recv_counts[j]) r = ncclRecv(rp + (size_t)roff[j] * es, (size_t)recv_counts[j], t, j, g_comm, s);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return fail(DSSM_E_RCCL, std::string("ncclSend/ncclRecv: ") + ncclGetErrorString(r));
    }
  }
  if (tail && tail_count) {
    ncclResult_t r = ncclAllReduce(tail, tail, (size_t)tail_count, tt, ncclSum, g_comm, s);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return fail(DSSM_E_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    }
  }
  RCCL_TRY(ncclGroupEnd());
  return DSSM_OK;
}

// ---- the data-parallel step graph (include/dssm.h dssm_plan_graph_build_dp_steps) -----------
// One collective of the exchange on the step's stream cs: the library's RCCL communicator (comm 0),
// a device copy of the same bytes (comm 1) or a kernel holding cs for the modelled link time (2).
struct DpComm {
  int mode;
  double gbps, latency_ns;
};
static int dp_collective(dssm_plan* P, const DpComm& k, int kind, int chunk, hipStream_t cs) {
  const int64_t sub = P->sub_elems();
  const int W = P->geo.ww;
  const int64_t blk = (int64_t)W * sub;  // chunk's elements in each wire
  const size_t tail = (size_t)(P->Lt.total - P->wire_end());
  float* tg = P->g + P->wire_end();
  // TAIL_IN_A2A: the last chunk's all-to-all carries the tail's all-reduce in its RCCL group
  const bool with_tail = kind == 0 && chunk == P->geo.wp - 1 && P->on(DSSM_OPT_TAIL_IN_A2A);
  // bytes this rank sends: all-to-all / all-gather (W-1) * sub bf16; all-reduce (ring) 2(W-1)/W fp32
  const double tail_bytes = 2.0 * (W - 1) / W * tail * 4;
  const double bytes = kind == 2 ? tail_bytes : (double)(W - 1) * sub * 2 + (with_tail ? tail_bytes : 0.0);
  if (k.mode == 2) {  // one fixed cost per launched group
    HIP_TRY(dssm::launch_spin(k.latency_ns + bytes / k.gbps, cs));
    return DSSM_OK;
  }
  if (k.mode == 3) {  // peer stores: the all-to-all happened inside the gradient pass (peer.hip)
    const dssm::PeerArgs a = peer_args(P);
    if (kind == 0) HIP_TRY(dssm::launch_peer_before_adam(a, cs));
    if (kind == 1) HIP_TRY(dssm::launch_peer_after_adam(a, cs));
    return DSSM_OK;  // kind 2: the tail rode in the push
  }
  uint16_t* gw = P->gwire + chunk * blk;
  uint16_t* st = const_cast<uint16_t*>(P->gstage) + chunk * blk;
  uint16_t* pw = P->pwire + chunk * blk;
  const bool mc = P->on(DSSM_OPT_MEMCPY_NODES);
  if (k.mode == 1) {  // same bytes through HBM (the tail's copy is skipped: 0.5 MB)
    if (kind == 0) HIP_TRY(device_copy(st, gw, blk * 2, cs, mc));
    if (kind == 1) HIP_TRY(device_copy(st, pw, blk * 2, cs, mc));
    return DSSM_OK;
  }
  if (kind == 0) return all_to_all_impl(gw, st, sub, ncclBfloat16, 2, cs, mc, with_tail ? tg : nullptr, tail);
  if (kind == 1) RCCL_TRY(ncclAllGather(pw + (int64_t)P->dp_rank * sub, pw, (size_t)sub, ncclBfloat16, g_comm, cs));
  if (kind == 2) RCCL_TRY(ncclAllReduce(tg, tg, tail, ncclFloat32, ncclSum, g_comm, cs));
  return DSSM_OK;
}

int dssm_plan_graph_build_dp_steps(dssm_plan* P, const int32_t* const* indptrs, const int32_t* const* indices,
                                   const float* const* values, int nsteps, float grad_scale, int comm,
                                   float link_gbps, float latency_us, int overlap, int with_probes,
                                   void* stream, int* graph_id) {
  if (!P || !graph_id || !indptrs || !indices || !values || nsteps < 1)
    return fail(DSSM_E_INVALID, "null argument or nsteps < 1");
  if (!stream) return fail(DSSM_E_INVALID, "graph capture needs a non-default stream");
  if (P->capturing) return fail(DSSM_E_INVALID, "already capturing");
  if (!P->pwire || !wire_gradient_pass(P))
    return fail(DSSM_E_INVALID, "the data-parallel graph needs the bf16 wire (dssm_plan_set_dp_wire) and the "
                                "wire gradient pass (HEAVY_IN_ADAM, WIRE_GRAD_PASS)");
  if (overlap)
    return fail(DSSM_E_INVALID, "overlap: removed (the two-stream variant measured slower than the one-stream "
                                "graph and its captured RCCL steps raced at world 1; DESIGN 6)");
  if (comm < 0 || comm > 3 || (comm == 2 && !(link_gbps > 0.f)))
    return fail(DSSM_E_INVALID, "comm: 0 RCCL, 1 device copies, 2 modelled (link_gbps > 0), 3 peer stores");
  if ((comm == 3) != P->peer_on())
    return fail(DSSM_E_INVALID, "comm 3 (peer stores) if and only if dssm_plan_set_dp_peers is set");
  if (comm == 0 && (!g_comm || g_world != P->geo.ww || g_rank != P->dp_rank))
    return fail(DSSM_E_INVALID, "comm 0 needs dssm_comm_init with the wire's world and rank");
  if (comm == 0 && P->geo.ww > 1 && P->gstage == P->gwire)
    return fail(DSSM_E_INVALID, "the all-to-all needs a stage distinct from grad_wire");
  for (int i = 0; i < nsteps; ++i)
    if (!indptrs[i] || (P->Lt.max_nnz && (!indices[i] || !values[i])))
      return fail(DSSM_E_INVALID, "null batch pointer");
  hipStream_t s = (hipStream_t)stream;
  const DpComm k{comm, (double)link_gbps, 1e3 * (double)latency_us};
  const int C = P->geo.wp;
  auto* g = new dssm_plan::GraphSlot();
  g->probes = with_probes != 0;
  if (g->probes)
    for (auto& pr : g->ev)
      for (hipEvent_t& e : pr) (void)hipEventCreate(&e);
  const int32_t* keep_ip = P->indptr;
  const int32_t* keep_ix = P->indices;
  const float* keep_v = P->values;
  const bool was_fwd = P->fwd_train_done;
  P->grads_clean = true;
  hipError_t e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    delete g;
    return fail(DSSM_E_HIP, std::string("hipStreamBeginCapture: ") + hipGetErrorString(e));
  }
  P->capturing = g;
  P->dp_defer_gradpass = true;
  P->rank_done_for = nullptr;
  int rc = DSSM_OK;
  // every node on the one captured stream, in dependency order (graph_topology checks the chain)
  // probes (event-record nodes, the last step only): its phases (DSSM_PROBE_DP_*) and Adam shard
  unsigned dp_mask = 1u << DSSM_PROBE_ADAM;
  for (int id = DSSM_PROBE_DP_FWD_BWD; id <= DSSM_PROBE_DP_SHADOW; ++id) dp_mask |= 1u << id;
  for (int i = 0; i < nsteps && !rc; ++i) {
    g->probes = with_probes != 0 && i == nsteps - 1;
    g->probe_mask = dp_mask;
    P->indptr = indptrs[i];
    P->indices = indices[i];
    P->values = values[i];
    P->probe_begin(DSSM_PROBE_DP_FWD_BWD, s);
    rc = dssm_plan_forward(P, 1, stream);
    if (!rc) rc = dssm_plan_backward(P, stream);
    P->probe_end(DSSM_PROBE_DP_FWD_BWD, s);
    // the gradient pass chunk by chunk, each chunk's all-to-all behind it (probes: chunk 0's)
    for (int c = 0; c < C && !rc; ++c) {
      if (c == 0) P->probe_begin(DSSM_PROBE_DP_GRAD_PASS, s);
      rc = launch_wire_gradient_pass(P, s, C > 1 ? c : -1);
      if (c == 0) P->probe_end(DSSM_PROBE_DP_GRAD_PASS, s);
      if (c == 0) P->probe_begin(DSSM_PROBE_DP_ALL_TO_ALL, s);
      if (!rc) rc = dp_collective(P, k, 0, c, s);
      if (c == 0) P->probe_end(DSSM_PROBE_DP_ALL_TO_ALL, s);
    }
    P->probe_begin(DSSM_PROBE_DP_TAIL, s);
    if (!rc && !P->on(DSSM_OPT_TAIL_IN_A2A) && comm != 3)  // the fp32 tail (b1's row: the last chunk's pass)
      rc = dp_collective(P, k, 2, 0, s);
    P->probe_end(DSSM_PROBE_DP_TAIL, s);
    // Adam chunk by chunk, each chunk's all-gather behind its Adam
    if (!rc && i + 1 < nsteps && P->opt[DSSM_OPT_RANK_IN_ADAM]) {
      P->host_rank_indptr = indptrs[i + 1];
      P->host_rank_indices = indices[i + 1];
    }
    P->dp_hook = [&](int c) -> int { return dp_collective(P, k, 1, c, s); };
    if (!rc) rc = dssm_plan_adam(P, grad_scale, stream);
    P->dp_hook = nullptr;
    // W1's shadow rebuilt chunk by chunk from the all-gathered wire (the next forward's operand).  With
    // one chunk the wire already holds W1 row-major: the region's next step reads it directly
    // (w1_wire, tight rows of stride n: RawRow8<u16t>) and only the last step rebuilds the shadow,
    // which the next region's first step and the eval forward read.
    // (peer stores: the shadow is rebuilt every step, behind the acquire of k_peer_shadow)
    const bool direct = C == 1 && P->geo.n == P->Lt.n[0] && i + 1 < nsteps && comm != 3;
    P->probe_begin(DSSM_PROBE_DP_SHADOW, s);
    if (!rc && comm == 3) {
      hipError_t e_ = dssm::launch_peer_shadow(P->pwire, P->shadows().seg[0], s);
      if (e_ != hipSuccess) rc = fail(DSSM_E_HIP, std::string("launch_peer_shadow: ") + hipGetErrorString(e_));
    }
    for (int c = 0; c < C && !rc && !direct && comm != 3; ++c) {
      hipError_t e_ = dssm::launch_wire_shadow(P->pwire, P->shadows().seg[0], P->geo, C > 1 ? c : -1, s);
      if (e_ != hipSuccess) rc = fail(DSSM_E_HIP, std::string("launch_wire_shadow: ") + hipGetErrorString(e_));
    }
    P->probe_end(DSSM_PROBE_DP_SHADOW, s);
    P->w1_wire = direct ? P->pwire : nullptr;
  }
  P->w1_wire = nullptr;
  P->dp_hook = nullptr;
  P->dp_defer_gradpass = false;
  P->host_rank_indptr = P->host_rank_indices = nullptr;
  P->rank_done_for = nullptr;
  g->probes = with_probes != 0;
  g->probe_mask = ~0u;
  P->capturing = nullptr;
  std::string err = rc ? g_err : std::string();
  hipGraph_t graph = nullptr;
  e = hipStreamEndCapture(s, &graph);
  P->indptr = keep_ip;
  P->indices = keep_ix;
  P->values = keep_v;
  P->grads_clean = true;
  P->fwd_train_done = was_fwd;
  if (rc || e != hipSuccess || !graph) {
    if (graph) hipGraphDestroy(graph);
    delete g;
    return fail(rc ? rc : DSSM_E_HIP, rc ? err : std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
  }
  graph_topology(graph, g->topo);
  e = hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0);
  hipGraphDestroy(graph);
  if (e != hipSuccess) {
    delete g;
    return fail(DSSM_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
  }
#if DSSM_GRAPH_UPLOAD
  (void)hipGraphUpload(g->exec, s);
#endif
  P->graphs.push_back(g);
  *graph_id = (int)P->graphs.size() - 1;
  return DSSM_OK;
}

int dssm_comm_destroy(void) {
  if (g_comm) {
    ncclCommDestroy(g_comm);
    g_comm = nullptr;
    g_world = 0;
  }
  return DSSM_OK;
}

}  // extern "C"
