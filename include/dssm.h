/*
 * dssm.h — C-ABI of libdssm.so, the MI355X (gfx950) DSSM two-tower training path.
 *
 * The reference (MC-Zealot/dssm) has no FFI: its boundary is the TF1.x graph-building
 * Python functions plus the Session feed/fetch contract.  Each entry point below names the
 * reference interface it replaces (file:line under the reference repo).  The Python host
 * mirror of that interface (dssm_amd/api.py) is the only caller; INTEGRATION.md shows the
 * ctypes binding.
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer owned by the caller unless stated otherwise; the
 *     library allocates nothing on the hot path (size the workspace with
 *     dssm_workspace_bytes()).
 *   - Every call is asynchronous on the given hipStream_t (passed as void*; NULL = default).
 *   - Return 0 on success, a negative DSSM_E* code on failure; dssm_last_error() returns a
 *     thread-local message for the last failure.  No C++ exception crosses the ABI.
 *   - A plan must not be used from two host threads at once.  Data parallelism is one process
 *     per GPU (one plan per process).
 *   - Dense activation buffers are row-major with a padded leading dimension
 *     ldp(n) = round_up(n, 8); pad columns are kept at zero.
 */
#ifndef DSSM_H
#define DSSM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSSM_ABI_VERSION 2
#define DSSM_MAX_LAYERS 8

enum { DSSM_OK = 0, DSSM_E_INVALID = -1, DSSM_E_HIP = -2, DSSM_E_RCCL = -3, DSSM_E_UNSUPPORTED = -4 };
enum { DSSM_F32 = 0, DSSM_BF16 = 1, DSSM_I32 = 2 /* collectives only */ };

/* Model/step configuration (semantic_matching/dssm/config.py:19-28 + new_dssm.py constants). */
typedef struct dssm_config {
  int abi_version;              /* must be DSSM_ABI_VERSION */
  int trigram_d;                /* TRIGRAM_D: sparse input width (new_dssm.py:44) */
  int n_layers;                 /* number of FC(+BN+ReLU) layers: 2 in new_dssm.py, 3 in the paper shape */
  int widths[DSSM_MAX_LAYERS];  /* L1_N, L2_N, ... (config.py:20-21); each a multiple of 4, <= 4096 */
  int query_bs;                 /* query_BS (config.py:19) */
  int neg;                      /* NEG (config.py:28); 1..15 */
  int max_nnz;                  /* capacity: non-zeros of one step over all BS*(2+NEG) rows */
  int compute_dtype;            /* DSSM_F32 (parity mode) or DSSM_BF16 (perf mode, fp32 master/optimizer) */
  float gamma;                  /* cosine scale, 20 (new_dssm.py:199) */
  float bn_eps;                 /* 1e-3 (new_dssm.py:87) */
  float ema_decay;              /* 0.5 (new_dssm.py:78) */
  float lr, beta1, beta2, adam_eps; /* AdamOptimizer(conf.learning_rate) TF1.x defaults (new_dssm.py:217) */
} dssm_config;

/* One trainable-variable segment of the flat parameter arena (fp32 elements). */
typedef struct dssm_segment {
  char name[32];   /* "fc1" = [W1; b1] as ((in+1) x out), "bn1_q_gamma", ... */
  int64_t offset;  /* element offset in the arena (multiple of 64) */
  int64_t rows, cols;
} dssm_segment;

typedef struct dssm_plan dssm_plan;

/* Plan-owned buffers the caller may read (fetches) — ids for dssm_plan_buffer(). */
enum {
  DSSM_BUF_LOSS = 0,        /* float[2]: loss (new_dssm.py:209), accuracy (:221) */
  DSSM_BUF_COS_SIM_RAW,     /* float[(NEG+1)*BS], index k*BS+j (new_dssm.py:197) */
  DSSM_BUF_COS_SIM,         /* float[BS*(NEG+1)], 20*cos (new_dssm.py:199) */
  DSSM_BUF_PROB,            /* float[BS*(NEG+1)] softmax (new_dssm.py:206) */
  DSSM_BUF_QUERY_NORM,      /* float[BS] query_norm_single (new_dssm.py:187) */
  DSSM_BUF_EMBED,           /* float[R*ldp(n_L)] embeddings: rows [q; pos; neg] (new_dssm.py:156-158) */
  DSSM_BUF_Z,               /* float[R*ldp(n_l)] pre-BN activations of layer `layer` */
  DSSM_BUF_BATCH_MEAN,      /* float[2*n_l]: batch mean, tower q then d (new_dssm.py:77) */
  DSSM_BUF_BATCH_VAR,       /* float[2*n_l] */
  DSSM_BUF_DZ,              /* dZ of layer `layer` (compute dtype, R*ldp) */
  DSSM_BUF_A = 11,          /* post-BN/ReLU activation of layer `layer` (R*ldp): the next product's
                               operand, bf16 in bf16 mode; fp32 embeddings for the last layer */
  DSSM_BUF_DA,              /* float[R*ldp(n_l)] d loss / d A of layer `layer` (the last: dy) */
  DSSM_BUF_COUNT
};

int dssm_abi_version(void);
const char* dssm_last_error(void);

/* ---- layout / sizing --------------------------------------------------------------------- */
int dssm_config_check(const dssm_config* cfg);
/* Elements of the flat parameter arena (== gradient, Adam m, Adam v arenas). */
int64_t dssm_param_count(const dssm_config* cfg);
/* Fills up to max_segs segments; returns the total number of segments. */
int dssm_param_layout(const dssm_config* cfg, dssm_segment* segs, int max_segs);
/* Elements of the EMA shadow arena: per layer, tower q mean|var then tower d mean|var. */
int64_t dssm_ema_count(const dssm_config* cfg);
size_t dssm_workspace_bytes(const dssm_config* cfg);

/* ---- plan: the whole training step (new_dssm.py:104-217) ------------------------------- */
int dssm_plan_create(const dssm_config* cfg, void* workspace, size_t workspace_bytes,
                     float* params, float* grads, float* adam_m, float* adam_v, float* ema,
                     dssm_plan** out);
int dssm_plan_destroy(dssm_plan* plan);
int dssm_plan_buffer(const dssm_plan* plan, int buffer_id, int layer, void** ptr, size_t* bytes);

/* Feed (utils/utils.py:45-61 + the three sparse placeholders new_dssm.py:111-114): one CSR
 * over rows [q(BS); pos(BS); neg(BS*NEG)], negative i of query j at row 2*BS + j*NEG + i.
 * nnz is read on device from indptr[rows]; it must not exceed cfg->max_nnz. */
int dssm_plan_set_batch(dssm_plan* plan, const int32_t* indptr, const int32_t* indices,
                        const float* values);
/* Refresh the bf16 weight shadows from the fp32 arena (after loading params; BF16 mode). */
int dssm_plan_sync_shadows(dssm_plan* plan, void* stream);
/* Forward through the loss (sess.run(loss)); train!=0 uses batch moments and updates the
 * EMA shadows (new_dssm.py:85 tf.cond true branch), train==0 uses the shadows. */
int dssm_plan_forward(dssm_plan* plan, int train, void* stream);
/* Backward of the last train-mode forward into the gradient arena (TF autodiff of :124-209). */
int dssm_plan_backward(dssm_plan* plan, void* stream);
/* ApplyAdam over the whole arena with TF1.x semantics, then beta*_power *= beta* (the powers
 * live on the device: dssm_plan_set/get_adam_state; they start at beta1, beta2 like TF's
 * beta1_power/beta2_power variables).  grad_scale multiplies every gradient (1/world for the
 * data-parallel mean).  Also refreshes the bf16 shadows. */
int dssm_plan_adam(dssm_plan* plan, float grad_scale, void* stream);
int dssm_plan_set_adam_state(dssm_plan* plan, float beta1_power, float beta2_power, void* stream);
int dssm_plan_get_adam_state(dssm_plan* plan, float* beta1_power, float* beta2_power, void* stream);
/* Single-GPU fast path (default on; = dssm_plan_set_option(DSSM_OPT_FUSED_W1_ADAM)): backward
 * leaves the light rows of dW1 un-materialized and dssm_plan_adam computes them inline from the CSC
 * transpose while updating W1, so a dense dW1 is never written or re-read; the split-K partial
 * slabs of dW_l (l >= 2) are likewise summed inside the Adam step instead of by a reduce launch.
 * Turn it off when the gradient arena must hold the full gradient (data-parallel exchange, or
 * inspecting the gradients). */
int dssm_plan_set_fused_w1_adam(dssm_plan* plan, int on);
/* Schedule options.  The plan never reads the environment: every alternative schedule is chosen
 * here, explicitly, and applies to the steps enqueued (or graphs captured) afterwards.  Defaults
 * are the measured-fastest schedule; the alternatives stay for parity tests and
 * for shapes the defaults do not support (a default the shape cannot run falls back by itself:
 * dssm_plan_schedule() reports what a step runs).
 *   FUSED_STATS     1: BN statistics fused into producers / consumers (bf16, BS % 64 == 0,
 *                      widths <= 512); 0: separate fixed-order statistics launches
 *   MERGED_CSC      1: the rank transpose's scan / scatter ride in the forward's launches
 *                      (with FUSED_STATS, BS % 128 == 0)
 *   HEAVY_IN_ADAM   1: dW1's heavy columns as work items inside the Adam launch
 *   SCATTER_IN_COS  1: the transpose's scatter as workgroups of the cosine launch (with MERGED_CSC)
 *   DW_IN_APPLY     1: dW_l split-K tiles inside the next BN-backward apply launch (FUSED_STATS)
 *   WIRE_GRAD_PASS  1: data parallel bf16 wire: dW1 written straight into the wire
 *   CSC_RANK        1: rank / scan / scatter transpose (D <= ~38k); 0: histogram / fill launches
 *   DETERMINISTIC   0; 1: fixed-order reductions only (separate statistics launches, every CSC
 *                      column in row order, heavy dW1 rows summed in item order): repeated runs
 *                      from the same state and batches are bit-identical
 *   FUSED_W1_ADAM   see dssm_plan_set_fused_w1_adam
 *   RANK_IN_ADAM    1: in multi-step graphs (dssm_plan_graph_build_steps) step i's Adam launch also
 *                      runs step i+1's CSC rank pass (with MERGED_CSC and FUSED_W1_ADAM), so that
 *                      step's forward skips the rank launch
 *   MEMCPY_NODES    0; 1 (diagnostics): the data-parallel graph's device copies (the all-to-all's own
 *                      chunk, the copy rehearsal) as hipMemcpyAsync -- memcpy nodes in a capture --
 *                      instead of the copy kernel
 *   BNB_IN_PAIR     1: bf16 fused schedule, last layer <= 128 wide: its BN backward is formed while the
 *                      dA pair launch stages its A operand (no BN-backward apply launch for it); 0: the
 *                      apply launch
 *   TAIL_IN_A2A     0; 1: dssm_plan_graph_build_dp_steps puts the fp32 tail's all-reduce into the last
 *                      chunk's all-to-all RCCL group (one collective launch fewer per step; dssm_amd/dist.py
 *                      turns it on after a start-up self-test of that mixed group at the real world size)
 *   FWD32           0; 1 (bf16 plans, fused-statistics schedule, no data-parallel wire): the forward
 *                      at the reference's precision -- the SpMM gathers the fp32 W1 masters and the
 *                      layers >= 2 run the fp32-parity g32 tiles on the fp32 W_l, writing the bf16
 *                      activations the bf16 backward reads -- so loss, cosine scores and embeddings
 *                      match new_dssm.py:117-213 at fp32 accuracy while the backward and the optimizer
 *                      stay the bf16 perf mode's (their gradients carry bf16 rounding) */
enum {
  DSSM_OPT_FUSED_STATS = 0,
  DSSM_OPT_MERGED_CSC,
  DSSM_OPT_HEAVY_IN_ADAM,
  DSSM_OPT_SCATTER_IN_COS,
  DSSM_OPT_DW_IN_APPLY,
  DSSM_OPT_WIRE_GRAD_PASS,
  DSSM_OPT_CSC_RANK,
  DSSM_OPT_DETERMINISTIC,
  DSSM_OPT_FUSED_W1_ADAM,
  DSSM_OPT_RANK_IN_ADAM,
  DSSM_OPT_MEMCPY_NODES,
  DSSM_OPT_BNB_IN_PAIR,
  DSSM_OPT_TAIL_IN_A2A,
  DSSM_OPT_FWD32,
  DSSM_OPT_COUNT
};
int dssm_plan_set_option(dssm_plan* plan, int option, int value);
/* The option's value (0 / 1), or -1 for a bad plan / option. */
int dssm_plan_get_option(const dssm_plan* plan, int option);
/* Sharded optimizer step (data parallel, ZeRO-1 style): dssm_plan_adam updates only arena
 * elements [begin, end) (multiples of 4; [0, param_count) restores the full step) -- the rank's
 * shard of a reduce-scattered gradient -- together with the bf16 shadows of those elements.  The
 * fused W1 Adam must be off.  DSSM_GRAPH_SHADOWS captures dssm_plan_sync_shadows (the shadows of
 * the all-gathered parameters). */
int dssm_plan_set_adam_range(dssm_plan* plan, int64_t begin, int64_t end);
/* Data-parallel bf16 wire (perf mode; replaces the fp32 gradient all-reduce of the reference's
 * single-process optimizer, new_dssm.py:215-217, when the batch is sharded over ranks).  W1's rows
 * -- arena elements [0, dssm_plan_wire_extent()) -- cross the links as bf16, in `chunks` pieces
 * (dssm_plan_graph_build_dp_steps; with one piece the next step's SpMM reads the parameter wire):
 *   - rank j's optimizer shard is W1 rows [j*chunks*S, (j+1)*chunks*S) (S = ceil(D / (world *
 *     chunks)) rows per sub-chunk; dssm_plan_dp_geometry); the wires hold sub-chunk (p, j) -- rows
 *     (j*chunks + p)*S + [0, S) -- at element ((p*world + j)*S)*n, so chunk p of every collective
 *     is one contiguous block of world*S*n elements (chunks == 1: the arena's own layout);
 *   - dssm_plan_backward ends by writing every rank's W1 gradient rows as bf16 into grad_wire (the
 *     caller all-to-alls chunk p of grad_wire into chunk p of stage);
 *   - dssm_plan_adam updates this rank's shard with the fp32 sum, in rank order, of the world's
 *     bf16 partials in stage (x grad_scale: each rank's gradient rounded to bf16 once), writes
 *     bf16(param) of the shard into param_wire (the caller all-gathers chunk p of it, in place),
 *     and updates the replicated fp32 tail [extent, param_count) -- b1, W2.., BN -- from the fp32
 *     gradient arena (the caller all-reduces that tail first) with its shadows;
 *   - dssm_plan_wire_shadows (graph part DSSM_GRAPH_WIRE_SHADOWS) rewrites W1's bf16 shadow from
 *     the all-gathered param_wire.
 * W1's fp32 master rows outside the rank's shard are then stale (all-gather them for a
 * checkpoint).  count: elements of each buffer (>= dssm_plan_dp_wire_size(world, chunks)).  stage
 * may be grad_wire at world 1 (the all-to-all is then the identity).  All NULL: off.  Needs bf16
 * mode and the fused W1 Adam off. */
int64_t dssm_plan_wire_extent(const dssm_plan* plan);
int64_t dssm_plan_dp_wire_size(const dssm_plan* plan, int world, int chunks);
int dssm_plan_set_dp_wire(dssm_plan* plan, int world, int rank, int chunks, uint16_t* grad_wire,
                          const uint16_t* stage, uint16_t* param_wire, int64_t count);
/* out[8] = {world, chunks, S, S*n (elements per rank per chunk), shard begin, shard end (this rank's W1
 * arena elements), extent, param_count}. */
int dssm_plan_dp_geometry(const dssm_plan* plan, int64_t* out);
int dssm_plan_wire_shadows(dssm_plan* plan, void* stream);
/* nsteps data-parallel training steps on the bf16 wire captured into ONE graph, step i on batch
 * (indptrs[i], ...), each step: forward, backward, the gradient pass (chunk by chunk), each chunk's
 * all-to-all, the fp32 tail all-reduce, Adam chunk by chunk, each chunk's all-gather, the shadow
 * rebuild per gathered chunk; step i+1's CSC rank pass rides in step i's Adam (with RANK_IN_ADAM).
 * overlap must be 0: every node on `stream` in that order (the two-stream variant, collectives on a
 * second captured stream, measured slower and raced under RCCL at world 1; removed in round 3).
 * comm: 0 = the library's RCCL communicator (dssm_comm_init; world / rank must match the wire's);
 * 1 = rehearsal on one GPU, each collective replaced by a device copy of its bytes; 2 = rehearsal,
 * each collective replaced by a kernel that holds its stream for latency_us + (bytes this rank
 * sends) / link_gbps (GB/s) -- the exchange's modelled time on the links; 3 = the peer-store
 * exchange (dssm_plan_set_dp_peers, below): no collectives, the shadow rebuilt every step.  with_probes: the Adam
 * probe brackets the last step's Adam launches. */
int dssm_plan_graph_build_dp_steps(dssm_plan* plan, const int32_t* const* indptrs,
                                   const int32_t* const* indices, const float* const* values,
                                   int nsteps, float grad_scale, int comm, float link_gbps,
                                   float latency_us, int overlap, int with_probes, void* stream,
                                   int* graph_id);
/* forward(train) + backward + adam: one sess.run(train_step) (new_dssm.py:267). */
int dssm_plan_train_step(dssm_plan* plan, void* stream);

/* hipGraph capture of a step for the CURRENT batch pointers (dssm_plan_set_batch): parts =
 * DSSM_GRAPH_FWD_BWD and/or DSSM_GRAPH_ADAM and/or DSSM_GRAPH_SHADOWS (data-parallel runs launch
 * the gradient collective between the first two).  Parts run in the order FWD_BWD, ADAM, the shadow
 * parts, except that a graph of FWD_BWD plus a shadow part WITHOUT ADAM runs the shadow refresh first
 * (the previous step's, then this step's forward + backward: data parallel saves a graph boundary per
 * step).  Replays then cost one launch per step.  with_probes: the graph records the timing
 * probes' events (read back for its last replay with dssm_plan_graph_probe_read).  stream must
 * not be the default stream.  Graphs are owned by the plan. */
enum { DSSM_GRAPH_FWD_BWD = 1, DSSM_GRAPH_ADAM = 2, DSSM_GRAPH_SHADOWS = 4, DSSM_GRAPH_WIRE_SHADOWS = 8 };
int dssm_plan_graph_build(dssm_plan* plan, int parts, float grad_scale, int with_probes,
                          void* stream, int* graph_id);
int dssm_plan_graph_launch(dssm_plan* plan, int graph_id, void* stream);
/* nsteps whole training steps (forward + backward + Adam, as dssm_plan_train_step) captured
 * back to back into ONE graph, step i on batch (indptrs[i], indices[i], values[i]): a replay
 * runs them with no host launch boundary between steps.  with_probes 1: the transpose / SpMM /
 * dW1 probes record the first step, the Adam probe the last; 2: the Adam probe alone.
 * The plan's current batch is left as it was. */
int dssm_plan_graph_build_steps(dssm_plan* plan, const int32_t* const* indptrs,
                                const int32_t* const* indices, const float* const* values,
                                int nsteps, int with_probes, void* stream, int* graph_id);

/* Kernel timing probes (bench/roofline): HIP events recorded on the launch stream around one
 * kernel family for up to max_samples launches (0 disables); read back the summed duration.
 * The DP_* probes time the phases of the LAST step of a data-parallel step graph
 * (dssm_plan_graph_build_dp_steps with probes): forward + backward (gradient pass excluded), the
 * wire gradient pass, the gradient all-to-all, the fp32 tail all-reduce, the parameter all-gather
 * and the W1 shadow rebuild; DSSM_PROBE_ADAM there is the Adam shard alone (its all-gather
 * excluded).  With wire chunks > 1 the gradient-pass / all-to-all / all-gather probes time chunk 0's
 * launch (the first gradient pass / all-to-all, the last all-gather). */
enum {
  DSSM_PROBE_SPMM_FWD = 0, DSSM_PROBE_DW1, DSSM_PROBE_ADAM, DSSM_PROBE_CSC,
  DSSM_PROBE_DP_FWD_BWD, DSSM_PROBE_DP_GRAD_PASS, DSSM_PROBE_DP_ALL_TO_ALL, DSSM_PROBE_DP_TAIL,
  DSSM_PROBE_DP_ALL_GATHER, DSSM_PROBE_DP_SHADOW, DSSM_PROBE_COUNT
};
int dssm_plan_probe_enable(dssm_plan* plan, int probe_id, int max_samples);
int dssm_plan_probe_read(dssm_plan* plan, int probe_id, float* total_ms, int* count);
/* 1 when the plan's bf16 train steps run with the batch-norm statistics fused into the producing /
 * consuming kernels (DSSM_OPT_FUSED_STATS, default on where supported: bf16, query_bs % 64 == 0,
 * widths <= 512, not DETERMINISTIC), else 0. */
int dssm_plan_fused_stats(dssm_plan* plan);
/* What a train step of this plan runs (bit set of DSSM_SCHED_*), for tests and reports that
 * must know which kernels produced a result. */
enum {
  DSSM_SCHED_FUSED_STATS = 1,      /* BN statistics fused into producers / consumers (bnfuse.h) */
  DSSM_SCHED_MERGED_CSC = 2,       /* CSC transpose split across the forward's launches */
  DSSM_SCHED_HEAVY_IN_ADAM = 4,    /* dW1 heavy columns as work items of the Adam launch */
  DSSM_SCHED_FUSED_W1_ADAM = 8,    /* dW1 light rows + dW_l slabs consumed inside Adam */
  DSSM_SCHED_WHOLEK = 16,          /* layers >= 2 on the whole-K bf16 NT / backward-pair GEMMs */
  DSSM_SCHED_DW_IN_APPLY = 32,     /* dW_l split-K tiles inside the next BN-backward apply launch */
  DSSM_SCHED_SCATTER_IN_COS = 64,  /* CSC scatter as workgroups of the cosine launch */
  DSSM_SCHED_DETERMINISTIC = 128,  /* fixed-order reductions: bit-identical repeated runs */
  DSSM_SCHED_NT32 = 256,           /* fp32: layers >= 2 on the fused fp32 MFMA tiles (g32.h) */
  DSSM_SCHED_BNB_IN_PAIR = 512,    /* the last layer's BN backward inside the dA pair's A staging */
  DSSM_SCHED_FWD32 = 1024          /* bf16 plan: the forward at fp32 accuracy (DSSM_OPT_FWD32) */
};
int dssm_plan_schedule(const dssm_plan* plan);
/* A train forward (either precision) leaves the loss / accuracy reduction to the backward's first
 * launch; call this before reading DSSM_BUF_LOSS after a train forward that was not followed by
 * dssm_plan_backward (no-op otherwise). */
int dssm_plan_finalize_loss(dssm_plan* plan, void* stream);
int dssm_plan_graph_probe_read(dssm_plan* plan, int graph_id, int probe_id, float* ms);
/* The shape of a captured graph as it was before instantiation (hipGraphGetNodes / GetEdges /
 * NodeGetType): out[8] = {nodes, edges, roots, kernel nodes, memcpy nodes, memset nodes, other
 * nodes, chain}.  chain = 1 when the graph is one path through every node, i.e. each node runs
 * after every node captured before it on the stream, whatever its type.  -1 entries: the runtime
 * could not report. */
int dssm_plan_graph_topology(const dssm_plan* plan, int graph_id, int64_t* out);

/* ---- fine-grained kernels (the functional API: add_layer / batch_normalization / cosine) -- */
/* FC1 (new_dssm.py:124-126): Z[r, :] = sum_k values[k] * W[indices[k], :] + bias.
 * W: [d x ldw] of w_dtype (ldw >= n, multiple of 4); Z: [rows x ldz] fp32, ldz = ldp(n).  bf16 W
 * with tight rows (ldw == n, not a multiple of 8: the parameter wire) needs 8 readable elements
 * after its last row (dssm_plan_dp_wire_size includes them). */
int dssm_spmm_csr_fwd(const int32_t* indptr, const int32_t* indices, const float* values, int rows,
                      const void* W, int w_dtype, int ldw, int n, const float* bias, float* Z,
                      int ldz, void* stream);
/* Epilogue activations of the functional forwards (the FC layer + tf.nn.relu of
 * archive/multi_view_dssm_v3.py:120-139 in one launch). */
enum { DSSM_ACT_NONE = 0, DSSM_ACT_RELU = 1 };
int dssm_spmm_csr_fwd_act(const int32_t* indptr, const int32_t* indices, const float* values, int rows,
                          const void* W, int w_dtype, int ldw, int n, const float* bias, float* Z,
                          int ldz, int act, void* stream);
/* ... with the output's storage chosen: z_dtype DSSM_F32, or DSSM_BF16 (RNE of the fp32 row sums;
 * needs bf16 W with ldw >= round_up(n, 8) and zero pads): the multi-view model's bf16 FC1
 * activation, the next layer's bf16 MFMA operand. */
int dssm_spmm_csr_fwd_ex(const int32_t* indptr, const int32_t* indices, const float* values, int rows,
                         const void* W, int w_dtype, int ldw, int n, const float* bias, void* Z, int z_dtype,
                         int ldz, int act, void* stream);
/* add_layer (archive/dssm_v3.py:44-53) on device: Z[M x ldz] = A[M x lda] . W[K x ldw] + bias,
 * inputs of dtype `dtype`, fp32 accumulate and output. */
int dssm_dense_fwd(const void* A, int lda, const void* W, int ldw, int dtype, int M, int K, int N,
                   const float* bias, float* Z, int ldz, void* stream);
int dssm_dense_fwd_act(const void* A, int lda, const void* W, int ldw, int dtype, int M, int K, int N,
                       const float* bias, float* Z, int ldz, int act, void* stream);
/* batch_normalization (new_dssm.py:62-88) + ReLU over rows [row0, row0+rows) of Z (one tower).
 * train!=0: batch moments, EMA update of ema_mean/ema_var; train==0: uses the EMA.
 * out: [rows x ldz] of out_dtype; batch_mean/var may be NULL.  ws: >= dssm_bn_ws_bytes(),
 * zero-filled before its first use (it holds re-armed completion tickets). */
size_t dssm_bn_ws_bytes(int rows, int ldz);
int dssm_bn_relu_fwd(const float* Z, int ldz, int rows, int n, const float* gamma, const float* beta,
                     float* ema_mean, float* ema_var, float eps, float decay, int train, int relu,
                     void* out, int out_dtype, float* batch_mean, float* batch_var, void* ws,
                     void* stream);
/* Cosine_Similarity + Loss (new_dssm.py:182-213) fused with their backward: y rows
 * [q; pos; neg] [R x ld] fp32 -> cos_sim_raw, cos_sim, prob, query_norm, loss[2] (loss, acc),
 * dy [R x ld] (d loss / d y).  ws: >= 2*ceil(BS/4) + 64 floats, zero-filled before its first
 * use (it holds a completion ticket the kernel re-arms). */
/* ... with the RNN tower's inverted dropout (dssm_rnn.py:139,146,153: tf.nn.dropout on the final states)
 * fused: rows read as x * m / keep with dssm_rnn_dropout's counter-based mask m (seed, step; mask index
 * r * n + c), the dropped rows written to y (NULL: not stored), and dy stored as d loss / d x =
 * (d loss / d y) * m * bwd_scale / keep -- the two dssm_rnn_dropout launches of the unfused form. */
int dssm_cosine_softmax_loss_dropout(const float* x, int ld, int n, int query_bs, int neg, float gamma, float keep,
                                     uint32_t seed, uint32_t step, float bwd_scale, float* y, float* cos_sim_raw,
                                     float* cos_sim, float* prob, float* query_norm, float* loss, float* dy,
                                     float* ws, void* stream);
int dssm_cosine_softmax_loss(const float* y, int ld, int n, int query_bs, int neg, float gamma,
                             float* cos_sim_raw, float* cos_sim, float* prob, float* query_norm,
                             float* loss, float* dy, float* ws, void* stream);
/* The same with the rows read through a map: merged row r of [q; pos; neg] is y row row_map[r]
 * (multi_view_dssm_v3's in-batch rotated negatives, Make_Negative_Item, without a gathered copy);
 * dy [R x ld] is in the merged layout. */
int dssm_cosine_softmax_loss_mapped(const float* y, int ld, const int32_t* row_map, int n, int query_bs, int neg,
                                    float gamma, float* cos_sim_raw, float* cos_sim, float* prob,
                                    float* query_norm, float* loss, float* dy, float* ws, void* stream);

/* ---- functional backward (the per-op gradients; the plan fuses them) ---------------------- */
/* tf.sparse_tensor_dense_matmul's weight gradient (new_dssm.py:124-126 autodiff, dense like
 * TF1.x): dWb [(D+1) x n] = [X | 1]^T dZ (row D = db).  dZ [rows x lddz] of dz_dtype (lddz % 8 ==
 * 0).  ws: dssm_spmm_bwd_ws_bytes() bytes, zero-filled before first use (CSC transpose scratch,
 * kept zero between calls). */
size_t dssm_spmm_bwd_ws_bytes(int rows, int D, int max_nnz);
int dssm_spmm_csr_bwd_w(const int32_t* indptr, const int32_t* indices, const float* values, int rows,
                        int D, int max_nnz, const void* dZ, int dz_dtype, int lddz, int n, float* dWb,
                        void* ws, void* stream);
/* The CSC transpose [X | 1]^T that the weight gradient above gathers over: column c
 * (< D) holds the batch entries of trigram c, column D the virtual ones column (row r at slot
 * col_ptr[D] + r).  col_ptr [D + 2], csc_row / csc_val / csc_col [max_nnz + rows].  row_order != 0:
 * every column's entries in ascending row order (the deterministic mode's transpose; scipy's
 * tocsc() order); 0: per-column order set by atomics.  ws: dssm_spmm_bwd_ws_bytes() bytes,
 * zero-filled before first use. */
int dssm_csc_transpose(const int32_t* indptr, const int32_t* indices, const float* values, int rows, int D,
                       int max_nnz, int row_order, int32_t* col_ptr, int32_t* csc_row, float* csc_val,
                       int32_t* csc_col, void* ws, void* stream);
/* add_layer / tf.matmul(x, W) + b autodiff (new_dssm.py:146-148): dA [M x ldda] = dZ W^T (dA may be
 * NULL), dWb [(K+1) x N] = [A | 1]^T dZ (row K = db).  A [M x lda], W [K x ldw], dZ [M x lddz] of
 * dtype; fp32 accumulation; slab: dssm_dense_bwd_slab_floats() floats (split-K partials). */
size_t dssm_dense_bwd_slab_floats(int M, int K, int N, int dtype);
int dssm_dense_bwd(const void* A, int lda, const void* W, int ldw, int dtype, int M, int K, int N,
                   const void* dZ, int lddz, float* dA, int ldda, float* dWb, float* slab, void* stream);
/* dssm_dense_bwd with the ReLU backward of the layer's input fused into dA: dA = (dZ W^T) where
 * mask [M x ldmask] > 0, else 0 (mask = the ReLU output that was the layer's input A; ReluGrad). */
int dssm_dense_bwd_masked(const void* A, int lda, const void* W, int ldw, int dtype, int M, int K, int N,
                          const void* dZ, int lddz, float* dA, int ldda, const float* mask, int ldmask,
                          float* dWb, float* slab, void* stream);
/* ... with dA stored as da_dtype (DSSM_F32, or DSSM_BF16: RNE) and the mask read as mask_dtype (the
 * bf16 activation itself): the multi-view model's bf16 backward. */
int dssm_dense_bwd_ex(const void* A, int lda, const void* W, int ldw, int dtype, int M, int K, int N,
                      const void* dZ, int lddz, void* dA, int da_dtype, int ldda, const void* mask, int mask_dtype,
                      int ldmask, float* dWb, float* slab, int* deferred_splits, void* stream);
/* (deferred_splits != NULL: when the weight gradient is split over K, the partials stay in slab
 * [splits x (K+1) x N] for dssm_spmm_bwd_w_adam to sum, *deferred_splits = splits; 0: dWb written.) */
/* batch_normalization + ReLU backward with batch statistics (new_dssm.py:62-88, :134-136; ReLU'(0) =
 * 0): from the forward's Z, gamma, beta and batch mean / biased variance (dssm_bn_relu_fwd's
 * batch_mean / batch_var), dout -> dz, dgamma, dbeta.  relu = 0: plain batch norm. */
int dssm_bn_relu_bwd(const float* Z, int ldz, int rows, int n, const float* gamma, const float* beta,
                     const float* batch_mean, const float* batch_var, float eps, int relu,
                     const float* dout, int ldd, float* dz, int lddz, float* dgamma, float* dbeta,
                     void* stream);
/* TF1.x ApplyAdam (new_dssm.py:215-217) over n flat elements with gradient x grad_scale;
 * state = device {beta1_power, beta2_power} (start at beta1, beta2), advanced after the update
 * when advance != 0 (an optimizer step spanning several calls advances on its last one). */
int dssm_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                   float beta2, float eps, float* state, float grad_scale, int advance, void* stream);
/* The same step over one or two ranges of the arrays in ONE launch (ranges = {begin0, end0[, begin1,
 * end1]}: element offsets, multiples of 4; 16-B aligned arrays; indices < 2^31), also writing each updated
 * weight of the given blocks (at most 4) as bf16 to its shadow: segment i covers elements [offset,
 * offset + rows * cols) of p (row-major, rows x cols: a [W; b] block's W rows), shadow ptr [rows x ld]
 * (ld >= cols; offset, cols, ld multiples of 4).  The bf16 weights the next forward reads, without a
 * refresh pass over the parameters (the multi-view model's bf16 mode: both trained towers, one launch). */
typedef struct dssm_shadow_seg {
  int64_t offset;
  int64_t rows;
  int cols;
  int ld;
  uint16_t* ptr;
} dssm_shadow_seg;
int dssm_adam_step_shadow(float* p, const float* g, float* m, float* v, const int64_t* ranges, int nranges,
                          float lr, float beta1, float beta2, float eps, float* state, float grad_scale, int advance,
                          const dssm_shadow_seg* segs, int nseg, void* stream);
/* One tower's FC1 weight gradient and optimizer step in one pass, the dense [dW1; db1] never stored
 * (the training-step plan's fused single-GPU Adam as a functional op; replaces dssm_spmm_csr_bwd_w +
 * that tower's dssm_adam_step_shadow): builds the batch's CSC transpose [X | 1]^T in ws, then ONE
 * launch applies TF1.x ApplyAdam (new_dssm.py:215-217) to
 *   - rows [0, D] of the tower's [W1; b1] block at p (row length n, n % 4 == 0): a touched row's
 *     gradient gathered from the transpose and dZ [rows x lddz] (dz_dtype), the ones column (db1)
 *     and any column with more than 64 entries as work items of 256 entries; an untouched row
 *     decays (gradient 0);
 *   - elements [rest_begin, rest_end) of p (multiples of 4): gradient g, or for
 *     [rest_begin, rest_begin + slab_count) the sum of splits partials slab[k * slab_count + i]
 *     (dssm_dense_bwd_ex's deferred split-K; splits == 0: g).
 * g's rows [0, D] must be zero and are left zero (heavy columns' atomics target); gradient x
 * grad_scale.  bf16: W1's rows also written to w1_shadow [D x ld_shadow] (NULL: none), the rest range
 * to the shadow segments (offsets relative to p).  The beta powers: group == 0, not advanced (call
 * dssm_adam_advance once every trained block of the step is updated); group = n > 0, this launch is
 * member `member` of the step's n launches (any streams, concurrent or not) sharing `tickets`
 * (dssm_adam_tickets_bytes(n) bytes, zero-filled once, re-armed by the launches), and the last of them
 * to finish advances the powers -- no separate launch, no join before it.  Needs the CSC rank path
 * (D <= 36800). */
size_t dssm_adam_tickets_bytes(int group);
/* build_csc = 0: the transpose is already in ws, built for the same batch by dssm_spmm_bwd_csc
 * earlier in stream order (e.g. on another stream while the loss runs), and only the optimizer
 * launches. */
int dssm_spmm_bwd_csc(const int32_t* indptr, const int32_t* indices, const float* values, int rows, int D,
                      int max_nnz, void* ws, void* stream);
int dssm_spmm_bwd_w_adam(const int32_t* indptr, const int32_t* indices, const float* values, int rows, int D,
                         int max_nnz, const void* dZ, int dz_dtype, int lddz, int n, float* p, float* g, float* m,
                         float* v, int64_t rest_begin, int64_t rest_end, const float* slab, int64_t slab_count,
                         int splits, uint16_t* w1_shadow, int ld_shadow, const dssm_shadow_seg* segs, int nseg,
                         float lr, float beta1, float beta2, float eps, float* state, float grad_scale,
                         int group, int member, void* tickets, int build_csc, void* ws, void* stream);
/* (dssm_tower_adam: the per-tower arguments above as one record, the form the C++ side validates) */
typedef struct dssm_tower_adam {
  const int32_t* indptr;
  const int32_t* indices;
  const float* values;
  int rows, D, max_nnz;
  const void* dZ;
  int dz_dtype, lddz, n;
  float *p, *g, *m, *v;
  int64_t rest_begin, rest_end;
  const float* slab;
  int64_t slab_count;
  int splits;
  uint16_t* w1_shadow;
  int ld_shadow;
  const dssm_shadow_seg* segs;
  int nseg;
  int build_csc;
  void* ws;
} dssm_tower_adam;
/* TF1.x AdamOptimizer._finish: beta1_power *= beta1, beta2_power *= beta2 (state on the device). */
int dssm_adam_advance(float* state, float beta1, float beta2, void* stream);
/* Measurement: HIP events around the next n_max dssm_adam_step optimizer launches (0: off); read
 * averages the recorded launches (in a captured graph, each launch's latest replay). */
int dssm_adam_probe(int n_max);
int dssm_adam_probe_read(double* avg_ms, int* count);
/* ... and the wall span of n recorded launches from index first (launches that ran concurrently on
 * several streams): the latest end minus the earliest start. */
int dssm_adam_probe_span(int first, int n, double* span_ms);
/* Row gather / scatter-add (Merge_Negative_Doc by index, its backward): dst[r] = src[map[r]];
 * dst[map[r]] += src[r] over r < n after dst (dst_rows x ldd) is cleared.  fp32. */
int dssm_rows_gather(const float* src, int lds, const int32_t* map, int n, int cols, float* dst, int ldd,
                     void* stream);
int dssm_rows_scatter_add(const float* src, int lds, const int32_t* map, int n, int cols, float* dst,
                          int ldd, int dst_rows, void* stream);
/* The scatter-add's inverse form (Merge_Negative_Doc's gradient without atomics): dst[r] = scale *
 * sum over j in [offs[r], offs[r+1]) of src[idx[j]], summed in list order, for r < n; with mask
 * (ld ldm) the result is 0 where mask[r] <= 0 (the ReLU backward of the rows' forward output). */
int dssm_rows_gather_sum(const float* src, int lds, const int32_t* offs, const int32_t* idx, int n, int cols,
                         float scale, const float* mask, int ldm, float* dst, int ldd, void* stream);
/* ... with dst stored as dst_dtype (DSSM_F32, or DSSM_BF16: RNE of the fp32 sum). */
int dssm_rows_gather_sum_ex(const float* src, int lds, const int32_t* offs, const int32_t* idx, int n, int cols,
                            float scale, const float* mask, int ldm, void* dst, int dst_dtype, int ldd,
                            void* stream);
/* tf.nn.relu and its gradient (ReluGrad: dx = y > 0 ? dy : 0); y may alias x. */
int dssm_relu(const float* x, int ldx, int rows, int cols, float* y, int ldy, void* stream);
int dssm_relu_bwd(const float* y, int ldy, const float* dy, int lddy, int rows, int cols, float* dx,
                  int lddx, void* stream);

/* ---- data parallel: the library's RCCL communicator ----------------------
 * One communicator per process (one process per GPU).  unique_id: 128 bytes from
 * dssm_comm_unique_id() on rank 0, shared by the caller (dssm_amd/dist.py broadcasts it through
 * torch.distributed's store: bootstrap only, no data).  Collectives are asynchronous on `stream`
 * and replace the reference's single-process optimizer (new_dssm.py:215-217) when the batch is
 * sharded over ranks; dtype DSSM_F32 or DSSM_BF16 (summed by RCCL in that type).  count is per rank
 * (reduce-scatter: recv count, send holds world * count; all-gather: send count; all-to-all: the
 * chunk each pair of ranks exchanges, chunk j of send goes to rank j and chunk j of recv comes from
 * rank j; send != recv).  In-place reduce-scatter / all-gather: recv == send + rank * count /
 * send == recv + rank * count. */
int dssm_comm_unique_id(void* out128);
int dssm_comm_init(int rank, int world, const void* unique_id128);
int dssm_comm_world(void);  /* world size, 0 before dssm_comm_init */
/* The communicator as RCCL sees it (ncclCommCount / ncclCommUserRank; -1 before dssm_comm_init) and
 * the linked RCCL's version (ncclGetVersion, e.g. 22703 for 2.27.3): for the N > 1 bench line. */
int dssm_comm_info(int* rccl_world, int* rccl_rank, int* rccl_version);
int dssm_allreduce_sum(void* buf, int64_t count, int dtype, void* stream);
int dssm_allreduce_sum_f32(float* buf, int64_t count, void* stream);
int dssm_reduce_scatter_sum(const void* send, void* recv, int64_t count, int dtype, void* stream);
int dssm_all_gather(const void* send, void* recv, int64_t count, int dtype, void* stream);
int dssm_all_to_all(const void* send, void* recv, int64_t count, int dtype, void* stream);
/* The same all-to-all with an fp32 all-reduce of tail[0, tail_count) in place inside its RCCL group
 * (ncclGroupStart; per peer ncclSend / ncclRecv; ncclAllReduce; ncclGroupEnd): exactly the call the
 * data-parallel step graph captures under plan option TAIL_IN_A2A, exported so the start-up
 * self-test (dssm_amd/dist.py) runs that mixed point-to-point / collective group at the real world
 * size, eagerly and captured, before the option is turned on. */
int dssm_all_to_all_tail(const void* send, void* recv, int64_t count, int dtype, float* tail,
                         int64_t tail_count, void* stream);
/* Variable-count all-to-all (the touched-row sparse gradient exchange, dssm_amd/dist.py
 * DataParallel(sparse=True)): send_counts[j] elements of send (consecutive, in rank order) go to
 * rank j, recv_counts[j] elements of recv come from rank j (host arrays of world entries; the own
 * entries equal).  tail != NULL: tail_count elements of tail summed over the ranks in place
 * (all-reduce) in the same RCCL group.  Replaces the dense all-to-all + tail all-reduce of the
 * zero schedule (new_dssm.py:215-217's gradient application, sharded). */
int dssm_all_to_allv(const void* send, const int64_t* send_counts, void* recv, const int64_t* recv_counts,
                     int dtype, void* tail, int64_t tail_count, int tail_dtype, void* stream);
int dssm_comm_destroy(void);

/* Peer-store exchange (DESIGN.md §6 "peer exchange"; dssm_amd/csrc/peer.hip): the bf16-wire
 * schedule with no collective library on the data path, replacing the gradient all-to-all, the
 * fp32 tail all-reduce and the parameter all-gather that stand in for the reference's fp32 gradient
 * reduction (new_dssm.py:215-217 over a sharded batch).  Each rank allocates its stage and parameter
 * wire (dssm_plan_dp_wire_size elements of bf16 each), its tail stage (world * (param_count -
 * extent) floats) and its flags (DSSM_PEER_FLAG_BYTES) with dssm_peer_alloc (fine-grained device
 * memory, zeroed), shares dssm_ipc_handle of each with every rank, maps the others' with
 * dssm_ipc_open, attaches its own stage / parameter wire with dssm_plan_set_dp_wire (one chunk) and
 * then the world's buffers, indexed by rank, with dssm_plan_set_dp_peers.  All ranks must attach
 * zeroed flags before any rank's first step (a host barrier).  Then:
 *   - dssm_plan_backward's gradient pass stores this rank's bf16 W1 gradient rows straight into each
 *     owner's stage (block `rank`), as the all-to-all would have delivered them;
 *   - dssm_plan_peer_exchange(phase 0), between backward and adam: the fp32 tail pushed to every
 *     rank, a wait for every rank's gradient pass of this step, the tails summed in rank order;
 *   - dssm_plan_adam stores bf16(W1) of the shard into every rank's parameter wire;
 *   - dssm_plan_peer_exchange(phase 1), after adam: this rank's "parameters ready" flag on every
 *     rank, a wait for every rank's;
 *   - dssm_plan_wire_shadows rebuilds W1's shadow from the parameter wire (behind an acquire).
 * dssm_plan_graph_build_dp_steps with comm 3 captures the same sequence.  Waits are bounded
 * (dssm_plan_set_peer_timeout, default 20 s): a timeout is recorded, later waits return at once, and
 * dssm_plan_peer_status reports {error (0: none, else 1 + flag index), steps exchanged}. */
#define DSSM_PEER_FLAG_BYTES 4096
int dssm_peer_alloc(int64_t bytes, void** out);
int dssm_peer_free(void* ptr);
/* *out = 1 when the current device can map peer_device's memory (hipDeviceCanAccessPeer; the same
 * device: 1): DataParallel checks every pair before opening any peer's handle. */
int dssm_peer_can_access(int peer_device, int* out);
int dssm_ipc_handle(void* ptr, void* out64);
int dssm_ipc_open(const void* handle64, void** out);
int dssm_ipc_close(void* ptr);
int dssm_plan_set_dp_peers(dssm_plan* plan, int world, uint16_t* const* stages, uint16_t* const* param_wires,
                           float* const* tails, unsigned* const* flags);
int dssm_plan_set_peer_timeout(dssm_plan* plan, double ms);
int dssm_plan_peer_exchange(dssm_plan* plan, int phase, void* stream);
int dssm_plan_peer_status(const dssm_plan* plan, unsigned* out2);
/* Start-up self-test at the real world size (every rank calls it once, together, before its first
 * step): each rank stores a synthetic pattern into its slot of every rank's tail stage and its shard
 * block of every rank's parameter wire, releases and flags as a step does, and reads all slots and
 * blocks back with the consumers' system-scope loads.  *mismatches = elements that differ (0: pass;
 * -1: a wait timed out).  Synchronous; the buffers it writes are overwritten by the next step. */
int dssm_plan_peer_selftest(dssm_plan* plan, int64_t* mismatches, void* stream);
/* Packed rows of the sparse exchange, stride n + 4 u16: [row id int32][pad][n u16 of src row id].
 * pack: packed row k from src row rows[k] (n % 4 == 0); unpack: dst row (id - row_base) = packed row
 * k's data for ids in [row_base, row_base + nrows) (others skipped). */
int dssm_rows_pack_u16(const uint16_t* src, int64_t n, const int32_t* rows, int64_t count, uint16_t* out,
                       void* stream);
int dssm_rows_unpack_u16(const uint16_t* in, int64_t n, int64_t count, int64_t row_base, int64_t nrows,
                         uint16_t* dst, void* stream);

/* ---- host data path (utils/utils.py:20-24, 45-61, 368-437; new_dssm.py:26-49) ---------------
 * Host memory only (no device pointers) except the feeder's outputs. */
/* pre_process (utils/utils.py:424-437) of one UTF-8 line: short links removed, only U+4E00..U+9FA5,
 * 0-9, A-Z, a-z kept.  Writes up to cap-1 bytes + NUL to out (may be NULL); *len = full length. */
int dssm_text_clean(const char* text, char* out, size_t cap, size_t* len);
/* CountVectorizer(token_pattern=r"(?u)\b\w+\b") (new_dssm.py:37-45) for pre_processed text:
 * lowercase, tokens = maximal runs of [0-9A-Za-z_] / U+4E00..U+9FA5, feature ids in code-point
 * order of the token strings (sklearn's sorted vocabulary_), counts per document as CSR. */
typedef struct dssm_vocab dssm_vocab;
int dssm_vocab_create(dssm_vocab** out);
int dssm_vocab_destroy(dssm_vocab* v);
int dssm_vocab_fit(dssm_vocab* v, const char* const* texts, int64_t n);   /* accumulate tokens */
int64_t dssm_vocab_finalize(dssm_vocab* v);                               /* -> TRIGRAM_D */
int64_t dssm_vocab_size(const dssm_vocab* v);
/* feature name i (get_feature_names()[i]) into out; returns its byte length */
int dssm_vocab_name(const dssm_vocab* v, int64_t i, char* out, size_t cap);
/* append a feature (restoring a saved vocabulary in id order) */
int dssm_vocab_add(dssm_vocab* v, const char* name);
/* CRC-32C (Castagnoli) of n host bytes, extending the finished CRC `crc` (0 to start): the checksum
 * TF1.x's tf.train.Saver V2 checkpoints carry per tensor and per index block (new_dssm.py:248,331;
 * dssm_amd/tfckpt.py).  SSE4.2 crc32 instructions, 8 bytes per step. */
uint32_t dssm_crc32c(uint32_t crc, const void* data, size_t n);
/* vectorizer.transform: indptr [n+1]; indices / values [cap] (NULL: count only) */
int dssm_vocab_transform(const dssm_vocab* v, const char* const* texts, int64_t n, int64_t* indptr,
                         int32_t* indices, float* values, int64_t cap, int64_t* nnz_out);
/* Asynchronous feeder of the step's combined device CSR (pull_batch, utils/utils.py:45-61): from the
 * three host CSR matrices m = query [N x D], doc [N x D], doc_neg [N*NEG x D] (caller-owned,
 * alive until destroy), a worker thread assembles batch b's rows [q; pos; neg] into a pinned slot
 * and copies it to the slot's device buffers on the feeder's stream.  submit(slot, b) queues it;
 * acquire(slot, stream) waits for the copy to be queued, makes `stream` wait for it on the device
 * and returns the device pointers (for dssm_plan_set_batch); release(slot, stream) after the step
 * reading them is enqueued makes the slot's next copy wait for that step. */
typedef struct dssm_feeder dssm_feeder;
int dssm_feeder_create(const int64_t* const* indptr, const int32_t* const* indices,
                       const float* const* values, const int64_t* rows, int query_bs, int neg,
                       int64_t max_nnz, int nslots, dssm_feeder** out);
int dssm_feeder_submit(dssm_feeder* f, int slot, int64_t batch);
int dssm_feeder_acquire(dssm_feeder* f, int slot, void* stream, const int32_t** indptr,
                        const int32_t** indices, const float** values, int64_t* nnz);
int dssm_feeder_release(dssm_feeder* f, int slot, void* stream);
int dssm_feeder_destroy(dssm_feeder* f);

/* ---- RNN tower (semantic_matching/dssm_rnn/dssm_rnn.py:100-217) ------------
 * Word-embedding lookup + one bidirectional GRU (tf.contrib.rnn.GRUCell(H) shared by the three
 * inputs, bidirectional_dynamic_rnn with per-row lengths) over rows [q(BS); pos(BS); neg(BS*NEG)],
 * fp32.  ids: [R x T] int32 (row r's tokens, valid up to lens[r], 1 <= lens[r] <= T); emb [V x E];
 * w[4] = {fw [Wg; bg] ((E+H+1) x 2H), fw [Wc; bc] ((E+H+1) x H), bw [Wg; bg], bw [Wc; bc]} (the last
 * row is the bias, the reference's _gate_bias / _candidate_bias).  E, H multiples of 4, E+H <= 512,
 * H <= 256.  ws: dssm_rnn_ws_floats() floats (step caches of the forward, read by the backward). */
size_t dssm_rnn_ws_floats(int R, int T, int E, int H);
/* y [R x ldy] = concat(final fw state, final bw state) (dssm_rnn.py:138-152) */
int dssm_rnn_forward(const int32_t* ids, const int32_t* lens, int R, int T, const float* emb, int E,
                     int H, const float* const* w, float* ws, float* y, int ldy, void* stream);
/* tf.nn.dropout(x, keep) (dssm_rnn.py:141,147,153) with a counter-based mask (seed, step): y = x *
 * mask * scale / keep; the backward is the same call on dy (scale folds the loss scale). */
int dssm_rnn_dropout(const float* x, float* y, int rows, int cols, int ld, float keep, uint32_t seed,
                     uint32_t step, float scale, void* stream);
/* Backward of dssm_rnn_forward for dy [R x lddy]: the dense embedding gradient into demb
 * (demb_elems = V*E floats, cleared first), [W; b] gradients written to gw[4] (shapes of w). */
int dssm_rnn_backward(const int32_t* ids, const int32_t* lens, int R, int T, int E, int H,
                      const float* const* w, const float* dy, int lddy, float* ws, float* demb,
                      int64_t demb_elems, float* const* gw, void* stream);
/* bf16 perf mode of the same tower (csrc/rnn_mfma.hip): the recurrences on v_mfma_f32_16x16x32_bf16
 * with each direction's weights resident in VGPRs (bf16 copies of the fp32 w[4] made by the
 * kernels), fp32 states / accumulation / gradients, bf16 step caches in ws.  Same arguments and
 * outputs as the fp32 calls plus V (the embedding table's rows, for its bf16 copy in ws).
 * Shapes: (E, H) in {(128, 128), (64, 128), (32, 32)} (dssm_rnn_bf16_supported), V <= 32768.
 * Workspace contract: ws (dssm_rnn_bf16_ws_bytes) must be ZERO-FILLED before its first use and
 * kept for this model alone: the backward's token-bucketing counts live in it, are assumed zero on
 * entry and are re-zeroed by the backward itself (no clear launch per step).  A ws allocated with
 * a plain hipMalloc and not cleared gives garbage start offsets (out-of-bounds position writes). */
int dssm_rnn_bf16_supported(int E, int H);
size_t dssm_rnn_bf16_ws_bytes(int R, int T, int E, int H, int V);
int dssm_rnn_bf16_forward(const int32_t* ids, const int32_t* lens, int R, int T, const float* emb, int V,
                          int E, int H, const float* const* w, void* ws, float* y, int ldy, void* stream);
int dssm_rnn_bf16_backward(const int32_t* ids, const int32_t* lens, int R, int T, int V, int E, int H,
                           const float* const* w, const float* dy, int lddy, void* ws, float* demb,
                           float* const* gw, void* stream);
/* The forward with emb16_current = 1: the workspace's bf16 copy of the embedding table (at byte
 * dssm_rnn_bf16_emb16_offset() of ws) is already bf16(emb) -- written by the last dssm_rnn_adam_ex
 * -- so the per-step conversion pass is skipped (0: as dssm_rnn_bf16_forward). */
size_t dssm_rnn_bf16_emb16_offset(int R, int T, int E, int H, int V);
int dssm_rnn_bf16_forward_ex(const int32_t* ids, const int32_t* lens, int R, int T, const float* emb, int V,
                             int E, int H, const float* const* w, void* ws, float* y, int ldy, int emb16_current,
                             void* stream);
/* Timing probes (benchmarks): record HIP events around the next n_max BPTT launches (n_max = 0:
 * off); read the average launch duration of the recorded ones (synchronizes on their events). */
int dssm_rnn_bf16_probe(int n_max);
int dssm_rnn_bf16_probe_read(double* avg_ms, int* count);
/* AdamOptimizer (dssm_rnn.py:218) over a flat arena: [0, n_sparse) the embedding table (TF1's
 * deduplicated IndexedSlices update, m*b1 + (1-b1) g form), the rest dense ApplyAdam; state =
 * device {beta1_power, beta2_power}, advanced after the update. */
int dssm_rnn_adam(float* p, const float* g, float* m, float* v, int64_t n_sparse, int64_t n,
                  float* state, float lr, float beta1, float beta2, float eps, void* stream);
/* ... also writing bf16(p) of [0, n_sparse) (the embedding table) to shadow (NULL: none): the bf16
 * recurrences' embedding copy, kept current by the optimizer. */
int dssm_rnn_adam_ex(float* p, const float* g, float* m, float* v, int64_t n_sparse, int64_t n,
                     float* state, float lr, float beta1, float beta2, float eps, uint16_t* shadow, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DSSM_H */
