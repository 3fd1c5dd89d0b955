// AdamOptimizer(lr).minimize(loss) (new_dssm.py:215-217) as TF1.x ApplyAdam over the flat
// parameter arena, dense (every element decays m/v every step, as TF does), fused with the
// refresh of the bf16 weight shadows that the perf-mode SpMM/GEMMs read.
//
//   alpha = lr * sqrt(1 - beta2^t) / (1 - beta1^t)   (fp32, like the TF kernel; the beta powers
//   live on the device and the step's last block multiplies them, so a captured step graph
//   needs no per-step host scalars)
//   m += (g - m) * (1 - beta1);  v += (g*g - v) * (1 - beta2)
//   p -= (m * alpha) / (sqrt(v) + eps)
//
// HBM-bound: 28 B/param (p, m, v read+write, g read) + 2 B/param of shadow.
//
// One launch (k_adam_step) per step, two block roles:
//  * fused W1 rows (single-GPU path): one wave per row of the [W1; b1] block computes the light
//    rows' gradient inline from the CSC transpose and dZ1 (gather.h) and applies Adam in the
//    same pass, so a dense dW1 is never written or re-read; heavy rows (summed by k_dw1_heavy
//    into the gradient arena) are read and cleared ("consume and clear": the atomic targets
//    start the next step at zero without a memset);
//  * dense float4 streaming over the rest of the arena (or all of it when unfused).
// The last block to finish advances the device beta powers.
#include "common.h"
#include "flat.h"
#include "gather.h"
#include "launch.h"

#include <algorithm>

#ifndef DSSM_ADAM_ORDER
#define DSSM_ADAM_ORDER 0
#endif
#ifndef DSSM_RANK_POS
#define DSSM_RANK_POS 1
#endif
#ifndef DSSM_ADAM_PRE_IDX
#define DSSM_ADAM_PRE_IDX 1
#endif
#ifndef DSSM_ADAM_GATHER_U  // rows in flight in the W1-row role's gather batches
#define DSSM_ADAM_GATHER_U 4
#endif
#ifndef DSSM_ADAM_HEAVY_U  // rows in flight in the heavy items' gather batches
#define DSSM_ADAM_HEAVY_U 8
#endif
#ifndef DSSM_ADAM_LATE_PMV
#define DSSM_ADAM_LATE_PMV 0
#endif
#ifdef DSSM_ADAM_WPE  // diagnostics builds: a minimum occupancy (waves per SIMD) for the step kernel
#define DSSM_ADAM_ATTR __attribute__((amdgpu_waves_per_eu(DSSM_ADAM_WPE)))
#else
#define DSSM_ADAM_ATTR
#endif

namespace dssm {
namespace {

// Diagnostics build only (-DDSSM_WG_TL): per-workgroup start / end stamps of k_adam_step
// (s_memrealtime, 100 MHz), read back by dssm_debug_adam_timeline (tools/wg_timeline.py).
#ifdef DSSM_WG_TL
__device__ unsigned long long g_adam_tl[8192][2];
#define ADAM_TL(idx)                                                                          \
  do {                                                                                        \
    if (threadIdx.x == 0 && blockIdx.x < 8192) g_adam_tl[blockIdx.x][idx] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define ADAM_TL(idx) \
  do {               \
  } while (0)
#endif

__device__ __forceinline__ void write_shadow4(const ShadowList& sh, int64_t i, float4 v) {
#pragma unroll 1
  for (int s = 0; s < sh.count; ++s) {
    const ShadowSeg& g = sh.seg[s];
    const int64_t rel = i - g.offset;
    if (rel >= 0 && rel < g.rows * g.cols) {
      const int64_t r = rel / g.cols;
      const int c = (int)(rel - r * g.cols);
      uint2 p;
      p.x = pack2bf(v.x, v.y);
      p.y = pack2bf(v.z, v.w);
      *reinterpret_cast<uint2*>(g.ptr + r * g.ld + c) = p;
      if (g.tptr) {
        g.tptr[(int64_t)(c + 0) * g.tld + r] = f2bf(v.x);
        g.tptr[(int64_t)(c + 1) * g.tld + r] = f2bf(v.y);
        g.tptr[(int64_t)(c + 2) * g.tld + r] = f2bf(v.z);
        g.tptr[(int64_t)(c + 3) * g.tld + r] = f2bf(v.w);
      }
      return;
    }
  }
}

__device__ __forceinline__ bool in_slabs(const SlabList& sl, int64_t i) {
  for (int s = 0; s < sl.count; ++s)
    if (i >= sl.seg[s].offset && i < sl.seg[s].offset + sl.seg[s].count) return true;
  return false;
}

// Gradient of element i..i+3: from a deferred split-K slab (fixed split order, as
// k_splitk_reduce would have summed it) or from the arena.
__device__ __forceinline__ float4 slab_grad4(const SlabList& sl, int64_t i, const float* g) {
#pragma unroll 1
  for (int s = 0; s < sl.count; ++s) {
    const SlabSeg& q = sl.seg[s];
    const int64_t rel = i - q.offset;
    if (rel >= 0 && rel < q.count) {
      const float* b = q.slab + rel;
      float4 acc = *reinterpret_cast<const float4*>(b);
      for (int z = 1; z < q.splits; ++z) {
        const float4 x = *reinterpret_cast<const float4*>(b + (size_t)z * q.count);
        acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
      }
      return acc;
    }
  }
  return *reinterpret_cast<const float4*>(g + i);
}


// One wave updates row c of [W1; b1] (CSC column c): light rows' gradient is gathered inline
// from the CSC transpose and dZ1, heavy rows' gradient (k_dw1_heavy) is read and cleared.
// A light row's CSC entries (index, value), lane j holding entry j: loaded one row ahead of the
// row's gather (DSSM_ADAM_PRE_IDX), so the row's chain starts at the dZ1 loads.
struct RowEntries {
  int i;
  float v;
};

// gradient pass by wire chunks (a.wchunk >= 0): is row c (c == D: b1's row, last chunk) in it
__device__ __forceinline__ bool in_chunk(const AdamStep& a, int c) {
  if (a.wchunk < 0) return true;
  if (c >= a.D) return a.wchunk == a.geo.wp - 1;
  return (c / a.geo.ws) % a.geo.wp == a.wchunk;
}
// the W1-row role's v-th row: every row [0, D] (wchunk < 0) or the chunk's rows, b1's row last
// (-1: a slot past W1's rows)
__device__ __forceinline__ int w1_role_rows(const AdamStep& a) {
  return a.wchunk < 0 ? a.D + 1 : a.geo.ww * a.geo.ws + 1;
}
__device__ __forceinline__ int w1_role_row(const AdamStep& a, int v) {
  if (a.wchunk < 0) return v;
  const int nv = a.geo.ww * a.geo.ws;
  if (v == nv) return a.wchunk == a.geo.wp - 1 ? a.D : -1;
  return wire_chunk_row(a.geo, a.wchunk, v, a.D);
}
__device__ __forceinline__ RowEntries row_entries(const AdamStep& a, int s, int e) {
  RowEntries r{0, 0.f};
  const int lane = lane_id();
  if (e - s <= kLightEntries && lane < e - s) {
    r.i = a.csc_row[s + lane];
    r.v = a.csc_val[s + lane];
  }
  return r;
}

// gradient pass: where W1 row c's bf16 gradient goes -- this rank's gradient wire, or (peer exchange,
// one wire chunk) the block of this rank in the stage of the row's owner j = c / geo.ws
__device__ __forceinline__ u16* grad_row(const AdamStep& a, int c) {
  if (a.npeer) return a.gpeer[c / a.geo.ws] + wire_row_off(a.geo, c);
  return a.gout + wire_row_off(a.geo, c);
}

template <typename TZ, bool WIRE>
__device__ __forceinline__ void w1_row(const AdamStep& a, int c, int s, int e, float alpha,
                                       const RowEntries* pre = nullptr) {
  const int lane = lane_id();
  const int n = a.n;
  const bool heavy = e - s > kLightEntries;
  if (heavy && a.item_blocks) return;  // updated by the heavy-item workgroups
  if (e == s && a.w1_flat) return;  // untouched: the flat roles' pass
  const TZ* dZ = static_cast<const TZ*>(a.dZ);
  for (int c0 = 0; c0 < n; c0 += 512) {
    const int cc = c0 + lane * 8;
    const int nvalid = n - cc;
    const size_t o = (size_t)c * n + cc;
    float P[8], M[8], V[8], G[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#if !DSSM_ADAM_LATE_PMV
    if (nvalid > 0 && !(WIRE && a.gout)) {  // stream loads first: independent of the gather chain below
      ld_stream8(a.p + o, nvalid, P);
      ld_stream8(a.m + o, nvalid, M);
      ld_stream8(a.v + o, nvalid, V);
    }
#endif
    if (heavy) {
      if (nvalid > 0) {
        load8(a.g + o, nvalid, G);
        *reinterpret_cast<float4*>(a.g + o) = make_float4(0.f, 0.f, 0.f, 0.f);
        if (nvalid > 4) *reinterpret_cast<float4*>(a.g + o + 4) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {
      if (pre) gather_batch<TZ, 2, DSSM_ADAM_GATHER_U>(pre->i, pre->v, e - s, dZ, a.lddz, cc, nvalid, G);
      else gather_accumulate<TZ, 2>(a.csc_row, a.csc_val, s, e, dZ, a.lddz, cc, nvalid, G);
    }
#if DSSM_ADAM_LATE_PMV
    if (nvalid > 0 && !a.gout) {  // after the gather: fewer live registers, higher occupancy
      ld_stream8(a.p + o, nvalid, P);
      ld_stream8(a.m + o, nvalid, M);
      ld_stream8(a.v + o, nvalid, V);
    }
#endif
    if (WIRE && nvalid > 0 && a.gout) {  // gradient pass: the row leaves as bf16 (bias row: fp32)
      const int k = nvalid >= 8 ? 8 : 4;
      if (c < a.D) {
        u16* q = grad_row(a, c) + cc;
        uint2 lo;
        lo.x = pack2bf(G[0], G[1]);
        lo.y = pack2bf(G[2], G[3]);
        uint2 hi;
        hi.x = pack2bf(G[4], G[5]);
        hi.y = pack2bf(G[6], G[7]);
        if (a.npeer) {  // peer exchange: into the owner's stage (launch.h st_sys8)
          st_sys8(q, lo);
          if (k == 8) st_sys8(q + 4, hi);
        } else {
          *reinterpret_cast<uint2*>(q) = lo;
          if (k == 8) *reinterpret_cast<uint2*>(q + 4) = hi;
        }
      } else {
        *reinterpret_cast<float4*>(a.g + o) = make_float4(G[0], G[1], G[2], G[3]);
        if (k == 8) *reinterpret_cast<float4*>(a.g + o + 4) = make_float4(G[4], G[5], G[6], G[7]);
      }
    } else if (nvalid > 0) {
      const int k = nvalid >= 8 ? 8 : 4;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (i < k) adam1(P[i], M[i], V[i], G[i] * a.gs, alpha, a.b1c, a.b2c, a.eps);
      st_stream4(a.p + o, make_float4(P[0], P[1], P[2], P[3]));
      st_stream4(a.m + o, make_float4(M[0], M[1], M[2], M[3]));
      st_stream4(a.v + o, make_float4(V[0], V[1], V[2], V[3]));
      if (k == 8) {
        st_stream4(a.p + o + 4, make_float4(P[4], P[5], P[6], P[7]));
        st_stream4(a.m + o + 4, make_float4(M[4], M[5], M[6], M[7]));
        st_stream4(a.v + o + 4, make_float4(V[4], V[5], V[6], V[7]));
      }
      if (a.shadow && c < a.D) {
        u16* q = a.shadow + (size_t)c * a.ldsh + cc;
        uint2 lo;
        lo.x = pack2bf(P[0], P[1]);
        lo.y = pack2bf(P[2], P[3]);
        *reinterpret_cast<uint2*>(q) = lo;
        if (k == 8) {
          uint2 hi;
          hi.x = pack2bf(P[4], P[5]);
          hi.y = pack2bf(P[6], P[7]);
          *reinterpret_cast<uint2*>(q + 4) = hi;
        }
      }
    }
  }
}

// Adam over one W1 row c whose gradient row sits in LDS (heavy-item workgroups).
template <bool WIRE>
__device__ __forceinline__ void w1_row_from(const AdamStep& a, int c, const float* grow, float alpha) {
  if (WIRE && a.gout && a.npeer && c < a.D) {  // peer exchange: 4-B stores into the owner's stage
    unsigned* q = reinterpret_cast<unsigned*>(grad_row(a, c));
    for (int j = threadIdx.x; j < a.n / 2; j += blockDim.x) st_sys4(q + j, pack2bf(grow[2 * j], grow[2 * j + 1]));
    return;
  }
  if (WIRE && a.gout) {  // gradient pass
    const int64_t wo = c < a.D ? wire_row_off(a.geo, c) : 0;
    for (int j = threadIdx.x; j < a.n; j += blockDim.x) {
      if (c < a.D) a.gout[wo + j] = f2bf(grow[j]);
      else a.g[(size_t)c * a.n + j] = grow[j];
    }
    return;
  }
  for (int j = threadIdx.x; j < a.n; j += blockDim.x) {
    const size_t o = (size_t)c * a.n + j;
    float P = a.p[o], M = a.m[o], V = a.v[o];
    adam1(P, M, V, grow[j] * a.gs, alpha, a.b1c, a.b2c, a.eps);
    a.p[o] = P;
    a.m[o] = M;
    a.v[o] = V;
    if (a.shadow && c < a.D) a.shadow[(size_t)c * a.ldsh + j] = f2bf(P);
  }
}

// Heavy W1 columns (> kLightEntries entries, the ones column included) inside the step: each
// work item {column, k} is kHeavyItem CSC entries, 64 per wave, the 4 partial rows summed in LDS.
// A one-item column is updated right here; a longer column's items add their rows to the
// gradient arena with fp32 atomics and arrive on the column's ticket: the last arrival takes
// the row with atomic exchanges (read and clear at the coherence point), updates it and
// re-arms the ticket.  Deterministic mode (heavy_slab): the items store their rows into the slab
// instead (write-through stores drained before the ticket, sc1 loads by the last arrival) and the last arrival sums
// them in item order, so the fp32 sum no longer depends on arrival order.
// LDS of one heavy-item workgroup: the 4 waves' partial rows, the summed row, the last-arrival flag
struct HeavyLds {
  float part[4][512];
  float grow[512];
  int last;
};

template <typename TZ, bool WIRE>
__device__ __forceinline__ void heavy_items(const AdamStep& a, float alpha, int hb, HeavyLds& L) {
  float(&part)[4][512] = L.part;
  float(&grow)[512] = L.grow;
  int& s_last = L.last;
  const int wv = threadIdx.x >> 6, lane = lane_id();
  const TZ* dZ = static_cast<const TZ*>(a.dZ);
  const int nitems = *a.heavy_n;
  for (int it = hb; it < nitems; it += a.item_blocks) {
    const int2 item = a.heavy_items[it];
    const int c = item.x;
    if constexpr (WIRE)
      if (!in_chunk(a, c)) continue;  // uniform over the workgroup
    const int cs = a.col_ptr[c], ce = a.col_ptr[c + 1];
    const int i0 = cs + item.y * kHeavyItem;
    const int s = min(ce, i0 + wv * (kHeavyItem / 4)), e = min(ce, s + kHeavyItem / 4);
    const int nit = (ce - cs + kHeavyItem - 1) / kHeavyItem;
    for (int c0 = 0; c0 < a.n; c0 += 512) {
      const int cc = c0 + lane * 8;
      const int nvalid = a.n - cc;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (s < e) gather_accumulate<TZ, 2, DSSM_ADAM_HEAVY_U>(a.csc_row, a.csc_val, s, e, dZ, a.lddz, cc, nvalid, acc);
#pragma unroll
      for (int i = 0; i < 8; ++i) part[wv][lane * 8 + i] = acc[i];
      __syncthreads();
      const int m = min(512, a.n - c0);
      for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const float v = part[0][i] + part[1][i] + part[2][i] + part[3][i];
        if (nit == 1) grow[c0 + i] = v;
        else if (a.heavy_slab)
          __hip_atomic_store(a.heavy_slab + (size_t)it * a.n + c0 + i, v, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        else atomicAdd(a.g + (size_t)c * a.n + c0 + i, v);
      }
      __syncthreads();
    }
    if (nit == 1) {
      w1_row_from<WIRE>(a, c, grow, alpha);
    } else {
      // Deterministic mode: the slab rows are write-through stores drained before this workgroup's
      // arrival and the last arrival reads them with sc1 loads (common.h last_block_arrival_wt).  Atomics mode: every access to the
      // column's row is a device-scope atomic performed at the coherence point, so the drained adds
      // need no L2 write-back (an agent-scope release here writes back the XCD's L2 per item:
      // measured +20 us on the Adam launch).
      bool last;
      if (a.heavy_slab) {
        last = last_block_arrival_wt(a.heavy_ticket + c, (unsigned)nit, &s_last);
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's adds performed
        __syncthreads();
        if (threadIdx.x == 0) {
          const unsigned t = __hip_atomic_fetch_add(a.heavy_ticket + c, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
          s_last = t == (unsigned)nit - 1;
          if (s_last) __hip_atomic_store(a.heavy_ticket + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        last = s_last != 0;
      }
      if (last) {
        if (a.heavy_slab) {
          const float* sl = a.heavy_slab + (size_t)(it - item.y) * a.n;
          for (int j = threadIdx.x; j < a.n; j += blockDim.x) {
            float acc = 0.f;
            for (int k = 0; k < nit; ++k)
              acc += __hip_atomic_load(sl + (size_t)k * a.n + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            grow[j] = acc;
          }
        } else {
          for (int j = threadIdx.x; j < a.n; j += blockDim.x)
            grow[j] = __hip_atomic_exchange(a.g + (size_t)c * a.n + j, 0.f, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        w1_row_from<WIRE>(a, c, grow, alpha);
      }
    }
    __syncthreads();
  }
}

// one LDS block shared by the two roles that use LDS (the hosted rank role's hash table, the heavy
// items' rows): 16.4 instead of 26.6 KB per workgroup, so LDS no longer caps the launch at 6
// workgroups per CU
constexpr size_t kAdamLdsBytes = sizeof(unsigned) * kRankHash > sizeof(HeavyLds) ? sizeof(unsigned) * kRankHash
                                                                                 : sizeof(HeavyLds);

// The whole optimizer step in one launch (k_adam_step's body, run as workgroup blk of nblk):
// blocks [0, w1_blocks) run the fused W1 rows (grid-stride over rows, one wave per row), the
// others stream the dense float4 range.  Every block
// reads the beta powers at its start; the last block to finish (relaxed agent-scope tickets: it
// only needs every other block to have READ them, which precedes their arrival) advances them
// (TF1.x AdamOptimizer._finish: beta1_power *= beta1, beta2_power *= beta2, fp32) and re-arms
// the ticket.
// WIRE: the data-parallel variants (gradient pass, chunked rows, bf16 wire / stage in the dense
// range); the single-GPU step compiles without them (their row remapping and per-element wire tests
// in the W1 and streaming loops cost the fused step 16 us: 57.5 -> 75 us measured)
template <typename TZ, bool WIRE>
__device__ __forceinline__ void adam_step_body(const AdamStep& a, const int blk, const unsigned nblk,
                                               unsigned char* s_lds) {
  ADAM_TL(0);
  const float b1p = a.st[0], b2p = a.st[1];
  const float alpha = a.lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
  // Block roles in dispatch order: the heavy-item blocks (the longest dependent chains) first,
  // then the W1-row gather blocks, then the flat/dense streaming blocks.  (Interleaving the
  // gathers with the streaming was measured slower: the heavy chains start late, 61 -> 86 us.)
  const int nr = a.rank.nblocks;
  // where the hosted rank workgroups sit in dispatch order (build knob DSSM_RANK_POS): 1 (default)
  // last, after the streaming blocks; 0 first; 2 right after the heavy items
#if DSSM_RANK_POS == 0
  const int rs = 0;
#elif DSSM_RANK_POS == 1
  const int rs = (int)nblk - nr;
#else
  const int rs = a.item_blocks;
#endif
  const int bx = blk;
  const bool is_rank = bx >= rs && bx < rs + nr;
  const int b0 = bx < rs ? bx : bx - nr;
  const int nh = a.item_blocks, nw = a.w1_blocks, nd = a.dense_blocks;
  // role order after the heavy items: W1 rows then streaming (0), or streaming first (1)
  const bool w1_role = DSSM_ADAM_ORDER == 0 ? (b0 >= nh && b0 < nh + nw) : (b0 >= nh + nd);
  if (is_rank) {
    csc_rank_role(a.rank, bx - rs, reinterpret_cast<unsigned*>(s_lds));
  } else if (b0 < nh) {
    heavy_items<TZ, WIRE>(a, alpha, b0, *reinterpret_cast<HeavyLds*>(s_lds));
  } else if (w1_role) {
    const int b = DSSM_ADAM_ORDER == 0 ? b0 - nh : b0 - nh - nd;
    // the next row's column range is loaded while this row is processed (one dependent load
    // fewer on each row's chain)
    const int stride = a.w1_blocks * 4;
    if constexpr (!WIRE) {
      // every row [0, D]; c stays wave-uniform (scalar row state: a lane-varying form of this loop,
      // a row-slot remapping through a lambda, measured 57.5 -> 75 us)
      int c = b * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      int s = 0, e = 0;
      if (c <= a.D) {
        s = a.col_ptr[c];
        e = a.col_ptr[c + 1];
      }
#if DSSM_ADAM_PRE_IDX
      // two rows ahead: the column range; one row ahead: the light row's CSC entries
      int sn = 0, en = 0;
      if (c + stride <= a.D) {
        sn = a.col_ptr[c + stride];
        en = a.col_ptr[c + stride + 1];
      }
      RowEntries ent = row_entries(a, s, e);
      for (; c <= a.D; c += stride) {
        const int c2 = c + 2 * stride;
        int s2 = 0, e2 = 0;
        if (c2 <= a.D) {
          s2 = a.col_ptr[c2];
          e2 = a.col_ptr[c2 + 1];
        }
        const RowEntries next = row_entries(a, sn, en);
        w1_row<TZ, false>(a, c, s, e, alpha, &ent);
        s = sn;
        e = en;
        sn = s2;
        en = e2;
        ent = next;
      }
#else
      for (; c <= a.D; c += stride) {
        const int cn = c + stride;
        int sn = 0, en = 0;
        if (cn <= a.D) {
          sn = a.col_ptr[cn];
          en = a.col_ptr[cn + 1];
        }
        w1_row<TZ, false>(a, c, s, e, alpha);
        s = sn;
        e = en;
      }
#endif
    } else {
      // rows by slot v: every row, or one wire chunk's rows (w1_role_row); wave-uniform
      const int nv = w1_role_rows(a);
      int v = b * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      auto range = [&](int vv, int& rs, int& re) {
        const int c = __builtin_amdgcn_readfirstlane(vv < nv ? w1_role_row(a, vv) : -1);
        rs = re = 0;
        if (c >= 0) {
          rs = a.col_ptr[c];
          re = a.col_ptr[c + 1];
        }
        return c;
      };
      int s, e;
      int c = range(v, s, e);
      int sn, en;
      int cn = range(v + stride, sn, en);
      for (; v < nv; v += stride) {
        if (c >= 0) w1_row<TZ, true>(a, c, s, e, alpha);
        c = cn;
        s = sn;
        e = en;
        cn = range(v + 2 * stride, sn, en);
      }
    }
  } else {
    const int bi = DSSM_ADAM_ORDER == 0 ? b0 - nh - nw : b0 - nh;
    if (WIRE && a.w1_flat && a.gout) {  // gradient pass: an untouched row's gradient is zero
      const int nv = w1_role_rows(a) - 1;  // W1 rows only (b1's row is never untouched)
      const int q = a.n / 4;
      const int64_t w4 = (int64_t)nv * q;
      for (int64_t i = (int64_t)bi * blockDim.x + threadIdx.x; i < w4;
           i += (int64_t)a.dense_blocks * blockDim.x) {
        const int vr = (int)(i / q);
        const int c = w1_role_row(a, vr);
        if (c < 0 || c >= a.D || a.col_ptr[c + 1] != a.col_ptr[c]) continue;
        uint2* z = reinterpret_cast<uint2*>(grad_row(a, c)) + (i - (int64_t)vr * q);
        if (a.npeer) st_sys8(z, make_uint2(0u, 0u));
        else *z = make_uint2(0u, 0u);
      }
    } else if (a.w1_flat) {
      // untouched W1 rows (no CSC entry, g = 0): float4 streaming, every lane busy
      FlatSlice f{a.p, a.m, a.v, a.shadow, a.ldsh, a.n, a.D, a.col_ptr, a.st, a.lr, a.b1c, a.b2c, a.eps,
                  0, (int64_t)(a.D + 1) * a.n / 4, a.dense_blocks};
#ifndef DSSM_ADAM_SKIP_UNTOUCHED  // diagnostics build: the untouched rows' cost (wrong results)
      flat_untouched(f, bi);
#endif
    }
    const int64_t na = a.d4_end - a.d4_begin, nt = a.t4_end - a.t4_begin;
    if (WIRE && a.slab_to_g) {  // gradient pass: g = the deferred split-K slabs' sums (fixed order)
      for (int64_t j = (int64_t)bi * blockDim.x + threadIdx.x; j < nt; j += (int64_t)a.dense_blocks * blockDim.x) {
        const int64_t i = a.t4_begin + j;
        if (in_slabs(a.slabs, i * 4))
          reinterpret_cast<float4*>(a.g)[i] = slab_grad4(a.slabs, i * 4, a.g);
      }
    } else
    for (int64_t j = (int64_t)bi * blockDim.x + threadIdx.x; j < na + nt;
         j += (int64_t)a.dense_blocks * blockDim.x) {
      const int64_t i = j < na ? a.d4_begin + j : a.t4_begin + (j - na);
      const bool wired = WIRE && i < a.wire4;
      float4 pp = ld_stream4(a.p + i * 4);
      float4 gg;
      if (WIRE && wired && a.gstage) {
        // one bf16 rounding per rank's gradient, the sum over ranks in fp32 (fixed rank order)
        gg = make_float4(0.f, 0.f, 0.f, 0.f);
        const uint2* st = reinterpret_cast<const uint2*>(a.gstage) + (i - a.gbase4);
        for (int k = 0; k < a.gparts; ++k) {
          const uint2 q = a.npeer ? ld_sys8(st + (int64_t)k * (a.gstride / 4)) : st[(int64_t)k * (a.gstride / 4)];
          gg.x += __uint_as_float(q.x << 16);
          gg.y += __uint_as_float(q.x & 0xffff0000u);
          gg.z += __uint_as_float(q.y << 16);
          gg.w += __uint_as_float(q.y & 0xffff0000u);
        }
      } else if (WIRE && wired) {
        const uint2 q = reinterpret_cast<const uint2*>(a.gwire)[i];
        gg = make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                         __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u));
      } else if (WIRE && a.ptail) {  // peer exchange: the world's tail partials, rank order
        const float* t = a.ptail + (i * 4 - a.tail0);
        uint2 lo = ld_sys8(t), hi = ld_sys8(t + 2);
        gg = make_float4(__uint_as_float(lo.x), __uint_as_float(lo.y), __uint_as_float(hi.x), __uint_as_float(hi.y));
        for (int k = 1; k < a.npeer; ++k) {
          lo = ld_sys8(t + k * a.tailn);
          hi = ld_sys8(t + k * a.tailn + 2);
          gg.x += __uint_as_float(lo.x);
          gg.y += __uint_as_float(lo.y);
          gg.z += __uint_as_float(hi.x);
          gg.w += __uint_as_float(hi.y);
        }
      } else {
        gg = slab_grad4(a.slabs, i * 4, a.g);
      }
      float4 mm = ld_stream4(a.m + i * 4);
      float4 vv = ld_stream4(a.v + i * 4);
      adam1(pp.x, mm.x, vv.x, gg.x * a.gs, alpha, a.b1c, a.b2c, a.eps);
      adam1(pp.y, mm.y, vv.y, gg.y * a.gs, alpha, a.b1c, a.b2c, a.eps);
      adam1(pp.z, mm.z, vv.z, gg.z * a.gs, alpha, a.b1c, a.b2c, a.eps);
      adam1(pp.w, mm.w, vv.w, gg.w * a.gs, alpha, a.b1c, a.b2c, a.eps);
      st_stream4(a.p + i * 4, pp);
      st_stream4(a.m + i * 4, mm);
      st_stream4(a.v + i * 4, vv);
      if (i * 4 >= a.clear_from)
        reinterpret_cast<float4*>(a.g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (WIRE && wired) {
        uint2 q;
        q.x = pack2bf(pp.x, pp.y);
        q.y = pack2bf(pp.z, pp.w);
        if (a.npeer) {
          for (int k = 0; k < a.npeer; ++k) st_sys8(reinterpret_cast<uint2*>(a.ppeer[k]) + (i + a.pwire_off4), q);
        } else {
          reinterpret_cast<uint2*>(a.pwire)[i + a.pwire_off4] = q;
        }
      } else if (a.sh.count) {
        write_shadow4(a.sh, i * 4, pp);
      }
    }
  }
#ifdef DSSM_WG_TL
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  __syncthreads();
  ADAM_TL(1);
  if (threadIdx.x == 0 && a.ticket) {
    // Two-level ticket: same-address atomics serialise (~6 ns each; one counter for ~8k blocks
    // measured +45 us), so blocks arrive on kAdamSubTickets counters 256 B apart and only the
    // last arrival of each moves the top counter.
    const unsigned k = (unsigned)blk % kAdamSubTickets;
    const unsigned nk = nblk / kAdamSubTickets + (k < nblk % kAdamSubTickets ? 1u : 0u);
    unsigned* sub = a.ticket + 64 * (k + 1);
    const unsigned t = __hip_atomic_fetch_add(sub, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == nk - 1) {
      __hip_atomic_store(sub, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned ntop = min(nblk, (unsigned)kAdamSubTickets);
      const unsigned u =
          __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (u == ntop - 1) {
        if (a.heavy_reset) *a.heavy_reset = 0;
        __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // a step of group_n launches (possibly concurrent, on other streams): the last launch to
        // finish advances (each launch's blocks have read the powers before they arrived)
        bool adv = true;
        if (a.group_ticket) {
          const unsigned g =
              __hip_atomic_fetch_add(a.group_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          adv = g == (unsigned)a.group_n - 1;
          if (adv) __hip_atomic_store(a.group_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (adv) {
          a.st[0] = b1p * a.beta1;
          a.st[1] = b2p * a.beta2;
        }
      }
    }
  }
}

template <typename TZ, bool WIRE>
__global__ __launch_bounds__(256) DSSM_ADAM_ATTR void k_adam_step(AdamStep a) {
  __shared__ __align__(16) unsigned char s_lds[kAdamLdsBytes];
  adam_step_body<TZ, WIRE>(a, blockIdx.x, gridDim.x, s_lds);
}

__global__ __launch_bounds__(256) void k_shadow_sync(const float* __restrict__ p, ShadowSeg g) {
  const int64_t n4 = g.rows * g.cols / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t rel = i * 4;
    const int64_t r = rel / g.cols;
    const int c = (int)(rel - r * g.cols);
    const float4 v = *reinterpret_cast<const float4*>(p + g.offset + rel);
    uint2 q;
    q.x = pack2bf(v.x, v.y);
    q.y = pack2bf(v.z, v.w);
    *reinterpret_cast<uint2*>(g.ptr + r * g.ld + c) = q;
    if (g.tptr) {
      g.tptr[(int64_t)(c + 0) * g.tld + r] = f2bf(v.x);
      g.tptr[(int64_t)(c + 1) * g.tld + r] = f2bf(v.y);
      g.tptr[(int64_t)(c + 2) * g.tld + r] = f2bf(v.z);
      g.tptr[(int64_t)(c + 3) * g.tld + r] = f2bf(v.w);
    }
  }
}

// The functional optimizer step with bf16 shadows (dssm_adam_step_shadow: the multi-view model's bf16
// mode): ApplyAdam over n4 float4 groups of a flat range, each updated weight also written as bf16 to
// its block's shadow, so no separate refresh pass re-reads the parameters.  The range is < 2^31
// elements (launcher), so a group's (row, column) in its block comes from 32-bit division (the
// 64-bit form of write_shadow4 is a long software sequence per group: 43 -> 51 us measured).
// One shadow segment's geometry held in registers across the grid-stride loop.
struct Seg32 {
  int off, end, cols, ld;
  u16* ptr;
};
__device__ __forceinline__ void put_shadow4(const Seg32& g, int i, float4 v) {
  const int rel = i - g.off;
  const int r = rel / g.cols, c = rel - r * g.cols;
  uint2 p;
  p.x = pack2bf(v.x, v.y);
  p.y = pack2bf(v.z, v.w);
  *reinterpret_cast<uint2*>(g.ptr + (size_t)r * g.ld + c) = p;
}
__global__ __launch_bounds__(256) void k_adam_flat_shadow(float* __restrict__ p, const float* __restrict__ g,
                                                          float* __restrict__ m, float* __restrict__ v,
                                                          AdamRanges rg, const float* __restrict__ st, float lr,
                                                          float b1c, float b2c, float eps, float gs, ShadowList sh) {
  const float alpha = lr * sqrtf(1.0f - st[1]) / (1.0f - st[0]);
  // at most four segments (a tower's [W1; b1] and [W2; b2] blocks, two towers), geometry in registers
  Seg32 s4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    s4[k] = k < sh.count ? Seg32{(int)sh.seg[k].offset, (int)(sh.seg[k].offset + sh.seg[k].rows * sh.seg[k].cols),
                                 sh.seg[k].cols, sh.seg[k].ld, sh.seg[k].ptr}
                         : Seg32{0, 0, 1, 0, nullptr};
  const int64_t n0 = rg.n4[0], nt = rg.n4[0] + rg.n4[1];
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nt; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = j < n0 ? rg.b4[0] + j : rg.b4[1] + (j - n0);
    float4 pp = ld_stream4(p + i * 4);
    const float4 gg = *reinterpret_cast<const float4*>(g + i * 4);
    float4 mm = ld_stream4(m + i * 4);
    float4 vv = ld_stream4(v + i * 4);
    adam1(pp.x, mm.x, vv.x, gg.x * gs, alpha, b1c, b2c, eps);
    adam1(pp.y, mm.y, vv.y, gg.y * gs, alpha, b1c, b2c, eps);
    adam1(pp.z, mm.z, vv.z, gg.z * gs, alpha, b1c, b2c, eps);
    adam1(pp.w, mm.w, vv.w, gg.w * gs, alpha, b1c, b2c, eps);
    st_stream4(p + i * 4, pp);
    st_stream4(m + i * 4, mm);
    st_stream4(v + i * 4, vv);
    const int e = (int)(i * 4);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (e >= s4[k].off && e < s4[k].end) {
        put_shadow4(s4[k], e, pp);
        break;
      }
  }
}

// the wire's W1 rows from the materialised fp32 gradient (one 4-element group per thread)
__global__ __launch_bounds__(256) void k_wire_pack(const float* __restrict__ g, u16* __restrict__ w,
                                                   int D, WireGeo geo) {
  const int q = geo.n / 4;
  const int64_t n4 = (int64_t)D * q;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / q);
    const float4 v = reinterpret_cast<const float4*>(g)[i];
    uint2 o;
    o.x = pack2bf(v.x, v.y);
    o.y = pack2bf(v.z, v.w);
    reinterpret_cast<uint2*>(w + wire_row_off(geo, r))[i - (int64_t)r * q] = o;
  }
}

// W1 shadow rows [rows x ld] from the bf16 parameter wire (row length g.cols == geo.n; W1 at
// arena offset 0): every row, or one chunk's rows; one 4-element group per thread
__global__ __launch_bounds__(256) void k_wire_shadow(const u16* __restrict__ w, ShadowSeg g, WireGeo geo,
                                                     int chunk) {
  const int q = g.cols / 4;
  const int nrows = chunk < 0 ? (int)g.rows : geo.ww * geo.ws;
  const int64_t n4 = (int64_t)nrows * q;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int v = (int)(i / q);
    const int r = chunk < 0 ? v : wire_chunk_row(geo, chunk, v, (int)g.rows);
    if (r < 0) continue;
    const int c = (int)(i - (int64_t)v * q) * 4;
    *reinterpret_cast<uint2*>(g.ptr + (int64_t)r * g.ld + c) =
        *reinterpret_cast<const uint2*>(w + wire_row_off(geo, r) + c);
  }
}

// the data-parallel rehearsal's modelled collective: one wave holds the stream for `ticks` of the
// 100 MHz real-time counter
__global__ void k_spin(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
}

int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

int grid_for(int64_t n4) {
  const int64_t g = (n4 + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

// the launch geometry of one step (block counts by role), checked
static hipError_t prepare_adam_step(AdamStep& a) {
  if ((a.d4_begin < 0) || (a.d4_end < a.d4_begin)) return hipErrorInvalidValue;
  a.b1c = 1.0f - a.beta1;
  a.b2c = 1.0f - a.beta2;
  // 2048 W1-row gather blocks: measured against 1024 / 4096 (+2-4 us each)
  const int w1_rows = a.wchunk < 0 ? a.D + 1 : a.geo.ww * a.geo.ws + 1;
  if (a.w1_blocks > 0) a.w1_blocks = std::min(cdiv(w1_rows, 4), kAdamW1Blocks);
  if (a.gout || a.no_advance) a.ticket = nullptr;  // the gradient pass / a non-final chunk advance nothing
  if (!a.ticket && !a.gout && !a.no_advance) return hipErrorInvalidValue;  // a step advances the beta powers
  if (a.group_ticket && (!a.ticket || a.group_n < 1)) return hipErrorInvalidValue;
  if (a.wchunk >= 0 && (!a.gout || !a.geo.ww || a.wchunk >= a.geo.wp)) return hipErrorInvalidValue;
  if (a.slab_to_g && (!a.gout || a.d4_end != a.d4_begin)) return hipErrorInvalidValue;  // gradient pass only
  if (a.w1_blocks == 0 || !a.heavy_items) a.item_blocks = 0;
  else a.item_blocks = std::min(a.item_blocks, kAdamItemBlocks);
  // rows with no entry this step stream through the flat role instead of a wave per row
  a.w1_flat = (a.w1_blocks > 0 && a.item_blocks > 0 && (a.n % 4) == 0) ? 1 : 0;
  if (a.t4_end < a.t4_begin || (a.wire4 > 0 && (!a.gwire || !a.pwire))) return hipErrorInvalidValue;
  if (a.npeer < 0 || a.npeer > kPeerMax) return hipErrorInvalidValue;
  if (a.npeer && a.gout && (a.geo.wp != 1 || a.geo.ww != a.npeer || (a.n % 2))) return hipErrorInvalidValue;
  for (int k = 0; k < a.npeer; ++k)
    if ((a.gout && !a.gpeer[k]) || (!a.gout && !a.ppeer[k])) return hipErrorInvalidValue;
  if (a.ptail && (!a.npeer || a.gout || a.tailn < 4 * (a.t4_end - a.t4_begin) || a.tail0 != 4 * a.t4_begin))
    return hipErrorInvalidValue;
  const int64_t flat_rows = a.wchunk < 0 ? (int64_t)a.D + 1 : (int64_t)a.geo.ww * a.geo.ws;
#ifdef DSSM_ADAM_SKIP_UNTOUCHED
  const int64_t n4 = a.d4_end - a.d4_begin + (a.t4_end - a.t4_begin) + 0 * flat_rows;
#else
  const int64_t n4 = a.d4_end - a.d4_begin + (a.t4_end - a.t4_begin) + (a.w1_flat ? flat_rows * a.n / 4 : 0);
#endif
  a.dense_blocks = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(n4, 256), kAdamDenseBlocks));
  if (a.rank.nblocks && !a.ticket) return hipErrorInvalidValue;  // the hosted rank needs a whole step
  return hipSuccess;
}

hipError_t launch_adam_step(AdamStep a, bool dz_bf16, hipStream_t s) {
  const hipError_t pe = prepare_adam_step(a);
  if (pe != hipSuccess) return pe;
  dim3 grid(a.rank.nblocks + a.item_blocks + a.w1_blocks + a.dense_blocks), block(256);
  const bool wire = a.gout || a.wchunk >= 0 || a.wire4 > 0 || a.gstage || a.gwire || a.pwire || a.slab_to_g ||
                    a.npeer;
#define DSSM_ADAM_LAUNCH(TZ)                                                         \
  if (wire) hipLaunchKernelGGL((k_adam_step<TZ, true>), grid, block, 0, s, a);       \
  else hipLaunchKernelGGL((k_adam_step<TZ, false>), grid, block, 0, s, a)
  if (dz_bf16) {
    DSSM_ADAM_LAUNCH(u16);
  } else {
    DSSM_ADAM_LAUNCH(float);
  }
#undef DSSM_ADAM_LAUNCH
  return hipGetLastError();
}

hipError_t launch_wire_pack(const float* g, uint16_t* wire, int D, WireGeo geo, hipStream_t s) {
  if (geo.n % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_wire_pack, dim3(grid_for((int64_t)D * geo.n / 4)), dim3(256), 0, s, g, wire, D, geo);
  return hipGetLastError();
}

hipError_t launch_wire_shadow(const uint16_t* wire, ShadowSeg seg, WireGeo geo, int chunk, hipStream_t s) {
  if (seg.cols % 4 || seg.cols != geo.n || (chunk >= 0 && (!geo.ww || chunk >= geo.wp)))
    return hipErrorInvalidValue;
  const int64_t rows = chunk < 0 ? seg.rows : (int64_t)geo.ww * geo.ws;
  hipLaunchKernelGGL(k_wire_shadow, dim3(grid_for(rows * seg.cols / 4)), dim3(256), 0, s, wire, seg, geo, chunk);
  return hipGetLastError();
}

// Device-to-device copy as a kernel node (the data-parallel graphs' own-chunk all-to-all copy and the
// copy rehearsal): ordered like every other kernel of the captured stream.  16-B lanes when both
// pointers and the size allow it, else 4-B, else bytes.
__global__ __launch_bounds__(256) void k_copy_bytes(void* __restrict__ dst, const void* __restrict__ src,
                                                    size_t bytes, int width) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (width == 16) {
    for (size_t i = t; i < bytes / 16; i += stride)
      static_cast<uint4*>(dst)[i] = static_cast<const uint4*>(src)[i];
  } else if (width == 4) {
    for (size_t i = t; i < bytes / 4; i += stride)
      static_cast<unsigned*>(dst)[i] = static_cast<const unsigned*>(src)[i];
  } else {
    for (size_t i = t; i < bytes; i += stride)
      static_cast<unsigned char*>(dst)[i] = static_cast<const unsigned char*>(src)[i];
  }
}

hipError_t launch_copy_bytes(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (!bytes) return hipSuccess;
  const uintptr_t a = (uintptr_t)dst | (uintptr_t)src | (uintptr_t)bytes;
  const int width = (a % 16 == 0) ? 16 : (a % 4 == 0) ? 4 : 1;
  const size_t items = bytes / width;
  const int grid = (int)std::max<size_t>(1, std::min<size_t>((items + 255) / 256, 2048));
  hipLaunchKernelGGL(k_copy_bytes, dim3(grid), dim3(256), 0, s, dst, src, bytes, width);
  return hipGetLastError();
}

hipError_t launch_adam_flat_shadow(float* p, const float* g, float* m, float* v, AdamRanges rg, const float* st,
                                  float lr, float beta1, float beta2, float eps, float gs, ShadowList sh,
                                  hipStream_t s) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 || sh.count > 4 || rg.nr < 1 || rg.nr > 2)
    return hipErrorInvalidValue;
  if (rg.nr == 1) rg.n4[1] = 0;
  for (int k = 0; k < rg.nr; ++k)
    if (rg.b4[k] < 0 || rg.n4[k] < 0 || (rg.b4[k] + rg.n4[k]) * 4 >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  for (int i = 0; i < sh.count; ++i)
    if (sh.seg[i].offset % 4 || sh.seg[i].cols % 4 || sh.seg[i].ld % 4 || sh.seg[i].tptr ||
        sh.seg[i].offset + sh.seg[i].rows * sh.seg[i].cols >= ((int64_t)1 << 31))
      return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_adam_flat_shadow, dim3(grid_for(rg.n4[0] + rg.n4[1])), dim3(256), 0, s, p, g, m, v, rg, st,
                     lr, 1.0f - beta1, 1.0f - beta2, eps, gs, sh);
  return hipGetLastError();
}

hipError_t launch_spin(double ns, hipStream_t s) {
  const unsigned long long ticks = ns > 0 ? (unsigned long long)(ns / 10.0 + 0.5) : 0ull;
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, ticks);
  return hipGetLastError();
}

hipError_t launch_shadow_sync(const float* p, ShadowList sh, hipStream_t s) {
  for (int i = 0; i < sh.count; ++i) {
    const int64_t n4 = sh.seg[i].rows * sh.seg[i].cols / 4;
    hipLaunchKernelGGL(k_shadow_sync, dim3(grid_for(n4)), dim3(256), 0, s, p, sh.seg[i]);
  }
  return hipGetLastError();
}

}  // namespace dssm

#ifdef DSSM_WG_TL
extern "C" int dssm_debug_adam_timeline(unsigned long long* out, int n) {
  if (n > 8192) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dssm::g_adam_tl), sizeof(unsigned long long) * 2 * n, 0) ==
                 hipSuccess ? 0 : -2;
}
#endif
