// Level-synchronous Boruvka fragment contraction on gfx950 — the MI355X restatement of the
// reference's GHS level loop. One Boruvka round here == one GHS level of the reference:
//
//   reference (thread / MPI path)                               this file
//   test/handle_test/accept/reject/report/handle_report         k_minedge: every fragment's minimum
//     ghs_implementation.py:235-353, _mpi.py:353-580              outgoing edge, key (w, eid)
//   REJECT marks an intra-fragment edge (:271-301, _mpi:429-491) k_minedge drops arcs whose ends
//                                                                 share a fragment (fused compaction)
//   changeroot/handle_changeroot + handle_connect                k_hook: fragment -> other fragment
//     (:155-199, :355-387; _mpi:167-287, :582-671)                of its best edge; mutual pair =>
//                                                                 smaller label is the new core
//   handle_initiate broadcast of the new fragment id             k_jump: pointer jumping to the root
//     (:201-233; _mpi:289-351)
//   termination (:389-413, :492-552; _mpi:685-743)               k_flag_next + select: fragments with
//                                                                 an outgoing edge; none left => done
//   BRANCH sweep u<v (:481-490; _mpi:750-779)                    in_mst[eid] set by k_hook
//
// Weight levels (filter). The rounds run on one WEIGHT LEVEL of the edges at a time, lightest
// level first: level i holds the canonical edges with tau_{i-1} <= w < tau_i. Kruskal's order
// makes MSF(G) restricted to keys < tau exactly the MSF of the lighter levels, so once a level
// has run to completion its fragments are final for every lighter edge, and an edge of a later
// level whose ends already share a fragment can never enter the MSF (cycle property). The
// level pass (k_level_select) drops those edges BEFORE they are ever turned into arcs: the
// reference's REJECT, applied to a whole weight class at once. On R-MAT most heavy edges fall
// inside the giant fragment; they are rejected through a 1-bit-per-vertex membership bitmap
// (n/8 bytes: 2 MiB at scale 24, resident in every XCD's 4 MiB L2) instead of a 64 MiB label
// gather.
//
// Data layout in HBM (SoA, 256-B aligned carves of one workspace):
//   canonical edges  u[m] v[m] w[m] u32 (caller's)         eid = position, key = w << 32 | eid
//   arcs X / Y       src[C] dst[C] u32, key[C] u64        a level's arcs, grouped by source
//   segments X / Y   start[G] count[G] prefix[G+1] u64    block-private output regions
//   lab[n] u32  fragment label map        best[n] u64  per-fragment min outgoing key
//   par[n] u32  hook parent               act[2][n] u32 active fragment lists
//   flags[n] u8 select flags              bits[n/64] u64 giant-fragment bitmap
//
// Compaction without hot atomics. A compacting kernel runs a fixed grid of G blocks; block b
// owns a contiguous virtual input range and writes its survivors, in order, to the FRONT of the
// same range of the output buffer, then records its count (padded to a multiple of 4 with dead
// arcs, so every 4-arc group stays 16-B aligned). The next round reads these G segments through
// the prefix table. No same-address atomics (they serialise at ~12 ns each on MI355X, measured),
// and the output is deterministic.
//
// Label invariant. Each level's arcs carry the fragment roots current at the level start
// (lab[root] == root), so a level's first round needs no gathers. From its second round on, the
// min-edge kernel rewrites surviving arcs as (lab[src], lab[dst], key): arcs of round r carry the
// labels of the fragments active at the start of round r-1, and lab[x] for exactly those labels
// is refreshed every round by k_jump. A vertex's fragment is found by following lab[] to a
// fixpoint (find_lab); k_resolve compresses every vertex to its root between levels.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace ghs {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }

constexpr uint32_t SEG_G = 2048;   // blocks of a compacting kernel (8 per CU) = output segments
constexpr int FIND_LAB_MAX_HOPS = 256;
constexpr uint32_t JUMP_MAX_STEPS = 1u << 26;

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// best[c] = min(best[c], k). A plain read first: best only ever decreases, so a stale read is
// never below the true value and skipping on best <= k is always safe.
__device__ __forceinline__ void flush_min(uint64_t *__restrict__ best, uint32_t c, uint64_t k) {
  uint64_t *p = best + c;
  if (*p > k) atomicMin(reinterpret_cast<unsigned long long *>(p), (unsigned long long)k);
}

// Block-wide exclusive offsets for a compaction step: each lane contributes `mine` items and
// gets the count of items of lower lanes of the whole block; *total = block total.
// Every thread of the block must call it (two barriers).
__device__ __forceinline__ uint32_t block_offsets(uint32_t mine, uint32_t *s_wcnt, uint32_t *total) {
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  uint32_t incl = mine;
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const uint32_t o = __shfl_up(incl, d);
    if (lane >= d) incl += o;
  }
  if (lane == WAVE - 1) s_wcnt[wid] = incl;
  __syncthreads();
  uint32_t before = incl - mine, t = 0;
#pragma unroll
  for (int w = 0; w < BLOCK / WAVE; ++w) {
    if (w < wid) before += s_wcnt[w];
    t += s_wcnt[w];
  }
  *total = t;
  __syncthreads();
  return before;
}

// ------------------------------------------------------------------------------------------
// Segmented input: virtual index v in [0, total) lives in segment s with
// prefix[s] <= v < prefix[s+1], physical index start[s] + (v - prefix[s]).
// ------------------------------------------------------------------------------------------
struct SegView {
  const uint64_t *start;
  const uint64_t *prefix;  // nseg + 1 entries
  uint32_t nseg;
  uint64_t total;
};

__device__ __forceinline__ uint32_t seg_find(const uint64_t *__restrict__ prefix, uint32_t lo, uint32_t hi, uint64_t v) {
  // largest s in [lo, hi] with prefix[s] <= v
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= v) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// ------------------------------------------------------------------------------------------
// Stage 1: minimum outgoing edge per fragment (+ fused REJECT filter / stream compaction).
//
// Each lane owns 4 consecutive arcs (16-B loads of src/dst, 2x16-B of key). Arcs are grouped by
// source, so equal source labels form runs; a wave-wide segmented min-scan over its 256 arcs
// (in-lane serial + 6-step cross-lane scan) leaves one candidate per run, and only run tails
// touch best[] — after a plain read, since best only ever decreases (a stale read is never
// smaller than the true value, so skipping on `best <= cand` is always safe).
// IDENT: labels are already current roots (a level's first round): no gathers, dst not read.
// COMPACT: survivors (inter-fragment arcs) are written relabelled to this block's output segment.
// Dead arcs (src == LABEL_NONE) pad segments and are skipped.
// ------------------------------------------------------------------------------------------
template <bool IDENT, bool COMPACT>
__global__ __launch_bounds__(BLOCK) void k_minedge(const uint32_t *__restrict__ src, const uint32_t *__restrict__ dst,
                                                   const uint64_t *__restrict__ key, SegView in,
                                                   const uint32_t *__restrict__ lab, uint64_t *__restrict__ best,
                                                   uint32_t *__restrict__ osrc, uint32_t *__restrict__ odst,
                                                   uint64_t *__restrict__ okey, uint64_t *__restrict__ oseg_start,
                                                   uint64_t *__restrict__ oseg_count) {
  __shared__ uint32_t s_wcnt[BLOCK / WAVE];
  __shared__ uint32_t s_seg[2];
  const int lane = threadIdx.x & (WAVE - 1);
  const uint64_t T = in.total;
  const uint64_t Q = ((T + gridDim.x - 1) / gridDim.x + 3) & ~3ull;  // multiple of 4
  const uint64_t vb = Q * blockIdx.x;
  const uint64_t ve = (vb + Q < T) ? vb + Q : T;
  if (threadIdx.x == 0) {
    s_seg[0] = vb < T ? seg_find(in.prefix, 0, in.nseg - 1, vb) : 0;
    s_seg[1] = ve > vb ? seg_find(in.prefix, 0, in.nseg - 1, ve - 1) : 0;
  }
  __syncthreads();
  const uint32_t slo = s_seg[0], shi = s_seg[1];
  uint64_t out_n = 0;  // survivors written so far by this block
  uint32_t carry_l = LABEL_NONE;  // wave-uniform deferred run (label, min key)
  uint64_t carry_v = KEY_NONE;

  for (uint64_t v0 = vb; v0 < ve; v0 += ARCS_PER_BLOCK) {
    const uint64_t v = v0 + (uint64_t)threadIdx.x * ARCS_PER_THREAD;
    uint32_t L[4], D[4];
    uint64_t K[4];
    bool valid[4];
    if (v < ve) {
      const uint32_t s = (slo == shi) ? slo : seg_find(in.prefix, slo, shi, v);
      const uint64_t seg_end = in.prefix[s + 1];
      const uint64_t i0 = in.start[s] + (v - in.prefix[s]);
      if (v + 4 <= seg_end && v + 4 <= ve && (i0 & 3) == 0) {
        const uint4 s4 = *reinterpret_cast<const uint4 *>(src + i0);
        L[0] = s4.x; L[1] = s4.y; L[2] = s4.z; L[3] = s4.w;
        if (!IDENT) {
          const uint4 d4 = *reinterpret_cast<const uint4 *>(dst + i0);
          D[0] = d4.x; D[1] = d4.y; D[2] = d4.z; D[3] = d4.w;
        }
        const ulonglong2 k01 = *reinterpret_cast<const ulonglong2 *>(key + i0);
        const ulonglong2 k23 = *reinterpret_cast<const ulonglong2 *>(key + i0 + 2);
        K[0] = k01.x; K[1] = k01.y; K[2] = k23.x; K[3] = k23.y;
#pragma unroll
        for (int j = 0; j < 4; ++j) valid[j] = L[j] != LABEL_NONE;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool in_range = v + j < ve && v + j < seg_end;
          L[j] = in_range ? src[i0 + j] : LABEL_NONE;
          D[j] = (!IDENT && in_range) ? dst[i0 + j] : 0u;
          K[j] = in_range ? key[i0 + j] : KEY_NONE;
          valid[j] = L[j] != LABEL_NONE;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        L[j] = LABEL_NONE; D[j] = 0; K[j] = KEY_NONE; valid[j] = false;
      }
    }
    uint64_t V[4];
    if (IDENT) {
#pragma unroll
      for (int j = 0; j < 4; ++j) V[j] = valid[j] ? K[j] : KEY_NONE;  // level arcs: src != dst
    } else {
      uint32_t cs[4], cd[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // 8 independent gathers in flight per lane
        cs[j] = lab[valid[j] ? L[j] : 0u];
        cd[j] = lab[valid[j] ? D[j] : 0u];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        L[j] = valid[j] ? cs[j] : LABEL_NONE;
        D[j] = cd[j];
        V[j] = (valid[j] && cs[j] != cd[j]) ? K[j] : KEY_NONE;
      }
    }

    uint32_t smask = 0;  // survivors (inter-fragment arcs), taken before the carry merge
#pragma unroll
    for (int j = 0; j < 4; ++j) smask |= (V[j] != KEY_NONE) ? (1u << j) : 0u;
    // Deferred run of the previous iteration (wave-uniform carry): a run that reaches the
    // wave's end is not flushed but carried, and merged into the next run of the same label
    // (min is associative, contiguity is not needed). A giant fragment's run of millions of
    // arcs then costs one atomic per wave instead of one per 256 arcs (same-address atomics
    // serialise at the memory side).
    if (lane == 0 && L[0] == carry_l && carry_l != LABEL_NONE) {
      V[0] = umin64(V[0], carry_v);
      carry_l = LABEL_NONE;  // merged
    }
    carry_l = __shfl(carry_l, 0);
    if (carry_l != LABEL_NONE && lane == 0) flush_min(best, carry_l, carry_v);  // not merged
    carry_l = LABEL_NONE;

    // ---- wave-wide segmented min over 256 arcs, segments = runs of equal source label
    const uint32_t prevL3 = __shfl_up(L[3], 1);
    bool H[4];
    H[0] = (lane == 0) || (L[0] != prevL3);
    H[1] = L[1] != L[0];
    H[2] = L[2] != L[1];
    H[3] = L[3] != L[2];
    uint64_t x = KEY_NONE;
    int f = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x = H[j] ? V[j] : umin64(x, V[j]);
      f |= H[j] ? 1 : 0;
    }
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
      const uint64_t xo = __shfl_up(x, d);
      const int fo = __shfl_up(f, d);
      if (lane >= d) {
        if (!f) x = umin64(x, xo);
        f |= fo;
      }
    }
    uint64_t run = __shfl_up(x, 1);
    if (lane == 0) run = KEY_NONE;
    const int nextH0 = __shfl_down(H[0] ? 1 : 0, 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      run = H[j] ? V[j] : umin64(run, V[j]);
      const bool wave_end = (j == 3) && (lane == WAVE - 1);
      const bool tail = (j < 3) ? H[j + 1] : (lane == WAVE - 1 || nextH0);
      if (tail && !wave_end && run != KEY_NONE) flush_min(best, L[j], run);
      if (wave_end) {
        carry_l = (run != KEY_NONE) ? L[3] : LABEL_NONE;
        carry_v = run;
      }
    }
    carry_l = __shfl(carry_l, WAVE - 1);
    carry_v = __shfl(carry_v, WAVE - 1);

    if (COMPACT) {
      const uint32_t mine = (uint32_t)__popc(smask);
      uint32_t total;
      const uint32_t before = block_offsets(mine, s_wcnt, &total);
      uint64_t pos = vb + out_n + before;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (smask & (1u << j)) {
          osrc[pos] = L[j];
          odst[pos] = D[j];
          okey[pos] = K[j];
          ++pos;
        }
      }
      out_n += total;
    }
  }
  if (lane == 0 && carry_l != LABEL_NONE) flush_min(best, carry_l, carry_v);
  if (COMPACT) {
    // pad to a multiple of 4 with dead arcs; stays inside [vb, vb + Q) and below the capacity
    // (the workspace reserves 4 * SEG_G spare arcs)
    const uint64_t padded = (out_n + 3) & ~3ull;
    if (threadIdx.x < padded - out_n) {
      const uint64_t pos = vb + out_n + threadIdx.x;
      osrc[pos] = LABEL_NONE;
      odst[pos] = 0;
      okey[pos] = KEY_NONE;
    }
    if (threadIdx.x == 0) {
      oseg_start[blockIdx.x] = vb;
      oseg_count[blockIdx.x] = (vb < T) ? padded : 0;
    }
  }
}

// exclusive scan of count[0..n) into prefix[0..n]; one block of 1024 threads
__global__ __launch_bounds__(1024) void k_scan_counts(const uint64_t *__restrict__ count, uint32_t n,
                                                      uint64_t *__restrict__ prefix, unsigned long long *__restrict__ total) {
  __shared__ uint64_t s_part[1024];
  const uint32_t per = (n + 1023) / 1024;
  const uint32_t b = threadIdx.x * per;
  uint64_t sum = 0;
  for (uint32_t i = 0; i < per && b + i < n; ++i) sum += count[b + i];
  s_part[threadIdx.x] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const uint64_t o = threadIdx.x >= (unsigned)d ? s_part[threadIdx.x - d] : 0;
    __syncthreads();
    s_part[threadIdx.x] += o;
    __syncthreads();
  }
  uint64_t run = s_part[threadIdx.x] - sum;
  for (uint32_t i = 0; i < per && b + i < n; ++i) {
    prefix[b + i] = run;
    run += count[b + i];
  }
  if (threadIdx.x == 1023) {
    prefix[n] = s_part[1023];
    *total = s_part[1023];
  }
}

__device__ __forceinline__ uint32_t find_lab(const uint32_t *__restrict__ lab, uint32_t x,
                                             unsigned long long *__restrict__ err) {
  uint32_t y = lab[x];
  int hops = 0;
  while (y != x) {
    x = y;
    y = lab[x];
    if (++hops > FIND_LAB_MAX_HOPS) {
      atomicOr(err, 1ull);
      break;
    }
  }
  return x;
}

// ------------------------------------------------------------------------------------------
// Stage 2: hook (CONNECT over the best edge). act == nullptr => fragments are 0..nact-1.
// Strict total order on keys => the hook graph's only cycles are mutual pairs; the smaller
// label stays root (the reference merges equal-level fragments over a shared core edge,
// ghs_implementation.py:186-196, initiator by (fragment_id, rank), ghs_implementation_mpi.py:
// 237-239). Every hook adds exactly one MSF edge; one pair of atomics per block for the totals.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_hook(const uint32_t *__restrict__ act, uint64_t nact,
                                                const uint64_t *__restrict__ best, const uint32_t *__restrict__ lab,
                                                const uint32_t *__restrict__ eu, const uint32_t *__restrict__ ev,
                                                uint32_t *__restrict__ par, uint8_t *__restrict__ in_mst,
                                                unsigned long long *__restrict__ acc /* [0] weight, [1] edges */,
                                                unsigned long long *__restrict__ err) {
  __shared__ unsigned long long s_w[BLOCK / WAVE], s_c[BLOCK / WAVE];
  unsigned long long wsum = 0, cnt = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < nact; i += (uint64_t)gridDim.x * BLOCK) {
    const uint32_t c = act ? act[i] : (uint32_t)i;
    const uint64_t k = best[c];
    uint32_t p = c;
    if (k != KEY_NONE) {
      const uint32_t eid = (uint32_t)k;
      const uint32_t la = find_lab(lab, eu[eid], err);
      const uint32_t lb = find_lab(lab, ev[eid], err);
      if (la != c && lb != c) atomicOr(err, 2ull);  // the chosen edge must leave c
      const uint32_t other = (la == c) ? lb : la;
      const bool mutual = best[other] == k;
      if (!(mutual && c < other)) {
        p = other;
        in_mst[eid] = 1;
        wsum += k >> 32;
        cnt += 1;
      }
    }
    par[c] = p;
  }
#pragma unroll
  for (int d = WAVE / 2; d > 0; d >>= 1) {
    wsum += __shfl_xor(wsum, d);
    cnt += __shfl_xor(cnt, d);
  }
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  if (lane == 0) {
    s_w[wid] = wsum;
    s_c[wid] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tw = 0, tc = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / WAVE; ++w) {
      tw += s_w[w];
      tc += s_c[w];
    }
    if (tc) {
      atomicAdd(acc + 0, tw);
      atomicAdd(acc + 1, tc);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Stage 3: pointer jumping (INITIATE broadcast of the new fragment id). Path splitting on par:
// concurrent compression only moves a pointer to an ancestor, so stale reads are still valid
// ancestors and every walk ends at its root. lab[c] = root.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_jump(const uint32_t *__restrict__ act, uint64_t nact, uint32_t *par,
                                                uint32_t *__restrict__ lab, unsigned long long *__restrict__ err) {
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < nact; i += (uint64_t)gridDim.x * BLOCK) {
    const uint32_t c = act ? act[i] : (uint32_t)i;
    uint32_t x = c;
    uint32_t px = par[x];
    uint32_t steps = 0;
    while (px != x) {
      const uint32_t ppx = par[px];
      if (ppx != px) par[x] = ppx;
      x = px;
      px = ppx;
      if (++steps > JUMP_MAX_STEPS) {
        atomicOr(err, 4ull);
        break;
      }
    }
    lab[c] = x;
  }
}

// ------------------------------------------------------------------------------------------
// Stage 3b: flags of the next active fragment list = roots that still had an outgoing edge
// (their best slot is reset). A root with no outgoing edge is finished for this level (the
// reference: "best_weight == inf at the core => terminate", ghs_implementation.py:316-320).
// The list is produced by an order-preserving select, so every rank of a multi-GPU run holds
// the same list in the same order and the all-reduce slots line up.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_flag_next(const uint32_t *__restrict__ act, uint64_t nact,
                                                     const uint32_t *__restrict__ par, uint64_t *__restrict__ best,
                                                     uint8_t *__restrict__ flags) {
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < nact; i += (uint64_t)gridDim.x * BLOCK) {
    const uint32_t c = act ? act[i] : (uint32_t)i;
    const bool keep = (par[c] == c) && (best[c] != KEY_NONE);
    if (keep) best[c] = KEY_NONE;
    flags[i] = keep ? 1 : 0;
  }
}

// ------------------------------------------------------------------------------------------
// Between levels: compress every vertex to its root (lab[v] = find(v)) and flag the roots.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_resolve(uint32_t n, uint32_t *lab, uint8_t *__restrict__ root_flag,
                                                   unsigned long long *__restrict__ err) {
  for (uint64_t v = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; v < n; v += (uint64_t)gridDim.x * BLOCK) {
    const uint32_t r = find_lab(lab, (uint32_t)v, err);
    lab[v] = r;
    root_flag[v] = (r == (uint32_t)v) ? 1 : 0;
  }
}

// giant-fragment membership bitmap: bit v = (lab[v] == giant); one u64 word per wave
__global__ __launch_bounds__(BLOCK) void k_bitmap(uint32_t n, const uint32_t *__restrict__ lab, uint32_t giant,
                                                  uint64_t *__restrict__ bits) {
  const uint64_t words = ((uint64_t)n + 63) / 64;
  for (uint64_t base = blockIdx.x * (uint64_t)BLOCK; base < (uint64_t)n; base += (uint64_t)gridDim.x * BLOCK) {
    const uint64_t v = base + threadIdx.x;
    const bool in = v < n && lab[v] == giant;
    const uint64_t b = __ballot(in);
    if ((threadIdx.x & (WAVE - 1)) == 0 && (v >> 6) < words) bits[v >> 6] = b;
  }
}

__global__ void k_sample_labels(uint32_t n, const uint32_t *__restrict__ lab, uint32_t nsamp, uint32_t *__restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nsamp; i += gridDim.x * blockDim.x) {
    const uint64_t v = ((uint64_t)i * n) / nsamp;
    out[i] = lab[v < n ? v : n - 1];
  }
}

__global__ void k_sample_weights(uint64_t cnt, const uint32_t *__restrict__ w, uint32_t nsamp, uint32_t *__restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nsamp; i += gridDim.x * blockDim.x) {
    const uint64_t e = ((uint64_t)i * cnt) / nsamp;
    out[i] = w[e];
  }
}

// ------------------------------------------------------------------------------------------
// Level pass. Splits the edges still pending into (a) this level's edges whose ends lie in
// different fragments -> (lab[u], lab[v], key) into this block's level staging region, and
// (b) heavier edges that also survive the fragment test -> (u, v, key) into this block's
// REMAINING region, the next level's input. Edges whose ends share a fragment are dropped for
// good (cycle property). Both outputs are block-private regions (deterministic, no atomics).
// FIRST: the input is the canonical list itself [e_lo, e_hi) (u, v, w; key built here),
// every vertex is its own fragment, and the pass also validates canonicity (u < v < n,
// strictly ascending) into err bit 8 — before any kernel indexes an array with these ids.
// Otherwise the input is the previous level's remaining regions (segmented view) and lab is
// fully resolved (one hop); the giant-fragment bitmap rejects most heavy edges without a
// label gather.
// ------------------------------------------------------------------------------------------
template <bool FIRST>
__global__ __launch_bounds__(BLOCK) void k_level_pass(uint32_t n, uint64_t e_lo, const uint32_t *__restrict__ eu,
                                                      const uint32_t *__restrict__ ev, const uint32_t *__restrict__ ew,
                                                      const uint32_t *__restrict__ ru, const uint32_t *__restrict__ rv,
                                                      const uint64_t *__restrict__ rkey, SegView in, uint64_t w_hi,
                                                      const uint32_t *__restrict__ lab,
                                                      const uint64_t *__restrict__ giant_bits,
                                                      uint32_t *__restrict__ lsrc, uint32_t *__restrict__ ldst,
                                                      uint64_t *__restrict__ lkey, uint64_t *__restrict__ lcount,
                                                      uint32_t *__restrict__ ou, uint32_t *__restrict__ ov,
                                                      uint64_t *__restrict__ okey, uint64_t *__restrict__ ostart,
                                                      uint64_t *__restrict__ ocount,
                                                      unsigned long long *__restrict__ err) {
  __shared__ uint32_t s_wcnt[BLOCK / WAVE];
  __shared__ uint32_t s_seg[2];
  const uint64_t T = in.total;
  const uint64_t Q = ((T + gridDim.x - 1) / gridDim.x + 3) & ~3ull;
  const uint64_t vb = Q * blockIdx.x;
  const uint64_t ve = (vb + Q < T) ? vb + Q : T;
  if (!FIRST) {
    if (threadIdx.x == 0) {
      s_seg[0] = vb < T ? seg_find(in.prefix, 0, in.nseg - 1, vb) : 0;
      s_seg[1] = ve > vb ? seg_find(in.prefix, 0, in.nseg - 1, ve - 1) : 0;
    }
    __syncthreads();
  }
  uint64_t nlev = 0, nrem = 0;
  bool bad = false;
  for (uint64_t v0 = vb; v0 < ve; v0 += ARCS_PER_BLOCK) {
    const uint64_t v = v0 + (uint64_t)threadIdx.x * 4;
    uint32_t a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    uint64_t k[4] = {KEY_NONE, KEY_NONE, KEY_NONE, KEY_NONE};
    bool live[4] = {false, false, false, false};
    if (FIRST) {
      const uint64_t e0 = e_lo + v;
      uint32_t w[4] = {0, 0, 0, 0};
      if (v + 4 <= ve && (e0 & 3) == 0) {
        const uint4 a4 = *reinterpret_cast<const uint4 *>(eu + e0);
        const uint4 b4 = *reinterpret_cast<const uint4 *>(ev + e0);
        const uint4 w4 = *reinterpret_cast<const uint4 *>(ew + e0);
        a[0] = a4.x; a[1] = a4.y; a[2] = a4.z; a[3] = a4.w;
        b[0] = b4.x; b[1] = b4.y; b[2] = b4.z; b[3] = b4.w;
        w[0] = w4.x; w[1] = w4.y; w[2] = w4.z; w[3] = w4.w;
#pragma unroll
        for (int j = 0; j < 4; ++j) live[j] = true;
      } else if (v < ve) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (v + j < ve) {
            a[j] = eu[e0 + j];
            b[j] = ev[e0 + j];
            w[j] = ew[e0 + j];
            live[j] = true;
          }
        }
      }
      if (v < ve) {  // canonical order: u < v < n, (u, v) strictly ascending
        uint32_t pa = 0, pb = 0;
        const bool has_prev = e0 > 0;
        if (has_prev) {
          pa = eu[e0 - 1];
          pb = ev[e0 - 1];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (live[j]) {
            bool ok = a[j] < b[j] && b[j] < n;
            if (j > 0 || has_prev) ok = ok && (pa < a[j] || (pa == a[j] && pb < b[j]));
            bad |= !ok;
            pa = a[j];
            pb = b[j];
            k[j] = ((uint64_t)w[j] << 32) | (uint32_t)(e0 + j);
            if (!ok) live[j] = false;  // never index with an unchecked id
          }
        }
      }
    } else if (v < ve) {
      const uint32_t sidx = (s_seg[0] == s_seg[1]) ? s_seg[0] : seg_find(in.prefix, s_seg[0], s_seg[1], v);
      const uint64_t seg_end = in.prefix[sidx + 1];
      const uint64_t i0 = in.start[sidx] + (v - in.prefix[sidx]);
      if (v + 4 <= seg_end && v + 4 <= ve && (i0 & 3) == 0) {
        const uint4 a4 = *reinterpret_cast<const uint4 *>(ru + i0);
        const uint4 b4 = *reinterpret_cast<const uint4 *>(rv + i0);
        const ulonglong2 k01 = *reinterpret_cast<const ulonglong2 *>(rkey + i0);
        const ulonglong2 k23 = *reinterpret_cast<const ulonglong2 *>(rkey + i0 + 2);
        a[0] = a4.x; a[1] = a4.y; a[2] = a4.z; a[3] = a4.w;
        b[0] = b4.x; b[1] = b4.y; b[2] = b4.z; b[3] = b4.w;
        k[0] = k01.x; k[1] = k01.y; k[2] = k23.x; k[3] = k23.y;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool in_range = v + j < ve && v + j < seg_end;
          a[j] = in_range ? ru[i0 + j] : LABEL_NONE;
          b[j] = in_range ? rv[i0 + j] : 0u;
          k[j] = in_range ? rkey[i0 + j] : KEY_NONE;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) live[j] = a[j] != LABEL_NONE;
      // REJECT a whole class at once: both ends in the giant fragment (1-bit bitmap in L2;
      // a is sorted within a region, so one word load usually serves a lane's 4 edges)
      uint32_t wa_idx = 0xffffffffu;
      uint64_t wa = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (live[j]) {
          if ((a[j] >> 6) != wa_idx) {
            wa_idx = a[j] >> 6;
            wa = giant_bits[wa_idx];
          }
          const bool ga = (wa >> (a[j] & 63)) & 1;
          if (ga && ((giant_bits[b[j] >> 6] >> (b[j] & 63)) & 1)) live[j] = false;
        }
      }
    }
    // fragment test + level/remaining split
    uint32_t la[4], lb[4];
    bool lev[4], rem[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      la[j] = a[j];
      lb[j] = b[j];
      if (!FIRST && live[j]) {
        la[j] = lab[a[j]];
        lb[j] = lab[b[j]];
        if (la[j] == lb[j]) live[j] = false;
      }
      const bool in_level = (k[j] >> 32) < w_hi;
      lev[j] = live[j] && in_level;
      rem[j] = live[j] && !in_level;
    }
    uint32_t mlev = 0, mrem = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mlev += lev[j] ? 1u : 0u;
      mrem += rem[j] ? 1u : 0u;
    }
    uint32_t tlev, trem;
    const uint32_t blev = block_offsets(mlev, s_wcnt, &tlev);
    const uint32_t brem = block_offsets(mrem, s_wcnt, &trem);
    uint64_t pl = vb + nlev + blev, pr = vb + nrem + brem;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (lev[j]) {
        lsrc[pl] = la[j];
        ldst[pl] = lb[j];
        lkey[pl] = k[j];
        ++pl;
      }
      if (rem[j]) {
        ou[pr] = a[j];
        ov[pr] = b[j];
        okey[pr] = k[j];
        ++pr;
      }
    }
    nlev += tlev;
    nrem += trem;
  }
  if (FIRST && bad) atomicOr(err, 8ull);
  // remaining regions padded to a multiple of 4 with dead entries (u = LABEL_NONE)
  const uint64_t padded = (nrem + 3) & ~3ull;
  if (threadIdx.x < padded - nrem) {
    const uint64_t pos = vb + nrem + threadIdx.x;
    ou[pos] = LABEL_NONE;
    ov[pos] = 0;
    okey[pos] = KEY_NONE;
  }
  if (threadIdx.x == 0) {
    lcount[blockIdx.x] = (vb < T) ? nlev : 0;
    ostart[blockIdx.x] = vb;
    ocount[blockIdx.x] = (vb < T) ? padded : 0;
  }
}

// staging segments -> dense forward arcs [0, S) of the level arc buffer (order preserved)
__global__ __launch_bounds__(BLOCK) void k_gather_segments(uint64_t T, const uint64_t *__restrict__ seg_prefix,
                                                           const uint32_t *__restrict__ ssrc,
                                                           const uint32_t *__restrict__ sdst,
                                                           const uint64_t *__restrict__ skey, uint32_t *__restrict__ dsrc,
                                                           uint32_t *__restrict__ ddst, uint64_t *__restrict__ dkey) {
  const uint64_t Q = ((T + gridDim.x - 1) / gridDim.x + 3) & ~3ull;
  const uint64_t vb = Q * blockIdx.x;
  const uint64_t cnt = seg_prefix[blockIdx.x + 1] - seg_prefix[blockIdx.x];
  const uint64_t dbase = seg_prefix[blockIdx.x];
  for (uint64_t i = threadIdx.x; i < cnt; i += BLOCK) {
    dsrc[dbase + i] = ssrc[vb + i];
    ddst[dbase + i] = sdst[vb + i];
    dkey[dbase + i] = skey[vb + i];
  }
}

__global__ void k_iota(uint32_t *__restrict__ a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}

// reverse arcs [S, 2S): src = sorted dst labels (already written), dst/key gathered by index
__global__ void k_fill_reverse(uint64_t S, const uint32_t *__restrict__ idx, uint32_t *__restrict__ asrc,
                               uint32_t *__restrict__ adst, uint64_t *__restrict__ akey) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < S; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t j = idx[i];
    adst[S + i] = asrc[j];
    akey[S + i] = akey[j];
  }
}

// flag every fragment that has an arc in the level: run heads of the (grouped) source labels
__global__ void k_mark_sources(uint64_t A, const uint32_t *__restrict__ src, uint8_t *__restrict__ flags) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < A; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = src[i];
    if (i == 0 || src[i - 1] != c) flags[c] = 1;
  }
}

__global__ void k_set_seg1(uint64_t *start, uint64_t *prefix, uint64_t total) {
  start[0] = 0;
  prefix[0] = 0;
  prefix[1] = total;
}

// dense all-reduce staging: int64 slot = key ^ 2^63 preserves unsigned order under signed MIN
__global__ void k_pack_best(const uint32_t *__restrict__ act, uint64_t nact, const uint64_t *__restrict__ best,
                            int64_t *__restrict__ dense) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nact; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = act ? act[i] : (uint32_t)i;
    dense[i] = (int64_t)(best[c] ^ 0x8000000000000000ull);
  }
}

__global__ void k_unpack_best(const uint32_t *__restrict__ act, uint64_t nact, uint64_t *__restrict__ best,
                              const int64_t *__restrict__ dense) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nact; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = act ? act[i] : (uint32_t)i;
    best[c] = (uint64_t)dense[i] ^ 0x8000000000000000ull;
  }
}

static inline unsigned grid_for(uint64_t items, uint64_t per_block, unsigned cap) {
  uint64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

static inline int bits_for(uint64_t maxval) {
  int b = 0;
  while (b < 64 && (maxval >> b)) ++b;
  return b ? b : 1;
}

}  // namespace ghs

using namespace ghs;

// ============================================================================================
// Solver handle
// ============================================================================================
struct ArcBuf {
  uint32_t *src = nullptr, *dst = nullptr;
  uint64_t *key = nullptr;
  uint64_t *seg_start = nullptr, *seg_count = nullptr, *seg_prefix = nullptr;
};

struct ghs_solver {
  uint32_t n = 0;
  uint64_t m = 0, e_lo = 0, e_hi = 0;
  const uint32_t *eu = nullptr, *ev = nullptr, *ew = nullptr;
  uint8_t *in_mst = nullptr;
  hipStream_t stream = nullptr;
  ghs_config_t cfg{};

  uint32_t *lab = nullptr, *par = nullptr, *act[2] = {nullptr, nullptr};
  uint64_t *best = nullptr, *bits = nullptr;
  uint8_t *flags = nullptr;
  uint32_t *sample = nullptr;
  ArcBuf buf[2];
  ArcBuf rem[2];             // remaining (not yet levelled) edges: u, v, key as block regions
  int rcur = 0;              // rem buffer holding the pending edges (level >= 1)
  uint64_t rem_total = 0;    // pending edges (incl. padding) after the last level pass
  uint32_t rem_nseg = 1;     // regions of the pending edges
  uint64_t cap_arcs = 0;
  void *cub_temp = nullptr;
  size_t cub_bytes = 0;
  unsigned long long *cnt = nullptr;    // device [0] scratch total, [1] active out, [2] weight, [3] edges, [4] err
  unsigned long long *h_cnt = nullptr;  // pinned host mirror
  uint32_t *h_sample = nullptr;         // pinned host sample buffer

  // level plan (identical on every rank: computed from the global canonical list)
  std::vector<uint64_t> thresholds;  // level i: [thr[i], thr[i+1])
  uint32_t level = 0;                // index of the level being processed
  bool level_open = false;
  uint64_t level_arcs = 0;           // arcs built for the current level (stats)

  // round state
  uint32_t round = 0;        // completed rounds (all levels)
  uint32_t level_round = 0;  // completed rounds in this level
  int phase = 0;             // 0: expect minedge, 1: expect contract, 2: done
  int cur = 0;               // arc buffer holding the live arcs
  bool cur_single = true;    // live arcs are one dense segment
  uint64_t cur_arcs = 0;
  int act_cur = 0;
  bool act_ident = true;     // fragments are 0..n-1
  uint64_t nact = 0;
  uint64_t edges_before = 0;

  std::vector<ghs_round_stats_t> stats;
  std::vector<hipEvent_t> ev_pool;
  std::chrono::steady_clock::time_point t0;
};

static std::mutex g_mutex;  // the one-shot entry points are serialised per process

static constexpr uint32_t NSAMPLE = 8192;    // labels sampled to find the giant fragment
static constexpr uint32_t NSAMPLE_W = 16384; // weights sampled for the level plan
static constexpr uint32_t NSAMPLE_MAX = NSAMPLE_W > NSAMPLE ? NSAMPLE_W : NSAMPLE;

static size_t cub_temp_bytes(uint32_t n, uint64_t cap) {
  size_t a = 0, b = 0, c = 0;
  const size_t items = n ? n : 1;
  (void)hipcub::DeviceSelect::Flagged(nullptr, a, (const uint32_t *)nullptr, (const uint8_t *)nullptr,
                                      (uint32_t *)nullptr, (unsigned long long *)nullptr, items);
  (void)hipcub::DeviceSelect::Flagged(nullptr, b, hipcub::CountingInputIterator<uint32_t>(0u),
                                      (const uint8_t *)nullptr, (uint32_t *)nullptr, (unsigned long long *)nullptr,
                                      items);
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, c, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                          (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                          (size_t)(cap ? cap : 1), 0, bits_for(n ? n - 1 : 0));
  return std::max(a, std::max(b, c)) + 256;
}

static size_t workspace_layout(uint32_t n, uint64_t local_edges, ghs_solver *s, char *base) {
  size_t off = 0;
  auto carve = [&](size_t bytes) -> char * {
    char *p = base ? base + off : nullptr;
    off = align_up(off + bytes, 256);
    return p;
  };
  const size_t N = (size_t)n;
  const uint64_t cap = 2 * local_edges + 4 * SEG_G;  // a level's arcs: <= 2 per selected edge (+ padding)
  char *p;
  p = carve(N * 4); if (s) s->lab = (uint32_t *)p;
  p = carve(N * 4); if (s) s->par = (uint32_t *)p;
  p = carve(N * 8); if (s) s->best = (uint64_t *)p;
  p = carve(N * 4); if (s) s->act[0] = (uint32_t *)p;
  p = carve(N * 4); if (s) s->act[1] = (uint32_t *)p;
  p = carve(N ? N : 1); if (s) s->flags = (uint8_t *)p;
  p = carve(((N + 63) / 64) * 8 + 8); if (s) s->bits = (uint64_t *)p;
  p = carve(NSAMPLE_MAX * 4); if (s) s->sample = (uint32_t *)p;
  for (int b = 0; b < 2; ++b) {
    p = carve(cap * 4); if (s) s->buf[b].src = (uint32_t *)p;
    p = carve(cap * 4); if (s) s->buf[b].dst = (uint32_t *)p;
    p = carve(cap * 8); if (s) s->buf[b].key = (uint64_t *)p;
    p = carve(SEG_G * 8); if (s) s->buf[b].seg_start = (uint64_t *)p;
    p = carve(SEG_G * 8); if (s) s->buf[b].seg_count = (uint64_t *)p;
    p = carve((SEG_G + 1) * 8); if (s) s->buf[b].seg_prefix = (uint64_t *)p;
  }
  const uint64_t rcap = local_edges + 4 * SEG_G;
  for (int b = 0; b < 2; ++b) {
    p = carve(rcap * 4); if (s) s->rem[b].src = (uint32_t *)p;
    p = carve(rcap * 4); if (s) s->rem[b].dst = (uint32_t *)p;
    p = carve(rcap * 8); if (s) s->rem[b].key = (uint64_t *)p;
    p = carve(SEG_G * 8); if (s) s->rem[b].seg_start = (uint64_t *)p;
    p = carve(SEG_G * 8); if (s) s->rem[b].seg_count = (uint64_t *)p;
    p = carve((SEG_G + 1) * 8); if (s) s->rem[b].seg_prefix = (uint64_t *)p;
  }
  const size_t cb = cub_temp_bytes(n, cap);
  p = carve(cb); if (s) { s->cub_temp = p; s->cub_bytes = cb; s->cap_arcs = cap; }
  p = carve(8 * sizeof(unsigned long long)); if (s) s->cnt = (unsigned long long *)p;
  return off;
}

static hipEvent_t round_event(ghs_solver *s, uint32_t round, int k) {
  if (round >= GHS_MAX_ROUND_STATS) return nullptr;
  const size_t idx = (size_t)round * 6 + k;
  while (s->ev_pool.size() <= idx) {
    hipEvent_t ev = nullptr;
    if (hipEventCreate(&ev) != hipSuccess) return nullptr;
    s->ev_pool.push_back(ev);
  }
  return s->ev_pool[idx];
}

static void record(ghs_solver *s, int k) {
  hipEvent_t ev = round_event(s, s->round, k);
  if (ev) (void)hipEventRecord(ev, s->stream);
}

static void default_config(ghs_config_t *c) {
  c->max_levels = 8;
  c->num_ranks = 1;
  c->level1_edges_per_vertex = 0.5;
  c->level_growth = 4.0;
}

// ---- level planning: thresholds from a sample of the GLOBAL canonical weights ----------------
static int plan_levels(ghs_solver *s) {
  s->thresholds.clear();
  s->thresholds.push_back(0);
  const uint32_t L = std::max<uint32_t>(1, std::min<uint32_t>(s->cfg.max_levels, 32));
  if (L > 1 && s->m > 0) {
    const uint32_t ns = (uint32_t)std::min<uint64_t>(NSAMPLE_W, s->m);
    k_sample_weights<<<grid_for(ns, 256, 256), 256, 0, s->stream>>>(s->m, s->ew, ns, s->sample);
    GHS_HIP_CHECK(hipGetLastError());
    GHS_HIP_CHECK(hipMemcpyAsync(s->h_sample, s->sample, ns * 4, hipMemcpyDeviceToHost, s->stream));
    GHS_HIP_CHECK(hipStreamSynchronize(s->stream));
    std::vector<uint32_t> w(s->h_sample, s->h_sample + ns);
    double target = s->cfg.level1_edges_per_vertex * (double)s->n;
    for (uint32_t i = 1; i < L; ++i) {
      const double frac = target / (double)s->m;
      if (frac >= 1.0) break;
      const size_t q = (size_t)(frac * ns);
      target *= std::max(1.01, s->cfg.level_growth);
      if (q == 0) continue;
      std::nth_element(w.begin(), w.begin() + q, w.end());
      const uint64_t thr = (uint64_t)w[q];
      if (thr > s->thresholds.back()) s->thresholds.push_back(thr);
    }
  }
  s->thresholds.push_back(1ull << 32);
  return GHS_OK;
}

// ---- open the next level: split pending edges, build the level's arcs, set the active list ---
// Returns GHS_OK with s->level_open set, or with the level skipped (single rank, no arcs).
static int open_level(ghs_solver *s) {
  const uint32_t lv = s->level;
  const uint64_t w_hi = s->thresholds[lv + 1];
  const bool first = (lv == 0);
  hipStream_t st = s->stream;
  ArcBuf &X = s->buf[0], &Y = s->buf[1];
  const int rin = s->rcur, rout = first ? 0 : (s->rcur ^ 1);
  ArcBuf &RI = s->rem[rin], &RO = s->rem[rout];

  if (!first) {
    // compress labels, find the giant fragment from a sample, build its bitmap
    k_resolve<<<grid_for(s->n, BLOCK, 16384), BLOCK, 0, st>>>(s->n, s->lab, s->flags, s->cnt + 4);
    const uint32_t ns = std::min<uint32_t>(NSAMPLE, s->n);
    k_sample_labels<<<grid_for(ns, 256, 256), 256, 0, st>>>(s->n, s->lab, ns, s->sample);
    GHS_HIP_CHECK(hipGetLastError());
    GHS_HIP_CHECK(hipMemcpyAsync(s->h_sample, s->sample, ns * 4, hipMemcpyDeviceToHost, st));
    GHS_HIP_CHECK(hipStreamSynchronize(st));
    std::vector<uint32_t> smp(s->h_sample, s->h_sample + ns);
    std::sort(smp.begin(), smp.end());
    uint32_t giant = smp[0];
    size_t best_run = 0;
    for (size_t i = 0; i < smp.size();) {
      size_t j = i;
      while (j < smp.size() && smp[j] == smp[i]) ++j;
      if (j - i > best_run) {
        best_run = j - i;
        giant = smp[i];
      }
      i = j;
    }
    k_bitmap<<<grid_for(s->n, BLOCK, 16384), BLOCK, 0, st>>>(s->n, s->lab, giant, s->bits);
    GHS_HIP_CHECK(hipGetLastError());
  }

  // 1. split: this level's surviving edges -> Y staging; heavier survivors -> RO regions
  const uint64_t T = first ? (s->e_hi - s->e_lo) : s->rem_total;
  const unsigned G = grid_for(T, ARCS_PER_BLOCK, SEG_G);
  SegView in{RI.seg_start, RI.seg_prefix, s->rem_nseg, T};
  if (T) {
    if (first)
      k_level_pass<true><<<G, BLOCK, 0, st>>>(s->n, s->e_lo, s->eu, s->ev, s->ew, nullptr, nullptr, nullptr, in, w_hi,
                                              s->lab, s->bits, Y.src, Y.dst, Y.key, Y.seg_count, RO.src, RO.dst,
                                              RO.key, RO.seg_start, RO.seg_count, s->cnt + 4);
    else
      k_level_pass<false><<<G, BLOCK, 0, st>>>(s->n, 0, nullptr, nullptr, nullptr, RI.src, RI.dst, RI.key, in, w_hi,
                                               s->lab, s->bits, Y.src, Y.dst, Y.key, Y.seg_count, RO.src, RO.dst,
                                               RO.key, RO.seg_start, RO.seg_count, s->cnt + 4);
    GHS_HIP_CHECK(hipGetLastError());
    k_scan_counts<<<1, 1024, 0, st>>>(Y.seg_count, G, Y.seg_prefix, s->cnt + 0);
    k_scan_counts<<<1, 1024, 0, st>>>(RO.seg_count, G, RO.seg_prefix, s->cnt + 5);
    // 2. dense forward arcs X[0, S) (order kept: grouped by the source's vertex)
    k_gather_segments<<<G, BLOCK, 0, st>>>(T, Y.seg_prefix, Y.src, Y.dst, Y.key, X.src, X.dst, X.key);
    GHS_HIP_CHECK(hipGetLastError());
  } else {
    GHS_HIP_CHECK(hipMemsetAsync(s->cnt, 0, 8, st));
    GHS_HIP_CHECK(hipMemsetAsync(s->cnt + 5, 0, 8, st));
  }
  GHS_HIP_CHECK(hipMemcpyAsync(s->h_cnt, s->cnt, 6 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  if (s->h_cnt[4] & 8) {
    s->phase = 2;
    GHS_FAIL(GHS_E_NONCANON, "edge list is not canonical (need u < v < n, strictly ascending (u, v))");
  }
  if (s->h_cnt[4]) {
    s->phase = 2;
    GHS_FAIL(GHS_E_STATE, "internal invariant violated (code " + std::to_string(s->h_cnt[4]) + ")");
  }
  const uint64_t S = s->h_cnt[0];
  s->rem_total = s->h_cnt[5];
  s->rem_nseg = G;
  s->rcur = rout;
  s->level_arcs = 2 * S;
  if (S == 0 && s->cfg.num_ranks <= 1) {  // nothing to merge at this level (single rank only:
    s->level_open = false;                // ranks must run the same rounds)
    return GHS_OK;
  }
  // 3. reverse arcs X[S, 2S): radix sort (dst label, index) -> grouped by dst label
  if (S) {
    uint32_t *idx_in = Y.src, *idx_out = Y.dst;  // Y's staging is consumed
    k_iota<<<grid_for(S, 256, 16384), 256, 0, st>>>(idx_in, S);
    size_t cb = s->cub_bytes;
    GHS_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(s->cub_temp, cb, X.dst, X.src + S, idx_in, idx_out, (size_t)S, 0,
                                                     bits_for(s->n - 1), st));
    k_fill_reverse<<<grid_for(S, 256, 16384), 256, 0, st>>>(S, idx_out, X.src, X.dst, X.key);
    GHS_HIP_CHECK(hipGetLastError());
  }
  s->cur = 0;
  s->cur_single = true;
  s->cur_arcs = 2 * S;
  k_set_seg1<<<1, 1, 0, st>>>(X.seg_start, X.seg_prefix, s->cur_arcs);
  GHS_HIP_CHECK(hipGetLastError());

  // 4. active fragments. Single rank: the fragments that have an arc in this level.
  //    Several ranks: every current root (first level: every vertex) — identical on every
  //    rank without an exchange; roots without arcs anywhere drop out after one round.
  size_t cb = s->cub_bytes;
  if (s->cfg.num_ranks <= 1) {
    GHS_HIP_CHECK(hipMemsetAsync(s->flags, 0, s->n, st));
    k_mark_sources<<<grid_for(2 * S, 256, 16384), 256, 0, st>>>(2 * S, X.src, s->flags);
    GHS_HIP_CHECK(hipGetLastError());
    GHS_HIP_CHECK(hipcub::DeviceSelect::Flagged(s->cub_temp, cb, hipcub::CountingInputIterator<uint32_t>(0u), s->flags,
                                                s->act[0], s->cnt + 1, (size_t)s->n, st));
    GHS_HIP_CHECK(hipMemcpyAsync(s->h_cnt + 1, s->cnt + 1, 8, hipMemcpyDeviceToHost, st));
    GHS_HIP_CHECK(hipStreamSynchronize(st));
    s->act_ident = false;
    s->act_cur = 0;
    s->nact = s->h_cnt[1];
  } else if (first) {
    s->act_ident = true;
    s->nact = s->n;
  } else {
    GHS_HIP_CHECK(hipcub::DeviceSelect::Flagged(s->cub_temp, cb, hipcub::CountingInputIterator<uint32_t>(0u), s->flags,
                                                s->act[0], s->cnt + 1, (size_t)s->n, st));
    GHS_HIP_CHECK(hipMemcpyAsync(s->h_cnt + 1, s->cnt + 1, 8, hipMemcpyDeviceToHost, st));
    GHS_HIP_CHECK(hipStreamSynchronize(st));
    s->act_ident = false;
    s->act_cur = 0;
    s->nact = s->h_cnt[1];
  }
  s->level_round = 0;
  s->level_open = true;
  return GHS_OK;
}

extern "C" {

int ghs_abi_version(void) { return GHS_MST_ABI_VERSION; }
const char *ghs_last_error(void) { return ghs::g_err.c_str(); }

int ghs_device_count(int *count) {
  if (!count) GHS_FAIL(GHS_E_ARG, "count is NULL");
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *count = c;
  return GHS_OK;
}

void ghs_default_config(ghs_config_t *cfg) {
  if (cfg) default_config(cfg);
}

size_t ghs_workspace_bytes(uint32_t n, uint64_t m, uint64_t local_edges) {
  (void)m;
  return workspace_layout(n, local_edges, nullptr, nullptr);
}

int ghs_solver_create(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                      uint64_t e_lo, uint64_t e_hi, const ghs_config_t *cfg, void *d_workspace,
                      size_t workspace_bytes, uint8_t *d_in_mst, void *stream, ghs_solver_t **out) {
  if (!out) GHS_FAIL(GHS_E_ARG, "out is NULL");
  *out = nullptr;
  if (m >= (1ull << 31)) GHS_FAIL(GHS_E_ARG, "m must be < 2^31");
  if (e_lo > e_hi || e_hi > m) GHS_FAIL(GHS_E_ARG, "bad edge range");
  if (m && (!d_u || !d_v || !d_w || !d_in_mst)) GHS_FAIL(GHS_E_ARG, "d_u/d_v/d_w/d_in_mst is NULL");
  if ((((uintptr_t)d_u) | ((uintptr_t)d_v) | ((uintptr_t)d_w)) & 15)
    GHS_FAIL(GHS_E_ARG, "d_u/d_v/d_w must be 16-byte aligned");
  const size_t need = workspace_layout(n, e_hi - e_lo, nullptr, nullptr);
  if (!d_workspace || workspace_bytes < need)
    GHS_FAIL(GHS_E_NOMEM, "workspace too small: need " + std::to_string(need) + " bytes");
  if (((uintptr_t)d_workspace) & 255) GHS_FAIL(GHS_E_ARG, "workspace must be 256-byte aligned");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) GHS_FAIL(GHS_E_NODEVICE, "no HIP device");

  ghs_solver *s = new ghs_solver();
  s->n = n; s->m = m; s->e_lo = e_lo; s->e_hi = e_hi;
  s->eu = d_u; s->ev = d_v; s->ew = d_w;
  s->in_mst = d_in_mst; s->stream = (hipStream_t)stream;
  if (cfg) s->cfg = *cfg; else default_config(&s->cfg);
  workspace_layout(n, e_hi - e_lo, s, (char *)d_workspace);
  auto fail = [&](hipError_t e, const char *what) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    if (s->h_cnt) (void)hipHostFree(s->h_cnt);
    if (s->h_sample) (void)hipHostFree(s->h_sample);
    delete s;
    return GHS_E_HIP;
  };
  hipError_t e;
  if ((e = hipHostMalloc((void **)&s->h_cnt, 8 * sizeof(unsigned long long), hipHostMallocDefault)) != hipSuccess)
    return fail(e, "hipHostMalloc");
  if ((e = hipHostMalloc((void **)&s->h_sample, NSAMPLE_MAX * 4, hipHostMallocDefault)) != hipSuccess)
    return fail(e, "hipHostMalloc");
  s->t0 = std::chrono::steady_clock::now();
  if (n) {
    if ((e = hipMemsetAsync(s->best, 0xff, (size_t)n * 8, s->stream)) != hipSuccess) return fail(e, "memset best");
    k_iota<<<grid_for(n, 256, 8192), 256, 0, s->stream>>>(s->lab, n);
  }
  if (m && (e = hipMemsetAsync(s->in_mst, 0, m, s->stream)) != hipSuccess) return fail(e, "memset in_mst");
  if ((e = hipMemsetAsync(s->cnt, 0, 8 * sizeof(unsigned long long), s->stream)) != hipSuccess)
    return fail(e, "memset counters");
  if ((e = hipGetLastError()) != hipSuccess) return fail(e, "init kernels");
  int rc = plan_levels(s);
  if (rc) {
    ghs_solver_destroy(s);
    return rc;
  }
  s->level = 0;
  s->level_open = false;
  s->phase = n ? 0 : 2;
  *out = s;
  return GHS_OK;
}

int ghs_solver_minedge(ghs_solver_t *s, uint64_t *num_active) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  if (s->phase == 2) {
    if (num_active) *num_active = 0;
    return GHS_OK;
  }
  if (s->phase != 0) GHS_FAIL(GHS_E_STATE, "minedge called twice without contract");
  if (s->round >= 16 * GHS_MAX_ROUND_STATS) GHS_FAIL(GHS_E_ROUNDCAP, "round cap exceeded");
  while (!s->level_open) {
    if (s->level + 1 >= s->thresholds.size()) {  // every level done
      s->phase = 2;
      if (num_active) *num_active = 0;
      return GHS_OK;
    }
    int rc = open_level(s);
    if (rc) return rc;
    if (!s->level_open) s->level += 1;  // skipped (no arcs)
  }
  record(s, 0);
  const uint64_t A = s->cur_arcs;
  const ArcBuf &I = s->buf[s->cur];
  ArcBuf &O = s->buf[s->cur ^ 1];
  if (A) {
    SegView in{I.seg_start, I.seg_prefix, s->cur_single ? 1u : SEG_G, A};
    const unsigned G = grid_for(A, ARCS_PER_BLOCK, SEG_G);
    if (s->level_round == 0) {
      k_minedge<true, false><<<G, BLOCK, 0, s->stream>>>(I.src, I.dst, I.key, in, s->lab, s->best, nullptr, nullptr,
                                                         nullptr, nullptr, nullptr);
    } else {
      // unused segment slots of O (when G < SEG_G) stay zero-count
      if (G < SEG_G) GHS_HIP_CHECK(hipMemsetAsync(O.seg_count + G, 0, (SEG_G - G) * 8, s->stream));
      k_minedge<false, true><<<G, BLOCK, 0, s->stream>>>(I.src, I.dst, I.key, in, s->lab, s->best, O.src, O.dst,
                                                         O.key, O.seg_start, O.seg_count);
      k_scan_counts<<<1, 1024, 0, s->stream>>>(O.seg_count, SEG_G, O.seg_prefix, s->cnt + 0);
    }
    GHS_HIP_CHECK(hipGetLastError());
  }
  record(s, 1);
  s->phase = 1;
  if (num_active) *num_active = s->nact;
  return GHS_OK;
}

int ghs_solver_pack_best(ghs_solver_t *s, int64_t *d_dense) {
  if (!s || (s->nact && !d_dense)) GHS_FAIL(GHS_E_ARG, "solver/dense is NULL");
  if (s->phase != 1) GHS_FAIL(GHS_E_STATE, "pack_best must follow minedge");
  if (s->nact) {
    const uint32_t *act = s->act_ident ? nullptr : s->act[s->act_cur];
    k_pack_best<<<grid_for(s->nact, 256, 16384), 256, 0, s->stream>>>(act, s->nact, s->best, d_dense);
    GHS_HIP_CHECK(hipGetLastError());
  }
  return GHS_OK;
}

int ghs_solver_unpack_best(ghs_solver_t *s, const int64_t *d_dense) {
  if (!s || (s->nact && !d_dense)) GHS_FAIL(GHS_E_ARG, "solver/dense is NULL");
  if (s->phase != 1) GHS_FAIL(GHS_E_STATE, "unpack_best must follow minedge");
  if (s->nact) {
    const uint32_t *act = s->act_ident ? nullptr : s->act[s->act_cur];
    k_unpack_best<<<grid_for(s->nact, 256, 16384), 256, 0, s->stream>>>(act, s->nact, s->best, d_dense);
    GHS_HIP_CHECK(hipGetLastError());
  }
  return GHS_OK;
}

int ghs_solver_contract(ghs_solver_t *s, int *done) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  if (s->phase == 2) {
    if (done) *done = 1;
    return GHS_OK;
  }
  if (s->phase != 1) GHS_FAIL(GHS_E_STATE, "contract must follow minedge");
  const uint32_t *act = s->act_ident ? nullptr : s->act[s->act_cur];
  const uint64_t nact = s->nact;
  const unsigned g = grid_for(nact, BLOCK, 16384);
  if (nact) {
    k_hook<<<grid_for(nact, BLOCK, 2048), BLOCK, 0, s->stream>>>(act, nact, s->best, s->lab, s->eu, s->ev, s->par,
                                                                 s->in_mst, s->cnt + 2, s->cnt + 4);
    GHS_HIP_CHECK(hipGetLastError());
  }
  record(s, 2);
  if (nact) {
    k_jump<<<g, BLOCK, 0, s->stream>>>(act, nact, s->par, s->lab, s->cnt + 4);
    GHS_HIP_CHECK(hipGetLastError());
  }
  record(s, 3);
  const int nb = s->act_ident ? 0 : (s->act_cur ^ 1);
  if (nact) {
    k_flag_next<<<g, BLOCK, 0, s->stream>>>(act, nact, s->par, s->best, s->flags);
    GHS_HIP_CHECK(hipGetLastError());
    size_t cb = s->cub_bytes;
    if (act) {
      GHS_HIP_CHECK(hipcub::DeviceSelect::Flagged(s->cub_temp, cb, act, s->flags, s->act[nb], s->cnt + 1, (size_t)nact,
                                                  s->stream));
    } else {
      GHS_HIP_CHECK(hipcub::DeviceSelect::Flagged(s->cub_temp, cb, hipcub::CountingInputIterator<uint32_t>(0u),
                                                  s->flags, s->act[nb], s->cnt + 1, (size_t)nact, s->stream));
    }
  } else {
    GHS_HIP_CHECK(hipMemsetAsync(s->cnt + 1, 0, 8, s->stream));
  }
  record(s, 4);
  GHS_HIP_CHECK(hipMemcpyAsync(s->h_cnt, s->cnt, 5 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s->stream));
  GHS_HIP_CHECK(hipStreamSynchronize(s->stream));
  if (s->h_cnt[4]) {
    s->phase = 2;
    GHS_FAIL(GHS_E_STATE, "internal invariant violated in round " + std::to_string(s->round + 1) + " (code " +
                              std::to_string(s->h_cnt[4]) + ")");
  }
  ghs_round_stats_t st{};
  st.level = s->level;
  st.level_arcs = s->level_round == 0 ? s->level_arcs : 0;
  st.live_arcs = s->cur_arcs;
  st.active_components = nact;
  st.hooks = s->h_cnt[3] - s->edges_before;
  s->edges_before = s->h_cnt[3];
  s->stats.push_back(st);

  // the arcs compacted by this round's min-edge kernel are the next round's input
  if (s->level_round >= 1 && s->cur_arcs) {
    s->cur ^= 1;
    s->cur_single = false;
    s->cur_arcs = s->h_cnt[0];
  }
  s->act_cur = nb;
  s->act_ident = false;
  s->nact = s->h_cnt[1];
  s->round += 1;
  s->level_round += 1;
  if (s->nact == 0) {  // level complete
    s->level_open = false;
    s->level += 1;
    const bool no_more = (s->level + 1 >= s->thresholds.size()) || (s->cfg.num_ranks <= 1 && s->rem_total == 0);
    s->phase = no_more ? 2 : 0;
  } else {
    s->phase = 0;
  }
  if (done) *done = (s->phase == 2);
  return GHS_OK;
}

int ghs_solver_finish(ghs_solver_t *s, ghs_result_t *result, ghs_round_stats_t *stats) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  if (s->phase != 2) GHS_FAIL(GHS_E_STATE, "finish before the loop terminated");
  GHS_HIP_CHECK(hipStreamSynchronize(s->stream));
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - s->t0).count();
  const uint32_t ns = (uint32_t)std::min<size_t>(s->stats.size(), GHS_MAX_ROUND_STATS);
  for (uint32_t r = 0; r < ns; ++r) {
    float t[4] = {0, 0, 0, 0};
    for (int k = 0; k < 4; ++k) {
      hipEvent_t a = round_event(s, r, k), b = round_event(s, r, k + 1);
      if (a && b) (void)hipEventElapsedTime(&t[k], a, b);
    }
    s->stats[r].ms_minedge = t[0];
    s->stats[r].ms_hook = t[1];
    s->stats[r].ms_jump = t[2];
    s->stats[r].ms_active = t[3];
    if (stats) stats[r] = s->stats[r];
  }
  if (result) {
    result->num_mst_edges = s->n ? s->h_cnt[3] : 0;
    result->total_weight = s->n ? s->h_cnt[2] : 0;
    result->rounds = s->round;
    result->num_stats = ns;
    result->levels = (uint32_t)(s->thresholds.size() - 1);
    result->ms_total = ms;
  }
  return GHS_OK;
}

int ghs_solver_destroy(ghs_solver_t *s) {
  if (!s) return GHS_OK;
  for (hipEvent_t e : s->ev_pool) (void)hipEventDestroy(e);
  if (s->h_cnt) (void)hipHostFree(s->h_cnt);
  if (s->h_sample) (void)hipHostFree(s->h_sample);
  delete s;
  return GHS_OK;
}

int ghs_mst_device(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                   const ghs_config_t *cfg, void *d_workspace, size_t workspace_bytes, uint8_t *d_in_mst, void *stream,
                   ghs_result_t *result, ghs_round_stats_t *stats) {
  std::lock_guard<std::mutex> lock(g_mutex);
  ghs_solver_t *s = nullptr;
  int rc = ghs_solver_create(n, m, d_u, d_v, d_w, 0, m, cfg, d_workspace, workspace_bytes, d_in_mst, stream, &s);
  if (rc) return rc;
  int done = (n == 0);
  while (!done) {
    if ((rc = ghs_solver_minedge(s, nullptr))) break;
    if ((rc = ghs_solver_contract(s, &done))) break;
  }
  if (!rc) rc = ghs_solver_finish(s, result, stats);
  ghs_solver_destroy(s);
  return rc;
}

}  // extern "C"
