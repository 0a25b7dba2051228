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

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace ghs {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }

constexpr uint32_t SEG_G = 2048;   // blocks of a compacting kernel (8 per CU) = output segments
constexpr uint32_t SEG_MAX = SEG_G * 4;  // segments of a wave-private output (one per wave)
// The compacting min-edge runs 6 blocks per CU (79 VGPRs): a grid of exactly 6 x 256 measured ~5%
// faster than 2048 (R-MAT s24: 1.75 vs 1.67 TB/s); the canonical passes keep 2048 (k_filter is
// fastest there).
constexpr uint32_t CMP_G = 1536;
constexpr int FIND_LAB_MAX_HOPS = 256;
// Rounds >= 1 of one rank: CONNECT in edge form (k_win over the compacted survivors, which carry
// the current roots) while live edges < EDGE_HOOK_RATIO x active fragments — lattice-like levels,
// where most fragments are still small (16384^2 grid: ~1.4 survivors per fragment) and k_hook's
// per-fragment gathers of the canonical endpoints dominate; fragment form (k_hook) otherwise.
// Chosen on the device from the exact counts; the host enqueues both only while its bound on the
// active fragments is at least EDGE_HOOK_MIN_BOUND.
#ifndef GHS_EDGE_HOOK_RATIO
#define GHS_EDGE_HOOK_RATIO 4
#endif
constexpr uint64_t EDGE_HOOK_RATIO = GHS_EDGE_HOOK_RATIO;
constexpr uint32_t HOOK_G = 2048;  // grid cap of the kernels ending in per-block total atomics
constexpr uint64_t EDGE_HOOK_MIN_BOUND = 1u << 20;
constexpr uint32_t JUMP_MAX_STEPS = 1u << 26;

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// best[c] = min(best[c], k). A plain read first: best only ever decreases, so a stale read is
// never below the true value and skipping on best <= k is always safe.
__device__ __forceinline__ void flush_min(uint64_t *__restrict__ best, uint32_t c, uint64_t k) {
  uint64_t *p = best + c;
  if (*p > k) atomicMin(reinterpret_cast<unsigned long long *>(p), (unsigned long long)k);
}

// Per-block LDS cache of fragment minima. A run tail (label L, min key k) lands in a
// direct-mapped slot: if the slot holds L (or is claimed for L now) the min is taken in LDS
// (native ds_min_u64), else it goes to best[] directly. The block flushes its slots once at the
// end. A fragment with arcs all over the stream (the giant) then costs one global update per
// block instead of one per run — same-address global operations serialise at the memory side
// (~12 ns each, MI355X_MICROARCH.md "fanin") and atomics drop the line from L2, so every later
// plain read of that slot misses too.
// k_filter: issue the random b-probe only for edges whose a-end is in the giant (1), or for
// every heavy edge beside the a-probes (0)
// k_resolve: 4 vertices per lane with their label walks interleaved — consecutive (1) or a grid
// stride apart (2) — or one per thread (0)
#ifndef GHS_RESOLVE4
#define GHS_RESOLVE4 1
#endif
#ifndef GHS_FILTER_GATED
#define GHS_FILTER_GATED 1
#endif
#ifndef GHS_HOT_BITS
#define GHS_HOT_BITS 9
#endif
constexpr int HOT_BITS = GHS_HOT_BITS;
// the compacting min-edge's parallel-edge filter: LDS pair slots per block,
// linear probes, and the host's bound on the active fragments below which the filtering variant
// is launched (it filters when the exact count is <= the solver's dedup_max: env GHS_DEDUP_MAX,
// default 0 = off — measured to cost about what it saves, DESIGN.md "Measured and rejected")
constexpr int DEDUP_SLOTS = 1024;
constexpr int DEDUP_PROBES = 16;
constexpr uint64_t DEDUP_BOUND_FACTOR = 32;
constexpr int HOT_SLOTS = 1 << HOT_BITS;

__device__ __forceinline__ void hot_init(uint32_t *s_hl, unsigned long long *s_hk) {
  for (int i = threadIdx.x; i < HOT_SLOTS; i += BLOCK) {
    s_hl[i] = LABEL_NONE;
    s_hk[i] = KEY_NONE;
  }
}

__device__ __forceinline__ void hot_min(uint32_t *s_hl, unsigned long long *s_hk, uint64_t *__restrict__ best,
                                        uint32_t L, uint64_t k) {
  const uint32_t slot = (L * 0x9E3779B1u) >> (32 - HOT_BITS);
  uint32_t cur = s_hl[slot];
  if (cur == LABEL_NONE) {
    cur = atomicCAS(&s_hl[slot], LABEL_NONE, L);
    if (cur == LABEL_NONE) cur = L;
  }
  if (cur == L)
    atomicMin(&s_hk[slot], (unsigned long long)k);
  else
    flush_min(best, L, k);
}

__device__ __forceinline__ void hot_flush(const uint32_t *s_hl, const unsigned long long *s_hk, uint64_t *__restrict__ best) {
  for (int i = threadIdx.x; i < HOT_SLOTS; i += BLOCK) {
    const uint32_t L = s_hl[i];
    if (L != LABEL_NONE && s_hk[i] != KEY_NONE) flush_min(best, L, s_hk[i]);
  }
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

// Wave-exclusive prefix sum of small per-lane counts (x < 2^B) from B ballots: bit k of every
// lane's count is one 64-bit ballot, and a lane's prefix is the sum over k of 2^k times the set bits
// below it (mbcnt). No cross-lane data movement — a shuffle scan is six dependent ds_bpermute
// round trips per tile — and the total is uniform (scalar popcounts).
template <int B>
__device__ __forceinline__ uint32_t wave_excl_small(uint32_t x, uint32_t *total) {
  uint32_t ex = 0, t = 0;
#pragma unroll
  for (int k = 0; k < B; ++k) {
    const uint64_t m = __ballot((x >> k) & 1u);
    ex += __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << k;
    t += (uint32_t)__popcll(m) << k;
  }
  *total = t;
  return ex;
}

// Wave-level offsets for a block-wide compaction step: *lane_excl = items of lower lanes of the
// wave, *wave_before = items of lower waves of the block, *wave_cnt = the wave's items,
// *total = the block's. mine < 8 (a lane's 4-entry tile). Every thread of the block must call it
// (two barriers).
template <int NT = BLOCK>
__device__ __forceinline__ void block_offsets_w(uint32_t mine, uint32_t *s_wcnt, uint32_t *lane_excl,
                                                uint32_t *wave_before, uint32_t *wave_cnt, uint32_t *total) {
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  uint32_t wc;
  *lane_excl = wave_excl_small<3>(mine, &wc);
  *wave_cnt = wc;
  if (lane == 0) s_wcnt[wid] = wc;
  __syncthreads();
  uint32_t before = 0, t = 0;
#pragma unroll
  for (int w = 0; w < NT / WAVE; ++w) {
    if (w < wid) before += s_wcnt[w];
    t += s_wcnt[w];
  }
  *wave_before = before;
  *total = t;
  __syncthreads();
}

// Two compaction streams' offsets with one pair of barriers: the per-lane counts (< 8 each; a
// block's totals < 2^16) are scanned by ballots and their wave totals packed into the two halves
// of one 32-bit LDS word, so the level / pending split of a tile costs one cross-wave step.
struct Offs2 {
  uint32_t lane_excl[2], wave_before[2], wave_cnt[2], total[2];
};
__device__ __forceinline__ Offs2 block_offsets_w2(uint32_t mine0, uint32_t mine1, uint32_t *s_wcnt) {
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  Offs2 o;
  o.lane_excl[0] = wave_excl_small<3>(mine0, &o.wave_cnt[0]);
  o.lane_excl[1] = wave_excl_small<3>(mine1, &o.wave_cnt[1]);
  if (lane == 0) s_wcnt[wid] = o.wave_cnt[0] | (o.wave_cnt[1] << 16);
  __syncthreads();
  uint32_t before = 0, t = 0;
#pragma unroll
  for (int w = 0; w < BLOCK / WAVE; ++w) {
    if (w < wid) before += s_wcnt[w];
    t += s_wcnt[w];
  }
  __syncthreads();
  o.wave_before[0] = before & 0xffffu; o.wave_before[1] = before >> 16;
  o.total[0] = t & 0xffffu;            o.total[1] = t >> 16;
  return o;
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Staged compaction of a wave's survivors: each lane puts its (<= 4) flagged items at
// lane_excl.. in the wave's private LDS region (256 entries), then the wave writes its
// contiguous output range [out, out + wave_cnt) with coalesced stores (lane i: items i, i + 64,
// ...) instead of 12 scattered per-lane stores.
// Buffer resource over [p, p + bytes) (bytes clipped to 2^31 - 1). Loads past the end return 0
// instead of faulting, so the streaming loops issue every load unconditionally: no branch around
// a load, hence no path-dependent outstanding-load count, and hipcc's waits stay counted
// (vmcnt(N)) instead of draining the prefetched tile (cdna_hip_programming.md T8/T20). Built
// from block-uniform values only.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint64_t bytes) {
  const int nb = (int)(bytes > 0x7fffffffull ? 0x7fffffffull : bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, nb, 0x00020000);
}

__device__ __forceinline__ uint4 ld_b128(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 0);
  return make_uint4(x.x, x.y, x.z, x.w);
}

// The same as a non-temporal (streaming) load: the canonical list is read once per pass, and
// default-policy lines of a 3-12 GB stream evict the L2-resident giant bitmap that the pass's
// random probes need (R-MAT s26: 8 MiB bitmap, 4 MiB L2 per XCD). cache policy bits: nt = 2.
#ifndef GHS_FILTER_NT
#define GHS_FILTER_NT 1
#endif
__device__ __forceinline__ uint4 ld_b128_nt(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, GHS_FILTER_NT ? 2 : 0);
  return make_uint4(x.x, x.y, x.z, x.w);
}

__device__ __forceinline__ uint32_t ld_b32(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, (int)byte_off, 0, 0);
}


// Buffer stores through a resource: a lane whose byte offset is >= the resource's size stores
// nothing (the bounds check drops it), so a masked store is still ONE instruction issued in
// every iteration. A streaming loop whose store count per iteration is fixed keeps hipcc's
// waits counted: with a data-dependent number of stores behind the prefetch loads it emits
// vmcnt(0) at the loop top, which also waits for every store acknowledgement.
constexpr uint32_t ST_DROP = 0xffffffffu;  // an offset past every resource
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_u32(const void *p, uint64_t bytes) {
  const uint32_t nb = (uint32_t)(bytes > 0xfffffffeull ? 0xfffffffeull : bytes);  // < ST_DROP
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)nb, 0x00020000);
}
__device__ __forceinline__ void st_b8(uint8_t v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b8(v, r, (int)off, 0, 0);
}
__device__ __forceinline__ void st_b32(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)off, 0, 0);
}
__device__ __forceinline__ void st_b64(uint64_t v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)v, (uint32_t)(v >> 32)}, r, (int)off, 0, 0);
}

// ------------------------------------------------------------------------------------------
// CSR input (ABI 9). The canonical list may come as row offsets off[0..n] (u32: m < 2^31) + v + w
// — the north_star's "CSR edge list in HBM", u implied: edge e of row r has u = r for
// off[r] <= e < off[r + 1]. The streaming passes then read 8 B per edge plus ~4 B per row instead of
// 12 B per edge.
// Per solve, the CSR pre-pass (k_csr_range, k_csr_check: off[]'s validation, k_csr_tiles,
// k_csr_bounds: the passes' cost-balanced partitions) writes trow[t] = the row holding edge
// E0 + 256 t for every 256-edge tile of the solver's range (trow[ntiles]: the row of its last edge). A streaming wave derives u for a tile [t0, t0 + 256) from R0 = trow[t] and R1 =
// trow[t + 1] (csr_tile_rows): the rows R0 + 1 .. R1 start inside the tile (or at its end); each
// writes its id into the LDS slot of its first edge (ds_max: the empty rows before a nonempty one
// share its slot), and a max-scan over the 256 slots (in-lane over a lane's 4, then a wave DPP scan)
// gives every edge its row. Slots a tile does not write hold earlier tiles' rows, all <= R0, so they
// never win the max (a private table is zeroed once per kernel, not per tile). The rows come from
// 64-row windows of off[]: the first one prefetched a tile ahead, the rest of a tile's windows
// (R1 - R0 > 64: lattices ~128; the sparse end of an R-MAT list, where high ids store few canonical
// edges, up to thousands of mostly empty rows per tile) issued 8 at a time — R1 is known up front.
// (The first version walked windows from R0 until one passed the tile's end, a dependent round trip
// per 64 rows: the waves owning the list's sparse end made k_select 1.9 ms against COO's 0.7.)
// A gather of u by edge id (the fragment-form hooks: one per hooked fragment) is a binary search
// over the edge's tile rows (trow), or over off[] for another rank's edge (csr_row), unless the
// caller also passed u (Ends).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {  // inclusive max over the wave (gfx9 DPP)
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));  // row_shr:1
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));  // row_shr:2
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));  // row_shr:4
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));  // row_shr:8
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));  // row_bcast:15
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return x;
}
// the value of lane - 1 (lane 0: 0)
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false);  // wave_shr:1
}

// the row of edge e: the largest r in [0, n - 1] with off[r] <= e (one thread, binary search)
__device__ __forceinline__ uint32_t csr_row(const uint32_t *__restrict__ off, uint32_t n, uint32_t e) {
  uint32_t lo = 0, hi = n ? n - 1 : 0;
  while (lo < hi) {
    const uint32_t mid = lo + ((hi - lo + 1) >> 1);
    if (off[mid] <= e) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// one 64-row window: lane i holds off[base + i] (0xffffffff past off[n]); the load is issued
// unconditionally (clamped index), so a caller can prefetch it
__device__ __forceinline__ uint32_t csr_win(const uint32_t *__restrict__ off, uint32_t n, uint32_t base) {
  const uint32_t r = base + (threadIdx.x & (WAVE - 1));
  const uint32_t o = off[min(r, n)];
  return r <= n ? o : 0xffffffffu;
}

// Rows of the wave tile [t0, t0 + 256): u[j] = the row of edge t0 + 4 * lane + j, from R0 (the row
// holding t0), R1 (the row holding t0 + 256, or the range's last edge) and w0 = csr_win(off, n,
// R0 + 1) (prefetched). s_head: the wave's 256-entry LDS table; CLEAR: zeroed first (a table
// sharing LDS with other per-tile data).
template <bool CLEAR>
__device__ __forceinline__ void csr_tile_rows(const uint32_t *__restrict__ off, uint32_t n, uint32_t R0, uint32_t R1,
                                              uint32_t t0, uint32_t *s_head, uint32_t u[4], uint32_t w0) {
  const uint32_t lane = threadIdx.x & (WAVE - 1), tend = t0 + 256u;
  if (CLEAR) {
    reinterpret_cast<uint4 *>(s_head)[lane] = make_uint4(0u, 0u, 0u, 0u);
    wave_sync_lds();
  }
  // rows starting strictly inside the tile (a row at t0 is R0 itself; rows past R1 start past tend)
  auto mark = [&](uint32_t o, uint32_t r) {
    if ((o > t0) & (o < tend)) atomicMax(&s_head[o - t0], r);
  };
  mark(w0, R0 + 1 + lane);
  for (uint32_t base = R0 + 1 + WAVE; base <= R1; base += 8 * WAVE) {  // more than 64 rows: up to 8 windows a trip
    const uint32_t cnt = min(8u, (R1 - base) / WAVE + 1);  // wave-uniform
    uint32_t o[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) o[k] = k < cnt ? csr_win(off, n, base + k * WAVE) : 0u;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k)
      if (k < cnt) mark(o[k], base + k * WAVE + lane);
  }
  wave_sync_lds();
  const uint4 h = reinterpret_cast<const uint4 *>(s_head)[lane];
  const uint32_t x0 = h.x, x1 = max(x0, h.y), x2 = max(x1, h.z), x3 = max(x2, h.w);
  const uint32_t base = max(R0, wave_shr1(wave_incl_max(x3)));
  u[0] = max(base, x0);
  u[1] = max(base, x1);
  u[2] = max(base, x2);
  u[3] = max(base, x3);
}

// canonical endpoints by edge id (the fragment-form hooks, the plan's span sample): u from the
// caller's u array, or — CSR input without one — a binary search over the row offsets
struct Ends {
  const uint32_t *u;     // nullptr: CSR input
  const uint32_t *off;   // CSR row offsets (n + 1 entries)
  const uint32_t *v;
  uint32_t n;
  const uint32_t *trow;  // CSR: the rows of the solver's 256-edge tiles (k_csr_tiles), nullptr before it ran
  uint64_t E0, E1;       // ... its edges [E0, E1) (trow[ntiles] is the row of edge E1 - 1: edges of the
                         // last tile past E1 are another rank's, their rows may lie beyond it)
};
__device__ __forceinline__ uint32_t end_u(const Ends &E, uint32_t eid) {
  if (E.u) return E.u[eid];
  // an edge of the solver's range: its tile's rows bound the search (~16 rows at s24: 4 steps, not 24)
  if (E.trow && eid >= E.E0 && eid < E.E1) {
    const uint64_t t = (eid - E.E0) >> 8;
    uint32_t hi = min(E.trow[t + 1], E.n - 1), lo = min(E.trow[t], hi);  // clamped: malformed offsets (err 8)
    while (lo < hi) {
      const uint32_t mid = lo + ((hi - lo + 1) >> 1);
      if (E.off[mid] <= eid) lo = mid; else hi = mid - 1;
    }
    return lo;
  }
  return csr_row(E.off, E.n, eid);
}

struct WaveStage {
  uint32_t a[WAVE * 4];
  uint32_t b[WAVE * 4];
  uint64_t k[WAVE * 4];
};

__device__ __forceinline__ void stage_write(WaveStage &ws, const uint32_t a[4], const uint32_t b[4], const uint64_t k[4],
                                            uint32_t mask, uint32_t lane_excl, uint32_t wave_cnt,
                                            uint32_t *__restrict__ oa, uint32_t *__restrict__ ob,
                                            uint64_t *__restrict__ ok, uint64_t out) {
  uint32_t p = lane_excl;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (mask & (1u << j)) {
      ws.a[p] = a[j];
      ws.b[p] = b[j];
      ws.k[p] = k[j];
      ++p;
    }
  }
  wave_sync_lds();
  const int lane = threadIdx.x & (WAVE - 1);
  for (uint32_t i = lane; i < wave_cnt; i += WAVE) {
    oa[out + i] = ws.a[i];
    ob[out + i] = ws.b[i];
    ok[out + i] = ws.k[i];
  }
  wave_sync_lds();  // the region is rewritten next iteration
}

// The same with a fixed store count: 4 rounds of 64 lanes (a wave stages <= 256 entries) to the
// block's output region through resources based at the region (ra/rb: 4-B entries, rk: 8-B
// keys); rel = the wave's first entry relative to the region. Lanes past wave_cnt drop.
__device__ __forceinline__ void stage_write_rs(WaveStage &ws, const uint32_t a[4], const uint32_t b[4],
                                               const uint64_t k[4], uint32_t mask, uint32_t lane_excl,
                                               uint32_t wave_cnt, __amdgpu_buffer_rsrc_t ra,
                                               __amdgpu_buffer_rsrc_t rb, __amdgpu_buffer_rsrc_t rk, uint32_t rel) {
  uint32_t p = lane_excl;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (mask & (1u << j)) {
      ws.a[p] = a[j];
      ws.b[p] = b[j];
      ws.k[p] = k[j];
      ++p;
    }
  }
  wave_sync_lds();
  const uint32_t lane = threadIdx.x & (WAVE - 1);
#pragma unroll
  for (uint32_t r = 0; r < 4; ++r) {
    const uint32_t i = lane + WAVE * r;
    const bool ok = i < wave_cnt;
    const uint32_t e = rel + i;
    st_b32(ws.a[i], ra, ok ? e * 4u : ST_DROP);
    st_b32(ws.b[i], rb, ok ? e * 4u : ST_DROP);
    st_b64(ws.k[i], rk, ok ? e * 8u : ST_DROP);
  }
  wave_sync_lds();  // the region is rewritten next iteration
}

// ------------------------------------------------------------------------------------------
// Wave-private sparse output. A streaming kernel whose waves each own a contiguous slice of the
// input also owns the same slice of the output (one segment per wave). Survivors of each
// 256-edge wave tile are appended to the wave's LDS buffer (WaveStage, 256 entries); the
// buffer goes to the output only when the next tile might not fit: full 64-lane stores, every
// ~30 tiles at level-0 selectivity instead of a block-wide offset computation (two barriers)
// and a staging round per tile. Measured: the per-tile staging was ~19% of k_select.
// ------------------------------------------------------------------------------------------
struct WaveOut {
  uint32_t cnt = 0;   // entries in the LDS buffer (wave-uniform)
  uint64_t pos = 0;   // next output index of the wave's slice
};

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t *total) {
  const int lane = threadIdx.x & (WAVE - 1);
  uint32_t incl = x;
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const uint32_t o = __shfl_up(incl, d);
    if (lane >= d) incl += o;
  }
  *total = __shfl(incl, WAVE - 1);
  return incl - x;
}

__device__ __forceinline__ void wave_flush(WaveStage &ws, WaveOut &wo, uint32_t *__restrict__ oa, uint32_t *__restrict__ ob,
                                           uint64_t *__restrict__ ok) {
  wave_sync_lds();
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  for (uint32_t i = lane; i < wo.cnt; i += WAVE) {
    oa[wo.pos + i] = ws.a[i];
    ob[wo.pos + i] = ws.b[i];
    ok[wo.pos + i] = ws.k[i];
  }
  wave_sync_lds();  // the buffer is refilled next
  wo.pos += wo.cnt;
  wo.cnt = 0;
}

__device__ __forceinline__ void wave_append(WaveStage &ws, WaveOut &wo, const uint32_t a[4], const uint32_t b[4],
                                            const uint64_t k[4], uint32_t mask, uint32_t *__restrict__ oa,
                                            uint32_t *__restrict__ ob, uint64_t *__restrict__ ok) {
  uint32_t tile;
  const uint32_t ex = wave_excl_small<3>((uint32_t)__popc(mask), &tile);
  if (tile == 0) return;
  if (wo.cnt + tile > WAVE * 4) wave_flush(ws, wo, oa, ob, ok);
  uint32_t p = wo.cnt + ex;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (mask & (1u << j)) {
      ws.a[p] = a[j];
      ws.b[p] = b[j];
      ws.k[p] = k[j];
      ++p;
    }
  }
  wo.cnt += tile;
}

// the wave's last flush, padding to a multiple of 4 with dead entries, and its segment entry
__device__ __forceinline__ void wave_finish(WaveStage &ws, WaveOut &wo, uint32_t *__restrict__ oa,
                                            uint32_t *__restrict__ ob, uint64_t *__restrict__ ok, uint64_t seg_begin,
                                            bool has_range, uint64_t *__restrict__ ostart, uint64_t *__restrict__ ocount,
                                            uint32_t seg) {
  if (wo.cnt) wave_flush(ws, wo, oa, ob, ok);
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t n = wo.pos - seg_begin, padded = (n + 3) & ~3ull;
  if (lane < padded - n) {
    oa[wo.pos + lane] = LABEL_NONE;
    ob[wo.pos + lane] = 0;
    ok[wo.pos + lane] = KEY_NONE;
  }
  if (lane == 0) {
    ostart[seg] = seg_begin;
    ocount[seg] = has_range ? padded : 0;
  }
}

// ------------------------------------------------------------------------------------------
// Segmented input: virtual index v in [0, total) lives in segment s with
// prefix[s] <= v < prefix[s+1], physical index start[s] + (v - prefix[s]).
// ------------------------------------------------------------------------------------------
struct SegView {
  const uint64_t *start;
  const uint64_t *prefix;  // nseg + 1 entries; prefix[nseg] = the virtual total (device-side)
  uint32_t nseg;
};

__device__ __forceinline__ uint32_t seg_find(const uint64_t *__restrict__ prefix, uint32_t lo, uint32_t hi, uint64_t v) {
  // largest s in [lo, hi] with prefix[s] <= v
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= v) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// The same search by one full wave (every lane of it calls): a 64-ary search — each step one load
// per lane and a ballot — so nseg <= 4096 takes 2 dependent loads and SEG_MAX 3, where the binary
// search by one thread took ~13, all of them on the critical path of a streaming kernel's first
// tile (the block waits on them at its first barrier). Both ends of a block's range at once.
__device__ __forceinline__ void seg_find_wave2(const uint64_t *__restrict__ prefix, uint32_t nseg, uint64_t v0,
                                               uint64_t v1, uint32_t *r0, uint32_t *r1) {
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  uint32_t lo0 = 0, c0 = nseg, lo1 = 0, c1 = nseg;  // candidates [lo, lo + c): prefix[lo] <= v
  while (c0 > 1 || c1 > 1) {
    const uint32_t st0 = (c0 + WAVE - 1) / WAVE, st1 = (c1 + WAVE - 1) / WAVE;
    const bool in0 = c0 > 1 && lane * st0 < c0, in1 = c1 > 1 && lane * st1 < c1;
    const uint64_t p0 = in0 ? prefix[lo0 + lane * st0] : ~0ull;
    const uint64_t p1 = in1 ? prefix[lo1 + lane * st1] : ~0ull;
    const uint64_t m0 = __ballot(in0 && p0 <= v0), m1 = __ballot(in1 && p1 <= v1);
    if (c0 > 1) {  // m0 has lane 0's bit: prefix[lo0] <= v0
      const uint32_t L = 63u - (uint32_t)__clzll((long long)m0);
      lo0 += L * st0;
      c0 = min(st0, c0 - L * st0);
    }
    if (c1 > 1) {
      const uint32_t L = 63u - (uint32_t)__clzll((long long)m1);
      lo1 += L * st1;
      c1 = min(st1, c1 - L * st1);
    }
  }
  *r0 = lo0;
  *r1 = lo1;
}

// a block's range [vb, ve) of T virtual entries -> its first and last region (wave 0 calls)
__device__ __forceinline__ void seg_range_wave(const uint64_t *__restrict__ prefix, uint32_t nseg, uint64_t vb,
                                               uint64_t ve, uint64_t T, uint32_t *s_seg) {
  uint32_t a = 0, b = 0;
  seg_find_wave2(prefix, nseg, vb < T ? vb : 0, ve > vb ? ve - 1 : 0, &a, &b);
  if (threadIdx.x == 0) {
    s_seg[0] = vb < T ? a : 0;
    s_seg[1] = ve > vb ? b : 0;
  }
}

// ------------------------------------------------------------------------------------------
// Segmented edge input: every region holds a multiple of 4 entries and starts at a multiple of
// 4 (dead entries, a == LABEL_NONE, pad the regions), so a lane's 4-entry tile at a virtual
// index v (a multiple of 4) lies wholly inside one region. Tiles past the block's range read
// the tile at index 0 (always allocated) and are masked, so every load is unconditional.
// ------------------------------------------------------------------------------------------
struct EdgeTile {
  uint4 a, b;
  ulonglong2 k01, k23;
};

__device__ __forceinline__ uint64_t tile_phys(const SegView &in, uint32_t slo, uint32_t shi, uint64_t v, uint64_t ve) {
  if (v >= ve) return 0;
  const uint32_t sidx = (slo == shi) ? slo : seg_find(in.prefix, slo, shi, v);
  return in.start[sidx] + (v - in.prefix[sidx]);
}

__device__ __forceinline__ void tile_load(EdgeTile &t, const uint32_t *__restrict__ ea, const uint32_t *__restrict__ eb,
                                          const uint64_t *__restrict__ ek, uint64_t i0) {
  t.a = *reinterpret_cast<const uint4 *>(ea + i0);
  t.b = *reinterpret_cast<const uint4 *>(eb + i0);
  t.k01 = *reinterpret_cast<const ulonglong2 *>(ek + i0);
  t.k23 = *reinterpret_cast<const ulonglong2 *>(ek + i0 + 2);
}

// ------------------------------------------------------------------------------------------
// Stage 1: minimum outgoing edge per fragment (+ fused REJECT filter / stream compaction),
// edge-centric: every live edge (a, b, key) of the level is a candidate for BOTH fragments.
//  a-side: the edges keep the canonical order (grouped by the a vertex), so equal a labels form
//    runs; a wave-wide segmented min-scan over its 256 edges (in-lane serial + 6-step cross-lane
//    scan) leaves one candidate per run, and only run tails touch the fragment minima.
//  b-side: one candidate per edge.
// Candidates go through the block's LDS cache (hot_min) and then best[] — after a plain read,
// since best only ever decreases (a stale read is never smaller than the true value, so skipping
// on `best <= cand` is always safe).
// IDENT: labels are already current roots (a level's first round): no label gathers.
// COMPACT: survivors (inter-fragment edges) are written relabelled to this block's output
// region (padded to a multiple of 4 with dead entries).
// ------------------------------------------------------------------------------------------
template <bool IDENT, bool COMPACT, bool DEDUP = false, bool CAND = true>
GHS_STREAM_KERNEL_6 void k_minedge(const uint32_t *__restrict__ src, const uint32_t *__restrict__ dst,
                                 const uint64_t *__restrict__ key, SegView in, const uint32_t *__restrict__ lab,
                                 uint64_t *__restrict__ best, uint32_t *__restrict__ osrc, uint32_t *__restrict__ odst,
                                 uint64_t *__restrict__ okey, uint64_t *__restrict__ oseg_start,
                                 uint64_t *__restrict__ oseg_count, bool aside,
                                 const unsigned long long *__restrict__ guard_nact,
                                 const unsigned long long *__restrict__ dedup_nact = nullptr, uint32_t dedup_max = 0) {
  __shared__ uint32_t s_wcnt[BLOCK / WAVE];
  __shared__ uint32_t s_seg[2];
  __shared__ uint32_t s_hl[CAND ? HOT_SLOTS : 1];
  __shared__ unsigned long long s_hk[CAND ? HOT_SLOTS : 1];
  __shared__ WaveStage s_stage[COMPACT ? BLOCK / WAVE : 1];
  __shared__ unsigned long long s_dp[DEDUP ? DEDUP_SLOTS : 1];  // fragment pair lo << 32 | hi
  __shared__ unsigned long long s_dk[DEDUP ? DEDUP_SLOTS : 1];  // its minimum key in this block
  const int lane = threadIdx.x & (WAVE - 1);
  // parallel-edge filter (DEDUP, few active fragments): survivors between the same two fragments
  // keep only their minimum key per block (the heavier ones close a cycle with it: never in the
  // MSF); the pairs live in an LDS hash and are emitted once at the end of the block
  const bool dd = DEDUP && *dedup_nact <= dedup_max;
  if (DEDUP) {
    for (int i = threadIdx.x; i < DEDUP_SLOTS; i += BLOCK) {
      s_dp[i] = ~0ull;
      s_dk[i] = KEY_NONE;
    }
  }
  // a pipelined single-rank level runs one round ahead of the host's termination check: a round
  // that starts with <= 1 active fragment is such a discarded lookahead round (the level is
  // complete) — its blocks write empty regions instead of streaming every remaining edge
  const bool noop = COMPACT && guard_nact && *guard_nact <= 1;
  const uint64_t T = noop ? 0 : in.prefix[in.nseg];
  if (CAND) hot_init(s_hl, s_hk);
  const uint64_t Q = ((T + gridDim.x - 1) / gridDim.x + 3) & ~3ull;  // multiple of 4
  const uint64_t vb = Q * blockIdx.x;
  const uint64_t ve = (vb + Q < T) ? vb + Q : T;
  if (threadIdx.x < WAVE) seg_range_wave(in.prefix, in.nseg, vb, ve, T, s_seg);
  __syncthreads();
  const uint32_t slo = s_seg[0], shi = s_seg[1];
  uint64_t out_n = 0;  // survivors written so far by this block
  uint32_t carry_l = LABEL_NONE;  // wave-uniform deferred a-side run (label, min key)
  uint64_t carry_v = KEY_NONE;
  EdgeTile cur, nxt;
  tile_load(cur, src, dst, key, tile_phys(in, slo, shi, vb + (uint64_t)threadIdx.x * ARCS_PER_THREAD, ve));

  for (uint64_t v0 = vb; v0 < ve; v0 += ARCS_PER_BLOCK) {
    const uint64_t v = v0 + (uint64_t)threadIdx.x * ARCS_PER_THREAD;
    const bool in_range = v < ve;
    uint32_t L[4] = {cur.a.x, cur.a.y, cur.a.z, cur.a.w};
    uint32_t D[4] = {cur.b.x, cur.b.y, cur.b.z, cur.b.w};
    const uint64_t K[4] = {cur.k01.x, cur.k01.y, cur.k23.x, cur.k23.y};
    bool valid[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) valid[j] = in_range & (L[j] != LABEL_NONE);
    uint32_t cs[4], cd[4];
    if (!IDENT) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // 8 independent gathers in flight per lane
        cs[j] = lab[valid[j] ? L[j] : 0u];
        cd[j] = lab[valid[j] ? D[j] : 0u];
      }
    }
    tile_load(nxt, src, dst, key, tile_phys(in, slo, shi, v + ARCS_PER_BLOCK, ve));
    uint64_t V[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!IDENT) {
        L[j] = valid[j] ? cs[j] : LABEL_NONE;
        D[j] = cd[j];
        V[j] = (valid[j] & (cs[j] != cd[j])) ? K[j] : KEY_NONE;
      } else {
        if (!valid[j]) L[j] = LABEL_NONE;
        V[j] = valid[j] ? K[j] : KEY_NONE;  // level edges: a != b
      }
    }

    uint32_t smask = 0;  // survivors (inter-fragment edges), taken before the carry merge
#pragma unroll
    for (int j = 0; j < 4; ++j) smask |= (V[j] != KEY_NONE) ? (1u << j) : 0u;
    // b-side: one candidate per live edge
    if (CAND) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (smask & (1u << j)) hot_min(s_hl, s_hk, best, D[j], V[j]);
    }
    if (CAND && aside) {
    // a-side. Deferred run of the previous iteration (wave-uniform carry): a run that reaches
    // the wave's end is not flushed but carried, and merged into the next run of the same label
    // (min is associative, contiguity is not needed).
    uint64_t X[4] = {V[0], V[1], V[2], V[3]};
    if (lane == 0 && L[0] == carry_l && carry_l != LABEL_NONE) {
      X[0] = umin64(X[0], carry_v);
      carry_l = LABEL_NONE;  // merged
    }
    carry_l = __shfl(carry_l, 0);
    if (carry_l != LABEL_NONE && lane == 0) hot_min(s_hl, s_hk, best, carry_l, carry_v);  // not merged
    carry_l = LABEL_NONE;

    // ---- wave-wide segmented min over 256 edges, segments = runs of equal a label
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
      x = H[j] ? X[j] : umin64(x, X[j]);
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
      run = H[j] ? X[j] : umin64(run, X[j]);
      const bool wave_end = (j == 3) && (lane == WAVE - 1);
      const bool tail = (j < 3) ? H[j + 1] : (lane == WAVE - 1 || nextH0);
      if (tail && !wave_end && run != KEY_NONE) hot_min(s_hl, s_hk, best, L[j], run);
      if (wave_end) {
        carry_l = (run != KEY_NONE) ? L[3] : LABEL_NONE;
        carry_v = run;
      }
    }
    carry_l = __shfl(carry_l, WAVE - 1);
    carry_v = __shfl(carry_v, WAVE - 1);
    }  // aside

    if (COMPACT) {
      if (DEDUP && dd) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (smask & (1u << j)) {
            const uint32_t lo = L[j] < D[j] ? L[j] : D[j], hi = L[j] < D[j] ? D[j] : L[j];
            const unsigned long long pk = ((unsigned long long)lo << 32) | hi;
            uint32_t slot = mix32(lo ^ (hi * 0x9E3779B1u)) & (DEDUP_SLOTS - 1);
            for (int t = 0; t < DEDUP_PROBES; ++t) {
              unsigned long long cur = s_dp[slot];
              if (cur == ~0ull) {
                cur = atomicCAS(&s_dp[slot], ~0ull, pk);
                if (cur == ~0ull) cur = pk;
              }
              if (cur == pk) {  // a plain read first: few pairs means many lanes on one slot
                if ((unsigned long long)K[j] < s_dk[slot]) atomicMin(&s_dk[slot], (unsigned long long)K[j]);
                smask &= ~(1u << j);  // absorbed; a full neighbourhood leaves it to the stream
                break;
              }
              slot = (slot + 1) & (DEDUP_SLOTS - 1);
            }
          }
        }
      }
      uint32_t lane_excl, wave_before, wave_cnt, total;
      block_offsets_w((uint32_t)__popc(smask), s_wcnt, &lane_excl, &wave_before, &wave_cnt, &total);
      stage_write(s_stage[threadIdx.x / WAVE], L, D, K, smask, lane_excl, wave_cnt, osrc, odst, okey,
                  vb + out_n + wave_before);
      out_n += total;
    }
    cur = nxt;
  }
  if (CAND) {
    if (lane == 0 && carry_l != LABEL_NONE) hot_min(s_hl, s_hk, best, carry_l, carry_v);
    __syncthreads();
    hot_flush(s_hl, s_hk, best);
  }
  if (DEDUP && dd) {  // the block's pair minima join its survivors (4 slots per lane per pass)
    for (int base = 0; base < DEDUP_SLOTS; base += BLOCK * 4) {
      uint32_t L[4], D[4], dmask = 0;
      uint64_t K[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = base + threadIdx.x * 4 + j;
        const unsigned long long pk = i < DEDUP_SLOTS ? s_dp[i] : ~0ull;
        L[j] = (uint32_t)(pk >> 32);
        D[j] = (uint32_t)pk;
        K[j] = i < DEDUP_SLOTS ? s_dk[i] : KEY_NONE;
        dmask |= (pk != ~0ull) ? (1u << j) : 0u;
      }
      uint32_t lane_excl, wave_before, wave_cnt, total;
      block_offsets_w((uint32_t)__popc(dmask), s_wcnt, &lane_excl, &wave_before, &wave_cnt, &total);
      stage_write(s_stage[threadIdx.x / WAVE], L, D, K, dmask, lane_excl, wave_cnt, osrc, odst, okey,
                  vb + out_n + wave_before);
      out_n += total;
    }
  }
  if (COMPACT) {
    // pad to a multiple of 4 with dead entries; stays inside [vb, vb + Q) and below the capacity
    // (the workspace reserves 4 * SEG_MAX spare entries)
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


// ------------------------------------------------------------------------------------------
// Level 0, round 0, a-side only (the b-side follows in k_minedge<IDENT> with aside = false).
// At level 0 a label IS the vertex, and the canonical order holds each vertex's a-edges as ONE
// run, so a run whose head and tail both lie inside a wave tile (their neighbours valid and
// different) has a single writer: its minimum goes to best[] with a plain store — no LDS cache,
// no read, no atomic. A run touching the tile's first or last entry, or a padding entry (a run
// cut by a region end), may have a second piece elsewhere and takes the atomic path. Every store
// here lands before the b-side's atomics (next launch). On a 16384^2 grid this removes about half
// of round 0's global atomics (one a-run per vertex).
// ------------------------------------------------------------------------------------------
GHS_STREAM_KERNEL_6 void k_seed_runs(const uint32_t *__restrict__ src, const uint64_t *__restrict__ key, SegView in,
                                     uint64_t *__restrict__ best) {
  __shared__ uint32_t s_seg[2];
  const int lane = threadIdx.x & (WAVE - 1);
  const uint64_t T = in.prefix[in.nseg];
  const uint64_t Q = ((T + gridDim.x - 1) / gridDim.x + 3) & ~3ull;
  const uint64_t vb = Q * blockIdx.x;
  const uint64_t ve = (vb + Q < T) ? vb + Q : T;
  if (threadIdx.x < WAVE) seg_range_wave(in.prefix, in.nseg, vb, ve, T, s_seg);
  __syncthreads();
  const uint32_t slo = s_seg[0], shi = s_seg[1];
  uint64_t ph = tile_phys(in, slo, shi, vb + (uint64_t)threadIdx.x * 4, ve);
  uint4 ca = *reinterpret_cast<const uint4 *>(src + ph);
  ulonglong2 c01 = *reinterpret_cast<const ulonglong2 *>(key + ph), c23 = *reinterpret_cast<const ulonglong2 *>(key + ph + 2);
  for (uint64_t v0 = vb; v0 < ve; v0 += ARCS_PER_BLOCK) {
    const uint64_t v = v0 + (uint64_t)threadIdx.x * 4;
    const bool in_range = v < ve;
    uint32_t L[4] = {ca.x, ca.y, ca.z, ca.w};
    const uint64_t K[4] = {c01.x, c01.y, c23.x, c23.y};
    const uint64_t pn = tile_phys(in, slo, shi, v + ARCS_PER_BLOCK, ve);
    ca = *reinterpret_cast<const uint4 *>(src + pn);
    c01 = *reinterpret_cast<const ulonglong2 *>(key + pn);
    c23 = *reinterpret_cast<const ulonglong2 *>(key + pn + 2);
    uint64_t X[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!in_range) L[j] = LABEL_NONE;
      X[j] = (L[j] != LABEL_NONE) ? K[j] : KEY_NONE;
    }
    const uint32_t prevL3 = __shfl_up(L[3], 1);
    const uint32_t nextL0 = __shfl_down(L[0], 1);
    bool H[4], TH[4], TT[4];
    H[0] = (lane == 0) || (L[0] != prevL3);
    TH[0] = (lane != 0) && (L[0] != prevL3) && (prevL3 != LABEL_NONE);
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      H[j] = L[j] != L[j - 1];
      TH[j] = H[j] && (L[j - 1] != LABEL_NONE);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) TT[j] = (L[j + 1] != L[j]) && (L[j + 1] != LABEL_NONE);
    TT[3] = (lane != WAVE - 1) && (nextL0 != L[3]) && (nextL0 != LABEL_NONE);
    // segmented min over runs (heads reset), carrying "the run's head is untrusted"
    uint64_t x = KEY_NONE;
    int f = 0, uu = 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x = H[j] ? X[j] : umin64(x, X[j]);
      uu = H[j] ? (TH[j] ? 0 : 1) : uu;
      f |= H[j] ? 1 : 0;
    }
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
      const uint64_t xo = __shfl_up(x, d);
      const int fo = __shfl_up(f, d);
      const int uo = __shfl_up(uu, d);
      if (lane >= d && !f) {
        x = umin64(x, xo);
        uu = uo;
      }
      if (lane >= d) f |= fo;
    }
    uint64_t run = __shfl_up(x, 1);
    int ru = __shfl_up(uu, 1);
    if (lane == 0) {
      run = KEY_NONE;
      ru = 1;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      run = H[j] ? X[j] : umin64(run, X[j]);
      ru = H[j] ? (TH[j] ? 0 : 1) : ru;
      // a run continuing into the next lane is finished there (the scan carries its minimum)
      const bool tail = (j < 3) ? (L[j + 1] != L[j]) : (lane == WAVE - 1 || nextL0 != L[3]);
      if (tail && run != KEY_NONE && L[j] != LABEL_NONE) {
        if (!ru && TT[j]) best[L[j]] = run;   // whole run inside the tile: the only writer
        else flush_min(best, L[j], run);      // a piece of a run: atomic
      }
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

// Dense label of an active root x (several ranks, dense levels): its rank among the level's
// active flags = chunk prefix + word prefix + the flags below x in its 64-bit word. The three
// tables (12 B per 64 vertices: 12 MB at s26) replace a vertex-sized position map (268 MB) whose
// random reads went to HBM.
// pk (k_rank_pack): the same per word in one 16-B entry {bits lo, bits hi, flags below the word}
// — one random gather per lookup instead of two (bits, wpre; cpre is 4 KiB at s26, cache-resident)
struct DenseRank {
  const uint64_t *bits = nullptr;  // active flags, 64 vertices per word
  const uint32_t *wpre = nullptr;  // flags below the word, within its chunk of 256 words
  const uint32_t *cpre = nullptr;  // flags below the chunk
  const uint4 *pk = nullptr;       // packed (nullptr: the three tables)
};
__device__ __forceinline__ uint32_t dense_rank(const DenseRank &r, uint32_t x) {
  const uint32_t w = x >> 6;
  const uint64_t below = (1ull << (x & 63)) - 1;
  if (r.pk) {
    const uint4 q = r.pk[w];
    return q.z + (uint32_t)__popcll((((uint64_t)q.y << 32) | q.x) & below);
  }
  return r.cpre[w >> 8] + r.wpre[w] + (uint32_t)__popcll(r.bits[w] & below);
}

__global__ void k_rank_pack(const uint64_t *__restrict__ bits, const uint32_t *__restrict__ wpre,
                            const uint32_t *__restrict__ cpre, uint64_t words, uint4 *__restrict__ pk) {
  for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < words; w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = bits[w];
    pk[w] = make_uint4((uint32_t)b, (uint32_t)(b >> 32), cpre[w >> 8] + wpre[w], 0u);
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
// Exclusive scan of count[0..n) into prefix[0..n] (prefix[n] = *total) by ONE 256-thread block.
// k_hook's last block runs it for the compaction of the same round (the consumers — the next
// round's min-edge and the round report — run later), which saves a launch per round.
__device__ void block_scan_counts(const uint64_t *__restrict__ count, uint32_t n, uint64_t *__restrict__ prefix,
                                  unsigned long long *__restrict__ total) {
  __shared__ uint64_t s_part[BLOCK];
  const uint32_t per = (n + BLOCK - 1) / BLOCK;
  const uint32_t b = threadIdx.x * per;
  uint64_t sum = 0;
  for (uint32_t i = 0; i < per && b + i < n; ++i) sum += count[b + i];
  s_part[threadIdx.x] = sum;
  __syncthreads();
  for (int d = 1; d < BLOCK; d <<= 1) {
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
  if (threadIdx.x == BLOCK - 1) {
    prefix[n] = s_part[BLOCK - 1];
    *total = s_part[BLOCK - 1];
  }
}

__global__ __launch_bounds__(BLOCK) void k_hook(const uint32_t *__restrict__ act, const unsigned long long *__restrict__ d_nact,
                                                const uint64_t *__restrict__ best, const uint32_t *__restrict__ lab,
                                                const Ends E, uint32_t *__restrict__ par, uint8_t *__restrict__ in_mst,
                                                unsigned long long *__restrict__ acc /* [0] weight, [1] edges */,
                                                unsigned long long *__restrict__ err,
                                                const uint64_t *__restrict__ scan_count, uint32_t scan_n,
                                                uint64_t *__restrict__ scan_prefix, unsigned long long *__restrict__ scan_total,
                                                bool resolved, const unsigned long long *__restrict__ guard_live,
                                                uint32_t own_lo, uint32_t own_hi,
                                                const uint32_t *__restrict__ vlab, DenseRank dr) {
  __shared__ unsigned long long s_w[BLOCK / WAVE], s_c[BLOCK / WAVE];
  unsigned long long wsum = 0, cnt = 0;
  const uint64_t nact = *d_nact;
  if (guard_live && *guard_live < EDGE_HOOK_RATIO * nact) return;  // k_win of this round hooks
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < nact; i += (uint64_t)gridDim.x * BLOCK) {
    const uint32_t c = act ? act[i] : (uint32_t)i;
    const uint64_t k = best[c];
    uint32_t p = c;
    if (k != KEY_NONE) {
      const uint32_t eid = (uint32_t)k;
      // a level's first round: k_resolve left every label a root (one read, no walk). A dense level
      // (several ranks): an endpoint's level-open root vlab[x] (resolved), its dense label
      // dense_rank(vlab[x]), then the walk through the dense labels
      uint32_t xa = end_u(E, eid), xb = E.v[eid];
      if (dr.bits) {
        xa = dense_rank(dr, vlab[xa]);
        xb = dense_rank(dr, vlab[xb]);
      }
      const uint32_t la = resolved ? lab[xa] : find_lab(lab, xa, err);
      const uint32_t lb = resolved ? lab[xb] : find_lab(lab, xb, err);
      if (la != c && lb != c) atomicOr(err, 2ull);  // the chosen edge must leave c
      const uint32_t other = (la == c) ? lb : la;
      const bool mutual = best[other] == k;
      if (!(mutual && c < other)) {
        p = other;
        // several ranks: each marks only the MSF flags of its own edge range [own_lo, own_hi)
        // (the totals count every hook on every rank)
        if (eid >= own_lo && eid < own_hi) in_mst[eid] = 1;
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
  if (scan_count && blockIdx.x == gridDim.x - 1) block_scan_counts(scan_count, scan_n, scan_prefix, scan_total);
}

// ------------------------------------------------------------------------------------------
// Stage 2, edge form (single rank, many small fragments): every live edge (a, b, key) whose key
// is the best of a fragment is that fragment's CONNECT edge — no gathers of the canonical
// endpoints and no label walks (the edge already carries the current roots). A fragment c hooks
// to the other end o unless the pair is mutual and c < o (the smaller label stays root, as in
// k_hook). par[c] == c holds for every active root, so only hooking fragments are written.
// ------------------------------------------------------------------------------------------
GHS_STREAM_KERNEL_6 void k_win(const uint32_t *__restrict__ src, const uint32_t *__restrict__ dst,
                             const uint64_t *__restrict__ key, SegView in, const uint64_t *__restrict__ best,
                             uint32_t *__restrict__ par, uint8_t *__restrict__ in_mst,
                             unsigned long long *__restrict__ acc /* [0] weight, [1] edges; nullptr: par only */,
                             const unsigned long long *__restrict__ guard_nact) {
  __shared__ uint32_t s_seg[2];
  __shared__ unsigned long long s_w[BLOCK / WAVE], s_c[BLOCK / WAVE];
  const uint64_t T = in.prefix[in.nseg];
  // device-side choice of the CONNECT form (rounds >= 1): the edge form only while the live
  // edges are fewer than EDGE_HOOK_RATIO x the active fragments (k_hook takes the other case)
  if (guard_nact && T >= EDGE_HOOK_RATIO * *guard_nact) return;
  const uint64_t Q = ((T + gridDim.x - 1) / gridDim.x + 3) & ~3ull;
  const uint64_t vb = Q * blockIdx.x;
  const uint64_t ve = (vb + Q < T) ? vb + Q : T;
  if (threadIdx.x < WAVE) seg_range_wave(in.prefix, in.nseg, vb, ve, T, s_seg);
  __syncthreads();
  const uint32_t slo = s_seg[0], shi = s_seg[1];
  unsigned long long wsum = 0, cnt = 0;
  EdgeTile cur, nxt;
  tile_load(cur, src, dst, key, tile_phys(in, slo, shi, vb + (uint64_t)threadIdx.x * 4, ve));
  for (uint64_t v0 = vb; v0 < ve; v0 += ARCS_PER_BLOCK) {
    const uint64_t v = v0 + (uint64_t)threadIdx.x * 4;
    const bool in_range = v < ve;
    const uint32_t A[4] = {cur.a.x, cur.a.y, cur.a.z, cur.a.w}, B[4] = {cur.b.x, cur.b.y, cur.b.z, cur.b.w};
    const uint64_t K[4] = {cur.k01.x, cur.k01.y, cur.k23.x, cur.k23.y};
    bool live[4];
    uint64_t ba[4], bb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      live[j] = in_range & (A[j] != LABEL_NONE);
      ba[j] = best[live[j] ? A[j] : 0u];
      bb[j] = best[live[j] ? B[j] : 0u];
    }
    tile_load(nxt, src, dst, key, tile_phys(in, slo, shi, v + ARCS_PER_BLOCK, ve));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool wa = live[j] & (ba[j] == K[j]), wb = live[j] & (bb[j] == K[j]);
      const bool ha = wa & !(wb & (A[j] < B[j]));  // a hooks to b
      const bool hb = wb & !(wa & (B[j] < A[j]));  // b hooks to a
      if (ha) par[A[j]] = B[j];
      if (hb) par[B[j]] = A[j];
      if (ha | hb) {
        in_mst[(uint32_t)K[j]] = 1;  // with acc == nullptr: the owner rank's mark (see k_unpack_hook)
        wsum += K[j] >> 32;
        cnt += 1;
      }
    }
    cur = nxt;
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
  if (threadIdx.x == 0 && acc) {
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

// Multi-rank CONNECT of a level's first round, owner-computes: every winning edge lives on exactly
// one rank, whose k_win (acc == nullptr) set par[c] = other for the fragments it holds the winner
// of. The dense slot of active fragment c carries par[c] ^ c — 0 on every other rank, so a MAX
// all-reduce yields the hook of every fragment on every rank (4 bytes per slot instead of
// k_hook's ~5 random gathers per fragment: the canonical endpoints, their labels, best[other]).
__global__ void k_pack_hook(const uint32_t *__restrict__ act, const unsigned long long *__restrict__ d_nact,
                            const uint32_t *__restrict__ par, int32_t *__restrict__ dense) {
  const uint64_t nact = *d_nact;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nact; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = act ? act[i] : (uint32_t)i;
    dense[i] = (int32_t)(par[c] ^ c);
  }
}

// ... and after the all-reduce: par and the totals on every rank, as k_hook would have written
// them. in_mst is NOT written here: the owner rank's k_win marked the edge (a random byte store
// per hook on every rank cost ~0.5 ms per level at s26 / 8 ranks), so after a multi-rank solve
// each rank holds the flags of the hooks it owned and the OR over the ranks is the MSF
// (DistributedMST.gather_in_mst).
__global__ void k_unpack_hook(const uint32_t *__restrict__ act, const unsigned long long *__restrict__ d_nact,
                              const int32_t *__restrict__ dense, const uint64_t *__restrict__ best,
                              uint32_t *__restrict__ par, unsigned long long *__restrict__ acc /* [0] weight, [1] edges */) {
  __shared__ unsigned long long s_w[BLOCK / WAVE], s_c[BLOCK / WAVE];
  unsigned long long wsum = 0, cnt = 0;
  const uint64_t nact = *d_nact;
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < nact; i += (uint64_t)gridDim.x * BLOCK) {
    const uint32_t x = (uint32_t)dense[i];
    if (x == 0) continue;
    const uint32_t c = act ? act[i] : (uint32_t)i;
    const uint64_t k = best[c];
    par[c] = c ^ x;
    wsum += k >> 32;
    cnt += 1;
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

// A dense level's opening round with the reduce-scatter protocol (the library loop, ABI 6): after a
// MIN reduce-scatter of the best slots, rank r holds the final minimum of its slot range only; it
// computes those fragments' hooks from the replicated canonical list (the edge's ends, their
// level-open roots vlab, their dense labels) as pairs eid << 32 | other; an all-gather of the pairs
// gives every rank every hook, and k_apply_pairs sets par (a mutual pair keeps its smaller member
// as the root), the MSF flags of the rank's own edge range and the totals — 8 + 8 bytes per slot
// on the wire instead of the all-reduce protocol's 2 x (8 + 4).
__device__ __forceinline__ void add_totals_one(unsigned long long wsum, unsigned long long cnt,
                                               unsigned long long *__restrict__ acc) {
  __shared__ unsigned long long s_w[BLOCK / WAVE], s_c[BLOCK / WAVE];
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

// the reduce-scatter protocol's partial totals (all-reduced by the caller) join the totals
__global__ void k_fold_partial(unsigned long long *__restrict__ cnt) {
  cnt[2] += cnt[11];  // C_WEIGHT += C_RS_WEIGHT, C_EDGES += C_RS_EDGES
  cnt[3] += cnt[12];
  cnt[11] = 0;
  cnt[12] = 0;
}

__global__ void k_pad_slots(uint64_t *__restrict__ best, const unsigned long long *__restrict__ d_nact, uint64_t padded) {
  const uint64_t i = *d_nact + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < padded) best[i] = KEY_NONE;
}

__global__ void k_hook_owner(const uint64_t *__restrict__ best, uint64_t lo, uint64_t hi, const Ends E,
                             const uint32_t *__restrict__ vlab, DenseRank dr, uint64_t *__restrict__ pairs,
                             unsigned long long *__restrict__ err) {
  for (uint64_t c = lo + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < hi; c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = best[c];
    uint64_t out = KEY_NONE;
    if (k != KEY_NONE) {
      const uint32_t eid = (uint32_t)k;
      const uint32_t da = dense_rank(dr, vlab[end_u(E, eid)]), db = dense_rank(dr, vlab[E.v[eid]]);
      if (da != (uint32_t)c && db != (uint32_t)c) atomicOr(err, 2ull);  // the chosen edge must leave c
      out = ((uint64_t)eid << 32) | (da == (uint32_t)c ? db : da);
    }
    pairs[c] = out;
  }
}

__global__ __launch_bounds__(BLOCK) void k_apply_pairs(const uint64_t *__restrict__ pairs,
                                                       const unsigned long long *__restrict__ d_nact,
                                                       const uint32_t *__restrict__ ew, uint32_t *__restrict__ par,
                                                       uint64_t *__restrict__ best, uint8_t *__restrict__ in_mst,
                                                       uint32_t own_lo, uint32_t own_hi,
                                                       unsigned long long *__restrict__ acc) {
  unsigned long long wsum = 0, cnt = 0;
  const uint64_t nact = *d_nact;
  for (uint64_t c = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; c < nact; c += (uint64_t)gridDim.x * BLOCK) {
    const uint64_t p = pairs[c];
    best[c] = p;  // every rank the same "had an outgoing edge" for the jump's keep test
    if (p == KEY_NONE) continue;
    const uint32_t o = (uint32_t)p, eid = (uint32_t)(p >> 32);
    par[c] = o;  // a mutual pair stays a 2-cycle: the jump keeps its smaller member as the root
    // the MSF flag and the totals of the rank's own edges only (1/N of the random reads); the
    // caller SUM-all-reduces the partial totals
    if (eid < own_lo || eid >= own_hi) continue;
    if ((uint32_t)pairs[o] == (uint32_t)c && (uint32_t)c < o) continue;  // counted by its partner's slot
    in_mst[eid] = 1;
    wsum += ew[eid];
    cnt += 1;
  }
  add_totals_one(wsum, cnt, acc);
}

// ------------------------------------------------------------------------------------------
// Stage 3: pointer jumping (INITIATE broadcast of the new fragment id), one fragment per thread
// (every walk of the round in flight at once). Path splitting on par: concurrent compression
// only moves a pointer to an ancestor, so stale reads are still valid ancestors and every walk
// ends at its root; lab[c] = root. Stage 3b: the next active list = roots that still had an
// outgoing edge (their best slot is reset); keep byte -> flags[i] for k_select_lb. A root with
// no outgoing edge is finished for the level (the reference: "best_weight == inf at the core =>
// terminate", ghs_implementation.py:316-320).
// A bucketed round's hooks (k_bmin) leave every mutual pair as a 2-cycle c <-> p over their
// shared edge (the reference's equal-level merge over a core edge, ghs_implementation.py:186-196):
// a walk that meets par[par[x]] == x ends at min(x, par[x]), the smaller label keeps the root, and
// that member writes par[c] = c. Such pairs exist only at the tree tops and their two pointers are
// never rewritten by path splitting (a walk at either member detects the pair first), so every
// concurrent walk sees the same root. acc != nullptr (bucketed rounds): the jump also counts the
// round's hooks — every fragment that ends below another root adds its best key's weight (each MSF
// edge once: a mutual pair's smaller member adds nothing).
// ------------------------------------------------------------------------------------------
// The jump's hook totals go to HOOK_SHARDS address pairs (one 64-B line each, by block) instead of
// one pair: same-address device atomics serialise at ~12 ns each, which capped the counting jump's
// grid at 2048 blocks (R-MAT s24: k_jump_ident 0.28 -> 0.46 ms in bucketed rounds). The last
// select tile of the round folds the shards into the totals (k_select_lb).
constexpr int HOOK_SHARDS = 64;   // == WAVE: one lane per shard in the fold
constexpr int SHARD_STRIDE = 8;   // u64 per shard (64 B)
__device__ __forceinline__ void add_totals(unsigned long long wsum, unsigned long long cnt,
                                           unsigned long long *__restrict__ acc) {
  acc += SHARD_STRIDE * (blockIdx.x % HOOK_SHARDS);
  __shared__ unsigned long long s_w[BLOCK / WAVE], s_c[BLOCK / WAVE];
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

// k_jump's path splitting starts after SPLIT_AFTER steps of a walk: a short walk (most of them)
// then only reads, instead of a random 4-B store per step that no later walk may need. 16384^2
// grid, level 0 rounds 1-3: 2.29 / 1.29 / 0.48 -> 1.85 / 1.17 / 0.43 ms (2 steps; 4 the same).
// k_jump_ident keeps splitting from the first step: the gradient grid's long hook chains need it
// (its level-0 jump 1.54 -> 1.83 ms with 2 steps, profiles/r03/ab_split/).
#ifndef GHS_SPLIT_AFTER
#define GHS_SPLIT_AFTER 2
#endif
constexpr uint32_t SPLIT_AFTER = GHS_SPLIT_AFTER;
__global__ __launch_bounds__(BLOCK) void k_jump(const uint32_t *__restrict__ act, const unsigned long long *__restrict__ d_nact,
                                                uint32_t *par, uint32_t *__restrict__ lab, uint64_t *__restrict__ best,
                                                uint8_t *__restrict__ flags, unsigned long long *__restrict__ err,
                                                unsigned long long *__restrict__ acc) {
  const uint64_t nact = *d_nact;
  unsigned long long wsum = 0, cnt = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < nact; i += (uint64_t)gridDim.x * BLOCK) {
    const uint32_t c = act ? act[i] : (uint32_t)i;
    if (!act && lab[c] != c) {  // identity list: not a root when the level opened, never a label
      flags[i] = 0;
      continue;
    }
    uint32_t x = c;
    uint32_t px = par[x];
    bool root = px == c;
    uint32_t steps = 0;
    while (px != x) {
      const uint32_t ppx = par[px];
      if (ppx == x) {  // x <-> px: a mutual pair at the top of the tree
        x = x < px ? x : px;
        break;
      }
      if (ppx != px && steps >= SPLIT_AFTER) par[x] = ppx;
      x = px;
      px = ppx;
      if (++steps > JUMP_MAX_STEPS) {
        atomicOr(err, 4ull);
        break;
      }
    }
    if (x == c && !root) {  // the smaller member of a mutual pair: it keeps the root
      par[c] = c;
      root = true;
    }
    if (x != c) {
      lab[c] = x;  // a root's label is already itself (k_resolve, then only hooks move it)
      if (acc) {
        wsum += best[c] >> 32;
        cnt += 1;
      }
    }
    const bool keep = root && best[c] != KEY_NONE;
    if (keep) best[c] = KEY_NONE;
    flags[i] = keep ? 1 : 0;
  }
  if (acc) add_totals(wsum, cnt, acc);
}

// Stage 3 over the identity list (a single-rank level's first round): every vertex, 4 per thread
// per step, the 4 a grid stride apart (coalesced 4-B loads of lab, par and best per wave), their
// walks advanced together: each step issues the par loads of every unfinished walk before any is
// used, so a lane keeps 4 dependent chains in flight, and walks started together are far apart on
// a chain (they do not duplicate each other's path splitting; gradient grid 55.7 -> 25.8 ms over
// consecutive vertices). A vertex that was not a root when the level opened (lab[c] != c) is never
// a label and is skipped; a root that did not hook only tests its best slot; a root that hooked
// walks. Mutual pairs and hook counting as in k_jump.
// lab_init (one rank, level 0's round 0): lab was never initialised (every vertex is a root at the
// level's open, so it is not read) and this pass writes every vertex's label — the solve's only
// n-sized label write before level 1 (the iota it replaces and the read cost one lab pass each).
__global__ __launch_bounds__(BLOCK) void k_jump_ident(uint32_t n, uint32_t *par, uint32_t *__restrict__ lab,
                                                      uint64_t *__restrict__ best, uint8_t *__restrict__ flags,
                                                      unsigned long long *__restrict__ err,
                                                      unsigned long long *__restrict__ acc, bool lab_init) {
  const uint64_t tg = blockIdx.x * (uint64_t)BLOCK + threadIdx.x, S = (uint64_t)gridDim.x * BLOCK;
  unsigned long long wsum = 0, cnt = 0;
  for (uint64_t i0 = tg * 4; i0 - tg * 4 < n; i0 += S * 4) {  // every thread while the chunk starts below n
    const uint64_t cb = i0 - tg * 4;                          // the grid's chunk of 4S vertices
#define JV(k) (cb + tg + S * (uint64_t)(k))
    uint32_t lc[4], pc[4];
    uint64_t bc[4];
    // par / best only for the level's roots (lab[c] == c): past level 0 on a lattice-like graph
    // almost no vertex is one (the 16384^2 grid's level 1: ~97% are not), and their par / best
    // lines need not be fetched (k_jump_ident per step: grid 3.98 -> 3.62 ms, gradient grid 2.91 ->
    // 2.42 ms; R-MAT s24 within its spread, 0.289-0.303 ms)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t vv = JV(k);
      lc[k] = vv < n ? (lab_init ? (uint32_t)vv : lab[vv]) : LABEL_NONE;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t vv = JV(k);
      const bool root = vv < n && lc[k] == (uint32_t)vv;
      pc[k] = root ? par[vv] : 0u;
      bc[k] = root ? best[vv] : KEY_NONE;
    }
    uint32_t kb = 0;
    uint32_t x[4], px[4], walking = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t c = (uint32_t)JV(k);
      x[k] = c;
      px[k] = pc[k];
      if (lc[k] != c) continue;  // not a root at the level's open (or past n)
      if (pc[k] == c) {          // still a root: kept iff it had an outgoing edge
        if (bc[k] != KEY_NONE) {
          best[c] = KEY_NONE;
          kb |= 1u << (8 * k);
        }
        continue;
      }
      walking |= 1u << k;  // hooked: walk to the root (path splitting)
    }
    const uint32_t hooked = walking;
    uint32_t steps = 0;
    while (walking) {
      uint32_t ppx[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) ppx[k] = par[(walking >> k) & 1u ? px[k] : 0u];  // finished: a harmless load
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!((walking >> k) & 1u)) continue;
        if (ppx[k] == x[k]) {  // x <-> px: a mutual pair at the top of the tree
          x[k] = x[k] < px[k] ? x[k] : px[k];
          walking &= ~(1u << k);
          continue;
        }
        if (ppx[k] != px[k]) par[x[k]] = ppx[k];
        x[k] = px[k];
        px[k] = ppx[k];
        if (px[k] == x[k]) walking &= ~(1u << k);
      }
      if (++steps > JUMP_MAX_STEPS) {
        atomicOr(err, 4ull);
        break;
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!((hooked >> k) & 1u)) continue;
      const uint32_t c = (uint32_t)JV(k);
      if (x[k] == c) {  // the smaller member of a mutual pair: stays a root, had an edge
        par[c] = c;
        best[c] = KEY_NONE;
        kb |= 1u << (8 * k);
      } else {
        if (!lab_init) lab[c] = x[k];
        if (acc) {
          wsum += bc[k] >> 32;
          cnt += 1;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (JV(k) < n) {
        flags[JV(k)] = (uint8_t)(kb >> (8 * k));
        if (lab_init) lab[JV(k)] = (hooked >> k) & 1u ? x[k] : (uint32_t)JV(k);  // coalesced: every vertex
      }
#undef JV
  }
  if (acc) add_totals(wsum, cnt, acc);
}

// ------------------------------------------------------------------------------------------
// Between levels. k_giant first: the giant fragment = the most frequent root among NSAMPLE
// evenly spaced vertices (ties: the smaller label), each sample resolved by its own walk and
// counted in an LDS hash table — one workgroup, no host round trip. Then k_resolve compresses
// every vertex to its root (lab[v] = find(v)) and writes the giant-membership bitmap in the same
// pass (bit v = lab[v] == giant, one ballot word per wave).
// ------------------------------------------------------------------------------------------
constexpr uint32_t NSAMPLE = 2048;  // the giant holds >= ~10% of the vertices: 2048 samples find it
constexpr uint32_t GIANT_SLOTS = 4096;
// Hot fragments: the sample's most frequent roots (at most HOT_K, each hit by >= HOT_MIN samples,
// i.e. holding >= ~n/1024 vertices), giant included. A bucketed level-first round reduces their
// candidates per block (k_bucket) instead of filling one bucket each. Stored after the giant's
// two words: giant[GIANT_HOT] = count, giant[GIANT_HOT + 1 ...] = labels.
constexpr uint32_t HOT_K = 64;
constexpr uint32_t HOT_MIN = 2;
constexpr uint32_t GIANT_HOT = 4;
__global__ __launch_bounds__(1024) void k_giant(uint32_t n, const uint32_t *lab, uint32_t *__restrict__ giant,
                                                unsigned long long *__restrict__ err) {
  __shared__ uint32_t s_lab[GIANT_SLOTS];
  __shared__ uint32_t s_cnt[GIANT_SLOTS];
  __shared__ uint32_t s_hist[NSAMPLE + 1];  // labels per sample count
  __shared__ uint32_t s_wsum[1024 / WAVE];
  __shared__ uint32_t s_thr, s_nhot;
  __shared__ unsigned long long s_best[1024 / WAVE];
  for (uint32_t i = threadIdx.x; i < GIANT_SLOTS; i += 1024) {
    s_lab[i] = LABEL_NONE;
    s_cnt[i] = 0;
  }
  for (uint32_t i = threadIdx.x; i <= NSAMPLE; i += 1024) s_hist[i] = 0;
  if (threadIdx.x == 0) {
    s_thr = NSAMPLE + 1;
    s_nhot = 0;
  }
  __syncthreads();
  const uint32_t ns = n < NSAMPLE ? n : NSAMPLE;
  for (uint32_t i = threadIdx.x; i < ns; i += 1024) {
    const uint32_t r = find_lab(lab, (uint32_t)(((uint64_t)i * n) / ns), err);
    uint32_t h = (r * 0x9E3779B1u) >> (32 - 12);
    for (;;) {  // linear probing: 4096 slots for <= 2048 keys always end
      uint32_t cur = s_lab[h];
      if (cur == LABEL_NONE) {
        cur = atomicCAS(&s_lab[h], LABEL_NONE, r);
        if (cur == LABEL_NONE) cur = r;
      }
      if (cur == r) {
        atomicAdd(&s_cnt[h], 1u);
        break;
      }
      h = (h + 1) & (GIANT_SLOTS - 1);
    }
  }
  __syncthreads();
  // pack (count, ~label) for a max: most frequent, then the smaller label
  unsigned long long best = 0;
  for (uint32_t i = threadIdx.x; i < GIANT_SLOTS; i += 1024) {
    if (s_lab[i] != LABEL_NONE) {
      const unsigned long long c = ((unsigned long long)s_cnt[i] << 32) | (0xffffffffu - s_lab[i]);
      best = c > best ? c : best;
    }
  }
#pragma unroll
  for (int d = WAVE / 2; d > 0; d >>= 1) {
    const unsigned long long o = __shfl_xor(best, d);
    best = o > best ? o : best;
  }
  if ((threadIdx.x & (WAVE - 1)) == 0) s_best[threadIdx.x / WAVE] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = 0;
    for (int w = 0; w < 1024 / WAVE; ++w) b = s_best[w] > b ? s_best[w] : b;
    giant[0] = 0xffffffffu - (uint32_t)b;
    giant[1] = (uint32_t)(b >> 32);  // sampled vertices in the giant (stats / debug)
  }
  // hot list: the smallest count threshold T >= HOT_MIN with at most HOT_K labels counted >= T
  // (suffix sums of the count histogram: thread t holds counts 2048 - 2t and 2047 - 2t)
  for (uint32_t i = threadIdx.x; i < GIANT_SLOTS; i += 1024)
    if (s_lab[i] != LABEL_NONE) atomicAdd(&s_hist[s_cnt[i]], 1u);
  __syncthreads();
  const uint32_t c0 = NSAMPLE - 2 * threadIdx.x, c1 = c0 - 1;
  const uint32_t h0 = s_hist[c0], h1 = s_hist[c1];
  const uint32_t lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  uint32_t incl = h0 + h1;
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const uint32_t o = __shfl_up(incl, d);
    if ((int)lane >= d) incl += o;
  }
  if (lane == WAVE - 1) s_wsum[wid] = incl;
  __syncthreads();
  uint32_t before = incl - h0 - h1;
  for (uint32_t w = 0; w < wid; ++w) before += s_wsum[w];
  const uint32_t S0 = before + h0, S1 = S0 + h1, S2 = S1 + (c1 > 1 ? s_hist[c1 - 1] : 0u);  // S(c0), S(c1), S(c1 - 1)
  if (c0 >= HOT_MIN && S0 <= HOT_K && (c0 == HOT_MIN || S1 > HOT_K)) s_thr = c0;
  if (c1 >= HOT_MIN && S1 <= HOT_K && (c1 == HOT_MIN || S2 > HOT_K)) s_thr = c1;
  __syncthreads();
  const uint32_t T = s_thr;
  for (uint32_t i = threadIdx.x; i < GIANT_SLOTS; i += 1024)
    if (s_lab[i] != LABEL_NONE && s_cnt[i] >= T) giant[GIANT_HOT + 1 + atomicAdd(&s_nhot, 1u)] = s_lab[i];
  __syncthreads();
  if (threadIdx.x == 0) giant[GIANT_HOT] = s_nhot;
}

__global__ __launch_bounds__(BLOCK) void k_resolve(uint32_t n, uint32_t *lab, const uint32_t *__restrict__ giant_ptr,
                                                   uint64_t *__restrict__ bits, unsigned long long *__restrict__ err) {
  const uint32_t giant = giant_ptr[0];
  const uint64_t words = ((uint64_t)n + 63) / 64;
#if GHS_RESOLVE4 == 2
  // 4 vertices per thread a grid stride S apart (their walks start far apart on a chain, as in
  // k_jump_ident), advanced together; each of the 4 is a coalesced wave slice of 64 vertices, so
  // the giant bits of slice k are one ballot = one 64-bit bitmap word (S is a multiple of 64)
  const uint64_t tg = blockIdx.x * (uint64_t)BLOCK + threadIdx.x, S = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t cb = 0; cb < (uint64_t)n; cb += 4 * S) {
    uint32_t x[4], y[4], walking = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t vv = cb + tg + S * k;
      x[k] = (uint32_t)vv;
      y[k] = vv < n ? lab[vv] : (uint32_t)vv;
      if (vv < n && y[k] != x[k]) walking |= 1u << k;
    }
    uint32_t hops = 0;
    while (walking) {
      uint32_t ny[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) ny[k] = lab[(walking >> k) & 1u ? y[k] : 0u];  // finished: a harmless load
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!((walking >> k) & 1u)) continue;
        x[k] = y[k];
        y[k] = ny[k];
        if (y[k] == x[k]) walking &= ~(1u << k);
      }
      if (++hops > FIND_LAB_MAX_HOPS) {
        atomicOr(err, 1ull);
        break;
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t vv = cb + tg + S * k;
      if (vv < n) lab[vv] = x[k];
      const uint64_t b = __ballot((vv < n) && x[k] == giant);
      if ((threadIdx.x & (WAVE - 1)) == 0 && (vv >> 6) < words) bits[vv >> 6] = b;
    }
  }
#elif GHS_RESOLVE4
  // 4 vertices per lane (16-B lab load/store), their label walks advanced together; a lane's 4
  // giant bits are OR-combined over 16 lanes into one 64-bit bitmap word
  const uint64_t n4 = (uint64_t)n & ~3ull;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  for (uint64_t i0 = (blockIdx.x * (uint64_t)BLOCK + threadIdx.x) * 4; i0 - lane * 4 < (uint64_t)n;
       i0 += (uint64_t)gridDim.x * BLOCK * 4) {
    uint32_t x[4], y[4], walking = 0;
    if (i0 < n4) {
      const uint4 l4 = *reinterpret_cast<const uint4 *>(lab + i0);
      y[0] = l4.x; y[1] = l4.y; y[2] = l4.z; y[3] = l4.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) y[k] = i0 + k < n ? lab[i0 + k] : (uint32_t)(i0 + k);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[k] = (uint32_t)(i0 + k);
      if (i0 + k < n && y[k] != x[k]) walking |= 1u << k;
    }
    uint32_t hops = 0;
    while (walking) {
      uint32_t ny[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) ny[k] = lab[(walking >> k) & 1u ? y[k] : 0u];  // finished: a harmless load
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!((walking >> k) & 1u)) continue;
        x[k] = y[k];
        y[k] = ny[k];
        if (y[k] == x[k]) walking &= ~(1u << k);
      }
      if (++hops > FIND_LAB_MAX_HOPS) {
        atomicOr(err, 1ull);
        break;
      }
    }
    uint64_t part = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) part |= (uint64_t)((i0 + k < n) & (x[k] == giant)) << (4 * (lane & 15) + k);
    if (i0 < n4) {
      *reinterpret_cast<uint4 *>(lab + i0) = make_uint4(x[0], x[1], x[2], x[3]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (i0 + k < n) lab[i0 + k] = x[k];
    }
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) part |= __shfl_xor(part, d);
    if ((lane & 15) == 0 && (i0 >> 6) < words) bits[i0 >> 6] = part;
  }
#else
  for (uint64_t base = blockIdx.x * (uint64_t)BLOCK; base < (uint64_t)n; base += (uint64_t)gridDim.x * BLOCK) {
    const uint64_t v = base + threadIdx.x;
    bool in = false;
    if (v < n) {
      const uint32_t r = find_lab(lab, (uint32_t)v, err);
      lab[v] = r;
      in = r == giant;
    }
    const uint64_t b = __ballot(in);
    if ((threadIdx.x & (WAVE - 1)) == 0 && (v >> 6) < words) bits[v >> 6] = b;
  }
#endif
}


// evenly spaced sample of the canonical list: weights (the level plan) and, in out[NSAMPLE_W + i],
// edge spans v - u (the plan's locality test for the bucketed rounds)
constexpr uint32_t NSAMPLE_W = 16384;  // edges sampled for the level plan
__global__ void k_sample_weights(uint64_t cnt, const Ends E, const uint32_t *__restrict__ w, uint32_t nsamp,
                                 uint32_t *__restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nsamp; i += gridDim.x * blockDim.x) {
    const uint64_t e = ((uint64_t)i * cnt) / nsamp;
    out[i] = w[e];
    out[NSAMPLE_W + i] = E.v[e] - end_u(E, (uint32_t)e);  // canonical: u < v (unvalidated here: only a heuristic)
  }
}

// Level plan on the device (no host round trip before the first pass): thresholds = order
// statistics of the weight sample, the same arithmetic as a host plan would do (target =
// level1 * n edges, x growth per level, double precision; the q-th smallest by a 4-pass radix
// select over the sample in LDS; equal thresholds merged). thr[0..count), thr[PLAN_MAX] = count.
constexpr uint32_t PLAN_MAX = 33;      // 0, up to 31 interior thresholds, 2^32
// thr[PLAN_LOCAL] = 1: the span sample is lattice-like (<= 1/32 of the sampled edges span more than
// n/64 ids): the single-rank solve runs bucketed rounds
constexpr uint32_t PLAN_LOCAL = PLAN_MAX + 1;
__global__ __launch_bounds__(1024) void k_plan(const uint32_t *__restrict__ sample, uint32_t ns_all, uint32_t ns,
                                               uint32_t n, uint64_t m, uint32_t L, double l1, double growth,
                                               uint64_t *__restrict__ thr) {
  __shared__ uint32_t s_w[NSAMPLE_W];
  __shared__ uint32_t s_hist[256];
  __shared__ uint32_t s_sel[2];
  __shared__ uint32_t s_far;
  if (threadIdx.x == 0) s_far = 0;
  __syncthreads();
  {
    uint32_t far = 0;
    for (uint32_t i = threadIdx.x; i < ns_all; i += 1024) far += sample[NSAMPLE_W + i] > n / 64 ? 1u : 0u;
    if (far) atomicAdd(&s_far, far);
  }
  for (uint32_t i = threadIdx.x; i < ns; i += 1024) s_w[i] = sample[i];
  __syncthreads();
  uint32_t cnt = 1;
  uint64_t last = 0;
  double target = l1 * (double)n;
  for (uint32_t lev = 1; lev < L && ns > 0; ++lev) {  // uniform across the block
    const double frac = target / (double)m;
    if (frac >= 1.0) break;
    const uint32_t q = (uint32_t)(frac * ns);  // non-decreasing: target grows every level
    target *= fmax(1.01, growth);
    if (q == 0) continue;
    uint32_t prefix = 0, pmask = 0, k = q;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (uint32_t i = threadIdx.x; i < 256; i += 1024) s_hist[i] = 0;
      __syncthreads();
      for (uint32_t i = threadIdx.x; i < ns; i += 1024) {
        const uint32_t x = s_w[i];
        if ((x & pmask) == prefix) atomicAdd(&s_hist[(x >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (threadIdx.x < WAVE) {  // one wave finds the digit: lane t owns bins 4t..4t+3
        const uint32_t t = threadIdx.x;
        const uint32_t c[4] = {s_hist[4 * t], s_hist[4 * t + 1], s_hist[4 * t + 2], s_hist[4 * t + 3]};
        const uint32_t sum = c[0] + c[1] + c[2] + c[3];
        uint32_t incl = sum;
#pragma unroll
        for (int d = 1; d < WAVE; d <<= 1) {
          const uint32_t o = __shfl_up(incl, d);
          if ((int)t >= d) incl += o;
        }
        const uint32_t excl = incl - sum;
        if (excl <= k && incl > k) {  // exactly one lane: the candidates number more than k
          uint32_t acc = excl, d = 4 * t;
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            if (acc + c[j] > k) break;
            acc += c[j];
            ++d;
          }
          s_sel[0] = prefix | (d << shift);
          s_sel[1] = k - acc;
        }
      }
      __syncthreads();
      prefix = s_sel[0];
      k = s_sel[1];
      pmask |= 255u << shift;
      __syncthreads();
    }
    if (threadIdx.x == 0 && (uint64_t)prefix > last) {
      thr[cnt++] = prefix;
      last = prefix;
    }
  }
  if (threadIdx.x == 0) {
    thr[0] = 0;
    thr[cnt++] = 1ull << 32;
    thr[PLAN_MAX] = cnt;
    thr[PLAN_LOCAL] = (ns_all > 0 && (uint64_t)s_far * 32 <= ns_all) ? 1 : 0;
  }
}

// ------------------------------------------------------------------------------------------
// SELECT (opens level 0): the first full stream over the caller's canonical list [e_lo, e_hi)
// (u, v, w: 12 B per edge; key = w << 32 | eid built here). The stream runs over the aligned
// range [E0, e_hi), E0 = e_lo & ~3 (edges below e_lo are masked), so every lane's 4-edge tile is
// one 16-B buffer load per array. Validates canonicity (u < v < n, (u, v) strictly ascending)
// into err bit 8 — before any kernel indexes an array with these ids — and emits the edges with
// w < w_hi into this block's level staging region (every vertex is its own fragment, so the
// labels are the endpoints); flags both ends active. Nothing else is written: the
// heavier edges stay where they are until k_filter. Block-private output regions: deterministic,
// no atomics; the next tile's loads are issued before the current one is compacted.
// CSR (ABI 9): u is derived from the row offsets (csr_tile_rows, the tiles' rows from k_csr_tiles,
// after k_csr_check validated the offsets: a wave's slice is a multiple of 256 edges, so its tiles are trow's).
// ------------------------------------------------------------------------------------------
// One pass over the row offsets of the solver's range [E0, e_hi) (T = e_hi - E0 edges), before
// k_select:
//  - trow[t] = the row holding edge E0 + 256 t (t < ntiles), trow[ntiles] = the row of the range's
//    last edge: every nonempty row writes the tile starts inside it (one writer per tile);
//  - the offsets' validation (off[0] = 0, nondecreasing, off[n] = m; err bit 8): k_select skips its
//    stream when it is set, so no tile walks rows from a garbage trow;
//  - the streaming passes' partitions balanced by cost instead of edge count: k_select's wave slices
//    (bsel, nsel + 1 bounds, 256-edge tiles) and k_filter's block ranges (bfil, nfil + 1 bounds,
//    1024-edge tiles). A tile costs its edges and its rows (the windows of row starts it scans): the
//    end of an R-MAT list holds the high vertex ids, which store few canonical edges — thousands of
//    mostly empty rows per tile — and with equal edge counts its waves ran ~10x longer than the rest.
//    Cost = CSR_EDGE_COST per edge + a row cost per row of the range; each row r of [Rb, Re] owns
//    the cost interval [C_r, C_r + len_r) (its row cost at its start, then its edges), the intervals
//    tile [0, C_tot), and bound k = the position of cost k * C_tot / N, written by the row whose
//    interval holds it (one writer per bound), rounded down to the tile grid.
//    The row costs were measured per pass (R-MAT s24, same box, profiles/r06/csr/): k_select's wave
//    slices at 2 edges per row (row cost 8) run 0.76 -> 0.58 ms against 0.5 edge (row cost 2), while
//    k_filter's blocks are best near 0.5 edge per row (1.66 ms; 1.68 at 2 edges, 1.69 at 6).
#ifndef GHS_CSR_ROW_SEL
#define GHS_CSR_ROW_SEL 8
#endif
#ifndef GHS_CSR_ROW_FIL
#define GHS_CSR_ROW_FIL 2
#endif
constexpr uint64_t CSR_EDGE_COST = 4, CSR_ROW_SEL = GHS_CSR_ROW_SEL, CSR_ROW_FIL = GHS_CSR_ROW_FIL;
// Rb, Re: the rows of the range's first and last edges (one wave: a 64-ary search each), once per
// solve, before the row pass and the bounds
__global__ __launch_bounds__(64) void k_csr_range(const uint32_t *__restrict__ off, uint32_t n, uint64_t E0, uint64_t e_hi,
                                                 uint32_t *__restrict__ rb) {
  const uint32_t lane = threadIdx.x;
  for (int q = 0; q < 2; ++q) {
    const uint64_t e = q ? e_hi - 1 : E0;
    uint32_t lo = 0, c = n ? n : 1;  // candidates [lo, lo + c): off[lo] <= e
    while (c > 1) {
      const uint32_t st = (c + WAVE - 1) / WAVE;
      const bool in = lane * st < c;
      const uint64_t bm = __ballot(in && off[lo + lane * st] <= e);
      const uint32_t L = bm ? 63u - (uint32_t)__clzll((long long)bm) : 0u;
      lo += L * st;
      c = min(st, c - L * st);
    }
    if (lane == 0) rb[q] = lo;
  }
}

// The offsets' validation: one coalesced pass over off (off[0] = 0, nondecreasing, off[n] = m).
__global__ __launch_bounds__(256) void k_csr_check(const uint32_t *__restrict__ off, uint32_t n, uint64_t m,
                                                   unsigned long long *__restrict__ err) {
  bool bad = false;
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x)
    bad |= off[r] > off[r + 1];
  if (blockIdx.x == 0 && threadIdx.x == 0) bad |= (off[0] != 0u) | ((uint64_t)off[n] != m);
  if (__any(bad) && (threadIdx.x & (WAVE - 1)) == 0) atomicOr(err, 8ull);
}

// trow: one thread per tile — the row holding edge E0 + 256 t (t = ntiles: the range's last edge)
// by a binary search over [Rb, Re] (its upper levels are shared by every tile, so they hit in the
// caches). (A row pass that wrote each row's tiles left the wave of the R-MAT hub rows thousands of
// tiles behind the rest, and computing the partitions there made it VALU-bound: ~0.1 ms at s24.)
// Malformed offsets land the searches anywhere in [Rb, Re]; k_select then streams nothing.
__global__ __launch_bounds__(256) void k_csr_tiles(const uint32_t *__restrict__ off, const uint32_t *__restrict__ rb,
                                                   uint64_t E0, uint64_t e_hi, uint32_t *__restrict__ trow) {
  const uint64_t T = e_hi - E0, ntiles = (T + 255) >> 8;
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t > ntiles) return;
  const uint64_t e = t < ntiles ? E0 + (t << 8) : e_hi - 1;
  uint32_t lo = rb[0], hi = rb[1] < lo ? lo : rb[1];  // the last r with off[r] <= e
  while (lo < hi) {
    const uint32_t mid = lo + ((hi - lo + 1) >> 1);
    if (off[mid] <= e) lo = mid; else hi = mid - 1;
  }
  trow[t] = lo;
}

// The streaming passes' partitions: one thread per bound. The cumulative cost C(r) =
// row_cost (r - Rb) + CSR_EDGE_COST a_r is nondecreasing in r, so bound k — the position of cost
// k S, S = ceil(C_tot / N) — lies in the last row r with C(r) <= k S (a binary search over
// [Rb, Re]); inside it, past the row's own cost, at edge a_r + (k S - C(r) - row_cost) / EDGE_COST,
// rounded down to the pass's tile grid. k = N, and every k with k S >= C_tot, is the range's end.
// bsel: k_select's nsel + 1 wave-slice bounds (256-edge tiles); bfil: k_filter's nfil + 1 block
// bounds (1024-edge tiles). Malformed offsets (k_csr_check's err bit 8) make the searches land
// anywhere in the range, never outside it: k_select then streams nothing.
__global__ __launch_bounds__(256) void k_csr_bounds(const uint32_t *__restrict__ off, const uint32_t *__restrict__ rb,
                                                    uint64_t E0, uint64_t e_hi, uint32_t *__restrict__ bsel,
                                                    uint32_t nsel, uint32_t *__restrict__ bfil, uint32_t nfil) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nsel + 1 + nfil) return;
  const bool sel = i <= nsel;
  const uint32_t k = sel ? i : i - (nsel + 1), N = sel ? nsel : nfil;
  const uint64_t row = sel ? CSR_ROW_SEL : CSR_ROW_FIL, ts = sel ? WAVE * 4 : ARCS_PER_BLOCK;
  uint32_t *bound = sel ? bsel : bfil;
  const uint64_t T = e_hi - E0;
  const uint32_t Rb = rb[0], Re = rb[1] < Rb ? Rb : rb[1];
  const uint64_t Ctot = row * (uint64_t)(Re - Rb + 1) + CSR_EDGE_COST * T;
  const uint64_t S = (Ctot + N - 1) / N, X = (uint64_t)k * S;
  if (k == N || X >= Ctot) {
    bound[k] = (uint32_t)T;
    return;
  }
  auto pos = [&](uint32_t r) -> uint64_t {  // a_r: the row's first edge of the range, relative to E0
    const uint64_t o = off[r];
    return o > E0 ? (o < e_hi ? o : e_hi) - E0 : 0;
  };
  uint32_t lo = Rb, hi = Re;  // the last r with C(r) <= X (C(Rb) = 0 <= X)
  while (lo < hi) {
    const uint32_t mid = lo + ((hi - lo + 1) >> 1);
    if (row * (uint64_t)(mid - Rb) + CSR_EDGE_COST * pos(mid) <= X) lo = mid; else hi = mid - 1;
  }
  const uint64_t a = pos(lo), d = X - (row * (uint64_t)(lo - Rb) + CSR_EDGE_COST * a);
  uint64_t x = d < row ? a : a + (d - row) / CSR_EDGE_COST;
  if (x > T) x = T;
  bound[k] = (uint32_t)(x / ts * ts);
}

template <bool CSR>
GHS_STREAM_KERNEL_6 void k_select(uint32_t n, uint64_t m, uint64_t e_lo, uint64_t e_hi, const uint32_t *__restrict__ eu,
                                const uint32_t *__restrict__ eoff, const uint32_t *__restrict__ ev,
                                const uint32_t *__restrict__ ew, const uint64_t *__restrict__ w_hi_p,
                                uint32_t *__restrict__ osrc, uint32_t *__restrict__ odst, uint64_t *__restrict__ okey,
                                uint64_t *__restrict__ ostart, uint64_t *__restrict__ ocount,
                                uint8_t *__restrict__ mark, unsigned long long *__restrict__ err,
                                const uint64_t *__restrict__ local_flag, uint32_t bs,
                                unsigned long long *__restrict__ long_flag, const uint32_t *__restrict__ trow,
                                const uint32_t *__restrict__ bnd) {
  const uint64_t w_hi = *w_hi_p;  // the level plan lives on the device (k_plan)
  // a lattice-like plan (k_plan's span sample): note any level-0 edge whose ends lie more than one
  // bucket (2^bs ids) apart — the windowed round 0 (k_wmin) then falls back to k_bucket / k_bmin
  const bool check_span = local_flag && *local_flag;
  __shared__ WaveStage s_stage[BLOCK / WAVE];
  __shared__ uint32_t s_head[CSR ? BLOCK / WAVE : 1][CSR ? WAVE * 4 : 1];
  // the wave index through readfirstlane: uniform in an SGPR, so every value derived from it
  // (the slice, its buffer descriptors) is scalar — a VGPR descriptor makes hipcc wrap each
  // buffer load in a waterfall loop
  const uint32_t lane = threadIdx.x & (WAVE - 1), wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const uint32_t gw = blockIdx.x * (BLOCK / WAVE) + wid;  // this wave's slice (and output segment)
  const uint64_t W = (uint64_t)gridDim.x * (BLOCK / WAVE);
  const uint64_t E0 = e_lo & ~3ull;
  const uint64_t T = e_hi - E0;
  // CSR: the slices k_csr_bounds balanced by cost (whole 256-edge tiles: the trow grid)
  const uint64_t Q = ((T + W - 1) / W + 3) & ~3ull;
  const uint64_t vb = CSR ? bnd[gw] : Q * gw;
  const uint64_t ve = CSR ? bnd[gw + 1] : ((vb + Q < T) ? vb + Q : T);
  const uint64_t eb = E0 + vb;  // first edge of this wave
  const uint64_t nbytes = ve > vb ? (ve - vb) * 4 : 0;
  const __amdgpu_buffer_rsrc_t ru = make_rsrc(CSR ? ev : eu + eb, CSR ? 0 : nbytes);
  const __amdgpu_buffer_rsrc_t rv = make_rsrc(ev + eb, nbytes);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(ew + eb, nbytes);
  bool bad = false, far = false;
  // the edge before each lane's tile; offset -4 (the wave's first tile) is out of range of the
  // descriptor and is replaced by the wave's predecessor edge, loaded once
  uint32_t bpa = 0, bpb = 0;
  // CSR: the rows holding this tile's first edge and the next tile's (R0, R1), the tile after that's
  // (R2, a scalar load one tile ahead), the first window of rows after R0 (prefetched), the last
  // edge's row of the previous tile
  uint32_t R0 = 0, R1 = 0, R2 = 0, w0 = 0, lastu = 0;
  uint64_t vend = ve;  // CSR: an offsets error (k_csr_check) empties the stream
  if (CSR) {
    reinterpret_cast<uint4 *>(s_head[wid])[lane] = make_uint4(0u, 0u, 0u, 0u);
    if (*err & 8ull) vend = vb;
    const uint64_t ntiles = (T + 255) >> 8;
    if (vend > vb) {
      R0 = trow[vb >> 8];
      R1 = trow[(vb >> 8) + 1];
      R2 = trow[min((vb >> 8) + 2, ntiles)];
      w0 = csr_win(eoff, n, R0 + 1);
    }
    // edge eb - 1 lies in the same row iff that row began before eb (else in a lower one)
    if (eb > 0 && vend > vb) {
      bpa = eoff[R0] < eb ? R0 : R0 - 1u;
      bpb = ev[eb - 1];
    }
  } else if (eb > 0 && ve > vb) {
    bpa = eu[eb - 1];
    bpb = ev[eb - 1];
  }
  const uint32_t lane_off = lane * 16u;  // byte offset of the lane's tile in an iteration
  WaveOut wo;
  wo.pos = vb;
  uint4 ca = CSR ? make_uint4(0u, 0u, 0u, 0u) : ld_b128(ru, lane_off);
  uint4 cb = ld_b128(rv, lane_off), cw = ld_b128(rw, lane_off);
  uint32_t cpa = CSR ? 0u : ld_b32(ru, lane_off - 4), cpb = ld_b32(rv, lane_off - 4);
  // Every tile's loads are consumed at the END of the iteration that issued them (the empty asm
  // "uses"): the loop header then receives no pending load from either edge and never drains
  // the (rare, variable) flush stores there.
  asm volatile("" ::"v"(ca.x), "v"(cb.x), "v"(cw.x), "v"(cpa), "v"(cpb));
  for (uint64_t v0 = vb; v0 < vend; v0 += WAVE * 4) {
    const uint64_t v = v0 + (uint64_t)lane * 4;
    const uint64_t e0 = E0 + v;
    uint32_t a[4] = {ca.x, ca.y, ca.z, ca.w};
    const uint32_t b[4] = {cb.x, cb.y, cb.z, cb.w}, w[4] = {cw.x, cw.y, cw.z, cw.w};
    // lane mask of the tile: edges in [e_lo, ve) (32-bit arithmetic, no branches)
    const uint32_t nv = v < ve ? (uint32_t)((ve - v) < 4 ? (ve - v) : 4) : 0u;
    const uint32_t nskip = e0 < e_lo ? (uint32_t)(e_lo - e0) : 0u;
    bool live[4], out[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) live[j] = ((uint32_t)j < nv) & ((uint32_t)j >= nskip);
    // next tile (out-of-range offsets read 0)
    const uint32_t noff = (uint32_t)(v0 + WAVE * 4 - vb) * 4u + lane_off;
    if (!CSR) ca = ld_b128(ru, noff);
    cb = ld_b128(rv, noff);
    cw = ld_b128(rw, noff);
    const uint32_t npa = CSR ? 0u : ld_b32(ru, noff - 4), npb = ld_b32(rv, noff - 4);
    uint32_t pcsr = 0;
    if (CSR) {  // after the next tile's stream loads: the rows' LDS / DPP chain runs under them
      csr_tile_rows<false>(eoff, n, R0, R1, (uint32_t)(E0 + v0), s_head[wid], a, w0);
      // the next tile: its rows and its first window, in flight during this tile
      R0 = R1;
      R1 = R2;
      R2 = trow[min((v0 >> 8) + 3, (T + 255) >> 8)];
      w0 = csr_win(eoff, n, R0 + 1);
      pcsr = lane ? wave_shr1(a[3]) : lastu;
      lastu = __builtin_amdgcn_readlane(a[3], 63);
    }
    // u < v < n and (u, v) strictly above the previous edge; bitwise (no short-circuit
    // branches: hipcc turns && / || chains into exec-mask control flow here)
    uint32_t pa = (v == vb) ? bpa : (CSR ? pcsr : cpa), pb = (v == vb) ? bpb : cpb;
    const uint32_t first = (e0 == 0) ? 1u : 0u;  // edge 0 has no predecessor
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t ordered = (j == 0 ? first : 0u) | (uint32_t)(pa < a[j]) | ((uint32_t)(pa == a[j]) & (uint32_t)(pb < b[j]));
      const uint32_t ok = (uint32_t)(a[j] < b[j]) & (uint32_t)(b[j] < n) & ordered;
      bad |= live[j] & (ok == 0u);
      live[j] = live[j] & (ok != 0u);  // never index with an unchecked id
      pa = a[j];
      pb = b[j];
      out[j] = live[j] & ((uint64_t)w[j] < w_hi);
      far |= out[j] & ((b[j] >> bs) > (a[j] >> bs) + 1u);
    }
    cpa = npa;
    cpb = npb;
    uint32_t omask = 0;
    uint64_t key[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      omask |= out[j] ? (1u << j) : 0u;
      key[j] = ((uint64_t)w[j] << 32) | (uint32_t)(e0 + j);
      if (mark && out[j]) {  // active fragments of the level (~3% of the edges)
        mark[a[j]] = 1;
        mark[b[j]] = 1;
      }
    }
    // in canonical (eid) order, within and across the output regions: the LDS tail's (w, index)
    // minima rely on it (k_tail_open checks it under GHS_OPT_CHECK_TOTALS)
    wave_append(s_stage[wid], wo, a, b, key, omask, osrc, odst, okey);
    asm volatile("" ::"v"(ca.x), "v"(cb.x), "v"(cw.x), "v"(cpa), "v"(cpb));  // next tile landed (see above)
  }
  if (bad) atomicOr(err, 8ull);
  if (check_span && __any(far) && lane == 0 && !*long_flag) atomicOr(long_flag, 1ull);
  wave_finish(s_stage[wid], wo, osrc, odst, okey, vb, vb < T, ostart, ocount, gw);
}

// ------------------------------------------------------------------------------------------
// FILTER + level split (opens level 1): re-streams the canonical list once level 0 is complete.
//  - w < w_lo: level 0, already decided -> dropped;
//  - both ends in the giant fragment (1-bit bitmap, resident in each XCD's L2) -> dropped for
//    good (cycle property: the reference's REJECT for a whole weight class);
//  - w < w_hi: a level-1 edge: its labels are gathered (the only gathers of the pass), and if
//    they differ it goes to this block's region of the level staging (lab[u], lab[v], key) and
//    both fragments are flagged active (mark);
//  - otherwise: pending (u, v, key) for the later levels, tested there against their labels.
// The b-probes are ~1 L2 request per heavy edge and do not overlap the stream (measured: they
// add), so the pass costs stream + probes; splitting level 1 here saves a pass over the pending
// edges.
// ------------------------------------------------------------------------------------------
// CSR: 70 VGPRs (the row derivation), i.e. 7 blocks per CU, and the grid sized to one residency wave
// (7 x 256 blocks); 8 waves forced (GHS_FILTER_CSR_W8=1: 62 VGPRs + 4 spilled) measured slower:
// R-MAT s24 k_filter 1.85 against 1.65 ms, same box)
#ifndef GHS_FILTER_CSR_W8
#define GHS_FILTER_CSR_W8 0
#endif
template <bool CSR>
__global__ __launch_bounds__(BLOCK, (CSR && GHS_FILTER_CSR_W8) ? 8 : GHS_STREAM_WAVES) __attribute__((amdgpu_num_sgpr(72))) void k_filter(uint32_t n, uint64_t e_lo, uint64_t e_hi, const uint32_t *__restrict__ eu,
                                const uint32_t *__restrict__ eoff, const uint32_t *__restrict__ trow,
                                const uint32_t *__restrict__ ev, const uint32_t *__restrict__ ew,
                                const uint64_t *__restrict__ w_range /* [w_lo, w_hi] */,
                                const uint64_t *__restrict__ giant_bits,
                                const uint32_t *__restrict__ giant_ptr,
                                const uint32_t *__restrict__ lab, uint32_t *__restrict__ lsrc,
                                uint32_t *__restrict__ ldst, uint64_t *__restrict__ lkey,
                                uint64_t *__restrict__ lstart, uint64_t *__restrict__ lcount,
                                uint32_t *__restrict__ osrc, uint32_t *__restrict__ odst,
                                uint64_t *__restrict__ okey, uint64_t *__restrict__ ostart,
                                uint64_t *__restrict__ ocount, uint8_t *__restrict__ mark,
                                const uint32_t *__restrict__ bnd) {
  const uint64_t w_lo = w_range[0], w_hi = w_range[1];  // the level plan (k_plan)
  __shared__ uint32_t s_wcnt[BLOCK / WAVE];
  __shared__ WaveStage s_stage[BLOCK / WAVE];
  const uint64_t E0 = e_lo & ~3ull;
  const uint64_t T = e_hi - E0;
  // CSR: the block ranges k_csr_bounds balanced by cost (whole 1024-edge tiles, so every wave's 256-edge
  // part starts on the trow grid)
  const uint64_t Q = ((T + gridDim.x - 1) / gridDim.x + 3) & ~3ull;
  const uint64_t vb = CSR ? bnd[blockIdx.x] : Q * blockIdx.x;
  const uint64_t ve = CSR ? bnd[blockIdx.x + 1] : ((vb + Q < T) ? vb + Q : T);
  const uint64_t eb = E0 + vb;  // first edge of this block
  const uint64_t nbytes = ve > vb ? (ve - vb) * 4 : 0;
  const __amdgpu_buffer_rsrc_t ru = make_rsrc(CSR ? ev : eu + eb, CSR ? 0 : nbytes);
  const __amdgpu_buffer_rsrc_t rv = make_rsrc(ev + eb, nbytes);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(ew + eb, nbytes);
  const uint32_t lane_off = threadIdx.x * 16u;
  const uint4 *bits4 = reinterpret_cast<const uint4 *>(giant_bits);
  const uint32_t *bits32 = reinterpret_cast<const uint32_t *>(giant_bits);
  const uint32_t giant = giant_ptr[0];
  bool touch_giant = false;  // a level edge of this block has an end in the giant
  uint64_t nlev = 0, nrem = 0;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  // CSR: the rows of the wave's part of the tile (k_csr_tiles' trow: R0 holds its first edge, R1
  // its end), the next tile's part's (loaded a tile ahead), and this part's first window (prefetched)
  const uint64_t ntiles = (T + 255) >> 8;
  auto trow_at = [&](uint64_t t) -> uint32_t { return trow[t < ntiles ? t : ntiles]; };
  const uint64_t t0w = (vb >> 8) + wid;  // the wave's part of the block's first tile
  uint32_t R0 = CSR ? trow_at(t0w) : 0u, R1 = CSR ? trow_at(t0w + 1) : 0u;
  uint32_t N0 = CSR ? trow_at(t0w + 4) : 0u, N1 = CSR ? trow_at(t0w + 5) : 0u;
  uint32_t w0 = CSR ? csr_win(eoff, n, R0 + 1) : 0u;
  uint4 ca = CSR ? make_uint4(0u, 0u, 0u, 0u) : ld_b128_nt(ru, lane_off);
  uint4 cb = ld_b128_nt(rv, lane_off), cw = ld_b128_nt(rw, lane_off);
  for (uint64_t v0 = vb; v0 < ve; v0 += ARCS_PER_BLOCK) {
    const uint64_t v = v0 + (uint64_t)threadIdx.x * 4;
    const uint64_t e0 = E0 + v;
    uint32_t a[4] = {ca.x, ca.y, ca.z, ca.w};
    const uint32_t b[4] = {cb.x, cb.y, cb.z, cb.w}, w[4] = {cw.x, cw.y, cw.z, cw.w};
    if (CSR) {
      const uint32_t r0 = R0, r1 = R1, w = w0;
      const uint64_t tw = ((v0 + ARCS_PER_BLOCK) >> 8) + wid;  // the wave's part of the next tile
      R0 = N0;
      R1 = N1;
      w0 = csr_win(eoff, n, R0 + 1);  // the next part's window, in flight during this tile
      N0 = trow_at(tw + 4);
      N1 = trow_at(tw + 5);
      const uint64_t vw = v0 + (uint64_t)wid * (WAVE * 4);  // the wave's part (wave-uniform)
      // the head table lives in the wave's staging area (free between the tiles' stage_write calls),
      // so the block stays at 20 KiB of LDS: 8 blocks per CU
      if (vw < ve) csr_tile_rows<true>(eoff, n, r0, r1, (uint32_t)(E0 + vw), s_stage[wid].a, a, w);
    }
    const uint32_t nv = v < ve ? (uint32_t)((ve - v) < 4 ? (ve - v) : 4) : 0u;
    const uint32_t nskip = e0 < e_lo ? (uint32_t)(e_lo - e0) : 0u;
    bool out[4];
    // probes, all issued before any is used. a is sorted: two 16-B probes cover the 128-vertex
    // blocks of a[0] and a[3]; an a[j] outside both (a tile spanning > 2 blocks) counts as
    // outside the giant, so its edge is kept — always safe. b is random: one 32-bit word per
    // edge. Lanes that need no probe read word 0 (one request per wave instruction).
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j] = ((uint32_t)j < nv) & ((uint32_t)j >= nskip) & ((uint64_t)w[j] >= w_lo);
    // block indices and probed words from the same guard (an unguarded lane probes block 0 and
    // says so): an in-range a is a checked vertex id; a masked one may not be
    const bool in0 = ((uint32_t)0 < nv) & (0u >= nskip), in3 = (3u < nv) & (3u >= nskip);
    const uint32_t A0 = in0 ? (a[0] >> 7) : 0u, A3 = in3 ? (a[3] >> 7) : 0u;
    const uint4 q0 = bits4[A0];
    const uint4 q3 = bits4[A3];
    uint32_t gbw[4];
#if !GHS_FILTER_GATED
#pragma unroll
    for (int j = 0; j < 4; ++j) gbw[j] = bits32[out[j] ? (b[j] >> 5) : 0u];
#endif
    uint32_t ga[4], gb[4];
#if GHS_FILTER_GATED
    // gated b-probes: only an edge whose a-end is in the giant can be dropped, so the random
    // b-probe (one L2 request) is issued for those edges alone, after the a-probes landed (the
    // sequential a-probes are near-always L2 hits); the next tile's stream loads follow them
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t blk = a[j] >> 7, wsel = (a[j] >> 5) & 3;
      const uint4 q = (blk == A0) ? q0 : q3;
      const bool odd = wsel & 1;
      const uint32_t lo = odd ? q.y : q.x, hi = odd ? q.w : q.z;
      const uint32_t word = (wsel & 2) ? hi : lo;
      ga[j] = ((blk == A0) | (blk == A3)) ? (word >> (a[j] & 31)) & 1u : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) gbw[j] = bits32[(out[j] & (ga[j] != 0u)) ? (b[j] >> 5) : 0u];
#endif
    // next tile (out-of-range offsets read 0)
    const uint32_t noff = (uint32_t)(v0 + ARCS_PER_BLOCK - vb) * 4u + lane_off;
    if (!CSR) ca = ld_b128_nt(ru, noff);
    cb = ld_b128_nt(rv, noff);
    cw = ld_b128_nt(rw, noff);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#if !GHS_FILTER_GATED
      const uint32_t blk = a[j] >> 7, wsel = (a[j] >> 5) & 3;
      const uint4 q = (blk == A0) ? q0 : q3;
      const bool odd = wsel & 1;  // two-level select (an == chain becomes a branch tree)
      const uint32_t lo = odd ? q.y : q.x, hi = odd ? q.w : q.z;
      const uint32_t word = (wsel & 2) ? hi : lo;
      ga[j] = ((blk == A0) | (blk == A3)) ? (word >> (a[j] & 31)) & 1u : 0u;
#endif
#if GHS_FILTER_GATED
      gb[j] = ga[j] & (gbw[j] >> (b[j] & 31));  // unprobed b: "not known in the giant" (lab gathered)
#else
      gb[j] = (gbw[j] >> (b[j] & 31)) & 1u;
#endif
      out[j] = out[j] & ((ga[j] & gb[j]) == 0u);  // bitwise (no && : keeps the probes unsunk)
    }
    // level-1 split: labels only for this level's edges, and only for ends outside the giant
    // (a set bit IS lab[x] == giant: the bitmap was built from the same labels)
    bool lev[4], rem[4];
    uint32_t la[4], lb[4];
    uint64_t key[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lev[j] = out[j] & ((uint64_t)w[j] < w_hi);
      rem[j] = out[j] & !lev[j];
      la[j] = lab[(lev[j] & (ga[j] == 0u)) ? a[j] : 0u];
      lb[j] = lab[(lev[j] & (gb[j] == 0u)) ? b[j] : 0u];
      la[j] = ga[j] ? giant : la[j];
      lb[j] = gb[j] ? giant : lb[j];
      key[j] = ((uint64_t)w[j] << 32) | (uint32_t)(e0 + j);
    }
    uint32_t lmask = 0, rmask = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lev[j] = lev[j] & (la[j] != lb[j]);
      lmask |= lev[j] ? (1u << j) : 0u;
      rmask |= rem[j] ? (1u << j) : 0u;
      if (lev[j] && mark) {  // active fragments of the level; the giant's flag once per block
        if (!ga[j]) mark[la[j]] = 1;
        if (!gb[j]) mark[lb[j]] = 1;
        touch_giant |= (ga[j] | gb[j]) != 0u;
      }
    }
    const Offs2 o = block_offsets_w2((uint32_t)__popc(lmask), (uint32_t)__popc(rmask), s_wcnt);
    // in canonical (eid) order, within and across the output regions: the LDS tail's (w, index)
    // minima rely on it (k_tail_open checks it under GHS_OPT_CHECK_TOTALS)
    stage_write(s_stage[threadIdx.x / WAVE], la, lb, key, lmask, o.lane_excl[0], o.wave_cnt[0], lsrc, ldst, lkey,
                vb + nlev + o.wave_before[0]);
    stage_write(s_stage[threadIdx.x / WAVE], a, b, key, rmask, o.lane_excl[1], o.wave_cnt[1], osrc, odst, okey,
                vb + nrem + o.wave_before[1]);
    nlev += o.total[0];
    nrem += o.total[1];
  }
  if (__syncthreads_or(touch_giant ? 1 : 0) && threadIdx.x == 0 && mark) mark[giant] = 1;
  // both outputs padded to a multiple of 4 with dead entries (a = LABEL_NONE)
  const uint64_t padded = (nrem + 3) & ~3ull, lpadded = (nlev + 3) & ~3ull;
  if (threadIdx.x < padded - nrem) {
    const uint64_t pos = vb + nrem + threadIdx.x;
    osrc[pos] = LABEL_NONE;
    odst[pos] = 0;
    okey[pos] = KEY_NONE;
  }
  if (threadIdx.x < lpadded - nlev) {
    const uint64_t pos = vb + nlev + threadIdx.x;
    lsrc[pos] = LABEL_NONE;
    ldst[pos] = 0;
    lkey[pos] = KEY_NONE;
  }
  if (threadIdx.x == 0) {
    lstart[blockIdx.x] = vb;
    lcount[blockIdx.x] = (vb < T) ? lpadded : 0;
    ostart[blockIdx.x] = vb;
    ocount[blockIdx.x] = (vb < T) ? padded : 0;
  }
}

// ------------------------------------------------------------------------------------------
// Level pass over the PENDING edges (levels >= 1). Splits them into (a) this level's edges whose
// ends lie in different fragments -> (lab[u], lab[v], key) into this block's level staging
// region, and (b) heavier edges that also survive the fragment test -> (u, v, key) into this
// block's REMAINING region, the next level's input. Edges whose ends share a fragment are
// dropped for good (cycle property). lab is fully resolved (one hop); the giant-fragment bitmap
// rejects most heavy edges without a label gather. Block-private regions, no atomics.
// ------------------------------------------------------------------------------------------
GHS_STREAM_KERNEL_6 void k_level_pass(const uint32_t *__restrict__ ru, const uint32_t *__restrict__ rv,
                                    const uint64_t *__restrict__ rkey, SegView in, const uint64_t *__restrict__ w_hi_p,
                                    const uint32_t *__restrict__ lab, const uint64_t *__restrict__ giant_bits,
                                    const uint32_t *__restrict__ giant_ptr,
                                    uint32_t *__restrict__ lsrc, uint32_t *__restrict__ ldst,
                                    uint64_t *__restrict__ lkey, uint64_t *__restrict__ lstart,
                                    uint64_t *__restrict__ lcount, uint32_t *__restrict__ ou, uint32_t *__restrict__ ov, uint64_t *__restrict__ okey,
                                    uint64_t *__restrict__ ostart, uint64_t *__restrict__ ocount,
                                    uint8_t *__restrict__ mark) {
  const uint64_t w_hi = *w_hi_p;  // the level plan (k_plan)
  __shared__ uint32_t s_wcnt[BLOCK / WAVE];
  __shared__ uint32_t s_seg[2];
  __shared__ WaveStage s_stage[BLOCK / WAVE];
  const uint64_t T = in.prefix[in.nseg];
  const uint64_t Q = ((T + gridDim.x - 1) / gridDim.x + 3) & ~3ull;
  const uint64_t vb = Q * blockIdx.x;
  const uint64_t ve = (vb + Q < T) ? vb + Q : T;
  if (threadIdx.x < WAVE) seg_range_wave(in.prefix, in.nseg, vb, ve, T, s_seg);
  __syncthreads();
  const uint32_t slo = s_seg[0], shi = s_seg[1];
  // regions hold multiples of 4 entries and start at multiples of 4, so a lane's 4-entry tile
  // is either wholly inside one region or past ve; past-ve tiles read a valid tile (index 0)
  // and are masked, so every load is unconditional
  auto tile_index = [&](uint64_t v) -> uint64_t {
    if (v >= ve) return 0;
    const uint32_t sidx = (slo == shi) ? slo : seg_find(in.prefix, slo, shi, v);
    return in.start[sidx] + (v - in.prefix[sidx]);
  };
  const uint4 *bits4 = reinterpret_cast<const uint4 *>(giant_bits);
  const uint32_t *bits32 = reinterpret_cast<const uint32_t *>(giant_bits);
  const uint32_t giant = giant_ptr[0];
  bool touch_giant = false;  // a level edge of this block has an end in the giant
  uint64_t nlev = 0, nrem = 0;
  uint64_t i0 = tile_index(vb + (uint64_t)threadIdx.x * 4);
  uint4 ca = *reinterpret_cast<const uint4 *>(ru + i0), cb = *reinterpret_cast<const uint4 *>(rv + i0);
  ulonglong2 ck01 = *reinterpret_cast<const ulonglong2 *>(rkey + i0);
  ulonglong2 ck23 = *reinterpret_cast<const ulonglong2 *>(rkey + i0 + 2);
  for (uint64_t v0 = vb; v0 < ve; v0 += ARCS_PER_BLOCK) {
    const uint64_t v = v0 + (uint64_t)threadIdx.x * 4;
    const bool valid = v < ve;
    const uint32_t a[4] = {ca.x, ca.y, ca.z, ca.w}, b[4] = {cb.x, cb.y, cb.z, cb.w};
    const uint64_t k[4] = {ck01.x, ck01.y, ck23.x, ck23.y};
    bool live[4], lev[4], rem[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) live[j] = valid & (a[j] != LABEL_NONE);
    // giant-bitmap probes (a sorted within a region: two 16-B probes cover a[0]'s and a[3]'s
    // 128-vertex blocks; an a[j] outside both counts as outside the giant — safe), issued
    // before the next tile's loads
    // block indices and probed words from the same guard (a dead entry has a == LABEL_NONE)
    const uint32_t A0 = live[0] ? (a[0] >> 7) : 0u, A3 = live[3] ? (a[3] >> 7) : 0u;
    const uint4 q0 = bits4[A0];
    const uint4 q3 = bits4[A3];
    uint32_t gbw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) gbw[j] = bits32[live[j] ? (b[j] >> 5) : 0u];
    // next tile
    i0 = tile_index(v + ARCS_PER_BLOCK);
    ca = *reinterpret_cast<const uint4 *>(ru + i0);
    cb = *reinterpret_cast<const uint4 *>(rv + i0);
    ck01 = *reinterpret_cast<const ulonglong2 *>(rkey + i0);
    ck23 = *reinterpret_cast<const ulonglong2 *>(rkey + i0 + 2);
    // REJECT a whole class at once: both ends in the giant fragment
    uint32_t ga[4], gb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t blk = a[j] >> 7, wsel = (a[j] >> 5) & 3;
      const uint4 q = (blk == A0) ? q0 : q3;
      const bool odd = wsel & 1;
      const uint32_t lo = odd ? q.y : q.x, hi = odd ? q.w : q.z;
      const uint32_t word = (wsel & 2) ? hi : lo;
      ga[j] = ((blk == A0) | (blk == A3)) ? (word >> (a[j] & 31)) & 1u : 0u;
      gb[j] = (gbw[j] >> (b[j] & 31)) & 1u;
      live[j] = live[j] & ((ga[j] & gb[j]) == 0u);
    }
    // level/remaining split; labels are gathered only for this level's edges (they become arcs
    // and need the fragment test) — heavier edges are carried forward raw, the bitmap of the
    // next level (a larger giant) rejects most of them without any gather
    uint32_t la[4], lb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool in_level = (k[j] >> 32) < w_hi;
      lev[j] = live[j] & in_level;
      rem[j] = live[j] & !in_level;
      la[j] = lab[(lev[j] & (ga[j] == 0u)) ? a[j] : 0u];  // ends in the giant: no gather
      lb[j] = lab[(lev[j] & (gb[j] == 0u)) ? b[j] : 0u];
      la[j] = ga[j] ? giant : la[j];
      lb[j] = gb[j] ? giant : lb[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) lev[j] = lev[j] & (la[j] != lb[j]);
    uint32_t mlev = 0, mrem = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mlev += lev[j] ? 1u : 0u;
      mrem += rem[j] ? 1u : 0u;
    }
    uint32_t lmask = 0, rmask = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lmask |= lev[j] ? (1u << j) : 0u;
      rmask |= rem[j] ? (1u << j) : 0u;
      if (lev[j] && mark) {  // active fragments of the level; the giant's flag once per block
        if (!ga[j]) mark[la[j]] = 1;
        if (!gb[j]) mark[lb[j]] = 1;
        touch_giant |= (ga[j] | gb[j]) != 0u;
      }
    }
    const Offs2 o = block_offsets_w2(mlev, mrem, s_wcnt);
    // in canonical (eid) order, within and across the output regions: the LDS tail's (w, index)
    // minima rely on it (k_tail_open checks it under GHS_OPT_CHECK_TOTALS)
    stage_write(s_stage[threadIdx.x / WAVE], la, lb, k, lmask, o.lane_excl[0], o.wave_cnt[0], lsrc, ldst, lkey,
                vb + nlev + o.wave_before[0]);
    stage_write(s_stage[threadIdx.x / WAVE], a, b, k, rmask, o.lane_excl[1], o.wave_cnt[1], ou, ov, okey,
                vb + nrem + o.wave_before[1]);
    nlev += o.total[0];
    nrem += o.total[1];
  }
  if (__syncthreads_or(touch_giant ? 1 : 0) && threadIdx.x == 0 && mark) mark[giant] = 1;
  // both outputs padded to a multiple of 4 with dead entries (a = LABEL_NONE)
  const uint64_t padded = (nrem + 3) & ~3ull, lpadded = (nlev + 3) & ~3ull;
  if (threadIdx.x < padded - nrem) {
    const uint64_t pos = vb + nrem + threadIdx.x;
    ou[pos] = LABEL_NONE;
    ov[pos] = 0;
    okey[pos] = KEY_NONE;
  }
  if (threadIdx.x < lpadded - nlev) {
    const uint64_t pos = vb + nlev + threadIdx.x;
    lsrc[pos] = LABEL_NONE;
    ldst[pos] = 0;
    lkey[pos] = KEY_NONE;
  }
  if (threadIdx.x == 0) {
    lstart[blockIdx.x] = vb;
    lcount[blockIdx.x] = (vb < T) ? lpadded : 0;
    ostart[blockIdx.x] = vb;
    ocount[blockIdx.x] = (vb < T) ? padded : 0;
  }
}

// ------------------------------------------------------------------------------------------
// Bucketed rounds (lattice-like graphs: the plan's sample of edge spans says nearly every edge
// joins vertices close in id). A round's per-fragment minima are taken in LDS instead of through
// global 64-bit atomics, which execute at the memory side (~27 G/s on MI355X, the lattice's
// bound): the live edges are grouped by target bucket (2^bs consecutive labels) and one workgroup
// per bucket keeps that bucket's minima in LDS (ds_min_u64), then finds every target's winning
// edge in a second sweep and hooks it — par[t] = other end, best[t] = key, in_mst[eid] = 1 —
// single writer per target, no global atomics and no separate CONNECT pass (the reference's
// TEST/ACCEPT/REPORT convergecast and CHANGEROOT/CONNECT, ghs_implementation.py:155-353, as two
// passes over a bucket). Mutual pairs stay 2-cycles for the jump (k_jump / k_jump_ident).
//  k_bucket  block g streams its share of the live edges twice: pass A counts records per bucket
//            (an edge is a record of bucket(a), and of bucket(b) when that differs), one LDS
//            scan turns the counts into offsets in the block's record region, written bucket-major
//            (O[t][g]: a bucket's offsets are contiguous), pass B writes the records (a, b, key)
//            at LDS cursors. On a lattice a block's edges touch a handful of buckets, so the
//            records leave in long runs.
//  k_bmin    one workgroup per bucket: its runs from every region (offsets and their scan in
//            LDS), min per target in LDS, winners.
// ------------------------------------------------------------------------------------------
constexpr uint32_t BK_G = 512;        // k_bucket blocks = record regions
constexpr uint32_t BK_T = 512;        // k_bucket threads
constexpr uint32_t BK_MAX_B = 16384;  // buckets: k_bucket's LDS counters (64 KiB)
constexpr uint32_t BM_T = 1024;       // k_bmin threads
#ifndef GHS_BK_TILES
#define GHS_BK_TILES 2
#endif
constexpr int BK_TILES = GHS_BK_TILES;  // k_bucket: 4-edge tiles per lane in flight

// The offsets table of a bucketed round, (nb + 1) x BK_G words. Block-major (region g's nb + 1
// offsets contiguous: k_bucket writes its row with coalesced stores; k_bmin's workgroup t reads one
// word per region) — GHS_BK_BLOCKMAJOR=0: bucket-major (a bucket's 512 offsets contiguous: k_bmin
// reads one row, but every k_bucket block writes a strided column, nb + 1 scattered 4-B stores).
#ifndef GHS_BK_BLOCKMAJOR
#define GHS_BK_BLOCKMAJOR 1
#endif
__device__ __forceinline__ uint64_t bk_off_index(uint32_t t, uint32_t g, uint32_t nb) {
  return GHS_BK_BLOCKMAJOR ? (uint64_t)g * (nb + 1) + t : (uint64_t)t * BK_G + g;
}

// a block's share of the T live edges (a multiple of 4: whole 4-entry tiles); region g of the
// records starts at 2 * quota * g (an edge gives at most two records)
__device__ __forceinline__ uint64_t bk_quota(uint64_t T) { return ((T + BK_G - 1) / BK_G + 3) & ~3ull; }

// the hot fragments of a level-first round in an LDS hash (HOT_K labels in HOT_HASH slots)
constexpr uint32_t HOT_HASH = 4 * HOT_K;
constexpr uint32_t HOT_MARK = 0x80000000u;  // a record's hot end (labels < n <= 2^28)
__device__ __forceinline__ uint32_t hot_slot(uint32_t x) { return (x * 0x9E3779B1u) >> 24; }
static_assert(HOT_HASH == 256, "hot_slot yields 8 bits");
__device__ __forceinline__ void hot_insert(uint32_t *s_hl, uint32_t *s_hi, uint32_t x, uint32_t idx) {
  for (uint32_t h = hot_slot(x);; h = (h + 1) & (HOT_HASH - 1)) {
    if (atomicCAS(&s_hl[h], LABEL_NONE, x) == LABEL_NONE) {
      s_hi[h] = idx;
      return;
    }
  }
}
// index of x among the hot labels, or -1 (the caller synchronised after the inserts)
__device__ __forceinline__ int hot_find(const uint32_t *s_hl, const uint32_t *s_hi, uint32_t x) {
  for (uint32_t h = hot_slot(x);; h = (h + 1) & (HOT_HASH - 1)) {
    const uint32_t l = s_hl[h];
    if (l == x) return (int)s_hi[h];
    if (l == LABEL_NONE) return -1;
  }
}

// exclusive scan over the NT threads of a block (NT / 64 waves); *total = the block's sum
template <uint32_t NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t mine, uint32_t *s_wsum, uint32_t *total) {
  const uint32_t lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  uint32_t incl = mine;
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const uint32_t o = __shfl_up(incl, d);
    if ((int)lane >= d) incl += o;
  }
  if (lane == WAVE - 1) s_wsum[wid] = incl;
  __syncthreads();
  uint32_t before = incl - mine, t = 0;
#pragma unroll
  for (uint32_t w = 0; w < NT / WAVE; ++w) {
    if (w < wid) before += s_wsum[w];
    t += s_wsum[w];
  }
  *total = t;
  __syncthreads();
  return before;
}

// Wave-aggregated LDS bump: every active lane (act) adds one to counter s_h[bkt]; lanes with equal
// buckets are served by one atomic of their leader, and each lane gets its own slot (the old
// counter value + its rank among the lanes of its bucket, in lane order: consecutive lanes of a
// run of equal buckets get consecutive slots, so their record stores coalesce). Lattice edges put
// one or two buckets in a wave instruction; after BK_AGG_ROUNDS distinct buckets the remaining
// lanes take one atomic each (random graphs, forced mode). Every lane of the wave must call it.
constexpr int BK_AGG_ROUNDS = 4;
template <bool RET>
__device__ __forceinline__ uint32_t lds_bump(uint32_t *s_h, uint32_t bkt, bool act) {
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint64_t pending = __ballot(act);
  uint32_t slot = 0;
  for (int it = 0; it < BK_AGG_ROUNDS && pending; ++it) {
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)pending) - 1;
    const uint32_t lb = __shfl(bkt, leader);
    const uint64_t same = __ballot(act && bkt == lb) & pending;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&s_h[lb], (uint32_t)__popcll(same));
    if (RET) {
      base = __shfl(base, leader);
      if ((same >> lane) & 1ull) slot = base + (uint32_t)__popcll(same & below);
    }
    pending &= ~same;
  }
  if ((pending >> lane) & 1ull) {
    const uint32_t b = atomicAdd(&s_h[bkt], 1u);
    if (RET) slot = b;
  }
  return slot;
}

__global__ __launch_bounds__(BK_T) void k_bucket(const uint32_t *__restrict__ src, const uint32_t *__restrict__ dst,
                                                 const uint64_t *__restrict__ key, SegView in, uint32_t bs,
                                                 uint32_t nb, uint4 *__restrict__ rec, uint32_t *__restrict__ O,
                                                 const unsigned long long *__restrict__ guard_nact,
                                                 const uint32_t *__restrict__ hot, uint64_t *__restrict__ best,
                                                 const unsigned long long *__restrict__ only_if) {
  __shared__ uint32_t s_h[BK_MAX_B + 1];
  __shared__ uint32_t s_seg[2];
  __shared__ uint32_t s_wsum[BK_T / WAVE];
  __shared__ uint32_t s_hl[HOT_HASH];          // hot label -> its index (linear probing)
  __shared__ uint32_t s_hi[HOT_HASH];
  __shared__ unsigned long long s_hmin[HOT_K];  // this block's minimum per hot fragment
  // a lookahead round past the level's end (<= 1 active fragment) writes empty regions
  const bool noop = guard_nact && *guard_nact <= 1;
  // a level's first round past level 0: the hot fragments' candidates (the giant's: most of the
  // level's edges) are reduced in LDS and leave the block as one atomicMin on best[] each, instead
  // of filling one bucket each that a single k_bmin workgroup would have to sweep. A record's hot
  // end is marked (bit 31: bucketed solves have n <= 2^28), so k_bmin never takes it as a target.
  if (only_if && !*only_if) return;  // the windowed round ran (k_wmin)
  // a no-op lookahead round: k_bmin reads no offsets either (its own guard), so nothing is written
  // (the offset table alone is (nb + 1) x BK_G words: ~0.1 ms on the 16384^2 grids)
  if (noop) return;
  const uint32_t nhot = hot ? hot[0] : 0u;
  const uint32_t hot0 = nhot ? hot[1] : LABEL_NONE;  // one hot fragment (R-MAT: the giant): a compare
  for (uint32_t i = threadIdx.x; i < HOT_HASH; i += BK_T) s_hl[i] = LABEL_NONE;
  if (threadIdx.x < HOT_K) s_hmin[threadIdx.x] = KEY_NONE;
  __syncthreads();
  if (threadIdx.x < nhot) hot_insert(s_hl, s_hi, hot[1 + threadIdx.x], threadIdx.x);
  auto hidx = [&](uint32_t x) -> int { return nhot == 1 ? (x == hot0 ? 0 : -1) : hot_find(s_hl, s_hi, x); };
  const uint64_t T = noop ? 0 : in.prefix[in.nseg];
  const uint64_t Q = bk_quota(T);
  const uint64_t vb = Q * blockIdx.x;
  const uint64_t ve = (vb + Q < T) ? vb + Q : T;
  for (uint32_t i = threadIdx.x; i <= nb; i += BK_T) s_h[i] = 0;
  if (threadIdx.x < WAVE) seg_range_wave(in.prefix, in.nseg, vb, ve, T, s_seg);
  __syncthreads();
  const uint32_t slo = s_seg[0], shi = s_seg[1];
  // pass A: records per bucket (the a and b ends only); every lane of a wave iterates while the
  // wave's first tile is in range (the bumps are wave-collective); BK_TILES 4-edge tiles per lane
  // per iteration, all loads issued before the first bump
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  constexpr uint64_t STRIDE = (uint64_t)BK_T * 4;
  for (uint64_t v0 = vb + (uint64_t)threadIdx.x * 4; v0 - lane * 4 < ve; v0 += STRIDE * BK_TILES) {
    uint4 a4[BK_TILES], b4[BK_TILES];
#pragma unroll
    for (int q = 0; q < BK_TILES; ++q) {
      const uint64_t i0 = tile_phys(in, slo, shi, v0 + STRIDE * q, ve);
      a4[q] = *reinterpret_cast<const uint4 *>(src + i0);
      b4[q] = *reinterpret_cast<const uint4 *>(dst + i0);
    }
#pragma unroll
    for (int q = 0; q < BK_TILES; ++q) {
      const uint64_t v = v0 + STRIDE * q;
      const uint32_t A[4] = {a4[q].x, a4[q].y, a4[q].z, a4[q].w}, B[4] = {b4[q].x, b4[q].y, b4[q].z, b4[q].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool live = (v < ve) & (A[j] != LABEL_NONE);  // past the range / region padding
        const uint32_t ba = A[j] >> bs, bb = B[j] >> bs;
        const bool ea = live && (!nhot || hidx(A[j]) < 0);
        const bool eb = live && (!nhot || hidx(B[j]) < 0) && (bb != ba || !ea);
        lds_bump<false>(s_h, ba, ea);
        lds_bump<false>(s_h, bb, eb);
      }
    }
  }
  __syncthreads();
  // counts -> offsets in place (each thread a run of consecutive buckets), s_h[nb] = total
  const uint32_t per = (nb + BK_T - 1) / BK_T, c0 = threadIdx.x * per;
  uint32_t sum = 0;
  for (uint32_t i = 0; i < per && c0 + i < nb; ++i) sum += s_h[c0 + i];
  uint32_t tot;
  uint32_t run = block_excl_scan<BK_T>(sum, s_wsum, &tot);
  for (uint32_t i = 0; i < per && c0 + i < nb; ++i) {
    const uint32_t c = s_h[c0 + i];
    s_h[c0 + i] = run;
    run += c;
  }
  if (threadIdx.x == 0) s_h[nb] = tot;
  __syncthreads();
  for (uint32_t t = threadIdx.x; t <= nb; t += BK_T) O[bk_off_index(t, blockIdx.x, nb)] = s_h[t];
  __syncthreads();  // the cursors below advance s_h
  // pass B: the records at the cursors of their buckets
  const uint64_t base = 2 * vb;
  for (uint64_t v0 = vb + (uint64_t)threadIdx.x * 4; v0 - lane * 4 < ve; v0 += STRIDE * BK_TILES) {
    uint4 a4[BK_TILES], b4[BK_TILES];
    ulonglong2 k01[BK_TILES], k23[BK_TILES];
#pragma unroll
    for (int q = 0; q < BK_TILES; ++q) {
      const uint64_t i0 = tile_phys(in, slo, shi, v0 + STRIDE * q, ve);
      a4[q] = *reinterpret_cast<const uint4 *>(src + i0);
      b4[q] = *reinterpret_cast<const uint4 *>(dst + i0);
      k01[q] = *reinterpret_cast<const ulonglong2 *>(key + i0);
      k23[q] = *reinterpret_cast<const ulonglong2 *>(key + i0 + 2);
    }
#pragma unroll
    for (int q = 0; q < BK_TILES; ++q) {
      const uint64_t v = v0 + STRIDE * q;
      const uint32_t A[4] = {a4[q].x, a4[q].y, a4[q].z, a4[q].w}, B[4] = {b4[q].x, b4[q].y, b4[q].z, b4[q].w};
      const uint64_t K[4] = {k01[q].x, k01[q].y, k23[q].x, k23[q].y};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool live = (v < ve) & (A[j] != LABEL_NONE);
        const uint32_t ba = A[j] >> bs, bb = B[j] >> bs;
        const int ha = (live && nhot) ? hidx(A[j]) : -1;
        const int hb = (live && nhot) ? hidx(B[j]) : -1;
        const bool ea = live && ha < 0;
        const bool eb = live && hb < 0 && (bb != ba || !ea);
        const uint32_t pa = lds_bump<true>(s_h, ba, ea);
        const uint32_t pb = lds_bump<true>(s_h, bb, eb);
        const uint4 r = make_uint4(A[j] | (ha >= 0 ? HOT_MARK : 0u), B[j] | (hb >= 0 ? HOT_MARK : 0u), (uint32_t)K[j],
                                   (uint32_t)(K[j] >> 32));
        if (ea) rec[base + pa] = r;
        if (eb) rec[base + pb] = r;
        if (ha >= 0 && K[j] < s_hmin[ha]) atomicMin(&s_hmin[ha], (unsigned long long)K[j]);
        if (hb >= 0 && K[j] < s_hmin[hb]) atomicMin(&s_hmin[hb], (unsigned long long)K[j]);
      }
    }
  }
  if (nhot) {
    __syncthreads();
    if (threadIdx.x < nhot && s_hmin[threadIdx.x] != KEY_NONE) flush_min(best, hot[1 + threadIdx.x], s_hmin[threadIdx.x]);
  }
}

// k_bmin: BM_ILP records in flight per lane; the bucket's non-empty runs listed first (a lattice
// bucket's records come from one to three block regions), so locating a record searches that
// short list
#ifndef GHS_BM_ILP
#define GHS_BM_ILP 8
#endif
constexpr int BM_ILP = GHS_BM_ILP;
#ifndef GHS_BM_COMPRESS
#define GHS_BM_COMPRESS 1
#endif

// The LDS core of a bucketed round (k_bmin over records, k_wmin over a window of the level's edge
// list): `sweep(f)` calls f(a, b, key) for every candidate edge of bucket t (block-wide: every
// thread calls it, each thread gets its share); s_min holds KEY_NONE in every slot.
// FULL (level 0's windowed round 0): best and par of EVERY vertex of the bucket below n are written
// (KEY_NONE / itself where nothing hooks), so the solve starts without initialising them.
// eu != nullptr (level 0: the labels are the vertices): a target's winner comes from its minimum's
// canonical ends (two gathers per target) instead of a second sweep over the candidates (k_wmin:
// its window is four times the bucket's edges and does not stay in L2 — PMC: every edge read 4x)
template <uint32_t BS, bool FULL, class Sweep>
__device__ __forceinline__ void bucket_round(uint32_t t, unsigned long long *s_min, Sweep sweep,
                                             uint32_t *__restrict__ par, uint64_t *__restrict__ best,
                                             uint8_t *__restrict__ in_mst, uint32_t n,
                                             const uint32_t *__restrict__ eu = nullptr,
                                             const uint32_t *__restrict__ ev = nullptr) {
  constexpr uint32_t SPAN = 1u << BS;
  const uint32_t tb = t << BS;
  // sweep 1: every target's minimum. A hot end (HOT_MARK) is never this bucket's target. A plain
  // read first (slots only decrease): records of a large fragment all target one slot, and
  // same-address LDS atomics of a wave serialise
  sweep([&](uint32_t a, uint32_t b, unsigned long long k) {
    if ((a >> BS) == t && k < s_min[a - tb]) atomicMin(&s_min[a - tb], k);
    if ((b >> BS) == t && k < s_min[b - tb]) atomicMin(&s_min[b - tb], k);
  });
  __syncthreads();
  // the bucket's minima leave LDS in target order (one writer per target, consecutive lanes on
  // consecutive slots): best[] and the MSF flag of every target's minimum edge. Scattered per-winner
  // stores from the record sweep below measured 22 GB of HBM writes per 16384^2-grid solve for
  // ~5 GB of payload (record order is not target order, and the records' stream evicts the
  // partially written lines).
  for (uint32_t i = threadIdx.x; i < SPAN; i += BM_T) {
    const uint64_t v = s_min[i];
    if (v != KEY_NONE) {
      best[tb + i] = v;
      in_mst[(uint32_t)v] = 1;
    } else if (FULL && tb + i < n) {
      best[tb + i] = KEY_NONE;
    }
  }
  __syncthreads();
  // winners: exactly one record per target holds its minimum (keys are unique); it replaces the
  // slot by a tag carrying the other end (bit 31 set: a key's eid is < 2^31, so a tag never equals
  // a key, and KEY_NONE's low word is not the tag's)
  constexpr uint64_t TAG = 0x80000000ull;
  if (eu) {
    for (uint32_t i = threadIdx.x; i < SPAN; i += BM_T) {
      const uint64_t v = s_min[i];
      if (v == KEY_NONE) continue;
      const uint32_t eid = (uint32_t)v, a = eu[eid], b = ev[eid];
      s_min[i] = ((uint64_t)(a == tb + i ? b : a) << 32) | TAG;
    }
  } else {
    sweep([&](uint32_t a, uint32_t b, unsigned long long k) {
      if ((a >> BS) == t && s_min[a - tb] == k) s_min[a - tb] = ((uint64_t)(b & ~HOT_MARK) << 32) | TAG;
      if ((b >> BS) == t && s_min[b - tb] == k) s_min[b - tb] = ((uint64_t)(a & ~HOT_MARK) << 32) | TAG;
    });
  }
  __syncthreads();
  // Hook chains inside the bucket, compressed here so the jump walks fewer random steps (a
  // lattice's horizontal hooks stay in their row's bucket). First a mutual pair inside the bucket
  // keeps its smaller member as the root (its slot is cleared: par is not written, so it stays a
  // root); pairs across buckets stay 2-cycles for the jump. Then pointer jumping over the tags:
  // a slot whose parent lies in the bucket and hooked too takes the parent's parent — pointers
  // only move to ancestors, so concurrent updates are safe. par then points at the first
  // ancestor outside the bucket, the in-bucket root, or a member of a cross-bucket pair.
  auto in_bucket = [&](uint64_t v) -> bool { return (uint32_t)v == (uint32_t)TAG && ((uint32_t)(v >> 32) >> BS) == t; };
  if (GHS_BM_COMPRESS) {
  for (uint32_t i = threadIdx.x; i < SPAN; i += BM_T) {
    const uint64_t v = s_min[i];
    if (!in_bucket(v)) continue;
    const uint32_t o = (uint32_t)(v >> 32) - tb;
    if (s_min[o] == (((uint64_t)(tb + i) << 32) | TAG) && i < o) s_min[i] = KEY_NONE;  // the pair's root
  }
  __syncthreads();
  for (int it = 0; it < (int)BS + 1; ++it) {
    int more = 0;
    for (uint32_t i = threadIdx.x; i < SPAN; i += BM_T) {
      const uint64_t v = s_min[i];
      if (!in_bucket(v)) continue;
      const uint64_t pv = s_min[(uint32_t)(v >> 32) - tb];
      if ((uint32_t)pv == (uint32_t)TAG) {  // the parent hooked: skip it
        s_min[i] = pv;
        more |= in_bucket(pv) ? 1 : 0;
      }
    }
    if (!__syncthreads_or(more)) break;  // one barrier: every thread sees the same answer
  }
  }  // GHS_BM_COMPRESS
  for (uint32_t i = threadIdx.x; i < SPAN; i += BM_T) {
    const uint64_t v = s_min[i];
    if ((uint32_t)v == (uint32_t)TAG) par[tb + i] = (uint32_t)(v >> 32);
    else if (FULL && tb + i < n) par[tb + i] = tb + i;
  }
}

// FULL: a bucket without candidates still initialises its vertices (see bucket_round)
template <uint32_t BS>
__device__ __forceinline__ void bucket_ident(uint32_t t, uint32_t *__restrict__ par, uint64_t *__restrict__ best,
                                             uint32_t n) {
  const uint32_t tb = t << BS;
  for (uint32_t i = threadIdx.x; i < (1u << BS); i += BM_T) {
    if (tb + i >= n) break;
    best[tb + i] = KEY_NONE;
    par[tb + i] = tb + i;
  }
}

template <uint32_t BS, bool FULL = false>
__global__ __launch_bounds__(BM_T) void k_bmin(const uint4 *__restrict__ rec, const uint32_t *__restrict__ O,
                                               SegView in, uint32_t *__restrict__ par, uint64_t *__restrict__ best,
                                               uint8_t *__restrict__ in_mst,
                                               const unsigned long long *__restrict__ guard_nact,
                                               const unsigned long long *__restrict__ only_if, uint32_t n = 0) {
  constexpr uint32_t SPAN = 1u << BS;
  __shared__ unsigned long long s_min[SPAN];
  __shared__ uint64_t s_pos[BK_G];  // non-empty run i: its first record's position
  __shared__ uint32_t s_pre[BK_G];  // ... and its first index in the bucket's record order
  __shared__ uint32_t s_wsum[BM_T / WAVE];
  if (only_if && !*only_if) return;  // the windowed round ran (k_wmin)
  // a round enqueued past its level's end (the pipelined loop's lookahead) exits before the block
  // scans: one bucket per block, n / 2^BS blocks — the 16384^2 gradient grid's no-op k_bmin took
  // 57 us through them (profiles/r06/final/rounds_grid-gradient.txt)
  if (guard_nact && *guard_nact <= 1) return;
  const uint64_t T = in.prefix[in.nseg];
  const uint64_t R2 = 2 * bk_quota(T);  // record region stride
  const uint32_t t = blockIdx.x;
  uint32_t cnt = 0, st = 0;
  if (threadIdx.x < BK_G) {
    st = O[bk_off_index(t, threadIdx.x, gridDim.x)];
    cnt = O[bk_off_index(t + 1, threadIdx.x, gridDim.x)] - st;
  }
  // records before each run (scan of the counts), then the non-empty runs' slots (scan of their flags)
  uint32_t R, NZ;
  const uint32_t before = block_excl_scan<BM_T>(cnt, s_wsum, &R);
  if (R == 0) {  // block-uniform: no record of this bucket
    if (FULL) bucket_ident<BS>(t, par, best, n);
    return;
  }
  const uint32_t zi = block_excl_scan<BM_T>(cnt ? 1u : 0u, s_wsum, &NZ);
  if (cnt) {
    s_pos[zi] = R2 * threadIdx.x + st;
    s_pre[zi] = before;
  }
  for (uint32_t i = threadIdx.x; i < SPAN; i += BM_T) s_min[i] = KEY_NONE;
  __syncthreads();
  auto locate = [&](uint32_t r) -> uint64_t {  // the non-empty run with s_pre <= r, the last one
    uint32_t lo = 0, hi = NZ - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (s_pre[mid] <= r) lo = mid; else hi = mid - 1;
    }
    return s_pos[lo] + (r - s_pre[lo]);
  };
  constexpr uint32_t STEP = BM_T * BM_ILP;
  auto sweep = [&](auto f) {
    for (uint32_t r0 = threadIdx.x; r0 < R; r0 += STEP) {
      uint32_t a[BM_ILP], b[BM_ILP];
      unsigned long long k[BM_ILP];
#pragma unroll
      for (int j = 0; j < BM_ILP; ++j) {
        const uint32_t r = r0 + j * BM_T;
        const uint64_t p = r < R ? locate(r) : 0;
        const uint4 x = rec[p];
        a[j] = r < R ? x.x : LABEL_NONE;
        b[j] = r < R ? x.y : LABEL_NONE;
        k[j] = r < R ? ((unsigned long long)x.w << 32 | x.z) : KEY_NONE;
      }
#pragma unroll
      for (int j = 0; j < BM_ILP; ++j) f(a[j], b[j], k[j]);
    }
  };
  bucket_round<BS, FULL>(t, s_min, sweep, par, best, in_mst, n);
}

// ------------------------------------------------------------------------------------------
// Windowed round 0 of level 0 on a lattice-like graph. The level-0 edge list is in canonical order
// (a = u ascending) and its labels are the vertices, so bucket t's candidates are the edges with a
// in bucket t and the edges with b in bucket t; when no level-0 edge has its ends more than one
// bucket apart (k_select's span flag), all of them lie in the list's run of buckets t - 1 and t.
// k_wmin reads that window straight from the edge list — no k_bucket records, no region search —
// and runs the bucketed round's LDS core on it. Blocks take buckets in XCD order (workgroup i runs
// on XCD i % 8): consecutive buckets run together on one XCD, so the row they share is read from
// HBM about once. If the span flag is set, k_wstarts / k_wmin exit and the k_bucket / k_bmin
// launches enqueued behind them run the round instead.
// k_wstarts: start[t] = the first virtual index whose edge has a >= t << bs (start[nb] = total):
// a search over the regions' first edges, then inside one region (its padding is at its end).
// ------------------------------------------------------------------------------------------
// k_wfirst (one block): F[r] = the first edge's a of region r, an empty region taking the next
// non-empty one's (suffix minimum; the regions are in canonical order) — level 0 of the gradient
// grid leaves whole runs of regions empty, which a search that skips them one by one crawls over
constexpr uint32_t WF_T = 1024;
__global__ __launch_bounds__(WF_T) void k_wfirst(SegView in, const uint32_t *__restrict__ src, uint32_t *__restrict__ F,
                                                 const unsigned long long *__restrict__ long_flag) {
  __shared__ uint32_t s_w[WF_T / WAVE];
  if (*long_flag) return;
  const uint32_t per = (in.nseg + WF_T - 1) / WF_T, r0 = threadIdx.x * per;
  uint32_t v[16];  // per <= 16: nseg <= SEG_MAX = 16384
  uint32_t run = LABEL_NONE;
#pragma unroll
  for (int j = 15; j >= 0; --j) {  // the thread's regions, last first: suffix minimum
    const uint32_t r = r0 + (uint32_t)j;
    uint32_t x = LABEL_NONE;
    if ((uint32_t)j < per && r < in.nseg && in.prefix[r + 1] > in.prefix[r]) x = src[in.start[r]];
    run = x < run ? x : run;
    v[j] = run;
  }
  // suffix minimum across threads: the minimum over the threads above (wave shuffles + LDS)
  const uint32_t lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  uint32_t incl = v[0];
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const uint32_t o = __shfl_down(incl, d);
    if (lane + d < WAVE) incl = o < incl ? o : incl;
  }
  if (lane == 0) s_w[wid] = incl;
  __syncthreads();
  uint32_t after = __shfl_down(incl, 1);
  if (lane == WAVE - 1) after = LABEL_NONE;
  for (uint32_t w = wid + 1; w < WF_T / WAVE; ++w) after = s_w[w] < after ? s_w[w] : after;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t r = r0 + (uint32_t)j;
    if ((uint32_t)j < per && r < in.nseg) F[r] = v[j] < after ? v[j] : after;
  }
}

// k_wstarts: start[t] = the first virtual index whose edge has a >= t << bs (start[nb] = total):
// the last region whose first edge lies below (F), then a search inside it (its padding is at its end)
__global__ __launch_bounds__(256) void k_wstarts(SegView in, const uint32_t *__restrict__ src, const uint32_t *__restrict__ F,
                                                 uint32_t bs, uint32_t nb, uint64_t *__restrict__ start,
                                                 const unsigned long long *__restrict__ long_flag) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t > nb || *long_flag) return;
  const uint64_t T = in.prefix[in.nseg];
  const uint64_t x = (uint64_t)t << bs;
  if (t == 0 || t == nb || T == 0) {
    start[t] = t == 0 ? 0 : T;
    return;
  }
  uint32_t lo = 0, hi = in.nseg - 1;  // the last region whose first edge has a < x (region 0 if none)
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if ((uint64_t)F[mid] < x) lo = mid; else hi = mid - 1;
  }
  const uint64_t p0 = in.start[lo], cnt = in.prefix[lo + 1] - in.prefix[lo];
  uint64_t l = 0, h = cnt;  // an empty region lo (then F[lo] >= x or lo = 0): l = 0
  while (l < h) {
    const uint64_t mid = (l + h) >> 1;
    if ((uint64_t)src[p0 + mid] < x) l = mid + 1; else h = mid;
  }
  start[t] = in.prefix[lo] + l;  // l == cnt: the next region's first edge (a >= x by F)
}

constexpr uint32_t WM_CHUNK = 32;
#ifndef GHS_WM_GATHER
#define GHS_WM_GATHER 1
#endif
constexpr bool WM_GATHER = GHS_WM_GATHER;  // k_wmin: winners from the canonical ends (bucket_round)
template <uint32_t BS>
__global__ __launch_bounds__(BM_T) void k_wmin(const uint32_t *__restrict__ src, const uint32_t *__restrict__ dst,
                                               const uint64_t *__restrict__ key, SegView in, uint32_t nb,
                                               const uint64_t *__restrict__ start, uint32_t *__restrict__ par,
                                               uint64_t *__restrict__ best, uint8_t *__restrict__ in_mst,
                                               const unsigned long long *__restrict__ long_flag, uint32_t n,
                                               const uint32_t *__restrict__ eu, const uint32_t *__restrict__ ev) {
  constexpr uint32_t SPAN = 1u << BS;
  __shared__ unsigned long long s_min[SPAN];
  __shared__ uint32_t s_seg[2];
  // XCD order: workgroup i runs on XCD i % 8; chunks of WM_CHUNK consecutive buckets go round-robin
  // to the XCDs, so a chunk's buckets (which share rows) run together on one XCD's L2 while a
  // spatially skewed level (the gradient grid's lighter half) still spreads over every XCD
  const uint32_t j = blockIdx.x / 8;
  const uint32_t t = ((j / WM_CHUNK) * 8 + blockIdx.x % 8) * WM_CHUNK + j % WM_CHUNK;
  if (t >= nb || *long_flag) return;
  const uint64_t wlo = start[t ? t - 1 : 0], whi = start[t + 1 < nb ? t + 1 : nb];
  if (whi <= wlo) {  // block-uniform: no edge with an end in this bucket
    bucket_ident<BS>(t, par, best, n);
    return;
  }
  if (threadIdx.x < WAVE) seg_range_wave(in.prefix, in.nseg, wlo, whi, whi, s_seg);
  for (uint32_t i = threadIdx.x; i < SPAN; i += BM_T) s_min[i] = KEY_NONE;
  __syncthreads();
  const uint32_t slo = s_seg[0], shi = s_seg[1];
  auto sweep = [&](auto f) {
    for (uint32_t sg = slo; sg <= shi; ++sg) {  // the window's part of each region it touches
      const uint64_t v0 = wlo > in.prefix[sg] ? wlo : in.prefix[sg];
      const uint64_t v1 = whi < in.prefix[sg + 1] ? whi : in.prefix[sg + 1];
      const uint64_t p0 = in.start[sg] + (v0 - in.prefix[sg]), len = v1 > v0 ? v1 - v0 : 0;
      constexpr uint32_t STEP = BM_T * BM_ILP;
      for (uint64_t r0 = threadIdx.x; r0 < len; r0 += STEP) {
        uint32_t a[BM_ILP], b[BM_ILP];
        unsigned long long k[BM_ILP];
#pragma unroll
        for (int j = 0; j < BM_ILP; ++j) {
          const uint64_t r = r0 + (uint64_t)j * BM_T;
          const uint64_t p = r < len ? p0 + r : p0;
          a[j] = src[p];
          b[j] = dst[p];
          k[j] = key[p];
          if (r >= len) a[j] = b[j] = LABEL_NONE;  // padding entries carry a == LABEL_NONE too
        }
#pragma unroll
        for (int j = 0; j < BM_ILP; ++j) f(a[j], a[j] == LABEL_NONE ? LABEL_NONE : b[j], k[j]);
      }
    }
  };
  bucket_round<BS, true>(t, s_min, sweep, par, best, in_mst, n, eu, ev);
}

// The hot fragments' CONNECT in a bucketed level-first round (one thread each): a fragment's
// minimum (reduced by k_bucket) is edge eid; the level's labels are resolved roots, so the other
// end's label is one read. A mutual pair stays a 2-cycle for the jump, as in k_bmin.
__global__ void k_hot_hook(const uint32_t *__restrict__ hot, const uint64_t *__restrict__ best, const Ends E,
                           const uint32_t *__restrict__ lab, uint32_t *__restrict__ par, uint8_t *__restrict__ in_mst,
                           unsigned long long *__restrict__ err) {
  if (threadIdx.x >= hot[0]) return;
  const uint32_t g = hot[1 + threadIdx.x];
  const uint64_t k = best[g];
  if (k == KEY_NONE) return;
  const uint32_t eid = (uint32_t)k;
  const uint32_t la = lab[end_u(E, eid)], lb = lab[E.v[eid]];
  if (la != g && lb != g) atomicOr(err, 2ull);
  par[g] = la == g ? lb : la;
  in_mst[eid] = 1;
}

// ------------------------------------------------------------------------------------------
// Dense levels (several ranks). Once a level's active list A (nact0 fragment roots, identical on
// every rank) is known, the level runs in a dense label space 0..nact0-1: a root's dense label is
// its rank among the level's flags (DenseRank: popc over the flag words + word / chunk prefixes),
// the rank's level edges are relabelled through it, and best / lab / par become nact0-sized arrays.
// The level-opening round's all-reduce slots are then best itself (sequential pack / unpack, no
// gathers and scatters over the vertex arrays through A), the jump runs over the dense identity
// list, and the whole level's state stays in nact0 * 16 B. At the level's end every fragment's
// root is mapped back to vertex labels (vlab[A[i]] = A[root(i)]). SURVEY.md §7(d) "dense relabel
// of live components" — the per-rank volume the vertex-indexed multi-rank rounds paid.
// ------------------------------------------------------------------------------------------
__global__ void k_dense_open(const uint32_t *__restrict__ act, const unsigned long long *__restrict__ d_nact,
                             uint32_t *__restrict__ vtx, uint32_t *__restrict__ dlab,
                             uint32_t *__restrict__ dpar, uint64_t *__restrict__ dbest,
                             unsigned long long *__restrict__ dense_count) {
  const uint64_t nact = *d_nact;
  const uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t0 == 0) *dense_count = nact;
  for (uint64_t i = t0; i < nact; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = act[i];
    vtx[i] = c;
    dlab[i] = (uint32_t)i;
    dpar[i] = (uint32_t)i;
    dbest[i] = KEY_NONE;
  }
}

// the rank's level edges (a, b: vertex labels of active roots) -> dense labels, in place; the
// regions' 4-entry tiles as in k_minedge (one region lookup per block range, 16-B accesses)
__device__ __forceinline__ uint32_t nz_bits16(uint4 f);  // bit k = byte k of the 16 is nonzero (below)

// the rank tables from the level's active flags (n bytes): one thread per 64-vertex word, a block
// (256 words) scans its counts; then one block scans the chunk totals
__global__ __launch_bounds__(BLOCK) void k_rank_words(const uint8_t *__restrict__ flags, uint64_t nf,
                                                      uint64_t *__restrict__ bits, uint32_t *__restrict__ wpre,
                                                      uint32_t *__restrict__ csum, bool from_words) {
  __shared__ uint32_t s_wcnt[BLOCK / WAVE];
  const uint64_t words = (nf + 63) / 64;
  const uint64_t wd = blockIdx.x * (uint64_t)BLOCK + threadIdx.x;
  uint64_t b = 0;
  if (from_words) {  // the merged words of the bitmap exchange are already in bits (k_merge_flag_words)
    if (wd < words) b = bits[wd];
  } else if (wd < words) {
    const uint64_t i0 = wd * 64;
    if (i0 + 64 <= nf) {
      const uint4 *f = reinterpret_cast<const uint4 *>(flags + i0);
#pragma unroll
      for (int q = 0; q < 4; ++q) b |= (uint64_t)nz_bits16(f[q]) << (16 * q);
    } else {
      for (uint64_t i = i0; i < nf; ++i) b |= (uint64_t)(flags[i] != 0) << (i - i0);
    }
  }
  uint32_t total;
  const uint32_t ex = block_offsets((uint32_t)__popcll(b), s_wcnt, &total);
  if (wd < words) {
    if (!from_words) bits[wd] = b;
    wpre[wd] = ex;
  }
  if (threadIdx.x == 0) csum[blockIdx.x] = total;
}

// merged level-open flags as words (several ranks, dense levels): the OR of the gathered
// bitmaps straight into the rank tables' word array (flags below n; bit n, the error byte, to its
// byte) — no flag bytes written, no select over n bytes
__global__ void k_merge_flag_words(const uint64_t *__restrict__ all, uint32_t nranks, uint64_t words, uint64_t n,
                                   uint64_t *__restrict__ out, uint8_t *__restrict__ err_byte) {
  const uint64_t nw = (n + 63) / 64;
  for (uint64_t wd = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; wd < words; wd += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t b = 0;
    for (uint32_t r = 0; r < nranks; ++r) b |= all[(uint64_t)r * words + wd];
    if (wd == n / 64) *err_byte = ((b >> (n % 64)) & 1u) ? 2 : 0;
    if (wd < nw) out[wd] = (wd == n / 64) ? (b & ((1ull << (n % 64)) - 1)) : b;
  }
}

// the level's fragments from the rank tables: vtx[rank(x)] = x for every set flag x (a thread per
// word), then the dense identity state
__global__ void k_dense_open_words(DenseRank dr, uint64_t words, uint32_t *__restrict__ vtx) {
  for (uint64_t wd = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; wd < words; wd += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t b = dr.bits[wd];
    uint32_t r = dr.cpre[wd >> 8] + dr.wpre[wd];
    while (b) {
      const int j = __ffsll((unsigned long long)b) - 1;
      vtx[r++] = (uint32_t)(wd * 64 + j);
      b &= b - 1;
    }
  }
}

__global__ void k_dense_init(const unsigned long long *__restrict__ d_nact, uint32_t *__restrict__ dlab,
                             uint32_t *__restrict__ dpar, uint64_t *__restrict__ dbest,
                             unsigned long long *__restrict__ dense_count) {
  const uint64_t nact = *d_nact;
  const uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t0 == 0) *dense_count = nact;
  for (uint64_t i = t0; i < nact; i += (uint64_t)gridDim.x * blockDim.x) {
    dlab[i] = (uint32_t)i;
    dpar[i] = (uint32_t)i;
    dbest[i] = KEY_NONE;
  }
}

__global__ __launch_bounds__(1024) void k_rank_chunks(uint32_t *__restrict__ csum, uint32_t nchunks,
                                                      unsigned long long *__restrict__ total_out) {
  __shared__ uint32_t s_part[1024];
  const uint32_t per = (nchunks + 1023) / 1024;
  const uint32_t b = threadIdx.x * per;
  uint32_t sum = 0;
  for (uint32_t i = 0; i < per && b + i < nchunks; ++i) sum += csum[b + i];
  s_part[threadIdx.x] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const uint32_t o = threadIdx.x >= (unsigned)d ? s_part[threadIdx.x - d] : 0;
    __syncthreads();
    s_part[threadIdx.x] += o;
    __syncthreads();
  }
  uint32_t run = s_part[threadIdx.x] - sum;  // exclusive, in place
  for (uint32_t i = 0; i < per && b + i < nchunks; ++i) {
    const uint32_t c = csum[b + i];
    csum[b + i] = run;
    run += c;
  }
  if (total_out && threadIdx.x == 1023) *total_out = s_part[1023];
}

__global__ __launch_bounds__(BLOCK) void k_relabel_dense(uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                         SegView in, DenseRank dr) {
  __shared__ uint32_t s_seg[2];
  const uint64_t T = in.prefix[in.nseg];
  const uint64_t Q = ((T + gridDim.x - 1) / gridDim.x + 3) & ~3ull;
  const uint64_t vb = Q * blockIdx.x;
  const uint64_t ve = (vb + Q < T) ? vb + Q : T;
  if (threadIdx.x < WAVE) seg_range_wave(in.prefix, in.nseg, vb, ve, T, s_seg);
  __syncthreads();
  const uint32_t slo = s_seg[0], shi = s_seg[1];
  for (uint64_t v = vb + (uint64_t)threadIdx.x * 4; v < ve; v += ARCS_PER_BLOCK) {
    const uint64_t i0 = tile_phys(in, slo, shi, v, ve);
    uint4 a = *reinterpret_cast<const uint4 *>(src + i0);
    uint4 b = *reinterpret_cast<const uint4 *>(dst + i0);
    uint32_t A[4] = {a.x, a.y, a.z, a.w}, B[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // region padding (a == LABEL_NONE) stays dead
      const bool live = A[j] != LABEL_NONE;
      const uint32_t pa = dense_rank(dr, live ? A[j] : 0u), pb = dense_rank(dr, live ? B[j] : 0u);
      A[j] = live ? pa : LABEL_NONE;
      B[j] = live ? pb : B[j];
    }
    *reinterpret_cast<uint4 *>(src + i0) = make_uint4(A[0], A[1], A[2], A[3]);
    *reinterpret_cast<uint4 *>(dst + i0) = make_uint4(B[0], B[1], B[2], B[3]);
  }
}

// level end: every dense fragment's root back to vertex labels
// write = false: the chains' check alone (the plan's last level, whose vertex labels nothing reads,
// under GHS_OPT_CHECK_TOTALS — ADVICE r05)
__global__ void k_dense_close(const uint32_t *__restrict__ vtx, const unsigned long long *__restrict__ d_nact,
                              const uint32_t *__restrict__ dlab, uint32_t *__restrict__ vlab,
                              unsigned long long *__restrict__ err, bool write) {
  const uint64_t nact = *d_nact;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nact; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = find_lab(dlab, (uint32_t)i, err);
    if (write) vlab[vtx[i]] = vtx[r];
  }
}

// Multi-rank error agreement: a rank's own error bits -> the error byte flags[n] of the level's
// exchanged flag buffer (2: non-canonical input, 1: another invariant), and after the caller's
// MAX all-reduce the combined byte -> this rank's error bits, so every rank fails in the same
// call instead of leaving the others blocked in the next collective.
__global__ void k_err_to_flag(const unsigned long long *__restrict__ err, uint8_t *__restrict__ flag) {
  const unsigned long long e = *err;
  *flag = (e & 8ull) ? 2 : (e ? 1 : 0);
}

__global__ void k_flag_to_err(const uint8_t *__restrict__ flag, unsigned long long *__restrict__ err) {
  const uint8_t f = *flag;
  if (f) atomicOr(err, f >= 2 ? 8ull : 32ull);
}

// Level-open flag exchange as bitmaps (several ranks): the n + 1 flag bytes (fragments + error
// byte) packed to bits — each rank contributes (n + 1) / 8 bytes to an all-gather instead of n + 1
// bytes to a MAX all-reduce (half the bytes on the wire per rank, one eighth in the buffer) — and
// the gathered bitmaps OR-ed back into the flag bytes. One wave per 64-bit word.
__device__ __forceinline__ uint32_t nz_bits16(uint4 f) {  // bit k = byte k of the 16 is nonzero
  const uint32_t w[4] = {f.x, f.y, f.z, f.w};
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) r |= (((w[k >> 2] >> (8 * (k & 3))) & 0xffu) ? 1u : 0u) << k;
  return r;
}

// one thread per 64-bit word: 64 flag bytes in four 16-B loads (a wave reads 4 KB contiguous)
__global__ void k_pack_flag_bits(const uint8_t *__restrict__ flags, uint64_t nf, uint64_t *__restrict__ bits) {
  const uint64_t words = (nf + 63) / 64;
  for (uint64_t wd = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; wd < words; wd += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i0 = wd * 64;
    uint64_t b = 0;
    if (i0 + 64 <= nf) {
      const uint4 *f = reinterpret_cast<const uint4 *>(flags + i0);
#pragma unroll
      for (int q = 0; q < 4; ++q) b |= (uint64_t)nz_bits16(f[q]) << (16 * q);
    } else {
      for (uint64_t i = i0; i < nf; ++i) b |= (uint64_t)(flags[i] != 0) << (i - i0);
    }
    bits[wd] = b;
  }
}

// one thread per word: OR of the ranks' words, 64 flag bytes written as four 16-B stores
__global__ void k_merge_flag_bits(const uint64_t *__restrict__ all, uint32_t nranks, uint64_t words, uint64_t nf,
                                  uint8_t *__restrict__ flags, uint8_t *__restrict__ err_byte) {
  for (uint64_t wd = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; wd < words; wd += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t b = 0;
    for (uint32_t r = 0; r < nranks; ++r) b |= all[(uint64_t)r * words + wd];
    const uint64_t i0 = wd * 64;
    if (i0 + 64 < nf) {  // wholly below the error byte
      uint4 *f = reinterpret_cast<uint4 *>(flags + i0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t bb = (uint32_t)(b >> (16 * q + 4 * k)) & 15u;  // 4 flags -> 4 bytes
          w[k] = (bb & 1u) | ((bb & 2u) << 7) | ((bb & 4u) << 14) | ((bb & 8u) << 21);
        }
        f[q] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    } else {
      for (uint64_t i = i0; i < nf; ++i) {
        const uint8_t x = (uint8_t)((b >> (i - i0)) & 1u);
        if (i + 1 < nf) flags[i] = x;
        else *err_byte = x ? 2 : 0;  // bit n: some rank saw bad input (or failed)
      }
    }
  }
}

__global__ void k_iota(uint32_t *__restrict__ a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}

// dense all-reduce staging: int64 slot = key ^ 2^63 preserves unsigned order under signed MIN
// `bound` slots (the host's count, >= the device's): a pipelined multi-rank round all-reduces a
// bound on its active fragments, the slots past the device count hold "no edge" on every rank
__global__ void k_pack_best(const uint32_t *__restrict__ act, const unsigned long long *__restrict__ d_nact,
                            const uint64_t *__restrict__ best, int64_t *__restrict__ dense, uint64_t bound) {
  const uint64_t nact = *d_nact;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < bound; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k = KEY_NONE;
    if (i < nact) k = best[act ? act[i] : (uint32_t)i];
    dense[i] = (int64_t)(k ^ 0x8000000000000000ull);
  }
}

__global__ void k_unpack_best(const uint32_t *__restrict__ act, const unsigned long long *__restrict__ d_nact,
                              uint64_t *__restrict__ best, const int64_t *__restrict__ dense) {
  const uint64_t nact = *d_nact;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nact; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = act ? act[i] : (uint32_t)i;
    best[c] = (uint64_t)dense[i] ^ 0x8000000000000000ull;
  }
}

// Result of a round, written into coherent pinned host memory by the round's last kernel; the
// host polls seq (written last).
constexpr int C_ERR_IDX = 4;  // == C_ERR (counter layout below)
constexpr int C_LONG_IDX = 10;  // == C_LONG

// A report carries a checksum of (seq, every field): the host accepts a slot only when the fields
// it read hash to the checksum it read. Nothing in the HIP memory model orders the field stores
// before the seq store for a host reader short of a system-scope release (whose L2 write-back held
// the next round's first kernel ~6 us, every round); round 4 saw a new seq beside a stale weight
// when the slot straddled two 64-B lines. With the checksum, a stale or torn field (the slot's
// previous report, or a store still in flight) fails the check and the host polls again, whatever
// order the stores land in.
struct alignas(64) RoundSlot {
  unsigned long long live_out, nact_out, edges;
  unsigned long long err;      // error bits (low word); bit 32: counter C_LONG, a level-0 edge spans > 1
                               // bucket (the windowed round fell back) — not an error
  unsigned long long seq;
  unsigned long long nact_in;  // active fragments this round started from (a level's first round: the level's)
  unsigned long long pending;  // pending edges after the level's pass (counter C_PENDING)
  unsigned long long weight;   // MSF weight so far (counter C_WEIGHT)
  unsigned long long chk;      // slot_checksum(seq, the fields above)
};
constexpr unsigned long long SLOT_SPAN = 1ull << 32;
__host__ __device__ __forceinline__ unsigned long long slot_err(unsigned long long e) { return e & 0xffffffffull; }

__host__ __device__ __forceinline__ unsigned long long slot_mix(unsigned long long h, unsigned long long x) {
  h ^= x + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  h ^= h >> 30;  // splitmix64 finalizer
  h *= 0xbf58476d1ce4e5b9ull;
  h ^= h >> 27;
  h *= 0x94d049bb133111ebull;
  h ^= h >> 31;
  return h;
}

__host__ __device__ __forceinline__ unsigned long long slot_checksum(unsigned long long seq, unsigned long long live_out,
                                                                     unsigned long long nact_out, unsigned long long edges,
                                                                     unsigned long long err, unsigned long long nact_in,
                                                                     unsigned long long pending, unsigned long long weight) {
  unsigned long long h = slot_mix(0x5107ull, seq);
  h = slot_mix(h, live_out);
  h = slot_mix(h, nact_out);
  h = slot_mix(h, edges);
  h = slot_mix(h, err);
  h = slot_mix(h, nact_in);
  h = slot_mix(h, pending);
  return slot_mix(h, weight);
}

__device__ __forceinline__ void write_report(RoundSlot *slot, unsigned long long seq, const unsigned long long *cnt,
                                             unsigned long long nact_out, unsigned long long nact_in) {
  // device-scope loads: the error bits may come from other workgroups of the writing launch
  const unsigned long long live = __hip_atomic_load(cnt + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long edges = __hip_atomic_load(cnt + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long err = __hip_atomic_load(cnt + C_ERR_IDX, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long pending = __hip_atomic_load(cnt + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long weight = __hip_atomic_load(cnt + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long span = __hip_atomic_load(cnt + C_LONG_IDX, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long e = slot_err(err) | (span ? SLOT_SPAN : 0ull);  // error bits + the span flag
  // system-scope stores to the coherent (uncached) host slot; the checksum makes the host's read
  // independent of the order in which they land
  __hip_atomic_store(&slot->live_out, live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&slot->nact_out, nact_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&slot->edges, edges, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&slot->err, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&slot->nact_in, nact_in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&slot->pending, pending, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&slot->weight, weight, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&slot->chk, slot_checksum(seq, live, nact_out, edges, e, nact_in, pending, weight),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(&slot->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_round_report(RoundSlot *slot, unsigned long long seq, const unsigned long long *cnt,
                               const unsigned long long *nact_out, const unsigned long long *nact_in) {
  write_report(slot, seq, cnt, *nact_out, *nact_in);
}

// ------------------------------------------------------------------------------------------
// Order-preserving select in ONE launch: out[k] = (act ? act[i] : i) for the k-th i < *d_count
// with flags[i] != 0; every rank of a multi-GPU run produces the same list in the same order.
// (Opening a level: the flagged vertices. A round: the fragments k_jump kept.)
//  - at most LB_MAX_TILES (1024) workgroups of 256 threads: <= 4 per CU, always co-resident
//    (cdna_hip_programming.md §1), so waiting on another tile of the launch cannot deadlock
//    whatever the dispatch order; a tile covers LB_GROUP * G items (G from the host).
//  - pass 1 counts the tile's flagged items, the tile publishes its count as one 8-byte granule
//    {tag = epoch, count} by an agent-scope atomic store (the data is the flag: G16 R2), then
//    sums the counts of all lower tiles (one wave, <= 16 agent-scope granule loads per lane,
//    re-polled until every tag matches; a granule of another launch carries another tag). No
//    ticket counter: one device-scope counter costs ~12 ns per arrival (MI355X_MICROARCH.md,
//    fanin) — 50 us for 4096 tiles, measured.
//  - pass 2 takes the keep bits again (from LDS when the tile has at most LB_KEEP_G groups, n <=
//    2^28 items: pass 1 kept them; else from the flags) and writes the tile's items at its prefix;
//    each wave owns a contiguous quarter of the tile and places its items by wave scans (the first
//    version's block-wide scan per 4096-item group cost two barriers each: 128 per tile on the
//    16384^2 grid's 268M-vertex selects).
//  - the last tile's prefix + count is the total: that block writes *d_total and, for a round,
//    the round report (live, active, edges, err, seq) to the pinned slot.
//  - every spin is bounded: a timeout sets err bit 16 and the block writes nothing.
// Replaces count + scan + write (3 launches). Fusing k_jump into pass 1 as well measured slower
// (6.88 vs 6.72 ms per step, R-MAT s24): 1024 co-resident tiles leave each lane 8 walks in lock
// step, where k_jump has every walk of the round in flight.
// ------------------------------------------------------------------------------------------
typedef __attribute__((address_space(1))) unsigned long long gu64;
constexpr uint32_t LB_MAX_TILES = 1024;
constexpr uint32_t LB_GROUP = BLOCK * 16;     // items per group: 16 keep bytes per lane (one 16-B load)
constexpr uint32_t LB_MAX_SPINS = 1u << 16;   // x (load latency + s_sleep) ~ 0.1 s, never reached in a sane run
constexpr uint32_t LB_KEEP_G = 64;            // tiles of up to 64 groups keep pass 1's bits in LDS (32 KiB)

__device__ __forceinline__ unsigned long long lb_granule(uint32_t tag, uint32_t v) {
  return ((unsigned long long)tag << 32) | v;
}

// sum of the counts of tiles [0, t); ONE wave (all 64 lanes); false on timeout
__device__ bool lb_prefix(unsigned long long *state, uint32_t t, uint32_t tag, uint64_t *out) {
  constexpr int R = LB_MAX_TILES / WAVE;
  const int lane = threadIdx.x & (WAVE - 1);
  gu64 *st = (gu64 *)state;
  uint32_t spins = 0;
  for (;;) {
    uint64_t sum = 0;
    bool ready = true;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t idx = (uint32_t)lane + (uint32_t)(WAVE * r);
      if (idx < t) {
        const unsigned long long g = __hip_atomic_load(st + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ready &= (uint32_t)(g >> 32) == tag;
        sum += (uint32_t)g;
      }
    }
    if (__all(ready)) {
#pragma unroll
      for (int d = WAVE / 2; d > 0; d >>= 1) sum += __shfl_xor(sum, d);
      *out = sum;
      return true;
    }
    if (++spins > LB_MAX_SPINS) return false;
    __builtin_amdgcn_s_sleep(2);
  }
}

__device__ __forceinline__ uint32_t keep_bits16(const uint8_t *__restrict__ flags, uint64_t i0, uint64_t count) {
  uint32_t bits = 0;
  if (i0 + 16 <= count) {
    const uint4 f = *reinterpret_cast<const uint4 *>(flags + i0);
    const uint32_t w[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) bits |= (((w[k >> 2] >> (8 * (k & 3))) & 0xffu) ? 1u : 0u) << k;
  } else {
    for (uint32_t k = 0; k < 16; ++k)
      if (i0 + k < count && flags[i0 + k]) bits |= 1u << k;
  }
  return bits;
}

__global__ __launch_bounds__(BLOCK) void k_select_lb(const uint8_t *__restrict__ flags, const uint32_t *__restrict__ act,
                                                     const unsigned long long *__restrict__ d_count, uint32_t groups,
                                                     uint32_t *__restrict__ out, unsigned long long *__restrict__ d_total,
                                                     unsigned long long *state, uint32_t tag, RoundSlot *slot,
                                                     unsigned long long seq, unsigned long long *cnt,
                                                     unsigned long long *shards) {
  __shared__ uint32_t s_wcnt[BLOCK / WAVE];
  __shared__ uint64_t s_excl;
  __shared__ int s_ok;
  __shared__ uint16_t s_keep[LB_KEEP_G * BLOCK];  // pass 1's keep bits (G <= LB_KEEP_G): no re-read
  const uint32_t t = blockIdx.x;
  const uint64_t count = *d_count;
  // the tile [tb, tb + G * LB_GROUP) as four contiguous wave ranges of G chunks of 1024 items (16
  // keep bytes per lane per chunk): each wave finds its items' positions with wave scans only (no
  // block barrier per chunk), in item order
  const uint32_t lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  constexpr uint32_t CHUNK = WAVE * 16;
  const uint64_t tb = (uint64_t)t * groups * LB_GROUP;
  const uint64_t wb = tb + (uint64_t)wid * groups * CHUNK;  // the wave's first item
  const uint32_t wl = wb >= count ? 0u : (uint32_t)umin64((uint64_t)groups, (count - wb + CHUNK - 1) / CHUNK);
  const bool keep_lds = groups <= LB_KEEP_G;
  uint32_t mine = 0;  // kept items of this lane (pass 1)
  for (uint32_t c = 0; c < wl; ++c) {
    const uint32_t bits = keep_bits16(flags, wb + (uint64_t)c * CHUNK + (uint64_t)lane * 16, count);
    if (keep_lds) s_keep[(wid * groups + c) * WAVE + lane] = (uint16_t)bits;
    mine += __popc(bits);
  }
#pragma unroll
  for (int d = WAVE / 2; d > 0; d >>= 1) mine += __shfl_xor(mine, d);
  if (lane == 0) s_wcnt[wid] = mine;
  __syncthreads();
  uint32_t tot = 0, wbefore = 0;
#pragma unroll
  for (uint32_t w = 0; w < BLOCK / WAVE; ++w) {
    wbefore += w < wid ? s_wcnt[w] : 0u;
    tot += s_wcnt[w];
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store((gu64 *)state + t, lb_granule(tag, tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_excl = 0;
    s_ok = 1;
  }
  if (t > 0 && threadIdx.x < WAVE) {
    uint64_t ex = 0;
    const bool ok = lb_prefix(state, t, tag, &ex);
    if (threadIdx.x == 0) {
      s_excl = ex;
      s_ok = ok ? 1 : 0;
      if (!ok) atomicOr(cnt + C_ERR_IDX, 16ull);
    }
  }
  __syncthreads();
  if (!s_ok) return;
  // pass 2: the keep bits again (LDS, or the flags) -> out, in item order
  uint64_t run = s_excl + wbefore;
  for (uint32_t c = 0; c < wl; ++c) {
    const uint64_t i0 = wb + (uint64_t)c * CHUNK + (uint64_t)lane * 16;
    uint32_t bits = keep_lds ? (uint32_t)s_keep[(wid * groups + c) * WAVE + lane] : keep_bits16(flags, i0, count);
    const uint32_t k0 = (uint32_t)__popc(bits);
    uint32_t incl = k0;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d);
      if (lane >= (uint32_t)d) incl += y;
    }
    uint64_t pos = run + (incl - k0);
    while (bits) {
      const int k = __ffs(bits) - 1;
      bits &= bits - 1;
      out[pos++] = act ? act[i0 + k] : (uint32_t)(i0 + k);
    }
    run += __shfl(incl, WAVE - 1);
  }
  if (t == gridDim.x - 1 && threadIdx.x < WAVE) {
    // a counting jump ran before (bucketed rounds): its sharded hook totals join the counters
    // (read and cleared by device atomics: the shards live at the memory side like the adds)
    if (shards) {
      unsigned long long fw = atomicExch(shards + SHARD_STRIDE * threadIdx.x, 0ull);
      unsigned long long fc = atomicExch(shards + SHARD_STRIDE * threadIdx.x + 1, 0ull);
#pragma unroll
      for (int d = WAVE / 2; d > 0; d >>= 1) {
        fw += __shfl_xor(fw, d);
        fc += __shfl_xor(fc, d);
      }
      if (threadIdx.x == 0 && fc) {
        (void)atomicAdd(cnt + 2, fw);  // C_WEIGHT, C_EDGES (returning: complete before the report)
        (void)atomicAdd(cnt + 3, fc);
      }
    }
    if (threadIdx.x == 0) {
      *d_total = s_excl + tot;
      if (slot) write_report(slot, seq, cnt, s_excl + tot, count);
    }
  }
}

// ------------------------------------------------------------------------------------------
// The LDS tail of a level (one rank). Once a level's active fragments fit a workgroup's LDS
// (<= TAIL_MAX), its remaining rounds — the reference's last TEST / REPORT / CHANGEROOT /
// INITIATE exchanges of a level, ghs_implementation.py:235-387 — run without any global atomic and
// without n-sized arrays: the fragments get dense ids 0..F0-1 (their order in the active list),
// every edge is relabelled ONCE to the dense pair of its fragments, and each later round keeps
// every root's minimum in LDS per block.
//   k_tail_map    dmap[act[i]] = i; the tail's control block, R = identity, the root list
//   k_tail_open   (round 0 of the tail) every live edge: a, b -> dmap (its dense fragments);
//                 intra-fragment edges dropped, the rest compacted in order to the block's region of
//                 the tail buffer as one 12-byte record (da | db << 16, key); each end's candidate
//                 min'ed into the block's LDS minima; the block's row: each minimum's key and other end
//   k_tail_hook   one slot per active root: the minimum over the blocks' rows and its other end
//                 (the CONNECT target), the MSF flag of the edge
//   k_tail_round  every block applies the last round's hooks in LDS — over the ROOTS only: mutual
//                 pairs keep the smaller root, pointer jumping among the roots, then every dense id's
//                 root through one lookup (R[d] = P[R[d]]), the next root list — identically in every
//                 block (no grid barrier: the launch boundaries order open -> hook -> round -> hook,
//                 so ranks sharing a device cannot deadlock it), then streams its records (a
//                 candidate only where R[da] != R[db]) into its LDS minima and row. A round that
//                 starts with <= 1 active root finishes the level instead: lab of every fragment of
//                 the level = its final root, the round report.
// The LDS minima carry (w << 32 | the record's index in the block's region) instead of the key:
// a block's region holds its records in canonical (eid) order — a level's live edges keep the
// canonical order within and across their regions (k_select / k_filter / k_level_pass emit it,
// every compaction keeps it) and the open compacts in order — so within a block that order IS the
// (w, eid) order, and each minimum's record is one load away: its true key for the row and its
// other end. (Round 4's hook found the other end through the canonical list and the label chains,
// and its prologue jumped pointers over all F0 dense ids.)
// Per round: one stream of the 12-byte records + two launch boundaries, instead of the round
// kernels' relabel gathers, LDS-cache misses to best[], hook, jump and select over n-sized arrays.
// ------------------------------------------------------------------------------------------
constexpr uint32_t TAIL_MAX = 12288;        // dense fragments: LDS minima 96 KiB + 2 x 24 KiB of u16 tables
constexpr uint32_t TAIL_T = 1024;           // threads of the streaming tail kernels (16 waves, 1 block per CU)
constexpr uint32_t TAIL_G = 256;            // their blocks = rows of `partial`
constexpr uint32_t TAIL_ROUNDS_MAX = 32;    // a tail round at least halves the roots: <= 14 rounds
constexpr uint32_t TAIL_HS = 16;            // k_tail_hook: slots per 256-thread block (16 row groups)
constexpr uint16_t TAIL_NONE = 0xffffu;     // a row's other end where the block has no candidate
static_assert(TAIL_MAX <= 32768, "dense ids are packed as 16-bit pairs");

struct TailCtl {
  uint32_t F0;        // dense fragments (the active list at the tail's start)
  uint32_t done;      // the level is complete (lab written)
  uint32_t rounds;    // tail rounds streamed (set when done)
  uint32_t err;
  uint64_t Q;         // each block's region stride in the tail buffer
  uint64_t nroots[TAIL_ROUNDS_MAX + 1];  // active roots of round r (its list: droot[r & 1])
  uint64_t live[TAIL_ROUNDS_MAX];        // live (inter-fragment) edges round r scanned
  uint64_t edges[TAIL_ROUNDS_MAX];       // MSF edges (C_EDGES) once round r's hooks are counted
};

struct TailBufs {
  TailCtl *ctl;
  uint32_t *dmap;      // root label -> dense id (n entries; only the tail's roots are meaningful)
  uint64_t *partial;   // TAIL_G rows x TAIL_MAX block minima (root-list order)
  uint16_t *poth;      // ... and each minimum's other end (dense root id at the time of the stream)
  uint32_t *R[2];      // dense id -> dense root during round r: R[r & 1]
  uint32_t *droot[2];  // round r's active roots (ascending dense ids): droot[r & 1]
  uint32_t *ghook;     // per dense root: CONNECT target (dense root) of its minimum edge
  uint64_t *gkey;      // per dense root: its minimum key (KEY_NONE: no outgoing edge)
  uint64_t *gloc;      // several ranks: this rank's own minimum (gkey is then MIN-all-reduced)
  uint32_t *blive;     // per block: live edges of the round it streamed
  uint32_t *bcnt;      // per block: records in its region of the tail buffer
  uint32_t *rec;       // the tail buffer: da | db << 16
  uint64_t *rkey;      //   ... and the key
};

// A tail in progress (run_tail's batches, or the stepwise ghs_solver_tail_* calls of several ranks)
struct TailRun {
  TailBufs tb{};
  const uint32_t *act0 = nullptr;
  uint32_t F0 = 0, round0 = 0, lr0 = 0, r = 1;  // r: the next tail round to stream
  unsigned hook_g = 1;
  bool multi = false;
};

__global__ void k_tail_map(const uint32_t *__restrict__ act, const unsigned long long *__restrict__ d_nact, TailBufs tb) {
  const uint32_t F = (uint32_t)*d_nact;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < F; i += gridDim.x * blockDim.x) {
    tb.dmap[act[i]] = i;
    tb.R[0][i] = i;
    tb.droot[0][i] = i;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    TailCtl *c = tb.ctl;
    c->F0 = F;
    c->done = 0;
    c->rounds = 0;
    c->err = 0;
    c->nroots[0] = F;
  }
}

// The labels the live edges carry (the previous round's active list, or every vertex after a
// level's identity round) -> the dense id of their fragment now: dmap[x] = dmap[lab[x]] (one hop:
// lab of those labels is current; a root's own entry is k_tail_map's and is not rewritten here),
// so k_tail_open relabels an end with ONE gather.
__global__ void k_tail_labels(const uint32_t *__restrict__ prev, const unsigned long long *__restrict__ d_nprev,
                              const uint32_t *__restrict__ lab, TailBufs tb) {
  const uint64_t np = *d_nprev;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < np; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t x = prev ? prev[i] : (uint32_t)i;
    const uint32_t l = lab[x];
    if (l != x) tb.dmap[x] = tb.dmap[l];
  }
}

__device__ __forceinline__ void lds_min_u64(unsigned long long *s, uint32_t i, uint64_t k) {
  if (k < s[i]) atomicMin(&s[i], (unsigned long long)k);  // a plain read first: slots only decrease
}

// a wave's survivors staged in LDS for coalesced stores (12-byte records)
struct TailStage {
  uint32_t p[WAVE * 4];
  uint64_t k[WAVE * 4];
};

// a block-local candidate: the key's weight with the record's index in the block's region (the
// region is in eid order, so this orders the block's candidates exactly as (w, eid))
__device__ __forceinline__ uint64_t tail_local(uint64_t key, uint32_t idx) { return (key & ~0xffffffffull) | idx; }

// The block's row (root-list order: root i of the round = droots[i]): each root's minimum
// record (one load: its index is in the LDS minimum) gives the true key and the other end's dense
// root (through R: rmap == nullptr is the identity, the open). Every record load in flight first.
__device__ __forceinline__ void tail_row_out(const TailBufs tb, const unsigned long long *s_best, const uint16_t *droots,
                                             uint32_t nroot, const uint32_t *__restrict__ pr, const uint64_t *__restrict__ pk,
                                             const uint16_t *rmap) {
  constexpr uint32_t PER = TAIL_MAX / TAIL_T;
  uint64_t *row = tb.partial + (uint64_t)blockIdx.x * TAIL_MAX;
  uint16_t *orow = tb.poth + (uint64_t)blockIdx.x * TAIL_MAX;
  uint32_t p[PER], d[PER];
  uint64_t k[PER];
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t i = threadIdx.x + q * TAIL_T;
    d[q] = i < nroot ? (droots ? droots[i] : i) : 0u;
    const uint64_t v = i < nroot ? s_best[d[q]] : KEY_NONE;
    const bool has = v != KEY_NONE;
    p[q] = has ? pr[(uint32_t)v] : 0u;
    k[q] = has ? pk[(uint32_t)v] : KEY_NONE;
  }
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t i = threadIdx.x + q * TAIL_T;
    if (i >= nroot) break;
    uint16_t o = TAIL_NONE;
    if (k[q] != KEY_NONE) {
      const uint32_t da = p[q] & 0xffffu, db = p[q] >> 16;
      const uint32_t ra = rmap ? rmap[da] : da, rb = rmap ? rmap[db] : db;
      o = (uint16_t)(ra == d[q] ? rb : ra);
    }
    row[i] = k[q];
    orow[i] = o;
  }
}

// check (GHS_OPT_CHECK_TOTALS): verify the invariant the (w, index) minima rest on — the
// block's region holds its records in strictly increasing eid order — after writing it
__global__ __launch_bounds__(TAIL_T) void k_tail_open(const uint32_t *__restrict__ src, const uint32_t *__restrict__ dst,
                                                      const uint64_t *__restrict__ key, SegView in, TailBufs tb,
                                                      bool check) {
  __shared__ unsigned long long s_best[TAIL_MAX];
  __shared__ TailStage s_stage[TAIL_T / WAVE];
  __shared__ uint32_t s_wcnt[TAIL_T / WAVE];
  __shared__ uint32_t s_seg[2];
  __shared__ uint32_t s_live;
  const uint32_t F = tb.ctl->F0;
  for (uint32_t i = threadIdx.x; i < F; i += TAIL_T) s_best[i] = KEY_NONE;
  const uint64_t T = in.prefix[in.nseg];
  const uint64_t Q = ((T + gridDim.x - 1) / gridDim.x + 3) & ~3ull;
  const uint64_t vb = Q * blockIdx.x;
  const uint64_t ve = (vb + Q < T) ? vb + Q : T;
  if (threadIdx.x < WAVE) seg_range_wave(in.prefix, in.nseg, vb, ve, T, s_seg);
  if (threadIdx.x == 0) {
    s_live = 0;
    if (blockIdx.x == 0) tb.ctl->Q = Q;
  }
  __syncthreads();
  const uint32_t slo = s_seg[0], shi = s_seg[1];
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  uint32_t *orec = tb.rec + vb;
  uint64_t *okey = tb.rkey + vb;
  constexpr uint64_t STEP = (uint64_t)TAIL_T * 4;
  uint32_t out_n = 0, live_n = 0;
  for (uint64_t v0 = vb; v0 < ve; v0 += STEP) {
    const uint64_t v = v0 + (uint64_t)threadIdx.x * 4;
    const bool in_range = v < ve;
    const uint64_t ph = tile_phys(in, slo, shi, v, ve);
    const uint4 a4 = *reinterpret_cast<const uint4 *>(src + ph), b4 = *reinterpret_cast<const uint4 *>(dst + ph);
    const ulonglong2 k01 = *reinterpret_cast<const ulonglong2 *>(key + ph),
                     k23 = *reinterpret_cast<const ulonglong2 *>(key + ph + 2);
    const uint32_t A[4] = {a4.x, a4.y, a4.z, a4.w}, B[4] = {b4.x, b4.y, b4.z, b4.w};
    const uint64_t K[4] = {k01.x, k01.y, k23.x, k23.y};
    uint32_t da[4], db[4], mask = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // the dense fragments now (k_tail_labels: one gather per end)
      const bool valid = in_range & (A[j] != LABEL_NONE);
      da[j] = tb.dmap[valid ? A[j] : 0u];
      db[j] = tb.dmap[valid ? B[j] : 0u];
      mask |= (valid & (da[j] != db[j])) ? (1u << j) : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (((mask >> j) & 1u) && (da[j] >= F || db[j] >= F)) {  // a live edge must join two active fragments
        atomicOr(&tb.ctl->err, 1u);
        mask &= ~(1u << j);
      }
    live_n += __popc(mask);
    // survivors -> this block's region of the tail buffer, in order; their candidates carry their index
    uint32_t lane_excl, wave_before, wave_cnt, total;
    block_offsets_w<TAIL_T>((uint32_t)__popc(mask), s_wcnt, &lane_excl, &wave_before, &wave_cnt, &total);
    TailStage &ws = s_stage[wid];
    uint32_t o = lane_excl;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((mask >> j) & 1u) {
        ws.p[o] = da[j] | (db[j] << 16);
        ws.k[o] = K[j];
        const uint64_t c = tail_local(K[j], out_n + wave_before + o);
        lds_min_u64(s_best, da[j], c);
        lds_min_u64(s_best, db[j], c);
        ++o;
      }
    wave_sync_lds();  // the wave's records leave LDS as consecutive stores
    for (uint32_t i = lane; i < wave_cnt; i += WAVE) {
      orec[out_n + wave_before + i] = ws.p[i];
      okey[out_n + wave_before + i] = ws.k[i];
    }
    wave_sync_lds();
    out_n += total;
  }
  for (int d = WAVE / 2; d > 0; d >>= 1) live_n += __shfl_xor(live_n, d);
  if ((threadIdx.x & (WAVE - 1)) == 0) atomicAdd(&s_live, live_n);
  __syncthreads();  // every wave's record stores drained: the row reads them back through L2
  if (check)
    for (uint32_t i = threadIdx.x + 1; i < out_n; i += TAIL_T)
      if ((uint32_t)okey[i - 1] >= (uint32_t)okey[i]) atomicOr(&tb.ctl->err, 1u);
  // the block's minima of every dense fragment (round 0: the root list is the identity)
  tail_row_out(tb, s_best, nullptr, F, orec, okey, nullptr);
  if (threadIdx.x == 0) {
    tb.bcnt[blockIdx.x] = out_n;
    tb.blive[blockIdx.x] = s_live;
  }
}

// One active root per slot (root-list order): the blocks' minima reduced (16 row groups per slot)
// with their other ends, the root's CONNECT target, its MSF flag. Block 0 also totals the
// streamed round's live edges.
// several ranks (multi): the minimum is this rank's only — kept in gloc as well, no MSF flag yet
// (k_tail_xhook writes it once the ranks agree on the minimum)
__global__ __launch_bounds__(256) void k_tail_hook(TailBufs tb, uint32_t r, uint8_t *__restrict__ in_mst,
                                                   uint32_t nblocks, unsigned long long *__restrict__ err,
                                                   bool multi) {
  __shared__ unsigned long long s_part[256];
  __shared__ uint32_t s_prow[256];
  TailCtl *c = tb.ctl;
  if (c->done) return;  // r: the round just streamed
  const uint32_t nroot = (uint32_t)c->nroots[r];
  if (blockIdx.x == 0 && threadIdx.x < WAVE) {
    uint64_t t = 0;
    for (uint32_t b = threadIdx.x; b < nblocks; b += WAVE) t += tb.blive[b];
    for (int d = WAVE / 2; d > 0; d >>= 1) t += __shfl_xor(t, d);
    if (threadIdx.x == 0) c->live[r] = t;
  }
  const uint32_t s = threadIdx.x % TAIL_HS, g = threadIdx.x / TAIL_HS;  // slot, row group
  const uint32_t i = blockIdx.x * TAIL_HS + s;
  if (blockIdx.x * TAIL_HS >= nroot) return;  // block-uniform
  constexpr uint32_t GROUPS = 256 / TAIL_HS;
  uint64_t m = KEY_NONE;
  uint32_t w = 0;
  if (i < nroot) {
    uint64_t x[TAIL_G / GROUPS];
#pragma unroll
    for (uint32_t k = 0; k < TAIL_G / GROUPS; ++k) {
      const uint32_t b = g + k * GROUPS;
      x[k] = b < nblocks ? tb.partial[(uint64_t)b * TAIL_MAX + i] : KEY_NONE;
    }
#pragma unroll
    for (uint32_t k = 0; k < TAIL_G / GROUPS; ++k)
      if (x[k] < m) {
        m = x[k];
        w = g + k * GROUPS;
      }
  }
  s_part[threadIdx.x] = m;
  s_prow[threadIdx.x] = w;
  __syncthreads();
  if (g != 0 || i >= nroot) return;
  for (uint32_t k = 1; k < GROUPS; ++k) {
    const uint64_t x = s_part[k * TAIL_HS + s];
    if (x < m) {
      m = x;
      w = s_prow[k * TAIL_HS + s];
    }
  }
  const uint32_t d = tb.droot[r & 1][i];
  uint32_t o = LABEL_NONE;
  if (m != KEY_NONE) {
    o = tb.poth[(uint64_t)w * TAIL_MAX + i];
    if (o >= c->F0 || o == d) {  // the minimum edge must leave root d towards another root
      atomicOr(err, 2ull);
      o = LABEL_NONE;
      m = KEY_NONE;
    } else if (!multi) {
      in_mst[(uint32_t)m] = 1;  // both members of a mutual pair mark the same edge
    }
  }
  tb.gkey[d] = m;
  tb.ghook[d] = o;
  if (multi) tb.gloc[d] = m;
}

// Several ranks, between the MIN all-reduce of gkey and the MAX all-reduce of ghook: a root whose
// global minimum is this rank's own keeps its CONNECT target (and the owner writes the MSF flag of
// its own edge); every other root's target is withdrawn (LABEL_NONE = -1 under the int32 MAX), so
// the all-reduce leaves the owner's target on every rank. Keys are (w << 32 | global eid): unique.
__global__ __launch_bounds__(256) void k_tail_xhook(TailBufs tb, uint32_t r, uint8_t *__restrict__ in_mst,
                                                    uint32_t e_lo, uint32_t e_hi) {
  const TailCtl *c = tb.ctl;
  if (c->done) return;
  const uint32_t nroot = (uint32_t)c->nroots[r];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nroot; i += gridDim.x * blockDim.x) {
    const uint32_t d = tb.droot[r & 1][i];
    const uint64_t g = tb.gkey[d];
    if (g != KEY_NONE && g == tb.gloc[d]) {
      const uint32_t eid = (uint32_t)g;
      if (eid >= e_lo && eid < e_hi) in_mst[eid] = 1;
    } else {
      tb.ghook[d] = LABEL_NONE;
    }
  }
}

// Every block applies the last round's hooks (identical LDS computation in every block, over the
// roots only), then streams its records — or, when <= 1 root stays active, block 0 finishes the level.
__global__ __launch_bounds__(TAIL_T) void k_tail_round(TailBufs tb, uint32_t r, const uint32_t *__restrict__ act0,
                                                       uint32_t *__restrict__ lab, unsigned long long *__restrict__ cnt,
                                                       unsigned long long *__restrict__ err) {
  __shared__ unsigned long long s_best[TAIL_MAX];  // the prologue's pointer table first (u32 view)
  __shared__ uint16_t s_R[TAIL_MAX];
  __shared__ uint16_t s_root[TAIL_MAX];
  __shared__ uint32_t s_wsum[TAIL_T / WAVE];
  __shared__ unsigned long long s_tw, s_tc;
  __shared__ uint32_t s_live;
  TailCtl *c = tb.ctl;
  if (c->done) return;
  const uint32_t F = c->F0;  // r: the round about to stream (round r - 1 hooked last)
  const uint32_t nprev = (uint32_t)c->nroots[r - 1];
  const uint32_t *prev = tb.droot[(r - 1) & 1];
  uint32_t *P = reinterpret_cast<uint32_t *>(s_best);  // dense pointer forest over the roots (prologue only)
  constexpr uint32_t MARK = 0x80000000u;
  if (threadIdx.x == 0) {
    s_tw = 0;
    s_tc = 0;
    s_live = 0;
  }
  // every global load of the prologue first: the dense ids' roots, the roots' hooks and keys
  constexpr uint32_t PER = TAIL_MAX / TAIL_T;
  const uint32_t *Rp = tb.R[(r - 1) & 1];
  uint32_t rr[PER], pd[PER], ph[PER];
  uint64_t pk[PER];
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t d = threadIdx.x + q * TAIL_T, i = d;
    rr[q] = d < F ? Rp[d] : 0u;
    pd[q] = i < nprev ? prev[i] : 0u;
  }
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t i = threadIdx.x + q * TAIL_T;
    ph[q] = i < nprev ? tb.ghook[pd[q]] : LABEL_NONE;
    pk[q] = i < nprev ? tb.gkey[pd[q]] : KEY_NONE;
  }
  // every dense id a root of itself (an inactive root of round r - 1 stays one), then the hooks of
  // round r - 1's active roots
  for (uint32_t d = threadIdx.x; d < F; d += TAIL_T) P[d] = d;
  __syncthreads();
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t i = threadIdx.x + q * TAIL_T;
    if (i < nprev && ph[q] != LABEL_NONE) P[pd[q]] = ph[q];
  }
  __syncthreads();
  // a mutual pair (d <-> o over their shared minimum) keeps its smaller member as the root
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t i = threadIdx.x + q * TAIL_T;
    if (i < nprev) {
      const uint32_t d = pd[q], o = P[d] & ~MARK;
      if (o != d && (P[o] & ~MARK) == d && d < o) atomicOr(&P[d], MARK);
    }
  }
  __syncthreads();
  unsigned long long tw = 0, tc = 0;
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t i = threadIdx.x + q * TAIL_T;
    if (i < nprev) {
      const uint32_t d = pd[q];
      if (P[d] & MARK) {
        P[d] = d;
      } else if (P[d] != d) {  // d hooked: one MSF edge
        tw += pk[q] >> 32;
        tc += 1;
      }
    }
  }
  __syncthreads();
  for (int it = 0; it < 32; ++it) {  // pointer jumping among the roots (a hook targets a root)
    int more = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
      const uint32_t i = threadIdx.x + q * TAIL_T;
      if (i < nprev) {
        const uint32_t d = pd[q], p = P[d], pp = P[p];
        if (pp != p) {
          P[d] = pp;
          more = 1;
        }
      }
    }
    if (!__syncthreads_or(more)) break;
  }
  // every dense id's root: its round r - 1 root's final root (a root that was not active keeps itself)
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t d = threadIdx.x + q * TAIL_T;
    if (d < F) s_R[d] = (uint16_t)P[rr[q]];
  }
  // next roots: round r - 1's roots that had an edge and stayed roots (ascending: a block scan)
  uint32_t keep = 0;
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t i = threadIdx.x + q * TAIL_T;
    if (i < nprev && pk[q] != KEY_NONE && P[pd[q]] == pd[q]) keep |= 1u << q;
  }
  uint32_t nroot = 0;
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {  // root-list order = prev order (chunks of TAIL_T)
    if (q * TAIL_T < nprev) {  // block-uniform
      uint32_t tot;
      const uint32_t k = (keep >> q) & 1u;
      const uint32_t before = block_excl_scan<TAIL_T>(k, s_wsum, &tot);
      if (k) s_root[nroot + before] = (uint16_t)pd[q];
      nroot += tot;
    }
  }
  for (int dd = WAVE / 2; dd > 0; dd >>= 1) {
    tw += __shfl_xor(tw, dd);
    tc += __shfl_xor(tc, dd);
  }
  if ((threadIdx.x & (WAVE - 1)) == 0 && tc) {
    atomicAdd(&s_tw, tw);
    atomicAdd(&s_tc, tc);
  }
  __syncthreads();
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) {
      if (s_tc) {
        (void)atomicAdd(cnt + 2, s_tw);  // C_WEIGHT, C_EDGES (returning: complete before the report)
        (void)atomicAdd(cnt + 3, s_tc);
      }
      const unsigned long long edges = __hip_atomic_load(cnt + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      c->edges[r - 1] = edges;
    }
    if (nroot <= 1 || r >= TAIL_ROUNDS_MAX) {
      // the level is complete: every fragment of the level takes its final root's label
      uint32_t xs[PER], roots[PER];
#pragma unroll
      for (uint32_t q = 0; q < PER; ++q) {  // every gather in flight, then the stores
        const uint32_t d = threadIdx.x + q * TAIL_T;
        xs[q] = d < F ? act0[d] : 0u;
        roots[q] = d < F ? act0[s_R[d]] : 0u;
      }
#pragma unroll
      for (uint32_t q = 0; q < PER; ++q) {
        const uint32_t d = threadIdx.x + q * TAIL_T;
        if (d < F && roots[q] != xs[q]) lab[xs[q]] = roots[q];
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        if (r >= TAIL_ROUNDS_MAX && nroot > 1) atomicOr(err, 4ull);
        if (c->err) atomicOr(err, 2ull);
        c->done = 1;
        c->rounds = r;
        cnt[0] = 0;  // C_LIVE: no live edge left in the level
      }
      return;
    }
    for (uint32_t d = threadIdx.x; d < F; d += TAIL_T) tb.R[r & 1][d] = s_R[d];
    for (uint32_t i = threadIdx.x; i < nroot; i += TAIL_T) tb.droot[r & 1][i] = s_root[i];
    if (threadIdx.x == 0) c->nroots[r] = nroot;
  }
  if (nroot <= 1 || r >= TAIL_ROUNDS_MAX) return;  // block 0 finishes the level
  // stream this block's records into the LDS minima of the current roots
  for (uint32_t i = threadIdx.x; i < nroot; i += TAIL_T) s_best[s_root[i]] = KEY_NONE;
  __syncthreads();
  const uint64_t base = c->Q * blockIdx.x;
  const uint32_t n = tb.bcnt[blockIdx.x];
  const uint32_t *pr = tb.rec + base;
  const uint64_t *prk = tb.rkey + base;
  uint32_t live_n = 0;
  for (uint32_t e0 = threadIdx.x * 4; e0 < n; e0 += TAIL_T * 4) {
    uint32_t p[4];
    uint64_t k[4];
    if (e0 + 4 <= n) {  // a region starts at a multiple of 4: 16-B aligned
      const uint4 qv = *reinterpret_cast<const uint4 *>(pr + e0);
      const ulonglong2 k01 = *reinterpret_cast<const ulonglong2 *>(prk + e0), k23 = *reinterpret_cast<const ulonglong2 *>(prk + e0 + 2);
      p[0] = qv.x; p[1] = qv.y; p[2] = qv.z; p[3] = qv.w;
      k[0] = k01.x; k[1] = k01.y; k[2] = k23.x; k[3] = k23.y;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[j] = e0 + j < n ? pr[e0 + j] : 0u;
        k[j] = e0 + j < n ? prk[e0 + j] : KEY_NONE;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (e0 + j >= n) continue;
      const uint32_t ra = s_R[p[j] & 0xffffu], rb = s_R[p[j] >> 16];
      if (ra == rb) continue;
      ++live_n;
      const uint64_t cand = tail_local(k[j], e0 + j);
      lds_min_u64(s_best, ra, cand);
      lds_min_u64(s_best, rb, cand);
    }
  }
  for (int dd = WAVE / 2; dd > 0; dd >>= 1) live_n += __shfl_xor(live_n, dd);
  if ((threadIdx.x & (WAVE - 1)) == 0) atomicAdd(&s_live, live_n);
  __syncthreads();
  tail_row_out(tb, s_best, s_root, nroot, pr, prk, s_R);
  if (threadIdx.x == 0) tb.blive[blockIdx.x] = s_live;
}

// the report of a batch of tail rounds (enqueued after its copy of the control block): nact_out 0
// when the level is complete, else the active roots of the last round streamed (more rounds follow)
__global__ void k_tail_report(const TailBufs tb, uint32_t last, RoundSlot *slot, unsigned long long seq,
                              unsigned long long *cnt) {
  const TailCtl *c = tb.ctl;
  write_report(slot, seq, cnt, c->done ? 0ull : (unsigned long long)c->nroots[last], c->F0);
}


static inline unsigned grid_for(uint64_t items, uint64_t per_block, unsigned cap) {
  uint64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Blocks of ONE residency wave of a fixed-grid streaming kernel on the current device (its occupancy
// in blocks per CU x the CUs), at most cap. A fixed grid past it runs a second, nearly empty wave of
// blocks at the end: k_select sits at 7 blocks per CU (its SGPRs) and k_level_pass at 6 (its VGPRs),
// so their 2048-block grids left 256 / 512 blocks to run alone after the rest. Cached per kernel
// and device (one occupancy query each).
#ifndef GHS_RESIDENT_GRIDS
#define GHS_RESIDENT_GRIDS 0
#endif
static unsigned resident_grid(const void *kernel, unsigned block, unsigned cap, bool on = GHS_RESIDENT_GRIDS) {
  if (!on) return cap;
  static std::mutex mu;
  static std::unordered_map<uint64_t, unsigned> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return cap;
  const uint64_t key = (uint64_t)(uintptr_t)kernel * 64 + (uint64_t)dev;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return std::min(it->second, cap);
  int nb = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, (int)block, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || nb <= 0 || cus <= 0)
    return cap;
  const unsigned g = (unsigned)(nb * cus);
  cache[key] = g;
  return std::min(g, cap);
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

// Device counters (cnt[], one 256-B line): every round's sizes stay on the device; kernels read
// them there, so the host launches a round without knowing them (grid sizes are upper bounds).
enum : int {
  C_LIVE = 0,     // live edges (virtual total incl. padding) written by the last compaction scan
  C_WEIGHT = 2,   // MSF weight so far
  C_EDGES = 3,    // MSF edges so far (== hooks)
  C_ERR = C_ERR_IDX,  // invariant / canonicity error bits
  C_PENDING = 5,  // pending edges (virtual total) after the last level pass
  C_N = 6,        // n (the count of the identity active list)
  C_NDENSE = 7,   // fragments of a dense level (several ranks): the count of its identity list
  C_ACT = 8,      // [8], [9]: lengths of the active lists act[0], act[1]
  C_LONG = 10,    // a level-0 edge spans more than one bucket (k_select, lattice-like plans)
  C_RS_WEIGHT = 11,  // [11], [12]: a rank's own-range part of the reduce-scatter round's totals
  C_COUNT = 16
};
static_assert(C_WEIGHT == 2 && C_EDGES == 3 && C_ERR == C_ERR_IDX && C_PENDING == 5 && C_LONG == C_LONG_IDX,
              "write_report reads the counters by index");

constexpr int SLOT_RING = 8;
// rounds enqueued ahead of the host's termination check (GHS_LOOKAHEAD: 0..4). R-MAT s24: 1 ->
// 6.40-6.43 ms per step, 2 -> 6.48-6.59, 3 -> 6.62 (each extra round of lookahead ends every
// level with one more no-op round of ~25 us; one round hides the host's reaction time).
constexpr int LOOKAHEAD = 1;
constexpr uint32_t LEVEL_ROUND_CAP = 64;  // hang guard: a level takes O(log n) rounds

// Host-side resources of a solve: pinned buffers and timing events. Creating them costs far
// more than a small solve (page-pinning, event objects), so the one-shot entry point keeps one
// set per device for the process and reuses it; a stepwise solver handle owns its own.
// counters: all zero, C_N = n (the vertex count as a device-side item count)
__global__ void k_init_counters(unsigned long long *cnt, uint32_t n, unsigned long long *shards) {
  for (int i = threadIdx.x; i < HOOK_SHARDS * SHARD_STRIDE; i += blockDim.x) shards[i] = 0ull;
  for (int i = threadIdx.x; i < C_COUNT; i += blockDim.x) cnt[i] = (i == C_N) ? (unsigned long long)n : 0ull;
}

struct HostRes {
  unsigned long long *h_cnt = nullptr;  // pinned mirror of the device counters
  RoundSlot *h_slot = nullptr;          // pinned, coherent ring of round reports (host view)
  RoundSlot *d_slot = nullptr;          // the same ring, device view
  uint32_t *h_sample = nullptr;         // pinned sample buffer
  TailCtl *h_tail = nullptr;            // pinned copy of the LDS tail's control block (its round stats)
  std::vector<hipEvent_t> ev_pool;      // timing events, 6 per round
  hipEvent_t pass_ev[4] = {};           // the canonical passes' events
  hipEvent_t plan_ev = nullptr;         // the weight sample has landed in h_sample
  hipEvent_t sync_ev = nullptr;         // the cancellable waits of a multi-rank solver (solver_sync)
  unsigned long long seq = 0;           // round reports issued through h_slot (monotonic across solves)
  std::vector<hipEvent_t> prof_ev;      // ghs_profile_enable: two events per launch
};

// Timing-only events: no system-scope fence when they are recorded (they are read only through
// hipEventElapsedTime after the stream is synchronized).
constexpr unsigned TIMING_EVENT_FLAGS = hipEventDisableSystemFence;

static int hostres_init(HostRes *r) {
  GHS_HIP_CHECK(hipHostMalloc((void **)&r->h_cnt, C_COUNT * sizeof(unsigned long long), hipHostMallocDefault));
  // round slots: written by the round's last kernel, read by the host after seq has landed
  GHS_HIP_CHECK(hipHostMalloc((void **)&r->h_slot, SLOT_RING * sizeof(RoundSlot), hipHostMallocMapped | hipHostMallocCoherent));
  GHS_HIP_CHECK(hipHostGetDevicePointer((void **)&r->d_slot, r->h_slot, 0));
  GHS_HIP_CHECK(hipHostMalloc((void **)&r->h_sample, 16384 * 4, hipHostMallocDefault));
  GHS_HIP_CHECK(hipHostMalloc((void **)&r->h_tail, sizeof(TailCtl), hipHostMallocDefault));
  for (int i = 0; i < 4; ++i) GHS_HIP_CHECK(hipEventCreateWithFlags(&r->pass_ev[i], TIMING_EVENT_FLAGS));
  GHS_HIP_CHECK(hipEventCreateWithFlags(&r->plan_ev, hipEventDisableTiming));
  GHS_HIP_CHECK(hipEventCreateWithFlags(&r->sync_ev, hipEventDisableTiming));
  memset(r->h_slot, 0, SLOT_RING * sizeof(RoundSlot));
  return GHS_OK;
}

static void hostres_free(HostRes *r) {
  for (hipEvent_t e : r->ev_pool) (void)hipEventDestroy(e);
  r->ev_pool.clear();
  for (hipEvent_t e : r->prof_ev) (void)hipEventDestroy(e);
  r->prof_ev.clear();
  for (int i = 0; i < 4; ++i)
    if (r->pass_ev[i]) (void)hipEventDestroy(r->pass_ev[i]);
  if (r->plan_ev) (void)hipEventDestroy(r->plan_ev);
  if (r->sync_ev) (void)hipEventDestroy(r->sync_ev);
  if (r->h_cnt) (void)hipHostFree(r->h_cnt);
  if (r->h_slot) (void)hipHostFree(r->h_slot);
  if (r->h_sample) (void)hipHostFree(r->h_sample);
  if (r->h_tail) (void)hipHostFree(r->h_tail);
  r->h_tail = nullptr;
  r->h_cnt = nullptr;
  r->h_slot = r->d_slot = nullptr;
  r->h_sample = nullptr;
}

struct ghs_solver {
  uint32_t n = 0;
  uint64_t m = 0, e_lo = 0, e_hi = 0;
  const uint32_t *eu = nullptr, *ev = nullptr, *ew = nullptr;
  const uint32_t *eoff = nullptr;  // CSR input (ABI 9): row offsets, eu == nullptr (or the caller's u for gathers)
  bool csr = false;
  uint32_t *trow = nullptr;        // CSR: the row of every 256-edge tile of the range (k_csr_tiles)
  uint32_t *bsel = nullptr, *bfil = nullptr;  // CSR: k_select's / k_filter's cost-balanced partitions
  unsigned csr_gsel = 0, csr_gfil = 0;        // ... and the grids they were computed for
  bool trow_ready = false;                    // k_csr_tiles ran this solve (ends_of may use trow)
  bool lab_lazy = false;                      // one rank: lab not yet initialised (ensure_lab / k_jump_ident)
  uint64_t last_nact_in = 0;                  // active fragments at the start of the last reported round
  bool tail_step = false;                     // a stepwise tail in progress (ghs_solver_tail_begin)
  TailRun trun;                               // ... its state
  uint8_t *in_mst = nullptr;
  hipStream_t stream = nullptr;
  ghs_config_t cfg{};

  uint32_t *lab = nullptr, *par = nullptr, *act[2] = {nullptr, nullptr};
  uint64_t *best = nullptr, *bits = nullptr;
  uint8_t *flags = nullptr;
  uint32_t *sample = nullptr;
  uint32_t *giant = nullptr;  // device [0] giant label, [1] its sampled vertex count
  unsigned long long *lb_state = nullptr;  // single-pass select: tile granules (zeroed at create)
  unsigned long long *hook_acc = nullptr;  // sharded hook totals of the counting jumps (bucketed rounds)
  uint32_t lb_epoch = 0;                   // tag of the last select launch
  ArcBuf buf[2];             // a level's edges (regions) and the round double buffer
  ArcBuf rem[2];             // pending (not yet levelled) edges: u, v, key as regions
  int rcur = 0;              // rem buffer holding the pending edges (level >= 1)
  uint32_t rem_nseg = 1;     // regions of the pending edges
  uint64_t rem_total = 0;    // pending edges (incl. padding) after the last level pass (host copy)
  bool pending_built = false; // the FILTER pass has run (levels >= 1 read the pending regions)
  bool debug = false;        // GHS_DEBUG=1: per-level sizes on stderr
  uint64_t cap_arcs = 0;
  unsigned long long *cnt = nullptr;    // device counters (C_*)
  HostRes own;                          // host resources owned by this handle (stepwise API)
  HostRes *res = nullptr;               // the resources in use (own, or the process pool)
  unsigned long long *h_cnt = nullptr;  // = res->h_cnt
  RoundSlot *h_slot = nullptr;          // = res->h_slot
  RoundSlot *d_slot = nullptr;          // = res->d_slot
  uint32_t *h_sample = nullptr;         // = res->h_sample
  uint64_t *h_thr = nullptr;            // the plan's host copy (in the pinned sample buffer)

  // level plan (identical on every rank: computed from the global canonical list)
  std::vector<uint64_t> thresholds;  // level i: [thr[i], thr[i+1]) — host copy, once plan_known
  uint64_t *d_thr = nullptr;          // the plan on the device (k_plan), read by the passes
  bool plan_known = false;
  uint32_t level = 0;                // index of the level being processed
  bool level_open = false;
  uint64_t level_arcs = 0;           // edges of the current level (incl. padding; stats)

  // round state (host view)
  uint32_t round = 0;        // completed rounds (all levels)
  uint32_t level_round = 0;  // rounds issued in this level
  int phase = 0;             // stepwise API: 0 expect minedge, 1 expect contract, 2 done
  int cur = 0;               // edge buffer holding the live edges
  uint32_t cur_nseg = 1;     // its regions
  uint64_t cur_arcs = 0;     // live edges at level start (exact)
  int act_cur = 0;
  bool act_ident = true;     // active fragments are 0..n-1 (count C_N)
  uint64_t nact = 0;         // active fragments: exact in the stepwise API, an upper bound when pipelined
  uint64_t level_nact = 0;   // active fragments at level start (exact)
  uint64_t edges_before = 0;

  std::vector<ghs_round_stats_t> stats;
  std::vector<uint8_t> ev_rec;  // per round: bit k = event k recorded
  hipEvent_t pass_ev[4] = {};   // around k_select [0,1] and k_filter [2,3] (from the host pool)
  bool filter_run = false;
  bool pending_exchange = false;  // multi-rank: a level's flags await the caller's OR all-reduce
  bool hooked = false;            // multi-rank: this round's CONNECT came through the hook exchange
  unsigned open_G = 1;            // regions of the level's edges (between the two halves)
  uint64_t select_out = 0, filter_out = 0;
  bool detail = false;          // GHS_DETAIL=1: time every stage (adds ~5.7 us per event)
  bool time_rounds = false;     // GHS_TIME_ROUNDS=1: time the compacting min-edge launches (bench)
  uint32_t seg_g = SEG_G;       // blocks of the streaming kernels (GHS_SEG_G, 256..SEG_G)
  uint32_t cmp_g = CMP_G;       // blocks (= output regions) of the compacting min-edge (GHS_MINEDGE_G)
  uint32_t ident_g = SEG_G;     // grid caps: round-0 min-edge (GHS_IDENT_G), k_win (GHS_WIN_G: 6
  uint32_t win_g = CMP_G;       // blocks/CU like the compaction, measured ~1% faster per step),
  uint32_t lp_g = SEG_G;        // the level pass (GHS_LP_G)
  bool open_async = false;      // the open level's counts arrive with its first round's report
  bool scan_pending = false;    // the last compaction's region counts are not scanned yet
  bool report_final = false;    // the last round report read holds the final weight / edge count
  unsigned long long rep_weight = 0, rep_edges = 0;
  const ArcBuf *scan_buf = nullptr;
  bool open_ident = false;      // the open level's first round runs over the identity list (level 0, one rank)
  bool arcs_known = true;       // cur_arcs holds the exact live edge count (else: unknown, grids sized for the bound)
  uint32_t lookahead = LOOKAHEAD;  // rounds in flight ahead of the termination check (GHS_LOOKAHEAD)
  std::chrono::steady_clock::time_point t0;
  char *ws_base = nullptr;      // the caller's workspace (carved by workspace_layout)
  bool seed_runs = true;        // level 0 round 0: a-side runs by k_seed_runs (GHS_SEED_RUNS=0: off)
  uint32_t dedup_max = 0;       // parallel-edge filter at <= this many active fragments (GHS_DEDUP_MAX)
  // dense levels (several ranks, see k_dense_open): the dense arrays, the vertex arrays they stand
  // in for while a level runs, and the level's fragment count
  uint32_t *dlab = nullptr, *dpar = nullptr, *dvtx = nullptr;
  uint64_t *drank_bits = nullptr;                  // dense labels by rank (DenseRank)
  bool words_merged = false;                       // this level's flags arrived as merged words
  bool rank_ready = false;                         // ... and the rank tables are built from them
  uint32_t *drank_wpre = nullptr, *drank_cpre = nullptr;
  uint4 *drank_pk = nullptr;  // the packed rank table (k_rank_pack; GHS_DENSE_PACK)
  uint64_t *dbest = nullptr;
  uint32_t *vlab = nullptr, *vpar = nullptr;
  uint64_t *flag_bits = nullptr;  // the packed level-open flags (ghs_solver_flag_bits)
  uint64_t *vbest = nullptr;
  bool dense_mode = false;      // several ranks and the dense arrays exist (GHS_DENSE=0: off)
  bool level_dense = false;     // the open level runs in dense labels
  bool rs_fold = false;         // apply_hooks left partial totals for contract to fold in
  uint64_t dense_n = 0;
  uint64_t hook_S = 0;          // the padded slot count of the last hook_slots (hook_owner's bound)
  bool tail_ran = false;        // a level finished in the LDS tail (k_tail_*)
  TailBufs tail{};              // the LDS tail's arrays (one rank; tail.ctl == nullptr: no tail)
  bool tail_on = true;          // GHS_OPT_NO_TAIL clears it
  bool check_totals = false;    // GHS_OPT_CHECK_TOTALS: report totals vs a stream-ordered counter copy per level
  uint32_t totals_checked = 0;  // levels whose totals were checked (diagnostic)
  // bucketed rounds (single rank, lattice-like graphs; k_bucket / k_bmin): the record buffers,
  // the offsets table, the bucket geometry, and the per-solve / per-round decisions
  uint4 *rec = nullptr;         // records (a, b, key): 16 B each
  uint64_t *wstart = nullptr;   // windowed round 0: each bucket's first edge (nb + 1)
  bool windowed = true;         // level 0 round 0 of a lattice-like solve windowed (k_wmin)
  bool windowed_enq = false;    // ... was enqueued this solve (it ran unless k_select's span flag was set)
  bool windowed_ran = false;    // ... and ran (the span flag of its round report was clear)
  bool state_init_pending = false;  // one rank: best / par initialised by level 0's first round
  uint32_t *bk_off = nullptr;
  uint32_t bk_bs = 13, bk_nb = 0;
  bool bucketed = false;        // this solve runs bucketed rounds (decided once the plan landed)
  bool bucket_decided = false;
  bool bucket_first_only = false;  // only the levels' first rounds (random-like graphs)
  bool lattice = false;            // the plan's span sample says lattice-like
  unsigned jump_ident_g = 16384;   // k_jump_ident's grid cap
  bool round_bucketed = false;  // the round being enqueued is bucketed
  // pipelined rounds of a multi-rank level (ghs_solver_contract_async, rounds >= 2): issued rounds
  // whose report is not read yet (oldest first), the latest exact active count and the level round
  // it starts, the live edges at the start of the oldest unread round
  struct PipeRound {
    unsigned long long seq;
    uint32_t round, level_round;
  };
  std::vector<PipeRound> pipe;
  uint64_t pipe_exact = 0;
  uint32_t pipe_exact_lr = 0;
  uint64_t pipe_live = 0;
  // multi-rank failure agreement: another rank's failure ends this solver's waits (the flags are
  // read with __atomic loads; set by ghs_solver_cancel / the driver's shared group flag)
  int cancel_flag = 0;
  const int *group_cancel = nullptr;
  bool prof = false;            // ghs_profile_enable: every launch bracketed by events
  uint32_t prof_id = 0;         // tag of this handle's profile records (creation order)
  struct ProfRec {
    ghs_kernel_record_t rec;
    size_t ev;                  // index of its first event in res->prof_ev
  };
  std::vector<ProfRec> prof_recs;
};

// ---- per-launch profile (ghs_profile_enable / ghs_profile_read) ------------------------------
// Every kernel launch of a solve bracketed by two HIP events on the solve's stream: the bench's
// per-kernel durations (and the dominant kernel of its roofline line) come from these. The
// events add idle time between launches (~5.7 us each), so the bench times its steps without
// them and profiles one extra step.
// internal accessors for the round loop of multi.hip (common.h)
hipStream_t ghs_solver_stream_of(const ghs_solver *s) { return s->stream; }
uint32_t ghs_solver_n_of(const ghs_solver *s) { return s->n; }
uint32_t ghs_solver_ranks_of(const ghs_solver *s) { return s->cfg.num_ranks; }
// the round's slots in place: a dense level's identity round (its first) keeps the active
// fragments' minima contiguous in best[0, nact) — an unsigned MIN all-reduce over best itself
// replaces pack_best / all-reduce / unpack_best (nullptr: use those)
void ghs_solver_set_group_cancel(ghs_solver *s, const int *flag) { s->group_cancel = flag; }
const ghs_config_t *ghs_solver_cfg_of(const ghs_solver *s) { return &s->cfg; }
uint32_t ghs_solver_round_of(const ghs_solver *s) { return s->round; }
uint64_t *ghs_solver_best_slots_of(ghs_solver *s) {
  return (s->phase == 1 && s->nact && s->act_ident && s->level_dense) ? s->best : nullptr;
}

static std::mutex g_prof_mutex;
static bool g_prof_on = false;
static std::vector<ghs_kernel_record_t> g_prof;
static uint32_t g_prof_next_id = 0;

static const char *const KERNEL_NAMES[GHS_K_COUNT] = {
    "k_select", "k_filter", "k_level_pass", "k_seed_runs", "k_minedge<IDENT>", "k_minedge<COMPACT>",
    "k_win", "k_hook", "k_jump_ident", "k_jump", "k_select_lb", "k_resolve", "k_giant", "k_scan_counts",
    "k_plan", "k_init", "k_pack_best", "k_unpack_best", "k_round_report", "k_pack_hook", "k_unpack_hook", "k_dense", "k_flag_bits", "k_bucket", "k_bmin", "k_wstarts", "k_wmin", "k_hot_hook",
    "k_tail_open", "k_tail_round", "k_tail_hook", "k_csr_trow"};

struct KtScope {
  ghs_solver *s;
  KtScope(ghs_solver *s_, uint32_t kernel, uint64_t items) : s(s_->prof ? s_ : nullptr) {
    if (!s) return;
    std::vector<hipEvent_t> &pool = s->res->prof_ev;
    const size_t idx = s->prof_recs.size() * 2;
    while (pool.size() < idx + 2) {
      hipEvent_t ev = nullptr;
      if (hipEventCreateWithFlags(&ev, TIMING_EVENT_FLAGS) != hipSuccess) {
        s = nullptr;
        return;
      }
      pool.push_back(ev);
    }
    ghs_solver::ProfRec r{};
    r.rec.kernel = kernel;
    r.rec.round = s->round;
    r.rec.level = s->level;
    r.rec.items = items;
    r.rec.solver = s->prof_id;
    r.ev = idx;
    s->prof_recs.push_back(r);
    (void)hipEventRecord(pool[idx], s->stream);
  }
  ~KtScope() {
    if (s) (void)hipEventRecord(s->res->prof_ev[s->prof_recs.back().ev + 1], s->stream);
  }
};
#define KT(kernel, items) KtScope _kt_scope(s, (kernel), (items))

static inline Ends ends_of(const ghs_solver *s) {
  return Ends{s->eu, s->eoff, s->ev, s->n, s->csr && s->trow_ready ? s->trow : nullptr, s->e_lo & ~3ull, s->e_hi};
}

static bool solver_cancelled(const ghs_solver *s) {
  return __atomic_load_n(&s->cancel_flag, __ATOMIC_ACQUIRE) ||
         (s->group_cancel && __atomic_load_n(s->group_cancel, __ATOMIC_ACQUIRE));
}

bool ghs_solver_cancelled_of(const ghs_solver *s) { return solver_cancelled(s); }

// wait until `ev` (recorded on the solver's stream) has completed. One rank: a blocking wait.
// Several ranks: a poll that another rank's failure ends (ghs_solver_cancel) — a rank whose peer
// failed would otherwise wait forever behind a collective the peer never joins.
static int event_wait(ghs_solver *s, hipEvent_t ev) {
  if (s->cfg.num_ranks <= 1 && !s->group_cancel) {
    GHS_HIP_CHECK(hipEventSynchronize(ev));
    return GHS_OK;
  }
  // a few tight polls, then a short sleep between polls: every poll is a runtime call, and several
  // rank threads of one process (ghs_mst_multi / ghs_mst_emulated) polling back to back contend
  // for the runtime's locks with each other's launches
  for (uint32_t spins = 0;; ++spins) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return GHS_OK;
    if (q != hipErrorNotReady) GHS_HIP_CHECK(q);
    if (solver_cancelled(s)) GHS_FAIL(GHS_E_STATE, "cancelled: another rank of the solve failed");
    if (spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(10));
  }
}

// every piece of work enqueued so far on the solver's stream has completed
static int solver_sync(ghs_solver *s) {
  if (s->cfg.num_ranks <= 1 && !s->group_cancel) {
    GHS_HIP_CHECK(hipStreamSynchronize(s->stream));
    return GHS_OK;
  }
  GHS_HIP_CHECK(hipEventRecord(s->res->sync_ev, s->stream));
  return event_wait(s, s->res->sync_ev);
}

// after the solve: durations into the process-wide profile (one stream sync)
static int prof_collect(ghs_solver *s) {
  if (!s->prof || s->prof_recs.empty()) return GHS_OK;
  if (int rc = solver_sync(s)) return rc;
  std::lock_guard<std::mutex> lock(g_prof_mutex);
  for (const auto &r : s->prof_recs) {
    ghs_kernel_record_t rec = r.rec;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, s->res->prof_ev[r.ev], s->res->prof_ev[r.ev + 1]) != hipSuccess) ms = -1.f;
    rec.ms = ms;
    g_prof.push_back(rec);
  }
  s->prof_recs.clear();
  return GHS_OK;
}

static std::mutex g_mutex;  // the one-shot entry points are serialised per process

// process-wide host resources of the one-shot entry point, one set per device (under g_mutex)
static HostRes *pooled_res(int *rc) {
  static std::unordered_map<int, HostRes *> pools;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  auto it = pools.find(dev);
  if (it != pools.end()) return it->second;
  HostRes *r = new HostRes();
  if ((*rc = hostres_init(r)) != GHS_OK) {
    hostres_free(r);
    delete r;
    return nullptr;
  }
  pools[dev] = r;
  return r;
}

static constexpr uint32_t NSAMPLE_MAX = NSAMPLE_W;

// the bucketed rounds' geometry: buckets of 2^bs labels (bs 13 or 14: a k_bmin slice of 64 or 128
// KiB of LDS), nb <= BK_MAX_B of them; false when n is too large for it (n > 2^28)
static bool bucket_geometry(uint32_t n, uint32_t *bs, uint32_t *nb) {
  if (n == 0) return false;
  const uint32_t b = n <= (1u << 27) ? 13u : 14u;
  const uint64_t k = ((uint64_t)n + (1ull << b) - 1) >> b;
  if (k > BK_MAX_B) return false;
  *bs = b;
  *nb = (uint32_t)k;
  return true;
}

// Arrays are staggered by WS_STAGGER bytes: with power-of-two n (R-MAT, 2^k-sided grids) the
// vertex arrays are power-of-two sized, so lab[v], par[v] and best[v] — which k_jump_ident and
// the hooks read at the same index — would sit at power-of-two distances and land in the same
// memory channels. 16384^2 grid, same box (profiles/r05/ab/stagger/): k_jump_ident 4.25 -> 4.00 ms,
// the step 37.5 -> 37.25 ms (2 repeats each; a 20.6-KiB stagger gave the same jump).
#ifndef GHS_WS_STAGGER
#define GHS_WS_STAGGER ((1u << 20) + 1024u)
#endif
constexpr size_t WS_STAGGER = GHS_WS_STAGGER;
static size_t workspace_layout(uint32_t n, uint64_t m, uint64_t local_edges, ghs_solver *s, char *base) {
  size_t off = 0;
  // only the vertex-sized arrays (read at the same index by the jumps and hooks) are staggered
  // (a stagger after every carve grew every workspace by ~60 MB, tiny graphs included)
  auto carve = [&](size_t bytes, bool stagger = false) -> char * {
    char *p = base ? base + off : nullptr;
    off = align_up(off + bytes, 256) + (stagger ? WS_STAGGER : 0);
    return p;
  };
  const size_t N = (size_t)n;
  // a level's edges (+ padding of the regions, + the heavy copy's last block: < T/256 + 2 groups)
  const uint64_t cap = local_edges + 4 * SEG_MAX + local_edges / 256 + 2 * 2048;
  char *p;
  const bool stg = N * 4 >= (4u << 20);  // small graphs: no stagger at all
  p = carve(N * 4, stg); if (s) s->lab = (uint32_t *)p;
  p = carve(N * 4, stg); if (s) s->par = (uint32_t *)p;
  p = carve(N * 8, stg); if (s) s->best = (uint64_t *)p;
  p = carve(N * 4, stg); if (s) s->act[0] = (uint32_t *)p;
  p = carve(N * 4, stg); if (s) s->act[1] = (uint32_t *)p;
  if (local_edges < m) {  // a rank of a multi-rank solve: the dense-level arrays
    p = carve(N * 4, stg); if (s) s->dlab = (uint32_t *)p;
    p = carve(N * 4, stg); if (s) s->dpar = (uint32_t *)p;
    p = carve((N + 64) * 8, stg); if (s) s->dbest = (uint64_t *)p;  // + padding of the reduce-scatter slots
    const size_t W = (N + 63) / 64;
    p = carve(W * 8); if (s) s->drank_bits = (uint64_t *)p;
    p = carve(W * 4); if (s) s->drank_wpre = (uint32_t *)p;
    p = carve(((W + BLOCK - 1) / BLOCK) * 4 + 4); if (s) s->drank_cpre = (uint32_t *)p;
    p = carve(W * 16); if (s) s->drank_pk = (uint4 *)p;
    p = carve(N * 4, stg); if (s) s->dvtx = (uint32_t *)p;
  }
  p = carve(N + 1); if (s) s->flags = (uint8_t *)p;  // + the multi-rank error byte flags[n]
  p = carve(((N + 127) / 128) * 16 + 16); if (s) s->bits = (uint64_t *)p;
  p = carve(((N + 1 + 63) / 64) * 8); if (s) s->flag_bits = (uint64_t *)p;
  p = carve(2 * NSAMPLE_MAX * 4); if (s) s->sample = (uint32_t *)p;  // weights + spans
  p = carve((PLAN_LOCAL + 1) * 8); if (s) s->d_thr = (uint64_t *)p;
  p = carve((GIANT_HOT + 1 + HOT_K) * 4); if (s) s->giant = (uint32_t *)p;  // giant, hot list
  p = carve(LB_MAX_TILES * 8); if (s) s->lb_state = (unsigned long long *)p;  // select tile granules
  p = carve(HOOK_SHARDS * SHARD_STRIDE * 8); if (s) s->hook_acc = (unsigned long long *)p;  // jump totals
  for (int b = 0; b < 2; ++b) {
    p = carve(cap * 4); if (s) s->buf[b].src = (uint32_t *)p;
    p = carve(cap * 4); if (s) s->buf[b].dst = (uint32_t *)p;
    p = carve(cap * 8); if (s) s->buf[b].key = (uint64_t *)p;
    p = carve(SEG_MAX * 8); if (s) s->buf[b].seg_start = (uint64_t *)p;
    p = carve(SEG_MAX * 8); if (s) s->buf[b].seg_count = (uint64_t *)p;
    p = carve((SEG_MAX + 1) * 8); if (s) s->buf[b].seg_prefix = (uint64_t *)p;
  }
  for (int b = 0; b < 2; ++b) {
    p = carve(cap * 4); if (s) s->rem[b].src = (uint32_t *)p;
    p = carve(cap * 4); if (s) s->rem[b].dst = (uint32_t *)p;
    p = carve(cap * 8); if (s) s->rem[b].key = (uint64_t *)p;
    p = carve(SEG_MAX * 8); if (s) s->rem[b].seg_start = (uint64_t *)p;
    p = carve(SEG_MAX * 8); if (s) s->rem[b].seg_count = (uint64_t *)p;
    p = carve((SEG_MAX + 1) * 8); if (s) s->rem[b].seg_prefix = (uint64_t *)p;
  }
  if (s) s->cap_arcs = cap;
  p = carve(C_COUNT * sizeof(unsigned long long)); if (s) s->cnt = (unsigned long long *)p;
  p = carve((local_edges / 256 + 8) * 4); if (s) s->trow = (uint32_t *)p;  // CSR: each 256-edge tile's row
  p = carve((SEG_MAX + 3) * 4); if (s) s->bsel = (uint32_t *)p;             // CSR: k_select's wave slices (+ Rb, Re)
  p = carve((SEG_G + 1) * 4); if (s) s->bfil = (uint32_t *)p;               // CSR: k_filter's block ranges
  {  // the LDS tail's arrays (its records go to the idle edge buffer); several ranks: dense levels
    p = carve(N * 4, stg); if (s) s->tail.dmap = (uint32_t *)p;
    p = carve((size_t)TAIL_G * TAIL_MAX * 8); if (s) s->tail.partial = (uint64_t *)p;
    p = carve((size_t)TAIL_G * TAIL_MAX * 2); if (s) s->tail.poth = (uint16_t *)p;
    for (int b = 0; b < 2; ++b) {
      p = carve(TAIL_MAX * 4); if (s) s->tail.R[b] = (uint32_t *)p;
      p = carve(TAIL_MAX * 4); if (s) s->tail.droot[b] = (uint32_t *)p;
    }
    p = carve(TAIL_MAX * 4); if (s) s->tail.ghook = (uint32_t *)p;
    p = carve(TAIL_MAX * 8); if (s) s->tail.gkey = (uint64_t *)p;
    p = carve(TAIL_MAX * 8); if (s) s->tail.gloc = (uint64_t *)p;
    p = carve(TAIL_G * 4); if (s) s->tail.blive = (uint32_t *)p;
    p = carve(TAIL_G * 4); if (s) s->tail.bcnt = (uint32_t *)p;
    p = carve(sizeof(TailCtl)); if (s) s->tail.ctl = (TailCtl *)p;
  }
  // bucketed rounds (single rank, n <= 2^28): records (an edge gives at most two) + offsets
  uint32_t bs = 0, nb = 0;
  if (local_edges == m && bucket_geometry(n, &bs, &nb)) {
    const uint64_t rc = 2 * cap + 8 * BK_G;
    p = carve(rc * 16); if (s) s->rec = (uint4 *)p;
    p = carve((size_t)(nb + 1) * BK_G * 4); if (s) s->bk_off = (uint32_t *)p;
    p = carve((size_t)(nb + 1) * 8 + SEG_MAX * 4); if (s) s->wstart = (uint64_t *)p;  // + region-first table
    if (s) {
      s->bk_bs = bs;
      s->bk_nb = nb;
    }
  }
  return off;
}

static hipEvent_t round_event(ghs_solver *s, uint32_t round, int k) {
  if (round >= GHS_MAX_ROUND_STATS) return nullptr;
  const size_t idx = (size_t)round * 6 + k;
  std::vector<hipEvent_t> &pool = s->res->ev_pool;
  while (pool.size() <= idx) {
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, TIMING_EVENT_FLAGS) != hipSuccess) return nullptr;
    pool.push_back(ev);
  }
  return pool[idx];
}

// Timing events cost ~5.7 us of GPU idle each between dependent kernels (measured), so rounds
// are not timed by default; GHS_TIME_ROUNDS=1 brackets the compacting min-edge launches (the
// bench's instrumented step), GHS_DETAIL=1 every stage of every round.
static void record(ghs_solver *s, int k) {
  hipEvent_t ev = round_event(s, s->round, k);
  if (!ev) return;
  if (hipEventRecord(ev, s->stream) != hipSuccess) return;
  if (s->ev_rec.size() <= s->round) s->ev_rec.resize(s->round + 1, 0);
  s->ev_rec[s->round] |= (uint8_t)(1u << k);
}

static uint32_t next_tag(ghs_solver *s) {
  if (++s->lb_epoch == 0) s->lb_epoch = 1;  // 0 is the zeroed state's tag
  return s->lb_epoch;
}

// Order-preserving select, one launch: (act ? act[i] : i) for the i < *d_count with flags[i] != 0
// (bound >= *d_count on the host sizes the grid). *d_total = kept items.
// slot != nullptr: the kernel also reports the round (seq) to the pinned slot.
static int select_lb(ghs_solver *s, const uint32_t *act, const unsigned long long *d_count, uint64_t bound,
                     uint32_t *out, unsigned long long *d_total, RoundSlot *slot = nullptr, unsigned long long seq = 0,
                     bool fold_hooks = false) {
  if (bound == 0) {
    GHS_HIP_CHECK(hipMemsetAsync(d_total, 0, 8, s->stream));
    if (slot) {
      KT(GHS_K_ROUND_REPORT, 0);
      k_round_report<<<1, 1, 0, s->stream>>>(slot, seq, s->cnt, d_total, d_count);
    }
    GHS_HIP_CHECK(hipGetLastError());
    return GHS_OK;
  }
  // tiles of G groups, at most LB_MAX_TILES of them (co-resident)
  const uint64_t per = (uint64_t)LB_MAX_TILES * LB_GROUP;
  const uint64_t G = (bound + per - 1) / per;
  const uint64_t nb = (bound + G * LB_GROUP - 1) / (G * LB_GROUP);
  if (nb > LB_MAX_TILES || G >= (1ull << 20)) GHS_FAIL(GHS_E_STATE, "select: bad tiling");
  KT(GHS_K_SELECT_LB, bound);
  k_select_lb<<<(unsigned)nb, BLOCK, 0, s->stream>>>(s->flags, act, d_count, (uint32_t)G, out, d_total, s->lb_state,
                                                     next_tag(s), slot, seq, s->cnt, fold_hooks ? s->hook_acc : nullptr);
  GHS_HIP_CHECK(hipGetLastError());
  return GHS_OK;
}

static void default_config(ghs_config_t *c) {
  c->max_levels = 8;
  c->num_ranks = 1;
  c->level1_edges_per_vertex = 0.0;  // auto: level1_auto()
  c->level_growth = 8.0;  // R-MAT s24 sweep (tools/sweep_levels.py): 3 levels, 0.5n / 4n / rest
  c->options = 0;
  c->dedup_max = 0;
  c->fault_rank = 0;
  c->fault_round = 0;
}

// level1_edges_per_vertex <= 0 picks the first level's size from the density. The first level
// should just reach the point where a giant fragment forms (the filter of the later levels drops
// the edges inside it) without paying for an extra level of n-sized passes: 0.5n edges for dense
// random-like graphs (R-MAT s24: 6.18 ms vs 6.98 at 1.0n), 1.2n for sparse lattice-like ones
// (just past bond percolation of the square lattice at half the edges; 16384^2 grid: 56 ms vs 72
// at 0.5n, profiles/r01/sweep_levels_*.jsonl; r03 with the bucketed level-0 rounds, two sweeps:
// grid 39.1 / 40.1 ms at 1.0n -> 38.8 / 39.4 at 1.2n, gradient grid 15.9 / 16.0 -> 15.7 / 15.3,
// profiles/r03/sweeps/; R-MAT 0.35-0.5n within the noise).
static double level1_auto(const ghs_config_t &c, uint32_t n, uint64_t m) {
  if (c.level1_edges_per_vertex > 0) return c.level1_edges_per_vertex;
  return (m >= 4ull * n) ? 0.5 : 1.2;
}

// ---- level planning: thresholds from a sample of the GLOBAL canonical weights ----------------
// On the device (k_sample_weights -> k_plan -> d_thr, read by the passes), so the first pass
// starts without a host round trip; the host's copy (pinned, behind plan_ev) is read only when
// it needs the number of levels — at the end of level 0 at the earliest.
// With several ranks every level costs each rank n-sized passes (resolve, select, flag exchange,
// dense open/close) while its edge work is divided by the ranks: once a rank's share of the list
// is below 3n edges, two levels (the first as planned, then everything heavier) beat three.
// R-MAT s26 (n = 2^26), emulated ranks (profiles/r02/plan_s26_*.jsonl): N = 8 (m/N = 2n): 8.29 ->
// 7.85 ms max-rank compute, 884 -> 825 MB wire per rank; N = 4 (3.9n): 10.85 -> 11.47 ms and
// N = 2: 16.5 -> 18.6 ms — kept at three there.
static uint32_t plan_levels_count(const ghs_solver *s) {
  uint32_t L = std::max<uint32_t>(1, std::min<uint32_t>(s->cfg.max_levels, 32));
  if (s->cfg.num_ranks > 1 && s->m / s->cfg.num_ranks < 3ull * s->n) L = std::min<uint32_t>(L, 2);
  return L;
}

static int plan_levels_enqueue(ghs_solver *s) {
  const uint32_t L = plan_levels_count(s);
  const uint32_t ns_all = (uint32_t)std::min<uint64_t>(NSAMPLE_W, s->m);
  const uint32_t ns = L > 1 ? ns_all : 0u;
  {
    KT(GHS_K_PLAN, ns);
    if (ns_all)
      k_sample_weights<<<grid_for(ns_all, 256, 256), 256, 0, s->stream>>>(s->m, ends_of(s), s->ew, ns_all, s->sample);
    k_plan<<<1, 1024, 0, s->stream>>>(s->sample, ns_all, ns, s->n, s->m, L, level1_auto(s->cfg, s->n, s->m),
                                      s->cfg.level_growth, s->d_thr);
  }
  GHS_HIP_CHECK(hipGetLastError());
  GHS_HIP_CHECK(hipMemcpyAsync(s->h_thr, s->d_thr, (PLAN_LOCAL + 1) * 8, hipMemcpyDeviceToHost, s->stream));
  GHS_HIP_CHECK(hipEventRecord(s->res->plan_ev, s->stream));
  s->plan_known = false;
  return GHS_OK;
}

// the host copy of the plan (waits for it the first time)
static int plan_sync(ghs_solver *s) {
  if (s->plan_known) return GHS_OK;
  if (int rc = event_wait(s, s->res->plan_ev)) return rc;
  const uint64_t cnt = s->h_thr[PLAN_MAX];
  if (cnt < 2 || cnt > PLAN_MAX) GHS_FAIL(GHS_E_STATE, "bad level plan");
  s->thresholds.assign(s->h_thr, s->h_thr + cnt);
  s->plan_known = true;
  return GHS_OK;
}

// every level done? (level 0 always exists: no wait for the plan before it)
static bool levels_done(ghs_solver *s) {
  if (s->level == 0 && !s->plan_known) return false;
  if (plan_sync(s)) return true;
  return s->level + 1 >= s->thresholds.size();
}


static int fail_counters(ghs_solver *s, unsigned long long err, const char *where) {
  s->phase = 2;
  if (err & 8) GHS_FAIL(GHS_E_NONCANON, "edge list is not canonical (need u < v < n, strictly ascending (u, v))");
  if (err == 32) GHS_FAIL(GHS_E_STATE, std::string("another rank failed ") + where);
  GHS_FAIL(GHS_E_STATE, std::string("internal invariant violated ") + where + " (code " + std::to_string(err) + ")");
}

static int open_level_finish(ghs_solver *s);
static void ensure_lab(ghs_solver *s);

// ---- open the next level: select its edges, set its active list (one host sync) --------------
// Returns GHS_OK with s->level_open set, with the level skipped (no edges), or — several ranks —
// with s->pending_exchange set (the caller OR-combines the flags, then open_level_finish).
static int open_level_async(ghs_solver *s);

static int open_level(ghs_solver *s, bool async_open = false) {
  s->report_final = false;
  const uint32_t lv = s->level;
  const uint64_t *d_range = s->d_thr + lv;  // this level's [w_lo, w_hi] on the device
  const bool first = (lv == 0);
  const bool single = s->cfg.num_ranks <= 1;
  hipStream_t st = s->stream;
  ArcBuf &Y = s->buf[1];

  if (!first) {
    ensure_lab(s);
    // find the giant fragment from a sample, compress labels and build its bitmap (on device)
    {
      KT(GHS_K_GIANT, 0);
      k_giant<<<1, 1024, 0, st>>>(s->n, s->lab, s->giant, s->cnt + C_ERR);
    }
    {
      KT(GHS_K_RESOLVE, s->n);
      k_resolve<<<grid_for(s->n, BLOCK, 16384), BLOCK, 0, st>>>(s->n, s->lab, s->giant, s->bits, s->cnt + C_ERR);
    }
    GHS_HIP_CHECK(hipGetLastError());
  }

  // 1. this level's edges -> regions of Y (level edges: a, b labels + key, canonical order).
  //    The pass also flags both ends of every level edge (the level's active fragments).
  // Single rank, async open: no active flags at all. Round 0 runs over the identity list of all
  // n vertices (k_win needs no list; k_jump skips the vertices that were not roots when the level
  // opened and keeps the roots that found an outgoing edge), which costs a sequential pass over
  // lab/par/best instead of 2 random flag stores per level edge inside the pass (their line
  // write-backs were ~0.25 GB per k_filter launch) plus the select.
  const bool ident0 = single && async_open;
  uint8_t *mark = ident0 ? nullptr : s->flags;
  if (!ident0) GHS_HIP_CHECK(hipMemsetAsync(s->flags, 0, (size_t)s->n + 1, st));
  s->open_ident = ident0;
  unsigned G = 1;
  const uint64_t TC = s->e_hi > s->e_lo ? s->e_hi - (s->e_lo & ~3ull) : 0;  // canonical passes stream [e_lo & ~3, e_hi)
  if (first) {
    // SELECT over the canonical list: level-0 edges only (validates the list)
    auto sel = s->csr ? k_select<true> : k_select<false>;
    G = grid_for(TC, ARCS_PER_BLOCK, resident_grid((const void *)sel, BLOCK, s->seg_g));
    if (TC) {
      if (s->csr) {
        // CSR: every 256-edge tile's row, the offsets' validation, and both passes' cost-balanced
        // partitions (k_select's G x 4 wave slices, k_filter's block ranges for its grid)
        auto filt = k_filter<true>;
        s->csr_gsel = G;
        s->csr_gfil = grid_for(TC, ARCS_PER_BLOCK,
                               resident_grid((const void *)filt, BLOCK, s->seg_g, GHS_RESIDENT_GRIDS || !GHS_FILTER_CSR_W8));
        s->trow_ready = true;
        KT(GHS_K_CSR_TROW, s->n);
        uint32_t *rb = s->bsel + SEG_MAX + 1;  // (2 words past k_select's bounds)
        const uint32_t nsel = G * (BLOCK / WAVE), nfil = s->csr_gfil;
        k_csr_range<<<1, 64, 0, st>>>(s->eoff, s->n, s->e_lo & ~3ull, s->e_hi, rb);
        k_csr_check<<<grid_for(s->n, 256 * 8, 2048), 256, 0, st>>>(s->eoff, s->n, s->m, s->cnt + C_ERR);
        k_csr_tiles<<<(unsigned)((TC + 255) / 256 / 256 + 1), 256, 0, st>>>(s->eoff, rb, s->e_lo & ~3ull, s->e_hi, s->trow);
        k_csr_bounds<<<(nsel + nfil + 2 + 255) / 256, 256, 0, st>>>(s->eoff, rb, s->e_lo & ~3ull, s->e_hi, s->bsel, nsel,
                                                                    s->bfil, nfil);
      }
      GHS_HIP_CHECK(hipEventRecord(s->res->pass_ev[0], st));
      {
        KT(GHS_K_SELECT, TC);
        sel<<<G, BLOCK, 0, st>>>(s->n, s->m, s->e_lo, s->e_hi, s->eu, s->eoff, s->ev, s->ew, d_range + 1, Y.src, Y.dst,
                                 Y.key, Y.seg_start, Y.seg_count, mark, s->cnt + C_ERR,
                                 s->wstart ? s->d_thr + PLAN_LOCAL : nullptr, s->bk_bs, s->cnt + C_LONG, s->trow,
                                 s->bsel);
      }
      GHS_HIP_CHECK(hipEventRecord(s->res->pass_ev[1], st));
      GHS_HIP_CHECK(hipGetLastError());
      G *= BLOCK / WAVE;  // one output segment per wave
      KT(GHS_K_SCAN, G);
      k_scan_counts<<<1, 1024, 0, st>>>(Y.seg_count, G, Y.seg_prefix, s->cnt + C_LIVE);
    } else {
      GHS_HIP_CHECK(hipMemsetAsync(Y.seg_prefix, 0, 16, st));
      GHS_HIP_CHECK(hipMemsetAsync(s->cnt + C_LIVE, 0, 8, st));
    }
    GHS_HIP_CHECK(hipMemsetAsync(s->cnt + C_PENDING, 0, 8, st));
  } else {
    const int rin = s->rcur, rout = s->rcur ^ 1;
    ArcBuf &RI = s->rem[rin], &RO = s->rem[rout];
    if (!s->pending_built) {
      // FILTER + level split over the canonical list once level 0 is complete: level-1 edges
      // not inside one fragment -> Y; heavier edges not inside the giant -> pending (rem[rout])
      // CSR input with the caller's u resident too: the COO form of the filter (the pass is
      // probe-bound, and deriving u costs it more than the 4 B/edge it saves: R-MAT s24 1.59 vs
      // 1.62-1.63 ms), while k_select keeps the CSR stream (0.53 vs 0.68 ms)
      const bool fcsr = s->csr && !s->eu;
      auto filt = fcsr ? k_filter<true> : k_filter<false>;
      G = fcsr ? s->csr_gfil : grid_for(TC, ARCS_PER_BLOCK, resident_grid((const void *)filt, BLOCK, s->seg_g));
      if (TC) {
        GHS_HIP_CHECK(hipEventRecord(s->res->pass_ev[2], st));
        {
          KT(GHS_K_FILTER, TC);
          filt<<<G, BLOCK, 0, st>>>(s->n, s->e_lo, s->e_hi, s->eu, s->eoff, s->trow, s->ev, s->ew, d_range, s->bits, s->giant, s->lab,
                                        Y.src, Y.dst, Y.key, Y.seg_start, Y.seg_count, RO.src, RO.dst, RO.key,
                                        RO.seg_start, RO.seg_count, mark, s->bfil);
        }
        GHS_HIP_CHECK(hipGetLastError());
        GHS_HIP_CHECK(hipEventRecord(s->res->pass_ev[3], st));
        s->filter_run = true;
        KT(GHS_K_SCAN, G);
        k_scan_counts<<<1, 1024, 0, st>>>(RO.seg_count, G, RO.seg_prefix, s->cnt + C_PENDING);
        k_scan_counts<<<1, 1024, 0, st>>>(Y.seg_count, G, Y.seg_prefix, s->cnt + C_LIVE);
      } else {
        GHS_HIP_CHECK(hipMemsetAsync(RO.seg_prefix, 0, 16, st));
        GHS_HIP_CHECK(hipMemsetAsync(Y.seg_prefix, 0, 16, st));
        GHS_HIP_CHECK(hipMemsetAsync(s->cnt + C_LIVE, 0, 8, st));
        GHS_HIP_CHECK(hipMemsetAsync(s->cnt + C_PENDING, 0, 8, st));
      }
      GHS_HIP_CHECK(hipGetLastError());
      s->pending_built = true;
    } else {
      // split the pending edges (total on the device): this level's inter-fragment edges -> Y;
      // heavier survivors -> RO regions. Fixed grid: block b owns 1/seg_g of the virtual range.
      G = resident_grid((const void *)k_level_pass, BLOCK, s->lp_g);
      SegView in{RI.seg_start, RI.seg_prefix, s->rem_nseg};
      {
      KT(GHS_K_LEVEL_PASS, s->rem_total);
      k_level_pass<<<G, BLOCK, 0, st>>>(RI.src, RI.dst, RI.key, in, d_range + 1, s->lab, s->bits, s->giant, Y.src, Y.dst, Y.key,
                                        Y.seg_start, Y.seg_count, RO.src, RO.dst, RO.key, RO.seg_start, RO.seg_count,
                                        mark);
      }
      GHS_HIP_CHECK(hipGetLastError());
      KT(GHS_K_SCAN, G);
      k_scan_counts<<<1, 1024, 0, st>>>(RO.seg_count, G, RO.seg_prefix, s->cnt + C_PENDING);
      k_scan_counts<<<1, 1024, 0, st>>>(Y.seg_count, G, Y.seg_prefix, s->cnt + C_LIVE);
      GHS_HIP_CHECK(hipGetLastError());
    }
    s->rem_nseg = G;
    s->rcur = rout;
  }

  if (!single) {  // the caller OR-combines the flags across ranks, then open_level_finish
    k_err_to_flag<<<1, 1, 0, st>>>(s->cnt + C_ERR, s->flags + s->n);  // travels with the flags
    GHS_HIP_CHECK(hipGetLastError());
    s->pending_exchange = true;
    s->open_G = G;
    return GHS_OK;
  }
  s->open_G = G;
  return async_open ? open_level_async(s) : open_level_finish(s);
}

// ---- dense levels (several ranks; kernels at k_dense_open) ------------------------------------
#ifndef GHS_DENSE_PACK
#define GHS_DENSE_PACK 1
#endif
static DenseRank dense_rank_of(const ghs_solver *s) {
  DenseRank r;
  r.bits = s->drank_bits;
  r.wpre = s->drank_wpre;
  r.cpre = s->drank_cpre;
  r.pk = GHS_DENSE_PACK ? s->drank_pk : nullptr;
  return r;
}

// after k_rank_chunks: the packed table every dense_rank lookup of the level reads
static void rank_pack(ghs_solver *s, uint64_t words) {
  if (GHS_DENSE_PACK && s->drank_pk)
    k_rank_pack<<<grid_for(words, 256, 8192), 256, 0, s->stream>>>(s->drank_bits, s->drank_wpre, s->drank_cpre, words,
                                                                  s->drank_pk);
}

static int dense_open(ghs_solver *s) {
  hipStream_t st = s->stream;
  const uint64_t nact = s->nact;
  {
    KT(GHS_K_DENSE, nact);
    const uint64_t words = ((uint64_t)s->n + 63) / 64;
    const uint32_t chunks = (uint32_t)((words + BLOCK - 1) / BLOCK);
    if (s->rank_ready) {  // rank tables from the merged words (open_level_finish)
      k_dense_open_words<<<grid_for(words, 256, 16384), 256, 0, st>>>(dense_rank_of(s), words, s->dvtx);
      k_dense_init<<<grid_for(nact, 256, 16384), 256, 0, st>>>(s->cnt + C_ACT, s->dlab, s->dpar, s->dbest,
                                                               s->cnt + C_NDENSE);
    } else {
      k_rank_words<<<chunks, BLOCK, 0, st>>>(s->flags, s->n, s->drank_bits, s->drank_wpre, s->drank_cpre, false);
      k_rank_chunks<<<1, 1024, 0, st>>>(s->drank_cpre, chunks, nullptr);
      rank_pack(s, words);
      k_dense_open<<<grid_for(nact, 256, 16384), 256, 0, st>>>(s->act[0], s->cnt + C_ACT, s->dvtx, s->dlab,
                                                               s->dpar, s->dbest, s->cnt + C_NDENSE);
    }
    s->rank_ready = false;
    const ArcBuf &Y = s->buf[s->cur];
    SegView in{Y.seg_start, Y.seg_prefix, s->cur_nseg};
    if (s->cur_arcs)
      k_relabel_dense<<<grid_for(s->cur_arcs, ARCS_PER_BLOCK, SEG_G), BLOCK, 0, st>>>(Y.src, Y.dst, in, dense_rank_of(s));
  }
  GHS_HIP_CHECK(hipGetLastError());
  s->vlab = s->lab; s->vpar = s->par; s->vbest = s->best;
  s->lab = s->dlab; s->par = s->dpar; s->best = s->dbest;
  s->level_dense = true;
  s->dense_n = nact;
  s->act_ident = true;  // round 0: every dense fragment 0..nact0-1 (count C_NDENSE)
  return GHS_OK;
}

static int dense_close(ghs_solver *s) {
  if (!s->level_dense) return GHS_OK;
  // the vertex labels are read only by a later level's open (k_resolve, the passes' label
  // gathers): after the plan's last level nothing reads them, so its close writes none (R-MAT
  // s26 x 8 ranks: level 1's close, ~0.2 ms per rank)
  (void)plan_sync(s);
  const bool last = s->level + 2 >= s->thresholds.size();
  if (!last || s->check_totals) {
    KT(GHS_K_DENSE, s->dense_n);
    k_dense_close<<<grid_for(s->dense_n, 256, 16384), 256, 0, s->stream>>>(s->dvtx, s->cnt + C_NDENSE, s->dlab, s->vlab,
                                                                           s->cnt + C_ERR, !last);
  }
  GHS_HIP_CHECK(hipGetLastError());
  s->lab = s->vlab; s->par = s->vpar; s->best = s->vbest;
  s->level_dense = false;
  return GHS_OK;
}

// ---- second half of opening a level: the active list and the one host sync ------------------
// The active fragments are those with an edge in this level — on a multi-rank solve, on ANY rank
// (the flags were OR-combined by the caller), so every rank selects the same list in the same
// order and the all-reduce slots line up.
static int dense_open(ghs_solver *s);
static int open_level_finish(ghs_solver *s) {
  hipStream_t st = s->stream;
  const uint32_t lv = s->level;
  const bool first = (lv == 0);
  if (int rc = plan_sync(s)) return rc;
  const uint64_t w_hi = s->thresholds[lv + 1];
  const unsigned G = s->open_G;
  if (s->pending_exchange) {  // several ranks: the combined error byte (any rank's error)
    k_flag_to_err<<<1, 1, 0, st>>>(s->flags + s->n, s->cnt + C_ERR);
    GHS_HIP_CHECK(hipGetLastError());
  }
  s->pending_exchange = false;
  const bool from_words = s->words_merged;
  s->words_merged = false;
  if (from_words) {
    // dense levels, bitmap exchange: the rank tables (and the count) from the merged words; the
    // fragment list follows in dense_open
    KT(GHS_K_DENSE, s->n);
    const uint64_t words = ((uint64_t)s->n + 63) / 64;
    const uint32_t chunks = (uint32_t)((words + BLOCK - 1) / BLOCK);
    k_rank_words<<<chunks, BLOCK, 0, st>>>(s->flags, s->n, s->drank_bits, s->drank_wpre, s->drank_cpre, true);
    k_rank_chunks<<<1, 1024, 0, st>>>(s->drank_cpre, chunks, s->cnt + C_ACT);
    rank_pack(s, words);
    GHS_HIP_CHECK(hipGetLastError());
  } else if (int rc = select_lb(s, nullptr, s->cnt + C_N, s->n, s->act[0], s->cnt + C_ACT)) {
    return rc;
  }
  s->rank_ready = from_words;
  s->act_ident = false;
  s->act_cur = 0;
  GHS_HIP_CHECK(hipMemcpyAsync(s->h_cnt, s->cnt, C_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  if (int rc = solver_sync(s)) return rc;
  if (s->h_cnt[C_ERR]) return fail_counters(s, s->h_cnt[C_ERR], "opening a level");
  const uint64_t S = s->h_cnt[C_LIVE];
  s->rem_total = s->h_cnt[C_PENDING];
  s->nact = s->h_cnt[C_ACT];
  if (first) s->select_out = S;
  else if (s->filter_run && !s->filter_out) s->filter_out = S + s->rem_total;
  if (s->debug) {
    uint32_t g[2] = {0, 0};
    (void)hipMemcpy(g, s->giant, 8, hipMemcpyDeviceToHost);
    fprintf(stderr, "[ghs] level %u open: w_hi=%llu level_edges=%llu active=%llu pending_after=%llu giant=%u (%u/2048 sampled)\n",
            lv, (unsigned long long)w_hi, (unsigned long long)S, (unsigned long long)s->nact,
            (unsigned long long)s->rem_total, first ? 0u : g[0], first ? 0u : g[1]);
  }
  s->level_arcs = S;
  if (s->nact == 0) {  // no edge of this level on any rank (every rank sees the same flags)
    s->level_open = false;
    return GHS_OK;
  }
  s->cur = 1;  // the level's edges are Y's G regions (S entries incl. padding)
  s->cur_nseg = G;
  s->cur_arcs = S;
  s->level_nact = s->nact;
  s->level_round = 0;
  s->level_open = true;
  if (s->dense_mode) return dense_open(s);
  return GHS_OK;
}

// ---- single rank: open the level without a host sync ---------------------------------------
// The active list is selected on the device and the level's first round is enqueued right
// behind it; the level's counts (edges, active fragments, pending edges, errors) come back with
// that round's report (run_level_pipelined). Until then the grids are sized for the bounds
// (n fragments, the streaming grid for the edges). An empty level runs one no-op round.
static int open_level_async(ghs_solver *s) {
  if (s->open_ident) {
    s->act_ident = true;  // every vertex (count C_N); see open_level
  } else {
    if (int rc = select_lb(s, nullptr, s->cnt + C_N, s->n, s->act[0], s->cnt + C_ACT)) return rc;
    s->act_ident = false;
  }
  s->act_cur = 0;
  s->nact = s->n;  // bound
  s->level_nact = s->n;
  s->cur = 1;
  s->cur_nseg = s->open_G;
  s->cur_arcs = 0;
  s->arcs_known = false;
  s->open_async = true;
  s->level_round = 0;
  s->level_open = true;
  return GHS_OK;
}

static inline unsigned long long *act_count(ghs_solver *s, int which) { return s->cnt + C_ACT + which; }
static inline const unsigned long long *cur_act_count(ghs_solver *s) {
  return s->act_ident ? s->cnt + (s->level_dense ? C_NDENSE : C_N) : act_count(s, s->act_cur);
}

// the pending region scan as its own launch (when no hook kernel follows to carry it)
static void flush_scan(ghs_solver *s) {
  KT(GHS_K_SCAN, s->cmp_g);
  k_scan_counts<<<1, 1024, 0, s->stream>>>(s->scan_buf->seg_count, s->cmp_g, s->scan_buf->seg_prefix, s->cnt + C_LIVE);
  s->scan_pending = false;
}

// ---- one round, enqueued without a host sync (sizes on the device; s->nact is a bound) --------
// Bucketed rounds (k_bucket + k_bmin, one rank): level 0's rounds while the host's bound on the
// active fragments is at least BUCKET_MIN_ACTIVE. Past level 0 a giant fragment exists, and its
// bucket's records all land on one k_bmin workgroup (16384^2 grid, level 1 round 0: k_bmin 10.0
// ms vs 5.6 ms for the atomic min-edge + CONNECT); below the bound large fragments do the same
// (the grid's level-0 rounds 4 and 5: 0.84 / 0.52 ms vs 0.55 / 0.17 ms), and the min-edge kernel's
// LDS cache of fragment minima absorbs their candidates anyway.
#ifndef GHS_BUCKET_MIN_ACTIVE
#define GHS_BUCKET_MIN_ACTIVE (1u << 23)
#endif
constexpr uint64_t BUCKET_MIN_ACTIVE = GHS_BUCKET_MIN_ACTIVE;
// a lattice-like solve also buckets the first round of every later level (the hot fragments
// excluded). Off: on the 16384^2 grid level 0 stops at the bond-percolation point, so level 1 has
// many large fragments below the hot list's size threshold, each filling one bucket (grid step
// 43.6 -> 48.3 ms, gradient grid 18.8 -> 20.5 ms, same box; profiles/r03/hot2).
#ifndef GHS_BK_LEVEL_FIRST
#define GHS_BK_LEVEL_FIRST 0
#endif
constexpr bool BK_LEVEL_FIRST = GHS_BK_LEVEL_FIRST;
// k_jump_ident's grid cap on lattice-like solves. Path-splitting walks on long hook chains (the
// gradient grid's columns) duplicate each other's work when too many start at once: the gradient
// grid's level-0 jump took 1.8 ms at 2048 blocks and 3.6 ms at 16384; random graphs (short
// chains) want every walk in flight (R-MAT s24 bucketed rounds: 0.46 ms at 2048 blocks, 0.34 at
// 16384).
#ifndef GHS_JUMP_LATTICE_G
#define GHS_JUMP_LATTICE_G 2048
#endif
constexpr unsigned JUMP_LATTICE_G = GHS_JUMP_LATTICE_G;
// a random-like graph's level 0 round 0 bucketed too (1) or by the a-run seeding + atomic min-edge +
// k_win (0). Level 0 has no giant to reduce, so nearly every edge becomes two records in random
// buckets, each a scattered 16-B store: R-MAT s26 round 0 2.56 ms bucketed vs 2.37 ms (s24 0.50
// vs 0.52 ms), same box (profiles/r03/l0ab).
#ifndef GHS_BK_RANDOM_L0
#define GHS_BK_RANDOM_L0 0
#endif
constexpr bool BK_RANDOM_L0 = GHS_BK_RANDOM_L0;

// hot != nullptr (a level's first round past level 0: the hot list of k_giant): the hot fragments'
// candidates are reduced by k_bucket into best[]; k_hot_hook then hooks them like k_bmin hooks a
// bucket's targets
static void enqueue_bmin(ghs_solver *s, const uint32_t *a, const uint32_t *b, const uint64_t *k, SegView in,
                         const unsigned long long *guard, uint64_t items, const uint32_t *hot,
                         const unsigned long long *only_if = nullptr, bool full = false) {
  {
    KT(GHS_K_BUCKET, items);
    k_bucket<<<BK_G, BK_T, 0, s->stream>>>(a, b, k, in, s->bk_bs, s->bk_nb, s->rec, s->bk_off, guard, hot, s->best,
                                         only_if);
  }
  {
    KT(GHS_K_BMIN, items);
    if (full) {  // level 0's windowed round falling back: every vertex's best / par written
      if (s->bk_bs == 13)
        k_bmin<13, true><<<s->bk_nb, BM_T, 0, s->stream>>>(s->rec, s->bk_off, in, s->par, s->best, s->in_mst, guard,
                                                           only_if, s->n);
      else
        k_bmin<14, true><<<s->bk_nb, BM_T, 0, s->stream>>>(s->rec, s->bk_off, in, s->par, s->best, s->in_mst, guard,
                                                           only_if, s->n);
    } else if (s->bk_bs == 13) {
      k_bmin<13><<<s->bk_nb, BM_T, 0, s->stream>>>(s->rec, s->bk_off, in, s->par, s->best, s->in_mst, guard, only_if);
    } else {
      k_bmin<14><<<s->bk_nb, BM_T, 0, s->stream>>>(s->rec, s->bk_off, in, s->par, s->best, s->in_mst, guard, only_if);
    }
  }
  if (hot) {
    KT(GHS_K_HOT_HOOK, 0);
    k_hot_hook<<<1, HOT_K, 0, s->stream>>>(hot, s->best, ends_of(s), s->lab, s->par, s->in_mst, s->cnt + C_ERR);
  }
}

static int enqueue_state_init(ghs_solver *s);

// the identity labels, unless already written (solver_begin leaves them to level 0's round 0)
static void ensure_lab(ghs_solver *s) {
  if (!s->lab_lazy) return;
  s->lab_lazy = false;
  k_iota<<<grid_for(s->n, 256, 8192), 256, 0, s->stream>>>(s->lab, s->n);
}

static int enqueue_minedge(ghs_solver *s) {
  const bool timed = s->detail || (s->time_rounds && s->level_round >= 1);
  if (timed) record(s, 0);
  if (s->level != 0 || s->level_round != 0) ensure_lab(s);  // round 0 of level 0 reads no label
  const ArcBuf &I = s->buf[s->cur];
  ArcBuf &O = s->buf[s->cur ^ 1];
  SegView in{I.seg_start, I.seg_prefix, s->cur_nseg};
  // GHS_OPT_BUCKETED (forced) runs every round bucketed: the test suite's coverage of them
  s->round_bucketed = s->bucketed && (s->bucket_first_only ? (s->level_round == 0 && (BK_RANDOM_L0 || s->level > 0))
                                      : ((s->level == 0 && s->nact >= BUCKET_MIN_ACTIVE) ||
                                         (BK_LEVEL_FIRST && s->level > 0 && s->level_round == 0) ||
                                         (s->cfg.options & GHS_OPT_BUCKETED)));
  const bool windowed0 = s->level_round == 0 && (s->cur_arcs || !s->arcs_known) && s->round_bucketed &&
                         s->level == 0 && s->lattice && s->windowed;
  if (s->state_init_pending) {
    s->state_init_pending = false;
    if (!windowed0)
      if (int rc = enqueue_state_init(s)) return rc;
  }
  if (s->level_round == 0) {
    if (s->cur_arcs || !s->arcs_known) {
      const unsigned g = s->arcs_known ? grid_for(s->cur_arcs, ARCS_PER_BLOCK, s->ident_g) : s->ident_g;
      const uint64_t items = s->arcs_known ? s->cur_arcs : 0;
      if (windowed0) {
        s->windowed_enq = true;
        // windowed round 0 (k_wmin over the edge list); k_bucket / k_bmin run instead only if a
        // level-0 edge spans more than one bucket (k_select's flag)
        const unsigned long long *far = s->cnt + C_LONG;
        {
          KT(GHS_K_WSTARTS, s->bk_nb);
          uint32_t *F = reinterpret_cast<uint32_t *>(s->wstart + s->bk_nb + 1);  // region-first table
          k_wfirst<<<1, WF_T, 0, s->stream>>>(in, I.src, F, far);
          k_wstarts<<<(s->bk_nb + 1 + 255) / 256, 256, 0, s->stream>>>(in, I.src, F, s->bk_bs, s->bk_nb, s->wstart, far);
        }
        {
          KT(GHS_K_WMIN, items);
          const unsigned wg = 8 * WM_CHUNK * ((s->bk_nb + 8 * WM_CHUNK - 1) / (8 * WM_CHUNK));
          if (s->bk_bs == 13)
            k_wmin<13><<<wg, BM_T, 0, s->stream>>>(I.src, I.dst, I.key, in, s->bk_nb, s->wstart, s->par, s->best,
                                                  s->in_mst, far, s->n, WM_GATHER ? s->eu : nullptr, s->ev);
          else
            k_wmin<14><<<wg, BM_T, 0, s->stream>>>(I.src, I.dst, I.key, in, s->bk_nb, s->wstart, s->par, s->best,
                                                  s->in_mst, far, s->n, WM_GATHER ? s->eu : nullptr, s->ev);
        }
        enqueue_bmin(s, I.src, I.dst, I.key, in, nullptr, items, nullptr, far, true);
      } else if (s->round_bucketed) {
        // the level's edges carry roots (past level 0: resolved, and the giant is one of them)
        enqueue_bmin(s, I.src, I.dst, I.key, in, nullptr, items, s->level > 0 ? s->giant + GIANT_HOT : nullptr);
      } else {
        // level 0 (labels are the vertices): a-side runs seeded first, mostly by plain stores
        const bool seed = s->level == 0 && s->seed_runs;
        if (seed) {
          KT(GHS_K_SEED_RUNS, items);
          k_seed_runs<<<g, BLOCK, 0, s->stream>>>(I.src, I.key, in, s->best);
        }
        KT(GHS_K_MINEDGE_IDENT, items);
        k_minedge<true, false><<<g, BLOCK, 0, s->stream>>>(I.src, I.dst, I.key, in, s->lab, s->best, nullptr, nullptr,
                                                           nullptr, nullptr, nullptr, !seed, nullptr);
      }
    }
  } else if (s->round_bucketed) {
    // relabel + drop intra-fragment edges (no candidates), scan the survivors' regions, bucket them
    const unsigned long long *guard = cur_act_count(s);
    {
      KT(GHS_K_MINEDGE_COMPACT, 0);
      k_minedge<false, true, false, false><<<s->cmp_g, BLOCK, 0, s->stream>>>(
          I.src, I.dst, I.key, in, s->lab, s->best, O.src, O.dst, O.key, O.seg_start, O.seg_count, false, guard);
    }
    s->scan_pending = true;
    s->scan_buf = &O;
    flush_scan(s);
    SegView oin{O.seg_start, O.seg_prefix, s->cmp_g};
    enqueue_bmin(s, O.src, O.dst, O.key, oin, guard, 0, nullptr, nullptr);
  } else {
    // fixed grid: every one of the seg_g blocks writes its region's count
    KT(GHS_K_MINEDGE_COMPACT, 0);
    // a round that starts with <= 1 active fragment is a discarded lookahead round (one rank, or the
    // pipelined rounds of several): it streams nothing
    const unsigned long long *guard = cur_act_count(s);
    if (s->dedup_max && s->nact <= DEDUP_BOUND_FACTOR * s->dedup_max)  // few fragments left: the parallel-edge filter
      k_minedge<false, true, true><<<s->cmp_g, BLOCK, 0, s->stream>>>(I.src, I.dst, I.key, in, s->lab, s->best, O.src,
                                                                 O.dst, O.key, O.seg_start, O.seg_count, true, guard,
                                                                 cur_act_count(s), s->dedup_max);
    else
      k_minedge<false, true><<<s->cmp_g, BLOCK, 0, s->stream>>>(I.src, I.dst, I.key, in, s->lab, s->best, O.src, O.dst,
                                                            O.key, O.seg_start, O.seg_count, true, guard);
    // the regions' prefix scan is left to the round's hook kernel (or a scan launch before the
    // next consumer): s->scan_pending
    s->scan_pending = true;
    s->scan_buf = &O;
  }
  GHS_HIP_CHECK(hipGetLastError());
  if (timed) record(s, 1);
  return GHS_OK;
}

// slot != nullptr: the round's last kernel reports (live, active, edges, err, seq) to it
static int enqueue_contract(ghs_solver *s, RoundSlot *slot = nullptr, unsigned long long seq = 0) {
  if (s->rs_fold) {  // the reduce-scatter round's totals, summed over the ranks by the caller
    k_fold_partial<<<1, 1, 0, s->stream>>>(s->cnt);
    GHS_HIP_CHECK(hipGetLastError());
    s->rs_fold = false;
  }
  const uint32_t *act = s->act_ident ? nullptr : s->act[s->act_cur];
  const unsigned long long *d_nact = cur_act_count(s);
  const uint64_t bound = s->nact;
  const int nb = s->act_ident ? 0 : (s->act_cur ^ 1);
  if (bound) {
    const unsigned g = grid_for(bound, BLOCK, 16384);  // grid-stride beyond 4M fragments
    // the hook kernels end with one pair of same-address atomics per block (the totals), which
    // serialise at ~12 ns each: at most HOOK_G blocks (16384 blocks cost ~0.4 ms in atomics)
    const unsigned gh = grid_for(bound, BLOCK, HOOK_G);
    // CONNECT: edge form while fragments are many and small (a level's first round: its edges
    // carry the current roots), fragment form otherwise (and always with several ranks: a
    // fragment's best edge may live on another rank)
    const bool edge_form =
        s->cfg.num_ranks <= 1 && s->level_round == 0 && (!s->arcs_known || s->cur_arcs < 8 * bound);
    if (edge_form && s->scan_pending) flush_scan(s);
    const bool dual = !edge_form && s->cfg.num_ranks <= 1 && s->level_round >= 1 && bound >= EDGE_HOOK_MIN_BOUND;
    // lab stays uninitialised only into the identity jump of a round whose hooks read no label
    const bool ident_jump = s->act_ident && (s->cfg.num_ranks <= 1 || s->level_dense);
    if (!(ident_jump && s->level == 0 && s->level_round == 0 && (s->round_bucketed || edge_form))) ensure_lab(s);
    if (s->round_bucketed) {
      // k_bmin hooked every fragment that has an outgoing edge; the jump resolves the mutual
      // pairs and counts the hooks
      if (s->scan_pending) flush_scan(s);
    } else if (s->hooked) {
      // multi-rank: par / in_mst / totals already written by ghs_solver_unpack_hook
      if (s->scan_pending) flush_scan(s);
    } else if (edge_form) {
      const ArcBuf &I = s->buf[s->cur];
      SegView in{I.seg_start, I.seg_prefix, s->cur_nseg};
      KT(GHS_K_WIN, s->arcs_known ? s->cur_arcs : 0);
      k_win<<<s->arcs_known ? grid_for(s->cur_arcs, ARCS_PER_BLOCK, s->win_g) : s->win_g, BLOCK, 0, s->stream>>>(I.src, I.dst, I.key, in, s->best,
                                                                                   s->par, s->in_mst, s->cnt + C_WEIGHT, nullptr);
    } else if (dual) {
      // this round's compaction output (the survivors, relabelled to the current roots)
      if (s->scan_pending) flush_scan(s);
      const ArcBuf &O = s->buf[s->cur ^ 1];
      SegView in{O.seg_start, O.seg_prefix, s->cmp_g};
      {
        KT(GHS_K_WIN, 0);
        k_win<<<s->win_g, BLOCK, 0, s->stream>>>(O.src, O.dst, O.key, in, s->best, s->par, s->in_mst, s->cnt + C_WEIGHT,
                                                 d_nact);
      }
      GHS_HIP_CHECK(hipGetLastError());
      KT(GHS_K_HOOK, 0);
      k_hook<<<gh, BLOCK, 0, s->stream>>>(act, d_nact, s->best, s->lab, ends_of(s), s->par, s->in_mst,
                                         s->cnt + C_WEIGHT, s->cnt + C_ERR, nullptr, 0, nullptr, nullptr, false,
                                         s->cnt + C_LIVE, (uint32_t)s->e_lo, (uint32_t)s->e_hi, nullptr, DenseRank());
    } else {
      const ArcBuf *sb = s->scan_pending ? s->scan_buf : nullptr;
      KT(GHS_K_HOOK, 0);
      k_hook<<<gh, BLOCK, 0, s->stream>>>(act, d_nact, s->best, s->lab, ends_of(s), s->par, s->in_mst,
                                         s->cnt + C_WEIGHT, s->cnt + C_ERR, sb ? sb->seg_count : nullptr, s->cmp_g,
                                         sb ? sb->seg_prefix : nullptr, s->cnt + C_LIVE, s->level_round == 0, nullptr,
                                         (uint32_t)s->e_lo, (uint32_t)s->e_hi, s->level_dense ? s->vlab : nullptr,
                                         s->level_dense ? dense_rank_of(s) : DenseRank());
      s->scan_pending = false;
    }
    GHS_HIP_CHECK(hipGetLastError());
    if (s->detail) record(s, 2);
    // Stage 3, then the next active list (one launch each)
    // a bucketed round's hooks are counted by the jump: its grid is capped (one pair of
    // same-address atomics per block)
    unsigned long long *acc = s->round_bucketed ? s->hook_acc : nullptr;
    if (s->act_ident && (s->cfg.num_ranks <= 1 || s->level_dense)) {
      const uint32_t ni = s->level_dense ? (uint32_t)s->dense_n : s->n;
      KT(GHS_K_JUMP_IDENT, ni);
      k_jump_ident<<<grid_for(((uint64_t)ni + 3) / 4, BLOCK, s->jump_ident_g), BLOCK, 0, s->stream>>>(
          ni, s->par, s->lab, s->best, s->flags, s->cnt + C_ERR, acc, s->lab_lazy);
      s->lab_lazy = false;
    } else {
      KT(GHS_K_JUMP, 0);
      k_jump<<<g, BLOCK, 0, s->stream>>>(act, d_nact, s->par, s->lab, s->best, s->flags, s->cnt + C_ERR, acc);
    }
    GHS_HIP_CHECK(hipGetLastError());
    if (s->detail) record(s, 3);
    if (int rc = select_lb(s, act, d_nact, bound, s->act[nb], act_count(s, nb), slot, seq, acc != nullptr)) return rc;
  } else {
    if (s->scan_pending) flush_scan(s);
    if (int rc = select_lb(s, act, d_nact, 0, s->act[nb], act_count(s, nb), slot, seq)) return rc;
  }
  if (s->detail) record(s, 4);
  return GHS_OK;
}

// spin until the round report with this seq has landed in the pinned slot and its fields match
// its checksum, and copy it to *out (the stream keeps running); a failed or drained stream without
// the report is an error, never a hang. The stream is queried only after SLOT_QUIET_MS of waiting:
// hipStreamQuery enqueues a marker behind the last launch, and its system-scope release idled the
// GPU ~5.6 us before every round >= 2.
constexpr int SLOT_QUIET_MS = 20;
constexpr int SLOT_QUERY_MS = 5;

// one read of the slot: true when seq is the expected one and the fields hash to the checksum
static bool slot_read(const RoundSlot *hs, unsigned long long seq, RoundSlot *out) {
  if (__atomic_load_n(&hs->seq, __ATOMIC_ACQUIRE) != seq) return false;
  RoundSlot r;
  r.live_out = __atomic_load_n(&hs->live_out, __ATOMIC_ACQUIRE);
  r.nact_out = __atomic_load_n(&hs->nact_out, __ATOMIC_ACQUIRE);
  r.edges = __atomic_load_n(&hs->edges, __ATOMIC_ACQUIRE);
  r.err = __atomic_load_n(&hs->err, __ATOMIC_ACQUIRE);
  r.nact_in = __atomic_load_n(&hs->nact_in, __ATOMIC_ACQUIRE);
  r.pending = __atomic_load_n(&hs->pending, __ATOMIC_ACQUIRE);
  r.weight = __atomic_load_n(&hs->weight, __ATOMIC_ACQUIRE);
  r.chk = __atomic_load_n(&hs->chk, __ATOMIC_ACQUIRE);
  r.seq = seq;
  if (r.chk != slot_checksum(seq, r.live_out, r.nact_out, r.edges, r.err, r.nact_in, r.pending, r.weight)) return false;
  *out = r;
  return true;
}

static uint64_t g_slot_retries = 0;  // reads whose seq had landed before every field did (diagnostic)

static int wait_slot(ghs_solver *s, const RoundSlot *hs, unsigned long long seq, RoundSlot *out) {
  if (slot_read(hs, seq, out)) return GHS_OK;
  const auto t0 = std::chrono::steady_clock::now();
  unsigned spins = 0;
  bool quiet = true;
  auto last_query = t0;
  bool retried = false;  // the report's seq landed before a field: counted once per report
  while (!slot_read(hs, seq, out)) {
    if (!retried && __atomic_load_n(&hs->seq, __ATOMIC_RELAXED) == seq) {
      retried = true;
      __atomic_fetch_add(&g_slot_retries, 1, __ATOMIC_RELAXED);
    }
    if ((spins & 255) == 0 && solver_cancelled(s)) GHS_FAIL(GHS_E_STATE, "cancelled: another rank of the solve failed");
    if ((++spins & 255) == 0 && quiet)
      quiet = std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(SLOT_QUIET_MS);
    if (!quiet) {
      // a long wait (a multi-rank solve's peers share the device, or the stream failed): sleep
      // between polls and query the stream only every SLOT_QUERY_MS — each query enqueues a marker
      // whose system-scope release idles the GPU, and 8 emulated rank threads querying every 50 us
      // fed back into ever longer waits (emulated s26 x8 solves of 3-6 s instead of ~80 ms)
      std::this_thread::sleep_for(std::chrono::microseconds(50));
      const auto now = std::chrono::steady_clock::now();
      if (now - last_query >= std::chrono::milliseconds(SLOT_QUERY_MS)) {
        last_query = now;
        const hipError_t q = hipStreamQuery(s->stream);
        if (q != hipSuccess && q != hipErrorNotReady) GHS_HIP_CHECK(q);
        if (q == hipSuccess && !slot_read(hs, seq, out)) {
          if (__atomic_load_n(&hs->seq, __ATOMIC_ACQUIRE) == seq)
            GHS_FAIL(GHS_E_STATE, "round report fails its checksum after the stream drained");
          GHS_FAIL(GHS_E_STATE, "round report missing after the stream drained");
        }
      }
    }
  }
  return GHS_OK;
}

// host-side bookkeeping after a round was enqueued (buffers / lists flip; no device values)
static void advance_round(ghs_solver *s) {
  if (s->level_round >= 1) {  // this round's min-edge kernel compacted into the other buffer
    s->cur ^= 1;
    s->cur_nseg = s->cmp_g;
  }
  s->act_cur = s->act_ident ? 0 : (s->act_cur ^ 1);
  s->act_ident = false;
  s->round += 1;
  s->level_round += 1;
}

static void push_stats(ghs_solver *s, uint32_t level_round, uint64_t live_in, uint64_t nact_in, uint64_t edges_total) {
  ghs_round_stats_t st{};
  st.level = s->level;
  st.level_arcs = level_round == 0 ? s->level_arcs : 0;
  st.live_arcs = live_in;
  st.active_components = nact_in;
  s->last_nact_in = nact_in;
  st.hooks = edges_total - s->edges_before;
  s->edges_before = edges_total;
  s->stats.push_back(st);
}

// GHS_OPT_CHECK_TOTALS: the device counters behind the level's last kernel (a stream-ordered copy)
// against the totals of the level's last report (the trailing lookahead rounds change no counter)
static int check_level_totals(ghs_solver *s) {
  if (!s->check_totals || !s->report_final) return GHS_OK;
  GHS_HIP_CHECK(hipMemcpyAsync(s->h_cnt, s->cnt, C_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, s->stream));
  if (int rc = solver_sync(s)) return rc;
  if (s->h_cnt[C_WEIGHT] != s->rep_weight || s->h_cnt[C_EDGES] != s->rep_edges)
    GHS_FAIL(GHS_E_STATE, "level " + std::to_string(s->level) + ": report totals (" + std::to_string(s->rep_weight) + ", " +
                              std::to_string(s->rep_edges) + ") differ from the device counters (" +
                              std::to_string(s->h_cnt[C_WEIGHT]) + ", " + std::to_string(s->h_cnt[C_EDGES]) + ")");
  ++s->totals_checked;
  return GHS_OK;
}

static void close_level(ghs_solver *s) {
  ensure_lab(s);  // a level 0 without rounds
  s->level_open = false;
  s->level += 1;
  (void)plan_sync(s);  // on failure thresholds stay empty: no further level
  const bool no_more =
      (s->level + 1 >= s->thresholds.size()) || (s->cfg.num_ranks <= 1 && s->pending_built && s->rem_total == 0);
  s->phase = no_more ? 2 : 0;
}

// ---- single-rank level loop: rounds are enqueued LOOKAHEAD ahead of the termination check ------
// Each round copies (live, active, edges, err) to a pinned slot behind an event; the host waits
// only for the round LOOKAHEAD back. Rounds past the last are no-ops on the device (zero active
// fragments, zero live inter-fragment edges) and are discarded.
// Bucketed rounds or not, once per solve (one rank): the plan's locality flag. The host waits for
// the plan copy here — k_sample_weights / k_plan run first on the stream, so the wait overlaps the
// first canonical pass already enqueued behind them.
static int decide_bucketed(ghs_solver *s) {
  s->bucket_decided = true;
  s->bucketed = false;
  s->bucket_first_only = false;
  s->lattice = false;
  s->jump_ident_g = 16384;
  const uint32_t opt = s->cfg.options;
  if (s->cfg.num_ranks > 1 || !s->rec || (opt & GHS_OPT_NO_BUCKETED)) return GHS_OK;
  if (opt & GHS_OPT_BUCKETED) {
    s->bucketed = true;
    return GHS_OK;
  }
  if (int rc = plan_sync(s)) return rc;
  s->lattice = s->h_thr[PLAN_LOCAL] != 0;
  if (s->lattice) s->jump_ident_g = JUMP_LATTICE_G;
  // lattice-like: level 0's rounds while >= BUCKET_MIN_ACTIVE fragments; otherwise (or forced by
  // GHS_OPT_BUCKETED_FIRST) the first round of every level
  s->bucketed = true;
  s->bucket_first_only = !s->lattice || (opt & GHS_OPT_BUCKETED_FIRST);
  return GHS_OK;
}


// ---- the LDS tail: the rest of a level once its active fragments fit LDS (one rank) ---------
// Enters at a round >= 1 of a level whose exact active count is in [2, TAIL_MAX] (the host has
// read every earlier report); enqueues batches of tail rounds (k_tail_round + k_tail_hook, no-ops
// once the level is done) behind k_tail_map + k_tail_open, each batch ending with a copy of the
// control block and its report; reads the tail's per-round stats from that copy and closes the
// level. Rounds whose launches follow the finishing round exit at once.
// Tail rounds per batch: the first batch is sized from the level's last observed contraction.
// F0 fragments shrinking by `decay` per round leave <= 1 root after L = log_decay(F0) rounds of
// hooks (the open's included), so k_tail_round r = ceil(L) is the finishing one and the batch holds
// exactly the launches the level needs. The contraction slows inside a level (R-MAT s24 level 0:
// 26x, 19x, 10x, 10x), so half a round of margin — none when the open's hooks alone are expected to
// finish (F0 <= decay): R-MAT s24 levels 0 and 1 and both tails of the 16384^2 grid then launch no
// round past the finishing one (profiles/r06/rounds_*.txt). An underestimate costs one more batch.
constexpr uint32_t TAIL_BATCH_MIN = 1, TAIL_BATCH_MAX = 8;

static uint32_t tail_first_batch(uint64_t F0, uint64_t prev_in) {
  const double decay = std::max(2.0, prev_in > F0 ? (double)prev_in / (double)F0 : 2.0);
  const double L = std::log((double)F0) / std::log(decay);
  const double est = (double)F0 <= decay ? 1.0 : std::ceil(L + 0.5);
  return (uint32_t)std::min<double>(TAIL_BATCH_MAX, std::max<double>(TAIL_BATCH_MIN, est));
}
constexpr uint64_t TAIL_TRY = 32ull * TAIL_MAX;  // a bound below this: read the exact count first

static bool tail_usable(const ghs_solver *s) {
  return s->tail_on && s->tail.ctl && s->cfg.num_ranks <= 1 && !s->level_dense && s->level_round >= 1 &&
         !s->act_ident;
}

// map + labels + open (round 0's stream of the tail)
static void tail_start(ghs_solver *s, TailRun &t, bool multi) {
  hipStream_t st = s->stream;
  ensure_lab(s);
  t.tb = s->tail;
  const ArcBuf &I = s->buf[s->cur], &O = s->buf[s->cur ^ 1];
  t.tb.rec = O.src;  // the idle edge buffer holds the tail's records
  t.tb.rkey = O.key;
  if (s->scan_pending) flush_scan(s);
  t.act0 = s->act[s->act_cur];
  const unsigned long long *d_nact = cur_act_count(s);
  SegView in{I.seg_start, I.seg_prefix, s->cur_nseg};
  t.F0 = (uint32_t)s->nact;
  t.hook_g = (t.F0 + TAIL_HS - 1) / TAIL_HS;
  t.round0 = s->round;
  t.lr0 = s->level_round;
  t.r = 1;
  t.multi = multi;
  KT(GHS_K_TAIL_OPEN, s->arcs_known ? s->cur_arcs : 0);
  k_tail_map<<<grid_for(t.F0, 256, 64), 256, 0, st>>>(t.act0, d_nact, t.tb);
  // the labels the edges carry: the previous round's list (after the level's identity round 0:
  // every vertex; a dense level's: every dense label)
  const bool prev_ident = t.lr0 == 1;
  const uint32_t *prev = prev_ident ? nullptr : s->act[s->act_cur ^ 1];
  const unsigned long long *d_nprev =
      prev_ident ? s->cnt + (s->level_dense ? C_NDENSE : C_N) : act_count(s, s->act_cur ^ 1);
  const uint64_t nprev_bound = prev_ident ? (s->level_dense ? s->dense_n : s->n) : s->level_nact;
  k_tail_labels<<<grid_for(nprev_bound, 256, 8192), 256, 0, st>>>(prev, d_nprev, s->lab, t.tb);
  k_tail_open<<<TAIL_G, TAIL_T, 0, st>>>(I.src, I.dst, I.key, in, t.tb, s->check_totals);
}

// round rr's hooks: every root's minimum over the blocks' rows (several ranks: this rank's own,
// agreed by tail_agree between the caller's two all-reduces)
static int tail_hook_local(ghs_solver *s, const TailRun &t, uint32_t rr) {
  s->round = t.round0 + rr;  // the profile's round index: the round whose stream they reduce
  KT(GHS_K_TAIL_HOOK, rr ? 0 : t.F0);
  k_tail_hook<<<t.hook_g, 256, 0, s->stream>>>(t.tb, rr, s->in_mst, TAIL_G, s->cnt + C_ERR, t.multi);
  GHS_HIP_CHECK(hipGetLastError());
  return GHS_OK;
}

static int tail_agree(ghs_solver *s, const TailRun &t, uint32_t rr) {
  s->round = t.round0 + rr;
  KT(GHS_K_TAIL_HOOK, 0);
  k_tail_xhook<<<t.hook_g, 256, 0, s->stream>>>(t.tb, rr, s->in_mst, (uint32_t)s->e_lo, (uint32_t)s->e_hi);
  GHS_HIP_CHECK(hipGetLastError());
  return GHS_OK;
}

static int tail_round_launch(ghs_solver *s, const TailRun &t, uint32_t r) {
  s->round = t.round0 + r;
  KT(GHS_K_TAIL_ROUND, 0);
  k_tail_round<<<TAIL_G, TAIL_T, 0, s->stream>>>(t.tb, r, t.act0, s->lab, s->cnt, s->cnt + C_ERR);
  GHS_HIP_CHECK(hipGetLastError());
  return GHS_OK;
}

// the control block (and the report, checksummed) behind the tail's launches so far: *nact_out = 0
// once the level is done
static int tail_report(ghs_solver *s, const TailRun &t, uint32_t last, unsigned long long *nact_out) {
  hipStream_t st = s->stream;
  const unsigned long long seq = ++s->res->seq;
  RoundSlot *dslot = &s->d_slot[seq % SLOT_RING];
  GHS_HIP_CHECK(hipMemcpyAsync(s->res->h_tail, t.tb.ctl, sizeof(TailCtl), hipMemcpyDeviceToHost, st));
  k_tail_report<<<1, 1, 0, st>>>(t.tb, last, dslot, seq, s->cnt);
  GHS_HIP_CHECK(hipGetLastError());
  RoundSlot rep;
  if (int rc = wait_slot(s, s->h_slot + (seq % SLOT_RING), seq, &rep)) return rc;
  if (slot_err(rep.err)) return fail_counters(s, slot_err(rep.err), "in the LDS tail");
  s->rep_weight = rep.weight;
  s->rep_edges = rep.edges;
  s->report_final = true;
  if (s->debug)
    fprintf(stderr, "[ghs] level %u tail report: nact_out %llu edges %llu weight %llu\n", s->level, rep.nact_out,
            rep.edges, rep.weight);
  *nact_out = rep.nact_out;
  return GHS_OK;
}

// the level is done (the last report read): the tail rounds' stats, then the level's close
static int tail_finish(ghs_solver *s, const TailRun &t) {
  const TailCtl &c = *s->res->h_tail;
  const uint32_t rounds = std::min(c.rounds, TAIL_ROUNDS_MAX);
  for (uint32_t k = 0; k < rounds; ++k) push_stats(s, t.lr0 + k, c.live[k], c.nroots[k], c.edges[k]);
  s->round = t.round0 + rounds;
  s->level_round = t.lr0 + rounds;
  s->tail_ran = true;
  if (s->ev_rec.size() > s->round) s->ev_rec.resize(s->round);
  if (int rc = check_level_totals(s)) return rc;
  if (int rc = dense_close(s)) return rc;
  close_level(s);
  return GHS_OK;
}

// coll != nullptr: one rank of several (a dense level, ghs_solver_tail_multi) — each round's hooks
// agree across the ranks through two small all-reduces (MIN of the F0 keys, MAX of the targets)
static int run_tail(ghs_solver *s, uint64_t prev_in, const GhsTailColl *coll = nullptr) {
  hipStream_t st = s->stream;
  TailRun t;
  tail_start(s, t, coll != nullptr);
  auto hook = [&](uint32_t rr) -> int {
    if (int rc = tail_hook_local(s, t, rr)) return rc;
    if (coll) {
      if (int rc = coll->min_u64(coll->ctx, t.tb.gkey, t.F0, st)) return rc;
      if (int rc = tail_agree(s, t, rr)) return rc;
      if (int rc = coll->max_i32(coll->ctx, reinterpret_cast<int32_t *>(t.tb.ghook), t.F0, st)) return rc;
    }
    return GHS_OK;
  };
  if (int rc = hook(0)) return rc;
  uint32_t batch = tail_first_batch(t.F0, prev_in);
  for (;;) {
    const uint32_t last = std::min(t.r + batch - 1, TAIL_ROUNDS_MAX);  // the batch's last round
    for (; t.r <= last; ++t.r) {
      // round r - 1's hooks, unless the open's (launched above): a batch ends with a round, not with
      // its hook kernel, so the round that finishes the level is not followed by a no-op hook launch
      // when it closes its batch (the hook comes first in the next batch otherwise)
      if (t.r > 1)
        if (int rc = hook(t.r - 1)) return rc;
      if (int rc = tail_round_launch(s, t, t.r)) return rc;
    }
    unsigned long long nact_out = 0;
    if (int rc = tail_report(s, t, last, &nact_out)) return rc;
    if (nact_out <= 1) break;
    if (t.r > TAIL_ROUNDS_MAX) return fail_counters(s, 4, "in the LDS tail (round cap)");
    // the next batch from the batch's last contraction (the report's copy of the control block:
    // nroots[last] = nact_out roots entering round last's stream, nroots[last - 1] before them),
    // sized like the first — R-MAT s26 level 0 (1189 -> 106 -> 14 -> 3 roots) then finishes in a
    // batch of 1 instead of a fixed 3 with two no-op launch pairs
    const TailCtl &c = *s->res->h_tail;
    batch = tail_first_batch(nact_out, last >= 1 ? c.nroots[last - 1] : t.F0);
  }
  return tail_finish(s, t);
}

// The multi-rank loop's LDS tail (ghs_solver_run, multi.hip): at a round >= 1 of a dense level whose
// active count is at most TAIL_MAX, the rounds still in flight are drained (their reports give the
// exact count — every rank reads the same reports, so every rank takes the same branch), then the
// level finishes in run_tail with the ranks' hooks agreed per round. Returns 0 when not applicable,
// 1 when the level finished (in the drain or the tail), 2 when that ended the solve, or an error.
int ghs_solver_tail_multi(ghs_solver *s, const GhsTailColl *coll) {
  if (!s || !coll) return 0;
  if (s->phase != 0 || !s->level_open || s->cfg.num_ranks <= 1 || !s->level_dense || !s->tail_on || !s->tail.ctl ||
      s->act_ident || s->level_round < 1 || s->nact > TAIL_MAX)
    return 0;
  while (!s->pipe.empty()) {  // the rounds in flight (pipelined contract): their reports, in order
    const ghs_solver::PipeRound p = s->pipe.front();
    s->pipe.erase(s->pipe.begin());
    RoundSlot rep;
    if (int rc = wait_slot(s, s->h_slot + (p.seq % SLOT_RING), p.seq, &rep)) return rc;
    if (slot_err(rep.err)) return fail_counters(s, slot_err(rep.err), ("in round " + std::to_string(p.round + 1)).c_str());
    push_stats(s, p.level_round, s->pipe_live, rep.nact_in, rep.edges);
    s->pipe_live = rep.live_out;
    s->pipe_exact = rep.nact_out;
    s->pipe_exact_lr = p.level_round + 1;
    s->nact = rep.nact_out;
    if (rep.nact_out <= 1) {  // the level ended with round p: the rounds enqueued after it are no-ops
      s->pipe.clear();
      s->round = p.round + 1;
      s->level_round = p.level_round + 1;
      if (int rc = dense_close(s)) return rc;
      close_level(s);
      return s->phase == 2 ? 2 : 1;
    }
  }
  if (s->nact < 2) return 0;  // (the synchronous contract closes such a level itself)
  if (int rc = run_tail(s, s->last_nact_in, coll)) return rc;
  return s->phase == 2 ? 2 : 1;
}

static bool tail_step_usable(const ghs_solver *s) {
  return s->phase == 0 && s->level_open && s->cfg.num_ranks > 1 && s->level_dense && s->tail_on && s->tail.ctl &&
         !s->act_ident && s->level_round >= 1 && s->nact >= 2 && s->nact <= TAIL_MAX && s->pipe.empty();
}

extern "C" {

// ---- the stepwise LDS tail (ABI 10; include/ghs_mst.h): the caller's collectives between the calls ----
int ghs_solver_tail_begin(ghs_solver_t *s, uint64_t *num_fragments) {
  if (!s || !num_fragments) GHS_FAIL(GHS_E_ARG, "solver/num_fragments is NULL");
  *num_fragments = 0;
  if (s->tail_step) GHS_FAIL(GHS_E_STATE, "a tail is already in progress");
  if (!tail_step_usable(s)) return GHS_OK;
  s->trun = TailRun();
  tail_start(s, s->trun, true);
  if (int rc = tail_hook_local(s, s->trun, 0)) return rc;
  s->tail_step = true;
  s->phase = 3;  // (minedge / contract refuse until the tail ends)
  *num_fragments = s->trun.F0;
  return GHS_OK;
}

int ghs_solver_tail_buffers(ghs_solver_t *s, uint64_t **d_keys, int32_t **d_hooks) {
  if (!s || !d_keys || !d_hooks) GHS_FAIL(GHS_E_ARG, "solver/keys/hooks is NULL");
  if (!s->tail_step) GHS_FAIL(GHS_E_STATE, "no tail in progress (ghs_solver_tail_begin)");
  *d_keys = s->tail.gkey;
  *d_hooks = reinterpret_cast<int32_t *>(s->tail.ghook);
  return GHS_OK;
}

int ghs_solver_tail_agree(ghs_solver_t *s) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  if (!s->tail_step) GHS_FAIL(GHS_E_STATE, "no tail in progress (ghs_solver_tail_begin)");
  return tail_agree(s, s->trun, s->trun.r - 1);
}

int ghs_solver_tail_round(ghs_solver_t *s, int *state) {
  if (!s || !state) GHS_FAIL(GHS_E_ARG, "solver/state is NULL");
  *state = 0;
  if (!s->tail_step) GHS_FAIL(GHS_E_STATE, "no tail in progress (ghs_solver_tail_begin)");
  TailRun &t = s->trun;
  if (t.r > TAIL_ROUNDS_MAX) {
    s->tail_step = false;
    return fail_counters(s, 4, "in the LDS tail (round cap)");
  }
  if (int rc = tail_round_launch(s, t, t.r)) return rc;
  unsigned long long nact_out = 0;
  if (int rc = tail_report(s, t, t.r, &nact_out)) {
    s->tail_step = false;
    return rc;
  }
  if (nact_out <= 1) {
    s->tail_step = false;
    s->phase = 0;
    if (int rc = tail_finish(s, t)) return rc;
    *state = s->phase == 2 ? 2 : 1;
    return GHS_OK;
  }
  if (int rc = tail_hook_local(s, t, t.r)) return rc;
  ++t.r;
  return GHS_OK;
}

}  // extern "C"


static int run_level_pipelined(ghs_solver *s) {
  if (!s->bucket_decided)
    if (int rc = decide_bucketed(s)) return rc;
  const uint32_t round0 = s->round;
  uint64_t live_prev = s->cur_arcs, nact_prev = s->level_nact;  // inputs of the next checked round
  uint32_t issued = 0, checked = 0;
  uint64_t last_in = s->level_nact;  // the active input of the last checked round
  double decay = 2.0;                 // its contraction (input / output fragments), at least 2
  std::vector<unsigned long long> seqs(LEVEL_ROUND_CAP + s->lookahead + 1);
  for (;;) {
    if (issued < checked + 1 + s->lookahead) {
      // the LDS tail: once the bound on the next round's active fragments is small, read the
      // outstanding reports (the exact count), then finish the level there if it fits
      // (only when the round in flight may leave few enough — predicted with the
      // last checked round's contraction — so a level contracting slowly above TAIL_MAX keeps its
      // lookahead)
      if (issued >= 1 && s->nact <= TAIL_TRY && tail_usable(s)) {
        if (checked < issued && (double)s->nact / decay <= 2.0 * TAIL_MAX) goto check;
        if (checked == issued && s->nact >= 2 && s->nact <= TAIL_MAX) {
          s->round = round0 + issued;
          return run_tail(s, last_in);
        }
      }
      if (issued >= LEVEL_ROUND_CAP) GHS_FAIL(GHS_E_ROUNDCAP, "round cap exceeded in a level");
      const unsigned long long seq = ++s->res->seq;
      seqs[issued] = seq;
      if (int rc = enqueue_minedge(s)) return rc;
      if (int rc = enqueue_contract(s, &s->d_slot[issued % SLOT_RING], seq)) return rc;
      advance_round(s);
      ++issued;
      continue;
    }
  check:
    RoundSlot r;
    if (int rc = wait_slot(s, s->h_slot + (checked % SLOT_RING), seqs[checked], &r)) return rc;
    const unsigned long long span_flag = r.err & SLOT_SPAN;
    r.err = slot_err(r.err);
    s->rep_weight = r.weight;
    s->rep_edges = r.edges;
    s->report_final = true;
    if (s->debug)
      fprintf(stderr, "[ghs] level %u round %u report: nact_in %llu nact_out %llu live_out %llu edges %llu weight %llu\n",
              s->level, checked, r.nact_in, r.nact_out, r.live_out, r.edges, r.weight);
    if (r.err) return fail_counters(s, r.err, ("in round " + std::to_string(round0 + checked + 1)).c_str());
    if (checked == 0 && s->open_async) {  // the level's counts, from its first round
      const uint64_t S = r.live_out;  // round 0 does not compact: its live edges are the level's
      s->open_async = false;
      s->arcs_known = true;
      s->cur_arcs = S;
      s->level_arcs = S;
      s->rem_total = r.pending;
      s->level_nact = r.nact_in;
      live_prev = S;
      nact_prev = r.nact_in;
      if (s->level == 0) s->select_out = S;
      else if (s->filter_run && !s->filter_out) s->filter_out = S + s->rem_total;
      if (s->level == 0 && s->windowed_enq) s->windowed_ran = span_flag == 0;
      if (s->debug) {
        uint32_t g[2] = {0, 0};
        (void)hipMemcpy(g, s->giant, 8, hipMemcpyDeviceToHost);
        fprintf(stderr, "[ghs] level %u open: level_edges=%llu active=%llu pending_after=%llu giant=%u (%u/2048 sampled)\n",
                s->level, (unsigned long long)S, (unsigned long long)r.nact_in, (unsigned long long)s->rem_total,
                s->level ? g[0] : 0u, s->level ? g[1] : 0u);
      }
      if (r.nact_in == 0) break;  // no edge in this level: its rounds were no-ops (checked stays 0)
    }
    push_stats(s, checked, live_prev, nact_prev, r.edges);
    if (r.nact_out) decay = std::max(2.0, (double)nact_prev / (double)r.nact_out);
    last_in = nact_prev;
    // the live edges of round k + 1: round 0 does not compact (its input is read again)
    live_prev = checked == 0 ? live_prev : r.live_out;
    nact_prev = r.nact_out;
    s->nact = r.nact_out;  // tighter bound for the rounds enqueued from here on
    ++checked;
    // level complete after round `checked`: no active fragment left, or one — every remaining
    // level edge then lies inside it (a fragment drops out only with no outgoing edge, so all
    // other fragments of the level were hooked into this tree)
    if (r.nact_out <= 1) break;
  }
  // rounds issued past the last real one were no-ops: rewind the round counter (their events
  // are forgotten and re-recorded by the next level)
  s->round = round0 + checked;
  if (s->ev_rec.size() > s->round) s->ev_rec.resize(s->round);
  if (int rc = check_level_totals(s)) return rc;
  close_level(s);
  return GHS_OK;
}

extern "C" {

int ghs_abi_version(void) { return GHS_MST_ABI_VERSION; }

int ghs_slot_retries(uint64_t *count) {
  if (!count) GHS_FAIL(GHS_E_ARG, "count is NULL");
  *count = __atomic_load_n(&g_slot_retries, __ATOMIC_RELAXED);
  return GHS_OK;
}

int ghs_profile_enable(int on) {
  std::lock_guard<std::mutex> lock(g_prof_mutex);
  g_prof_on = on != 0;
  g_prof.clear();
  return GHS_OK;
}

int ghs_profile_read(ghs_kernel_record_t *out, uint32_t capacity, uint32_t *count) {
  if (!count) GHS_FAIL(GHS_E_ARG, "count is NULL");
  std::lock_guard<std::mutex> lock(g_prof_mutex);
  const uint32_t n = (uint32_t)std::min<size_t>(g_prof.size(), capacity);
  if (n && !out) GHS_FAIL(GHS_E_ARG, "out is NULL");
  for (uint32_t i = 0; i < n; ++i) out[i] = g_prof[i];
  *count = n;
  g_prof.erase(g_prof.begin(), g_prof.begin() + n);
  return GHS_OK;
}

const char *ghs_kernel_name(uint32_t kernel) { return kernel < GHS_K_COUNT ? KERNEL_NAMES[kernel] : "?"; }
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
  return workspace_layout(n, m, local_edges, nullptr, nullptr);
}

// Every vertex a root without a candidate: best = KEY_NONE, par = itself.
static int enqueue_state_init(ghs_solver *s) {
  KT(GHS_K_INIT, s->n);
  hipError_t e;
  if ((e = hipMemsetAsync(s->best, 0xff, (size_t)s->n * 8, s->stream)) != hipSuccess) GHS_FAIL(GHS_E_HIP, std::string("memset best: ") + hipGetErrorString(e));
  k_iota<<<grid_for(s->n, 256, 8192), 256, 0, s->stream>>>(s->par, s->n);  // every root: par[r] == r
  GHS_HIP_CHECK(hipGetLastError());
  return GHS_OK;
}

// The per-solve start of a solver: plan, state arrays, counters (create, and reset between solves).
static int solver_begin(ghs_solver *s) {
  hipError_t e;
  const uint32_t n = s->n;
  s->h_cnt = s->res->h_cnt;
  s->h_slot = s->res->h_slot;
  s->d_slot = s->res->d_slot;
  s->h_sample = s->res->h_sample;
  s->h_thr = reinterpret_cast<uint64_t *>(s->res->h_sample);
  s->t0 = std::chrono::steady_clock::now();
  if (int rc = plan_levels_enqueue(s)) return rc;
  KT(GHS_K_INIT, n);
  if (n) {
    // several ranks with dense levels: every level runs on the dense arrays (k_dense_open sets
    // them up), so the vertex-sized best / par are never read — only lab is (s26: 805 MB of
    // writes per rank saved)
    // one rank: best / par are initialised in front of level 0's first round, or not at all when
    // that round is the windowed one (its kernels write every vertex's slots: grid 3 GB of writes)
    if (!s->dense_mode) {
      if (s->cfg.num_ranks <= 1) {
        s->state_init_pending = true;
      } else if (int rc = enqueue_state_init(s)) {
        return rc;
      }
    }
    // one rank: level 0's round 0 writes every label in its k_jump_ident (nothing reads lab before
    // it); any other first reader initialises it through ensure_lab
    s->lab_lazy = s->cfg.num_ranks <= 1 && !s->dense_mode;
    if (!s->lab_lazy) k_iota<<<grid_for(n, 256, 8192), 256, 0, s->stream>>>(s->lab, n);
  }
  // only the solver's own edge range: it never writes a flag outside [e_lo, e_hi)
  if (s->e_hi > s->e_lo && (e = hipMemsetAsync(s->in_mst + s->e_lo, 0, s->e_hi - s->e_lo, s->stream)) != hipSuccess) GHS_FAIL(GHS_E_HIP, std::string("memset in_mst: ") + hipGetErrorString(e));
  if ((e = hipMemsetAsync(s->lb_state, 0, LB_MAX_TILES * 8, s->stream)) != hipSuccess) GHS_FAIL(GHS_E_HIP, std::string("memset select state: ") + hipGetErrorString(e));
  k_init_counters<<<1, 64, 0, s->stream>>>(s->cnt, n, s->hook_acc);
  if ((e = hipGetLastError()) != hipSuccess) GHS_FAIL(GHS_E_HIP, std::string("init kernels: ") + hipGetErrorString(e));
  s->level = 0;
  s->level_open = false;
  s->phase = n ? 0 : 2;
  return GHS_OK;
}

// pool: the one-shot entry point's process-wide host resources (nullptr: the handle owns its own).
// Passed explicitly, not through a global, so concurrent creators (the multi-rank drivers' threads)
// never adopt another caller's pinned counters.
// d_off != nullptr: CSR input (ABI 9) — the row offsets stream in place of u; d_u may then be NULL
// (gathers of u by edge id search the offsets) or the caller's u (used for those gathers only)
static int solver_create(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_off, const uint32_t *d_v,
                         const uint32_t *d_w, uint64_t e_lo, uint64_t e_hi, const ghs_config_t *cfg, void *d_workspace,
                         size_t workspace_bytes, uint8_t *d_in_mst, void *stream, HostRes *pool, ghs_solver_t **out) {
  if (!out) GHS_FAIL(GHS_E_ARG, "out is NULL");
  *out = nullptr;
  if (m >= (1ull << 31)) GHS_FAIL(GHS_E_ARG, "m must be < 2^31");
  if (e_lo > e_hi || e_hi > m) GHS_FAIL(GHS_E_ARG, "bad edge range");
  if (cfg && (cfg->num_ranks < 1 || cfg->num_ranks > GHS_MAX_RANKS)) GHS_FAIL(GHS_E_ARG, "num_ranks must be in [1, GHS_MAX_RANKS]");
  if (m && ((!d_u && !d_off) || !d_v || !d_w || !d_in_mst)) GHS_FAIL(GHS_E_ARG, "d_u (d_off)/d_v/d_w/d_in_mst is NULL");
  if (d_off && m && n == 0) GHS_FAIL(GHS_E_ARG, "CSR input with edges needs n >= 1");
  // (a CSR caller's d_u too: the level-opening filter streams it when present)
  if ((((uintptr_t)d_u) | ((uintptr_t)d_v) | ((uintptr_t)d_w)) & 15)
    GHS_FAIL(GHS_E_ARG, "d_u/d_v/d_w must be 16-byte aligned");
  if (((uintptr_t)d_off) & 3) GHS_FAIL(GHS_E_ARG, "d_off must be 4-byte aligned");
  const size_t need = workspace_layout(n, m, e_hi - e_lo, nullptr, nullptr);
  if (!d_workspace || workspace_bytes < need)
    GHS_FAIL(GHS_E_NOMEM, "workspace too small: need " + std::to_string(need) + " bytes");
  if (((uintptr_t)d_workspace) & 255) GHS_FAIL(GHS_E_ARG, "workspace must be 256-byte aligned");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) GHS_FAIL(GHS_E_NODEVICE, "no HIP device");

  ghs_solver *s = new ghs_solver();
  s->n = n; s->m = m; s->e_lo = e_lo; s->e_hi = e_hi;
  s->eu = d_u; s->ev = d_v; s->ew = d_w;
  s->eoff = d_off; s->csr = d_off != nullptr;
  s->in_mst = d_in_mst; s->stream = (hipStream_t)stream;
  if (cfg) s->cfg = *cfg; else default_config(&s->cfg);
  // path options come from the caller's config only (ABI 5): the library reads no environment
  // variable that changes the algorithm or a launch shape (GHS_AB_ENV builds excepted, below)
  const uint32_t opt = s->cfg.options;
  s->debug = (opt & GHS_OPT_DEBUG) != 0;
  s->detail = (opt & GHS_OPT_DETAIL) != 0;
  s->time_rounds = (opt & GHS_OPT_TIME_ROUNDS) != 0;
  s->seed_runs = (opt & GHS_OPT_NO_SEED_RUNS) == 0;
  s->windowed = (opt & GHS_OPT_NO_WINDOW) == 0;
  s->tail_on = (opt & GHS_OPT_NO_TAIL) == 0;
  s->check_totals = (opt & GHS_OPT_CHECK_TOTALS) != 0;
  s->dedup_max = s->cfg.dedup_max;
  {
    std::lock_guard<std::mutex> lock(g_prof_mutex);
    s->prof = g_prof_on;
    s->prof_id = g_prof_next_id++;
  }
#if GHS_AB_ENV
  // A/B builds only (make AB=1): launch-shape experiments from the environment
  if (const char *la = getenv("GHS_LOOKAHEAD")) {  // rounds in flight ahead of the check
    const long v = strtol(la, nullptr, 10);
    s->lookahead = (uint32_t)(v < 0 ? 0 : (v > 4 ? 4 : v));
  }
  auto grid_env = [](const char *name, uint32_t *dst) {  // per-kernel grids
    if (const char *g = getenv(name)) {
      const long v = strtol(g, nullptr, 10);
      *dst = (uint32_t)(v < 256 ? 256 : (v > (long)SEG_G ? SEG_G : v));
    }
  };
  grid_env("GHS_MINEDGE_G", &s->cmp_g);
  grid_env("GHS_IDENT_G", &s->ident_g);
  grid_env("GHS_WIN_G", &s->win_g);
  grid_env("GHS_LP_G", &s->lp_g);
  grid_env("GHS_SEG_G", &s->seg_g);
#endif
  s->ws_base = (char *)d_workspace;
  workspace_layout(n, m, e_hi - e_lo, s, s->ws_base);
  s->dense_mode = s->cfg.num_ranks > 1 && s->dlab != nullptr && (opt & GHS_OPT_NO_DENSE) == 0;

  if (pool) {
    s->res = pool;
  } else {
    s->res = &s->own;
    if (int rc = hostres_init(&s->own)) {
      ghs_solver_destroy(s);
      return rc;
    }
  }
  if (int rc = solver_begin(s)) {
    ghs_solver_destroy(s);
    return rc;
  }
  *out = s;
  return GHS_OK;
}

int ghs_solver_create(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                      uint64_t e_lo, uint64_t e_hi, const ghs_config_t *cfg, void *d_workspace,
                      size_t workspace_bytes, uint8_t *d_in_mst, void *stream, ghs_solver_t **out) {
  return solver_create(n, m, d_u, nullptr, d_v, d_w, e_lo, e_hi, cfg, d_workspace, workspace_bytes, d_in_mst, stream,
                       nullptr, out);
}

int ghs_solver_create_csr(uint32_t n, uint64_t m, const uint32_t *d_off, const uint32_t *d_u, const uint32_t *d_v,
                          const uint32_t *d_w, uint64_t e_lo, uint64_t e_hi, const ghs_config_t *cfg, void *d_workspace,
                          size_t workspace_bytes, uint8_t *d_in_mst, void *stream, ghs_solver_t **out) {
  if (m && !d_off) GHS_FAIL(GHS_E_ARG, "d_off is NULL");
  return solver_create(n, m, d_u, d_off ? d_off : nullptr, d_v, d_w, e_lo, e_hi, cfg, d_workspace, workspace_bytes,
                       d_in_mst, stream, nullptr, out);
}

}  // extern "C"

int ghs_solver_create_pooled(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                             uint64_t e_lo, uint64_t e_hi, const ghs_config_t *cfg, void *d_workspace,
                             size_t workspace_bytes, uint8_t *d_in_mst, void *stream, void *hostres,
                             ghs_solver_t **out) {
  if (!hostres) GHS_FAIL(GHS_E_ARG, "host resources are NULL");
  return solver_create(n, m, d_u, nullptr, d_v, d_w, e_lo, e_hi, cfg, d_workspace, workspace_bytes, d_in_mst, stream,
                       static_cast<HostRes *>(hostres), out);
}

void *ghs_hostres_new(int *rc) {
  HostRes *r = new HostRes();
  if ((*rc = hostres_init(r)) != GHS_OK) {
    hostres_free(r);
    delete r;
    return nullptr;
  }
  return r;
}

void ghs_hostres_delete(void *res) {
  if (!res) return;
  HostRes *r = static_cast<HostRes *>(res);
  hostres_free(r);
  delete r;
}

extern "C" {

// stepwise API: one round per minedge/contract pair, exact counts after every contract
int ghs_solver_minedge(ghs_solver_t *s, uint64_t *num_active) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  if (s->phase == 2) {
    if (num_active) *num_active = 0;
    return GHS_OK;
  }
  if (s->phase != 0) GHS_FAIL(GHS_E_STATE, "minedge called twice without contract");
  if (s->round >= 16 * GHS_MAX_ROUND_STATS) GHS_FAIL(GHS_E_ROUNDCAP, "round cap exceeded");
  while (!s->level_open) {
    if (s->pending_exchange) {  // the caller has OR-combined the level's flags
      if (int rc = open_level_finish(s)) return rc;
      if (!s->level_open) s->level += 1;  // no edge of this level on any rank
      continue;
    }
    if (levels_done(s)) {  // every level done
      s->phase = 2;
      if (num_active) *num_active = 0;
      return GHS_OK;
    }
    int rc = open_level(s);
    if (rc) return rc;
    if (s->pending_exchange) {
      if (num_active) *num_active = 0;
      return GHS_NEED_EXCHANGE;
    }
    if (!s->level_open) s->level += 1;  // skipped (no edges)
  }
  if (int rc = enqueue_minedge(s)) return rc;
  s->phase = 1;
  if (num_active) *num_active = s->nact;
  return GHS_OK;
}

int ghs_solver_exchange_buffer(ghs_solver_t *s, uint8_t **d_flags, uint64_t *bytes) {
  if (!s || !d_flags || !bytes) GHS_FAIL(GHS_E_ARG, "solver/d_flags/bytes is NULL");
  if (!s->pending_exchange) GHS_FAIL(GHS_E_STATE, "no exchange pending");
  if (int rc = solver_sync(s)) return rc;  // the flags are complete before the caller reads them
  *d_flags = s->flags;
  *bytes = (uint64_t)s->n + 1;  // n fragment flags + the error byte
  return GHS_OK;
}

int ghs_solver_flag_bits(ghs_solver_t *s, uint64_t **d_bits, uint64_t *words) {
  if (int rc = ghs_solver_flag_bits_async(s, d_bits, words)) return rc;
  if (int rc = solver_sync(s)) return rc;  // complete before the caller's collective reads it
  return GHS_OK;
}

}  // extern "C"

// the pack without the trailing sync: for a caller whose collective is enqueued on the solver's
// own stream (ghs_solver_run)
int ghs_solver_flag_bits_async(ghs_solver *s, uint64_t **d_bits, uint64_t *words) {
  if (!s || !d_bits || !words) GHS_FAIL(GHS_E_ARG, "solver/d_bits/words is NULL");
  if (!s->pending_exchange) GHS_FAIL(GHS_E_STATE, "no exchange pending");
  const uint64_t nf = (uint64_t)s->n + 1, nw = (nf + 63) / 64;
  {
    KT(GHS_K_FLAG_BITS, nw);
    k_pack_flag_bits<<<grid_for(nw, 256, 16384), 256, 0, s->stream>>>(s->flags, nf, s->flag_bits);
  }
  GHS_HIP_CHECK(hipGetLastError());
  *d_bits = s->flag_bits;
  *words = nw;
  return GHS_OK;
}

extern "C" {

int ghs_solver_merge_flag_bits(ghs_solver_t *s, const uint64_t *d_all, uint32_t nranks) {
  if (!s || !d_all || nranks == 0) GHS_FAIL(GHS_E_ARG, "solver/d_all is NULL or nranks is 0");
  if (!s->pending_exchange) GHS_FAIL(GHS_E_STATE, "no exchange pending");
  const uint64_t nf = (uint64_t)s->n + 1, nw = (nf + 63) / 64;
  {
    KT(GHS_K_FLAG_BITS, nw);
    if (s->dense_mode) {  // the level opens from the merged words (no flag bytes, no select over n)
      k_merge_flag_words<<<grid_for(nw, 256, 16384), 256, 0, s->stream>>>(d_all, nranks, nw, s->n, s->drank_bits,
                                                                          s->flags + s->n);
      s->words_merged = true;
    } else {
      k_merge_flag_bits<<<grid_for(nw, 256, 16384), 256, 0, s->stream>>>(d_all, nranks, nw, nf, s->flags,
                                                                         s->flags + s->n);
    }
  }
  GHS_HIP_CHECK(hipGetLastError());
  return GHS_OK;
}

int ghs_solver_pack_best(ghs_solver_t *s, int64_t *d_dense) {
  if (!s || (s->nact && !d_dense)) GHS_FAIL(GHS_E_ARG, "solver/dense is NULL");
  if (s->phase != 1) GHS_FAIL(GHS_E_STATE, "pack_best must follow minedge");
  if (s->nact) {
    const uint32_t *act = s->act_ident ? nullptr : s->act[s->act_cur];
    KT(GHS_K_PACK, s->nact);
    k_pack_best<<<grid_for(s->nact, 256, 16384), 256, 0, s->stream>>>(act, cur_act_count(s), s->best, d_dense, s->nact);
    GHS_HIP_CHECK(hipGetLastError());
  }
  return GHS_OK;
}

int ghs_solver_best_slots(ghs_solver_t *s, uint64_t **d_slots, uint64_t *count) {
  if (!s || !d_slots || !count) GHS_FAIL(GHS_E_ARG, "solver/slots/count is NULL");
  if (s->phase != 1) GHS_FAIL(GHS_E_STATE, "best_slots must follow minedge");
  *d_slots = ghs_solver_best_slots_of(s);
  *count = *d_slots ? s->nact : 0;
  return GHS_OK;
}

int ghs_solver_unpack_best(ghs_solver_t *s, const int64_t *d_dense) {
  if (!s || (s->nact && !d_dense)) GHS_FAIL(GHS_E_ARG, "solver/dense is NULL");
  if (s->phase != 1) GHS_FAIL(GHS_E_STATE, "unpack_best must follow minedge");
  if (s->nact) {
    const uint32_t *act = s->act_ident ? nullptr : s->act[s->act_cur];
    KT(GHS_K_UNPACK, s->nact);
    k_unpack_best<<<grid_for(s->nact, 256, 16384), 256, 0, s->stream>>>(act, cur_act_count(s), s->best, d_dense);
    GHS_HIP_CHECK(hipGetLastError());
  }
  return GHS_OK;
}

int ghs_solver_hook_local(ghs_solver_t *s, int32_t *d_dense, uint64_t *count) {
  if (!s || !count) GHS_FAIL(GHS_E_ARG, "solver/count is NULL");
  *count = 0;
  if (s->phase != 1) GHS_FAIL(GHS_E_STATE, "hook_local must follow unpack_best");
  // a level's first round with several ranks (its edges carry the current roots); labels and
  // fragment ids must fit the int32 MAX exchange
  if (s->cfg.num_ranks <= 1 || s->level_round != 0 || !s->nact || s->hooked || s->n > (1u << 31)) return GHS_OK;
  if (!d_dense) GHS_FAIL(GHS_E_ARG, "dense is NULL");
  const uint32_t *act = s->act_ident ? nullptr : s->act[s->act_cur];
  if (s->cur_arcs || !s->arcs_known) {
    const ArcBuf &I = s->buf[s->cur];
    SegView in{I.seg_start, I.seg_prefix, s->cur_nseg};
    KT(GHS_K_WIN, s->arcs_known ? s->cur_arcs : 0);
    k_win<<<s->arcs_known ? grid_for(s->cur_arcs, ARCS_PER_BLOCK, s->win_g) : s->win_g, BLOCK, 0, s->stream>>>(
        I.src, I.dst, I.key, in, s->best, s->par, s->in_mst, nullptr, nullptr);
  }
  KT(GHS_K_PACK_HOOK, s->nact);
  k_pack_hook<<<grid_for(s->nact, 256, 16384), 256, 0, s->stream>>>(act, cur_act_count(s), s->par, d_dense);
  GHS_HIP_CHECK(hipGetLastError());
  *count = s->nact;
  return GHS_OK;
}

int ghs_solver_unpack_hook(ghs_solver_t *s, const int32_t *d_dense) {
  if (!s || (s->nact && !d_dense)) GHS_FAIL(GHS_E_ARG, "solver/dense is NULL");
  if (s->phase != 1 || s->cfg.num_ranks <= 1 || s->level_round != 0 || s->hooked)
    GHS_FAIL(GHS_E_STATE, "unpack_hook must follow hook_local");
  if (s->nact) {
    const uint32_t *act = s->act_ident ? nullptr : s->act[s->act_cur];
    KT(GHS_K_UNPACK_HOOK, s->nact);
    k_unpack_hook<<<grid_for(s->nact, BLOCK, HOOK_G), BLOCK, 0, s->stream>>>(act, cur_act_count(s), d_dense, s->best,
                                                                            s->par, s->cnt + C_WEIGHT);
    GHS_HIP_CHECK(hipGetLastError());
  }
  s->hooked = true;
  return GHS_OK;
}

int ghs_solver_hook_slots(ghs_solver_t *s, uint32_t nranks, uint64_t **d_slots, uint64_t *padded) {
  if (!s || !d_slots || !padded || nranks == 0) GHS_FAIL(GHS_E_ARG, "solver/slots/padded is NULL or nranks == 0");
  *d_slots = nullptr;
  *padded = 0;
  if (s->phase != 1) GHS_FAIL(GHS_E_STATE, "hook_slots must follow minedge");
  // the padding (< nranks slots past nact) lives in dbest's and the communicator's 64 spare slots
  if (nranks != s->cfg.num_ranks) GHS_FAIL(GHS_E_ARG, "hook_slots: nranks differs from the solver's num_ranks");
  if (nranks > GHS_MAX_RANKS) GHS_FAIL(GHS_E_ARG, "hook_slots: more than GHS_MAX_RANKS ranks");
  s->hook_S = 0;
  // a dense level's opening round (its slots are best itself, in dense-label order)
  if (s->cfg.num_ranks <= 1 || s->level_round != 0 || !s->nact || s->hooked || !s->act_ident || !s->level_dense)
    return GHS_OK;
  const uint64_t S = (s->nact + nranks - 1) / nranks * nranks;
  if (S > s->nact) {
    k_pad_slots<<<(unsigned)((S - s->nact + 255) / 256 + 1), 256, 0, s->stream>>>(s->best, cur_act_count(s), S);
    GHS_HIP_CHECK(hipGetLastError());
  }
  *d_slots = s->best;
  *padded = S;
  s->hook_S = S;
  return GHS_OK;
}

int ghs_solver_hook_owner(ghs_solver_t *s, uint32_t rank, uint64_t per, uint64_t *d_pairs) {
  if (!s || !d_pairs) GHS_FAIL(GHS_E_ARG, "solver/pairs is NULL");
  if (s->phase != 1 || !s->level_dense || !s->act_ident || s->level_round != 0 || s->hooked)
    GHS_FAIL(GHS_E_STATE, "hook_owner must follow hook_slots and the reduce-scatter");
  if (rank >= s->cfg.num_ranks || (uint64_t)(rank + 1) * per > s->hook_S || per * s->cfg.num_ranks != s->hook_S)
    GHS_FAIL(GHS_E_ARG, "hook_owner: rank / slice outside the padded slots of hook_slots");
  const uint64_t lo = (uint64_t)rank * per, hi = lo + per;
  if (per) {
    KT(GHS_K_PACK_HOOK, per);
    k_hook_owner<<<grid_for(per, 256, 16384), 256, 0, s->stream>>>(s->best, lo, hi, ends_of(s), s->vlab,
                                                                   dense_rank_of(s), d_pairs, s->cnt + C_ERR);
    GHS_HIP_CHECK(hipGetLastError());
  }
  return GHS_OK;
}

int ghs_solver_apply_hooks(ghs_solver_t *s, const uint64_t *d_pairs, uint64_t **d_partial) {
  if (!s || (s->nact && !d_pairs) || !d_partial) GHS_FAIL(GHS_E_ARG, "solver/pairs/partial is NULL");
  *d_partial = reinterpret_cast<uint64_t *>(s->cnt + C_RS_WEIGHT);
  if (s->phase != 1 || !s->level_dense || !s->act_ident || s->level_round != 0 || s->hooked)
    GHS_FAIL(GHS_E_STATE, "apply_hooks must follow hook_owner and the all-gather");
  if (s->nact) {
    KT(GHS_K_UNPACK_HOOK, s->nact);
    k_apply_pairs<<<grid_for(s->nact, BLOCK, HOOK_G), BLOCK, 0, s->stream>>>(
        d_pairs, cur_act_count(s), s->ew, s->par, s->best, s->in_mst, (uint32_t)s->e_lo, (uint32_t)s->e_hi,
        s->cnt + C_RS_WEIGHT);
    GHS_HIP_CHECK(hipGetLastError());
  }
  s->hooked = true;
  s->rs_fold = true;  // contract folds the (all-reduced) partial totals in first
  return GHS_OK;
}

int ghs_solver_contract(ghs_solver_t *s, int *done) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  if (s->phase == 2) {
    if (done) *done = 1;
    return GHS_OK;
  }
  if (s->phase != 1) GHS_FAIL(GHS_E_STATE, "contract must follow minedge");
  s->report_final = false;
  const uint64_t live_in = s->level_round <= 1 ? s->cur_arcs : s->h_cnt[C_LIVE];
  const uint64_t nact_in = s->nact;
  if (int rc = enqueue_contract(s)) return rc;
  s->hooked = false;
  const int nb = s->act_ident ? 0 : (s->act_cur ^ 1);
  GHS_HIP_CHECK(hipMemcpyAsync(s->h_cnt, s->cnt, C_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, s->stream));
  if (int rc = solver_sync(s)) return rc;
  if (s->h_cnt[C_ERR]) return fail_counters(s, s->h_cnt[C_ERR], ("in round " + std::to_string(s->round + 1)).c_str());
  push_stats(s, s->level_round, live_in, nact_in, s->h_cnt[C_EDGES]);
  s->nact = s->h_cnt[C_ACT + nb];
  advance_round(s);
  if (s->nact <= 1) {  // level complete (one active fragment: its remaining edges are internal)
    if (int rc = dense_close(s)) return rc;
    close_level(s);
  } else {
    s->phase = 0;
  }
  if (done) *done = (s->phase == 2);
  return GHS_OK;
}

}  // extern "C"

// Multi-rank round loop (ghs_solver_run), pipelined: rounds >= 2 of a level are contracted without
// a host sync. The round's last kernel reports to a pinned slot; the host reads the report of the
// round BEFORE the one just enqueued (one round in flight), so round r + 1 is enqueued while round r
// still runs. Round r + 1's collective count is a bound: every active fragment of a round hooks or
// is hooked by another active one, so a round's active fragments are at most half the previous
// round's — floor(exact >> rounds since the latest exact count); the packed slots past the device
// count hold "no edge" on every rank, and every rank computes the same bounds. Rounds 0 and 1 keep
// the synchronous contract (round 1's bound from round 0's count would be far too loose: R-MAT s26
// x8, level 1: 11.7M bound vs 195K active). A level whose report shows <= 1 active fragment ends;
// the one round already enqueued past it is a no-op on the device (guards on the device counts).
int ghs_solver_contract_async(ghs_solver *s, int *done) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  if (s->phase == 2) {
    if (done) *done = 1;
    return GHS_OK;
  }
#ifndef GHS_PIPE_MULTI
#define GHS_PIPE_MULTI 1
#endif
  if (s->cfg.num_ranks <= 1 || s->level_round < 2 || !GHS_PIPE_MULTI) {
    const int rc = ghs_solver_contract(s, done);
    if (!rc && s->phase == 0 && s->level_round == 2) {  // round 2 comes next: its count is exact
      s->pipe.clear();
      s->pipe_exact = s->nact;
      s->pipe_exact_lr = 2;
      s->pipe_live = s->h_cnt[C_LIVE];
    }
    return rc;
  }
  if (s->phase != 1) GHS_FAIL(GHS_E_STATE, "contract must follow minedge");
  s->report_final = false;
  const unsigned long long seq = ++s->res->seq;
  if (int rc = enqueue_contract(s, &s->d_slot[seq % SLOT_RING], seq)) return rc;
  s->hooked = false;
  s->pipe.push_back({seq, s->round, s->level_round});
  advance_round(s);
  bool level_done = false;
  while (s->pipe.size() > 1 && !level_done) {  // read every report but the newest round's
    const ghs_solver::PipeRound p = s->pipe.front();
    s->pipe.erase(s->pipe.begin());
    RoundSlot rep;
    if (int rc = wait_slot(s, s->h_slot + (p.seq % SLOT_RING), p.seq, &rep)) return rc;
    const unsigned long long err = slot_err(rep.err), nact_in = rep.nact_in, nact_out = rep.nact_out;
    const unsigned long long live_out = rep.live_out, edges = rep.edges;
    if (err) return fail_counters(s, err, ("in round " + std::to_string(p.round + 1)).c_str());
    push_stats(s, p.level_round, s->pipe_live, nact_in, edges);
    s->pipe_live = live_out;
    s->pipe_exact = nact_out;  // the active fragments at the start of round p + 1
    s->pipe_exact_lr = p.level_round + 1;
    if (nact_out <= 1) {  // the level ended with round p: later rounds are no-ops
      level_done = true;
      s->round = p.round + 1;
      s->level_round = p.level_round + 1;
    }
  }
  if (level_done) {
    s->pipe.clear();
    if (int rc = dense_close(s)) return rc;
    close_level(s);
  } else {
    s->nact = s->pipe_exact >> (s->level_round - s->pipe_exact_lr);  // bound for the next round
    if (s->nact <= 1) {
      // the bound says the level is over (<= 1 fragment can remain): the rounds in flight finish
      // it; wait for them so their stats and errors are read, then close the level
      while (!s->pipe.empty()) {
        const ghs_solver::PipeRound p = s->pipe.front();
        s->pipe.erase(s->pipe.begin());
        RoundSlot rep;
        if (int rc = wait_slot(s, s->h_slot + (p.seq % SLOT_RING), p.seq, &rep)) return rc;
        if (slot_err(rep.err)) return fail_counters(s, slot_err(rep.err), ("in round " + std::to_string(p.round + 1)).c_str());
        push_stats(s, p.level_round, s->pipe_live, rep.nact_in, rep.edges);
        s->pipe_live = rep.live_out;
      }
      if (int rc = dense_close(s)) return rc;
      close_level(s);
    } else {
      s->phase = 0;
    }
  }
  if (done) *done = (s->phase == 2);
  return GHS_OK;
}

extern "C" {

int ghs_solver_finish(ghs_solver_t *s, ghs_result_t *result, ghs_round_stats_t *stats) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  if (s->phase != 2) GHS_FAIL(GHS_E_STATE, "finish before the loop terminated");
  if (s->report_final && !s->check_totals) {
    // the pipelined loop's last report (checksum-validated) holds the final totals: no copy, no
    // sync (a trailing no-op lookahead round may still run on the stream; it changes no counter)
    s->h_cnt[C_WEIGHT] = s->rep_weight;
    s->h_cnt[C_EDGES] = s->rep_edges;
  } else {
    GHS_HIP_CHECK(hipMemcpyAsync(s->h_cnt, s->cnt, C_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, s->stream));
    if (int rc = solver_sync(s)) return rc;
  }
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - s->t0).count();
  if (int rc = prof_collect(s)) return rc;
  const uint32_t ns = (uint32_t)std::min<size_t>(s->stats.size(), GHS_MAX_ROUND_STATS);
  for (uint32_t r = 0; r < ns; ++r) {
    float t[4] = {0, 0, 0, 0};
    const uint8_t rec = r < s->ev_rec.size() ? s->ev_rec[r] : 0;
    for (int k = 0; k < 4; ++k) {
      if (((rec >> k) & 3) != 3) continue;  // both ends recorded
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
    result->num_mst_edges = s->n ? s->h_cnt[C_EDGES] : 0;
    result->total_weight = s->n ? s->h_cnt[C_WEIGHT] : 0;
    result->rounds = s->round;
    result->num_stats = ns;
    result->levels = (plan_sync(s) == GHS_OK) ? (uint32_t)(s->thresholds.size() - 1) : 0u;
    result->ms_total = ms;
    float t = 0;
    result->ms_select = (s->e_hi > s->e_lo && hipEventElapsedTime(&t, s->res->pass_ev[0], s->res->pass_ev[1]) == hipSuccess) ? t : 0.f;
    t = 0;
    result->ms_filter = (s->filter_run && hipEventElapsedTime(&t, s->res->pass_ev[2], s->res->pass_ev[3]) == hipSuccess) ? t : 0.f;
    result->canon_edges = s->e_hi - s->e_lo;
    result->select_out = s->select_out;
    result->filter_out = s->filter_out;
    result->pass_flags = (s->bucketed ? 1u : 0u) | (s->lattice ? 2u : 0u) | (s->windowed_ran ? 4u : 0u) |
                         (s->tail_ran ? 8u : 0u);
    result->ms_setup = result->ms_solve = result->ms_gather = 0;
    result->reused = 0;
    result->reserved = 0;
  }
  return GHS_OK;
}

int ghs_solver_reset(ghs_solver_t *s) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  // a fresh round state over the same inputs, workspace, knobs and host resources
  ghs_solver t;
  t.n = s->n; t.m = s->m; t.e_lo = s->e_lo; t.e_hi = s->e_hi;
  t.eu = s->eu; t.ev = s->ev; t.ew = s->ew; t.eoff = s->eoff; t.csr = s->csr;
  t.in_mst = s->in_mst; t.stream = s->stream; t.cfg = s->cfg;
  t.debug = s->debug; t.lookahead = s->lookahead; t.seed_runs = s->seed_runs; t.dedup_max = s->dedup_max;
  t.windowed = s->windowed;
  t.tail_on = s->tail_on;
  t.check_totals = s->check_totals;
  t.detail = s->detail; t.time_rounds = s->time_rounds;
  t.group_cancel = s->group_cancel;
  { std::lock_guard<std::mutex> lock(g_prof_mutex); t.prof = g_prof_on; }
  t.prof_id = s->prof_id;
  t.seg_g = s->seg_g; t.cmp_g = s->cmp_g; t.ident_g = s->ident_g; t.win_g = s->win_g; t.lp_g = s->lp_g;
  t.ws_base = s->ws_base;
  workspace_layout(t.n, t.m, t.e_hi - t.e_lo, &t, t.ws_base);
  t.dense_mode = s->dense_mode;
  const bool owned = s->res == &s->own;
  HostRes *pool = s->res;
  t.own = std::move(s->own);
  s->own = HostRes();
  *s = std::move(t);
  s->res = owned ? &s->own : pool;
  return solver_begin(s);
}

int ghs_solver_cancel(ghs_solver_t *s) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  __atomic_store_n(&s->cancel_flag, 1, __ATOMIC_RELEASE);
  return GHS_OK;
}

int ghs_solver_destroy(ghs_solver_t *s) {
  if (!s) return GHS_OK;
  if (s->res == &s->own) hostres_free(&s->own);
  delete s;
  return GHS_OK;
}

// the one-shot solve of ghs_mst_device / ghs_mst_device_csr
static int mst_device(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_off, const uint32_t *d_v,
                      const uint32_t *d_w, const ghs_config_t *cfg, void *d_workspace, size_t workspace_bytes,
                      uint8_t *d_in_mst, void *stream, ghs_result_t *result, ghs_round_stats_t *stats) {
  std::lock_guard<std::mutex> lock(g_mutex);
  ghs_solver_t *s = nullptr;
  ghs_config_t c;
  if (cfg) c = *cfg; else default_config(&c);
  c.num_ranks = 1;  // one device holds every edge
  int rc = GHS_OK;
  HostRes *pool = pooled_res(&rc);
  if (!pool) return rc;
  rc = solver_create(n, m, d_u, d_off, d_v, d_w, 0, m, &c, d_workspace, workspace_bytes, d_in_mst, stream, pool, &s);
  if (rc) return rc;
  while (!rc && s->phase != 2) {
    if (!s->level_open) {
      if (levels_done(s)) {
        s->phase = 2;
        break;
      }
      rc = open_level(s, /*async_open=*/true);  // no host sync: the counts come with round 0
      if (rc) break;
    }
    rc = run_level_pipelined(s);
  }
  if (!rc) rc = ghs_solver_finish(s, result, stats);
  ghs_solver_destroy(s);
  return rc;
}

int ghs_mst_device(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                   const ghs_config_t *cfg, void *d_workspace, size_t workspace_bytes, uint8_t *d_in_mst, void *stream,
                   ghs_result_t *result, ghs_round_stats_t *stats) {
  return mst_device(n, m, d_u, nullptr, d_v, d_w, cfg, d_workspace, workspace_bytes, d_in_mst, stream, result, stats);
}

int ghs_mst_device_csr(uint32_t n, uint64_t m, const uint32_t *d_off, const uint32_t *d_u, const uint32_t *d_v,
                       const uint32_t *d_w, const ghs_config_t *cfg, void *d_workspace, size_t workspace_bytes,
                       uint8_t *d_in_mst, void *stream, ghs_result_t *result, ghs_round_stats_t *stats) {
  if (m && !d_off) GHS_FAIL(GHS_E_ARG, "d_off is NULL");
  return mst_device(n, m, d_u, d_off, d_v, d_w, cfg, d_workspace, workspace_bytes, d_in_mst, stream, result, stats);
}

}  // extern "C"
