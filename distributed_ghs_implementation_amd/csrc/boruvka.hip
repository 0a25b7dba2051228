// Level-synchronous Boruvka fragment contraction on gfx950 — the MI355X restatement of the
// reference's GHS level loop. One round here == one GHS level of the reference:
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
//   termination (:389-413, :492-552; _mpi:685-743)               k_flag_next + select: fragments with an
//                                                                 outgoing edge; none left => done
//   BRANCH sweep u<v (:481-490; _mpi:750-779)                    in_mst[eid] set by k_hook
//
// Data layout in HBM (all SoA, 256-B aligned):
//   arcs   src[A] u32 | dst[A] u32 | key[A] u64     key = w << 32 | eid, grouped by src
//   lab[n]  u32  fragment label map (see "label invariant" below)
//   best[n] u64  per-fragment minimum outgoing key (atomicMin target)
//   par[n]  u32  hook parent
//   act[2][n] u32 active fragment lists (double buffer)
//   arc double buffers for the compacted, relabelled arcs of rounds >= 2
//
// Label invariant. Round 1 scans the input arcs with the identity labelling. From round 2 on
// the min-edge kernel rewrites every surviving arc as (lab[src], lab[dst], key), so the arcs of
// round r carry the labels of the fragments that were active at the START of round r-1, and
// lab[x] for exactly those labels is refreshed every round to the current root (k_jump).
// A vertex's current fragment is found by following lab[] to a fixpoint (find_lab): roots
// satisfy lab[x] == x, and the chain is at most one hop longer per round.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "common.h"

namespace ghs {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }

__device__ __forceinline__ uint32_t wave_prefix_count(uint64_t ballot) {
  // number of set bits of `ballot` in lanes below this one
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(ballot >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ballot, 0u));
}

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// ------------------------------------------------------------------------------------------
// Stage 1: minimum outgoing edge per fragment (+ fused self-loop filter / stream compaction).
//
// Each lane owns 4 consecutive arcs (16-B loads of src/dst, 2x16-B of key). Arcs are grouped by
// source, so equal source labels form runs; a wave-wide segmented min-scan over its 256 arcs
// (in-lane serial + 6-step cross-lane scan) leaves one candidate per run, and only run tails
// touch best[] — with a plain read first, since best only ever decreases (a stale read can only
// be larger than the true value, so skipping on `best <= cand` is always correct).
// IDENT: round 1, labels are vertex ids (no gathers, dst not read). COMPACT: write surviving
// arcs relabelled; block-local order is preserved, blocks claim output ranges atomically.
// ------------------------------------------------------------------------------------------
template <bool IDENT, bool COMPACT>
__global__ __launch_bounds__(BLOCK) void k_minedge(const uint32_t *__restrict__ src, const uint32_t *__restrict__ dst,
                                                   const uint64_t *__restrict__ key, uint64_t A,
                                                   const uint32_t *__restrict__ lab, uint64_t *__restrict__ best,
                                                   uint32_t *__restrict__ osrc, uint32_t *__restrict__ odst,
                                                   uint64_t *__restrict__ okey, unsigned long long *__restrict__ out_count) {
  __shared__ uint32_t s_wcnt[BLOCK / WAVE];
  __shared__ unsigned long long s_base;
  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = threadIdx.x / WAVE;
  const uint64_t nchunks = (A + ARCS_PER_BLOCK - 1) / ARCS_PER_BLOCK;

  for (uint64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const uint64_t i0 = chunk * ARCS_PER_BLOCK + (uint64_t)threadIdx.x * ARCS_PER_THREAD;
    uint32_t L[4], D[4];
    uint64_t K[4];
    bool valid[4];
    if (i0 + 4 <= A) {
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
      for (int j = 0; j < 4; ++j) valid[j] = true;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        valid[j] = i0 + j < A;
        L[j] = valid[j] ? src[i0 + j] : 0u;
        D[j] = (!IDENT && valid[j]) ? dst[i0 + j] : 0u;
        K[j] = valid[j] ? key[i0 + j] : KEY_NONE;
      }
    }
    uint64_t V[4];
    if (IDENT) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        V[j] = valid[j] ? K[j] : KEY_NONE;  // canonical arcs are never self-loops
        L[j] = valid[j] ? L[j] : LABEL_NONE;
      }
    } else {
      uint32_t cs[4], cd[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // 8 independent gathers in flight per lane
        cs[j] = lab[L[j]];
        cd[j] = lab[D[j]];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        L[j] = valid[j] ? cs[j] : LABEL_NONE;
        D[j] = cd[j];
        V[j] = (valid[j] && cs[j] != cd[j]) ? K[j] : KEY_NONE;
      }
    }

    // ---- wave-wide segmented min over the 256 arcs, segments = runs of equal source label
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
      const bool tail = (j < 3) ? H[j + 1] : (lane == WAVE - 1 || nextH0);
      if (tail && run != KEY_NONE) {
        uint64_t *p = best + L[j];
        if (*p > run) atomicMin(reinterpret_cast<unsigned long long *>(p), (unsigned long long)run);
      }
    }

    if (COMPACT) {
      // ---- ballot + prefix-sum stream compaction of inter-fragment arcs (REJECT filter)
      uint32_t before = 0, wave_total = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint64_t b = __ballot(V[j] != KEY_NONE);
        before += wave_prefix_count(b);
        wave_total += (uint32_t)__popcll(b);
      }
      if (lane == 0) s_wcnt[wid] = wave_total;
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < BLOCK / WAVE; ++w) t += s_wcnt[w];
        s_base = t ? atomicAdd(out_count, (unsigned long long)t) : 0ull;
      }
      __syncthreads();
      uint64_t pos = s_base + before;
      for (int w = 0; w < wid; ++w) pos += s_wcnt[w];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (V[j] != KEY_NONE) {
          osrc[pos] = L[j];
          odst[pos] = D[j];
          okey[pos] = K[j];
          ++pos;
        }
      }
      __syncthreads();
    }
  }
}

// Bounded walks: a chain longer than these bounds means a broken invariant; the kernel sets
// the error word (checked by the host after every round) instead of spinning forever.
constexpr int FIND_LAB_MAX_HOPS = 256;        // >= rounds + 2 (rounds <= 64)
constexpr uint32_t JUMP_MAX_STEPS = 1u << 26;

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
// label stays root (the reference merges equal-level fragments on a shared core edge,
// ghs_implementation.py:186-196, and picks the initiator by (fragment_id, rank),
// ghs_implementation_mpi.py:237-239). Every hook adds exactly one MSF edge.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_hook(const uint32_t *__restrict__ act, uint64_t nact,
                                                const uint64_t *__restrict__ best, const uint32_t *__restrict__ lab,
                                                const uint32_t *__restrict__ eu, const uint32_t *__restrict__ ev,
                                                uint32_t *__restrict__ par, uint8_t *__restrict__ in_mst,
                                                unsigned long long *__restrict__ acc /* [0] weight, [1] edges */,
                                                unsigned long long *__restrict__ err) {
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i - threadIdx.x < nact;
       i += (uint64_t)gridDim.x * BLOCK) {
    unsigned long long wsum = 0, cnt = 0;
    if (i < nact) {
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
          wsum = k >> 32;
          cnt = 1;
        }
      }
      par[c] = p;
    }
#pragma unroll
    for (int d = WAVE / 2; d > 0; d >>= 1) {
      wsum += __shfl_xor(wsum, d);
      cnt += __shfl_xor(cnt, d);
    }
    if ((threadIdx.x & (WAVE - 1)) == 0 && cnt) {
      atomicAdd(acc + 0, wsum);
      atomicAdd(acc + 1, cnt);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Stage 3: pointer jumping (INITIATE broadcast of the new fragment id). Path splitting on par:
// concurrent compression only ever moves a pointer to an ancestor, so stale reads are still
// valid ancestors and every walk ends at its root. lab[c] = root.
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
// Stage 3b: next active fragment list = roots that still had an outgoing edge; reset their
// best slot. (A root with no outgoing edge is a finished MSF component: the reference's
// "best_weight == inf at the core => terminate", ghs_implementation.py:316-320.)
// The list itself is produced by an order-preserving select (hipcub::DeviceSelect::Flagged),
// so every rank of a multi-GPU run holds the same list in the same order — the all-reduce
// slots line up without any exchange of the list.
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

__global__ void k_iota(uint32_t *__restrict__ a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
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

}  // namespace ghs

using namespace ghs;

// ============================================================================================
// Solver handle
// ============================================================================================
struct ghs_solver {
  uint32_t n = 0;
  uint64_t m = 0;
  const uint32_t *eu = nullptr, *ev = nullptr;
  const uint32_t *in_src = nullptr, *in_dst = nullptr;
  const uint64_t *in_key = nullptr;
  uint64_t num_arcs = 0;
  uint8_t *in_mst = nullptr;
  hipStream_t stream = nullptr;

  uint32_t *lab = nullptr, *par = nullptr, *act[2] = {nullptr, nullptr};
  uint64_t *best = nullptr;
  uint32_t *bsrc[2] = {nullptr, nullptr}, *bdst[2] = {nullptr, nullptr};
  uint64_t *bkey[2] = {nullptr, nullptr};
  uint8_t *flags = nullptr;
  void *cub_temp = nullptr;
  size_t cub_bytes = 0;
  unsigned long long *cnt = nullptr;    // device [0] arcs out, [1] active out, [2] weight, [3] edges
  unsigned long long *h_cnt = nullptr;  // pinned host mirror

  // round state
  uint32_t round = 0;      // completed rounds
  int phase = 0;           // 0: expect minedge, 1: expect contract, 2: done
  int cur_buf = -1;        // -1: arcs are the input arrays
  uint64_t cur_arcs = 0;
  int act_cur = 0;
  bool act_ident = true;   // round 1: fragments are 0..n-1
  uint64_t nact = 0;
  uint64_t edges_before = 0;

  std::vector<ghs_round_stats_t> stats;
  std::vector<hipEvent_t> ev_pool;  // 5 per round (up to GHS_MAX_ROUND_STATS rounds)
  std::chrono::steady_clock::time_point t0;
};

static std::mutex g_mutex;  // calls are serialised per process

static size_t select_temp_bytes(uint32_t n) {
  size_t a = 0, b = 0;
  const size_t items = n ? n : 1;
  (void)hipcub::DeviceSelect::Flagged(nullptr, a, (const uint32_t *)nullptr, (const uint8_t *)nullptr,
                                      (uint32_t *)nullptr, (unsigned long long *)nullptr, items);
  (void)hipcub::DeviceSelect::Flagged(nullptr, b, hipcub::CountingInputIterator<uint32_t>(0u),
                                      (const uint8_t *)nullptr, (uint32_t *)nullptr, (unsigned long long *)nullptr,
                                      items);
  return (a > b ? a : b) + 256;
}

static size_t workspace_layout(uint32_t n, uint64_t num_arcs, ghs_solver *s, char *base) {
  size_t off = 0;
  auto carve = [&](size_t bytes) -> char * {
    char *p = base ? base + off : nullptr;
    off = align_up(off + bytes, 256);
    return p;
  };
  const size_t N = (size_t)n;
  char *p;
  p = carve(N * 4); if (s) s->lab = (uint32_t *)p;
  p = carve(N * 4); if (s) s->par = (uint32_t *)p;
  p = carve(N * 8); if (s) s->best = (uint64_t *)p;
  p = carve(N * 4); if (s) s->act[0] = (uint32_t *)p;
  p = carve(N * 4); if (s) s->act[1] = (uint32_t *)p;
  for (int b = 0; b < 2; ++b) {
    p = carve(num_arcs * 4); if (s) s->bsrc[b] = (uint32_t *)p;
    p = carve(num_arcs * 4); if (s) s->bdst[b] = (uint32_t *)p;
    p = carve(num_arcs * 8); if (s) s->bkey[b] = (uint64_t *)p;
  }
  p = carve(N ? N : 1); if (s) s->flags = (uint8_t *)p;
  size_t cb = select_temp_bytes(n);
  p = carve(cb); if (s) { s->cub_temp = p; s->cub_bytes = cb; }
  p = carve(8 * sizeof(unsigned long long)); if (s) s->cnt = (unsigned long long *)p;
  return off;
}

static int check_dev_ptr16(const void *p, uint64_t count, const char *name) {
  if (count && !p) GHS_FAIL(GHS_E_ARG, std::string(name) + " is NULL");
  if (((uintptr_t)p) & 15) GHS_FAIL(GHS_E_ARG, std::string(name) + " must be 16-byte aligned");
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

size_t ghs_workspace_bytes(uint32_t n, uint64_t m, uint64_t num_arcs) {
  (void)m;
  return workspace_layout(n, num_arcs, nullptr, nullptr);
}

int ghs_solver_create(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_asrc,
                      const uint32_t *d_adst, const uint64_t *d_akey, uint64_t num_arcs, void *d_workspace,
                      size_t workspace_bytes, uint8_t *d_in_mst, void *stream, ghs_solver_t **out) {
  if (!out) GHS_FAIL(GHS_E_ARG, "out is NULL");
  *out = nullptr;
  if (m >= (1ull << 32)) GHS_FAIL(GHS_E_ARG, "m must be < 2^32 (eid is 32-bit)");
  if (num_arcs >= (1ull << 40)) GHS_FAIL(GHS_E_ARG, "num_arcs too large");
  int rc;
  if ((rc = check_dev_ptr16(d_asrc, num_arcs, "d_asrc"))) return rc;
  if ((rc = check_dev_ptr16(d_adst, num_arcs, "d_adst"))) return rc;
  if ((rc = check_dev_ptr16(d_akey, num_arcs, "d_akey"))) return rc;
  if (m && (!d_u || !d_v || !d_in_mst)) GHS_FAIL(GHS_E_ARG, "d_u/d_v/d_in_mst is NULL");
  const size_t need = workspace_layout(n, num_arcs, nullptr, nullptr);
  if (!d_workspace || workspace_bytes < need)
    GHS_FAIL(GHS_E_NOMEM, "workspace too small: need " + std::to_string(need) + " bytes");
  if (((uintptr_t)d_workspace) & 255) GHS_FAIL(GHS_E_ARG, "workspace must be 256-byte aligned");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) GHS_FAIL(GHS_E_NODEVICE, "no HIP device");

  ghs_solver *s = new ghs_solver();
  s->n = n; s->m = m; s->eu = d_u; s->ev = d_v;
  s->in_src = d_asrc; s->in_dst = d_adst; s->in_key = d_akey; s->num_arcs = num_arcs;
  s->in_mst = d_in_mst; s->stream = (hipStream_t)stream;
  workspace_layout(n, num_arcs, s, (char *)d_workspace);
  auto fail = [&](hipError_t e, const char *what) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    if (s->h_cnt) (void)hipHostFree(s->h_cnt);
    delete s;
    return GHS_E_HIP;
  };
  hipError_t e;
  if ((e = hipHostMalloc((void **)&s->h_cnt, 8 * sizeof(unsigned long long), hipHostMallocDefault)) != hipSuccess)
    return fail(e, "hipHostMalloc");
  if (n) {
    if ((e = hipMemsetAsync(s->best, 0xff, (size_t)n * 8, s->stream)) != hipSuccess) return fail(e, "memset best");
    k_iota<<<grid_for(n, 256, 8192), 256, 0, s->stream>>>(s->lab, n);
  }
  if (m && (e = hipMemsetAsync(s->in_mst, 0, m, s->stream)) != hipSuccess) return fail(e, "memset in_mst");
  if ((e = hipMemsetAsync(s->cnt, 0, 8 * sizeof(unsigned long long), s->stream)) != hipSuccess)
    return fail(e, "memset counters");
  if ((e = hipGetLastError()) != hipSuccess) return fail(e, "init kernels");
  s->cur_arcs = num_arcs;
  s->nact = n;
  s->act_ident = true;
  s->phase = n ? 0 : 2;
  s->t0 = std::chrono::steady_clock::now();
  *out = s;
  return GHS_OK;
}

static hipEvent_t round_event(ghs_solver *s, uint32_t round, int k) {
  if (round >= GHS_MAX_ROUND_STATS) return nullptr;
  const size_t idx = (size_t)round * 5 + k;
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

int ghs_solver_minedge(ghs_solver_t *s, uint64_t *num_active) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  if (s->phase == 2) {
    if (num_active) *num_active = 0;
    return GHS_OK;
  }
  if (s->phase != 0) GHS_FAIL(GHS_E_STATE, "minedge called twice without contract");
  if (s->round >= 64) GHS_FAIL(GHS_E_ROUNDCAP, "round cap exceeded");
  record(s, 0);
  const uint64_t A = s->cur_arcs;
  if (A) {
    const unsigned grid = grid_for(A, ARCS_PER_BLOCK, 8192);
    if (s->round == 0) {
      k_minedge<true, false><<<grid, BLOCK, 0, s->stream>>>(s->in_src, s->in_dst, s->in_key, A, s->lab, s->best,
                                                            nullptr, nullptr, nullptr, nullptr);
    } else {
      const int ob = (s->cur_buf == 0) ? 1 : 0;
      const uint32_t *isrc = s->cur_buf < 0 ? s->in_src : s->bsrc[s->cur_buf];
      const uint32_t *idst = s->cur_buf < 0 ? s->in_dst : s->bdst[s->cur_buf];
      const uint64_t *ikey = s->cur_buf < 0 ? s->in_key : s->bkey[s->cur_buf];
      GHS_HIP_CHECK(hipMemsetAsync(s->cnt, 0, sizeof(unsigned long long), s->stream));
      k_minedge<false, true><<<grid, BLOCK, 0, s->stream>>>(isrc, idst, ikey, A, s->lab, s->best, s->bsrc[ob],
                                                            s->bdst[ob], s->bkey[ob], s->cnt);
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
  k_hook<<<g, BLOCK, 0, s->stream>>>(act, nact, s->best, s->lab, s->eu, s->ev, s->par, s->in_mst, s->cnt + 2,
                                     s->cnt + 4);
  GHS_HIP_CHECK(hipGetLastError());
  record(s, 2);
  k_jump<<<g, BLOCK, 0, s->stream>>>(act, nact, s->par, s->lab, s->cnt + 4);
  GHS_HIP_CHECK(hipGetLastError());
  record(s, 3);
  const int nb = s->act_ident ? 0 : (s->act_cur ^ 1);
  k_flag_next<<<g, BLOCK, 0, s->stream>>>(act, nact, s->par, s->best, s->flags);
  GHS_HIP_CHECK(hipGetLastError());
  size_t cb = s->cub_bytes;
  if (act) {
    GHS_HIP_CHECK(hipcub::DeviceSelect::Flagged(s->cub_temp, cb, act, s->flags, s->act[nb], s->cnt + 1, (size_t)nact,
                                                s->stream));
  } else {
    GHS_HIP_CHECK(hipcub::DeviceSelect::Flagged(s->cub_temp, cb, hipcub::CountingInputIterator<uint32_t>(0u), s->flags,
                                                s->act[nb], s->cnt + 1, (size_t)nact, s->stream));
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
  st.live_arcs = s->cur_arcs;
  st.active_components = nact;
  st.hooks = s->h_cnt[3] - s->edges_before;
  s->edges_before = s->h_cnt[3];
  s->stats.push_back(st);

  // advance: arcs compacted this round (rounds >= 2) become next round's input
  if (s->round >= 1) {
    s->cur_buf = (s->cur_buf == 0) ? 1 : 0;
    s->cur_arcs = s->h_cnt[0];
  }
  s->act_cur = nb;
  s->act_ident = false;
  s->nact = s->h_cnt[1];
  s->round += 1;
  if (s->nact == 0) {
    s->phase = 2;
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
  const double ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - s->t0).count();
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
    result->ms_total = ms;
  }
  return GHS_OK;
}

int ghs_solver_destroy(ghs_solver_t *s) {
  if (!s) return GHS_OK;
  for (hipEvent_t e : s->ev_pool) (void)hipEventDestroy(e);
  if (s->h_cnt) (void)hipHostFree(s->h_cnt);
  delete s;
  return GHS_OK;
}

int ghs_mst_device(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_asrc,
                   const uint32_t *d_adst, const uint64_t *d_akey, uint64_t num_arcs, void *d_workspace,
                   size_t workspace_bytes, uint8_t *d_in_mst, void *stream, ghs_result_t *result,
                   ghs_round_stats_t *stats) {
  std::lock_guard<std::mutex> lock(g_mutex);
  ghs_solver_t *s = nullptr;
  int rc = ghs_solver_create(n, m, d_u, d_v, d_asrc, d_adst, d_akey, num_arcs, d_workspace, workspace_bytes,
                             d_in_mst, stream, &s);
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
