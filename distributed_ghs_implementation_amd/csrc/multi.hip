// The multi-rank round loop in the library, and its drivers.
//
//   ghs_solver_run     one rank's whole solve: the stepwise protocol of include/ghs_mst.h with the
//                      collectives of a ghs_comm enqueued on the solver's own stream — the round
//                      loop that distributed.py run_rounds drives from Python, in one host call
//   ghs_comm_*         an RCCL communicator per rank (ncclCommInitRank from a unique id the caller
//                      broadcasts: one process per GPU, e.g. under torch.distributed)
//   ghs_mst_multi      one process driving N devices: an RCCL clique (ncclCommInitAll), one host
//                      thread per device, each running ghs_solver_run
//   ghs_mst_emulated   N ranks on ONE device with in-process collectives of the same semantics
//                      (test / diagnostic: the exact N-rank loop, checkable on one GPU)
//
// This is the library form of the reference's MPI path (ghs_implementation_mpi.py:884-954:
// mpiexec -n <vertices> ranks exchanging pickled point-to-point messages, then Barrier + gather of
// the BRANCH edges to rank 0, :760-779) with one rank per GPU and these collectives:
//   level open    flags (n fragment bits + error bit)     all-gather, OR on the device
//   level round 0 best keys of the dense fragments        reduce-scatter MIN (uint64, in place)
//                 the slot owners' hooks (eid, other)     all-gather (uint64)
//   later rounds  best keys of the active fragments       all-reduce MIN  (int64, key ^ 2^63)
//   (the stepwise protocol's level round 0 — all-reduce MIN of the slots, owner-computed hooks
//   as int32 MAX all-reduce — stays available to callers driving their own collectives)
// Each rank holds the replicated canonical list and owns the contiguous canonical-edge range
// [r*m/N, (r+1)*m/N) (4-aligned) — the same partition as the Python driver (device.py edge_range).
// Every rank writes the MSF flags of its own range only; the result is their concatenation.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <thread>
#include <vector>

#include "common.h"

namespace ghs {

// In-process collectives of ghs_mst_emulated: every rank's buffers live on the same device. A
// generation barrier; a rank that fails aborts the group so the others leave instead of waiting.
struct EmuGroup {
  explicit EmuGroup(int n) : nranks(n), ptrs(n, nullptr) {}
  int nranks;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<const void *> ptrs;
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return false;
    const uint64_t g = gen;
    if (++arrived == nranks) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    cv.wait(lk, [&] { return gen != g || aborted; });
    return !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
};

}  // namespace ghs

namespace {

__global__ void k_emu_min_i64(int64_t *__restrict__ dst, const int64_t *__restrict__ src, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i] < dst[i] ? src[i] : dst[i];
}
__global__ void k_emu_min_u64(uint64_t *__restrict__ dst, const uint64_t *__restrict__ src, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i] < dst[i] ? src[i] : dst[i];
}
__global__ void k_emu_sum_u64(uint64_t *__restrict__ dst, const uint64_t *__restrict__ src, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] += src[i];
}
__global__ void k_emu_max_i32(int32_t *__restrict__ dst, const int32_t *__restrict__ src, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i] > dst[i] ? src[i] : dst[i];
}

inline unsigned emu_grid(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return (unsigned)(g < 4096 ? (g ? g : 1) : 4096);
}

}  // namespace

struct ghs_comm {
  int nranks = 1, rank = 0, dev = 0;
  ncclComm_t nccl = nullptr;
  bool own_nccl = false;
  ghs::EmuGroup *emu = nullptr;
  int32_t *agree = nullptr;      // device int of the setup agreement (RCCL)
  int *group_cancel = nullptr;   // ghs_mst_multi: set by the first failing rank of the clique
  bool rs_hooks = true;          // dense level-opening rounds: reduce-scatter protocol (ABI 6)
  // device scratch of the loop (grown on demand)
  int64_t *dense = nullptr;
  int32_t *hook = nullptr;
  uint64_t *gathered = nullptr;
  uint64_t *pairs = nullptr;     // the reduce-scatter protocol's hook pairs (n + 64 slots)
  size_t dense_cap = 0, gathered_cap = 0, pairs_cap = 0;
};

namespace {

#define COMM_NCCL(expr)                                                                            \
  do {                                                                                             \
    ncclResult_t _r = (expr);                                                                      \
    if (_r != ncclSuccess) GHS_FAIL(GHS_E_HIP, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)
#define COMM_BARRIER(c)                                                                            \
  do {                                                                                             \
    if (!(c)->emu->barrier()) GHS_FAIL(GHS_E_STATE, "another rank of the emulated group failed");  \
  } while (0)

int comm_scratch(ghs_comm *c, uint32_t n) {
  const size_t slots = (size_t)n + 1, words = ((size_t)n + 1 + 63) / 64;
  if (c->dense_cap < slots) {
    if (c->dense) (void)hipFree(c->dense);
    if (c->hook) (void)hipFree(c->hook);
    c->dense = nullptr;
    c->hook = nullptr;
    c->dense_cap = 0;
    GHS_HIP_CHECK(hipMalloc((void **)&c->dense, slots * 8));
    GHS_HIP_CHECK(hipMalloc((void **)&c->hook, slots * 4));
    c->dense_cap = slots;
  }
  if (c->pairs_cap < slots + 64) {
    if (c->pairs) (void)hipFree(c->pairs);
    c->pairs = nullptr;
    c->pairs_cap = 0;
    GHS_HIP_CHECK(hipMalloc((void **)&c->pairs, (slots + 64) * 8));
    c->pairs_cap = slots + 64;
  }
  if (c->gathered_cap < words * c->nranks) {
    if (c->gathered) (void)hipFree(c->gathered);
    c->gathered = nullptr;
    c->gathered_cap = 0;
    GHS_HIP_CHECK(hipMalloc((void **)&c->gathered, words * c->nranks * 8));
    c->gathered_cap = words * c->nranks;
  }
  return GHS_OK;
}

int coll_allgather_u64(ghs_comm *c, const uint64_t *send, uint64_t *recv, size_t count, hipStream_t st) {
  if (c->nccl) {
    COMM_NCCL(ncclAllGather(send, recv, count, ncclUint64, c->nccl, st));
    return GHS_OK;
  }
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  c->emu->ptrs[c->rank] = send;
  COMM_BARRIER(c);
  for (int r = 0; r < c->nranks; ++r)  // (an in-place gather's own slice is already there)
    if (recv + (size_t)r * count != c->emu->ptrs[r] && count)
      GHS_HIP_CHECK(hipMemcpyAsync(recv + (size_t)r * count, c->emu->ptrs[r], count * 8, hipMemcpyDeviceToDevice, st));
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  COMM_BARRIER(c);  // every rank has read every send buffer
  return GHS_OK;
}

// in-place MIN reduce-scatter over uint64: buf holds nranks x per slots; rank r keeps slice r
int coll_reducescatter_min_u64(ghs_comm *c, uint64_t *buf, size_t per, hipStream_t st) {
  if (c->nccl) {
    COMM_NCCL(ncclReduceScatter(buf, buf + (size_t)c->rank * per, per, ncclUint64, ncclMin, c->nccl, st));
    return GHS_OK;
  }
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  c->emu->ptrs[c->rank] = buf;
  COMM_BARRIER(c);
  uint64_t *mine = buf + (size_t)c->rank * per;  // every rank reduces its own slice from the others
  for (int r = 0; r < c->nranks; ++r)
    if (r != c->rank && per)
      k_emu_min_u64<<<emu_grid(per), 256, 0, st>>>(mine, (const uint64_t *)c->emu->ptrs[r] + (size_t)c->rank * per, per);
  GHS_HIP_CHECK(hipGetLastError());
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  COMM_BARRIER(c);  // every rank has read every buffer
  return GHS_OK;
}

// in-place all-reduce: MIN over int64 or uint64, MAX over int32
template <typename T>
int coll_allreduce(ghs_comm *c, T *buf, size_t count, hipStream_t st) {
  constexpr bool is_min = sizeof(T) == 8;
  constexpr bool is_u64 = std::is_same<T, uint64_t>::value;
  if (c->nccl) {
    COMM_NCCL(ncclAllReduce(buf, buf, count, is_u64 ? ncclUint64 : (is_min ? ncclInt64 : ncclInt32),
                            is_min ? ncclMin : ncclMax, c->nccl, st));
    return GHS_OK;
  }
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  c->emu->ptrs[c->rank] = buf;
  COMM_BARRIER(c);
  if (c->rank == 0) {  // rank 0 reduces every buffer into its own
    for (int r = 1; r < c->nranks; ++r) {
      if (is_u64)
        k_emu_min_u64<<<emu_grid(count), 256, 0, st>>>((uint64_t *)buf, (const uint64_t *)c->emu->ptrs[r], count);
      else if (is_min)
        k_emu_min_i64<<<emu_grid(count), 256, 0, st>>>((int64_t *)buf, (const int64_t *)c->emu->ptrs[r], count);
      else
        k_emu_max_i32<<<emu_grid(count), 256, 0, st>>>((int32_t *)buf, (const int32_t *)c->emu->ptrs[r], count);
    }
    GHS_HIP_CHECK(hipGetLastError());
    GHS_HIP_CHECK(hipStreamSynchronize(st));
  }
  COMM_BARRIER(c);
  if (c->rank != 0) {
    GHS_HIP_CHECK(hipMemcpyAsync(buf, c->emu->ptrs[0], count * sizeof(T), hipMemcpyDeviceToDevice, st));
    GHS_HIP_CHECK(hipStreamSynchronize(st));
  }
  COMM_BARRIER(c);  // rank 0's buffer is free again
  return GHS_OK;
}

// in-place SUM all-reduce over uint64 (the reduce-scatter round's partial totals: 2 words)
int coll_allreduce_sum_u64(ghs_comm *c, uint64_t *buf, size_t count, hipStream_t st) {
  if (c->nccl) {
    COMM_NCCL(ncclAllReduce(buf, buf, count, ncclUint64, ncclSum, c->nccl, st));
    return GHS_OK;
  }
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  c->emu->ptrs[c->rank] = buf;
  COMM_BARRIER(c);
  if (c->rank == 0) {
    for (int r = 1; r < c->nranks; ++r)
      k_emu_sum_u64<<<1, 64, 0, st>>>(buf, (const uint64_t *)c->emu->ptrs[r], count);
    GHS_HIP_CHECK(hipGetLastError());
    GHS_HIP_CHECK(hipStreamSynchronize(st));
  }
  COMM_BARRIER(c);
  if (c->rank != 0) {
    GHS_HIP_CHECK(hipMemcpyAsync(buf, c->emu->ptrs[0], count * 8, hipMemcpyDeviceToDevice, st));
    GHS_HIP_CHECK(hipStreamSynchronize(st));
  }
  COMM_BARRIER(c);
  return GHS_OK;
}

// Setup agreement, before a rank's first collective: every rank contributes its setup status and
// learns whether any rank failed (int32 MAX over RCCL; the emulated group's barrier). A rank whose
// workspace allocation or copy failed thereby fails the call on every rank instead of leaving the
// others blocked in the level-open all-gather. Returns GHS_OK or this rank's error (its own, or
// GHS_E_STATE for a peer's).
int comm_agree(ghs_comm *c, int local_rc, hipStream_t st) {
  if (c->emu) {
    if (local_rc) {
      c->emu->abort();
      return local_rc;
    }
    COMM_BARRIER(c);
    return GHS_OK;
  }
  if (!c->nccl || !c->agree) return local_rc;
  const int32_t mine = local_rc ? 1 : 0;
  int32_t any = 1;
  GHS_HIP_CHECK(hipMemcpyAsync(c->agree, &mine, 4, hipMemcpyHostToDevice, st));
  COMM_NCCL(ncclAllReduce(c->agree, c->agree, 1, ncclInt32, ncclMax, c->nccl, st));
  GHS_HIP_CHECK(hipMemcpyAsync(&any, c->agree, 4, hipMemcpyDeviceToHost, st));
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  if (local_rc) return local_rc;
  if (any) GHS_FAIL(GHS_E_STATE, "another rank failed during setup");
  return GHS_OK;
}

// A rank's solve failed mid-loop: tell the rest of the clique (its waits end: solver_sync polls
// the group flag) and abort this rank's communicator, which ends its RCCL kernels still waiting
// for peers, so its stream drains; the handle is not destroyed again afterwards.
int loop_fail(ghs_comm *c, int rc) {
  if (!c) return rc;
  if (c->group_cancel) __atomic_store_n(c->group_cancel, 1, __ATOMIC_RELEASE);
  if (c->emu) c->emu->abort();
  if (c->nccl) {
    (void)ncclCommAbort(c->nccl);
    c->nccl = nullptr;
  }
  return rc;
}

#define LOOP_CHECK(expr)                  \
  do {                                    \
    const int _rc = (expr);               \
    if (_rc < 0) return loop_fail(c, _rc); \
  } while (0)

int run_loop(ghs_solver_t *s, ghs_comm *c) {
  const uint32_t nr = ghs_solver_ranks_of(s);
  const bool multi = nr > 1;
  hipStream_t st = ghs_solver_stream_of(s);
  if (multi) {
    if (hipSetDevice(c->dev) != hipSuccess) {
      ghs::set_error("hipSetDevice of the communicator's device failed");
      return loop_fail(c, GHS_E_HIP);
    }
    LOOP_CHECK(comm_scratch(c, ghs_solver_n_of(s)));
  }
  const ghs_config_t *cf = ghs_solver_cfg_of(s);
  const GhsTailColl tcoll{c,
                          [](void *x, uint64_t *b, size_t n, hipStream_t q) {
                            return coll_allreduce<uint64_t>(static_cast<ghs_comm *>(x), b, n, q);
                          },
                          [](void *x, int32_t *b, size_t n, hipStream_t q) {
                            return coll_allreduce<int32_t>(static_cast<ghs_comm *>(x), b, n, q);
                          }};
  for (uint32_t guard = 0;; ++guard) {
    if (guard > 16 * GHS_MAX_ROUND_STATS) {
      ghs::set_error("round cap exceeded");
      return loop_fail(c, GHS_E_ROUNDCAP);
    }
    // test hook (ghs_config_t.fault_round): this rank fails between rounds while its peers go on
    // into the next collective — their waits must end through the group's cancel path
    if (multi && cf->fault_round && cf->fault_rank == (uint32_t)c->rank + 1 && ghs_solver_round_of(s) >= cf->fault_round) {
      ghs::set_error("injected mid-solve failure (fault_round)");
      return loop_fail(c, GHS_E_STATE);
    }
    if (multi) {  // a dense level's last rounds in the LDS tail (few active fragments)
      const int t = ghs_solver_tail_multi(s, &tcoll);
      if (t < 0) return loop_fail(c, t);
      if (t == 2) return GHS_OK;
      if (t == 1) continue;
    }
    uint64_t count = 0;
    int rc = ghs_solver_minedge(s, &count);
    while (rc == GHS_NEED_EXCHANGE) {  // a level opened: OR its fragment flags (+ error bit)
      uint64_t *bits = nullptr;
      uint64_t words = 0;
      LOOP_CHECK(c->nccl ? ghs_solver_flag_bits_async(s, &bits, &words) : ghs_solver_flag_bits(s, &bits, &words));
      LOOP_CHECK(coll_allgather_u64(c, bits, c->gathered, words, st));
      LOOP_CHECK(ghs_solver_merge_flag_bits(s, c->gathered, nr));
      rc = ghs_solver_minedge(s, &count);
    }
    LOOP_CHECK(rc);
    uint64_t *hs = nullptr, S = 0;
    if (multi && count && c->rs_hooks) LOOP_CHECK(ghs_solver_hook_slots(s, nr, &hs, &S));
    if (S) {
      // a dense level's opening round: reduce-scatter of the best slots, owner-computed hooks,
      // all-gather of the (eid, other) pairs — 16 instead of 24 ring bytes per slot
      const uint64_t per = S / nr;
      LOOP_CHECK(coll_reducescatter_min_u64(c, hs, per, st));
      LOOP_CHECK(ghs_solver_hook_owner(s, (uint32_t)c->rank, per, c->pairs));
      LOOP_CHECK(coll_allgather_u64(c, c->pairs + (size_t)c->rank * per, c->pairs, per, st));
      uint64_t *partial = nullptr;
      LOOP_CHECK(ghs_solver_apply_hooks(s, c->pairs, &partial));
      LOOP_CHECK(coll_allreduce_sum_u64(c, partial, 2, st));
    } else if (multi && count) {
      if (uint64_t *slots = ghs_solver_best_slots_of(s)) {  // a dense level's first round: best in place
        LOOP_CHECK(coll_allreduce<uint64_t>(c, slots, count, st));
      } else {
        LOOP_CHECK(ghs_solver_pack_best(s, c->dense));
        LOOP_CHECK(coll_allreduce<int64_t>(c, c->dense, count, st));
        LOOP_CHECK(ghs_solver_unpack_best(s, c->dense));
      }
      uint64_t hooks = 0;
      LOOP_CHECK(ghs_solver_hook_local(s, c->hook, &hooks));
      if (hooks) {
        LOOP_CHECK(coll_allreduce<int32_t>(c, c->hook, hooks, st));
        LOOP_CHECK(ghs_solver_unpack_hook(s, c->hook));
      }
    }
    int done = 0;
    LOOP_CHECK(ghs_solver_contract_async(s, &done));
    if (done) return GHS_OK;
  }
}

void comm_free(ghs_comm *c) {
  if (!c) return;
  if (hipSetDevice(c->dev) == hipSuccess) {
    for (void *p : {(void *)c->dense, (void *)c->hook, (void *)c->gathered, (void *)c->agree, (void *)c->pairs})
      if (p) (void)hipFree(p);
  }
  if (c->nccl && c->own_nccl) ncclCommDestroy(c->nccl);
  delete c;
}

// the ranks' edge ranges balanced by the cost density 1 + RANGE_BETA * (1 - e / m) over the canonical
// list — the closed form of device.py range_split / edge_range (see there), 4-aligned
#ifndef GHS_RANGE_BETA
#define GHS_RANGE_BETA 0.2
#endif
uint64_t range_split(uint64_t m, int k, int N) {
  const double b = GHS_RANGE_BETA;
  if (k <= 0) return 0;
  if (k >= N) return m;
  if (b == 0.0) return ((m * (uint64_t)k) / (uint64_t)N) & ~3ull;
  const double t = (double)k / (double)N * (1.0 + b / 2.0);
  const double x = ((1.0 + b) - std::sqrt((1.0 + b) * (1.0 + b) - 2.0 * b * t)) / b;
  const uint64_t e = (uint64_t)(x * (double)m);
  return (e < m ? e : m) & ~3ull;
}
void edge_range(uint64_t m, int r, int N, uint64_t *lo, uint64_t *hi) {
  *lo = range_split(m, r, N);
  *hi = (r == N - 1) ? m : range_split(m, r + 1, N);
  if (*hi < *lo) *hi = *lo;
}

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// The drivers' per-rank state, kept across calls (ghs_release_cache): a rank's stream, workspace,
// replicated canonical copy and flags (ghs_mst_multi), and pinned report ring — a call of the same
// shape then allocates nothing. Per-call allocation of ~N workspaces (s26 x 8 emulated: 8 x ~11 GB)
// was the suspected cause of the multi-second emulated calls of round 3.
struct RankState {
  int dev = 0;
  hipStream_t stream = nullptr;
  void *canon = nullptr;       // ghs_mst_multi: u, v, w replicated per device
  void *ws = nullptr;
  size_t ws_bytes = 0;
  uint8_t *in_mst = nullptr;   // ghs_mst_multi: m flags per device (own range written)
  void *hostres = nullptr;     // pinned counters / report ring / events of the rank's solver
};

// one rank of a driver call: its cached state, this call's solver and outcome
struct Rank {
  RankState *st = nullptr;
  ghs_solver_t *solver = nullptr;
  ghs_comm *comm = nullptr;
  int rc = GHS_OK;
  std::string err;
  ghs_result_t result{};
  std::vector<ghs_round_stats_t> stats;
  double ms_setup = 0, ms_solve = 0, ms_gather = 0;
};

struct DriverCache {
  int kind = 0;  // 1 = ghs_mst_multi, 2 = ghs_mst_emulated
  std::vector<int> devs;
  uint32_t n = 0;
  uint64_t m = 0;
  std::vector<RankState> ranks;
  std::vector<ghs_comm> comms;  // ghs_mst_multi's clique (nccl) and both drivers' collective scratch
};
std::mutex g_drv_mu;           // one driver call at a time per process (they share the cache)
DriverCache *g_drv = nullptr;

void cache_free(DriverCache *c) {
  if (!c) return;
  for (RankState &x : c->ranks) {
    if (hipSetDevice(x.dev) != hipSuccess) continue;
    if (x.stream) (void)hipStreamSynchronize(x.stream);
    for (void *p : {x.canon, x.ws, (void *)x.in_mst})
      if (p) (void)hipFree(p);
    if (x.stream) (void)hipStreamDestroy(x.stream);
    ghs_hostres_delete(x.hostres);
  }
  for (ghs_comm &k : c->comms) {
    if (hipSetDevice(k.dev) != hipSuccess) continue;
    if (k.nccl) ncclCommDestroy(k.nccl);  // (one aborted by loop_fail was nulled there)
    k.nccl = nullptr;
    for (void *p : {(void *)k.dense, (void *)k.hook, (void *)k.gathered, (void *)k.agree, (void *)k.pairs})
      if (p) (void)hipFree(p);
  }
  delete c;
}

// the cache of this call's shape (g_drv_mu held): the one kept from an earlier call of the same
// shape, or a fresh one (another shape's is freed first: one shape's state at a time)
DriverCache *cache_acquire(int kind, const std::vector<int> &devs, uint32_t n, uint64_t m, bool *reused) {
  if (g_drv && g_drv->kind == kind && g_drv->devs == devs && g_drv->n == n && g_drv->m == m) {
    *reused = true;
    return g_drv;
  }
  cache_free(g_drv);
  g_drv = new DriverCache;
  g_drv->kind = kind;
  g_drv->devs = devs;
  g_drv->n = n;
  g_drv->m = m;
  const int N = (int)devs.size();
  g_drv->ranks.resize(N);
  g_drv->comms.resize(N);
  for (int i = 0; i < N; ++i) {
    g_drv->ranks[i].dev = devs[i];
    g_drv->comms[i].nranks = N;
    g_drv->comms[i].rank = i;
    g_drv->comms[i].dev = devs[i];
  }
  *reused = false;
  return g_drv;
}

// after a call: a failed call leaves no state behind (aborted communicators, cancelled solvers),
// and a successful one keeps it only when the caller asked (GHS_OPT_KEEP_CACHE): the cached
// workspaces are invisible to the caller's allocator (s26 x 8 emulated: ~8 x 11 GB on one device)
void cache_release_on(int rc, const ghs_config_t *cfg) {
  const bool keep = rc == GHS_OK && cfg && (cfg->options & GHS_OPT_KEEP_CACHE);
  if (keep || !g_drv) return;
  cache_free(g_drv);
  g_drv = nullptr;
}

inline double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int rank_fail(Rank &d, int rc) {
  d.rc = rc;
  d.err = ghs_last_error();
  if (d.comm && d.comm->emu) d.comm->emu->abort();
  if (d.comm && d.comm->group_cancel) __atomic_store_n(d.comm->group_cancel, 1, __ATOMIC_RELEASE);
  return rc;
}

// create the rank's solver over device-resident u/v/w (workspace and pinned resources from the
// cache, allocated on first use), agree with the other ranks that every setup succeeded, and run it
// to completion. setup_rc: the driver's own setup of this rank (stream, copies) — a failed rank
// still joins the agreement, so its peers leave too. t0: the rank's start (phase times).
int rank_solve(Rank &d, int r, int N, uint32_t n, uint64_t m, const uint32_t *du, const uint32_t *dv,
               const uint32_t *dw, uint8_t *d_in_mst, const ghs_config_t *cfg, int setup_rc,
               std::chrono::steady_clock::time_point t0) {
  RankState &x = *d.st;
  int rc = setup_rc;
  uint64_t lo, hi;
  edge_range(m, r, N, &lo, &hi);
  const size_t wsb = ghs_workspace_bytes(n, m, hi - lo);
  ghs_config_t c2;
  if (cfg) c2 = *cfg; else ghs_default_config(&c2);
  c2.num_ranks = (uint32_t)N;
  if (!rc && hipSetDevice(x.dev) != hipSuccess) {
    ghs::set_error("hipSetDevice failed");
    rc = GHS_E_HIP;
  }
  if (!rc && c2.fault_rank && c2.fault_round && N == 1) {  // a one-rank loop has no round exchange to fail in
    ghs::set_error("fault_round needs num_ranks > 1");
    rc = GHS_E_ARG;
  }
  if (!rc && c2.fault_rank == (uint32_t)r + 1 && c2.fault_round == 0) {  // test hook (ghs_config_t.fault_rank)
    ghs::set_error("injected setup failure (fault_rank)");
    rc = GHS_E_NOMEM;
  }
  if (!rc && x.ws_bytes < wsb) {
    if (x.ws) (void)hipFree(x.ws);
    x.ws = nullptr;
    x.ws_bytes = 0;
    if (hipMalloc(&x.ws, wsb) != hipSuccess) {
      ghs::set_error("hipMalloc of a rank workspace failed");
      rc = GHS_E_NOMEM;
    } else {
      x.ws_bytes = wsb;
    }
  }
  if (!rc && !x.hostres) x.hostres = ghs_hostres_new(&rc);
  if (!rc) rc = ghs_solver_create_pooled(n, m, du, dv, dw, lo, hi, &c2, x.ws, x.ws_bytes, d_in_mst, x.stream, x.hostres,
                                         &d.solver);
  if (rc < 0) d.err = ghs_last_error();
  const int agreed = comm_agree(d.comm, rc < 0 ? rc : GHS_OK, x.stream);
  d.ms_setup = ms_since(t0);
  if (agreed < 0) {
    if (!rc) d.err = ghs_last_error();
    d.rc = agreed;
    if (d.comm && d.comm->group_cancel) __atomic_store_n(d.comm->group_cancel, 1, __ATOMIC_RELEASE);
    return agreed;
  }
  const auto t1 = std::chrono::steady_clock::now();
  rc = ghs_solver_run(d.solver, d.comm);
  if (rc < 0) return rank_fail(d, rc);
  d.stats.assign(GHS_MAX_ROUND_STATS, ghs_round_stats_t{});
  rc = ghs_solver_finish(d.solver, &d.result, d.stats.data());
  d.ms_solve = ms_since(t1);
  if (rc < 0) return rank_fail(d, rc);
  return GHS_OK;
}

// the call's solver goes; the rank's cached state stays (its stream drained)
void rank_detach(Rank &d) {
  if (!d.st || hipSetDevice(d.st->dev) != hipSuccess) return;
  if (d.solver) ghs_solver_destroy(d.solver);
  d.solver = nullptr;
  if (d.st->stream) (void)hipStreamSynchronize(d.st->stream);
}

// a rank's error that only reports another rank's failure (a cancelled wait, a failed agreement)
bool peer_error(const Rank &x) {
  return x.rc == GHS_E_STATE && (x.err.rfind("cancelled", 0) == 0 || x.err.rfind("another rank", 0) == 0);
}

// the first failing rank's own error (over those that only saw a peer fail), then the totals agree
// on every rank; the host phase times are the maxima over the ranks
int collect(std::vector<Rank> &d, bool reused, ghs_result_t *result, ghs_round_stats_t *stats, std::string *err) {
  for (auto &x : d)
    if (x.rc && !peer_error(x)) {
      *err = x.err;
      return x.rc;
    }
  for (auto &x : d)
    if (x.rc) {
      *err = x.err;
      return x.rc;
    }
  for (size_t i = 1; i < d.size(); ++i)
    if (d[i].result.total_weight != d[0].result.total_weight || d[i].result.num_mst_edges != d[0].result.num_mst_edges) {
      *err = "ranks disagree on the MSF totals";
      return GHS_E_STATE;
    }
  if (result) {
    *result = d[0].result;
    result->ms_setup = result->ms_solve = result->ms_gather = 0;
    for (auto &x : d) {
      result->ms_setup = std::max(result->ms_setup, x.ms_setup);
      result->ms_solve = std::max(result->ms_solve, x.ms_solve);
      result->ms_gather = std::max(result->ms_gather, x.ms_gather);
    }
    result->reused = reused ? 1u : 0u;
  }
  if (stats)
    for (uint32_t i = 0; i < d[0].result.num_stats; ++i) stats[i] = d[0].stats[i];
  return GHS_OK;
}

}  // namespace

extern "C" int ghs_comm_unique_id(uint8_t *id) {
  if (!id) GHS_FAIL(GHS_E_ARG, "id is NULL");
  static_assert(sizeof(ncclUniqueId) == GHS_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId u;
  COMM_NCCL(ncclGetUniqueId(&u));
  memcpy(id, &u, GHS_COMM_ID_BYTES);
  return GHS_OK;
}

extern "C" int ghs_comm_init(int nranks, int rank, const uint8_t *id, ghs_comm_t **out) {
  if (!out || !id || nranks < 1 || nranks > GHS_MAX_RANKS || rank < 0 || rank >= nranks)
    GHS_FAIL(GHS_E_ARG, "bad communicator arguments");
  *out = nullptr;
  ghs_comm *c = new ghs_comm;
  c->nranks = nranks;
  c->rank = rank;
  if (hipGetDevice(&c->dev) != hipSuccess) {
    delete c;
    GHS_FAIL(GHS_E_NODEVICE, "no current HIP device");
  }
  ncclUniqueId u;
  memcpy(&u, id, GHS_COMM_ID_BYTES);
  const ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    GHS_FAIL(GHS_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  c->own_nccl = true;
  if (hipMalloc((void **)&c->agree, 4) != hipSuccess) {
    ncclCommDestroy(c->nccl);
    delete c;
    GHS_FAIL(GHS_E_NOMEM, "hipMalloc of the communicator's agreement word failed");
  }
  *out = c;
  return GHS_OK;
}

extern "C" int ghs_comm_destroy(ghs_comm_t *comm) {
  comm_free(comm);
  return GHS_OK;
}

extern "C" int ghs_solver_run(ghs_solver_t *s, ghs_comm_t *comm) {
  if (!s) GHS_FAIL(GHS_E_ARG, "solver is NULL");
  const uint32_t nr = ghs_solver_ranks_of(s);
  if (nr > 1 && (!comm || comm->nranks != (int)nr))
    GHS_FAIL(GHS_E_ARG, "a solver of " + std::to_string(nr) + " ranks needs a communicator of as many ranks");
  if (nr > 1 && !comm->nccl && !comm->emu) GHS_FAIL(GHS_E_STATE, "the communicator was aborted by an earlier failure");
  if (comm && comm->group_cancel) ghs_solver_set_group_cancel(s, comm->group_cancel);
  int prev = 0;
  const bool have_prev = hipGetDevice(&prev) == hipSuccess;
  const int rc = run_loop(s, comm);
  if (have_prev) (void)hipSetDevice(prev);  // the caller's current device, as it was
  return rc;
}

extern "C" int ghs_mst_multi(uint32_t n, uint64_t m, const uint32_t *u, const uint32_t *v, const uint32_t *w,
                             int num_gpus, const int *devices, const ghs_config_t *cfg, uint8_t *in_mst,
                             ghs_result_t *result, ghs_round_stats_t *stats) {
  if (num_gpus < 1 || num_gpus > GHS_MAX_RANKS) GHS_FAIL(GHS_E_ARG, "num_gpus must be in [1, GHS_MAX_RANKS]");
  if (m && (!u || !v || !w || !in_mst)) GHS_FAIL(GHS_E_ARG, "NULL host pointer");
  if (m >= (1ull << 31)) GHS_FAIL(GHS_E_ARG, "m must be < 2^31");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) GHS_FAIL(GHS_E_NODEVICE, "no HIP device");
  std::vector<int> devs(num_gpus);
  for (int i = 0; i < num_gpus; ++i) {
    devs[i] = devices ? devices[i] : i;
    if (devs[i] < 0 || devs[i] >= ndev) GHS_FAIL(GHS_E_ARG, "device " + std::to_string(devs[i]) + " not visible");
    for (int j = 0; j < i; ++j)
      if (devs[j] == devs[i]) GHS_FAIL(GHS_E_ARG, "devices must be distinct (one rank per GPU)");
  }
  std::lock_guard<std::mutex> lock(g_drv_mu);
  const auto t0 = std::chrono::steady_clock::now();
  int prev = 0;
  (void)hipGetDevice(&prev);
  bool reused = false;
  DriverCache *C = cache_acquire(1, devs, n, m, &reused);
  std::vector<Rank> d(num_gpus);
  int rc = GHS_OK;
  std::string err;
  if (!C->comms[0].nccl) {  // a fresh cache: the clique (kept with the cache)
    std::vector<ncclComm_t> nc(num_gpus, nullptr);
    const ncclResult_t nr = ncclCommInitAll(nc.data(), num_gpus, devs.data());
    if (nr != ncclSuccess) {
      rc = GHS_E_HIP;
      err = std::string("ncclCommInitAll: ") + ncclGetErrorString(nr);
    } else {
      for (int i = 0; i < num_gpus; ++i) C->comms[i].nccl = nc[i];
    }
  }
  int group_failed = 0;  // set by the first failing rank: the others' waits end (solver_sync)
  for (int i = 0; i < num_gpus; ++i) {
    ghs_comm &k = C->comms[i];
    k.own_nccl = false;
    k.group_cancel = &group_failed;
    d[i].st = &C->ranks[i];
    d[i].comm = &k;
    if (rc == GHS_OK && !k.agree && (hipSetDevice(devs[i]) != hipSuccess || hipMalloc((void **)&k.agree, 4) != hipSuccess)) {
      rc = GHS_E_NOMEM;
      err = "hipMalloc of the setup-agreement word failed";
    }
  }
  if (rc == GHS_OK) {
    // one thread per device: stream, H2D copies of the replicated list, then the solve (the
    // collectives in lock step); the copies of the devices proceed in parallel
    std::vector<std::thread> th;
    for (int i = 0; i < num_gpus; ++i)
      th.emplace_back([&, i] {
        Rank &x = d[i];
        RankState &st = *x.st;
        // setup errors are carried into rank_solve, whose agreement fails every rank together
        int setup = GHS_OK;
        const size_t cb = al256(m * 4);
        if (hipSetDevice(st.dev) != hipSuccess ||
            (!st.stream && hipStreamCreateWithFlags(&st.stream, hipStreamNonBlocking) != hipSuccess)) {
          ghs::set_error("device setup failed");
          setup = GHS_E_HIP;
        } else if ((!st.canon && hipMalloc(&st.canon, 3 * cb + 256) != hipSuccess) ||
                   (!st.in_mst && hipMalloc((void **)&st.in_mst, m ? m : 1) != hipSuccess)) {
          ghs::set_error("hipMalloc of the device's canonical copy failed");
          setup = GHS_E_NOMEM;
        } else {
          const char *c = (const char *)st.canon;
          if (m && (hipMemcpyAsync((void *)c, u, m * 4, hipMemcpyHostToDevice, st.stream) != hipSuccess ||
                    hipMemcpyAsync((void *)(c + cb), v, m * 4, hipMemcpyHostToDevice, st.stream) != hipSuccess ||
                    hipMemcpyAsync((void *)(c + 2 * cb), w, m * 4, hipMemcpyHostToDevice, st.stream) != hipSuccess)) {
            ghs::set_error("H2D copy of the canonical list failed");
            setup = GHS_E_HIP;
          }
        }
        const char *c = (const char *)st.canon;
        if (rank_solve(x, i, num_gpus, n, m, (const uint32_t *)c, (const uint32_t *)(c ? c + cb : nullptr),
                       (const uint32_t *)(c ? c + 2 * cb : nullptr), st.in_mst, cfg, setup, t0))
          return;
        const auto t2 = std::chrono::steady_clock::now();
        uint64_t lo, hi;
        edge_range(m, i, num_gpus, &lo, &hi);
        if (hi > lo && (hipMemcpyAsync(in_mst + lo, st.in_mst + lo, hi - lo, hipMemcpyDeviceToHost, st.stream) != hipSuccess ||
                        hipStreamSynchronize(st.stream) != hipSuccess)) {
          ghs::set_error("D2H copy of the flags failed");
          rank_fail(x, GHS_E_HIP);
        }
        x.ms_gather = ms_since(t2);
      });
    for (auto &t : th) t.join();
    rc = collect(d, reused, result, stats, &err);
  }
  for (auto &x : d) rank_detach(x);
  for (ghs_comm &k : C->comms) k.group_cancel = nullptr;
  cache_release_on(rc, cfg);
  (void)hipSetDevice(prev);
  if (rc) GHS_FAIL(rc, err);
  return GHS_OK;
}

extern "C" int ghs_mst_emulated(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                                int num_ranks, const ghs_config_t *cfg, uint8_t *d_in_mst, ghs_result_t *result,
                                ghs_round_stats_t *stats) {
  if (num_ranks < 1 || num_ranks > GHS_MAX_RANKS) GHS_FAIL(GHS_E_ARG, "num_ranks must be in [1, GHS_MAX_RANKS]");
  if (m && (!d_u || !d_v || !d_w || !d_in_mst)) GHS_FAIL(GHS_E_ARG, "NULL device pointer");
  if (m >= (1ull << 31)) GHS_FAIL(GHS_E_ARG, "m must be < 2^31");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) GHS_FAIL(GHS_E_NODEVICE, "no current HIP device");
  std::lock_guard<std::mutex> lock(g_drv_mu);
  const auto t0 = std::chrono::steady_clock::now();
  bool reused = false;
  DriverCache *C = cache_acquire(2, std::vector<int>(num_ranks, dev), n, m, &reused);
  ghs::EmuGroup group(num_ranks);
  std::vector<Rank> d(num_ranks);
  int group_failed = 0;
  for (int i = 0; i < num_ranks; ++i) {
    C->comms[i].emu = &group;
    C->comms[i].group_cancel = &group_failed;
    d[i].st = &C->ranks[i];
    d[i].comm = &C->comms[i];
  }
  std::vector<std::thread> th;
  for (int i = 0; i < num_ranks; ++i)
    th.emplace_back([&, i] {
      Rank &x = d[i];
      RankState &st = *x.st;
      int setup = GHS_OK;
      if (hipSetDevice(dev) != hipSuccess ||
          (!st.stream && hipStreamCreateWithFlags(&st.stream, hipStreamNonBlocking) != hipSuccess)) {
        ghs::set_error("stream creation failed");
        setup = GHS_E_HIP;
      }
      if (rank_solve(x, i, num_ranks, n, m, d_u, d_v, d_w, d_in_mst, cfg, setup, t0)) return;
      const auto t2 = std::chrono::steady_clock::now();
      if (hipStreamSynchronize(st.stream) != hipSuccess) {
        ghs::set_error("stream sync failed");
        rank_fail(x, GHS_E_HIP);
      }
      x.ms_gather = ms_since(t2);
    });
  for (auto &t : th) t.join();
  std::string err;
  const int rc = collect(d, reused, result, stats, &err);
  for (auto &x : d) rank_detach(x);
  for (ghs_comm &k : C->comms) {
    k.emu = nullptr;
    k.group_cancel = nullptr;
  }
  cache_release_on(rc, cfg);
  (void)hipSetDevice(dev);
  if (rc) GHS_FAIL(rc, err);
  return GHS_OK;
}

extern "C" int ghs_release_cache(void) {
  std::lock_guard<std::mutex> lock(g_drv_mu);
  int prev = 0;
  const bool have = hipGetDevice(&prev) == hipSuccess;
  cache_free(g_drv);
  g_drv = nullptr;
  if (have) (void)hipSetDevice(prev);
  ghs_release_eid_temps();
  return GHS_OK;
}
