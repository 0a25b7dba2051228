// Single-process multi-GPU solve: one call drives N devices of one node as an RCCL clique
// (ncclCommInitAll), one host thread per device. This is the library form of the reference's
// MPI path (ghs_implementation_mpi.py:884-954: mpiexec -n <vertices> ranks exchanging pickled
// point-to-point messages, then Barrier + gather of the BRANCH edges to rank 0, :760-779) with
// one rank per GPU and the collectives of include/ghs_mst.h's stepwise protocol:
//   level open   flags (n fragment bits + error bit)     all-gather, OR on the device
//   every round  best keys of the active fragments       all-reduce MIN  (int64, key ^ 2^63)
//   level round 0 owner-computed hooks (par ^ fragment)  all-reduce MAX  (int32)
// Each device holds the replicated canonical list and owns the contiguous canonical-edge range
// [r*m/N, (r+1)*m/N) (4-aligned) — the same partition as the Python driver (distributed.py).
// Every device writes the MSF flags of its own range only; the result is their concatenation.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace {

struct DevRes {
  int dev = 0;
  hipStream_t stream = nullptr;
  void *canon = nullptr;       // u, v, w (replicated)
  void *ws = nullptr;          // solver workspace
  uint8_t *in_mst = nullptr;   // m flags (own range written)
  int64_t *dense = nullptr;    // all-reduce slots (<= n)
  int32_t *dense_hook = nullptr;
  uint64_t *gathered = nullptr;  // num_gpus x the level-open flag bitmap
  ghs_solver_t *solver = nullptr;
  ncclComm_t comm = nullptr;
  int rc = GHS_OK;
  std::string err;
  ghs_result_t result{};
  std::vector<ghs_round_stats_t> stats;
};

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

void edge_range(uint64_t m, int r, int N, uint64_t *lo, uint64_t *hi) {
  *lo = ((m * (uint64_t)r) / (uint64_t)N) & ~3ull;
  *hi = (r == N - 1) ? m : (((m * (uint64_t)(r + 1)) / (uint64_t)N) & ~3ull);
}

#define MULTI_HIP(expr)                                                                            \
  do {                                                                                             \
    hipError_t _e = (expr);                                                                        \
    if (_e != hipSuccess) {                                                                        \
      d.err = std::string(#expr) + ": " + hipGetErrorString(_e);                                   \
      return GHS_E_HIP;                                                                            \
    }                                                                                              \
  } while (0)
#define MULTI_NCCL(expr)                                                                           \
  do {                                                                                             \
    ncclResult_t _r = (expr);                                                                      \
    if (_r != ncclSuccess) {                                                                       \
      d.err = std::string(#expr) + ": " + ncclGetErrorString(_r);                                  \
      return GHS_E_HIP;                                                                            \
    }                                                                                              \
  } while (0)
#define MULTI_GHS(expr)                                                                            \
  do {                                                                                             \
    int _rc = (expr);                                                                              \
    if (_rc < 0) {                                                                                 \
      d.err = ghs_last_error();                                                                    \
      return _rc;                                                                                  \
    }                                                                                              \
  } while (0)

// setup on the device's thread: buffers, H2D copies of the canonical list, the solver
int setup(DevRes &d, int r, int N, uint32_t n, uint64_t m, const uint32_t *u, const uint32_t *v, const uint32_t *w,
          const ghs_config_t *cfg) {
  MULTI_HIP(hipSetDevice(d.dev));
  MULTI_HIP(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  uint64_t lo, hi;
  edge_range(m, r, N, &lo, &hi);
  const size_t cb = al256(m * 4);
  MULTI_HIP(hipMalloc(&d.canon, 3 * cb + 256));
  char *c = (char *)d.canon;
  if (m) {
    MULTI_HIP(hipMemcpyAsync(c, u, m * 4, hipMemcpyHostToDevice, d.stream));
    MULTI_HIP(hipMemcpyAsync(c + cb, v, m * 4, hipMemcpyHostToDevice, d.stream));
    MULTI_HIP(hipMemcpyAsync(c + 2 * cb, w, m * 4, hipMemcpyHostToDevice, d.stream));
  }
  const size_t wsb = ghs_workspace_bytes(n, m, hi - lo);
  MULTI_HIP(hipMalloc(&d.ws, wsb));
  MULTI_HIP(hipMalloc((void **)&d.in_mst, m ? m : 1));
  MULTI_HIP(hipMalloc((void **)&d.dense, ((size_t)n + 1) * 8));
  MULTI_HIP(hipMalloc((void **)&d.dense_hook, ((size_t)n + 1) * 4));
  MULTI_HIP(hipMalloc((void **)&d.gathered, (size_t)N * (((size_t)n + 1 + 63) / 64) * 8));
  ghs_config_t c2;
  if (cfg) c2 = *cfg; else ghs_default_config(&c2);
  c2.num_ranks = (uint32_t)N;
  MULTI_GHS(ghs_solver_create(n, m, (const uint32_t *)c, (const uint32_t *)(c + cb), (const uint32_t *)(c + 2 * cb),
                              lo, hi, &c2, d.ws, wsb, d.in_mst, d.stream, &d.solver));
  return GHS_OK;
}

// the round loop of one device (distributed.py run_rounds, in C++): every device makes the same
// sequence of collective calls because every device sees the same counts
int run(DevRes &d, uint64_t m, int r, int N, uint8_t *in_mst_out) {
  MULTI_HIP(hipSetDevice(d.dev));
  for (uint32_t guard = 0;; ++guard) {
    if (guard > 16 * GHS_MAX_ROUND_STATS) {
      d.err = "round cap exceeded";
      return GHS_E_ROUNDCAP;
    }
    uint64_t count = 0;
    int rc = ghs_solver_minedge(d.solver, &count);
    while (rc == GHS_NEED_EXCHANGE) {  // a level opened: OR its fragment flags (+ error bit)
      uint64_t *bits = nullptr;
      uint64_t words = 0;
      MULTI_GHS(ghs_solver_flag_bits(d.solver, &bits, &words));
      MULTI_NCCL(ncclAllGather(bits, d.gathered, words, ncclUint64, d.comm, d.stream));
      MULTI_GHS(ghs_solver_merge_flag_bits(d.solver, d.gathered, (uint32_t)N));
      rc = ghs_solver_minedge(d.solver, &count);
    }
    MULTI_GHS(rc);
    if (count) {
      MULTI_GHS(ghs_solver_pack_best(d.solver, d.dense));
      MULTI_NCCL(ncclAllReduce(d.dense, d.dense, count, ncclInt64, ncclMin, d.comm, d.stream));
      MULTI_GHS(ghs_solver_unpack_best(d.solver, d.dense));
      uint64_t hooks = 0;
      MULTI_GHS(ghs_solver_hook_local(d.solver, d.dense_hook, &hooks));
      if (hooks) {
        MULTI_NCCL(ncclAllReduce(d.dense_hook, d.dense_hook, hooks, ncclInt32, ncclMax, d.comm, d.stream));
        MULTI_GHS(ghs_solver_unpack_hook(d.solver, d.dense_hook));
      }
    }
    int done = 0;
    MULTI_GHS(ghs_solver_contract(d.solver, &done));
    if (done) break;
  }
  d.stats.assign(GHS_MAX_ROUND_STATS, ghs_round_stats_t{});
  MULTI_GHS(ghs_solver_finish(d.solver, &d.result, d.stats.data()));
  uint64_t lo, hi;
  edge_range(m, r, N, &lo, &hi);
  if (in_mst_out && hi > lo) {
    MULTI_HIP(hipMemcpyAsync(in_mst_out + lo, d.in_mst + lo, hi - lo, hipMemcpyDeviceToHost, d.stream));
    MULTI_HIP(hipStreamSynchronize(d.stream));
  }
  return GHS_OK;
}

void release(DevRes &d) {
  if (hipSetDevice(d.dev) != hipSuccess) return;
  if (d.solver) ghs_solver_destroy(d.solver);
  if (d.comm) ncclCommDestroy(d.comm);
  if (d.stream) (void)hipStreamSynchronize(d.stream);
  for (void *p : {d.canon, d.ws, (void *)d.in_mst, (void *)d.dense, (void *)d.dense_hook, (void *)d.gathered})
    if (p) (void)hipFree(p);
  if (d.stream) (void)hipStreamDestroy(d.stream);
}

}  // namespace

extern "C" int ghs_mst_multi(uint32_t n, uint64_t m, const uint32_t *u, const uint32_t *v, const uint32_t *w,
                             int num_gpus, const int *devices, const ghs_config_t *cfg, uint8_t *in_mst,
                             ghs_result_t *result, ghs_round_stats_t *stats) {
  if (num_gpus < 1) GHS_FAIL(GHS_E_ARG, "num_gpus must be >= 1");
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
  int prev = 0;
  (void)hipGetDevice(&prev);
  std::vector<DevRes> d(num_gpus);
  std::vector<ncclComm_t> comms(num_gpus);
  int rc = GHS_OK;
  std::string err;
  {
    const ncclResult_t nr = ncclCommInitAll(comms.data(), num_gpus, devs.data());
    if (nr != ncclSuccess) {
      rc = GHS_E_HIP;
      err = std::string("ncclCommInitAll: ") + ncclGetErrorString(nr);
    }
  }
  for (int i = 0; i < num_gpus; ++i) {
    d[i].dev = devs[i];
    d[i].comm = rc == GHS_OK ? comms[i] : nullptr;
  }
  // setup (threads: the H2D copies of the replicated list proceed in parallel)
  if (rc == GHS_OK) {
    std::vector<std::thread> th;
    for (int i = 0; i < num_gpus; ++i)
      th.emplace_back([&, i] { d[i].rc = setup(d[i], i, num_gpus, n, m, u, v, w, cfg); });
    for (auto &t : th) t.join();
    for (auto &x : d)
      if (x.rc && rc == GHS_OK) {
        rc = x.rc;
        err = x.err;
      }
  }
  // the solve: one thread per device, collectives in lock step
  if (rc == GHS_OK) {
    std::vector<std::thread> th;
    for (int i = 0; i < num_gpus; ++i) th.emplace_back([&, i] { d[i].rc = run(d[i], m, i, num_gpus, in_mst); });
    for (auto &t : th) t.join();
    for (auto &x : d)
      if (x.rc && rc == GHS_OK) {
        rc = x.rc;
        err = x.err;
      }
  }
  if (rc == GHS_OK) {
    for (int i = 1; i < num_gpus; ++i)
      if (d[i].result.total_weight != d[0].result.total_weight || d[i].result.num_mst_edges != d[0].result.num_mst_edges) {
        rc = GHS_E_STATE;
        err = "devices disagree on the MSF totals";
      }
  }
  if (rc == GHS_OK) {
    if (result) *result = d[0].result;
    if (stats) for (uint32_t i = 0; i < d[0].result.num_stats; ++i) stats[i] = d[0].stats[i];
  }
  for (auto &x : d) release(x);
  (void)hipSetDevice(prev);
  if (rc) GHS_FAIL(rc, err);
  return GHS_OK;
}
