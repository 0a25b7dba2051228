// TEST-ONLY stand-in for the RCCL entry points libghs_mst.so calls (csrc/multi.hip), so that the
// library's real COMM_NCCL branches — the in-place ncclReduceScatter(buf, buf + rank * per, ...),
// ncclAllGather, the uint64 / int64 / int32 all-reduces and the setup agreement — run at N > 1 on a
// ONE-GPU box, where RCCL itself refuses two ranks on one device ("Duplicate GPU detected"). It is
// linked only into a test build of the library (tests/rccl_stub/libghs_mst_rcclstub.so, Makefile
// target `rcclstub`), never into the shipped libghs_mst.so, which links librccl.
//
// Semantics follow NCCL's: every rank of a communicator calls the same collective with the same
// count / type / op (checked: a mismatch fails the call on every rank with ncclInvalidUsage); the
// result is written to recvbuff on the caller's stream; in-place is recvbuff == sendbuff (all-reduce),
// recvbuff == sendbuff + rank * recvcount (reduce-scatter), sendbuff == recvbuff + rank * sendcount
// (all-gather), any other overlap is ncclInvalidArgument. NCCL leaves the other slices of an in-place
// reduce-scatter's send buffer undefined: the stub poisons them, so a caller relying on them breaks.
// Implementation: host-synchronous — each rank syncs its stream (send data ready), stages its send
// buffer into a device scratch of the group, barriers with the other rank threads, computes its own
// output from the stages with a kernel, syncs, barriers again. ncclCommAbort wakes every waiter.
#include <hip/hip_runtime.h>

#include "nccl_rename.h"  // the stub defines the renamed entry points the test build calls
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

enum Kind { K_ALLREDUCE = 1, K_REDUCESCATTER = 2, K_ALLGATHER = 3 };

struct Call {
  int kind = 0;
  const void *send = nullptr;
  void *recv = nullptr;
  size_t count = 0;
  int dt = -1, op = -1;
};

struct Group {
  int nranks = 0;
  int refs = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<Call> calls;
  std::vector<void *> stage;
  std::vector<size_t> stage_cap;
  std::vector<int> devs;
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
};

std::mutex g_mu;
std::map<std::string, Group *> g_groups;
std::atomic<uint64_t> g_next{1};
std::atomic<uint64_t> g_calls{0};

size_t dt_size(int dt) {
  switch (dt) {
    case ncclInt32: return 4;
    case ncclInt64: case ncclUint64: return 8;
    default: return 0;
  }
}

template <typename T, int OP>
__global__ void k_fold(T *__restrict__ dst, const T *__restrict__ src, size_t n, bool first) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T s = src[i];
    if (first) { dst[i] = s; continue; }
    const T d = dst[i];
    dst[i] = OP == ncclSum ? (T)(d + s) : OP == ncclMin ? (s < d ? s : d) : (s > d ? s : d);
  }
}

__global__ void k_poison(uint8_t *p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = 0xA5;
}

unsigned grid(size_t n) {
  const size_t g = (n + 255) / 256;
  return (unsigned)(g < 4096 ? (g ? g : 1) : 4096);
}

template <typename T>
ncclResult_t fold(int op, T *dst, const T *src, size_t n, bool first, hipStream_t st) {
  if (op == ncclSum) k_fold<T, ncclSum><<<grid(n), 256, 0, st>>>(dst, src, n, first);
  else if (op == ncclMin) k_fold<T, ncclMin><<<grid(n), 256, 0, st>>>(dst, src, n, first);
  else if (op == ncclMax) k_fold<T, ncclMax><<<grid(n), 256, 0, st>>>(dst, src, n, first);
  else return ncclInvalidArgument;
  return hipGetLastError() == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

ncclResult_t fold_dt(int dt, int op, void *dst, const void *src, size_t n, bool first, hipStream_t st) {
  if (dt == ncclInt32) return fold<int32_t>(op, (int32_t *)dst, (const int32_t *)src, n, first, st);
  if (dt == ncclInt64) return fold<int64_t>(op, (int64_t *)dst, (const int64_t *)src, n, first, st);
  if (dt == ncclUint64) return fold<uint64_t>(op, (uint64_t *)dst, (const uint64_t *)src, n, first, st);
  return ncclInvalidArgument;
}

bool overlap(const void *a, size_t an, const void *b, size_t bn) {
  const char *x = (const char *)a, *y = (const char *)b;
  return x < y + bn && y < x + an;
}

}  // namespace

struct ncclComm {
  Group *g = nullptr;
  int rank = 0;
  int dev = 0;
};

namespace {

ncclResult_t collective(ncclComm *c, Call call, hipStream_t st) {
  if (!c || !c->g) return ncclInvalidArgument;
  Group *g = c->g;
  const int N = g->nranks, r = c->rank;
  const size_t es = dt_size(call.dt);
  if (!es) return ncclInvalidArgument;
  g_calls.fetch_add(1);
  // argument rules (NCCL): in place exactly at the documented offset, else disjoint buffers
  const size_t sb = call.count * es * (call.kind == K_REDUCESCATTER ? N : 1);
  const size_t rb = call.count * es * (call.kind == K_ALLGATHER ? N : 1);
  bool bad_args = false;
  if (call.count && overlap(call.send, sb, call.recv, rb)) {
    const char *s = (const char *)call.send, *d = (const char *)call.recv;
    if (call.kind == K_ALLREDUCE) bad_args = s != d;
    if (call.kind == K_REDUCESCATTER) bad_args = d != s + (size_t)r * call.count * es;
    if (call.kind == K_ALLGATHER) bad_args = s != d + (size_t)r * call.count * es;
  }
  if (hipSetDevice(c->dev) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return ncclUnhandledCudaError;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    g->calls[r] = call;
  }
  if (!g->barrier()) return ncclRemoteError;
  // every rank checks every rank's call: all fail together on a mismatch
  for (int q = 0; q < N; ++q) {
    const Call &o = g->calls[q];
    if (o.kind != call.kind || o.count != call.count || o.dt != call.dt || o.op != call.op) {
      fprintf(stderr, "[nccl_stub] rank %d: collective mismatch with rank %d (kind %d/%d count %zu/%zu dt %d/%d op %d/%d)\n",
              r, q, call.kind, o.kind, call.count, o.count, call.dt, o.dt, call.op, o.op);
      g->barrier();
      return ncclInvalidUsage;
    }
  }
  // stage this rank's send buffer (recv may alias it: the others read the stage, never the buffer)
  if (g->stage_cap[r] < sb) {
    if (g->stage[r]) (void)hipFree(g->stage[r]);
    g->stage[r] = nullptr;
    g->stage_cap[r] = 0;
    if (hipMalloc(&g->stage[r], sb ? sb : 8) != hipSuccess) return ncclSystemError;
    g->stage_cap[r] = sb;
  }
  if (sb && hipMemcpyAsync(g->stage[r], call.send, sb, hipMemcpyDeviceToDevice, st) != hipSuccess) return ncclUnhandledCudaError;
  if (hipStreamSynchronize(st) != hipSuccess) return ncclUnhandledCudaError;
  if (!g->barrier()) return ncclRemoteError;
  ncclResult_t res = bad_args ? ncclInvalidArgument : ncclSuccess;
  if (!bad_args && call.count) {
    const size_t n = call.count;
    if (call.kind == K_ALLREDUCE) {
      for (int q = 0; q < N && res == ncclSuccess; ++q) res = fold_dt(call.dt, call.op, call.recv, g->stage[q], n, q == 0, st);
    } else if (call.kind == K_REDUCESCATTER) {
      for (int q = 0; q < N && res == ncclSuccess; ++q)
        res = fold_dt(call.dt, call.op, call.recv, (const char *)g->stage[q] + (size_t)r * n * es, n, q == 0, st);
      // NCCL leaves the rest of an in-place send buffer undefined: poison it
      if (res == ncclSuccess && (const char *)call.recv == (const char *)call.send + (size_t)r * n * es) {
        if (r > 0) k_poison<<<grid(r * n * es), 256, 0, st>>>((uint8_t *)call.send, (size_t)r * n * es);
        if (r < N - 1)
          k_poison<<<grid((N - 1 - r) * n * es), 256, 0, st>>>((uint8_t *)call.recv + n * es, (size_t)(N - 1 - r) * n * es);
      }
    } else {
      for (int q = 0; q < N; ++q)
        if (hipMemcpyAsync((char *)call.recv + (size_t)q * n * es, g->stage[q], n * es, hipMemcpyDeviceToDevice, st) !=
            hipSuccess)
          res = ncclUnhandledCudaError;
    }
  }
  if (hipStreamSynchronize(st) != hipSuccess && res == ncclSuccess) res = ncclUnhandledCudaError;
  if (!g->barrier()) return ncclRemoteError;  // every rank has read every stage
  return res;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
  if (!id) return ncclInvalidArgument;
  memset(id, 0, sizeof(*id));
  const uint64_t k = g_next.fetch_add(1);
  snprintf(id->internal, sizeof(id->internal), "nccl_stub:%llu:%p", (unsigned long long)k, (void *)&g_next);
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId commId, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  const std::string key(commId.internal, strnlen(commId.internal, sizeof(commId.internal)));
  std::lock_guard<std::mutex> lk(g_mu);
  Group *&g = g_groups[key];
  if (!g) {
    g = new Group;
    g->nranks = nranks;
    g->calls.resize(nranks);
    g->stage.assign(nranks, nullptr);
    g->stage_cap.assign(nranks, 0);
  }
  if (g->nranks != nranks) return ncclInvalidUsage;
  ncclComm *c = new ncclComm;
  c->g = g;
  c->rank = rank;
  if (hipGetDevice(&c->dev) != hipSuccess) c->dev = 0;
  ++g->refs;
  *comm = c;
  return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t *comm, int ndev, const int *devlist) {
  if (!comm || ndev < 1) return ncclInvalidArgument;
  ncclUniqueId id;
  ncclGetUniqueId(&id);
  int prev = 0;
  (void)hipGetDevice(&prev);
  for (int i = 0; i < ndev; ++i) {
    (void)hipSetDevice(devlist ? devlist[i] : i);
    if (ncclResult_t r = ncclCommInitRank(&comm[i], ndev, id, i)) return r;
  }
  (void)hipSetDevice(prev);
  return ncclSuccess;
}

static void drop(ncclComm *c) {
  std::lock_guard<std::mutex> lk(g_mu);
  Group *g = c->g;
  if (g && --g->refs == 0) {
    for (auto it = g_groups.begin(); it != g_groups.end(); ++it)
      if (it->second == g) {
        g_groups.erase(it);
        break;
      }
    for (void *p : g->stage)
      if (p) (void)hipFree(p);
    delete g;
  }
  delete c;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (comm) drop(comm);
  return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (!comm) return ncclSuccess;
  {
    std::lock_guard<std::mutex> lk(comm->g->mu);
    comm->g->aborted = true;
    comm->g->cv.notify_all();
  }
  drop(comm);
  return ncclSuccess;
}

const char *ncclGetErrorString(ncclResult_t result) {
  switch (result) {
    case ncclSuccess: return "no error (nccl_stub)";
    case ncclInvalidArgument: return "invalid argument (nccl_stub)";
    case ncclInvalidUsage: return "invalid usage: ranks called different collectives (nccl_stub)";
    case ncclRemoteError: return "a peer aborted the communicator (nccl_stub)";
    default: return "error (nccl_stub)";
  }
}

ncclResult_t ncclAllReduce(const void *sendbuff, void *recvbuff, size_t count, ncclDataType_t datatype, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream) {
  return collective(comm, Call{K_ALLREDUCE, sendbuff, recvbuff, count, (int)datatype, (int)op}, stream);
}

ncclResult_t ncclReduceScatter(const void *sendbuff, void *recvbuff, size_t recvcount, ncclDataType_t datatype,
                               ncclRedOp_t op, ncclComm_t comm, hipStream_t stream) {
  return collective(comm, Call{K_REDUCESCATTER, sendbuff, recvbuff, recvcount, (int)datatype, (int)op}, stream);
}

ncclResult_t ncclAllGather(const void *sendbuff, void *recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, hipStream_t stream) {
  return collective(comm, Call{K_ALLGATHER, sendbuff, recvbuff, sendcount, (int)datatype, -1}, stream);
}

// test introspection: collectives executed by this process (the test asserts the RCCL branches ran)
uint64_t nccl_stub_calls(void) { return g_calls.load(); }

}  // extern "C"
