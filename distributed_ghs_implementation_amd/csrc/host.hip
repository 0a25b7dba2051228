// Host-buffer entry point: GHSAlgorithm.run / MPI collect_results equivalent
// (ghs_implementation.py:442-490, ghs_implementation_mpi.py:673-779) for callers that hold the
// canonical edge list in host memory (the reference's own FFI-free Python flow, small graphs).
#include <hip/hip_runtime.h>

#include <string>

#include "common.h"

namespace {
struct DevBuf {
  void *p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};
}  // namespace

extern "C" int ghs_mst_host(uint32_t n, uint64_t m, const uint32_t *u, const uint32_t *v, const uint32_t *w,
                            uint8_t *in_mst, ghs_result_t *result, ghs_round_stats_t *stats) {
  if (m && (!u || !v || !w || !in_mst)) GHS_FAIL(GHS_E_ARG, "NULL host pointer");
  if (m >= (1ull << 31)) GHS_FAIL(GHS_E_ARG, "m must be < 2^31");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) GHS_FAIL(GHS_E_NODEVICE, "no HIP device");
  // canonicity is validated on the device by the solve's first pass (k_select, GHS_E_NONCANON
  // before any id indexes an array): no serial host loop in front of the copy
  const size_t ws = ghs_workspace_bytes(n, m, m);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t off_u = 0, off_v = off_u + al(m * 4), off_w = off_v + al(m * 4), off_mst = off_w + al(m * 4),
               off_ws = off_mst + al(m ? m : 1), total = off_ws + al(ws);
  DevBuf buf;
  GHS_HIP_CHECK(hipMalloc(&buf.p, total));
  char *b = (char *)buf.p;
  hipStream_t st = nullptr;
  if (m) {
    GHS_HIP_CHECK(hipMemcpyAsync(b + off_u, u, m * 4, hipMemcpyHostToDevice, st));
    GHS_HIP_CHECK(hipMemcpyAsync(b + off_v, v, m * 4, hipMemcpyHostToDevice, st));
    GHS_HIP_CHECK(hipMemcpyAsync(b + off_w, w, m * 4, hipMemcpyHostToDevice, st));
  }
  int rc = ghs_mst_device(n, m, (uint32_t *)(b + off_u), (uint32_t *)(b + off_v), (uint32_t *)(b + off_w), nullptr,
                          b + off_ws, ws, (uint8_t *)(b + off_mst), st, result, stats);
  if (rc) return rc;
  if (m) GHS_HIP_CHECK(hipMemcpy(in_mst, b + off_mst, m, hipMemcpyDeviceToHost));
  return GHS_OK;
}
