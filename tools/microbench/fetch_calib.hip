// Calibration of the rocprofv3 FETCH_SIZE / WRITE_SIZE counters on gfx950 for the access patterns
// of the MST kernels (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for wide coalesced reads).
// Each kernel moves a KNOWN number of bytes: run under `rocprofv3 --pmc FETCH_SIZE` (and a
// separate `--pmc WRITE_SIZE` pass) and divide the counter by the printed expectation.
//   k_cal_stream   16 B per lane coalesced reads of S bytes                     expect S
//   k_cal_gather4  N random 4-B reads from a 1 GiB table (distinct lines)       expect N x 64 B (one 64-B sector each)
//   k_cal_gather8  N random 8-B reads                                           expect N x 64 B
//   k_cal_atomic8  N random u64 atomicMin (no return)                           expect N x 64 B (memory-side RMW)
//   k_cal_store4   N random 4-B stores                                          expect N x 64 B written
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
__global__ void k_cal_stream(const uint4 *__restrict__ p, size_t n16, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_cal_gather4(const uint32_t *__restrict__ tab, uint32_t mask, size_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += tab[(hash32((uint32_t)i) & mask) & ~15u];  // one word per 64-B sector, distinct sectors
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_cal_gather8(const uint64_t *__restrict__ tab, uint32_t mask, size_t n, uint32_t *out) {
  uint64_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += tab[(hash32((uint32_t)i) & mask) & ~7u];
  if (acc == 0x12345678u) out[0] = (uint32_t)acc;
}
__global__ void k_cal_atomic8(unsigned long long *tab, uint32_t mask, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t h = hash32((uint32_t)i);
    atomicMin(&tab[(h & mask) & ~7u], (unsigned long long)h);
  }
}
__global__ void k_cal_store4(uint32_t *tab, uint32_t mask, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    tab[(hash32((uint32_t)i) & mask) & ~15u] = (uint32_t)i;
}

int main() {
  const size_t TAB = 1ull << 30;  // 1 GiB: far beyond L2 (4 MiB / XCD) and the 256 MiB MALL
  const size_t N = 1ull << 22;    // 4M accesses: ~1.6% of the table's 64-B sectors -> distinct w.h.p.
  void *tab; CK(hipMalloc(&tab, TAB)); CK(hipMemset(tab, 1, TAB));
  uint32_t *out; CK(hipMalloc(&out, 64));
  const size_t S = 1ull << 30;
  k_cal_stream<<<4096, 256>>>((const uint4 *)tab, S / 16, out);
  k_cal_gather4<<<4096, 256>>>((const uint32_t *)tab, (uint32_t)(TAB / 4 - 1), N, out);
  k_cal_gather8<<<4096, 256>>>((const uint64_t *)tab, (uint32_t)(TAB / 8 - 1), N, out);
  k_cal_atomic8<<<4096, 256>>>((unsigned long long *)tab, (uint32_t)(TAB / 8 - 1), N);
  k_cal_store4<<<4096, 256>>>((uint32_t *)tab, (uint32_t)(TAB / 4 - 1), N);
  CK(hipDeviceSynchronize());
  printf("expect k_cal_stream  fetch %zu B\n", S);
  printf("expect k_cal_gather4 fetch %zu B (N x 64)\n", N * 64);
  printf("expect k_cal_gather8 fetch %zu B (N x 64)\n", N * 64);
  printf("expect k_cal_atomic8 fetch/write %zu B (N x 64)\n", N * 64);
  printf("expect k_cal_store4  write %zu B (N x 64)\n", N * 64);
  return 0;
}
