// Microbenchmark 2: random u32 gather rate vs table size and memory-level parallelism (ILP per
// thread), plus XCD-sliced tables (block b reads only slice b%8 of the table).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

// Index computed in-register (no index stream) so that only the gather is measured.
template <int ILP>
__global__ void k_gather_ilp(const uint32_t* __restrict__ tab, uint32_t mask, size_t n, uint32_t* out, int xcd_slices) {
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x * ILP;
  uint32_t slice_base = 0, slice_mask = mask;
  if (xcd_slices > 1) {  // table split into xcd_slices parts; block b uses part b % xcd_slices
    uint32_t part = (mask + 1) / xcd_slices;
    slice_base = (blockIdx.x % xcd_slices) * part;
    slice_mask = part - 1;
  }
  for (size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) * ILP; i < n; i += stride) {
    uint32_t v[ILP];
#pragma unroll
    for (int j = 0; j < ILP; ++j) v[j] = tab[slice_base + (hash32((uint32_t)(i + j)) & slice_mask)];
#pragma unroll
    for (int j = 0; j < ILP; ++j) acc += v[j];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int ILP>
__global__ void k_atomic_ilp(unsigned long long* tab, uint32_t mask, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * ILP;
  for (size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) * ILP; i < n; i += stride) {
#pragma unroll
    for (int j = 0; j < ILP; ++j) { uint32_t h = hash32((uint32_t)(i + j)); atomicMin(&tab[h & mask], (unsigned long long)h); }
  }
}

int main() {
  const size_t NG = 1ull << 28;
  uint32_t* tab; CK(hipMalloc(&tab, 1ull << 30)); CK(hipMemset(tab, 0, 1ull << 30));
  uint32_t* out; CK(hipMalloc(&out, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float ms;
  int block = 256;
  for (int lg : {18, 20, 21, 22, 24, 26, 28}) {   // table entries (x4 bytes)
    uint32_t mask = (1u << lg) - 1;
    for (int grid : {2048, 8192}) {
      auto run = [&](auto kern, const char* name, int xs) -> int {
        kern<<<grid, block>>>(tab, mask, NG, out, xs);
        CK(hipEventRecord(e0)); kern<<<grid, block>>>(tab, mask, NG, out, xs); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("table %7.2f MiB grid %5d %-6s xcd_slices=%d: %.3f ms  %.1f G gathers/s\n", (4.0 * (mask + 1)) / 1048576.0, grid, name, xs, ms, NG / ms / 1e6);
        return 0;
      };
      if (run(k_gather_ilp<1>, "ilp1", 1)) return 1;
      if (run(k_gather_ilp<4>, "ilp4", 1)) return 1;
      if (run(k_gather_ilp<8>, "ilp8", 1)) return 1;
      if (lg >= 22) if (run(k_gather_ilp<8>, "ilp8", 8)) return 1;
    }
  }
  unsigned long long* at; CK(hipMalloc(&at, 1ull << 30)); CK(hipMemset(at, 0xff, 1ull << 30));
  const size_t NA = 1ull << 26;
  for (int lg : {16, 19, 22, 24, 27}) {
    uint32_t mask = (1u << lg) - 1;
    for (int ilp : {1, 4}) {
      CK(hipEventRecord(e0));
      if (ilp == 1) k_atomic_ilp<1><<<8192, block>>>(at, mask, NA); else k_atomic_ilp<4><<<8192, block>>>(at, mask, NA);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      printf("atomicMin u64 table %7.2f MiB ilp%d: %.3f ms %.1f G atomics/s\n", (8.0 * (mask + 1)) / 1048576.0, ilp, ms, NA / ms / 1e6);
    }
  }
  printf("done\n");
  return 0;
}
