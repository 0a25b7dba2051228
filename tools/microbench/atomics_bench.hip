// Microbenchmark: what the MST stage-1 design depends on, on gfx950.
//  (1) streaming read of 16 B/lane; (2) random u32 gather from tables of various sizes;
//  (3) random 64-bit atomicMin (no return) into tables of various sizes;
//  (4) atomicMin where a wave's 64 lanes hit runs of equal addresses.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

__global__ void k_stream(const uint4* __restrict__ a, size_t n4, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = a[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_gather(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ tab, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    acc += tab[idx[i]];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_atomic_rand(unsigned long long* tab, uint32_t mask, size_t n, uint32_t salt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = hash32((uint32_t)i ^ salt);
    atomicMin(&tab[h & mask], ((unsigned long long)h << 20) | (i & 0xfffff));
  }
}

// runs: lanes in groups of `run` consecutive lanes hit the same address
__global__ void k_atomic_runs(unsigned long long* tab, uint32_t mask, size_t n, uint32_t run, uint32_t salt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = hash32((uint32_t)(i / run) ^ salt);
    atomicMin(&tab[h & mask], ((unsigned long long)hash32((uint32_t)i) << 20));
  }
}

// wave-reduced: one lane per run of `run` lanes issues
__global__ void k_atomic_sparse(unsigned long long* tab, uint32_t mask, size_t n, uint32_t run, uint32_t salt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if ((i % run) == 0) {
      uint32_t h = hash32((uint32_t)(i / run) ^ salt);
      atomicMin(&tab[h & mask], ((unsigned long long)hash32((uint32_t)i) << 20));
    }
  }
}

int main() {
  const size_t NS = 1ull << 28;  // 256M uint4 = 4 GiB
  uint4* a; CK(hipMalloc(&a, NS * 16)); CK(hipMemset(a, 1, NS * 16));
  uint32_t* out; CK(hipMalloc(&out, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float ms;
  int grid = 256 * 8, block = 256;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0)); k_stream<<<grid, block>>>(a, NS, out); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("stream 16B/lane  4GiB: %.3f ms  %.1f GB/s\n", ms, NS * 16 / ms / 1e6);
  }
  // gather: 256M random indices into tables of 16 MiB .. 1 GiB
  const size_t NG = 1ull << 28;
  uint32_t* idx = (uint32_t*)a;  // reuse
  std::vector<uint32_t> h(1);
  for (int lg = 22; lg <= 28; lg += 2) {
    size_t tsz = 1ull << lg;
    uint32_t* tab; CK(hipMalloc(&tab, tsz * 4)); CK(hipMemset(tab, 0, tsz * 4));
    // fill idx with random in [0,tsz)
    std::vector<uint32_t> hi(NG);
    for (size_t i = 0; i < NG; ++i) { uint32_t x = (uint32_t)i * 2654435761u; x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15; hi[i] = x & (tsz - 1); }
    CK(hipMemcpy(idx, hi.data(), NG * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0)); k_gather<<<grid, block>>>(idx, tab, NG, out); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("gather u32 table %5zu MiB: %.3f ms  %.2f G gathers/s (idx stream %.0f GB/s)\n", tsz * 4 >> 20, ms, NG / ms / 1e6, NG * 4 / ms / 1e6);
    }
    CK(hipFree(tab));
  }
  // atomics
  const size_t NA = 1ull << 26;
  for (int lg = 20; lg <= 26; lg += 2) {
    size_t tsz = 1ull << lg;
    unsigned long long* tab; CK(hipMalloc(&tab, tsz * 8)); CK(hipMemset(tab, 0xff, tsz * 8));
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0)); k_atomic_rand<<<grid, block>>>(tab, (uint32_t)(tsz - 1), NA, rep * 77); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("atomicMin u64 random, table %5zu MiB: %.3f ms  %.2f G atomics/s\n", tsz * 8 >> 20, ms, NA / ms / 1e6);
    }
    for (uint32_t run : {4u, 16u, 64u}) {
      CK(hipEventRecord(e0)); k_atomic_runs<<<grid, block>>>(tab, (uint32_t)(tsz - 1), NA, run, 5); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("  runs=%2u same-address lanes: %.3f ms  %.2f G lane-atomics/s\n", run, ms, NA / ms / 1e6);
      CK(hipEventRecord(e0)); k_atomic_sparse<<<grid, block>>>(tab, (uint32_t)(tsz - 1), NA, run, 5); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("  one lane per %2u issues:      %.3f ms  %.2f G issued-atomics/s\n", run, ms, NA / run / ms / 1e6);
    }
    CK(hipFree(tab));
  }
  printf("done\n");
  return 0;
}
