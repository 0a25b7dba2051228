// rocPRIM/hipCUB radix sort throughput on gfx950 for the arc-build shapes (u32 key, u32 value).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
__global__ void fill(uint32_t* k, uint32_t* v, size_t n, uint32_t mask) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u; x ^= x >> 15; x *= 0x2c1b3c6dU; x ^= x >> 12;
    k[i] = x & mask; v[i] = (uint32_t)i;
  }
}
int main() {
  for (size_t n : {(size_t)67108864, (size_t)268435456, (size_t)536870912}) {
    uint32_t *k0, *k1, *v0, *v1; void* tmp = nullptr; size_t tb = 0;
    CK(hipMalloc(&k0, n * 4)); CK(hipMalloc(&k1, n * 4)); CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&v1, n * 4));
    for (int bits : {24, 26}) {
      fill<<<4096, 256>>>(k0, v0, n, (1u << bits) - 1);
      tb = 0; CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0, k1, v0, v1, n, 0, bits));
      CK(hipMalloc(&tmp, tb));
      hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a)); CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k0, k1, v0, v1, n, 0, bits)); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        printf("SortPairs u32/u32 n=%zu bits=%d: %.3f ms  %.2f G pairs/s\n", n, bits, ms, n / ms / 1e6);
      }
      // DoubleBuffer variant
      hipcub::DoubleBuffer<uint32_t> dk(k0, k1), dv(v0, v1);
      size_t tb2 = 0; CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, dk, dv, n, 0, bits));
      void* tmp2; CK(hipMalloc(&tmp2, tb2));
      fill<<<4096, 256>>>(k0, v0, n, (1u << bits) - 1);
      CK(hipEventRecord(a)); CK(hipcub::DeviceRadixSort::SortPairs(tmp2, tb2, dk, dv, n, 0, bits)); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      printf("SortPairs DoubleBuffer n=%zu bits=%d: %.3f ms  %.2f G pairs/s (temp %zu MB)\n", n, bits, ms, n / ms / 1e6, tb2 >> 20);
      CK(hipFree(tmp)); CK(hipFree(tmp2));
    }
    CK(hipFree(k0)); CK(hipFree(k1)); CK(hipFree(v0)); CK(hipFree(v1));
  }
  return 0;
}
