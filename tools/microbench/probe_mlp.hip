// Random 32-bit probes into a 2 MiB table (L2-resident): rate vs probes in flight per lane and
// occupancy. P independent probes per lane per iteration.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int P>
__global__ __launch_bounds__(256) void k(uint64_t M, const uint32_t *__restrict__ bits, uint32_t nwords, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t t = blockIdx.x; t * 256 * P < M; t += gridDim.x) {
    const uint64_t i = (t * 256 + threadIdx.x) * P;
    uint32_t v[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      uint32_t h = (uint32_t)(i + p) * 2654435761u;
      h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12;
      v[p] = bits[h % nwords];
    }
#pragma unroll
    for (int p = 0; p < P; ++p) acc ^= v[p];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const uint64_t M = 256000000ull;
  for (uint32_t nwords : {(1u << 24) / 32, (1u << 20) / 32, (1u << 26) / 32}) {
    uint32_t *bits, *o;
    CK(hipMalloc(&bits, (size_t)nwords * 4)); CK(hipMalloc(&o, 1 << 26));
    CK(hipMemset(bits, 0x55, (size_t)nwords * 4));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int grid : {2048, 8192}) {
      for (int P : {4, 8, 16}) {
        float best = 1e9;
        for (int rep = 0; rep < 4; ++rep) {
          CK(hipEventRecord(e0));
          if (P == 4) k<4><<<grid, 256>>>(M, bits, nwords, o);
          if (P == 8) k<8><<<grid, 256>>>(M, bits, nwords, o);
          if (P == 16) k<16><<<grid, 256>>>(M, bits, nwords, o);
          CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
          float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
        }
        printf("table %6u KiB grid %5d P %2d  %8.1f us  %6.1f G probes/s\n", nwords * 4 / 1024, grid, P, best * 1e3, M / (best * 1e-3) / 1e9);
      }
    }
    CK(hipFree(bits)); CK(hipFree(o));
  }
  return 0;
}
