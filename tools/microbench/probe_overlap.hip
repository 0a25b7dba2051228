// Does a 12 B/edge stream overlap with one random 2 MiB-bitmap probe per edge (k_filter's shape)
// when the stream is prefetched D tiles ahead? probe_bench measured the SUM of the two with no
// prefetch; here D = 0, 1, 2, 3 (tile = 4 edges per lane; probe index from the streamed v).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int D>
__global__ __launch_bounds__(256) void k(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b,
                                         const uint32_t *__restrict__ c, uint64_t M, const uint32_t *__restrict__ bits,
                                         uint32_t nwords, uint32_t *out) {
  uint32_t acc = 0;
  const uint64_t step = (uint64_t)gridDim.x * 1024;
  uint64_t t = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
  uint4 qa[D + 1], qb[D + 1], qc[D + 1];
#pragma unroll
  for (int d = 0; d <= D; ++d) {
    const uint64_t i = t + d * step;
    const uint64_t ii = i < M ? i : 0;
    qa[d] = *(const uint4 *)(a + ii); qb[d] = *(const uint4 *)(b + ii); qc[d] = *(const uint4 *)(c + ii);
  }
  for (; t < M; t += step) {
    const uint4 x = qa[0], y = qb[0], z = qc[0];
#pragma unroll
    for (int d = 0; d < D; ++d) { qa[d] = qa[d + 1]; qb[d] = qb[d + 1]; qc[d] = qc[d + 1]; }
    {
      const uint64_t i = t + (D + 1) * step;
      const uint64_t ii = i < M ? i : 0;
      qa[D] = *(const uint4 *)(a + ii); qb[D] = *(const uint4 *)(b + ii); qc[D] = *(const uint4 *)(c + ii);
    }
    const uint32_t p0 = bits[(y.x >> 5) % nwords], p1 = bits[(y.y >> 5) % nwords];
    const uint32_t p2 = bits[(y.z >> 5) % nwords], p3 = bits[(y.w >> 5) % nwords];
    acc ^= ((p0 >> (y.x & 31)) & 1) + ((p1 >> (y.y & 31)) & 1) + ((p2 >> (y.z & 31)) & 1) + ((p3 >> (y.w & 31)) & 1);
    acc ^= x.x ^ x.y ^ x.z ^ x.w ^ z.x ^ z.y ^ z.z ^ z.w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ void k_fill(uint32_t *b, uint64_t M, uint32_t nv) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < M; i += 256ull * gridDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12;
    b[i] = h % nv;
  }
}

template <int D>
static float run(const uint32_t *a, const uint32_t *b, const uint32_t *c, uint64_t M, const uint32_t *bits, uint32_t nw,
                 uint32_t *o, int grid) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  float best = 1e9;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0);
    k<D><<<grid, 256>>>(a, b, c, M, bits, nw, o);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const uint64_t M = 260000000ull;
  const uint32_t nv = 1u << 24, nw = nv / 32;  // 16.8M vertices -> 2 MiB bitmap
  uint32_t *a, *b, *c, *o, *bits;
  CK(hipMalloc(&a, M * 4)); CK(hipMalloc(&b, M * 4)); CK(hipMalloc(&c, M * 4));
  CK(hipMalloc(&o, 1 << 26)); CK(hipMalloc(&bits, nw * 4));
  CK(hipMemset(a, 1, M * 4)); CK(hipMemset(c, 3, M * 4)); CK(hipMemset(bits, 0x55, nw * 4));
  k_fill<<<8192, 256>>>(b, M, nv);
  CK(hipDeviceSynchronize());
  for (int grid : {1024, 2048, 4096}) {
    printf("grid %d: D0 %.1f us  D1 %.1f us  D2 %.1f us  D3 %.1f us\n", grid, run<0>(a, b, c, M, bits, nw, o, grid) * 1e3,
           run<1>(a, b, c, M, bits, nw, o, grid) * 1e3, run<2>(a, b, c, M, bits, nw, o, grid) * 1e3,
           run<3>(a, b, c, M, bits, nw, o, grid) * 1e3);
  }
  return 0;
}
