// Random-probe microbenchmark for the FILTER pass shape: M random 32-bit probes into a 2 MiB
// bitmap (L2-resident per XCD), alone and beside a 12 B/edge stream.
//   probe     : 4 independent probes per lane per iteration, no stream
//   stream    : the 3-array stream alone (16-B loads)
//   both      : stream + 4 probes per lane (indices from the streamed data)
//   both_nt   : as both, stream loads nontemporal (do not allocate in L2)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void k(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b,
                                         const uint32_t *__restrict__ c, uint64_t M, const uint32_t *__restrict__ bits,
                                         uint32_t nwords, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t t = blockIdx.x; t * 1024 < M; t += gridDim.x) {
    const uint64_t i = t * 1024 + threadIdx.x * 4;
    uint4 x, y, z;
    if (MODE == 0) {
      uint32_t h = (uint32_t)i * 2654435761u;
      x = make_uint4(h, h * 747796405u, h * 2891336453u, h ^ (h >> 13) * 1664525u);
      y = x; z = x;
    } else if (MODE == 3) {
      typedef uint32_t v4 __attribute__((ext_vector_type(4)));
      v4 xa = __builtin_nontemporal_load((const v4 *)(a + i));
      v4 ya = __builtin_nontemporal_load((const v4 *)(b + i));
      v4 za = __builtin_nontemporal_load((const v4 *)(c + i));
      x = make_uint4(xa.x, xa.y, xa.z, xa.w); y = make_uint4(ya.x, ya.y, ya.z, ya.w); z = make_uint4(za.x, za.y, za.z, za.w);
    } else {
      x = *(const uint4 *)(a + i); y = *(const uint4 *)(b + i); z = *(const uint4 *)(c + i);
    }
    if (MODE == 1) {
      acc ^= x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w ^ z.x ^ z.y ^ z.z ^ z.w;
    } else {
      const uint32_t p0 = bits[(y.x * 2654435761u) % nwords], p1 = bits[(y.y * 2654435761u) % nwords];
      const uint32_t p2 = bits[(y.z * 2654435761u) % nwords], p3 = bits[(y.w * 2654435761u) % nwords];
      acc ^= p0 ^ p1 ^ p2 ^ p3 ^ x.x ^ z.w;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ void k_fill(uint32_t *b, uint64_t M) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < M; i += 256ull * gridDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12;
    b[i] = h;
  }
}

int main() {
  const uint64_t M = 260000000ull;
  const uint32_t nwords = (1u << 24) / 32;  // 16.8M vertices -> 2 MiB
  uint32_t *a, *b, *c, *o, *bits;
  CK(hipMalloc(&a, M * 4)); CK(hipMalloc(&b, M * 4)); CK(hipMalloc(&c, M * 4));
  CK(hipMalloc(&o, 1 << 26)); CK(hipMalloc(&bits, nwords * 4));
  CK(hipMemset(a, 1, M * 4)); CK(hipMemset(b, 7, M * 4)); CK(hipMemset(c, 3, M * 4)); CK(hipMemset(bits, 0x55, nwords * 4));
  k_fill<<<8192, 256>>>(b, M);  // b holds random values: random probe indices
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char *names[4] = {"probe", "stream", "both", "both_nt"};
  for (int grid : {2048, 8192}) {
    for (int mode = 0; mode < 4; ++mode) {
      float best = 1e9;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0));
        if (mode == 0) k<0><<<grid, 256>>>(a, b, c, M, bits, nwords, o);
        if (mode == 1) k<1><<<grid, 256>>>(a, b, c, M, bits, nwords, o);
        if (mode == 2) k<2><<<grid, 256>>>(a, b, c, M, bits, nwords, o);
        if (mode == 3) k<3><<<grid, 256>>>(a, b, c, M, bits, nwords, o);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
      }
      printf("grid %5d %-8s %8.1f us  %6.1f G probes/s  %6.0f GB/s stream\n", grid, names[mode], best * 1e3,
             mode == 1 ? 0.0 : M / (best * 1e-3) / 1e9, mode == 0 ? 0.0 : 12.0 * M / (best * 1e-3) / 1e9);
    }
  }
  return 0;
}
