// Streaming-read microbenchmark for the canonical passes' shape: 3 u32 arrays of M elements
// (12 B per edge), 256-thread blocks, 16-B loads per lane. Variants:
//   contig  : block b owns the contiguous range [b*Q, (b+1)*Q) (the compaction layout)
//   stride  : grid-stride over 1024-edge tiles (all blocks sweep the arrays together)
//   contig+scan : contig + a block-wide prefix (2 barriers) per tile, like block_offsets
//   wave    : each wave owns a contiguous slice (k_select's layout: 256 edges per wave step)
// Prints GB/s (12 B per edge read).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void k_read(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b,
                                              const uint32_t *__restrict__ c, uint64_t M, uint32_t *out) {
  __shared__ uint32_t s[8];
  uint32_t acc = 0;
  if (MODE == 3) {
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t W = (uint64_t)gridDim.x * 4, gw = blockIdx.x * 4ull + wid;
    const uint64_t Q = ((M + W - 1) / W + 255) & ~255ull;
    const uint64_t vb = Q * gw, ve = vb + Q < M ? vb + Q : M;
    for (uint64_t v0 = vb; v0 < ve; v0 += 256) {
      const uint64_t i = v0 + lane * 4;
      if (i + 4 <= ve) {
        uint4 x = *(const uint4 *)(a + i), y = *(const uint4 *)(b + i), z = *(const uint4 *)(c + i);
        acc ^= x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w ^ z.x ^ z.y ^ z.z ^ z.w;
      }
    }
  } else if (MODE == 1) {
    for (uint64_t t = blockIdx.x; t * 1024 < M; t += gridDim.x) {
      const uint64_t i = t * 1024 + threadIdx.x * 4;
      if (i + 4 <= M) {
        uint4 x = *(const uint4 *)(a + i), y = *(const uint4 *)(b + i), z = *(const uint4 *)(c + i);
        acc ^= x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w ^ z.x ^ z.y ^ z.z ^ z.w;
      }
    }
  } else {
    const uint64_t Q = ((M + gridDim.x - 1) / gridDim.x + 1023) & ~1023ull;
    const uint64_t vb = Q * blockIdx.x, ve = vb + Q < M ? vb + Q : M;
    for (uint64_t v0 = vb; v0 < ve; v0 += 1024) {
      const uint64_t i = v0 + threadIdx.x * 4;
      uint32_t mine = 0;
      if (i + 4 <= ve) {
        uint4 x = *(const uint4 *)(a + i), y = *(const uint4 *)(b + i), z = *(const uint4 *)(c + i);
        acc ^= x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w ^ z.x ^ z.y ^ z.z ^ z.w;
        mine = (x.x & 1) + (y.y & 1);
      }
      if (MODE == 2) {
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        uint32_t incl = mine;
        for (int d = 1; d < 64; d <<= 1) { uint32_t o = __shfl_up(incl, d); if (lane >= d) incl += o; }
        if (lane == 63) s[wid] = incl;
        __syncthreads();
        uint32_t tot = s[0] + s[1] + s[2] + s[3];
        __syncthreads();
        acc += tot + incl;
      }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const uint64_t M = 260000000ull;
  uint32_t *a, *b, *c, *o;
  CK(hipMalloc(&a, M * 4)); CK(hipMalloc(&b, M * 4)); CK(hipMalloc(&c, M * 4));
  CK(hipMalloc(&o, 1 << 26));
  CK(hipMemset(a, 1, M * 4)); CK(hipMemset(b, 2, M * 4)); CK(hipMemset(c, 3, M * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char *names[4] = {"contig", "stride", "contig+scan", "wave"};
  for (int grid : {1024, 2048, 4096, 8192}) {
    for (int mode = 0; mode < 4; ++mode) {
      float best = 1e9;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0));
        if (mode == 0) k_read<0><<<grid, 256>>>(a, b, c, M, o);
        if (mode == 1) k_read<1><<<grid, 256>>>(a, b, c, M, o);
        if (mode == 2) k_read<2><<<grid, 256>>>(a, b, c, M, o);
        if (mode == 3) k_read<3><<<grid, 256>>>(a, b, c, M, o);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
      }
      printf("grid %5d %-12s %8.1f us  %7.0f GB/s\n", grid, names[mode], best * 1e3, 12.0 * M / (best * 1e-3) / 1e9);
    }
  }
  return 0;
}
