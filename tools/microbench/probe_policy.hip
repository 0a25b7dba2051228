// Random 32-bit probes into a 2 MiB bitmap (the k_filter giant test) under different cache
// policies of the probe load, alone and beside the 12 B/edge stream. The question: does a probe
// that does not allocate in the CU's L1 (or asks L2 for less than a line) raise the probe rate?
//   aux bits (gfx950 buffer loads): 1 = sc0, 2 = nt, 16 = sc1
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int AUX>
__device__ __forceinline__ uint32_t probe(__amdgpu_buffer_rsrc_t r, uint32_t word) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, (int)(word * 4u), 0, AUX);
}

template <int AUX, bool STREAM>
__global__ __launch_bounds__(256) void k(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b,
                                         const uint32_t *__restrict__ c, uint64_t M, const uint32_t *bits,
                                         uint32_t nwords, uint32_t *out) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(bits), (short)0, (int)(nwords * 4), 0x00020000);
  uint32_t acc = 0;
  for (uint64_t t = blockIdx.x; t * 1024 < M; t += gridDim.x) {
    const uint64_t i = t * 1024 + threadIdx.x * 4;
    uint4 x, y, z;
    if (STREAM) {
      x = *(const uint4 *)(a + i); y = *(const uint4 *)(b + i); z = *(const uint4 *)(c + i);
    } else {
      uint32_t h = (uint32_t)i * 2654435761u;
      y = make_uint4(h, h * 747796405u, h * 2891336453u, h ^ (h >> 13) * 1664525u);
      x = y; z = y;
    }
    const uint32_t p0 = probe<AUX>(r, (y.x * 2654435761u) % nwords), p1 = probe<AUX>(r, (y.y * 2654435761u) % nwords);
    const uint32_t p2 = probe<AUX>(r, (y.z * 2654435761u) % nwords), p3 = probe<AUX>(r, (y.w * 2654435761u) % nwords);
    acc ^= p0 ^ p1 ^ p2 ^ p3 ^ x.x ^ z.w;
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

template <int AUX, bool STREAM>
static float run(const uint32_t *a, const uint32_t *b, const uint32_t *c, uint64_t M, const uint32_t *bits, uint32_t nw,
                 uint32_t *o, int grid) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float best = 1e9;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(e0);
    k<AUX, STREAM><<<grid, 256>>>(a, b, c, M, bits, nw, o);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const uint64_t M = 260000000ull;
  uint32_t *a, *b, *c, *o, *bits;
  CK(hipMalloc(&a, M * 4)); CK(hipMalloc(&b, M * 4)); CK(hipMalloc(&c, M * 4));
  CK(hipMalloc(&o, 1 << 26)); CK(hipMalloc(&bits, (1u << 26)));
  CK(hipMemset(a, 1, M * 4)); CK(hipMemset(c, 3, M * 4)); CK(hipMemset(bits, 0x55, 1u << 26));
  k_fill<<<8192, 256>>>(b, M);
  CK(hipDeviceSynchronize());
  for (uint32_t mib : {2u, 8u}) {
    const uint32_t nw = mib * (1u << 20) / 4;
    const int grid = 4096;
#define ROW(AUX, ST, name) { float ms = run<AUX, ST>(a, b, c, M, bits, nw, o, grid); \
      printf("%2u MiB %-10s %-6s %8.1f us  %6.1f G probes/s\n", mib, name, ST ? "stream" : "alone", ms * 1e3, M / (ms * 1e-3) / 1e9); }
    ROW(0, false, "plain") ROW(1, false, "sc0") ROW(2, false, "nt") ROW(3, false, "sc0|nt") ROW(16, false, "sc1") ROW(17, false, "sc0|sc1")
    ROW(0, true, "plain") ROW(1, true, "sc0") ROW(2, true, "nt") ROW(3, true, "sc0|nt") ROW(16, true, "sc1") ROW(17, true, "sc0|sc1")
  }
  return 0;
}
