// Stage-1 ceiling: what one min-edge round over a level's live edges can reach on
// MI355X, so that stage1_roofline (24 B per live edge over the min-edge kernels' time) is judged
// against an achievable number. A shared library driven by tools/stage1_ceiling.py, which hands it
// the R-MAT s24 level-0 edge set (the edges of the engine's first level: a ascending, b random,
// key = w << 32 | eid) as device pointers. Each variant is one kernel over the E records; the driver
// times it with HIP events and converts to the 24 B model.
//   stream        read a, b, key (16 B per record), nothing else: the HBM stream bound
//   a_seg         + the a-side minimum per run of equal a (wave segmented min, one read-checked
//                 atomicMin per run tail into best[a])
//   b_gather      + a random 8-B read of best[b] per record (no update): the random-read floor
//   b_atomic      + a random 64-bit atomicMin into best[b] per record (no read-check)
//   ideal         a_seg + read-checked b atomicMin: the minimum work of an unbucketed round
//   b_sorted      both sides as segmented minima over records already grouped by b (a second,
//                 b-sorted copy of the records, built outside the timing): an upper bound for any
//                 design that removes the random best[] traffic (it still streams 2 x 16 B)
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int WAVE = 64;

__device__ __forceinline__ void min_rc(unsigned long long *best, uint32_t i, unsigned long long k) {
  if (best[i] > k) atomicMin(best + i, k);
}

// one record per lane per step, grid-stride over runs of 64 consecutive records per wave (so the
// segmented min sees consecutive records)
template <int KIND>
__global__ __launch_bounds__(256) void k_round(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b,
                                                const unsigned long long *__restrict__ key, uint64_t E,
                                                unsigned long long *__restrict__ best, unsigned long long *sink) {
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / WAVE;
  const uint64_t nw = (uint64_t)gridDim.x * blockDim.x / WAVE;
  unsigned long long acc = 0;
  for (uint64_t base = wave * WAVE; base < E; base += nw * WAVE) {
    const uint64_t i = base + lane;
    const bool v = i < E;
    const uint32_t A = v ? a[i] : 0xffffffffu, B = v ? b[i] : 0u;
    const unsigned long long K = v ? key[i] : ~0ull;
    if (KIND == 0) {
      acc ^= A ^ B ^ K;
      continue;
    }
    if (KIND == 1 || KIND == 4 || KIND == 5) {  // segmented min over runs of equal A (A ascending)
      unsigned long long m = K;
      for (int d = 1; d < WAVE; d <<= 1) {
        const unsigned long long o = __shfl_down(m, d);
        const uint32_t oa = __shfl_down(A, d);
        if (lane + d < WAVE && oa == A && o < m) m = o;
      }
      // m of the run's FIRST lane holds the run's min (every later lane of the run folds forward)
      const uint32_t pa = __shfl_up(A, 1);
      const bool head = lane == 0 || pa != A;
      if (v && head) min_rc(best, A, m);
    }
    if (KIND == 5) {  // b grouped too: the same segmented min over runs of equal B
      unsigned long long m = K;
      for (int d = 1; d < WAVE; d <<= 1) {
        const unsigned long long o = __shfl_down(m, d);
        const uint32_t ob = __shfl_down(B, d);
        if (lane + d < WAVE && ob == B && o < m) m = o;
      }
      const uint32_t pb = __shfl_up(B, 1);
      if (v && (lane == 0 || pb != B)) min_rc(best, B, m);
    }
    if (KIND == 2 && v) acc += best[B];
    if (KIND == 3 && v) atomicMin(best + B, K);
    if (KIND == 4 && v) min_rc(best, B, K);
  }
  if (acc == 0x1234567ull) sink[0] = acc;
}
}  // namespace

extern "C" int s1_run(int kind, const uint32_t *a, const uint32_t *b, const unsigned long long *key, uint64_t E,
                      unsigned long long *best, unsigned long long *sink, int grid, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (kind) {
    case 0: k_round<0><<<grid, 256, 0, st>>>(a, b, key, E, best, sink); break;
    case 1: k_round<1><<<grid, 256, 0, st>>>(a, b, key, E, best, sink); break;
    case 2: k_round<2><<<grid, 256, 0, st>>>(a, b, key, E, best, sink); break;
    case 3: k_round<3><<<grid, 256, 0, st>>>(a, b, key, E, best, sink); break;
    case 4: k_round<4><<<grid, 256, 0, st>>>(a, b, key, E, best, sink); break;
    case 5: k_round<5><<<grid, 256, 0, st>>>(a, b, key, E, best, sink); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
