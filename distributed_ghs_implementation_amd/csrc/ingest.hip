// Ingest: canonical edge list -> symmetric arc list (the device graph the Boruvka rounds scan),
// and the synthetic generators of BASELINE.json configs 3-5 (R-MAT s24/s26, 2D grid 16k^2).
//
// The arc list is the device form of the reference's per-node neighbour files: node_<id>.json
// holds {"neighbors": {nbr: w}} for every vertex (create_graph_files.py:56-74), i.e. every
// undirected edge once from each side; ghs_implementation_mpi.py:74-92 loads exactly that per
// rank. Here it is one array of 2m arcs grouped by source, built with a rocPRIM radix sort.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <string>

#include "common.h"

namespace ghs {

static inline unsigned grid_cap(uint64_t items, unsigned per_block, unsigned cap) {
  uint64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

static inline int bits_for(uint64_t maxval) {  // bits needed to represent values <= maxval
  int b = 0;
  while (b < 64 && (maxval >> b)) ++b;
  return b ? b : 1;
}

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// canonical check: u < v < n and (u, v) strictly ascending
__global__ void k_check_canonical(uint32_t n, uint64_t m, const uint32_t *__restrict__ u, const uint32_t *__restrict__ v,
                                  unsigned int *__restrict__ bad) {
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < m; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t a = u[e], b = v[e];
    bool ok = a < b && b < n;
    if (ok && e > 0) {
      const uint32_t pa = u[e - 1], pb = v[e - 1];
      ok = (pa < a) || (pa == a && pb < b);
    }
    if (!ok) atomicOr(bad, 1u);
  }
}

// first e with u[e] >= lo and first e with u[e] >= hi (u ascending): one wave, binary search
__global__ void k_range_bounds(uint64_t m, const uint32_t *__restrict__ u, uint32_t lo, uint32_t hi,
                               unsigned long long *__restrict__ out) {
  if (threadIdx.x > 1) return;
  const uint32_t target = threadIdx.x == 0 ? lo : hi;
  uint64_t a = 0, b = m;
  while (a < b) {
    const uint64_t mid = (a + b) / 2;
    if (u[mid] < target) a = mid + 1; else b = mid;
  }
  out[threadIdx.x] = a;
}

__global__ void k_count_rev(uint64_t m, const uint32_t *__restrict__ v, uint32_t lo, uint32_t hi,
                            unsigned long long *__restrict__ cnt) {
  unsigned long long c = 0;
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < m; e += (uint64_t)gridDim.x * blockDim.x)
    c += (v[e] >= lo && v[e] < hi) ? 1 : 0;
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

// Arc ids: a < m is the forward arc u[a] -> v[a]; a >= m is the reverse arc v[a-m] -> u[a-m].
// Forward arcs of the range are the contiguous slice [bounds[0], bounds[1]) of the canonical
// list (sorted by u); reverse arcs are selected by v in [lo, hi) with a ballot compaction.
// Output: keys (source) and ids, forward slice first, then reverse arcs (block order).
__global__ void k_arc_keys_range(uint64_t m, const uint32_t *__restrict__ u, const uint32_t *__restrict__ v,
                                 uint32_t lo, uint32_t hi, unsigned long long *__restrict__ bounds,
                                 uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
  __shared__ uint32_t s_wcnt[4];
  __shared__ unsigned long long s_base;
  const uint64_t f0 = bounds[0], f1 = bounds[1], nf = f1 - f0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (uint64_t base = blockIdx.x * (uint64_t)blockDim.x; base < m; base += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t e = base + threadIdx.x;
    if (e >= f0 && e < f1) {
      keys[e - f0] = u[e];
      vals[e - f0] = (uint32_t)e;
    }
    uint32_t ve = 0;
    const bool sel = e < m && (ve = v[e], ve >= lo && ve < hi);
    const uint64_t b = __ballot(sel);
    if (lane == 0) s_wcnt[wid] = (uint32_t)__popcll(b);
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t t = s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
      s_base = t ? atomicAdd(bounds + 2, (unsigned long long)t) : 0ull;
    }
    __syncthreads();
    if (sel) {
      uint64_t pos = nf + s_base +
                     __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
      for (int w = 0; w < wid; ++w) pos += s_wcnt[w];
      keys[pos] = ve;
      vals[pos] = (uint32_t)(e + m);
    }
    __syncthreads();
  }
}

// in place: adst[p] holds the sorted arc id on entry
__global__ void k_arc_fill(uint64_t A, uint64_t m, const uint32_t *__restrict__ u, const uint32_t *__restrict__ v,
                           const uint32_t *__restrict__ w, uint32_t *__restrict__ adst, uint64_t *__restrict__ akey) {
  for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < A; p += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t a = adst[p];
    const bool fwd = a < m;
    const uint32_t e = fwd ? a : (uint32_t)(a - m);
    adst[p] = fwd ? v[e] : u[e];
    akey[p] = ((uint64_t)w[e] << 32) | e;
  }
}

// ---- R-MAT ---------------------------------------------------------------------------------
// Graph500 quadrant probabilities as exact integer thresholds on a uniform 32-bit draw.
constexpr uint32_t RMAT_TA = (uint32_t)((57ull << 32) / 100);
constexpr uint32_t RMAT_TAB = (uint32_t)((76ull << 32) / 100);
constexpr uint32_t RMAT_TABC = (uint32_t)((95ull << 32) / 100);

__host__ __device__ __forceinline__ uint32_t rmat_perm(uint32_t x, uint32_t scale, uint64_t seed) {
  // bijection on [0, 2^scale): odd multiply, xorshift, odd multiply, xor constant (all mod 2^scale)
  const uint32_t mask = (scale >= 32) ? 0xffffffffu : ((1u << scale) - 1u);
  const uint32_t c1 = (uint32_t)splitmix64(seed ^ 0x1111) | 1u;
  const uint32_t c2 = (uint32_t)splitmix64(seed ^ 0x2222) | 1u;
  const uint32_t c3 = (uint32_t)splitmix64(seed ^ 0x3333);
  x = (x * c1) & mask;
  x ^= x >> ((scale + 1) / 2);
  x = (x * c2) & mask;
  x ^= x >> ((scale + 2) / 3);
  return (x ^ c3) & mask;
}

// tuple t -> packed canonical key (min << scale | max), or all-ones (2*scale bits) for a self-loop
__host__ __device__ __forceinline__ uint64_t rmat_tuple(uint64_t t, uint32_t scale, uint64_t seed) {
  uint64_t state = splitmix64(seed ^ splitmix64(t + 0x5bd1e995ull));
  uint32_t uu = 0, vv = 0;
  uint64_t bits = 0;
  for (uint32_t l = 0; l < scale; ++l) {
    if ((l & 1) == 0) {
      state += 0x9e3779b97f4a7c15ull;
      bits = splitmix64(state);
    }
    const uint32_t r = (l & 1) ? (uint32_t)(bits >> 32) : (uint32_t)bits;
    const uint32_t bu = r >= RMAT_TAB ? 1u : 0u;
    const uint32_t bv = (r >= RMAT_TA && r < RMAT_TAB) || r >= RMAT_TABC ? 1u : 0u;
    uu = (uu << 1) | bu;
    vv = (vv << 1) | bv;
  }
  uu = rmat_perm(uu, scale, seed);
  vv = rmat_perm(vv, scale, seed);
  if (uu == vv) return (scale >= 32) ? ~0ull : ((1ull << (2 * scale)) - 1ull);
  const uint32_t a = uu < vv ? uu : vv, b = uu < vv ? vv : uu;
  return ((uint64_t)a << scale) | b;
}

__global__ void k_rmat_tuples(uint64_t T, uint32_t scale, uint64_t seed, uint64_t *__restrict__ keys) {
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < T; t += (uint64_t)gridDim.x * blockDim.x)
    keys[t] = rmat_tuple(t, scale, seed);
}

__global__ void k_rmat_decode(uint64_t m, uint32_t scale, uint64_t wseed, const uint64_t *__restrict__ keys,
                              uint32_t *__restrict__ u, uint32_t *__restrict__ v, uint32_t *__restrict__ w) {
  const uint64_t mask = (1ull << scale) - 1ull;
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < m; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[e];
    u[e] = (uint32_t)(k >> scale);
    v[e] = (uint32_t)(k & mask);
    w[e] = mix32((uint32_t)e ^ (uint32_t)wseed);
  }
}

// ---- grid ----------------------------------------------------------------------------------
__global__ void k_grid(uint32_t k, uint32_t mode, uint64_t wseed, uint32_t *__restrict__ u, uint32_t *__restrict__ v,
                       uint32_t *__restrict__ w) {
  const uint64_t n = (uint64_t)k * k;
  for (uint64_t x = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; x < n; x += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = (uint32_t)(x / k), c = (uint32_t)(x % k);
    uint64_t e = (r < k - 1) ? (uint64_t)r * (2ull * k - 1) + 2ull * c
                             : (uint64_t)(k - 1) * (2ull * k - 1) + c;
    if (c < k - 1) {
      u[e] = (uint32_t)x; v[e] = (uint32_t)(x + 1);
      w[e] = mode ? (uint32_t)e : mix32((uint32_t)e ^ (uint32_t)wseed);
      ++e;
    }
    if (r < k - 1) {
      u[e] = (uint32_t)x; v[e] = (uint32_t)(x + k);
      w[e] = mode ? (uint32_t)e : mix32((uint32_t)e ^ (uint32_t)wseed);
    }
  }
}

}  // namespace ghs

using namespace ghs;

extern "C" {

size_t ghs_build_arcs_temp_bytes(uint32_t n, uint64_t m) {
  size_t cub = 0;
  const uint64_t A = 2 * m;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cub, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                          (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)(A ? A : 1), 0,
                                          bits_for(n ? n - 1 : 0));
  return align256(cub) + 256;
}

int ghs_count_arcs_range(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, uint32_t src_lo,
                         uint32_t src_hi, void *d_temp, size_t temp_bytes, void *stream, uint64_t *num_arcs) {
  hipStream_t st = (hipStream_t)stream;
  if (!num_arcs) GHS_FAIL(GHS_E_ARG, "num_arcs is NULL");
  *num_arcs = 0;
  if (src_hi > n || src_lo > src_hi) GHS_FAIL(GHS_E_ARG, "bad source range");
  if (m == 0 || src_lo == src_hi) return GHS_OK;
  if (!d_u || !d_v || !d_temp || temp_bytes < 256) GHS_FAIL(GHS_E_ARG, "NULL pointer / temp too small");
  unsigned long long *cnt = reinterpret_cast<unsigned long long *>(d_temp);  // [0] fwd lo, [1] fwd hi, [2] rev
  GHS_HIP_CHECK(hipMemsetAsync(cnt, 0, 3 * sizeof(unsigned long long), st));
  k_range_bounds<<<1, 64, 0, st>>>(m, d_u, src_lo, src_hi, cnt);
  k_count_rev<<<grid_cap(m, 256, 4096), 256, 0, st>>>(m, d_v, src_lo, src_hi, cnt + 2);
  GHS_HIP_CHECK(hipGetLastError());
  unsigned long long h[3];
  GHS_HIP_CHECK(hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, st));
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  *num_arcs = (h[1] - h[0]) + h[2];
  return GHS_OK;
}

int ghs_build_arcs_range(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                         uint32_t src_lo, uint32_t src_hi, uint32_t *d_asrc, uint32_t *d_adst, uint64_t *d_akey,
                         uint64_t arc_capacity, void *d_temp, size_t temp_bytes, void *stream, uint64_t *num_arcs) {
  hipStream_t st = (hipStream_t)stream;
  if (!num_arcs) GHS_FAIL(GHS_E_ARG, "num_arcs is NULL");
  *num_arcs = 0;
  if (src_hi > n || src_lo > src_hi) GHS_FAIL(GHS_E_ARG, "bad source range");
  if (m == 0 || src_lo == src_hi) return GHS_OK;
  if (m >= (1ull << 31)) GHS_FAIL(GHS_E_ARG, "m must be < 2^31 (arc ids are 32-bit)");
  if (!d_u || !d_v || !d_w || !d_asrc || !d_adst || !d_akey || !d_temp) GHS_FAIL(GHS_E_ARG, "NULL pointer");
  if ((((uintptr_t)d_asrc) | ((uintptr_t)d_adst) | ((uintptr_t)d_akey) | ((uintptr_t)d_temp)) & 15)
    GHS_FAIL(GHS_E_ARG, "arc arrays and temp must be 16-byte aligned");
  if (temp_bytes < ghs_build_arcs_temp_bytes(n, m)) GHS_FAIL(GHS_E_NOMEM, "temp too small");
  unsigned long long *cnt = reinterpret_cast<unsigned long long *>(d_temp);  // [0..2] range, [3] canon flag
  void *cub_temp = (char *)d_temp + 256;
  size_t cub_bytes = temp_bytes - 256;

  GHS_HIP_CHECK(hipMemsetAsync(cnt, 0, 4 * sizeof(unsigned long long), st));
  k_check_canonical<<<grid_cap(m, 256, 16384), 256, 0, st>>>(n, m, d_u, d_v, (unsigned int *)(cnt + 3));
  k_range_bounds<<<1, 64, 0, st>>>(m, d_u, src_lo, src_hi, cnt);
  k_count_rev<<<grid_cap(m, 256, 4096), 256, 0, st>>>(m, d_v, src_lo, src_hi, cnt + 2);
  GHS_HIP_CHECK(hipGetLastError());
  unsigned long long h[4];
  GHS_HIP_CHECK(hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, st));
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  if (h[3]) GHS_FAIL(GHS_E_NONCANON, "edge list is not canonical (need u < v < n, strictly ascending (u, v))");
  const uint64_t nf = h[1] - h[0], nr = h[2], A = nf + nr;
  if (A > arc_capacity) GHS_FAIL(GHS_E_NOMEM, "arc capacity too small: need " + std::to_string(A));
  if (A == 0) return GHS_OK;
  // keys_in / vals_in live in d_akey's storage (A * 8 bytes = A * 4 + A * 4); sorted keys land
  // directly in d_asrc, sorted arc ids in d_adst (then rewritten in place by k_arc_fill).
  uint32_t *keys_in = reinterpret_cast<uint32_t *>(d_akey);
  uint32_t *vals_in = keys_in + A;
  GHS_HIP_CHECK(hipMemsetAsync(cnt + 2, 0, sizeof(unsigned long long), st));
  k_arc_keys_range<<<grid_cap(m, 256, 16384), 256, 0, st>>>(m, d_u, d_v, src_lo, src_hi, cnt, keys_in, vals_in);
  GHS_HIP_CHECK(hipGetLastError());
  GHS_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(cub_temp, cub_bytes, keys_in, d_asrc, vals_in, d_adst, (size_t)A, 0,
                                                   bits_for(n - 1), st));
  k_arc_fill<<<grid_cap(A, 256, 16384), 256, 0, st>>>(A, m, d_u, d_v, d_w, d_adst, d_akey);
  GHS_HIP_CHECK(hipGetLastError());
  *num_arcs = A;
  return GHS_OK;
}

int ghs_build_arcs(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                   uint32_t *d_asrc, uint32_t *d_adst, uint64_t *d_akey, void *d_temp, size_t temp_bytes,
                   void *stream) {
  uint64_t A = 0;
  return ghs_build_arcs_range(n, m, d_u, d_v, d_w, 0, n, d_asrc, d_adst, d_akey, 2 * m, d_temp, temp_bytes, stream, &A);
}

int ghs_check_canonical(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, void *stream, int *ok) {
  hipStream_t st = (hipStream_t)stream;
  if (!ok) GHS_FAIL(GHS_E_ARG, "ok is NULL");
  *ok = 1;
  if (m == 0) return GHS_OK;
  if (!d_u || !d_v) GHS_FAIL(GHS_E_ARG, "NULL pointer");
  unsigned int *bad = nullptr;
  GHS_HIP_CHECK(hipMallocAsync((void **)&bad, sizeof(unsigned int), st));
  GHS_HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(unsigned int), st));
  k_check_canonical<<<grid_cap(m, 256, 16384), 256, 0, st>>>(n, m, d_u, d_v, bad);
  unsigned int h_bad = 0;
  hipError_t e = hipMemcpyAsync(&h_bad, bad, sizeof(h_bad), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFreeAsync(bad, st);
  GHS_HIP_CHECK(e);
  *ok = h_bad ? 0 : 1;
  return GHS_OK;
}

size_t ghs_rmat_temp_bytes(uint32_t scale, uint32_t edgefactor) {
  const uint64_t T = (uint64_t)edgefactor << scale;
  size_t sort_b = 0, uniq_b = 0;
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, sort_b, (const uint64_t *)nullptr, (uint64_t *)nullptr, (size_t)T, 0,
                                         (int)(2 * scale));
  (void)hipcub::DeviceSelect::Unique(nullptr, uniq_b, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                     (uint64_t *)nullptr, (size_t)T);
  return 2 * align256(T * 8) + align256(sort_b > uniq_b ? sort_b : uniq_b) + 256;
}

int ghs_rmat_generate(uint32_t scale, uint32_t edgefactor, uint64_t seed, uint64_t wseed, uint32_t *d_u,
                      uint32_t *d_v, uint32_t *d_w, uint64_t *m_out, void *d_temp, size_t temp_bytes, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!m_out || !d_u || !d_v || !d_w || !d_temp) GHS_FAIL(GHS_E_ARG, "NULL pointer");
  if (scale < 1 || scale > 31) GHS_FAIL(GHS_E_ARG, "scale must be in [1, 31]");
  const uint64_t T = (uint64_t)edgefactor << scale;
  if (T == 0 || T >= (1ull << 32)) GHS_FAIL(GHS_E_ARG, "edgefactor * 2^scale must be in [1, 2^32)");
  if (temp_bytes < ghs_rmat_temp_bytes(scale, edgefactor)) GHS_FAIL(GHS_E_NOMEM, "temp too small");
  char *base = (char *)d_temp;
  uint64_t *ka = (uint64_t *)base;
  uint64_t *kb = (uint64_t *)(base + align256(T * 8));
  uint64_t *nsel = (uint64_t *)(base + 2 * align256(T * 8));
  void *cub_temp = base + 2 * align256(T * 8) + 256;
  size_t cub_bytes = temp_bytes - (2 * align256(T * 8) + 256);

  k_rmat_tuples<<<grid_cap(T, 256, 16384), 256, 0, st>>>(T, scale, seed, ka);
  GHS_HIP_CHECK(hipGetLastError());
  GHS_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(cub_temp, cub_bytes, ka, kb, (size_t)T, 0, (int)(2 * scale), st));
  GHS_HIP_CHECK(hipcub::DeviceSelect::Unique(cub_temp, cub_bytes, kb, ka, nsel, (size_t)T, st));
  uint64_t cnt = 0, last = 0;
  GHS_HIP_CHECK(hipMemcpyAsync(&cnt, nsel, 8, hipMemcpyDeviceToHost, st));
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  if (cnt) {
    GHS_HIP_CHECK(hipMemcpyAsync(&last, ka + (cnt - 1), 8, hipMemcpyDeviceToHost, st));
    GHS_HIP_CHECK(hipStreamSynchronize(st));
    if (last == ((1ull << (2 * scale)) - 1ull)) --cnt;  // the self-loop marker sorts last
  }
  k_rmat_decode<<<grid_cap(cnt, 256, 16384), 256, 0, st>>>(cnt, scale, wseed, ka, d_u, d_v, d_w);
  GHS_HIP_CHECK(hipGetLastError());
  *m_out = cnt;
  return GHS_OK;
}

int ghs_grid_generate(uint32_t k, uint32_t mode, uint64_t wseed, uint32_t *d_u, uint32_t *d_v, uint32_t *d_w,
                      void *stream) {
  if (k < 2) return GHS_OK;
  if ((uint64_t)k * k >= (1ull << 32)) GHS_FAIL(GHS_E_ARG, "k*k must be < 2^32");
  if (!d_u || !d_v || !d_w) GHS_FAIL(GHS_E_ARG, "NULL pointer");
  const uint64_t n = (uint64_t)k * k;
  k_grid<<<grid_cap(n, 256, 16384), 256, 0, (hipStream_t)stream>>>(k, mode, wseed, d_u, d_v, d_w);
  GHS_HIP_CHECK(hipGetLastError());
  return GHS_OK;
}

}  // extern "C"
