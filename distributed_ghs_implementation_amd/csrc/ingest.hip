// Ingest: the synthetic generators of BASELINE.json configs 3-5 (R-MAT s24/s26, 2D grid 16k^2)
// and the device-side canonicity check. A generator's output is the canonical edge list of
// include/ghs_mst.h (u < v, ascending (u, v), unique) — the device form of the reference's
// graph files (create_graph_files.py:43-89 writes every undirected edge once in
// graph_metadata.json). The reference's generator is networkx's seeded ER G(n, p)
// (create_graph_files.py:13-40); R-MAT and grids are the BASELINE scales it cannot reach. The
// canonical sort/dedupe is a rocPRIM radix sort of 64-bit (min << scale | max) keys, then a
// two-pass unique + decode (k_uniq_*).
// The CPU restatement of both generators (test infrastructure) is oracle/generators.c.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/device/device_reduce.hpp>
#include <rocprim/iterator/transform_iterator.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <mutex>
#include <unordered_map>

#include <string>

#include "common.h"

namespace ghs {

static inline unsigned grid_cap(uint64_t items, unsigned per_block, unsigned cap) {
  uint64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
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

// CSR row offsets of a canonical list (ABI 9, ghs_csr_offsets): off[r] = the first edge of row r.
// Edge e writes the offsets of the rows (u[e - 1], u[e]] (every row from 0 for e = 0, up to n for
// e = m): each row's entry is written exactly once, by the edge that starts it or by the first
// edge past it when it is empty. u ascending is required (the solve validates the offsets).
__global__ void k_csr_offsets(uint32_t n, uint64_t m, const uint32_t *__restrict__ u, uint32_t *__restrict__ off) {
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e <= m; e += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t lo = e == 0 ? -1 : (int64_t)u[e - 1];
    const int64_t hi = e == m ? (int64_t)n : (int64_t)min(u[e], n);
    for (int64_t r = lo + 1; r <= hi; ++r) off[r] = (uint32_t)e;
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

// Unique + decode of the sorted keys in two passes over them (rocPRIM's unique, a partition
// over 2 GB of keys at s24, took 8 ms; these are streaming passes): a key is kept when it differs
// from its predecessor and is not the self-loop marker (which sorts last). Pass 1 counts the kept
// keys per tile, one block scans the tile counts, pass 2 writes each kept key's (u, v, w) at its
// rank — the weight hashes the output position, as the canonical list's edge id.
constexpr int UQ_BLOCK = 256;
constexpr int UQ_ROWS = 16;  // a tile is UQ_ROWS rows of UQ_BLOCK consecutive keys
constexpr uint64_t UQ_TILE = (uint64_t)UQ_BLOCK * UQ_ROWS;

__device__ __forceinline__ bool uq_keep(const uint64_t *__restrict__ keys, uint64_t i, uint64_t T, uint64_t marker,
                                        uint64_t *k_out) {
  if (i >= T) return false;
  const uint64_t k = keys[i];
  *k_out = k;
  return k != marker && (i == 0 || keys[i - 1] != k);
}

__global__ __launch_bounds__(UQ_BLOCK) void k_uniq_count(const uint64_t *__restrict__ keys, uint64_t T, uint64_t marker,
                                                         uint32_t *__restrict__ tile_cnt) {
  __shared__ uint32_t s_w[UQ_BLOCK / 64];
  const uint64_t base = blockIdx.x * UQ_TILE;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < UQ_ROWS; ++j) {
    uint64_t k;
    c += uq_keep(keys, base + (uint64_t)j * UQ_BLOCK + threadIdx.x, T, marker, &k) ? 1u : 0u;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x / 64] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < UQ_BLOCK / 64; ++w) t += s_w[w];
    tile_cnt[blockIdx.x] = t;
  }
}

// exclusive scan of the tile counts in place (one block of 1024), total to *total
__global__ __launch_bounds__(1024) void k_uniq_scan(uint32_t *__restrict__ cnt, uint32_t ntiles,
                                                    uint64_t *__restrict__ total) {
  __shared__ uint32_t s_part[1024];
  const uint32_t per = (ntiles + 1023) / 1024;
  const uint32_t b = threadIdx.x * per;
  uint32_t sum = 0;
  for (uint32_t i = 0; i < per && b + i < ntiles; ++i) sum += cnt[b + i];
  s_part[threadIdx.x] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const uint32_t o = threadIdx.x >= (unsigned)d ? s_part[threadIdx.x - d] : 0;
    __syncthreads();
    s_part[threadIdx.x] += o;
    __syncthreads();
  }
  uint32_t run = s_part[threadIdx.x] - sum;
  for (uint32_t i = 0; i < per && b + i < ntiles; ++i) {
    const uint32_t c = cnt[b + i];
    cnt[b + i] = run;
    run += c;
  }
  if (threadIdx.x == 1023) *total = s_part[1023];
}

__global__ __launch_bounds__(UQ_BLOCK) void k_uniq_write(const uint64_t *__restrict__ keys, uint64_t T, uint64_t marker,
                                                         const uint32_t *__restrict__ tile_off, uint32_t scale,
                                                         uint64_t wseed, uint32_t *__restrict__ u,
                                                         uint32_t *__restrict__ v, uint32_t *__restrict__ w) {
  __shared__ uint32_t s_cnt[UQ_ROWS][UQ_BLOCK / 64];
  const uint64_t base = blockIdx.x * UQ_TILE;
  const int lane = threadIdx.x & 63, wid = threadIdx.x / 64;
  const uint64_t lt = (1ull << lane) - 1ull;
  uint64_t kk[UQ_ROWS];
  uint64_t masks[UQ_ROWS];
#pragma unroll
  for (int j = 0; j < UQ_ROWS; ++j) {
    const bool keep = uq_keep(keys, base + (uint64_t)j * UQ_BLOCK + threadIdx.x, T, marker, &kk[j]);
    masks[j] = __ballot(keep);
    if (lane == 0) s_cnt[j][wid] = (uint32_t)__popcll(masks[j]);
  }
  __syncthreads();
  const uint64_t vmask = (1ull << scale) - 1ull;
  uint32_t row_base = tile_off[blockIdx.x];
#pragma unroll
  for (int j = 0; j < UQ_ROWS; ++j) {
    uint32_t before = 0, row = 0;
#pragma unroll
    for (int x = 0; x < UQ_BLOCK / 64; ++x) {
      const uint32_t c = s_cnt[j][x];
      before += x < wid ? c : 0u;
      row += c;
    }
    if ((masks[j] >> lane) & 1ull) {
      const uint32_t o = row_base + before + (uint32_t)__popcll(masks[j] & lt);
      u[o] = (uint32_t)(kk[j] >> scale);
      v[o] = (uint32_t)(kk[j] & vmask);
      w[o] = mix32(o ^ (uint32_t)wseed);
    }
    row_base += row;
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

int ghs_csr_offsets(uint32_t n, uint64_t m, const uint32_t *d_u, uint32_t *d_off, void *stream) {
  if (!d_off || (m && !d_u)) GHS_FAIL(GHS_E_ARG, "NULL pointer");
  if (m >= (1ull << 31)) GHS_FAIL(GHS_E_ARG, "m must be < 2^31");
  k_csr_offsets<<<grid_cap(m + 1, 256, 16384), 256, 0, (hipStream_t)stream>>>(n, m, d_u, d_off);
  GHS_HIP_CHECK(hipGetLastError());
  return GHS_OK;
}

size_t ghs_rmat_temp_bytes(uint32_t scale, uint32_t edgefactor) {
  const uint64_t T = (uint64_t)edgefactor << scale;
  size_t sort_b = 0;
  (void)rocprim::radix_sort_keys(nullptr, sort_b, (const uint64_t *)nullptr, (uint64_t *)nullptr, (size_t)T, 0u,
                                 2u * scale);
  const size_t tiles_b = align256(((T + UQ_TILE - 1) / UQ_TILE) * 4);
  return 2 * align256(T * 8) + align256(sort_b > tiles_b ? sort_b : tiles_b) + 256;
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
  void *prim_temp = base + 2 * align256(T * 8) + 256;
  size_t prim_bytes = temp_bytes - (2 * align256(T * 8) + 256);
  const uint64_t ntiles = (T + UQ_TILE - 1) / UQ_TILE;
  uint32_t *tiles = (uint32_t *)prim_temp;  // reused after the sort
  const uint64_t marker = (1ull << (2 * scale)) - 1ull;  // a self-loop's key (sorts last)

  k_rmat_tuples<<<grid_cap(T, 256, 16384), 256, 0, st>>>(T, scale, seed, ka);
  GHS_HIP_CHECK(hipGetLastError());
  GHS_HIP_CHECK(rocprim::radix_sort_keys(prim_temp, prim_bytes, ka, kb, (size_t)T, 0u, 2u * scale, st));
  k_uniq_count<<<(unsigned)ntiles, UQ_BLOCK, 0, st>>>(kb, T, marker, tiles);
  k_uniq_scan<<<1, 1024, 0, st>>>(tiles, (uint32_t)ntiles, nsel);
  k_uniq_write<<<(unsigned)ntiles, UQ_BLOCK, 0, st>>>(kb, T, marker, tiles, scale, wseed, d_u, d_v, d_w);
  GHS_HIP_CHECK(hipGetLastError());
  uint64_t cnt = 0;
  GHS_HIP_CHECK(hipMemcpyAsync(&cnt, nsel, 8, hipMemcpyDeviceToHost, st));
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  *m_out = cnt;
  return GHS_OK;
}

struct FlagOne {
  __host__ __device__ uint32_t operator()(uint8_t f) const { return f ? 1u : 0u; }
};

}  // extern "C"

// ghs_flags_to_eids' per-device temporary storage (grown on demand), freed by ghs_release_cache
// (it used to be held until the process ended, outside torch's allocator's view)
namespace {
struct EidTemp {
  void *p = nullptr;
  size_t bytes = 0;
  uint32_t *h_cnt = nullptr;  // pinned: the selected count
  uint32_t *d_cnt = nullptr;
};
std::mutex g_eid_mu;
std::unordered_map<int, EidTemp> g_eid_temps;
}  // namespace

void ghs_release_eid_temps() {
  std::lock_guard<std::mutex> lock(g_eid_mu);
  int cur = 0;
  const bool have = hipGetDevice(&cur) == hipSuccess;
  for (auto &kv : g_eid_temps) {
    (void)hipSetDevice(kv.first);
    if (kv.second.p) (void)hipFree(kv.second.p);
    if (kv.second.d_cnt) (void)hipFree(kv.second.d_cnt);
    if (kv.second.h_cnt) (void)hipHostFree(kv.second.h_cnt);
  }
  g_eid_temps.clear();
  if (have) (void)hipSetDevice(cur);
}

extern "C" {

// The MSF edge ids of a flag range (a rank's own range for collect_results,
// ghs_implementation_mpi.py:760-779): rocPRIM's flagged select over a counting input. Its temporary
// storage is kept per device (grown on demand); the count comes back through pinned memory.
int ghs_flags_to_eids(const uint8_t *d_in_mst, uint64_t lo, uint64_t hi, uint32_t *d_eids, uint64_t capacity,
                      uint64_t *count, void *stream) {
  if (!count || (hi > lo && (!d_in_mst || !d_eids))) GHS_FAIL(GHS_E_ARG, "NULL pointer");
  if (hi < lo || hi >= (1ull << 32)) GHS_FAIL(GHS_E_ARG, "bad range (need lo <= hi < 2^32)");
  *count = 0;
  if (hi == lo) return GHS_OK;
  std::lock_guard<std::mutex> lock(g_eid_mu);
  int dev = 0;
  GHS_HIP_CHECK(hipGetDevice(&dev));
  EidTemp &t = g_eid_temps[dev];
  hipStream_t st = (hipStream_t)stream;
  const size_t N = (size_t)(hi - lo);
  rocprim::counting_iterator<uint32_t> in((uint32_t)lo);
  size_t need = 0;
  GHS_HIP_CHECK(rocprim::select(nullptr, need, in, d_in_mst + lo, d_eids, (uint32_t *)nullptr, N, st));
  if (!t.h_cnt) {
    GHS_HIP_CHECK(hipHostMalloc((void **)&t.h_cnt, sizeof(uint32_t), hipHostMallocDefault));
    GHS_HIP_CHECK(hipMalloc((void **)&t.d_cnt, sizeof(uint32_t)));
  }
  if (t.bytes < need) {
    if (t.p) (void)hipFree(t.p);
    t.p = nullptr;
    t.bytes = 0;
    GHS_HIP_CHECK(hipMalloc(&t.p, need));
    t.bytes = need;
  }
  // the output holds at most `capacity` ids: when the range is longer, count the flags first
  // (rocPRIM writes every selected id) and refuse the call instead of writing past it
  if (N > capacity) {
    auto ones = rocprim::make_transform_iterator(d_in_mst + lo, FlagOne());
    size_t rneed = 0;
    GHS_HIP_CHECK(rocprim::reduce(nullptr, rneed, ones, t.d_cnt, 0u, N, rocprim::plus<uint32_t>(), st));
    if (rneed > need) need = rneed;
    if (t.bytes < need) {
      if (t.p) (void)hipFree(t.p);
      t.p = nullptr;
      t.bytes = 0;
      GHS_HIP_CHECK(hipMalloc(&t.p, need));
      t.bytes = need;
    }
    GHS_HIP_CHECK(rocprim::reduce(t.p, rneed, ones, t.d_cnt, 0u, N, rocprim::plus<uint32_t>(), st));
    GHS_HIP_CHECK(hipMemcpyAsync(t.h_cnt, t.d_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    GHS_HIP_CHECK(hipStreamSynchronize(st));
    if (*t.h_cnt > capacity) GHS_FAIL(GHS_E_NOMEM, "more flagged edges than the output's capacity");
  }
  GHS_HIP_CHECK(rocprim::select(t.p, need, in, d_in_mst + lo, d_eids, t.d_cnt, N, st));
  GHS_HIP_CHECK(hipMemcpyAsync(t.h_cnt, t.d_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  GHS_HIP_CHECK(hipStreamSynchronize(st));
  *count = *t.h_cnt;
  return GHS_OK;
}

int ghs_rmat_tuples(uint32_t scale, uint32_t edgefactor, uint64_t seed, uint64_t *d_keys, void *stream) {
  if (!d_keys) GHS_FAIL(GHS_E_ARG, "NULL pointer");
  if (scale < 1 || scale > 31) GHS_FAIL(GHS_E_ARG, "scale must be in [1, 31]");
  const uint64_t T = (uint64_t)edgefactor << scale;
  if (T == 0 || T >= (1ull << 32)) GHS_FAIL(GHS_E_ARG, "edgefactor * 2^scale must be in [1, 2^32)");
  k_rmat_tuples<<<grid_cap(T, 256, 16384), 256, 0, (hipStream_t)stream>>>(T, scale, seed, d_keys);
  GHS_HIP_CHECK(hipGetLastError());
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
