// Where the CSR row derivation's time goes (round 6): a k_select-shaped stream (wave-private slices
// of 256-edge tiles, next tile's loads in flight) over the R-MAT s24 list in COO form and in CSR
// form, with the row derivation switched in piece by piece. Driven by tools/csr_rows_bench.py.
//   0 COO: u, v, w streamed (12 B/edge), checksum
//   1 CSR: v, w streamed, u = the tile's first row (no derivation)
//   2 CSR: + the offsets window loaded per tile (prefetched one tile ahead), no LDS
//   3 CSR: + head table writes + in-lane max (no wave scan)
//   4 CSR: + the wave DPP scan (the full derivation)
//   5 CSR: 4 + one trow store per tile (lane 0)
//   6 CSR: v, w + an offsets window per tile at a data-independent row (t0 / 16): the load alone
//   7 CSR: the window of the next tile from this tile's ballot (one window per tile, no inner loop)
//   8 CSR: 7 with the window loaded as 16-B per lane (256 rows) from an aligned base
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
  return x;
}
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t csr_row(const uint32_t *off, uint32_t n, uint32_t e) {
  uint32_t lo = 0, hi = n - 1;
  while (lo < hi) {
    const uint32_t mid = lo + ((hi - lo + 1) >> 1);
    if (off[mid] <= e) lo = mid; else hi = mid - 1;
  }
  return lo;
}

template <int K>
__global__ __launch_bounds__(256) void k_rows(uint32_t n, uint32_t m, const uint32_t *__restrict__ u,
                                              const uint32_t *__restrict__ off, const uint32_t *__restrict__ v,
                                              const uint32_t *__restrict__ w, uint32_t *__restrict__ trow,
                                              uint32_t *sink) {
  __shared__ uint32_t s_head[4][256];
  const uint32_t lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint32_t gw = blockIdx.x * 4 + wid, W = gridDim.x * 4;
  const uint32_t Q = ((m + W - 1) / W + 255) & ~255u;
  const uint32_t vb = Q * gw, ve = min(vb + Q, m);
  uint32_t acc = 0;
  if (vb >= ve) return;
  reinterpret_cast<uint4 *>(s_head[wid])[lane] = make_uint4(0, 0, 0, 0);
  uint32_t row = K ? csr_row(off, n, vb) : 0;
  auto win = [&](uint32_t r, uint32_t &o, uint32_t &o2) {
    const uint32_t ri = r + 1 + lane;
    const uint32_t a = off[min(ri, n)], b = off[min(ri + 1, n)];
    o = ri <= n ? a : 0xffffffffu;
    o2 = ri < n ? b : 0xffffffffu;
  };
  uint32_t o = 0, o2 = 0;
  if (K >= 2) win(row, o, o2);
  if (K == 8) o = off[min(row + 1 + lane, n)];
  const uint32_t i0 = vb + lane * 4;
  uint4 cu = K == 0 ? *reinterpret_cast<const uint4 *>(u + min(i0, m - 4)) : make_uint4(0, 0, 0, 0);
  uint4 cv = *reinterpret_cast<const uint4 *>(v + min(i0, m - 4)), cw = *reinterpret_cast<const uint4 *>(w + min(i0, m - 4));
  for (uint32_t t0 = vb; t0 < ve; t0 += 256) {
    uint32_t a[4] = {cu.x, cu.y, cu.z, cu.w};
    const uint32_t b[4] = {cv.x, cv.y, cv.z, cv.w}, ww[4] = {cw.x, cw.y, cw.z, cw.w};
    if (K == 1) {
      for (int j = 0; j < 4; ++j) a[j] = row;
    }
    if (K == 6) {
      uint32_t oo = 0, oo2 = 0;
      win(t0 >> 4, oo, oo2);
      acc += oo;
      for (int j = 0; j < 4; ++j) a[j] = row;
    }
    if (K == 7) {
      const uint32_t tend = t0 + 256;
      const uint64_t le = __ballot(o <= tend);
      row += (uint32_t)__popcll(le);
      win(row, o, o2);
      for (int j = 0; j < 4; ++j) a[j] = row;
    }
    if (K == 8) {
      const uint32_t tend = t0 + 256;
      const uint64_t le = __ballot(o <= tend);
      row += (uint32_t)__popcll(le);
      const uint32_t base = (row + 1) & ~3u;
      const uint4 q = *reinterpret_cast<const uint4 *>(off + min(base + lane * 4, n - 4));
      o = q.x;
      acc += q.y ^ q.z ^ q.w;
      for (int j = 0; j < 4; ++j) a[j] = row;
    }
    if (K >= 2 && K <= 5) {
      if (K == 5 && lane == 0) trow[t0 >> 8] = row;
      const uint32_t rin = row, tend = t0 + 256;
      uint32_t r = row;
      for (;;) {
        const uint32_t ri = r + 1 + lane;
        if (K >= 3 && (ri < n) & (o < o2) & (o > t0) & (o < tend)) s_head[wid][o - t0] = ri;
        const uint64_t le = __ballot(o <= tend);
        if (le != ~0ull) {
          r += (uint32_t)__popcll(le);
          break;
        }
        r += 64;
        win(r, o, o2);
      }
      row = min(r, n - 1);
      win(row, o, o2);  // next tile's window
      if (K >= 3) {
        __builtin_amdgcn_wave_barrier();
        const uint4 h = reinterpret_cast<const uint4 *>(s_head[wid])[lane];
        const uint32_t x0 = h.x, x1 = max(x0, h.y), x2 = max(x1, h.z), x3 = max(x2, h.w);
        const uint32_t base = K >= 4 ? max(rin, wave_shr1(wave_incl_max(x3))) : rin;
        a[0] = max(base, x0); a[1] = max(base, x1); a[2] = max(base, x2); a[3] = max(base, x3);
      } else {
        for (int j = 0; j < 4; ++j) a[j] = rin;
      }
    }
    const uint32_t ni = min(t0 + 256 + lane * 4, m - 4);
    if (K == 0) cu = *reinterpret_cast<const uint4 *>(u + ni);
    cv = *reinterpret_cast<const uint4 *>(v + ni);
    cw = *reinterpret_cast<const uint4 *>(w + ni);
    for (int j = 0; j < 4; ++j) acc += (a[j] < b[j]) + ww[j];
    asm volatile("" ::"v"(cv.x), "v"(cw.x), "v"(cu.x));
  }
  if (acc == 0x1234567u) sink[0] = acc;
}
}  // namespace

extern "C" int csr_rows_run(int kind, uint32_t n, uint32_t m, const uint32_t *u, const uint32_t *off, const uint32_t *v,
                            const uint32_t *w, uint32_t *trow, uint32_t *sink, int grid, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (kind) {
    case 0: k_rows<0><<<grid, 256, 0, st>>>(n, m, u, off, v, w, trow, sink); break;
    case 1: k_rows<1><<<grid, 256, 0, st>>>(n, m, u, off, v, w, trow, sink); break;
    case 2: k_rows<2><<<grid, 256, 0, st>>>(n, m, u, off, v, w, trow, sink); break;
    case 3: k_rows<3><<<grid, 256, 0, st>>>(n, m, u, off, v, w, trow, sink); break;
    case 4: k_rows<4><<<grid, 256, 0, st>>>(n, m, u, off, v, w, trow, sink); break;
    case 5: k_rows<5><<<grid, 256, 0, st>>>(n, m, u, off, v, w, trow, sink); break;
    case 6: k_rows<6><<<grid, 256, 0, st>>>(n, m, u, off, v, w, trow, sink); break;
    case 7: k_rows<7><<<grid, 256, 0, st>>>(n, m, u, off, v, w, trow, sink); break;
    case 8: k_rows<8><<<grid, 256, 0, st>>>(n, m, u, off, v, w, trow, sink); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
