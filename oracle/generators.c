/*
 * ORACLE — test infrastructure only. CPU restatement of the synthetic generators of
 * BASELINE.json configs 3-5, to pin the GPU generators of libghs_mst.so
 * (distributed_ghs_implementation_amd/csrc/ingest.hip) tuple for tuple (SURVEY.md §8(d):
 * "fixed seeds, reproducible by both CPU oracle and GPU generator").
 *
 * The reference's own generator is networkx's seeded ER G(n, p) with randint(1, 10) weights
 * (create_graph_files.py:13-40); it never reaches R-MAT or grid scale, so these generators are
 * the build's, restated here from their specification:
 *   R-MAT (Graph500 A, B, C, D = .57, .19, .19, .05): tuple t draws `scale` quadrant choices from
 *   a splitmix64 stream seeded by (seed, t), 2 choices per 64-bit draw (low word first), each a
 *   uniform 32-bit value against the integer thresholds floor(.57 * 2^32), floor(.76 * 2^32),
 *   floor(.95 * 2^32); quadrant bits (u, v): [0, A) -> (0, 0), [A, A+B) -> (0, 1),
 *   [A+B, A+B+C) -> (1, 0), [A+B+C, 1) -> (1, 1); then both ends go through the seeded vertex
 *   bijection rmat_perm. The canonical list (self-loops dropped, pairs deduplicated, sorted by
 *   (min, max)) gets weights w[e] = mix32(e ^ wseed), unique by construction.
 * Used by tests/test_generators.py (CPU: internal consistency) and tests/test_gpu_parity.py
 * (GPU vs this file, bit-exact).
 */
#include <stdint.h>
#include <stddef.h>

static uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

uint32_t oracle_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

/* the seeded bijection on [0, 2^scale): odd multiply, xorshift, odd multiply, xor constant */
static uint32_t rmat_perm(uint32_t x, uint32_t scale, uint64_t seed) {
  const uint32_t mask = scale >= 32 ? 0xffffffffu : ((1u << scale) - 1u);
  const uint32_t c1 = (uint32_t)splitmix64(seed ^ 0x1111) | 1u;
  const uint32_t c2 = (uint32_t)splitmix64(seed ^ 0x2222) | 1u;
  const uint32_t c3 = (uint32_t)splitmix64(seed ^ 0x3333);
  x = (x * c1) & mask;
  x ^= x >> ((scale + 1) / 2);
  x = (x * c2) & mask;
  x ^= x >> ((scale + 2) / 3);
  return (x ^ c3) & mask;
}

/* raw (permuted) endpoint pair of every tuple: uu[t], vv[t] for t < edgefactor << scale */
int oracle_rmat_pairs(uint32_t scale, uint32_t edgefactor, uint64_t seed, uint32_t *uu, uint32_t *vv) {
  if (scale < 1 || scale > 31 || !uu || !vv) return -1;
  const uint32_t TA = (uint32_t)((57ull << 32) / 100), TAB = (uint32_t)((76ull << 32) / 100),
                 TABC = (uint32_t)((95ull << 32) / 100);
  const uint64_t T = (uint64_t)edgefactor << scale;
  for (uint64_t t = 0; t < T; ++t) {
    uint64_t state = splitmix64(seed ^ splitmix64(t + 0x5bd1e995ull));
    uint64_t draw = 0;
    uint32_t a = 0, b = 0;
    for (uint32_t l = 0; l < scale; ++l) {
      if (l % 2 == 0) {
        state += 0x9e3779b97f4a7c15ull;
        draw = splitmix64(state);
      }
      const uint32_t r = (l % 2) ? (uint32_t)(draw >> 32) : (uint32_t)draw;
      uint32_t qu, qv;
      if (r < TA) { qu = 0; qv = 0; }
      else if (r < TAB) { qu = 0; qv = 1; }
      else if (r < TABC) { qu = 1; qv = 0; }
      else { qu = 1; qv = 1; }
      a = (a << 1) | qu;
      b = (b << 1) | qv;
    }
    uu[t] = rmat_perm(a, scale, seed);
    vv[t] = rmat_perm(b, scale, seed);
  }
  return 0;
}

/* weights of a canonical list of m edges: w[e] = mix32(e ^ wseed) */
void oracle_hash_weights(uint64_t m, uint64_t wseed, uint32_t *w) {
  for (uint64_t e = 0; e < m; ++e) w[e] = oracle_mix32((uint32_t)e ^ (uint32_t)wseed);
}
