/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by, or called from the product
 * path (distributed_ghs_implementation_amd/). Only tests/ and bench.py's cpu_baseline leg load it.
 *
 * The all-cores CPU baseline SURVEY.md §8(d) asks for beside the serial Kruskal: an OpenMP
 * Borůvka over the canonical edge list, computing the same canonical MSF as oracle/kruskal.c
 * (strict key (w, eid) == (w, min(u,v), max(u,v)); keys are unique, so the MSF is unique and
 * Borůvka and Kruskal agree edge for edge — checked by tests/test_oracle.py).
 *
 * It restates the reference's GHS phases as CPU rounds, like the GPU path does:
 *   min outgoing edge per fragment  (test / accept / reject / report, ghs_implementation.py:235-353)
 *   hook over it, mutual pair broken by the smaller id  (changeroot / connect, :155-199, :355-387)
 *   relabel every vertex to its new root  (initiate, :201-233)
 *   stop when no fragment has an outgoing edge  (termination, :389-413)
 * Each thread keeps a static chunk of the edge list and compacts its live edges in place
 * (intra-fragment edges dropped: the reference's REJECT), so later rounds read only survivors.
 */
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_E_ARG (-1)
#define ORC_E_NOMEM (-3)

static inline void amin_u64(uint64_t *p, uint64_t k) {
  uint64_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (k < cur && !__atomic_compare_exchange_n(p, &cur, k, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
}

/* Canonical input (u < v, ascending (u, v), unique; not re-validated here — kruskal.c's
 * oracle_check_canonical does that). in_mst: m bytes, zeroed here. threads <= 0: OpenMP default. */
int oracle_boruvka_omp(uint32_t n, uint64_t m, const uint32_t *u, const uint32_t *v, const uint32_t *w,
                       int threads, uint8_t *in_mst, uint64_t *total_weight, uint64_t *num_edges,
                       uint32_t *rounds_out) {
  if ((m && (!u || !v || !w || !in_mst)) || !total_weight || !num_edges || m > 0xffffffffull)
    return ORC_E_ARG;
  if (m) memset(in_mst, 0, m);
  *total_weight = 0;
  *num_edges = 0;
  if (rounds_out) *rounds_out = 0;
  if (n == 0 || m == 0) return ORC_OK;
  const int T = threads > 0 ? threads : omp_get_max_threads();
  uint32_t *comp = malloc((size_t)n * sizeof *comp);
  uint32_t *par = malloc((size_t)n * sizeof *par);
  uint32_t *nr = malloc((size_t)n * sizeof *nr);
  uint64_t *best = malloc((size_t)n * sizeof *best);
  uint32_t *live = malloc((size_t)m * sizeof *live);
  if (!comp || !par || !nr || !best || !live) {
    free(comp); free(par); free(nr); free(best); free(live);
    return ORC_E_NOMEM;
  }
  uint64_t tw = 0, ne = 0, round_hooks = 0;
  int moved = 0; /* pointer doubling: some parent moved this pass */
  uint32_t rounds = 0;
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    const uint64_t lo = m * (uint64_t)t / (uint64_t)nt, hi = m * (uint64_t)(t + 1) / (uint64_t)nt;
    for (uint64_t e = lo; e < hi; ++e) live[e] = (uint32_t)e;
    uint64_t mine = hi - lo;
#pragma omp for schedule(static)
    for (uint64_t x = 0; x < n; ++x) {
      comp[x] = (uint32_t)x;
      best[x] = UINT64_MAX;
    }
    for (;;) {
      /* min outgoing edge per fragment; intra-fragment edges leave the thread's live chunk */
      uint64_t k = lo;
      for (uint64_t i = lo; i < lo + mine; ++i) {
        const uint32_t e = live[i];
        const uint32_t cu = comp[u[e]], cv = comp[v[e]];
        if (cu == cv) continue;
        live[k++] = e;
        const uint64_t key = ((uint64_t)w[e] << 32) | e;
        amin_u64(&best[cu], key);
        amin_u64(&best[cv], key);
      }
      mine = k - lo;
#pragma omp barrier
#pragma omp single
      {
        round_hooks = 0;
        rounds++;
      }
      /* hook every root over its best edge; a mutual pair keeps the smaller id as root */
      uint64_t my_w = 0, my_e = 0;
#pragma omp for schedule(static)
      for (uint64_t x = 0; x < n; ++x) {
        const uint32_t c = (uint32_t)x;
        if (comp[c] != c) continue;
        const uint64_t b = best[c];
        par[c] = c;
        if (b == UINT64_MAX) continue;
        const uint32_t e = (uint32_t)b;
        const uint32_t a = comp[u[e]], d = comp[v[e]];
        const uint32_t other = a == c ? d : a;
        if (best[other] == b && c < other) continue; /* the mutual pair's root */
        par[c] = other;
        in_mst[e] = 1; /* one hook per edge: the mutual pair hooks once */
        my_w += w[e];
        my_e += 1;
      }
#pragma omp atomic
      tw += my_w;
#pragma omp atomic
      ne += my_e;
#pragma omp atomic
      round_hooks += my_e;
#pragma omp barrier
      if (round_hooks == 0) break; /* every thread reads the same total */
      /* new root of every old root (parent chains are acyclic after the mutual break): pointer
       * doubling until no parent moves — chains can be long (gradient grids: thousands of hops),
       * where a plain walk per root would be quadratic. par only moves to an ancestor, so the
       * racy in-place updates converge to the roots. */
      for (;;) {
#pragma omp single
        moved = 0;
        int my_moved = 0;
#pragma omp for schedule(static)
        for (uint64_t x = 0; x < n; ++x) {
          if (comp[x] != (uint32_t)x) continue;
          const uint32_t p = par[x], pp = par[p];
          if (pp != p) {
            par[x] = pp;
            my_moved = 1;
          }
        }
        if (my_moved) {
#pragma omp atomic write
          moved = 1;
        }
#pragma omp barrier
        int any;
#pragma omp atomic read
        any = moved;
#pragma omp barrier
        if (!any) break;
      }
#pragma omp for schedule(static)
      for (uint64_t x = 0; x < n; ++x) {
        if (comp[x] != (uint32_t)x) continue;
        nr[x] = par[x];
        best[x] = UINT64_MAX;
      }
      /* every vertex's label is an old root: one lookup resolves it */
#pragma omp for schedule(static)
      for (uint64_t x = 0; x < n; ++x) comp[x] = nr[comp[x]];
    }
  }
  free(comp); free(par); free(nr); free(best); free(live);
  *total_weight = tw;
  *num_edges = ne;
  if (rounds_out) *rounds_out = rounds;
  return ORC_OK;
}
