"""ORACLE — test infrastructure only. CPU restatements the GPU path is checked against.

* `kruskal_py`      pure-Python canonical Kruskal (small cases), the definition of the contract.
* `canonicalize_py` pure-Python nx.Graph-style canonicalisation (self-loops dropped, last write
                    wins on duplicate pairs, output sorted by (min, max)).
* `kruskal_c` / `canonicalize_c`  the same in C (oracle/kruskal.c via ctypes), for the large
                    parity cases and the bench's cpu_baseline (kind "port").
* `boruvka_omp_c`   OpenMP Borůvka on all given cores (oracle/boruvka_omp.c): the same canonical
                    MSF (unique keys), the bench's all-cores CPU baseline.
* `rmat_pairs_c` / `rmat_canonical` / `grid_canonical`  the synthetic generators restated
                    (oracle/generators.c, numpy): the GPU generators are checked against them
                    tuple for tuple (SURVEY §8(d) "reproducible by both CPU oracle and GPU generator").

Reference anchors: the MST the reference verifies against is NetworkX Kruskal
(ghs_implementation.py:746, create_graph_files.py:141, check_mst.py:9); the raw-edge semantics
follow nx.Graph.add_edge as used at ghs_implementation.py:425-426 and create_graph_files.py:65-87.
Pinned by tests/golden/*.json (NetworkX canonical MSF + the reference thread GHS outputs).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    """Load oracle/_build/liboracle.so (built by `make -C oracle` / __graft_entry__.build())."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle library missing: {path} (run `make -C oracle`)")
        L = ctypes.CDLL(path)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_kruskal.argtypes = [ctypes.c_uint32, ctypes.c_uint64, u32p, u32p, u32p, u8p, u64p, u64p]
        L.oracle_kruskal.restype = ctypes.c_int
        L.oracle_canonicalize.argtypes = [ctypes.c_uint32, ctypes.c_uint64, u32p, u32p, u32p,
                                          u32p, u32p, u32p, u64p]
        L.oracle_canonicalize.restype = ctypes.c_int
        L.oracle_check_canonical.argtypes = [ctypes.c_uint32, ctypes.c_uint64, u32p, u32p]
        L.oracle_check_canonical.restype = ctypes.c_int
        L.oracle_boruvka_omp.argtypes = [ctypes.c_uint32, ctypes.c_uint64, u32p, u32p, u32p, ctypes.c_int,
                                         u8p, u64p, u64p, u32p]
        L.oracle_boruvka_omp.restype = ctypes.c_int
        L.oracle_rmat_pairs.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, u32p, u32p]
        L.oracle_rmat_pairs.restype = ctypes.c_int
        L.oracle_hash_weights.argtypes = [ctypes.c_uint64, ctypes.c_uint64, u32p]
        L.oracle_hash_weights.restype = None
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def canonicalize_py(n, edges):
    """nx.Graph semantics: drop self-loops, last write wins, sort by (min, max)."""
    last = {}
    for u, v, w in edges:
        u, v, w = int(u), int(v), int(w)
        if not (0 <= u < n and 0 <= v < n):
            raise ValueError("vertex out of range")
        if u == v:
            continue
        last[(min(u, v), max(u, v))] = w
    keys = sorted(last)
    return [(a, b, last[(a, b)]) for a, b in keys]


def canonicalize_py_any(n, edges):
    """canonicalize_py for any comparable weights (kept as given)."""
    last = {}
    for u, v, w in edges:
        u, v = int(u), int(v)
        if not (0 <= u < n and 0 <= v < n):
            raise ValueError("vertex out of range")
        if u == v:
            continue
        last[(min(u, v), max(u, v))] = w
    return [(a, b, last[(a, b)]) for a, b in sorted(last)]


def kruskal_py(n, canon_edges):
    """Canonical Kruskal under key (w, eid) on a canonical edge list -> (in_mst list, weight)."""
    parent = list(range(n))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    order = sorted(range(len(canon_edges)), key=lambda e: (canon_edges[e][2], e))
    in_mst = [0] * len(canon_edges)
    tw = 0
    for e in order:
        a, b, w = canon_edges[e]
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[ra] = rb
            in_mst[e] = 1
            tw += w
    return in_mst, tw


def canonicalize_c(n, u, v, w):
    u = np.ascontiguousarray(u, dtype=np.uint32)
    v = np.ascontiguousarray(v, dtype=np.uint32)
    w = np.ascontiguousarray(w, dtype=np.uint32)
    m = len(u)
    cu = np.empty(max(m, 1), np.uint32)
    cv = np.empty(max(m, 1), np.uint32)
    cw = np.empty(max(m, 1), np.uint32)
    mo = ctypes.c_uint64(0)
    rc = lib().oracle_canonicalize(n, m, _p(u, ctypes.c_uint32), _p(v, ctypes.c_uint32), _p(w, ctypes.c_uint32),
                                   _p(cu, ctypes.c_uint32), _p(cv, ctypes.c_uint32), _p(cw, ctypes.c_uint32),
                                   ctypes.byref(mo))
    if rc != 0:
        raise ValueError(f"oracle_canonicalize failed rc={rc}")
    k = mo.value
    return cu[:k].copy(), cv[:k].copy(), cw[:k].copy()


def kruskal_c(n, u, v, w):
    """C canonical Kruskal on canonical arrays -> (in_mst uint8[m], total_weight, num_edges)."""
    u = np.ascontiguousarray(u, dtype=np.uint32)
    v = np.ascontiguousarray(v, dtype=np.uint32)
    w = np.ascontiguousarray(w, dtype=np.uint32)
    m = len(u)
    in_mst = np.zeros(max(m, 1), np.uint8)
    tw = ctypes.c_uint64(0)
    k = ctypes.c_uint64(0)
    rc = lib().oracle_kruskal(n, m, _p(u, ctypes.c_uint32), _p(v, ctypes.c_uint32), _p(w, ctypes.c_uint32),
                              _p(in_mst, ctypes.c_uint8), ctypes.byref(tw), ctypes.byref(k))
    if rc != 0:
        raise ValueError(f"oracle_kruskal failed rc={rc}")
    return in_mst[:m], tw.value, k.value


def boruvka_omp_c(n, u, v, w, threads=0):
    """OpenMP Borůvka on canonical arrays -> (in_mst uint8[m], total_weight, num_edges, rounds).
    threads <= 0: the OpenMP default (OMP_NUM_THREADS)."""
    u = np.ascontiguousarray(u, dtype=np.uint32)
    v = np.ascontiguousarray(v, dtype=np.uint32)
    w = np.ascontiguousarray(w, dtype=np.uint32)
    m = len(u)
    in_mst = np.zeros(max(m, 1), np.uint8)
    tw = ctypes.c_uint64(0)
    k = ctypes.c_uint64(0)
    r = ctypes.c_uint32(0)
    rc = lib().oracle_boruvka_omp(n, m, _p(u, ctypes.c_uint32), _p(v, ctypes.c_uint32), _p(w, ctypes.c_uint32),
                                  int(threads), _p(in_mst, ctypes.c_uint8), ctypes.byref(tw), ctypes.byref(k),
                                  ctypes.byref(r))
    if rc != 0:
        raise ValueError(f"oracle_boruvka_omp failed rc={rc}")
    return in_mst[:m], tw.value, k.value, r.value


def mix32_np(x):
    """The bijective 32-bit mixer of the weight hash (oracle/generators.c oracle_mix32), numpy."""
    x = np.asarray(x, dtype=np.uint32).copy()
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def rmat_pairs_c(scale, edgefactor, seed):
    """Raw R-MAT tuples (uu[t], vv[t]) after the vertex permutation (oracle/generators.c)."""
    T = edgefactor << scale
    uu = np.empty(max(T, 1), np.uint32)
    vv = np.empty(max(T, 1), np.uint32)
    rc = lib().oracle_rmat_pairs(scale, edgefactor, seed, _p(uu, ctypes.c_uint32), _p(vv, ctypes.c_uint32))
    if rc != 0:
        raise ValueError("oracle_rmat_pairs failed")
    return uu[:T], vv[:T]


def hash_weights(m, wseed):
    w = np.empty(max(m, 1), np.uint32)
    lib().oracle_hash_weights(m, wseed, _p(w, ctypes.c_uint32))
    return w[:m]


def rmat_canonical(scale, edgefactor=16, seed=1, wseed=2):
    """The canonical R-MAT graph: tuples -> self-loops dropped, pairs deduplicated, sorted by
    (min, max) (canonicalize_c) -> w[e] = mix32(e ^ wseed). Returns (n, u, v, w)."""
    n = 1 << scale
    uu, vv = rmat_pairs_c(scale, edgefactor, seed)
    cu, cv, _ = canonicalize_c(n, uu, vv, np.zeros(len(uu), np.uint32))
    return n, cu, cv, hash_weights(len(cu), wseed)


def grid_canonical(k, mode=0, wseed=2):
    """k x k grid, vertex r*k + c, right and down edges in canonical order (for each vertex x: its
    right edge (x, x+1), then its down edge (x, x+k)); w = eid (mode 1, "road-like" gradient) or
    mix32(eid ^ wseed). Returns (n, u, v, w)."""
    n = k * k
    x = np.arange(n, dtype=np.int64)
    r, c = x // k, x % k
    right = np.stack([x, x + 1], 1)[c < k - 1]
    down = np.stack([x, x + k], 1)[r < k - 1]
    e = np.concatenate([right, down])
    order = np.lexsort((e[:, 1], e[:, 0]))
    e = e[order]
    m = len(e)
    eid = np.arange(m, dtype=np.uint32)
    w = eid.copy() if mode else mix32_np(eid ^ np.uint32(wseed & 0xFFFFFFFF))
    return n, e[:, 0].astype(np.uint32), e[:, 1].astype(np.uint32), w
