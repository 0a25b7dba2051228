"""Host front-end of the MST engine: the reference's call surfaces over the HIP C-ABI.

`GHSAlgorithm` mirrors ghs_implementation.py:416-552 (constructor (num_nodes, edges), run()
returning the MST edges as (u, v) with u < v, `.graph[u][v]["weight"]` lookups used by the
reference's harness at :741-743/:770). `minimum_spanning_forest` is the array-level call.
Both run the gfx950 kernels of libghs_mst.so; there is no CPU path.

Deliberate differences from the reference (all documented in DESIGN.md):
  * the result is exact and deterministic: canonical Kruskal order (w, min(u,v), max(u,v)),
    identical to NetworkX's MST on a canonically built graph; the reference's GHS is not
    (SURVEY.md §8c);
  * isolated vertices / disconnected inputs give a spanning forest instead of NetworkXError
    (ghs_implementation.py:433-436);
  * `timeout` is accepted for signature compatibility; the engine terminates by construction
    (at most ceil(log2 n) + 1 rounds; a hang guard raises GHS_E_ROUNDCAP);
  * weights: any numbers, as nx.Graph accepts (ghs_implementation.py:417-440). Integers in
    [0, 2^32) go to the engine as they are; others (negative, float, larger) as their dense rank
    (order-preserving, ties kept: the same MSF), and results report the caller's values.
"""
import ctypes
import time

import numpy as np

from . import _native
from .graph import CanonicalGraph, canonicalize, mst_result_dict


class MSTResult:
    """Spanning forest of a CanonicalGraph: in_mst mask over canonical edge ids + totals."""

    def __init__(self, graph, in_mst, total_weight, rounds, stats, ms_total):
        self.graph = graph
        self.in_mst = in_mst.astype(bool)
        # the engine sums uint32 weights; for rank-mapped weights (graph.weights) the caller's
        # own values are summed over the same edges
        self.total_weight = int(total_weight) if graph.weights is None else graph.total_weight(self.in_mst)
        self.rounds = int(rounds)
        self.stats = stats
        self.ms_total = float(ms_total)

    @property
    def num_edges(self):
        return int(self.in_mst.sum())

    def edges(self):
        """MST edges as sorted (u, v) tuples with u < v (GHSAlgorithm.run's return value)."""
        return [(a, b) for a, b, _ in self.triples()]

    def triples(self):
        return self.graph.edge_triples(self.in_mst)

    def to_dict(self, algorithm="Boruvka (HIP)"):
        return mst_result_dict(self.triples(), algorithm)


def minimum_spanning_forest(graph, num_gpus=1, devices=None, config=None):
    """Run the HIP engine on a CanonicalGraph (host arrays) -> MSTResult. num_gpus > 1 (or an
    explicit device list): one process drives that many GPUs of this node as an RCCL clique
    (ghs_mst_multi: the MPI path's multi-rank solve as one call; `config`: its ghs_config_t)."""
    if not isinstance(graph, CanonicalGraph):
        raise TypeError("expected a CanonicalGraph (use graph.canonicalize)")
    L = _native.load()
    _native.require_gpu()
    m = graph.m
    in_mst = np.zeros(max(m, 1), dtype=np.uint8)
    res = _native.Result()
    stats = (_native.RoundStats * _native.GHS_MAX_ROUND_STATS)()
    u, v, w = graph.u, graph.v, graph.w
    if num_gpus > 1 or devices is not None:
        devs = list(range(num_gpus)) if devices is None else [int(d) for d in devices]
        arr = (ctypes.c_int * len(devs))(*devs)
        cfg = ctypes.byref(config) if config is not None else None
        _native.check(L.ghs_mst_multi(graph.n, m, u.ctypes.data, v.ctypes.data, w.ctypes.data, len(devs), arr,
                                      cfg, in_mst.ctypes.data, ctypes.byref(res), stats))
    else:
        _native.check(L.ghs_mst_host(graph.n, m, u.ctypes.data, v.ctypes.data, w.ctypes.data, in_mst.ctypes.data,
                                     ctypes.byref(res), stats))
    st = [stats[i].as_dict() for i in range(res.num_stats)]
    out = MSTResult(graph, in_mst[:m], res.total_weight, res.rounds, st, res.ms_total)
    if out.num_edges != res.num_mst_edges:
        raise _native.GHSError(_native.GHS_E_STATE, "in_mst count disagrees with the device edge counter")
    return out


class _WeightView:
    """Minimal `graph[u][v]["weight"]` view (the reference harness reads weights this way)."""

    def __init__(self, graph):
        self._adj = {}
        for a, b, c in graph.edge_triples():
            self._adj.setdefault(a, {})[b] = {"weight": c}
            self._adj.setdefault(b, {})[a] = {"weight": c}

    def __getitem__(self, u):
        return self._adj[u]

    def __contains__(self, u):
        return u in self._adj


class GHSAlgorithm:
    """Drop-in for ghs_implementation.GHSAlgorithm (ghs_implementation.py:416-490).

    GHSAlgorithm(num_nodes, edges) with edges = [(u, v, w), ...]; run() -> [(u, v), ...].
    """

    def __init__(self, num_nodes, edges):
        self.num_nodes = int(num_nodes)
        self.edges = list(edges)
        self.canonical = canonicalize(self.num_nodes, edges=self.edges)
        self.graph = _WeightView(self.canonical)
        self.result = None

    def run(self, timeout=10):
        """Compute the MST; returns sorted (u, v) pairs with u < v (the reference returned the
        same pairs in set order, ghs_implementation.py:481-490)."""
        del timeout  # terminates by construction (see module docstring)
        t0 = time.perf_counter()
        self.result = minimum_spanning_forest(self.canonical)
        self.elapsed = time.perf_counter() - t0
        return self.result.edges()

    @property
    def mst_weight(self):
        return None if self.result is None else self.result.total_weight

    def mst_triples(self):
        return [] if self.result is None else self.result.triples()
