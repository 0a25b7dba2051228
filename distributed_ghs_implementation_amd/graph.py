"""Graph inputs/outputs in the reference's formats, and the canonical edge list.

Reference formats (create_graph_files.py:43-89, ghs_implementation_mpi.py:74-92, :811-820):
  <dir>/node_<id>.json       {"node_id": id, "neighbors": {"<nbr>": w, ...}, "num_neighbors": k}
  <dir>/graph_metadata.json  {"num_nodes": n, "num_edges": m, "edges": [[u, v, w], ...]}
  <dir>/mst_result_mpi.json  {"mst_edges": [[u, v, w], ...], "total_weight": W,
                              "num_edges": k, "algorithm": "GHS (MPI)"}
Our result file is ghs_mst.json with the mst_result_mpi.json schema (README.md:8,74 promise
ghs_mst.json), "algorithm": "Boruvka (HIP)", edges sorted ascending.

Canonical edge list (the contract of include/ghs_mst.h): self-loops dropped, each unordered
pair once as (min, max) with the LAST weight given for it (nx.Graph.add_edge overwrites, which
is how every reference entry point builds its graph: ghs_implementation.py:425-426,
check_mst.py:6-7), sorted ascending by (min, max); eid = position. The engine computes on uint32
weights: integers in [0, 2^32) (the reference draws random.randint(1, 10):
create_graph_files.py:38, ghs_implementation.py:718) go through unchanged; any other numeric
weights (negative, float, > 2^32 — nx.Graph, and so the reference's GHSAlgorithm at
ghs_implementation.py:417-440, accepts any comparable weight) are replaced by their dense rank
among the distinct values, an order-preserving map that keeps ties tied, so the MSF edge set is
the same; the original values are kept (`CanonicalGraph.weights`) for the reported weights.

Binary format for large graphs (.mstbin, little endian): 8-byte magic b"MSTBIN1\\0", uint32 n,
uint32 flags (bit 0 = canonical), uint64 m, then u[m], v[m], w[m] as uint32 arrays.
"""
import json
import os
import re

import numpy as np

MAGIC = b"MSTBIN1\0"
_NODE_RE = re.compile(r"^node_(\d+)\.json$")


class CanonicalGraph:
    """n vertices + canonical (u < v, ascending, unique) uint32 arrays u, v, w. `weights`: the
    caller's original weights in canonical order when w holds their ranks (else None)."""

    __slots__ = ("n", "u", "v", "w", "weights")

    def __init__(self, n, u, v, w, weights=None):
        self.n = int(n)
        self.u = np.ascontiguousarray(u, dtype=np.uint32)
        self.v = np.ascontiguousarray(v, dtype=np.uint32)
        self.w = np.ascontiguousarray(w, dtype=np.uint32)
        self.weights = None if weights is None else np.asarray(weights)
        if not (len(self.u) == len(self.v) == len(self.w)):
            raise ValueError("u, v, w must have equal length")
        if self.weights is not None and len(self.weights) != len(self.w):
            raise ValueError("weights must align with the canonical edges")

    @property
    def m(self):
        return len(self.u)

    def check(self):
        """Raise ValueError unless u < v < n and (u, v) strictly ascending."""
        u = self.u.astype(np.int64)
        v = self.v.astype(np.int64)
        if self.m == 0:
            return self
        if not np.all(u < v) or int(v.max()) >= self.n:
            raise ValueError("canonical edge list needs u < v < n")
        key = (self.u.astype(np.uint64) << np.uint64(32)) | self.v.astype(np.uint64)
        if not np.all(key[1:] > key[:-1]):
            raise ValueError("canonical edge list must be strictly ascending in (u, v)")
        return self

    def weight_of(self, i):
        """The caller's weight of canonical edge i (a Python int or float)."""
        if self.weights is None:
            return int(self.w[i])
        x = self.weights[i]
        return x.item() if hasattr(x, "item") else x

    def total_weight(self, mask):
        """Sum of the caller's weights over a mask of canonical edges."""
        if self.weights is None:
            return int(self.w[np.asarray(mask, bool)].astype(np.uint64).sum())
        sel = self.weights[np.asarray(mask, bool)]
        return sum(x.item() if hasattr(x, "item") else x for x in sel)

    def edge_triples(self, mask=None):
        idx = np.arange(self.m) if mask is None else np.flatnonzero(mask)
        return [(int(self.u[i]), int(self.v[i]), self.weight_of(i)) for i in idx]


def _as_weight_array(ws):
    """Weights -> (uint32 engine weights, the original values or None). Integers in [0, 2^32)
    pass unchanged; other numeric weights are replaced by their dense rank (order-preserving,
    ties stay tied)."""
    w = np.asarray(ws)
    if w.size == 0:
        return np.zeros(0, np.uint32), None
    if w.dtype.kind == "O":  # Python ints beyond int64, mixed int / float
        try:
            w = np.asarray(ws, dtype=np.float64) if any(isinstance(x, float) for x in ws) \
                else np.asarray([int(x) for x in ws], dtype=object)
        except (TypeError, ValueError) as exc:
            raise ValueError("weights must be numbers") from exc
    if w.dtype.kind == "b":
        w = w.astype(np.int64)
    if w.dtype.kind in "iu" and int(w.min()) >= 0 and int(w.max()) < (1 << 32):
        return w.astype(np.uint32), None
    if w.dtype.kind == "f" and np.any(np.isnan(w)):
        raise ValueError("weights must not be NaN")
    if w.dtype.kind not in "iufO":
        raise ValueError("weights must be numbers")
    if w.dtype.kind == "O":
        uniq = sorted(set(w.tolist()))
        rank = {x: i for i, x in enumerate(uniq)}
        return np.array([rank[x] for x in w.tolist()], dtype=np.uint32), w
    uniq = np.unique(w)
    return np.searchsorted(uniq, w).astype(np.uint32), w


def canonicalize(num_nodes, edges=None, u=None, v=None, w=None):
    """Raw edges -> CanonicalGraph with nx.Graph semantics (see module docstring).

    Pass either `edges` = iterable of (u, v, w) or arrays u, v, w.
    """
    n = int(num_nodes)
    if n < 0 or n >= (1 << 32):
        raise ValueError("num_nodes must be in [0, 2^32)")
    if edges is not None:
        edges = list(edges)
        if edges:
            arr = np.array([(int(a), int(b)) for a, b, _ in edges], dtype=np.int64).reshape(-1, 2)
            u, v = arr[:, 0], arr[:, 1]
            w, orig = _as_weight_array([c for _, _, c in edges])
        else:
            u = v = np.zeros(0, np.int64)
            w, orig = np.zeros(0, np.uint32), None
    else:
        u = np.asarray(u, dtype=np.int64)
        v = np.asarray(v, dtype=np.int64)
        w, orig = _as_weight_array(w)
    if len(u):
        if u.min() < 0 or v.min() < 0 or u.max() >= n or v.max() >= n:
            raise ValueError(f"vertex id out of range [0, {n})")
    keep = u != v
    a = np.minimum(u, v)[keep]
    b = np.maximum(u, v)[keep]
    w = w[keep]
    if orig is not None:
        orig = orig[keep]
    key = (a.astype(np.uint64) << np.uint64(32)) | b.astype(np.uint64)
    # stable sort by key; for repeated keys keep the LAST occurrence (nx add_edge overwrite)
    order = np.argsort(key, kind="stable")
    ks = key[order]
    last = np.ones(len(ks), dtype=bool)
    if len(ks) > 1:
        last[:-1] = ks[1:] != ks[:-1]
    sel = order[last]
    if orig is not None:
        # ranks were taken over every given value; the canonical list keeps the same order
        return CanonicalGraph(n, a[sel], b[sel], w[sel], weights=orig[sel])
    return CanonicalGraph(n, a[sel], b[sel], w[sel])


# ---------------------------------------------------------------- reference directory formats
def read_graph_dir(graph_dir):
    """Read a create_graph_files.py directory -> CanonicalGraph.

    Uses graph_metadata.json when present (the complete edge list, create_graph_files.py:79-87);
    otherwise the node_<id>.json neighbour files the MPI ranks load (ghs_implementation_mpi.py:
    74-92). Missing directory / files raise FileNotFoundError (the reference only printed).
    """
    meta_path = os.path.join(graph_dir, "graph_metadata.json")
    if os.path.exists(meta_path):
        with open(meta_path) as f:
            meta = json.load(f)
        n = int(meta["num_nodes"])
        return canonicalize(n, edges=[tuple(e) for e in meta["edges"]])
    return read_node_files(graph_dir)


def read_node_files(graph_dir):
    """node_<id>.json files -> CanonicalGraph (each edge appears in both endpoint files)."""
    ids = []
    for name in os.listdir(graph_dir):
        mt = _NODE_RE.match(name)
        if mt:
            ids.append(int(mt.group(1)))
    if not ids:
        raise FileNotFoundError(f"no graph_metadata.json or node_<id>.json files in {graph_dir}")
    n = max(ids) + 1
    edges = []
    for i in sorted(ids):
        with open(os.path.join(graph_dir, f"node_{i}.json")) as f:
            node = json.load(f)
        nid = int(node.get("node_id", i))
        for nbr, wt in node["neighbors"].items():
            edges.append((nid, int(nbr), wt))
    g = canonicalize(n, edges=edges)
    return g


def write_graph_dir(graph, graph_dir):
    """Write the reference's per-node files + metadata for a CanonicalGraph
    (same schema as create_graph_files.py:43-89; no PNG)."""
    os.makedirs(graph_dir, exist_ok=True)
    nbrs = [dict() for _ in range(graph.n)]
    for a, b, c in graph.edge_triples():
        nbrs[a][b] = c
        nbrs[b][a] = c
    for i in range(graph.n):
        with open(os.path.join(graph_dir, f"node_{i}.json"), "w") as f:
            json.dump({"node_id": i, "neighbors": {str(k): v for k, v in nbrs[i].items()},
                       "num_neighbors": len(nbrs[i])}, f, indent=2)
    with open(os.path.join(graph_dir, "graph_metadata.json"), "w") as f:
        json.dump({"num_nodes": graph.n, "num_edges": graph.m,
                   "edges": [list(e) for e in graph.edge_triples()]}, f, indent=2)


def mst_result_dict(mst_triples, algorithm="Boruvka (HIP)"):
    """The mst_result_mpi.json schema (ghs_implementation_mpi.py:811-816), edges sorted."""
    edges = sorted([int(a), int(b), c if isinstance(c, (int, float)) else c.item()] for a, b, c in mst_triples)
    return {"mst_edges": edges, "total_weight": sum(e[2] for e in edges),
            "num_edges": len(edges), "algorithm": algorithm}


def write_result(path, mst_triples, algorithm="Boruvka (HIP)"):
    res = mst_result_dict(mst_triples, algorithm)
    with open(path, "w") as f:
        json.dump(res, f, indent=2)
    return res


# ---------------------------------------------------------------- binary format
def write_mstbin(path, graph):
    with open(path, "wb") as f:
        f.write(MAGIC)
        f.write(np.array([graph.n, 1], dtype="<u4").tobytes())
        f.write(np.array([graph.m], dtype="<u8").tobytes())
        for arr in (graph.u, graph.v, graph.w):
            f.write(np.ascontiguousarray(arr, dtype="<u4").tobytes())


def read_mstbin(path, mmap=True):
    with open(path, "rb") as f:
        if f.read(8) != MAGIC:
            raise ValueError(f"{path}: not an .mstbin file")
        n, flags = np.frombuffer(f.read(8), dtype="<u4")
        (m,) = np.frombuffer(f.read(8), dtype="<u8")
    m = int(m)
    off = 24
    if mmap:
        arr = np.memmap(path, dtype="<u4", mode="r", offset=off, shape=(3 * m,))
    else:
        arr = np.fromfile(path, dtype="<u4", offset=off, count=3 * m)
    g = CanonicalGraph(int(n), arr[:m], arr[m:2 * m], arr[2 * m:3 * m])
    if not (int(flags) & 1):
        g = canonicalize(g.n, u=g.u, v=g.v, w=g.w)
    return g
