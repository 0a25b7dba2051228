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
check_mst.py:6-7), sorted ascending by (min, max); eid = position. Weights are non-negative
integers < 2^32 (the reference draws random.randint(1, 10): create_graph_files.py:38,
ghs_implementation.py:718).

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
    """n vertices + canonical (u < v, ascending, unique) uint32 arrays u, v, w."""

    __slots__ = ("n", "u", "v", "w")

    def __init__(self, n, u, v, w):
        self.n = int(n)
        self.u = np.ascontiguousarray(u, dtype=np.uint32)
        self.v = np.ascontiguousarray(v, dtype=np.uint32)
        self.w = np.ascontiguousarray(w, dtype=np.uint32)
        if not (len(self.u) == len(self.v) == len(self.w)):
            raise ValueError("u, v, w must have equal length")

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
        key = (u << 32) | v
        if not np.all(key[1:] > key[:-1]):
            raise ValueError("canonical edge list must be strictly ascending in (u, v)")
        return self

    def edge_triples(self, mask=None):
        idx = np.arange(self.m) if mask is None else np.flatnonzero(mask)
        return [(int(self.u[i]), int(self.v[i]), int(self.w[i])) for i in idx]


def _as_weight_array(ws):
    w = np.asarray(ws)
    if w.size == 0:
        return np.zeros(0, np.uint32)
    if w.dtype.kind == "f":
        if not np.all(np.isfinite(w)) or not np.all(w == np.floor(w)):
            raise ValueError("weights must be integers (the reference uses random.randint weights)")
        w = w.astype(np.int64)
    elif w.dtype.kind not in "iu":
        w = np.array([int(x) for x in ws], dtype=np.int64)
    w = w.astype(np.int64)
    if np.any(w < 0) or np.any(w >= (1 << 32)):
        raise ValueError("weights must lie in [0, 2^32)")
    return w.astype(np.uint32)


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
            w = _as_weight_array([c for _, _, c in edges])
        else:
            u = v = np.zeros(0, np.int64)
            w = np.zeros(0, np.uint32)
    else:
        u = np.asarray(u, dtype=np.int64)
        v = np.asarray(v, dtype=np.int64)
        w = _as_weight_array(w)
    if len(u):
        if u.min() < 0 or v.min() < 0 or u.max() >= n or v.max() >= n:
            raise ValueError(f"vertex id out of range [0, {n})")
    keep = u != v
    a = np.minimum(u, v)[keep]
    b = np.maximum(u, v)[keep]
    w = w[keep]
    key = (a << 32) | b
    # stable sort by key; for repeated keys keep the LAST occurrence (nx add_edge overwrite)
    order = np.argsort(key, kind="stable")
    ks = key[order]
    last = np.ones(len(ks), dtype=bool)
    if len(ks) > 1:
        last[:-1] = ks[1:] != ks[:-1]
    sel = order[last]
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
    edges = sorted([int(a), int(b), int(c)] for a, b, c in mst_triples)
    return {"mst_edges": edges, "total_weight": int(sum(e[2] for e in edges)),
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
