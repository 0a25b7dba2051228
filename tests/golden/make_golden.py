"""Generate the golden fixtures under tests/golden/ (run in the dev container only).

This script is the ONLY place that imports the reference (read-only at /root/reference) — it is
never run by the test suite, smoke() or bench.py, and nothing it imports travels to the GPU box.
What it commits is data: input graphs exactly as the reference's own generators produce them,
the MST NetworkX computes for them, and the edge set the reference's thread GHS returns where it
was run.

Sources of each fixture (reference file:line):
  readme6      README.md:45-49 sample graph; expected W=20 at README.md:60
  simple3      create_simple_test.py:11-50 (3 nodes, expected W=3 at :50)
  cgf_n6       create_graph_files.create_random_graph(6, 0.5, 42) (create_graph_files.py:13-40,
               defaults at :151-175); README_MPI.md:228-235 shows W=11 for it
  thread_cfgN  ghs_implementation.create_random_graph(n, p, seed) for the 6 configs at
               ghs_implementation.py:787-794
  cgf_n1000_p001 / cgf_n1000_p05  create_graph_files.create_random_graph(1000, p, 42)
  ties_*       tie-stress multigraphs (self-loops, duplicates, isolated vertices, equal weights),
               our own generator; pinned by NetworkX only (the reference cannot run them:
               ghs_implementation.py:433-436 raises on isolated vertices)

The expected MSF is NetworkX 3.4.2 `minimum_spanning_tree` (the reference's own verifier:
ghs_implementation.py:746, create_graph_files.py:141, check_mst.py:9) on a graph built
CANONICALLY: add_nodes_from(range(n)), then the de-duplicated edges added in ascending
(min(u,v), max(u,v)) order, duplicates resolved last-write-wins like nx.Graph.add_edge.
Under that construction NetworkX's stable-sort Kruskal equals Kruskal under the strict key
(w, min(u,v), max(u,v)) — asserted below for every fixture.

Usage (from the repo root, dev container):  python tests/golden/make_golden.py [--with-ghs]
"""
import argparse
import contextlib
import gzip
import io
import json
import os
import random
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def canonical_nx_mst(n, edges):
    import networkx as nx
    last = {}
    for u, v, w in edges:
        if u == v:
            continue
        last[(min(u, v), max(u, v))] = int(w)
    G = nx.Graph()
    G.add_nodes_from(range(n))
    for (a, b) in sorted(last):
        G.add_edge(a, b, weight=last[(a, b)])
    T = nx.minimum_spanning_tree(G, weight="weight")
    mst = sorted((min(a, b), max(a, b), last[(min(a, b), max(a, b))]) for a, b in T.edges())
    # cross-check: pure Kruskal under the strict key (w, min, max)
    parent = list(range(n))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    kr = []
    for (a, b), w in sorted(last.items(), key=lambda t: (t[1], t[0][0], t[0][1])):
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[ra] = rb
            kr.append((a, b, w))
    assert sorted(kr) == mst, "NetworkX canonical MST != strict-key Kruskal"
    return [list(e) for e in mst], sum(e[2] for e in mst)


def run_ref_thread_ghs(n, edges, timeout=15):
    """Run ghs_implementation.GHSAlgorithm (the reference thread path) and return its edge set."""
    sys.path.insert(0, REF)
    import ghs_implementation as gi
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        ghs = gi.GHSAlgorithm(n, [tuple(e) for e in edges])
        res = ghs.run(timeout=timeout)
    g = ghs.graph
    return sorted([min(u, v), max(u, v), g[u][v]["weight"]] for u, v in res)


def dump(name, n, edges, source, ghs_edges=None, compress=False):
    mst, W = canonical_nx_mst(n, edges)
    fx = {
        "name": name,
        "source": source,
        "num_nodes": n,
        "num_edges": len(edges),
        "edges": [list(map(int, e)) for e in edges],
        "expected_mst_edges": mst,
        "expected_total_weight": W,
    }
    if ghs_edges is not None:
        fx["reference_thread_ghs_edges"] = ghs_edges
        fx["reference_thread_ghs_weight"] = sum(e[2] for e in ghs_edges)
        fx["reference_thread_ghs_matches"] = ghs_edges == mst
    path = os.path.join(HERE, name + (".json.gz" if compress else ".json"))
    data = json.dumps(fx, separators=(",", ":")).encode()
    if compress:
        with gzip.GzipFile(path, "wb", mtime=0) as f:
            f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data)
    print(f"{name}: n={n} m={len(edges)} W={W}" + (
        f" ghs_match={fx['reference_thread_ghs_matches']}" if ghs_edges is not None else ""))


def tie_stress(seed, n, m, wmax, p_self=0.05, p_dup=0.1):
    rng = random.Random(seed)
    edges = []
    for _ in range(m):
        u = rng.randrange(n)
        v = u if rng.random() < p_self else rng.randrange(n)
        edges.append((u, v, rng.randint(1, wmax)))
        if rng.random() < p_dup and edges:
            a, b, _ = edges[rng.randrange(len(edges))]
            edges.append((b, a, rng.randint(1, wmax)))
    return edges


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--with-ghs", action="store_true", help="also run the reference thread GHS")
    args = ap.parse_args()
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    scratch = tempfile.mkdtemp(prefix="ghs_golden_")
    os.chdir(scratch)  # the reference writes PNG/JSON into cwd
    sys.path.insert(0, REF)
    import create_graph_files as cgf
    import ghs_implementation as gi

    readme = [(0, 1, 1), (0, 2, 4), (1, 2, 2), (1, 3, 5), (2, 3, 3), (2, 4, 7), (3, 4, 6),
              (3, 5, 8), (4, 5, 9)]
    dump("readme6", 6, readme, "README.md:45-49",
         run_ref_thread_ghs(6, readme) if args.with_ghs else None)
    dump("simple3", 3, [(0, 1, 1), (0, 2, 2)], "create_simple_test.py:11-50",
         run_ref_thread_ghs(3, [(0, 1, 1), (0, 2, 2)]) if args.with_ghs else None)

    G = cgf.create_random_graph(6, 0.5, 42)
    e6 = [(u, v, G[u][v]["weight"]) for u, v in G.edges()]
    dump("cgf_n6", 6, e6, "create_graph_files.create_random_graph(6,0.5,42)",
         run_ref_thread_ghs(6, e6) if args.with_ghs else None)
    # the reference's file format for this graph, written by the reference's own writer
    # (create_graph_files.py:43-89; its PNG is not kept)
    gdir = os.path.join(HERE, "graph_data_n6")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        cgf.visualize_graph = lambda graph, output_dir: None  # skip the matplotlib PNG
        cgf.create_node_files(G, gdir)

    cfgs = [(5, 0.5, 42), (6, 0.4, 100), (7, 0.6, 200), (6, 0.7, 300), (10, 0.8, 400), (20, 0.3, 500)]
    for i, (n, p, s) in enumerate(cfgs, 1):
        nn, edges = gi.create_random_graph(num_nodes=n, edge_probability=p, seed=s)
        dump(f"thread_cfg{i}", nn, edges, f"ghs_implementation.create_random_graph({n},{p},{s}) "
             f"(ghs_implementation.py:787-794 config {i})",
             run_ref_thread_ghs(nn, edges) if args.with_ghs else None)

    for p, tag in [(0.01, "p001"), (0.5, "p05")]:
        G = cgf.create_random_graph(1000, p, 42)
        e = [(u, v, G[u][v]["weight"]) for u, v in G.edges()]
        dump(f"cgf_n1000_{tag}", 1000, e, f"create_graph_files.create_random_graph(1000,{p},42)",
             None, compress=(tag == "p05"))

    for i, (n, m, wmax) in enumerate([(8, 30, 2), (50, 200, 1), (200, 600, 3), (300, 400, 5),
                                      (1000, 5000, 10), (64, 2000, 1)]):
        dump(f"ties_{i}", n, tie_stress(1000 + i, n, m, wmax), f"tie-stress seed {1000 + i}")
    dump("empty", 4, [], "edge case: 4 isolated vertices")
    dump("selfloops", 3, [(0, 0, 1), (1, 1, 2), (0, 2, 5)], "edge case: self-loops dropped")


if __name__ == "__main__":
    main()
