"""Result verification — the reference's check_mst.py and experiment record, as library code.

check_mst.py:1-20 loads graph_metadata.json, recomputes the MST with NetworkX and prints the
expected edges, total weight, edge count and whether the graph / MST are connected;
ghs_implementation.py:721-776 (run_experiment) compares a run with nx.minimum_spanning_tree and
records {"experiment", "num_nodes", "num_edges", "mst_edges", "mst_weight", "networkx_weight",
"is_correct", "edges_found", "edges_expected"} into ghs_experiments.json.

`verify_forest` checks a result against its graph without any MST solver: every result edge is a
graph edge with the same weight, the result is a forest (components(T) == n - |T|), and it spans
every component of the graph (components(T) == components(G)). Optimality is checked against
NetworkX (the reference's own verifier; third-party, optional) when it is importable and the
graph is small enough for it (`nx_max_edges`); otherwise `weight_matches_networkx` is None.
This module never calls the HIP engine, so it also verifies results produced elsewhere.
"""
import numpy as np

NX_MAX_EDGES = 2_000_000  # NetworkX needs ~0.9 GB per 1M edges


def _components(n, a, b):
    """Number of connected components of the graph (n vertices, edges a[i]-b[i])."""
    if n == 0:
        return 0
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    a = np.asarray(a, dtype=np.int64)
    b = np.asarray(b, dtype=np.int64)
    mat = coo_matrix((np.ones(a.size, dtype=np.int8), (a, b)), shape=(n, n))
    return int(connected_components(mat, directed=False, return_labels=False))


def networkx_msf(graph):
    """(edges [(u, v, w)] sorted, total weight) of nx.minimum_spanning_tree on the graph built as
    the reference's verifiers build it (ghs_implementation.py:746, check_mst.py:3-9), with every
    vertex added first so isolated vertices are allowed. Raises ImportError without NetworkX."""
    import networkx as nx
    G = nx.Graph()
    G.add_nodes_from(range(graph.n))
    gw = graph.w if graph.weights is None else graph.weights
    for a, b, c in zip(graph.u.tolist(), graph.v.tolist(), gw.tolist()):
        G.add_edge(a, b, weight=c)
    T = nx.minimum_spanning_tree(G, weight="weight")
    edges = sorted((min(a, b), max(a, b), d["weight"]) for a, b, d in T.edges(data=True))
    return edges, sum(e[2] for e in edges)


def verify_forest(graph, mst_triples, use_networkx=True, nx_max_edges=NX_MAX_EDGES):
    """Check `mst_triples` [(u, v, w)] against the canonical `graph`. Returns a report dict;
    report["ok"] is True iff every structural check passes and (when it ran) the NetworkX
    weight matches."""
    triples = list(mst_triples)
    t = np.asarray([(a, b) for a, b, _ in triples], dtype=np.int64).reshape(-1, 2)
    tw = [c for _, _, c in triples]  # the caller's weights (ints, or any numbers: graph.weights)
    tu = np.minimum(t[:, 0], t[:, 1])
    tv = np.maximum(t[:, 0], t[:, 1])
    rep = {"num_nodes": graph.n, "num_edges": graph.m, "mst_edges": int(len(t)),
           "mst_weight": sum(tw) if tw else 0}
    # every result edge is a graph edge with the graph's weight (canonical order: searchsorted)
    gkey = (graph.u.astype(np.uint64) << np.uint64(32)) | graph.v.astype(np.uint64)
    tkey = (tu.astype(np.uint64) << np.uint64(32)) | tv.astype(np.uint64)
    pos = np.searchsorted(gkey, tkey)
    found = (pos < graph.m) & (gkey[np.minimum(pos, max(graph.m - 1, 0))] == tkey) if graph.m else np.zeros(len(t), bool)
    rep["edges_in_graph"] = bool(found.all())
    gw = graph.w.astype(np.int64) if graph.weights is None else graph.weights
    rep["weights_match_graph"] = bool(rep["edges_in_graph"] and
                                      all(gw[p] == c for p, c in zip(pos[found].tolist(), np.asarray(tw, dtype=object)[found])))
    rep["duplicate_edges"] = int(len(tkey) - len(np.unique(tkey)))
    cg = _components(graph.n, graph.u, graph.v)
    ct = _components(graph.n, tu, tv)
    rep["graph_components"] = cg
    rep["graph_connected"] = cg == 1
    rep["mst_connected"] = ct == 1
    rep["is_forest"] = ct == graph.n - len(t)
    rep["spans_components"] = ct == cg
    rep["edges_expected"] = graph.n - cg
    ok = (rep["edges_in_graph"] and rep["weights_match_graph"] and rep["duplicate_edges"] == 0
          and rep["is_forest"] and rep["spans_components"])
    rep["networkx_weight"] = None
    rep["weight_matches_networkx"] = None
    rep["edge_set_matches_networkx"] = None
    if use_networkx and graph.m <= nx_max_edges:
        try:
            nx_edges, nx_w = networkx_msf(graph)
        except ImportError:
            nx_edges = None
        if nx_edges is not None:
            rep["networkx_weight"] = nx_w
            rep["weight_matches_networkx"] = nx_w == rep["mst_weight"]
            # informational under weight ties (the MST edge set is then not unique)
            rep["edge_set_matches_networkx"] = [e[:2] for e in nx_edges] == sorted(zip(tu.tolist(), tv.tolist()))
            ok = ok and rep["weight_matches_networkx"]
    rep["ok"] = bool(ok)
    return rep


def experiment_record(experiment, graph, mst_triples, num_input_edges=None, **kw):
    """One ghs_experiments.json entry (ghs_implementation.py:766-776 schema) for a result."""
    rep = verify_forest(graph, mst_triples, **kw)
    edges = sorted([int(a), int(b), c] for a, b, c in mst_triples)
    correct = rep["ok"] if rep["networkx_weight"] is None else bool(rep["ok"] and rep["weight_matches_networkx"])
    return {"experiment": experiment, "num_nodes": graph.n,
            "num_edges": graph.m if num_input_edges is None else int(num_input_edges),
            "mst_edges": edges, "mst_weight": rep["mst_weight"],
            "networkx_weight": rep["networkx_weight"], "is_correct": correct,
            "edges_found": rep["mst_edges"], "edges_expected": rep["edges_expected"]}


def format_report(rep, mst_triples=None, max_edges=50):
    """check_mst.py-style text (check_mst.py:10-20)."""
    lines = []
    if mst_triples is not None and len(mst_triples) <= max_edges:
        lines.append("MST edges:")
        for a, b, c in sorted(mst_triples):
            lines.append(f"  ({a},{b}): {c}")
        lines.append("")
    lines.append(f"Total weight: {rep['mst_weight']}")
    lines.append(f"Number of edges: {rep['mst_edges']} (expected {rep['edges_expected']})")
    if rep["networkx_weight"] is not None:
        lines.append(f"NetworkX MST weight: {rep['networkx_weight']}")
    else:
        lines.append("NetworkX MST weight: not checked (networkx missing or graph too large)")
    lines.append(f"\nOriginal graph connected: {rep['graph_connected']}")
    lines.append(f"MST connected: {rep['mst_connected']}")
    lines.append(f"Forest: {rep['is_forest']}  spans every component: {rep['spans_components']}  "
                 f"edges in graph with its weights: {rep['edges_in_graph'] and rep['weights_match_graph']}")
    lines.append(f"Status: {'CORRECT' if rep['ok'] else 'INCORRECT'}")
    return "\n".join(lines)
