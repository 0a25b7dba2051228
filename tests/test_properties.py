"""Property-based tie-stress tests (hypothesis; SURVEY.md §4 "tie-stress property tests").

CPU: on arbitrary raw multigraphs (duplicates, self-loops, isolated vertices, tiny weight
alphabets so ties are everywhere) the oracle's pieces agree with each other and with their
definitions: canonicalisation (C vs Python, nx.Graph last-write-wins), canonical Kruskal (C vs
Python), the OpenMP Borůvka CPU baseline vs Kruskal, the independent torch Borůvka checker vs
Kruskal, the numpy step restatement driven by the product's run_rounds (one rank), and the
product's own canonicalisation / rank-mapped weights. The MSF invariants are checked directly
too: forest, spans every component, minimal under the strict key (every non-tree edge is the
heaviest key on the tree path it closes — the cycle property).

GPU (marked gpu): the same generated graphs through GHSAlgorithm / the device API are bit-exact
with the oracle.
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from distributed_ghs_implementation_amd import graph as G
from oracle import oracle

SETTINGS = dict(deadline=None, suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])


@st.composite
def raw_graphs(draw, max_n=40, max_m=160, weights=st.integers(0, 3)):
    n = draw(st.integers(1, max_n))
    m = draw(st.integers(0, max_m))
    edges = draw(st.lists(st.tuples(st.integers(0, n - 1), st.integers(0, n - 1), weights), min_size=m, max_size=m))
    return n, edges


def _cycle_property_holds(n, canon, in_mst):
    """Every non-tree edge (a, b) has the largest strict key (w, eid) on the cycle it closes."""
    adj = [[] for _ in range(n)]
    for e, (a, b, w) in enumerate(canon):
        if in_mst[e]:
            adj[a].append((b, (w, e)))
            adj[b].append((a, (w, e)))
    for e, (a, b, w) in enumerate(canon):
        if in_mst[e]:
            continue
        # max key on the tree path a -> b (iterative DFS); None if b unreachable (then e would
        # join two components: a minimum spanning forest never leaves such an edge out)
        stack, seen, best = [(a, None)], {a}, {a: None}
        while stack:
            x, mx = stack.pop()
            if x == b:
                break
            for y, k in adj[x]:
                if y not in seen:
                    seen.add(y)
                    nk = k if mx is None or k > mx else mx
                    best[y] = nk
                    stack.append((y, nk))
        if b not in best or best[b] is None or best[b] > (w, e):
            return False
    return True


@settings(max_examples=150, **SETTINGS)
@given(raw_graphs())
def test_oracle_pieces_agree_on_tie_stress(g):
    n, edges = g
    canon = oracle.canonicalize_py(n, edges)
    e = np.array(edges, dtype=np.int64).reshape(-1, 3)
    cu, cv, cw = oracle.canonicalize_c(n, e[:, 0], e[:, 1], e[:, 2])
    assert [(int(a), int(b), int(c)) for a, b, c in zip(cu, cv, cw)] == canon
    pg = G.canonicalize(n, edges=edges)
    assert pg.edge_triples() == canon
    in_py, w_py = oracle.kruskal_py(n, canon)
    in_c, w_c, k_c = oracle.kruskal_c(n, cu, cv, cw)
    assert list(in_c) == in_py and w_c == w_py and k_c == sum(in_py)
    in_omp, w_omp, k_omp, _ = oracle.boruvka_omp_c(n, cu, cv, cw, threads=2)
    assert np.array_equal(in_omp, in_c) and (w_omp, k_omp) == (w_c, k_c)
    # forest spanning every component, minimal under the strict key
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    def comps(us, vs):
        mat = coo_matrix((np.ones(len(us)), (np.asarray(us), np.asarray(vs))), shape=(n, n))
        return connected_components(mat, directed=False, return_labels=False)
    t = [i for i, f in enumerate(in_py) if f]
    assert comps([canon[i][0] for i in t], [canon[i][1] for i in t]) == n - len(t)  # a forest
    assert comps([a for a, _, _ in canon], [b for _, b, _ in canon]) == n - len(t)  # spanning
    assert _cycle_property_holds(n, canon, in_py)


@settings(max_examples=60, **SETTINGS)
@given(raw_graphs(max_n=30, max_m=120))
def test_torch_checker_and_step_restatement_agree(g):
    import torch

    from distributed_ghs_implementation_amd.distributed import run_rounds
    from oracle.boruvka_steps import CpuStepper
    from torch_boruvka import msf_boruvka
    n, edges = g
    canon = oracle.canonicalize_py(n, edges)
    in_py, w_py = oracle.kruskal_py(n, canon)
    u = np.array([a for a, _, _ in canon], np.int64)
    v = np.array([b for _, b, _ in canon], np.int64)
    w = np.array([c for _, _, c in canon], np.int64)
    got = msf_boruvka(n, torch.from_numpy(u), torch.from_numpy(v), torch.from_numpy(w))
    assert got.numpy().astype(int).tolist() == in_py
    st_ = CpuStepper(n, u, v, w, 0, len(u), (0, 2, 1 << 32))  # two weight levels
    run_rounds(st_, lambda t: None, allreduce_max=lambda t: None)
    assert st_.in_mst.tolist() == in_py and st_.finish()[0] == w_py


@settings(max_examples=80, **SETTINGS)
@given(raw_graphs(max_n=25, max_m=100, weights=st.one_of(st.integers(-5, 5), st.sampled_from([0.5, -2.25, 1e12, 3.0]))))
def test_rank_mapped_weights_keep_the_msf(g):
    n, edges = g
    pg = G.canonicalize(n, edges=edges)
    canon = oracle.canonicalize_py_any(n, edges)
    assert pg.edge_triples() == canon
    ref_in, ref_w = oracle.kruskal_py(n, canon)
    got_in, _, _ = oracle.kruskal_c(n, pg.u, pg.v, pg.w)
    assert list(got_in) == ref_in
    assert pg.total_weight(got_in.astype(bool)) == pytest.approx(ref_w, rel=1e-12, abs=1e-9)


@pytest.mark.gpu
@settings(max_examples=40, **SETTINGS)
@given(raw_graphs(max_n=60, max_m=300))
def test_gpu_engine_on_tie_stress(g):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_ghs_implementation_amd import GHSAlgorithm
    n, edges = g
    canon = oracle.canonicalize_py(n, edges)
    in_py, w_py = oracle.kruskal_py(n, canon)
    ghs = GHSAlgorithm(n, edges)
    assert ghs.run() == [(a, b) for (a, b, _), f in zip(canon, in_py) if f]
    assert ghs.mst_weight == w_py
