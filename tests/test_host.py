"""Host logic of the product package (no GPU): canonicalisation, reference file formats,
binary format, result schema. Checked against the oracle's independent restatement."""
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN, fixture_names, load_fixture
from distributed_ghs_implementation_amd import graph as G
from oracle import oracle


@pytest.mark.parametrize("name", fixture_names())
def test_canonicalize_matches_oracle(name):
    fx = load_fixture(name)
    g = G.canonicalize(fx["num_nodes"], edges=fx["edges"])
    assert g.edge_triples() == oracle.canonicalize_py(fx["num_nodes"], fx["edges"])
    g.check()


def test_canonicalize_random_duplicates_last_write_wins():
    rng = random.Random(3)
    for _ in range(50):
        n = rng.randint(1, 30)
        edges = [(rng.randrange(n), rng.randrange(n), rng.randint(0, 5)) for _ in range(rng.randint(0, 80))]
        g = G.canonicalize(n, edges=edges)
        assert g.edge_triples() == oracle.canonicalize_py(n, edges)


def test_canonicalize_validation():
    with pytest.raises(ValueError):
        G.canonicalize(3, edges=[(0, 3, 1)])
    with pytest.raises(ValueError):
        G.canonicalize(3, edges=[(0, 1, float("nan"))])
    with pytest.raises(ValueError):
        G.canonicalize(3, edges=[(0, 1, "heavy")])
    g = G.canonicalize(3, edges=[(0, 1, 2.0)])
    assert g.edge_triples() == [(0, 1, 2)]
    assert G.canonicalize(0, edges=[]).m == 0


@pytest.mark.parametrize("kind", ["negative", "float", "huge", "mixed"])
def test_non_u32_weights_rank_mapped(kind):
    """nx.Graph (so the reference's GHSAlgorithm, ghs_implementation.py:417-440) takes any
    numeric weight. Non-u32 weights go to the engine as their dense rank: order and ties are
    kept, so canonical Kruskal on the ranks picks exactly the edges Kruskal picks on the
    original values (oracle.kruskal_py handles any comparable weights), and the reported
    triples / weight are the caller's values."""
    rng = random.Random(7)
    for _ in range(40):
        n = rng.randint(2, 40)
        def wt():
            if kind == "negative":
                return rng.randint(-5, 5)
            if kind == "float":
                return rng.choice([0.5, -1.25, 3.0, 2.75, 1e9, -1e-3])
            if kind == "huge":
                return rng.choice([1 << 40, (1 << 40) + 1, 7, 1 << 63])
            return rng.choice([1, 2.5, -3, 1 << 33])
        edges = [(rng.randrange(n), rng.randrange(n), wt()) for _ in range(rng.randint(1, 120))]
        g = G.canonicalize(n, edges=edges)
        canon = oracle.canonicalize_py_any(n, edges)
        assert g.edge_triples() == canon
        ref_in, ref_w = oracle.kruskal_py(n, canon)
        got_in, _, _ = oracle.kruskal_c(n, g.u, g.v, g.w)
        assert list(got_in) == ref_in
        assert g.total_weight(got_in.astype(bool)) == pytest.approx(ref_w, rel=1e-12)  # float sums: order differs


def test_read_reference_graph_dir():
    # directory written by the reference's own create_node_files (create_graph_files.py:43-89)
    d = os.path.join(GOLDEN, "graph_data_n6")
    g = G.read_graph_dir(d)
    fx = load_fixture("cgf_n6.json")
    assert g.n == 6 and g.edge_triples() == oracle.canonicalize_py(6, fx["edges"])
    g2 = G.read_node_files(d)  # the MPI ranks' view (ghs_implementation_mpi.py:74-92)
    assert g2.edge_triples() == g.edge_triples()


def test_write_graph_dir_roundtrip(tmp_path):
    fx = load_fixture("thread_cfg5.json")
    g = G.canonicalize(fx["num_nodes"], edges=fx["edges"])
    G.write_graph_dir(g, str(tmp_path))
    assert G.read_graph_dir(str(tmp_path)).edge_triples() == g.edge_triples()
    os.remove(tmp_path / "graph_metadata.json")
    assert G.read_graph_dir(str(tmp_path)).edge_triples() == g.edge_triples()
    node0 = json.load(open(tmp_path / "node_0.json"))
    assert set(node0) == {"node_id", "neighbors", "num_neighbors"}


def test_missing_graph_dir_raises(tmp_path):
    with pytest.raises(FileNotFoundError):
        G.read_graph_dir(str(tmp_path))


def test_mstbin_roundtrip(tmp_path):
    fx = load_fixture("ties_4.json")
    g = G.canonicalize(fx["num_nodes"], edges=fx["edges"])
    p = str(tmp_path / "g.mstbin")
    G.write_mstbin(p, g)
    h = G.read_mstbin(p)
    assert h.n == g.n and np.array_equal(h.u, g.u) and np.array_equal(h.v, g.v) and np.array_equal(h.w, g.w)


def test_result_schema(tmp_path):
    res = G.write_result(str(tmp_path / "ghs_mst.json"), [(3, 5, 2), (0, 2, 2), (0, 3, 1)])
    on_disk = json.load(open(tmp_path / "ghs_mst.json"))
    assert on_disk == res
    # same keys as ghs_implementation_mpi.py:811-816
    assert set(res) == {"mst_edges", "total_weight", "num_edges", "algorithm"}
    assert res["mst_edges"] == [[0, 2, 2], [0, 3, 1], [3, 5, 2]]
    assert res["total_weight"] == 5 and res["num_edges"] == 3


def _fixture_graph_and_result(name):
    fx = load_fixture(name)
    g = G.canonicalize(fx["num_nodes"], edges=fx["edges"])
    return g, [tuple(e) for e in fx["expected_mst_edges"]], fx


@pytest.mark.parametrize("name", fixture_names())
def test_verify_accepts_oracle_msf(name):
    """verify.py (the check_mst.py equivalent) accepts the pinned canonical MSF of every fixture."""
    from distributed_ghs_implementation_amd.verify import verify_forest
    g, exp, fx = _fixture_graph_and_result(name)
    rep = verify_forest(g, exp)
    assert rep["ok"], rep
    assert rep["mst_weight"] == fx["expected_total_weight"]
    assert rep["mst_edges"] == rep["edges_expected"]
    if rep["networkx_weight"] is not None:
        assert rep["weight_matches_networkx"]


def test_verify_rejects_broken_results():
    from distributed_ghs_implementation_amd.verify import verify_forest
    g, exp, _ = _fixture_graph_and_result("readme6.json")
    assert verify_forest(g, exp)["ok"]
    assert not verify_forest(g, exp[:-1])["spans_components"]          # an edge missing
    extra = [e for e in g.edge_triples() if e not in exp][0]
    assert not verify_forest(g, exp + [extra])["is_forest"]            # a cycle
    bad_w = [(exp[0][0], exp[0][1], exp[0][2] + 1)] + exp[1:]
    assert not verify_forest(g, bad_w)["weights_match_graph"]          # wrong weight
    assert not verify_forest(g, [(0, 5, 1)] + exp[1:])["edges_in_graph"]  # not a graph edge
    # a spanning tree that is not minimum: structurally fine, rejected by the NetworkX weight
    pytest.importorskip("networkx")
    heavier = [e for e in exp if e != (0, 1, 1)] + [(0, 2, 4)]
    rep = verify_forest(g, heavier)
    assert rep["is_forest"] and rep["spans_components"] and not rep["ok"]


def test_experiment_record_schema():
    """ghs_experiments.json entry (ghs_implementation.py:766-776)."""
    from distributed_ghs_implementation_amd.verify import experiment_record
    g, exp, fx = _fixture_graph_and_result("readme6.json")
    rec = experiment_record(1, g, exp)
    assert list(rec) == ["experiment", "num_nodes", "num_edges", "mst_edges", "mst_weight", "networkx_weight",
                         "is_correct", "edges_found", "edges_expected"]
    assert rec["mst_weight"] == 20 and rec["is_correct"] and rec["edges_found"] == rec["edges_expected"] == 5


def test_cli_check_result_without_gpu(tmp_path):
    """`python -m distributed_ghs_implementation_amd --graph-dir D --check-result F`: the
    check_mst.py flow on the reference's own graph-file directory, no GPU needed."""
    from distributed_ghs_implementation_amd.__main__ import main
    g, exp, _ = _fixture_graph_and_result("readme6.json")
    d = tmp_path / "graph"
    G.write_graph_dir(g, str(d))
    good = tmp_path / "good.json"
    G.write_result(str(good), exp)
    assert main(["--graph-dir", str(d), "--check-result", str(good)]) == 0
    bad = tmp_path / "bad.json"
    G.write_result(str(bad), exp[:-1])
    assert main(["--graph-dir", str(d), "--check-result", str(bad)]) == 1
