"""GPU parity: the HIP path (through the C-ABI) vs the oracle, bit-exact on MSF edge sets.

Small/medium sizes compare against oracle Kruskal on the same canonical input; the BASELINE
sizes (R-MAT s24, the 16384^2 grids) are compared bit-exact with an independent plain-torch
Boruvka (tests/torch_boruvka.py, itself pinned against the oracle on CPU) and checked by
size-independent properties: a connected grid gives n - 1 edges, the flags do not depend on
the level plan or on the rank partition, and repeated solves are identical.
"""
import os
import numpy as np
import pytest

from conftest import fixture_names, load_fixture

pytestmark = pytest.mark.gpu


def _oracle():
    from oracle import oracle
    return oracle


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_ghs_implementation_amd import _native
    assert _native.device_count() > 0
    return torch


@pytest.mark.parametrize("name", fixture_names())
def test_golden_fixtures_through_ghsalgorithm(name, torch_cuda):
    from distributed_ghs_implementation_amd import GHSAlgorithm
    fx = load_fixture(name)
    ghs = GHSAlgorithm(fx["num_nodes"], [tuple(e) for e in fx["edges"]])
    edges = ghs.run(timeout=5)
    exp = fx["expected_mst_edges"]
    assert edges == [(a, b) for a, b, _ in exp]
    assert ghs.mst_weight == fx["expected_total_weight"]
    assert [list(t) for t in ghs.mst_triples()] == exp
    for a, b in edges:  # reference harness reads weights as ghs.graph[u][v]["weight"]
        assert ghs.graph[a][b]["weight"] == ghs.graph[b][a]["weight"]


def _random_graph(rng, n, m, wmax):
    u = rng.integers(0, n, m)
    v = rng.integers(0, n, m)
    w = rng.integers(0, wmax + 1, m)
    return u, v, w


@pytest.mark.parametrize("seed,n,m,wmax", [(1, 10, 30, 2), (2, 100, 400, 1), (3, 1000, 3000, 3), (4, 5000, 40000, 10),
                                           (5, 20000, 60000, 1000), (6, 3000, 300000, 0), (7, 50000, 20000, 5),
                                           (8, 100000, 1000000, 1 << 31), (9, 2, 1, 7), (10, 1, 0, 1)])
def test_random_tie_graphs_vs_oracle(seed, n, m, wmax, torch_cuda):
    from distributed_ghs_implementation_amd import canonicalize, minimum_spanning_forest
    ora = _oracle()
    rng = np.random.default_rng(seed)
    u, v, w = _random_graph(rng, n, m, wmax)
    g = canonicalize(n, u=u, v=v, w=w)
    r = minimum_spanning_forest(g)
    ref_in, ref_tw, ref_k = ora.kruskal_c(n, g.u, g.v, g.w)
    assert np.array_equal(r.in_mst, ref_in.astype(bool))
    assert r.total_weight == ref_tw and r.num_edges == ref_k


def test_noncanonical_device_input_rejected(torch_cuda):
    import torch
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceEdges, DeviceMST
    t = lambda a: torch.tensor(a, dtype=torch.int32, device="cuda")
    for u, v in [([1, 0], [2, 3]), ([0, 0], [1, 9]), ([2], [1]), ([0, 0], [1, 1])]:
        e = DeviceEdges(4, t(u), t(v), t([1] * len(u)))
        with pytest.raises(_native.GHSError) as ei:
            DeviceMST(e).run()
        assert ei.value.code == _native.GHS_E_NONCANON


CONFIGS = [dict(max_levels=1), dict(), dict(max_levels=6, level1_edges_per_vertex=0.25, level_growth=2.0),
           dict(max_levels=16, level1_edges_per_vertex=0.01, level_growth=1.5)]


@pytest.mark.parametrize("cfg", CONFIGS)
@pytest.mark.parametrize("scale", [10, 14, 18])
def test_rmat_device_vs_oracle(scale, cfg, torch_cuda):
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
    ora = _oracle()
    e = generate_rmat(scale, 16, seed=1, wseed=2)
    g = e.to_host()
    g.check()
    assert len(np.unique(g.w)) == g.m  # unique weights by construction
    eng = DeviceMST(e, config=_native.make_config(**cfg))
    res, stats = eng.run()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(eng.in_mst_host(), ref_in.astype(bool))
    assert res.total_weight == ref_tw and res.num_mst_edges == ref_k
    assert sum(st["hooks"] for st in stats) == ref_k or res.rounds > len(stats)


@pytest.mark.parametrize("cfg", CONFIGS[:3])
@pytest.mark.parametrize("k,mode", [(2, 0), (3, 1), (64, 0), (257, 1), (1024, 0), (1024, 1)])
def test_grid_device_vs_oracle(k, mode, cfg, torch_cuda):
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_grid
    ora = _oracle()
    e = generate_grid(k, mode)
    g = e.to_host()
    g.check()
    assert g.m == 2 * k * (k - 1)
    eng = DeviceMST(e, config=_native.make_config(**cfg))
    res, _ = eng.run()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(eng.in_mst_host(), ref_in.astype(bool))
    assert res.num_mst_edges == k * k - 1 == ref_k


@pytest.mark.parametrize("cfg", CONFIGS)
def test_tie_heavy_levels_vs_oracle(cfg, torch_cuda):
    """Equal weights across level thresholds (a whole weight class lands in one level)."""
    from distributed_ghs_implementation_amd import _native, canonicalize
    from distributed_ghs_implementation_amd.device import DeviceEdges, DeviceMST
    ora = _oracle()
    rng = np.random.default_rng(11)
    n, m = 30000, 400000
    g = canonicalize(n, u=rng.integers(0, n, m), v=rng.integers(0, n, m), w=rng.integers(0, 4, m))
    eng = DeviceMST(DeviceEdges.from_host(g), config=_native.make_config(**cfg))
    res, _ = eng.run()
    ref_in, ref_tw, _ = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(eng.in_mst_host(), ref_in.astype(bool)) and res.total_weight == ref_tw


def test_stepwise_solver_equals_monolithic(torch_cuda):
    """The multi-GPU step API at world size 1 (pack -> identity all-reduce -> unpack) must give
    the same flags as ghs_mst_device."""
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
    from distributed_ghs_implementation_amd.distributed import HipStepper, run_rounds
    e = generate_rmat(16, 16, seed=5, wseed=6)
    a = DeviceMST(e)
    ra, _ = a.run()
    b = DeviceMST(e)
    st = HipStepper(b)
    run_rounds(st, lambda t: None)
    rb, _ = st.finish()
    assert np.array_equal(a.in_mst_host(), b.in_mst_host())
    assert ra.total_weight == rb.total_weight and ra.rounds == rb.rounds
    # the same handle again after ghs_solver_reset (what DistributedMST does per solve)
    b.in_mst.fill_(7)
    st.reset()
    run_rounds(st, lambda t: None)
    rc, _ = st.finish()
    st.close()
    assert np.array_equal(a.in_mst_host(), b.in_mst_host())
    assert rc.total_weight == ra.total_weight and rc.rounds == ra.rounds


def _emulate_ranks(e, world, cfg=None, bitmaps=True, rs=False):
    """`world` edge-range engines on one GPU stepping in lock step, the collectives emulated with
    torch.maximum / torch.minimum (exactly what RCCL's MAX / MIN all-reduce compute). rs: a dense
    level's opening round through the reduce-scatter protocol (hook_slots / reduce-scatter MIN /
    hook_owner / all-gather / apply_hooks, ABI 6) instead of all-reduce + owner hooks. Returns the
    MSF flags assembled from the ranks' own slices (each rank writes only [e_lo, e_hi)) and every
    rank's (total weight, MSF edges)."""
    import torch
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, edge_range
    from distributed_ghs_implementation_amd.distributed import HipStepper
    cfg = cfg or _native.make_config(num_ranks=world)
    engines = [DeviceMST(e, *edge_range(e.m, r, world), config=cfg) for r in range(world)]
    assert sum(x.e_hi - x.e_lo for x in engines) == e.m
    for x in engines:  # a sentinel outside each rank's own range: it must never be written
        x.in_mst.fill_(7)
    steppers = [HipStepper(x) for x in engines]
    try:
        done = False
        while not done:
            # a dense level's LDS tail (ABI 10): MIN of the F keys (unsigned), agree, MAX of the hooks
            F = [s.tail_begin() for s in steppers]
            assert len(set(F)) == 1
            if F[0]:
                bufs = [s.tail_buffers(F[0]) for s in steppers]
                sign = torch.tensor(-(1 << 63), dtype=torch.int64, device=bufs[0][0].device)
                while True:
                    red = bufs[0][0] ^ sign
                    for k, _ in bufs[1:]:
                        red = torch.minimum(red, k ^ sign)
                    red ^= sign
                    for k, _ in bufs:
                        k.copy_(red)
                    for s in steppers:
                        s.tail_agree()
                    hmax = bufs[0][1].clone()
                    for _, h in bufs[1:]:
                        hmax = torch.maximum(hmax, h)
                    for _, h in bufs:
                        h.copy_(hmax)
                    states = [s.tail_round() for s in steppers]
                    assert len(set(states)) == 1
                    if states[0]:
                        break
                done = states[0] == 2
                continue
            counts = [s.minedge() for s in steppers]
            while counts[0] is None:  # a level opened: OR-combine the fragment flags
                assert all(c is None for c in counts)
                if bitmaps:  # packed bitmaps, all-gathered (emulated: concatenated), OR-ed on device
                    gathered = torch.cat([s.flag_bits().clone() for s in steppers])
                    for s in steppers:
                        s.merge_flag_bits(gathered, world)
                else:  # the n + 1 flag bytes, all-reduced with MAX (emulated)
                    bufs = [s.exchange_buffer() for s in steppers]
                    red = bufs[0].clone()
                    for b in bufs[1:]:
                        red = torch.maximum(red, b)
                    for b in bufs:
                        b.copy_(red)
                counts = [s.minedge() for s in steppers]
            assert len(set(counts)) == 1
            slots = [s.hook_slots(world) for s in steppers] if rs and counts[0] else [None]
            assert len(set(x is None for x in slots)) == 1
            if slots[0] is not None:  # reduce-scatter MIN (unsigned) + the owners' pairs all-gathered
                S = int(slots[0].numel())
                assert S % world == 0 and S >= counts[0]
                sign = torch.tensor(-(1 << 63), dtype=torch.int64, device=slots[0].device)
                red = slots[0] ^ sign
                for v in slots[1:]:
                    red = torch.minimum(red, v ^ sign)
                red ^= sign
                per = S // world
                for r, v in enumerate(slots):  # each rank receives its own slice only
                    v[r * per:(r + 1) * per].copy_(red[r * per:(r + 1) * per])
                pairs = torch.full((S,), -2, dtype=torch.int64, device=slots[0].device)
                for r, st in enumerate(steppers):
                    st.hook_owner(r, per, pairs)
                assert not bool((pairs == -2).any())  # every slot written by its owner
                partial = [st.apply_hooks(pairs) for st in steppers]
                tot = sum(pt.clone() for pt in partial)  # the SUM all-reduce of the partial totals
                for pt in partial:
                    pt.copy_(tot)
            elif counts[0]:
                dense = [s.pack(counts[0]).clone() for s in steppers]
                red = dense[0]
                for d in dense[1:]:
                    red = torch.minimum(red, d)
                for s in steppers:
                    s.unpack(red)
                hooks = [s.hook_local() for s in steppers]  # owner-computes hook (a level's round 0)
                assert len(set(h is None for h in hooks)) == 1
                if hooks[0] is not None:
                    nz = sum((h != 0).to(torch.int64) for h in hooks)
                    assert int(nz.max().item()) <= 1  # one owner per winning edge
                    hmax = hooks[0].clone()
                    for h in hooks[1:]:
                        hmax = torch.maximum(hmax, h)
                    for s in steppers:
                        s.unpack_hook(hmax)
            dones = [s.contract() for s in steppers]
            assert len(set(dones)) == 1
            done = dones[0]
        totals = []
        for s in steppers:
            res, _ = s.finish()
            totals.append((res.total_weight, res.num_mst_edges))
        # owner-written flags: the MSF is the concatenation of the ranks' own slices, and no rank
        # wrote outside its range
        flags = torch.empty(e.m, dtype=torch.uint8, device=e.device)
        for x in engines:
            flags[x.e_lo:x.e_hi] = x.in_mst[x.e_lo:x.e_hi]
            assert bool((x.in_mst[: x.e_lo] == 7).all()) and bool((x.in_mst[x.e_hi: e.m] == 7).all())
        assert int(flags.max().item() if e.m else 0) <= 1
        return flags, totals
    finally:
        for s in steppers:
            s.close()


@pytest.mark.parametrize("world,graph,bitmaps,rs", [(2, "rmat", True, False), (3, "rmat", False, False),
                                                    (8, "rmat", True, False), (8, "grid", True, False),
                                                    (5, "grid-gradient", True, False), (8, "readme", True, False),
                                                    (8, "readme", False, False), (4, "ties", True, False),
                                                    (4, "ties", False, False), (2, "rmat", True, True),
                                                    (8, "rmat", True, True), (8, "grid", True, True),
                                                    (5, "grid-gradient", True, True), (8, "readme", True, True),
                                                    (3, "ties", True, True), (4, "forest", True, True)])
def test_partitioned_ranks_emulated_on_one_gpu(world, graph, bitmaps, rs, torch_cuda):
    """`world` edge-range engines on one GPU, all-reduces emulated: the OR of the ranks' flags is
    canonical Kruskal's MSF (oracle) and every rank reports the oracle's totals."""
    from distributed_ghs_implementation_amd import canonicalize
    from distributed_ghs_implementation_amd.device import DeviceEdges, generate_grid, generate_rmat
    ora = _oracle()
    if graph == "rmat":
        e = generate_rmat(15, 16, seed=3, wseed=4)
    elif graph == "readme":  # 9 edges over 8 ranks: most ranks own no edge at all
        e = DeviceEdges.from_host(canonicalize(6, edges=[(0, 1, 1), (0, 2, 4), (1, 2, 2), (1, 3, 5), (2, 3, 3),
                                                         (2, 4, 7), (3, 4, 6), (3, 5, 8), (4, 5, 9)]))
    elif graph == "ties":  # equal weights across ranks: the (w, eid) tie-break must hold globally
        rng = np.random.default_rng(12)
        n, m = 3000, 20000
        e = DeviceEdges.from_host(canonicalize(n, u=rng.integers(0, n, m), v=rng.integers(0, n, m),
                                               w=rng.integers(0, 3, m)))
    elif graph == "forest":  # many components, isolated vertices
        e = _test_graph("forest")
    else:
        e = generate_grid(257, 1 if graph == "grid-gradient" else 0)
    flags, totals = _emulate_ranks(e, world, bitmaps=bitmaps, rs=rs)
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(flags.cpu().numpy().astype(bool), ref_in.astype(bool))
    assert set(totals) == {(ref_tw, ref_k)}


def test_partitioned_noncanonical_fails_on_every_rank(torch_cuda):
    """A non-canonical edge in ONE rank's range: every rank returns GHS_E_NONCANON from the same
    minedge call (the error byte travels with the exchanged flags), so no rank would be left
    waiting in a collective."""
    import torch
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceEdges, DeviceMST, edge_range, generate_rmat
    from distributed_ghs_implementation_amd.distributed import HipStepper
    e = generate_rmat(12, 16, seed=1, wseed=2)
    world = 4
    lo, hi = edge_range(e.m, 2, world)
    v = e.v.clone()
    v[(lo + hi) // 2] = e.u[(lo + hi) // 2]  # u == v inside rank 2's range
    bad = DeviceEdges(e.n, e.u, v, e.w)
    cfg = _native.make_config(num_ranks=world)
    steppers = [HipStepper(DeviceMST(bad, *edge_range(e.m, r, world), config=cfg)) for r in range(world)]
    try:
        assert all(s.minedge() is None for s in steppers)  # level 0 opened on every rank
        bufs = [s.exchange_buffer() for s in steppers]
        assert all(b.numel() == e.n + 1 for b in bufs)  # n flags + the error byte
        red = bufs[0].clone()
        for b in bufs[1:]:
            red = torch.maximum(red, b)
        for b in bufs:
            b.copy_(red)
        for s in steppers:
            with pytest.raises(_native.GHSError) as ei:
                s.minedge()
            assert ei.value.code == _native.GHS_E_NONCANON
    finally:
        for s in steppers:
            s.close()


@pytest.fixture(scope="module")
def rmat_s26_reference(torch_cuda):
    """BASELINE config 4's graph (R-MAT s26, ~1.05B canonical edges) and its single-GPU MSF,
    checked bit-exact against the independent torch Boruvka (full-size parity of config 4)."""
    torch = torch_cuda
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
    from torch_boruvka import msf_boruvka
    e = generate_rmat(26, 16, seed=1, wseed=2)
    eng = DeviceMST(e)
    res, _ = eng.run()
    flags = eng.in_mst[: e.m].clone()
    del eng
    torch.cuda.empty_cache()
    ref = msf_boruvka(e.n, e.u, e.v, e.w)
    assert torch.equal(flags.bool(), ref), "s26 single-GPU MSF differs from the torch Boruvka checker"
    del ref
    _oracle_full_size(e, flags, res)
    torch.cuda.empty_cache()
    w = (e.w.to(torch.int64) & 0xFFFFFFFF)
    assert int(flags.sum().item()) == res.num_mst_edges
    assert int(w[flags.bool()].sum().item()) == res.total_weight
    del w
    yield e, flags, (res.total_weight, res.num_mst_edges)
    del e
    torch.cuda.empty_cache()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_partitioned_s26_emulated(world, rmat_s26_reference, torch_cuda):
    """BASELINE config 4 (R-MAT s26 edge-partitioned over 2/4/8 ranks, all-reduces emulated on
    one GPU): the OR of the ranks' flags is the s26 MSF (single GPU == torch Boruvka checker)
    and every rank reports the same totals."""
    torch = torch_cuda
    e, ref_flags, ref_tot = rmat_s26_reference
    flags, totals = _emulate_ranks(e, world)
    assert torch.equal(flags, ref_flags)
    assert set(totals) == {ref_tot}
    del flags
    torch.cuda.empty_cache()


def _test_graph(graph):
    from distributed_ghs_implementation_amd import canonicalize
    from distributed_ghs_implementation_amd.device import DeviceEdges, generate_grid, generate_rmat
    if graph == "rmat":
        return generate_rmat(15, 16, seed=3, wseed=4)
    if graph == "rmat20":  # the bucketed filter's waves hold several groups each
        return generate_rmat(20, 24, seed=5, wseed=6)
    if graph == "readme":  # 9 edges: most of 8 ranks own no edge at all
        return DeviceEdges.from_host(canonicalize(6, edges=[(0, 1, 1), (0, 2, 4), (1, 2, 2), (1, 3, 5), (2, 3, 3),
                                                            (2, 4, 7), (3, 4, 6), (3, 5, 8), (4, 5, 9)]))
    if graph == "ties":
        rng = np.random.default_rng(12)
        n, m = 3000, 20000
        return DeviceEdges.from_host(canonicalize(n, u=rng.integers(0, n, m), v=rng.integers(0, n, m),
                                                  w=rng.integers(0, 3, m)))
    if graph == "forest":  # many components, isolated vertices
        rng = np.random.default_rng(13)
        n, m = 50000, 20000
        return DeviceEdges.from_host(canonicalize(n, u=rng.integers(0, n, m), v=rng.integers(0, n, m),
                                                  w=rng.integers(0, 50, m)))
    return generate_grid(257, 1 if graph == "grid-gradient" else 0)


@pytest.mark.parametrize("world,graph", [(2, "rmat"), (3, "ties"), (8, "rmat"), (8, "grid"), (5, "grid-gradient"),
                                         (8, "readme"), (4, "forest"), (1, "rmat")])
def test_native_loop_emulated_vs_oracle(world, graph, torch_cuda):
    """ghs_solver_run — the library's own multi-rank round loop, the one DistributedMST runs over
    RCCL — with `world` rank solvers on this GPU (ghs_mst_emulated: a host thread and a stream per
    rank, in-process collectives): the assembled own-range flags and every rank's totals equal
    oracle Kruskal."""
    from distributed_ghs_implementation_amd.device import emulated_mst
    ora = _oracle()
    e = _test_graph(graph)
    res, stats, flags = emulated_mst(e, world)
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(flags.cpu().numpy().astype(bool), ref_in.astype(bool))
    assert (res.total_weight, res.num_mst_edges) == (ref_tw, ref_k)
    assert len(stats) == res.num_stats
    # rounds >= 2 of a level are pipelined (read from the round reports): every round's stats once
    assert sum(st["hooks"] for st in stats) == ref_k or res.rounds > len(stats)
    assert res.rounds == len(stats) or res.rounds > 64


@pytest.mark.parametrize("world,graph", [(2, "rmat"), (8, "rmat"), (3, "ties"), (4, "grid"), (5, "grid-gradient"),
                                         (4, "forest"), (8, "rmat20"), (8, "readme")])
def test_native_loop_multi_rank_tail_vs_oracle(world, graph, torch_cuda):
    """The LDS tail in the multi-rank loop (a dense level once <= TAIL_MAX fragments stay active:
    ghs_solver_tail_multi drains the pipelined rounds, then every tail round's hooks are agreed by
    a MIN all-reduce of the F0 keys and a MAX all-reduce of the CONNECT targets; the owner rank
    writes the MSF flag): flags and totals equal oracle Kruskal and the loop without the tail
    (GHS_OPT_NO_TAIL); pass_flags bit 3 says the tail ran."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import emulated_mst
    ora = _oracle()
    e = _test_graph(graph)
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    res, stats, flags = emulated_mst(e, world)
    res0, _, flags0 = emulated_mst(e, world, config=_native.make_config(options=_native.OPT_NO_TAIL))
    for r, f in ((res, flags), (res0, flags0)):
        assert np.array_equal(f.cpu().numpy().astype(bool), ref_in.astype(bool))
        assert (r.total_weight, r.num_mst_edges) == (ref_tw, ref_k)
    assert not res0.pass_flags & 8
    if graph in ("rmat", "rmat20", "grid", "ties"):
        assert res.pass_flags & 8
    assert sum(st["hooks"] for st in stats) == ref_k
    assert res.rounds == len(stats)


@pytest.mark.parametrize("dedup_max", [128, 1000000000])
@pytest.mark.parametrize("graph,world", [("rmat", 1), ("ties", 1), ("forest", 1), ("grid", 1), ("rmat", 4),
                                         ("ties", 3)])
def test_parallel_edge_filter_vs_oracle(graph, world, dedup_max, torch_cuda):
    """The compacting min-edge's parallel-edge filter (ghs_config_t.dedup_max: per block, survivors between
    the same two fragments keep only their minimum key) at <= 128 active fragments and in every
    compacting round: the oracle's MSF, single GPU and through the multi-rank loop."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, emulated_mst
    cfg = _native.make_config(dedup_max=dedup_max)
    ora = _oracle()
    e = _test_graph(graph)
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    if world == 1:
        eng = DeviceMST(e, config=cfg)
        res, _ = eng.run()
        flags = eng.in_mst_host()
    else:
        res, _, f = emulated_mst(e, world, config=cfg)
        flags = f.cpu().numpy().astype(bool)
    assert np.array_equal(flags, ref_in.astype(bool))
    assert (res.total_weight, res.num_mst_edges) == (ref_tw, ref_k)


def test_native_loop_emulated_noncanonical_fails_together(torch_cuda):
    """A non-canonical edge in one rank's range: ghs_mst_emulated returns GHS_E_NONCANON (every
    rank leaves the loop at the same step — no rank left waiting in a collective)."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceEdges, edge_range, emulated_mst, generate_rmat
    e = generate_rmat(12, 16, seed=1, wseed=2)
    lo, hi = edge_range(e.m, 1, 4)
    v = e.v.clone()
    v[(lo + hi) // 2] = e.u[(lo + hi) // 2]
    with pytest.raises(_native.GHSError) as ei:
        emulated_mst(DeviceEdges(e.n, e.u, v, e.w), 4)
    assert ei.value.code == _native.GHS_E_NONCANON


@pytest.mark.parametrize("world,fault", [(4, 2), (4, 1), (3, 3), (1, 1)])
def test_rank_setup_failure_fails_every_rank(world, fault, torch_cuda):
    """One rank's setup fails (ghs_config_t.fault_rank = 1 + rank: its workspace is refused):
    ghs_mst_emulated returns an error from every rank (the setup agreement before the first
    collective) instead of hanging, and the same graph then solves normally."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import emulated_mst, generate_rmat
    ora = _oracle()
    e = generate_rmat(12, 16, seed=1, wseed=2)
    cfg = _native.make_config(fault_rank=fault)
    with pytest.raises(_native.GHSError) as ei:
        emulated_mst(e, world, config=cfg)
    assert ei.value.code in (_native.GHS_E_NOMEM, _native.GHS_E_STATE)
    res, _, flags = emulated_mst(e, world)
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(flags.cpu().numpy().astype(bool), ref_in.astype(bool))


@pytest.mark.parametrize("world,fault,round_", [(4, 2, 1), (4, 4, 3), (2, 1, 2)])
def test_rank_mid_solve_failure_fails_every_rank(world, fault, round_, torch_cuda):
    """One rank fails INSIDE the round loop (ghs_config_t.fault_round: after `round_` rounds, while
    its peers go on into the next collective): every rank returns an error instead of hanging (the
    group's cancel flag ends their waits), the failing rank's own error is reported, the drivers'
    cached state is dropped, and the next call solves normally — then a call of the same shape runs
    on the cached state (ABI 7: no allocation)."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import emulated_mst, generate_rmat
    ora = _oracle()
    e = generate_rmat(13, 16, seed=3, wseed=4)
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    with pytest.raises(_native.GHSError) as ei:
        emulated_mst(e, world, config=_native.make_config(fault_rank=fault, fault_round=round_))
    assert ei.value.code == _native.GHS_E_STATE
    assert "injected mid-solve failure" in str(ei.value)
    keep = _native.make_config(options=_native.OPT_KEEP_CACHE)
    for k in range(2):
        res, _, flags = emulated_mst(e, world, config=keep)
        assert np.array_equal(flags.cpu().numpy().astype(bool), ref_in.astype(bool))
        assert (res.total_weight, res.num_mst_edges) == (ref_tw, ref_k)
        assert res.reused == k  # the failed call left nothing cached; the second call reuses
        assert res.ms_setup > 0 and res.ms_solve > 0
    _native.release_cache()


def test_fault_round_rejected_with_one_rank(torch_cuda):
    """fault_round on a one-rank loop (no exchange to fail in) is GHS_E_ARG, not a
    silent success."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import emulated_mst, generate_rmat
    e = generate_rmat(11, 16, seed=1, wseed=2)
    with pytest.raises(_native.GHSError) as ei:
        emulated_mst(e, 1, config=_native.make_config(fault_rank=1, fault_round=1))
    assert ei.value.code == _native.GHS_E_ARG


def test_driver_cache_follows_the_shape(torch_cuda):
    """The drivers' cache holds one shape: another graph (or rank count) allocates afresh, the
    same one reuses; ghs_mst_multi's 1-rank clique is cached too (its second call reuses)."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import emulated_mst, generate_rmat
    from distributed_ghs_implementation_amd.mst import minimum_spanning_forest
    ora = _oracle()
    a, b = generate_rmat(11, 16, seed=1, wseed=2), generate_rmat(12, 16, seed=1, wseed=2)
    keep = _native.make_config(options=_native.OPT_KEEP_CACHE)
    seen = []
    # the last call is without OPT_KEEP_CACHE: it runs on the kept state, then frees it (ABI 8)
    for e, world, cfg in ((a, 2, keep), (a, 2, keep), (b, 2, keep), (b, 3, keep), (b, 3, None), (b, 3, keep)):
        res, _, flags = emulated_mst(e, world, config=cfg)
        g = e.to_host()
        ref_in, _, _ = ora.kruskal_c(g.n, g.u, g.v, g.w)
        assert np.array_equal(flags.cpu().numpy().astype(bool), ref_in.astype(bool))
        seen.append(res.reused)
    assert seen == [0, 1, 0, 0, 1, 0]
    g = b.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    for k in range(2):
        r = minimum_spanning_forest(g, devices=[0], config=keep)
        assert np.array_equal(r.in_mst, ref_in.astype(bool))
    _native.release_cache()


@pytest.mark.parametrize("world", [2, 4])
def test_driver_cache_reuse_with_other_graph_same_shape(world, torch_cuda):
    """the cached per-rank state re-solving a DIFFERENT graph of the same (n, m) — other
    edges, other weights — so leftover workspace contents (tail buffers, collective scratch, report
    rings) cannot pass for fresh memory: both graphs' MSFs equal the oracle's, the second call runs
    on the first's state (reused = 1)."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceEdges, emulated_mst, generate_rmat
    ora = _oracle()
    a, b = generate_rmat(13, 16, seed=1, wseed=2), generate_rmat(13, 16, seed=9, wseed=10)
    mm = min(a.m, b.m) & ~3
    graphs = [DeviceEdges(x.n, x.u[:mm], x.v[:mm], x.w[:mm]) for x in (a, b)]  # a canonical prefix is canonical
    keep = _native.make_config(options=_native.OPT_KEEP_CACHE)
    for i, e in enumerate(graphs + graphs[:1]):
        res, _, flags = emulated_mst(e, world, config=keep)
        g = e.to_host()
        ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
        assert np.array_equal(flags.cpu().numpy().astype(bool), ref_in.astype(bool)), i
        assert (res.total_weight, res.num_mst_edges) == (ref_tw, ref_k)
        assert res.reused == (1 if i else 0)
    _native.release_cache()


def test_multi_gpu_entry_setup_failure(torch_cuda):
    """ghs_mst_multi (a 1-rank RCCL clique on the box's device) with its rank's setup failing:
    the setup agreement's RCCL all-reduce runs and the call returns the error."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import generate_rmat
    from distributed_ghs_implementation_amd.mst import minimum_spanning_forest
    g = generate_rmat(12, 16, seed=1, wseed=2).to_host()
    with pytest.raises(_native.GHSError) as ei:
        minimum_spanning_forest(g, devices=[0], config=_native.make_config(fault_rank=1))
    assert ei.value.code == _native.GHS_E_NOMEM


def test_native_loop_rccl_comm_one_rank(torch_cuda):
    """ghs_comm_unique_id / ghs_comm_init (ncclCommInitRank, 1 rank on this GPU) + ghs_solver_run
    on a solver handle, twice (reset between solves): the oracle's MSF; a 2-rank solver refuses a
    1-rank communicator."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
    from distributed_ghs_implementation_amd.distributed import HipStepper
    ora = _oracle()
    e = generate_rmat(14, 16, seed=7, wseed=8)
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    comm = _native.Comm(1, 0, _native.comm_unique_id())
    eng = DeviceMST(e)
    st = HipStepper(eng)
    try:
        for _ in range(2):
            st.run_native(comm)
            res, _ = st.finish()
            assert np.array_equal(eng.in_mst_host(), ref_in.astype(bool))
            assert (res.total_weight, res.num_mst_edges) == (ref_tw, ref_k)
            st.reset()
    finally:
        st.close()
    two = DeviceMST(e, 0, e.m // 2 & ~3, _native.make_config(num_ranks=2))
    st2 = HipStepper(two)
    try:
        with pytest.raises(_native.GHSError) as ei:
            st2.run_native(comm)
        assert ei.value.code == _native.GHS_E_ARG
    finally:
        st2.close()
        comm.close()


@pytest.mark.parametrize("world", [8])
def test_native_loop_s26_emulated(world, rmat_s26_reference, torch_cuda):
    """BASELINE config 4 through the library's round loop (ghs_mst_emulated, 8 ranks on this
    GPU): the s26 MSF of the single-GPU solve (== torch Boruvka checker)."""
    torch = torch_cuda
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import emulated_mst
    e, ref_flags, ref_tot = rmat_s26_reference
    res, _, flags = emulated_mst(e, world)
    _native.release_cache()  # ~N workspaces of s26 stay cached otherwise
    assert torch.equal(flags, ref_flags)
    assert (res.total_weight, res.num_mst_edges) == ref_tot
    del flags
    torch.cuda.empty_cache()


@pytest.mark.parametrize("scale,ef,seed,wseed", [(12, 16, 1, 2), (16, 16, 1, 2), (18, 16, 3, 4), (14, 8, 9, 0),
                                                 (1, 1, 1, 2), (2, 3, 5, 6), (3, 1, 7, 8), (10, 3, 1, 2),
                                                 (13, 5, 2, 3)])
def test_rmat_generator_matches_oracle(scale, ef, seed, wseed, torch_cuda):
    """Generator parity: the raw GPU tuples equal oracle/generators.c tuple for
    tuple, and the GPU canonical list (rocPRIM radix sort, then the k_uniq_* unique + decode:
    self-loops dropped, hashed weights) equals the oracle's canonicalisation of the same tuples,
    bit-exact. Tiny and ragged sizes cover partial unique tiles (4096 keys) and all-self-loop
    outcomes."""
    import torch
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import _ptr, _stream, generate_rmat
    ora = _oracle()
    L = _native.load()
    T = ef << scale
    keys = torch.empty(T, dtype=torch.int64, device="cuda")
    _native.check(L.ghs_rmat_tuples(scale, ef, seed, _ptr(keys), _stream()))
    k = keys.cpu().numpy().view(np.uint64)
    uu, vv = ora.rmat_pairs_c(scale, ef, seed)
    a = np.minimum(uu, vv).astype(np.uint64)
    b = np.maximum(uu, vv).astype(np.uint64)
    exp = np.where(uu == vv, np.uint64((1 << (2 * scale)) - 1), (a << np.uint64(scale)) | b)
    assert np.array_equal(k, exp)
    g = generate_rmat(scale, ef, seed=seed, wseed=wseed).to_host()
    n, cu, cv, cw = ora.rmat_canonical(scale, ef, seed, wseed)
    assert g.n == n and g.m == len(cu)
    assert np.array_equal(g.u, cu) and np.array_equal(g.v, cv) and np.array_equal(g.w, cw)


@pytest.mark.parametrize("k,mode,wseed", [(2, 0, 2), (3, 1, 2), (257, 0, 2), (1000, 1, 2), (1024, 0, 77)])
def test_grid_generator_matches_oracle(k, mode, wseed, torch_cuda):
    from distributed_ghs_implementation_amd.device import generate_grid
    ora = _oracle()
    g = generate_grid(k, mode, wseed=wseed).to_host()
    n, u, v, w = ora.grid_canonical(k, mode, wseed)
    assert g.n == n and g.m == len(u) == 2 * k * (k - 1)
    assert np.array_equal(g.u, u) and np.array_equal(g.v, v) and np.array_equal(g.w, w)


def test_check_canonical_utility(torch_cuda):
    import ctypes
    import torch
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import _ptr, _stream, generate_rmat
    L = _native.load()
    e = generate_rmat(12, 16, seed=1, wseed=2)
    ok = ctypes.c_int(0)
    _native.check(L.ghs_check_canonical(e.n, e.m, _ptr(e.u), _ptr(e.v), _stream(), ctypes.byref(ok)))
    assert ok.value == 1
    v = e.v.clone()
    v[e.m // 2] = e.u[e.m // 2]  # u == v breaks u < v
    _native.check(L.ghs_check_canonical(e.n, e.m, _ptr(e.u), _ptr(v), _stream(), ctypes.byref(ok)))
    assert ok.value == 0


def test_rmat_s20_oracle_and_determinism(torch_cuda):
    """Larger scale: bit-exact vs oracle Kruskal, and two runs give identical flags."""
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
    ora = _oracle()
    e = generate_rmat(20, 16, seed=1, wseed=2)
    eng = DeviceMST(e)
    r1, _ = eng.run()
    f1 = eng.in_mst_host()
    r2, _ = eng.run()
    f2 = eng.in_mst_host()
    assert np.array_equal(f1, f2) and r1.total_weight == r2.total_weight
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(f1, ref_in.astype(bool))


def _host_plan(w, n, m, max_levels=8, l1=0.0, growth=8.0, nsample=16384):
    """The level plan's formula (boruvka.hip k_plan, level1_auto) restated: order statistics of
    an evenly spaced weight sample."""
    if l1 <= 0:
        l1 = 0.5 if m >= 4 * n else 1.2
    L = max(1, min(max_levels, 32))
    thr = [0]
    if L > 1 and m > 0:
        ns = min(nsample, m)
        idx = (np.arange(ns, dtype=np.uint64) * np.uint64(m)) // np.uint64(ns)
        smp = np.sort(w[idx.astype(np.int64)].astype(np.uint64))
        target = l1 * float(n)
        for _ in range(1, L):
            frac = target / float(m)
            if frac >= 1.0:
                break
            q = int(frac * ns)
            target *= max(1.01, growth)
            if q == 0:
                continue
            t = int(smp[q])
            if t > thr[-1]:
                thr.append(t)
    thr.append(1 << 32)
    return thr


@pytest.mark.parametrize("scale,cfg", [(16, {}), (18, dict(max_levels=6, level1_edges_per_vertex=0.25, level_growth=2.0))])
def test_device_level_plan_matches_formula(scale, cfg, torch_cuda):
    """k_plan (device radix select) gives the thresholds of the formula: same level count, and
    level 0 holds exactly the edges below the first threshold (+ <= 3 padding entries per
    output region)."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
    e = generate_rmat(scale, 16, seed=7, wseed=8)
    g = e.to_host()
    kw = dict(max_levels=8, l1=0.0, growth=8.0)
    kw.update({"max_levels": cfg.get("max_levels", 8), "l1": cfg.get("level1_edges_per_vertex", 0.0),
               "growth": cfg.get("level_growth", 8.0)})
    thr = _host_plan(g.w, g.n, g.m, **kw)
    eng = DeviceMST(e, config=_native.make_config(**cfg))
    res, stats = eng.run()
    assert res.levels == len(thr) - 1
    below = int((g.w.astype(np.uint64) < np.uint64(thr[1])).sum())
    lvl0 = stats[0]["level_arcs"]
    assert below <= lvl0 <= below + 3 * 4 * 2048


def _oracle_full_size(e, flags, res):
    """The oracle at BASELINE size: oracle/boruvka_omp.c (the all-cores CPU restatement, pinned to
    canonical Kruskal on every golden fixture and random tie-heavy graphs in tests/test_oracle.py)
    over the same canonical arrays, flags compared edge for edge, totals with the GPU's."""
    ora = _oracle()
    cu, cv, cw = (t.cpu().numpy() for t in (e.u, e.v, e.w))
    ref, tw, k, _ = ora.boruvka_omp_c(e.n, cu, cv, cw)
    del cu, cv, cw
    got = flags.cpu().numpy().astype(bool)
    assert np.array_equal(got, ref.astype(bool)), "HIP MSF differs from the oracle at full size"
    assert (tw, k) == (res.total_weight, res.num_mst_edges)


def _full_size_checks(e, eng, res, torch):
    """BASELINE-size checks: the oracle (bit-exact, all cores), the independent torch Boruvka
    (bit-exact), determinism, and a second execution path (one weight level, i.e. no giant
    filter) giving the same flags."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST
    from torch_boruvka import msf_boruvka
    flags = eng.in_mst[: e.m].clone()
    _oracle_full_size(e, flags, res)
    ref = msf_boruvka(e.n, e.u, e.v, e.w)
    assert torch.equal(flags.bool(), ref), "HIP MSF differs from the torch Boruvka checker"
    del ref
    torch.cuda.empty_cache()
    assert int(flags.sum().item()) == res.num_mst_edges
    w = (e.w.to(torch.int64) & 0xFFFFFFFF)
    assert int(w[flags.bool()].sum().item()) == res.total_weight
    r2, _ = eng.run()
    assert torch.equal(eng.in_mst[: e.m], flags) and r2.total_weight == res.total_weight
    one = DeviceMST(e, config=_native.make_config(max_levels=1))
    r1, _ = one.run()
    assert torch.equal(one.in_mst[: e.m], flags) and r1.total_weight == res.total_weight
    return flags


def test_rmat_s24_full_size(torch_cuda):
    """BASELINE config 3 (R-MAT s24, 260M canonical edges) at full size."""
    torch = torch_cuda
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
    e = generate_rmat(24, 16, seed=1, wseed=2)
    eng = DeviceMST(e)
    res, _ = eng.run()
    assert res.levels >= 2  # the default plan exercises the giant filter
    _full_size_checks(e, eng, res, torch)


@pytest.mark.parametrize("mode", [0, 1])
def test_grid_16k_full_size(mode, torch_cuda):
    """BASELINE config 5 (16384^2 grid, 537M edges; mode 1 = gradient weights) at full size:
    connected, so exactly n - 1 MSF edges."""
    torch = torch_cuda
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_grid
    k = 16384
    e = generate_grid(k, mode)
    assert e.m == 2 * k * (k - 1)
    eng = DeviceMST(e)
    res, _ = eng.run()
    assert res.num_mst_edges == k * k - 1
    _full_size_checks(e, eng, res, torch)


def test_cli_graph_dir_with_check(tmp_path, torch_cuda):
    """The reference's CLI flow end to end on the reference's own graph-file directory
    (create_graph_files.py output): --graph-dir D -> ghs_mst.json, then --check (check_mst.py)."""
    import json
    import shutil

    from conftest import GOLDEN
    from distributed_ghs_implementation_amd.__main__ import main
    d = tmp_path / "graph_data"
    shutil.copytree(os.path.join(GOLDEN, "graph_data_n6"), d)
    assert main(["--graph-dir", str(d), "--check", "--quiet"]) == 0
    res = json.load(open(d / "ghs_mst.json"))
    assert res["total_weight"] == 11 and res["num_edges"] == 5  # README_MPI.md:228-235


@pytest.mark.parametrize("seed", [1, 2])
def test_any_numeric_weights_through_ghsalgorithm(seed, torch_cuda):
    """Negative / float / > 2^32 weights (nx.Graph accepts them, so the reference's GHSAlgorithm
    does: ghs_implementation.py:417-440) go through the engine as dense ranks: the same edges as
    canonical Kruskal on the original values, reported with the caller's weights."""
    import random
    from distributed_ghs_implementation_amd import GHSAlgorithm
    ora = _oracle()
    rng = random.Random(seed)
    n = 2000
    pool = [-7.5, -1, 0, 0.25, 3, 3.0000001, 1 << 40, -(1 << 35), 1e12]
    edges = [(rng.randrange(n), rng.randrange(n), rng.choice(pool)) for _ in range(12000)]
    ghs = GHSAlgorithm(n, edges)
    got = ghs.run()
    canon = ora.canonicalize_py_any(n, edges)
    ref_in, ref_w = ora.kruskal_py(n, canon)
    assert got == [(a, b) for (a, b, _), f in zip(canon, ref_in) if f]
    assert ghs.mst_weight == pytest.approx(ref_w, rel=1e-12)
    assert ghs.mst_triples() == [t for t, f in zip(canon, ref_in) if f]


@pytest.mark.parametrize("name", ["readme6.json", "cgf_n1000_p05.json.gz", "ties_4.json", "empty.json"])
def test_multi_gpu_entry_one_device_vs_oracle(name, torch_cuda):
    """ghs_mst_multi (one process, RCCL clique via ncclCommInitAll, one host thread per device)
    on the box's one device: the same flags as canonical Kruskal. The collective calls of the
    multi-rank protocol run (a 1-rank RCCL communicator); N > 1 needs an 8-GPU node."""
    from distributed_ghs_implementation_amd import canonicalize, minimum_spanning_forest
    ora = _oracle()
    fx = load_fixture(name)
    g = canonicalize(fx["num_nodes"], edges=fx["edges"])
    r = minimum_spanning_forest(g, devices=[0])
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(r.in_mst, ref_in.astype(bool))
    assert r.total_weight == ref_tw == fx["expected_total_weight"] and r.num_edges == ref_k


def test_multi_gpu_entry_rmat_and_bad_devices(torch_cuda):
    import torch
    from distributed_ghs_implementation_amd import _native, minimum_spanning_forest
    from distributed_ghs_implementation_amd.device import generate_rmat
    ora = _oracle()
    g = generate_rmat(18, 16, seed=1, wseed=2).to_host()
    r = minimum_spanning_forest(g, devices=[0])
    ref_in, ref_tw, _ = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(r.in_mst, ref_in.astype(bool)) and r.total_weight == ref_tw
    with pytest.raises(_native.GHSError) as ei:  # one rank per GPU
        minimum_spanning_forest(g, devices=[0, 0])
    assert ei.value.code == _native.GHS_E_ARG
    with pytest.raises(_native.GHSError) as ei:
        minimum_spanning_forest(g, num_gpus=torch.cuda.device_count() + 1)
    assert ei.value.code == _native.GHS_E_ARG
    # a non-canonical list fails through the multi-GPU entry as well (error byte of the exchange)
    from distributed_ghs_implementation_amd.graph import CanonicalGraph
    bad = CanonicalGraph(g.n, g.u.copy(), g.v.copy(), g.w)
    bad.v[g.m // 2] = bad.u[g.m // 2]
    with pytest.raises(_native.GHSError) as ei:
        minimum_spanning_forest(bad, devices=[0])
    assert ei.value.code == _native.GHS_E_NONCANON


def test_cli_generator_and_multi_gpu_flag(tmp_path, torch_cuda):
    import json
    from distributed_ghs_implementation_amd.__main__ import main
    out = tmp_path / "r.json"
    assert main(["--generator", "rmat", "--scale", "12", "--gpus", "1", "--output", str(out), "--check", "--quiet"]) == 0
    res = json.load(open(out))
    ora = _oracle()
    n, u, v, w = ora.rmat_canonical(12, 16, 1, 2)
    _, ref_tw, ref_k = ora.kruskal_c(n, u, v, w)
    assert res["total_weight"] == ref_tw and res["num_edges"] == ref_k


@pytest.mark.parametrize("graph", ["rmat", "rmat20", "ties", "forest", "readme", "grid", "grid-gradient"])
@pytest.mark.parametrize("levels", [None, 1])
@pytest.mark.parametrize("mode", ["every", "first"])
def test_bucketed_rounds_vs_oracle(graph, levels, mode, torch_cuda):
    """Bucketed rounds (k_bucket groups the live edges by target bucket, k_bmin takes every
    fragment's minimum in LDS and hooks it; mutual pairs resolved by the jump) forced onto every
    round of every graph kind (GHS_OPT_BUCKETED), or onto every level's first round
    (GHS_OPT_BUCKETED_FIRST; past level 0 the giant fragment's candidates are reduced per block
    and hooked by k_giant_hook): the oracle's MSF and totals, the same flags as the unbucketed
    rounds, and pass_flags says they ran."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST
    ora = _oracle()
    e = _test_graph(graph)
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    kw = {} if levels is None else {"max_levels": levels}
    opt = _native.OPT_BUCKETED if mode == "every" else _native.OPT_BUCKETED_FIRST
    on = DeviceMST(e, config=_native.make_config(options=opt, **kw))
    res, _ = on.run()
    assert res.pass_flags & 1
    assert np.array_equal(on.in_mst_host(), ref_in.astype(bool))
    assert (res.total_weight, res.num_mst_edges) == (ref_tw, ref_k)
    res2, _ = on.run()  # repeat on the same workspace
    assert (res2.total_weight, res2.num_mst_edges) == (ref_tw, ref_k)
    off = DeviceMST(e, config=_native.make_config(options=_native.OPT_NO_BUCKETED, **kw))
    res0, _ = off.run()
    assert not res0.pass_flags & 1
    assert np.array_equal(off.in_mst_host(), ref_in.astype(bool))


@pytest.mark.parametrize("k,mode", [(2048, 0), (2048, 1), (1500, 0)])
def test_bucketed_auto_on_lattices(k, mode, torch_cuda):
    """The default path finds lattices lattice-like (the plan's span sample: bucketed level-0
    rounds) and R-MAT not (bucketed first rounds of every level, the giant excluded past level 0);
    grids large enough for bucketed rounds past the first (>= 2^20 active fragments) and the
    R-MAT graph match the oracle."""
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_grid, generate_rmat
    ora = _oracle()
    e = generate_grid(k, mode)
    eng = DeviceMST(e)
    res, stats = eng.run()
    assert res.pass_flags & 1 and res.pass_flags & 2
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(eng.in_mst_host(), ref_in.astype(bool))
    assert (res.total_weight, res.num_mst_edges) == (ref_tw, ref_k) and ref_k == g.n - 1
    r = generate_rmat(16, 16, seed=1, wseed=2)
    eng_r = DeviceMST(r)
    res_r, _ = eng_r.run()
    assert res_r.pass_flags & 1 and not res_r.pass_flags & 2
    h = r.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(h.n, h.u, h.v, h.w)
    assert np.array_equal(eng_r.in_mst_host(), ref_in.astype(bool))
    assert (res_r.total_weight, res_r.num_mst_edges) == (ref_tw, ref_k)


@pytest.mark.parametrize("k,mode,extra", [(3000, 0, 0), (3000, 1, 0), (2900, 0, 64)])
def test_windowed_round0_vs_oracle(k, mode, extra, torch_cuda):
    """Level 0 round 0 of a lattice-like solve with >= 2^23 vertices runs windowed (k_wmin over the
    level-0 edge list's run of two buckets, no records). `extra` lightest edges spanning many
    buckets set k_select's span flag, and the round falls back to k_bucket / k_bmin on the device.
    Both match the oracle, as does the record path forced by GHS_OPT_NO_WINDOW."""
    from distributed_ghs_implementation_amd import _native, canonicalize
    from distributed_ghs_implementation_amd.device import DeviceEdges, DeviceMST, generate_grid
    ora = _oracle()
    e = generate_grid(k, mode)
    if extra:
        g = e.to_host()
        rng = np.random.default_rng(7)
        u = rng.integers(0, g.n // 2, extra)
        v = u + rng.integers(g.n // 4, g.n // 2, extra)
        w = rng.integers(0, 16, extra)  # the lightest weights: level-0 edges
        e = DeviceEdges.from_host(canonicalize(g.n, u=np.concatenate([g.u, u]), v=np.concatenate([g.v, v]),
                                               w=np.concatenate([g.w, w])))
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    for opt in (0, _native.OPT_NO_WINDOW):
        eng = DeviceMST(e, config=_native.make_config(options=opt) if opt else None)
        res, _ = eng.run()
        assert res.pass_flags & 1 and res.pass_flags & 2  # lattice-like, bucketed level-0 rounds
        # pass_flags bit 2: the windowed round ran (not with long edges: k_select's span flag)
        assert bool(res.pass_flags & _native.PASS_WINDOWED) == (opt == 0 and extra == 0)
        assert np.array_equal(eng.in_mst_host(), ref_in.astype(bool))
        assert (res.total_weight, res.num_mst_edges) == (ref_tw, ref_k)


@pytest.mark.parametrize("graph", ["rmat", "rmat20", "ties", "forest", "readme", "grid", "grid-gradient"])
@pytest.mark.parametrize("levels", [None, 1])
@pytest.mark.parametrize("opt", ["default", "bucketed", "first"])
def test_lds_tail_vs_oracle(graph, levels, opt, torch_cuda):
    """The LDS tail (k_tail_*: a level's rounds once its active fragments fit LDS — dense fragment
    ids, 12-byte records, per-block LDS minima, hooks and pointer jumping in LDS): the oracle's MSF
    and totals on every graph kind and level plan, with the per-round kernels before it either
    unbucketed or bucketed; the same flags as with the tail off (GHS_OPT_NO_TAIL); the round stats
    add up (hooks = MSF edges) and pass_flags bit 3 says the tail ran."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST
    ora = _oracle()
    e = _test_graph(graph)
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    kw = {} if levels is None else {"max_levels": levels}
    base = {"default": 0, "bucketed": _native.OPT_BUCKETED, "first": _native.OPT_BUCKETED_FIRST}[opt]
    on = DeviceMST(e, config=_native.make_config(options=base, **kw))
    for _ in range(2):  # twice on the same workspace
        res, stats = on.run()
        assert np.array_equal(on.in_mst_host(), ref_in.astype(bool))
        assert (res.total_weight, res.num_mst_edges) == (ref_tw, ref_k)
        assert sum(st["hooks"] for st in stats) == ref_k
    off = DeviceMST(e, config=_native.make_config(options=base | _native.OPT_NO_TAIL, **kw))
    res0, stats0 = off.run()
    assert not res0.pass_flags & _native.PASS_TAIL
    assert np.array_equal(off.in_mst_host(), ref_in.astype(bool))
    assert res0.rounds == res.rounds  # the tail runs the same Boruvka rounds
    # the tail takes over a level at its first round past round 0 that starts with 2..TAIL_MAX
    # active fragments (per the per-round path's stats)
    st0 = list(stats0)
    eligible = any(0 < i and st0[i - 1]["level"] == st["level"] and 2 <= st["active_components"] <= 12288
                   for i, st in enumerate(st0))
    assert bool(res.pass_flags & _native.PASS_TAIL) == eligible, (graph, st0)


@pytest.mark.parametrize("graph", ["rmat", "rmat20", "ties", "forest", "readme", "grid", "grid-gradient"])
@pytest.mark.parametrize("opt", ["default", "no_tail", "bucketed"])
def test_report_totals_match_ordered_counters(graph, opt, torch_cuda):
    """VERDICT r04 #4 / ADVICE r04: the running totals the host takes from each level's last round
    report (a checksum-validated pinned slot) equal a stream-ordered copy of the device counters made
    behind the level's last kernel (GHS_OPT_CHECK_TOTALS: the library compares them at the end of
    EVERY level and fails with GHS_E_STATE if they differ), on the tail and non-tail paths; the
    solve's totals then come from that copy and equal the oracle's."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST
    ora = _oracle()
    e = _test_graph(graph)
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    base = {"default": 0, "no_tail": _native.OPT_NO_TAIL, "bucketed": _native.OPT_BUCKETED}[opt]
    for levels in (None, 1):
        kw = {} if levels is None else {"max_levels": levels}
        eng = DeviceMST(e, config=_native.make_config(options=base | _native.OPT_CHECK_TOTALS, **kw))
        for _ in range(2):
            res, _ = eng.run()
            assert np.array_equal(eng.in_mst_host(), ref_in.astype(bool))
            assert (res.total_weight, res.num_mst_edges) == (ref_tw, ref_k)
    assert _native.slot_retries() >= 0


@pytest.mark.parametrize("seed,n,m,wmax", [(21, 300, 2000, 1), (22, 12000, 40000, 3), (23, 13000, 26000, 100),
                                           (24, 40000, 400000, 0), (25, 200000, 300000, 7)])
def test_lds_tail_tie_heavy_and_sizes(seed, n, m, wmax, torch_cuda):
    """Tie-heavy random multigraphs around the tail's capacity (12288 dense fragments; graphs whose
    first explicit round has just fewer or more fragments than that), all-equal weights: the
    strict (w, eid) order decides every tie exactly as Kruskal."""
    from distributed_ghs_implementation_amd import canonicalize
    from distributed_ghs_implementation_amd.device import DeviceEdges, DeviceMST
    ora = _oracle()
    rng = np.random.default_rng(seed)
    cg = canonicalize(n, u=rng.integers(0, n, m), v=rng.integers(0, n, m), w=rng.integers(0, wmax + 1, m))
    e = DeviceEdges.from_host(cg)
    g = e.to_host()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    for levels in (None, 1):
        from distributed_ghs_implementation_amd import _native
        eng = DeviceMST(e, config=_native.make_config(**({} if levels is None else {"max_levels": levels})))
        res, _ = eng.run()
        assert np.array_equal(eng.in_mst_host(), ref_in.astype(bool))
        assert (res.total_weight, res.num_mst_edges) == (ref_tw, ref_k)


@pytest.mark.parametrize("lo,hi,cap", [(0, 0, 1), (0, 1000, None), (3, 997, None), (0, 100000, 5000), (12345, 90001, 20000)])
def test_flags_to_eids(lo, hi, cap, torch_cuda):
    """ABI 8 ghs_flags_to_eids (the device-side compaction a rank's MSF slice is gathered in):
    the ascending ids of the flagged edges of [lo, hi), as torch.nonzero would give them; a
    capacity below the flagged count is refused (GHS_E_NOMEM) without writing."""
    torch = torch_cuda
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import flags_to_eids
    g = torch.Generator().manual_seed(lo + hi)
    flags = (torch.rand(100001, generator=g) < 0.03).to(torch.uint8).cuda()
    want = torch.nonzero(flags[lo:hi]).flatten().cpu() + lo
    got = flags_to_eids(flags, lo, hi, cap)
    assert torch.equal(got.cpu(), want)
    if want.numel() > 1:
        with pytest.raises(_native.GHSError) as ei:
            flags_to_eids(flags, lo, hi, want.numel() - 1)
        assert ei.value.code == _native.GHS_E_NOMEM
