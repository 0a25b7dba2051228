"""GPU parity of the CSR entry (ABI 9: ghs_mst_device_csr / ghs_solver_create_csr): the canonical
list as row offsets + v + w, u derived on the device from the offsets (csr_tile_rows). Every case
is compared bit-exact with the oracle (canonical Kruskal, oracle/kruskal.c) and with the COO entry
on the same graph; the offsets' validation is checked with malformed inputs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _oracle():
    from oracle import oracle
    return oracle


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _offsets(n, u):
    return np.searchsorted(np.asarray(u, dtype=np.int64), np.arange(n + 1), side="left").astype(np.uint32)


def _csr_edges(g, keep_u=False):
    import torch
    from distributed_ghs_implementation_amd.device import DeviceEdges
    e = DeviceEdges.from_host(g)
    off = torch.from_numpy(_offsets(g.n, g.u).view(np.int32).copy()).cuda()
    return DeviceEdges(g.n, e.u if keep_u else None, e.v, e.w, off)


def _solve(e, cfg=None, csr=True):
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST
    eng = DeviceMST(e, config=cfg if cfg is not None else _native.make_config(), csr=csr)
    res, _ = eng.run()
    return eng.in_mst_host(), res


def _check(g, e, cfg=None):
    ora = _oracle()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    got, res = _solve(e, cfg)
    assert np.array_equal(got, ref_in.astype(bool))
    assert res.total_weight == ref_tw and res.num_mst_edges == ref_k
    return got


@pytest.mark.parametrize("keep_u", [False, True])
@pytest.mark.parametrize("seed,n,m,wmax", [(1, 10, 30, 2), (2, 100, 400, 1), (3, 1000, 3000, 3), (4, 5000, 40000, 10),
                                           (5, 20000, 60000, 1000), (6, 3000, 300000, 0), (7, 50000, 20000, 5),
                                           (8, 100000, 1000000, 1 << 31), (9, 2, 1, 7), (10, 1, 0, 1)])
def test_csr_random_tie_graphs_vs_oracle(seed, n, m, wmax, keep_u, torch_cuda):
    from distributed_ghs_implementation_amd import canonicalize
    rng = np.random.default_rng(seed)
    g = canonicalize(n, u=rng.integers(0, n, m), v=rng.integers(0, n, m), w=rng.integers(0, wmax + 1, m))
    _check(g, _csr_edges(g, keep_u))


CONFIGS = [dict(max_levels=1), dict(), dict(max_levels=6, level1_edges_per_vertex=0.25, level_growth=2.0),
           dict(max_levels=16, level1_edges_per_vertex=0.01, level_growth=1.5)]


@pytest.mark.parametrize("keep_u", [False, True])
@pytest.mark.parametrize("cfg", CONFIGS)
@pytest.mark.parametrize("scale", [10, 14, 18])
def test_csr_rmat_vs_oracle_and_coo(scale, cfg, keep_u, torch_cuda):
    """keep_u: both forms resident (bench.py's N = 1 default): k_select streams the CSR form,
    k_filter the COO one."""
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import generate_rmat
    e = generate_rmat(scale, 16, seed=1, wseed=2)
    g = e.to_host()
    c = _native.make_config(**cfg)
    got = _check(g, e.with_csr() if keep_u else e.csr_only(), c)
    coo, _ = _solve(e, c, csr=False)
    assert np.array_equal(got, coo)


@pytest.mark.parametrize("opt", ["BUCKETED", "NO_BUCKETED", "BUCKETED_FIRST", "NO_TAIL", "NO_SEED_RUNS",
                                 "CHECK_TOTALS"])
def test_csr_rmat_forced_paths(opt, torch_cuda):
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import generate_rmat
    e = generate_rmat(16, 16, seed=7, wseed=8)
    g = e.to_host()
    _check(g, e.csr_only(), _native.make_config(options=getattr(_native, "OPT_" + opt)))


@pytest.mark.parametrize("keep_u", [False, True])
@pytest.mark.parametrize("k,mode", [(2, 0), (3, 1), (257, 0), (257, 1), (1024, 0), (1024, 1)])
def test_csr_grid_vs_oracle(k, mode, keep_u, torch_cuda):
    """Lattices: ~2 edges per row (several 64-row windows per tile), the windowed round 0 with
    (keep_u) and without (the sweep form) the canonical u."""
    from distributed_ghs_implementation_amd.device import DeviceEdges, generate_grid
    e = generate_grid(k, mode)
    g = e.to_host()
    e.with_csr()
    ce = DeviceEdges(e.n, e.u if keep_u else None, e.v, e.w, e.off)
    got, res = _solve(ce)
    ora = _oracle()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(got, ref_in.astype(bool)) and res.num_mst_edges == k * k - 1 == ref_k


def _graph(kind):
    from distributed_ghs_implementation_amd import canonicalize
    rng = np.random.default_rng(21)
    if kind == "star":  # one row holds every edge: it spans thousands of tiles
        n = 300000
        return canonicalize(n, u=np.zeros(n - 1, np.int64), v=np.arange(1, n), w=rng.integers(0, 50, n - 1))
    if kind == "sparse_rows":  # long runs of empty rows between the nonempty ones (windows loop)
        n = 2_000_000
        a = np.sort(rng.choice(n - 1, 3000, replace=False))
        return canonicalize(n, u=a, v=a + 1 + rng.integers(0, 5, a.size).clip(max=0), w=rng.integers(0, 9, a.size))
    if kind == "path":  # one edge per row
        n = 200000
        return canonicalize(n, u=np.arange(n - 1), v=np.arange(1, n), w=rng.integers(0, 3, n - 1))
    if kind == "last_rows":  # edges only among the highest vertices (rows 0..n-k empty)
        n = 500000
        u = rng.integers(n - 2000, n, 40000)
        v = rng.integers(n - 2000, n, 40000)
        return canonicalize(n, u=u, v=v, w=rng.integers(0, 100, u.size))
    if kind == "mixed":  # hubs, empty gaps and short rows interleaved
        n = 400000
        hubs = rng.choice(n, 20, replace=False)
        u = np.concatenate([np.repeat(hubs, 5000), rng.integers(0, n, 200000)])
        v = np.concatenate([rng.integers(0, n, 100000), rng.integers(0, n, 200000)])
        return canonicalize(n, u=u, v=v, w=rng.integers(0, 1000, u.size))
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["star", "sparse_rows", "path", "last_rows", "mixed"])
@pytest.mark.parametrize("cfg", [dict(), dict(max_levels=1), dict(max_levels=8, level1_edges_per_vertex=0.05)])
def test_csr_row_shapes_vs_oracle(kind, cfg, torch_cuda):
    from distributed_ghs_implementation_amd import _native
    g = _graph(kind)
    _check(g, _csr_edges(g), _native.make_config(**cfg))


def test_csr_empty_and_isolated(torch_cuda):
    import torch
    from distributed_ghs_implementation_amd.device import DeviceEdges
    for n in (1, 7, 100000):  # no edges at all: every vertex isolated
        off = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
        z = torch.empty(0, dtype=torch.int32, device="cuda")
        got, res = _solve(DeviceEdges(n, None, z, z, off))
        assert got.size == 0 and res.num_mst_edges == 0 and res.total_weight == 0


def test_csr_offsets_builder_matches_searchsorted(torch_cuda):
    from distributed_ghs_implementation_amd.device import generate_rmat
    e = generate_rmat(14, 16, seed=3, wseed=4).with_csr()
    u = e.u.cpu().numpy().view(np.uint32)
    assert np.array_equal(e.off.cpu().numpy().view(np.uint32), _offsets(e.n, u))
    assert np.array_equal(e.csr_only().u_host(), u)


@pytest.mark.parametrize("bad", ["decreasing", "first_nonzero", "last_not_m", "v_not_ascending", "v_equals_u",
                                 "v_out_of_range"])
def test_csr_malformed_rejected(bad, torch_cuda):
    import torch
    from distributed_ghs_implementation_amd import _native, canonicalize
    from distributed_ghs_implementation_amd.device import DeviceEdges, DeviceMST
    rng = np.random.default_rng(5)
    n = 5000
    g = canonicalize(n, u=rng.integers(0, n, 40000), v=rng.integers(0, n, 40000), w=rng.integers(0, 9, 40000))
    off = _offsets(n, g.u).astype(np.int64)
    v = g.v.astype(np.int64).copy()
    r = int(np.argmax(np.diff(off) >= 3))  # a row with >= 3 edges
    if bad == "decreasing":
        off[r + 1], off[r + 2] = off[r + 2], off[r + 1]
        if off[r + 1] == off[r + 2]:
            off[r + 1] += 1
    elif bad == "first_nonzero":
        off[0] = 1
    elif bad == "last_not_m":
        off[n] = g.m - 1
    elif bad == "v_not_ascending":
        v[off[r]], v[off[r] + 1] = v[off[r] + 1], v[off[r]]
    elif bad == "v_equals_u":
        v[off[r]] = r
    elif bad == "v_out_of_range":
        v[off[r + 1] - 1] = n
    t = lambda a: torch.from_numpy(a.astype(np.uint32).view(np.int32).copy()).cuda()
    e = DeviceEdges(n, None, t(v), t(g.w), t(off))
    with pytest.raises(_native.GHSError) as ei:
        DeviceMST(e, csr=True).run()
    assert ei.value.code == _native.GHS_E_NONCANON


@pytest.mark.parametrize("world", [2, 3, 8])
def test_csr_partitioned_ranks_emulated(world, torch_cuda):
    """Rank edge ranges starting inside rows (ghs_solver_create_csr, the stepwise loop with
    emulated collectives): the OR of the ranks' slices is the oracle's MSF."""
    from test_gpu_parity import _emulate_ranks
    from distributed_ghs_implementation_amd.device import generate_rmat
    e = generate_rmat(15, 16, seed=3, wseed=4)
    g = e.to_host()
    flags, totals = _emulate_ranks(e.csr_only(), world, rs=True)
    ora = _oracle()
    ref_in, ref_tw, ref_k = ora.kruskal_c(g.n, g.u, g.v, g.w)
    assert np.array_equal(flags.cpu().numpy().astype(bool), ref_in.astype(bool))
    assert set(totals) == {(ref_tw, ref_k)}


def test_csr_rmat_s24_equals_coo(torch_cuda):
    """BASELINE config 3 at full size: the CSR solve's flags equal the COO solve's (which the
    torch Boruvka checker pins in test_gpu_parity), and the totals match the flags."""
    torch = torch_cuda
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
    e = generate_rmat(24, 16, seed=1, wseed=2)
    a = DeviceMST(e, csr=False)
    ra, _ = a.run()
    fa = a.in_mst[: e.m].clone()
    del a
    torch.cuda.empty_cache()
    c = e.csr_only()
    b = DeviceMST(c)
    rb, _ = b.run()
    assert torch.equal(fa, b.in_mst[: e.m])
    assert (ra.total_weight, ra.num_mst_edges) == (rb.total_weight, rb.num_mst_edges)
    del b
    torch.cuda.empty_cache()
    h = DeviceMST(e.with_csr())  # both forms (bench.py's N = 1 default): CSR k_select, COO k_filter
    rh, _ = h.run()
    assert torch.equal(fa, h.in_mst[: e.m])
    assert (ra.total_weight, ra.num_mst_edges) == (rh.total_weight, rh.num_mst_edges)
    w = e.w.to(torch.int64) & 0xFFFFFFFF
    assert int(w[fa.bool()].sum().item()) == rb.total_weight
