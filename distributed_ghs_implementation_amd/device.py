"""Device-resident pipeline (torch supplies device memory and the stream; HIP does the work).

    edges = generate_rmat(24)                    # canonical u, v, w in HBM (BASELINE config 3)
    eng = DeviceMST(edges)                       # workspace allocated once
    res, stats = eng.run()                       # canonical edges -> in_mst flags + weight

`DeviceMST.run()` is the timed unit of bench.py: from the device-resident canonical edge list to
the in_mst flags and total weight (BASELINE.md "Definitions") — validation, the weight-level
plan, every level's filter + arc build, and all Boruvka rounds. Nothing falls back to the CPU:
without the HIP library or a GPU the constructors raise.
"""
import ctypes

import torch

from . import _native


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else ctypes.c_void_p(0)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class DeviceEdges:
    """Canonical edge list in HBM: n, u/v/w as int32 tensors holding uint32 bit patterns. `off`
    (ABI 9, optional): the CSR row offsets of the same list (n + 1 entries, `with_csr()`); an
    engine built with csr=True streams (off, v, w) — 8 B per edge instead of 12 — and u may then
    be dropped (`csr_only()`)."""

    def __init__(self, n, u, v, w, off=None):
        self.n = int(n)
        self.u, self.v, self.w = u, v, w
        self.off = off

    @property
    def m(self):
        return int(self.v.numel())

    def with_csr(self):
        """Add the CSR row offsets (built on the device from the sorted u)."""
        if self.off is None:
            L = _native.load()
            off = torch.empty(self.n + 1, dtype=torch.int32, device=self.device)
            _native.check(L.ghs_csr_offsets(self.n, self.m, _ptr(self.u), _ptr(off), _stream()))
            self.off = off
        return self

    def csr_only(self):
        """The CSR form alone (u released): off, v, w."""
        self.with_csr()
        return DeviceEdges(self.n, None, self.v, self.w, self.off)

    @property
    def device(self):
        return self.v.device

    @classmethod
    def from_host(cls, graph, device="cuda"):
        """CanonicalGraph (numpy) -> device tensors (H2D copy)."""
        def dev(a):
            return torch.from_numpy(a.view("int32").copy()).to(device)
        return cls(graph.n, dev(graph.u), dev(graph.v), dev(graph.w))

    def u_host(self):
        """u as a host uint32 array (expanded from the offsets for a CSR-only list)."""
        import numpy as np
        if self.u is not None:
            return self.u.cpu().numpy().view("uint32")
        off = self.off.cpu().numpy().view("uint32").astype(np.int64)
        return np.repeat(np.arange(self.n, dtype=np.uint32), np.diff(off))

    def to_host(self):
        from .graph import CanonicalGraph
        return CanonicalGraph(self.n, self.u_host(), self.v.cpu().numpy().view("uint32"),
                              self.w.cpu().numpy().view("uint32"))


def generate_rmat(scale, edgefactor=16, seed=1, wseed=2, device="cuda"):
    """R-MAT (Graph500 A,B,C,D = .57,.19,.19,.05), self-loops dropped, de-duplicated, canonical,
    unique hashed weights — generated and sorted on the GPU."""
    L = _native.load()
    _native.require_gpu()
    T = edgefactor << scale
    dev = torch.device(device)
    u = torch.empty(T, dtype=torch.int32, device=dev)
    v = torch.empty(T, dtype=torch.int32, device=dev)
    w = torch.empty(T, dtype=torch.int32, device=dev)
    tb = L.ghs_rmat_temp_bytes(scale, edgefactor)
    tmp = torch.empty(tb, dtype=torch.uint8, device=dev)
    m = ctypes.c_uint64(0)
    _native.check(L.ghs_rmat_generate(scale, edgefactor, seed, wseed, _ptr(u), _ptr(v), _ptr(w), ctypes.byref(m),
                                      _ptr(tmp), tb, _stream()))
    del tmp
    mm = m.value
    # views of the first m entries (the buffers hold T >= m; at edgefactor 16 m is ~97% of T, so
    # keeping the tail is cheaper than copying 12 B per edge into exact-size tensors)
    return DeviceEdges(1 << scale, u[:mm], v[:mm], w[:mm])


def generate_grid(k, mode=0, wseed=2, device="cuda"):
    """k x k grid graph (right + down edges), canonical; mode 1 = gradient ("road-like") weights."""
    L = _native.load()
    _native.require_gpu()
    dev = torch.device(device)
    m = 2 * k * (k - 1) if k >= 2 else 0
    u = torch.empty(m, dtype=torch.int32, device=dev)
    v = torch.empty(m, dtype=torch.int32, device=dev)
    w = torch.empty(m, dtype=torch.int32, device=dev)
    _native.check(L.ghs_grid_generate(k, mode, wseed, _ptr(u), _ptr(v), _ptr(w), _stream()))
    return DeviceEdges(k * k, u, v, w)


# The ranks' edge ranges are balanced by a cost density over the canonical list instead of by edge
# count: c(x) = 1 + RANGE_BETA * (1 - x) at relative position x = e / m. A canonical edge is stored at
# its smaller end, so the list's early edges have small u and their heavier ends spread over the
# whole vertex range: rank 0's k_filter probes reach all of the giant bitmap (8 MiB at s26, beyond
# one XCD's L2) and the last rank's only its top part — R-MAT s26 x 8 with equal counts ran k_filter
# 1.70 ms on rank 0 against 1.16 on rank 7 (profiles/r05/final/emu_s26_w8_per_rank.txt). The same
# closed form is in csrc/multi.hip (ghs_mst_multi / ghs_mst_emulated). beta = 0.2 measured best over
# {0, 0.2, 0.4} on the s26 x 8 emulation: slowest rank's kernels 6.46 -> 6.08 ms (profiles/r06/).
RANGE_BETA = 0.2


def range_split(m, k, world, beta=None):
    """The first edge of rank k's range: F(x_k) = k / world * F(1) for F(x) = x + beta (x - x^2 / 2),
    4-aligned (the 16-byte vector loads of the level pass stay aligned)."""
    import math
    b = RANGE_BETA if beta is None else float(beta)
    if k <= 0:
        return 0
    if k >= world:
        return m
    if b == 0.0:
        return ((m * k) // world) & ~3
    t = k / world * (1.0 + b / 2.0)
    x = ((1.0 + b) - math.sqrt((1.0 + b) ** 2 - 2.0 * b * t)) / b
    return min(m, int(x * m)) & ~3


def edge_range(m, rank, world, beta=None):
    """Contiguous canonical-edge range owned by `rank` (range_split: cost-balanced, 4-aligned)."""
    lo = range_split(m, rank, world, beta)
    hi = m if rank == world - 1 else range_split(m, rank + 1, world, beta)
    return lo, max(lo, hi)


class DeviceMST:
    """Preallocated single-GPU engine for one DeviceEdges graph (or one rank's edge range).
    csr=None: the CSR entry (ghs_mst_device_csr) whenever the edges carry offsets."""

    def __init__(self, edges, e_lo=0, e_hi=None, config=None, csr=None):
        L = self.L = _native.load()
        _native.require_gpu()
        self.edges = edges
        n, m = edges.n, edges.m
        self.e_lo = int(e_lo)
        self.e_hi = m if e_hi is None else int(e_hi)
        self.config = config if config is not None else _native.make_config()
        dev = edges.device
        self.ws_bytes = int(L.ghs_workspace_bytes(n, m, self.e_hi - self.e_lo))
        self.ws = torch.empty(max(self.ws_bytes, 256), dtype=torch.uint8, device=dev)
        self.in_mst = torch.zeros(max(m, 1), dtype=torch.uint8, device=dev)
        self.csr = (edges.off is not None) if csr is None else bool(csr)
        if self.csr:
            edges.with_csr()

    def run(self):
        """Canonical edges (HBM) -> in_mst flags + totals. Returns (Result, [round stats])."""
        e = self.edges
        res = _native.Result()
        stats = (_native.RoundStats * _native.GHS_MAX_ROUND_STATS)()
        if self.csr:
            _native.check(self.L.ghs_mst_device_csr(e.n, e.m, _ptr(e.off), _ptr(e.u), _ptr(e.v), _ptr(e.w),
                                                    ctypes.byref(self.config), _ptr(self.ws), self.ws_bytes,
                                                    _ptr(self.in_mst), _stream(), ctypes.byref(res), stats))
        else:
            _native.check(self.L.ghs_mst_device(e.n, e.m, _ptr(e.u), _ptr(e.v), _ptr(e.w), ctypes.byref(self.config),
                                                _ptr(self.ws), self.ws_bytes, _ptr(self.in_mst), _stream(),
                                                ctypes.byref(res), stats))
        return res, _native.RoundStatsList(stats, res.num_stats)

    def in_mst_host(self):
        return self.in_mst[: self.edges.m].cpu().numpy().astype(bool)


def flags_to_eids(in_mst, lo, hi, capacity=None):
    """The edge ids e in [lo, hi) with in_mst[e] != 0, ascending, as an int64 device tensor — on the
    device (ghs_flags_to_eids: a flagged select), never through torch.nonzero (whose first call per
    process loaded for ~100 s with 4 ranks sharing one GPU, the gloo rehearsal's stall)."""
    lo, hi = int(lo), int(hi)
    cap = (hi - lo) if capacity is None else int(capacity)
    out = torch.empty(max(cap, 1), dtype=torch.int32, device=in_mst.device)
    cnt = ctypes.c_uint64(0)
    _native.check(_native.load().ghs_flags_to_eids(_ptr(in_mst), lo, hi, _ptr(out), cap, ctypes.byref(cnt), _stream()))
    return out[: cnt.value].to(torch.int64)


def emulated_mst(edges, num_ranks, config=None):
    """The multi-rank loop of an N-GPU solve (ghs_solver_run, every rank its own solver, stream
    and host thread over its edge range) with all N ranks on THIS device and in-process
    collectives (ghs_mst_emulated) — the N-rank protocol checked on one GPU. Returns
    (Result, [round stats], in_mst uint8 tensor of m flags)."""
    L = _native.load()
    _native.require_gpu()
    cfg = config if config is not None else _native.make_config()
    in_mst = torch.zeros(max(edges.m, 1), dtype=torch.uint8, device=edges.device)
    torch.cuda.synchronize(edges.device)  # the rank streams read u/v/w written on torch's stream
    res = _native.Result()
    stats = (_native.RoundStats * _native.GHS_MAX_ROUND_STATS)()
    _native.check(L.ghs_mst_emulated(edges.n, edges.m, _ptr(edges.u), _ptr(edges.v), _ptr(edges.w), int(num_ranks),
                                     ctypes.byref(cfg), _ptr(in_mst), ctypes.byref(res), stats))
    return res, _native.RoundStatsList(stats, res.num_stats), in_mst[: edges.m]
