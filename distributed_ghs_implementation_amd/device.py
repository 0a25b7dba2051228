"""Device-resident pipeline (torch supplies device memory and the stream; HIP does the work).

    edges = generate_rmat(24)                    # canonical u, v, w in HBM (BASELINE config 3)
    eng = DeviceMST(edges)                       # arc + workspace buffers, allocated once
    res = eng.run()                              # canonical edges -> in_mst flags + weight

`DeviceMST.run()` is the timed unit of bench.py: from the device-resident canonical edge list to
the in_mst flags and total weight (BASELINE.md "Definitions"): symmetric arc build (radix sort by
source) + the Boruvka rounds. Nothing falls back to the CPU: without the HIP library or a GPU the
constructors raise.
"""
import ctypes

import torch

from . import _native


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else ctypes.c_void_p(0)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class DeviceEdges:
    """Canonical edge list in HBM: n, u/v/w as int32 tensors holding uint32 bit patterns."""

    def __init__(self, n, u, v, w):
        self.n = int(n)
        self.u, self.v, self.w = u, v, w

    @property
    def m(self):
        return int(self.u.numel())

    @property
    def device(self):
        return self.u.device

    @classmethod
    def from_host(cls, graph, device="cuda"):
        """CanonicalGraph (numpy) -> device tensors (H2D copy)."""
        def dev(a):
            return torch.from_numpy(a.view("int32").copy()).to(device)
        return cls(graph.n, dev(graph.u), dev(graph.v), dev(graph.w))

    def to_host(self):
        from .graph import CanonicalGraph
        return CanonicalGraph(self.n, self.u.cpu().numpy().view("uint32"), self.v.cpu().numpy().view("uint32"),
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
    # keep exact-size tensors (clone so the oversize buffers are released)
    return DeviceEdges(1 << scale, u[:mm].clone(), v[:mm].clone(), w[:mm].clone())


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


class DeviceMST:
    """Preallocated single-GPU engine for one DeviceEdges graph (or one rank's source range)."""

    def __init__(self, edges, src_lo=0, src_hi=None):
        L = self.L = _native.load()
        _native.require_gpu()
        self.edges = edges
        n, m = edges.n, edges.m
        self.src_lo = int(src_lo)
        self.src_hi = n if src_hi is None else int(src_hi)
        dev = edges.device
        self.temp_bytes = int(L.ghs_build_arcs_temp_bytes(n, m))
        self.temp = torch.empty(max(self.temp_bytes, 256), dtype=torch.uint8, device=dev)
        cnt = ctypes.c_uint64(0)
        if self.src_lo == 0 and self.src_hi == n:
            cnt.value = 2 * m
        else:
            _native.check(L.ghs_count_arcs_range(n, m, _ptr(edges.u), _ptr(edges.v), self.src_lo, self.src_hi,
                                                 _ptr(self.temp), self.temp_bytes, _stream(), ctypes.byref(cnt)))
        self.num_arcs = int(cnt.value)
        A = max(self.num_arcs, 1)
        self.asrc = torch.empty(A, dtype=torch.int32, device=dev)
        self.adst = torch.empty(A, dtype=torch.int32, device=dev)
        self.akey = torch.empty(A, dtype=torch.int64, device=dev)
        self.ws_bytes = int(L.ghs_workspace_bytes(n, m, self.num_arcs))
        self.ws = torch.empty(max(self.ws_bytes, 256), dtype=torch.uint8, device=dev)
        self.in_mst = torch.zeros(max(m, 1), dtype=torch.uint8, device=dev)

    def build_arcs(self):
        e = self.edges
        got = ctypes.c_uint64(0)
        _native.check(self.L.ghs_build_arcs_range(e.n, e.m, _ptr(e.u), _ptr(e.v), _ptr(e.w), self.src_lo, self.src_hi,
                                                  _ptr(self.asrc), _ptr(self.adst), _ptr(self.akey), self.num_arcs,
                                                  _ptr(self.temp), self.temp_bytes, _stream(), ctypes.byref(got)))
        if got.value != self.num_arcs:
            raise _native.GHSError(_native.GHS_E_STATE, f"built {got.value} arcs, expected {self.num_arcs}")

    def solve(self):
        """Boruvka rounds on the built arcs -> (Result, [round stats])."""
        e = self.edges
        res = _native.Result()
        stats = (_native.RoundStats * _native.GHS_MAX_ROUND_STATS)()
        _native.check(self.L.ghs_mst_device(e.n, e.m, _ptr(e.u), _ptr(e.v), _ptr(self.asrc), _ptr(self.adst),
                                            _ptr(self.akey), self.num_arcs, _ptr(self.ws), self.ws_bytes,
                                            _ptr(self.in_mst), _stream(), ctypes.byref(res), stats))
        return res, [stats[i].as_dict() for i in range(res.num_stats)]

    def run(self):
        """Canonical edges (HBM) -> in_mst flags + totals. Returns (Result, stats)."""
        self.build_arcs()
        return self.solve()

    def in_mst_host(self):
        return self.in_mst[: self.edges.m].cpu().numpy().astype(bool)
