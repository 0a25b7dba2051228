"""Worker of tests/test_gpu_rccl_stub.py (runs in its own process: it loads the TEST build of the
library, tests/rccl_stub/libghs_mst_rcclstub.so, whose RCCL entry points are the in-process stub of
tests/rccl_stub/nccl_stub.hip). N ranks as N host threads on the box's one GPU, each through the
product's multi-rank entry points exactly as a process per GPU would call them — ghs_comm_init from
one unique id, ghs_solver_create(_csr) over its edge range, ghs_solver_run — so the library's real
COMM_NCCL branches (csrc/multi.hip: the level-open all-gather, the in-place reduce-scatter MIN of a
dense level's opening round, the pairs' in-place all-gather, the SUM / MIN / MAX all-reduces, the
setup agreement) execute at N > 1. Prints one JSON line per case: the OR of the ranks' own-range flags
against the oracle's Kruskal MSF, every rank's totals, and the stub's collective count."""
import ctypes
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
STUB = os.path.join(ROOT, "tests", "rccl_stub")
os.environ["GHS_MST_LIB"] = os.path.join(STUB, "libghs_mst_rcclstub.so")
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributed_ghs_implementation_amd import _native, canonicalize  # noqa: E402
from distributed_ghs_implementation_amd.device import (DeviceEdges, DeviceMST, edge_range, generate_grid,  # noqa: E402
                                                       generate_rmat)
from distributed_ghs_implementation_amd.distributed import HipStepper  # noqa: E402
from oracle import oracle  # noqa: E402


def stub_calls():
    return ctypes.CDLL(os.path.join(STUB, "libnccl_stub.so")).nccl_stub_calls()


def graph(kind):
    if kind == "rmat12":
        return generate_rmat(12, 16, seed=1, wseed=2)
    if kind == "rmat15":
        return generate_rmat(15, 16, seed=3, wseed=4)
    if kind == "grid":
        return generate_grid(257, 0)
    if kind == "grid-gradient":
        return generate_grid(129, 1)
    if kind == "readme":  # 9 edges: most of 8 ranks own none
        return DeviceEdges.from_host(canonicalize(6, edges=[(0, 1, 1), (0, 2, 4), (1, 2, 2), (1, 3, 5), (2, 3, 3),
                                                            (2, 4, 7), (3, 4, 6), (3, 5, 8), (4, 5, 9)]))
    if kind == "ties":
        rng = np.random.default_rng(12)
        n, m = 3000, 20000
        return DeviceEdges.from_host(canonicalize(n, u=rng.integers(0, n, m), v=rng.integers(0, n, m),
                                                  w=rng.integers(0, 3, m)))
    if kind == "forest":
        rng = np.random.default_rng(13)
        n, m = 20000, 12000
        return DeviceEdges.from_host(canonicalize(n, u=rng.integers(0, n, m), v=rng.integers(0, n, m),
                                                  w=rng.integers(0, 50, m)))
    raise ValueError(kind)


def solve(e, N, options=0, fault_rank=0, fault_round=0):
    uid = _native.comm_unique_id()
    cfg = _native.make_config(num_ranks=N, options=options, fault_rank=fault_rank, fault_round=fault_round)
    engines = [DeviceMST(e, *edge_range(e.m, r, N), config=cfg) for r in range(N)]
    for x in engines:
        x.in_mst.fill_(7)  # a sentinel outside each rank's own range: never written
    streams = [torch.cuda.Stream() for _ in range(N)]
    torch.cuda.synchronize()
    out = [None] * N

    def rank(r):
        try:
            with torch.cuda.stream(streams[r]):
                st = HipStepper(engines[r])
                comm = _native.Comm(N, r, uid)
                L = engines[r].L
                rc = L.ghs_solver_run(st.h, comm.h)
                if rc < 0:
                    out[r] = {"rc": int(rc), "err": L.ghs_last_error().decode()}
                else:
                    res, _ = st.finish()
                    out[r] = {"rc": 0, "weight": int(res.total_weight), "edges": int(res.num_mst_edges)}
                streams[r].synchronize()
                st.close()
                comm.close()
        except Exception as ex:  # noqa: BLE001
            out[r] = {"rc": -100, "err": repr(ex)}

    th = [threading.Thread(target=rank, args=(r,)) for r in range(N)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    hung = [r for r, t in enumerate(th) if t.is_alive()]
    torch.cuda.synchronize()
    flags = torch.empty(max(e.m, 1), dtype=torch.uint8, device="cuda")[: e.m]
    sentinel_ok = True
    for x in engines:
        flags[x.e_lo:x.e_hi] = x.in_mst[x.e_lo:x.e_hi]
        sentinel_ok &= bool((x.in_mst[: x.e_lo] == 7).all()) and bool((x.in_mst[x.e_hi: e.m] == 7).all())
    return out, flags, sentinel_ok, hung


def main():
    cases = json.loads(sys.argv[1])
    for c in cases:
        e = graph(c["graph"])
        if c.get("csr"):
            e = e.csr_only()
        g = e.to_host()
        before = stub_calls()
        out, flags, sentinel_ok, hung = solve(e, c["N"], c.get("options", 0), c.get("fault_rank", 0),
                                              c.get("fault_round", 0))
        ref_in, ref_tw, ref_k = oracle.kruskal_c(g.n, g.u, g.v, g.w)
        rec = dict(c, ranks=out, hung=hung, sentinel_ok=sentinel_ok, collectives=stub_calls() - before,
                   oracle=[int(ref_tw), int(ref_k)])
        if all(o and o["rc"] == 0 for o in out):
            rec["flags_match"] = bool(np.array_equal(flags.cpu().numpy().astype(bool), ref_in.astype(bool)))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
