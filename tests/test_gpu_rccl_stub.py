"""The real RCCL branches of the library's multi-rank loop (csrc/multi.hip COMM_NCCL: ncclAllGather,
the in-place ncclReduceScatter(buf, buf + rank * per, ...), the uint64 / int64 / int32 all-reduces,
the setup agreement) executed at N = 2 ... 8 on the box's ONE GPU. RCCL itself
refuses two ranks on one device, so a TEST build of the library links an in-process RCCL stand-in
(tests/rccl_stub/nccl_stub.hip: NCCL's semantics and in-place rules, the undefined slices of an
in-place reduce-scatter poisoned, mismatched calls failing every rank); the shipped libghs_mst.so
links librccl and is not involved. Each case runs in a worker process (tests/gpu_workers/
rccl_stub_solve.py) with one host thread per rank through ghs_comm_init + ghs_solver_run, and is
checked against the oracle's Kruskal MSF."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB_LIB = os.path.join(ROOT, "tests", "rccl_stub", "libghs_mst_rcclstub.so")

pytestmark = pytest.mark.gpu


def _run(cases, timeout=300):
    if not os.path.exists(STUB_LIB):
        pytest.fail("tests/rccl_stub/libghs_mst_rcclstub.so missing: build it with "
                    "`make -C distributed_ghs_implementation_amd/csrc rcclstub` (__graft_entry__.build())")
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gpu_workers", "rccl_stub_solve.py"),
                        json.dumps(cases)], capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    recs = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(recs) == len(cases), p.stdout[-2000:] + p.stderr[-2000:]
    return recs


CASES = [dict(graph="rmat12", N=2), dict(graph="rmat15", N=3), dict(graph="rmat15", N=8),
         dict(graph="grid", N=4), dict(graph="grid-gradient", N=5), dict(graph="readme", N=8),
         dict(graph="ties", N=4), dict(graph="forest", N=3),
         dict(graph="rmat15", N=4, options=0x2),          # GHS_OPT_NO_DENSE: int64 MIN + int32 MAX all-reduces
         dict(graph="rmat15", N=4, csr=True),             # the CSR form (ghs_solver_create_csr)
         dict(graph="grid", N=8, csr=True)]


def test_rccl_branches_match_oracle():
    for r in _run(CASES):
        ranks = r["ranks"]
        assert all(x["rc"] == 0 for x in ranks), r
        assert not r["hung"] and r["sentinel_ok"], r
        assert r["flags_match"], r
        assert {(x["weight"], x["edges"]) for x in ranks} == {tuple(r["oracle"])}, r
        assert r["collectives"] > 0, r  # the stub's entry points (the COMM_NCCL branches) ran


def test_rccl_branch_mid_solve_failure_fails_every_rank():
    """One rank fails after its first rounds (ghs_config_t.fault_round): it aborts its communicator
    (ncclCommAbort), which ends its peers' collectives — every rank returns an error, none hangs."""
    (r,) = _run([dict(graph="rmat15", N=4, fault_rank=3, fault_round=2)])
    assert not r["hung"], r
    assert all(x["rc"] < 0 for x in r["ranks"]), r
