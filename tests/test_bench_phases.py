"""bench.py's N>1 failure agreement on CPU (gloo, world 2): a phase that raises on ONE rank ends
every rank with PhaseFailed naming the phase and the failing rank — no rank is left waiting in the
next collective (the N=4 rehearsal went silent)."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import datetime

    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    out = []
    try:
        assert bench.agreed("ok phase", lambda: rank * 10, rank, world, dist, "cpu") == rank * 10

        def bad():
            if rank == 1:
                raise ValueError("boom")
            return 1

        try:
            bench.agreed("bad phase", bad, rank, world, dist, "cpu")
            out.append("no failure")
        except bench.PhaseFailed as ex:
            out.append(str(ex))
    finally:
        dist.destroy_process_group()
    q.put((rank, out))


def test_phase_failure_ends_every_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    for r in range(2):
        assert len(got[r]) == 1 and "bad phase" in got[r][0] and "[1]" in got[r][0], got
    assert "boom" in got[1][0]
