"""The multi-rank orchestration (distributed.run_rounds + edge_range partition + all-reduce
MIN) on CPU with the gloo backend, world_size 2 and 3, with one and with several weight levels.
The per-rank compute is the oracle's numpy stepper (oracle/boruvka_steps.py) standing in for the
HIP stepper, including the owner-computes CONNECT exchange of a level's first round (hook_local,
int32 MAX all-reduce, unpack_hook: distributed.run_rounds drives it exactly as for HipStepper)
and the reduce-scatter CONNECT of the library loop (hook_slots, reduce-scatter MIN, hook_owner,
pair all-gather, apply_hooks, SUM of the partial totals; distributed.TorchRs over gloo).
The totals must equal canonical Kruskal on every rank and the OR of the ranks' MSF flags must
equal Kruskal's edge set (an owner-computed hook marks its edge on the owning rank only)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import load_fixture


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, u, v, w, thr, out, owner_hooks, use_rs):
    import torch.distributed as dist

    from distributed_ghs_implementation_amd.device import edge_range
    from distributed_ghs_implementation_amd.distributed import TorchRs, run_rounds
    from oracle.boruvka_steps import CpuStepper
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = edge_range(len(u), rank, world)
    st = CpuStepper(n, u, v, w, lo, hi, thr, ranks=world if owner_hooks else 1)
    st.rs = use_rs

    def ar(t):
        dist.all_reduce(t, op=dist.ReduceOp.MIN)

    def ar_max(t):
        dist.all_reduce(t, op=dist.ReduceOp.MAX)

    rounds = run_rounds(st, ar, allreduce_max=ar_max, rs=TorchRs() if use_rs else None)
    total, count = st.finish()
    out[rank] = (st.in_mst.tolist(), total, count, rounds, st.hooks_exchanged)
    dist.barrier()
    dist.destroy_process_group()


def _run(world, n, u, v, w, thr, owner_hooks=True, use_rs=False):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, u, v, w, thr, out, owner_hooks, use_rs), nprocs=world,
             join=True)
    return dict(out)


@pytest.mark.parametrize("world,name,levels,owner_hooks,use_rs", [
    (2, "ties_4.json", 1, True, False), (2, "cgf_n1000_p001.json", 3, True, False),
    (3, "ties_2.json", 2, True, False), (2, "ties_5.json", 3, True, False), (2, "ties_5.json", 3, False, False),
    (2, "cgf_n1000_p001.json", 3, True, True), (3, "ties_2.json", 2, True, True), (3, "ties_5.json", 3, True, True)])
def test_gloo_ranks_match_kruskal(world, name, levels, owner_hooks, use_rs):
    from oracle import oracle
    fx = load_fixture(name)
    n = fx["num_nodes"]
    e = np.array(fx["edges"], dtype=np.int64).reshape(-1, 3)
    u, v, w = oracle.canonicalize_c(n, e[:, 0], e[:, 1], e[:, 2])
    ref_in, ref_tw, ref_k = oracle.kruskal_c(n, u, v, w)
    qs = np.quantile(w, np.linspace(0, 1, levels + 1)[1:-1]).astype(np.int64).tolist() if levels > 1 else []
    thr = [0] + sorted(set(int(q) + 1 for q in qs)) + [1 << 32]
    out = _run(world, n, u, v, w, thr, owner_hooks, use_rs)
    assert len(out) == world
    flags = np.zeros(len(u), np.uint8)
    for rank in range(world):
        in_mst, total, count, rounds, exchanged = out[rank]
        flags |= np.array(in_mst, np.uint8)
        assert total == ref_tw == fx["expected_total_weight"]
        assert count == ref_k
        assert rounds <= (len(thr) - 1) * (int(np.ceil(np.log2(max(n, 2)))) + 2)
        assert (exchanged > 0) == owner_hooks  # the int32 MAX hook exchange really ran
        if not owner_hooks:  # fragment-form hooks on every rank: each rank holds the whole MSF
            assert np.array_equal(np.array(in_mst, np.uint8), ref_in)
    assert np.array_equal(flags, ref_in)


def test_failure_watch_keys_are_per_instance():
    """a failure key left in the store by one DistributedMST's failed solve must not
    cancel another instance's solve (a retry, another group on the same store). The key carries the
    instance's nonce (its RCCL unique id) and the solve index."""
    import threading

    import torch.distributed as dist
    from distributed_ghs_implementation_amd.distributed import DistributedMST, _FailureWatch

    class Stepper:
        def __init__(self):
            self.cancelled = threading.Event()

        def cancel(self):
            self.cancelled.set()

    store = dist.HashStore()
    a, b = DistributedMST.__new__(DistributedMST), DistributedMST.__new__(DistributedMST)
    a._nonce, b._nonce = "aaaa", "bbbb"
    a._solves = b._solves = 1
    assert a._failure_key() != b._failure_key()
    # instance a fails: its key is set
    wa = _FailureWatch(store, a._failure_key(), Stepper())
    wa.report()
    wa.stop()
    # instance b (same solve index, same store) is NOT cancelled ...
    sb = Stepper()
    wb = _FailureWatch(store, b._failure_key(), sb, period=0.005)
    assert not sb.cancelled.wait(0.1)
    # ... but a peer of b reporting b's key cancels it
    _FailureWatch(store, b._failure_key(), Stepper()).report()
    assert sb.cancelled.wait(2.0)
    wb.stop()
