"""Worker of tests/test_gpu_distributed.py (launched by torch.distributed.run, one process per
rank, all sharing the box's one GPU over gloo): the product's multi-GPU driver
(DistributedMST: edge-range partition, level flag MAX exchange, MIN all-reduce of the best
slots, owner-computes hook exchange) end to end across real processes. Rank 0 checks the OR of
the ranks' MSF flags against canonical Kruskal (oracle) and writes a JSON verdict."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def fault(out_path, scale):
    """Mode "fault": rank 1's setup is made to fail (ghs_config_t.fault_rank = 2); every rank must
    raise from the DistributedMST constructor (the setup agreement) instead of hanging."""
    import torch
    import torch.distributed as dist

    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import generate_rmat
    from distributed_ghs_implementation_amd.distributed import DistributedMST
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    e = generate_rmat(scale, 16, seed=1, wseed=2)
    code = 0
    try:
        DistributedMST(e, rank, world, config=_native.make_config(num_ranks=world, fault_rank=2))
    except _native.GHSError as ex:
        code = ex.code
    codes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(codes, torch.tensor([code], dtype=torch.int64))
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"world": world, "codes": [int(c.item()) for c in codes]}, f)
    dist.barrier()
    dist.destroy_process_group()


def main():
    out_path, scale = sys.argv[1], int(sys.argv[2])
    if len(sys.argv) > 3 and sys.argv[3] == "fault":
        return fault(out_path, scale)
    import numpy as np
    import torch
    import torch.distributed as dist

    from distributed_ghs_implementation_amd.device import generate_rmat
    from distributed_ghs_implementation_amd.distributed import DistributedMST
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    e = generate_rmat(scale, 16, seed=1, wseed=2)
    eng = DistributedMST(e, rank, world)
    results = []
    collected = None
    for _ in range(2):  # the second solve reuses the handle (ghs_solver_reset)
        res, _ = eng.run()
        flags = eng.in_mst_host()
        results.append((res.total_weight, res.num_mst_edges, flags))
        collected = eng.collect_mst(0)  # the reference's collect_results: MSF edge ids on rank 0
    eng.close()
    tot = torch.tensor([results[-1][0], results[-1][1]], dtype=torch.int64)
    allt = [torch.zeros_like(tot) for _ in range(world)]
    dist.all_gather(allt, tot)
    if rank == 0:
        from oracle import oracle
        g = e.to_host()
        ref_in, ref_tw, ref_k = oracle.kruskal_c(g.n, g.u, g.v, g.w)
        verdict = {
            "world": world, "m": g.m,
            "flags_match_oracle": all(bool(np.array_equal(r[2], ref_in.astype(bool))) for r in results),
            "totals_match_oracle": all((r[0], r[1]) == (ref_tw, ref_k) for r in results),
            "ranks_agree": all(t.tolist() == allt[0].tolist() for t in allt),
            "collected_match_oracle": bool(np.array_equal(collected.cpu().numpy(), np.flatnonzero(ref_in))),
        }
        with open(out_path, "w") as f:
            json.dump(verdict, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
