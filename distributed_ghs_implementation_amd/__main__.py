"""CLI mirroring `mpiexec -n N python ghs_implementation_mpi.py --graph-dir D`
(ghs_implementation_mpi.py:884-954) and the thread path's result JSON.

    python -m distributed_ghs_implementation_amd --graph-dir graph_data
        reads graph_metadata.json (or node_<id>.json files), runs the HIP engine on one GPU,
        writes <graph-dir>/ghs_mst.json in the mst_result_mpi.json schema
        ({"mst_edges", "total_weight", "num_edges", "algorithm"}), prints a summary.
    --mpi-compat   also write <graph-dir>/mst_result_mpi.json (same content)
    --graph FILE   read an .mstbin binary graph instead of a directory
    --output FILE  result path (default <graph-dir>/ghs_mst.json)
    --check        verify the result after the run (verify.py: forest, spans every component,
                   weight vs NetworkX when available — the reference's check_mst.py)
    --check-result FILE
                   verify an existing result JSON against the graph; no GPU, no solve

    --gpus N       one process drives N GPUs of this node (RCCL clique, ghs_mst_multi)
    --generator {rmat,grid} --scale S --seed X
                   solve a synthetic BASELINE graph generated on the GPU instead of reading one
                   (R-MAT 2^S vertices, edgefactor 16; grid: --scale is the side k)

Multi-GPU, one process per GPU:
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        -m distributed_ghs_implementation_amd --graph-dir D
"""
import argparse
import os
import sys
import time


def main(argv=None):
    ap = argparse.ArgumentParser(description="MI355X Boruvka MST (drop-in for ghs_implementation_mpi.py)")
    ap.add_argument("--graph-dir", type=str, default="graph_data", help="Graph data directory (default: graph_data)")
    ap.add_argument("--graph", type=str, default=None, help=".mstbin graph file")
    ap.add_argument("--output", type=str, default=None)
    ap.add_argument("--mpi-compat", action="store_true")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--check", action="store_true", help="verify the result (check_mst.py)")
    ap.add_argument("--check-result", type=str, default=None, help="verify an existing result JSON only")
    ap.add_argument("--gpus", type=int, default=1, help="GPUs driven by this one process (RCCL clique)")
    ap.add_argument("--generator", choices=["rmat", "grid"], default=None, help="synthetic graph instead of a file")
    ap.add_argument("--scale", type=int, default=16, help="R-MAT scale (2^scale vertices) / grid side k")
    ap.add_argument("--seed", type=int, default=1, help="generator seed (weights: seed + 1)")
    args = ap.parse_args(argv)

    from . import graph as G

    t0 = time.perf_counter()
    if args.generator:
        from .device import generate_grid, generate_rmat
        e = (generate_rmat(args.scale, 16, seed=args.seed, wseed=args.seed + 1) if args.generator == "rmat"
             else generate_grid(args.scale, 0, wseed=args.seed + 1))
        g = e.to_host()
        del e
    else:
        g = G.read_mstbin(args.graph) if args.graph else G.read_graph_dir(args.graph_dir)
    t_read = time.perf_counter() - t0

    if args.check_result:
        import json

        from .verify import format_report, verify_forest
        with open(args.check_result) as f:
            triples = [tuple(e) for e in json.load(f)["mst_edges"]]
        rep = verify_forest(g, triples)
        print(format_report(rep, triples))
        return 0 if rep["ok"] else 1

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist

        from .device import DeviceEdges
        from .distributed import DistributedMST
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
        edges = DeviceEdges.from_host(g)
        d = DistributedMST(edges)
        res, _ = d.run()
        in_mst = d.in_mst_host()
        triples = g.edge_triples(in_mst)
        rounds, ms = res.rounds, res.ms_total
        dist.barrier()
        dist.destroy_process_group()
    else:
        from .mst import minimum_spanning_forest
        r = minimum_spanning_forest(g, num_gpus=args.gpus)
        triples, rounds, ms = r.triples(), r.rounds, r.ms_total
    if rank != 0:
        return 0
    if args.output:
        out = args.output
    elif args.generator:
        out = "ghs_mst.json"
    else:
        out = os.path.join(args.graph_dir if not args.graph else os.path.dirname(args.graph) or ".", "ghs_mst.json")
    res = G.write_result(out, triples)
    if args.mpi_compat:
        G.write_result(os.path.join(os.path.dirname(out), "mst_result_mpi.json"), triples)
    if not args.quiet:
        print("=" * 70)
        print("Boruvka MST on MI355X (HIP) — drop-in for the GHS MPI path")
        print("=" * 70)
        print(f"Nodes: {g.n}  Edges: {g.m}  GPUs: {max(world, args.gpus)}")
        print(f"MST edges: {res['num_edges']}  Total MST weight: {res['total_weight']}")
        print(f"Rounds (GHS levels): {rounds}  engine time: {ms:.3f} ms  read: {t_read * 1e3:.1f} ms")
        if res["num_edges"] == g.n - 1:
            print("Spanning tree: n-1 edges")
        else:
            print(f"Spanning forest: {g.n - res['num_edges']} components")
        print(f"Results saved to: {out}")
    if args.check:
        from .verify import format_report, verify_forest
        rep = verify_forest(g, triples)
        print(format_report(rep, triples))
        return 0 if rep["ok"] else 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
