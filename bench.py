"""Benchmark: MST edges processed/sec on R-MAT (BASELINE.json metric) + % HBM roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scale S] [--workload rmat|grid]

A step = one full MST of the device-resident canonical edge list (BASELINE.md "Definitions"):
validation, the weight-level plan, every level's pass and all Boruvka rounds -> in_mst flags +
total weight.
Inputs are generated on the GPU before the timed region (synthetic R-MAT, Graph500 parameters,
unique hashed weights — no dataset download). N=1: R-MAT scale 24 (BASELINE config 3).
N>1 (torch.distributed.run, one rank per GPU, RCCL all-reduce MIN per round): every rank holds
the replicated canonical list and streams its contiguous canonical-edge range; scale
min(26, 24 + log2 N) (config 4: s26 on 8 GPUs).

Rank 0 prints ONE JSON line. `roofline` is for the dominant kernel of the step (largest
time over the timed steps) among the instrumented ones: k_filter (canonical stream + giant-bitmap
filter + level-1 split; 12 B per canonical edge read + 16 B per entry written), k_select
(validation + level-0 split; same accounting) and the compacting min-edge kernel (24 B per live
edge + 16 B per survivor). Durations are HIP events recorded by libghs_mst.so on the launch
stream: k_filter / k_select inside the timed steps, the min-edge launches in one extra
instrumented step after them (GHS_TIME_ROUNDS=1; per-round events would add idle time to the
timed steps); all three are listed under "kernels". `traffic` comes from the
committed PMC profile (profiles/**/<workload>_pmc.json: rocprofv3 FETCH_SIZE / WRITE_SIZE passes,
gfx950-corrected, tools/gpu/pmc_traffic.sh) when one exists for this workload, else null.
CPU baselines on bounded samples (same generator, smaller scale), rank 0 at N=1 only:
`cpu_baseline` = the all-cores OpenMP Borůvka (oracle/boruvka_omp.c, kind "port",
OMP_NUM_THREADS threads) on R-MAT s23; `cpu_baseline_serial` = the oracle's C Kruskal (1 thread)
on R-MAT s21; `cpu_baseline_networkx` = NetworkX Kruskal (the reference's verifier) on R-MAT s16.
"""
import argparse
import glob
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MST edges processed/sec (R-MAT s24 1 GPU, s26 8 GPU) + % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=int, default=None)
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--workload", choices=["rmat", "grid", "grid-gradient"], default="rmat")
    ap.add_argument("--grid-k", type=int, default=16384)
    ap.add_argument("--cpu-scale", type=int, default=21, help="R-MAT scale of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--omp-scale", type=int, default=23, help="R-MAT scale of the OpenMP Boruvka baseline sample")
    ap.add_argument("--nx-scale", type=int, default=16, help="R-MAT scale of the NetworkX baseline sample")
    ap.add_argument("--verify", action="store_true", help="check the result against the oracle (slow at s24)")
    ap.add_argument("--stats", action="store_true", help="print per-round stats to stderr")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N>1 (nccl = RCCL; gloo only to rehearse ranks sharing a GPU)")
    ap.add_argument("--verify-ranks", action="store_true", help="N>1: check every rank holds the same MSF")
    return ap.parse_args()


def minedge_roofline(all_stats):
    """The compacting min-edge kernel (rounds >= 2 of a level; SURVEY.md 8(d) stage 1): 24 B per
    live edge read (a 4 + b 4 + key 8 + lab[a] 4 + lab[b] 4) + 16 B per surviving edge written.
    Returns (achieved GB/s, bytes per launch, avg ms per launch, launches) or None."""
    tot_bytes = 0.0
    tot_ms = 0.0
    launches = 0
    for stats in all_stats:
        for r, st in enumerate(stats):
            first_of_level = r == 0 or stats[r - 1]["level"] != st["level"]
            if first_of_level or st["live_arcs"] == 0 or st["ms_minedge"] <= 0:
                continue
            nxt = stats[r + 1] if r + 1 < len(stats) else None
            survivors = nxt["live_arcs"] if nxt is not None and nxt["level"] == st["level"] else 0
            tot_bytes += 24.0 * st["live_arcs"] + 16.0 * survivors
            tot_ms += st["ms_minedge"]
            launches += 1
    if launches == 0 or tot_ms <= 0:
        return None
    return tot_bytes / (tot_ms * 1e-3) / 1e9, tot_bytes / launches, tot_ms / launches, launches


def pass_roofline(results, which):
    """A canonical pass (one launch per step): 12 B per canonical edge streamed (u, v, w) + 16 B
    per entry written. k_filter's bitmap probes hit the L2-resident bitmap and are not HBM bytes.
    Returns (achieved GB/s, bytes per launch, avg ms per launch, launches) or None."""
    ms = [getattr(r, "ms_" + which) for r in results]
    out = [getattr(r, which + "_out") for r in results]
    if not ms or min(ms) <= 0:
        return None
    bpl = 12.0 * results[0].canon_edges + 16.0 * out[0]
    avg = sum(ms) / len(ms)
    return bpl / (avg * 1e-3) / 1e9, bpl, avg, len(ms)


def load_traffic(workload_tag, kernel):
    """Per-launch HBM bytes of `kernel` from a committed PMC profile (profiles/**/*_pmc.json)."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*_pmc.json"), recursive=True)):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        k = d.get("kernels", {}).get(kernel)
        if d.get("workload") == workload_tag and k and k.get("traffic_bytes_per_launch"):
            best = dict(k, _path=os.path.relpath(p, ROOT))
    return best


def roofline_obj(roof, kernel, tag, note):
    ach, bpl, msl, launches = roof
    traffic = load_traffic(tag, kernel)
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": (round(traffic["traffic_bytes_per_launch"]) if traffic else None),
            "kernel": kernel, "note": note, "algorithmic_bytes_per_launch": round(bpl),
            "avg_launch_ms": round(msl, 4), "launches": launches,
            "traffic_source": traffic["_path"] if traffic else None}


def cpu_baseline(scale, edgefactor):
    """Oracle C Kruskal (1 thread) on R-MAT(scale) generated by the same GPU generator."""
    import numpy as np  # noqa: F401

    from distributed_ghs_implementation_amd.device import generate_rmat
    from oracle import oracle
    e = generate_rmat(scale, edgefactor, seed=1, wseed=2)
    g = e.to_host()
    del e
    oracle.kruskal_c(min(g.n, 1024), g.u[:0], g.v[:0], g.w[:0])  # load the library outside the timing
    t0 = time.perf_counter()
    _, tw, k = oracle.kruskal_c(g.n, g.u, g.v, g.w)
    dt = time.perf_counter() - t0
    return {"value": g.m / dt, "unit": "edges/s", "cores": 1, "kind": "port",
            "sample": f"R-MAT scale {scale} edgefactor {edgefactor} (same generator/seeds as the GPU workload, "
                      f"{g.m} canonical edges) through oracle/kruskal.c canonical Kruskal, 1 thread, "
                      f"{dt:.2f} s; host os.cpu_count()={os.cpu_count()}",
            "seconds": dt}


def omp_baseline(scale, edgefactor, threads=None):
    """The all-cores CPU baseline: oracle/boruvka_omp.c, an OpenMP Borůvka
    over the canonical list (same canonical MSF, parity in tests/test_oracle.py), on R-MAT(scale)
    from the same generator. threads: OMP_NUM_THREADS (16 on the GPU box), else the process's
    CPUs capped at 16. Its weight/edge count is checked against one GPU solve of the same graph."""
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
    from oracle import oracle
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or min(16, len(os.sched_getaffinity(0)))
    e = generate_rmat(scale, edgefactor, seed=1, wseed=2)
    gres, _ = DeviceMST(e).run()
    g = e.to_host()
    del e
    oracle.boruvka_omp_c(min(g.n, 1024), g.u[:0], g.v[:0], g.w[:0], threads=threads)  # load outside the timing
    t0 = time.perf_counter()
    _, tw, k, rounds = oracle.boruvka_omp_c(g.n, g.u, g.v, g.w, threads=threads)
    dt = time.perf_counter() - t0
    ok = (tw, k) == (gres.total_weight, gres.num_mst_edges)
    return {"value": g.m / dt, "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": f"R-MAT scale {scale} edgefactor {edgefactor} ({g.m} canonical edges) through "
                      f"oracle/boruvka_omp.c OpenMP Boruvka, {threads} threads, {rounds} rounds, {dt:.2f} s; "
                      f"weight/edges {'==' if ok else '!='} the GPU solve of the same graph; "
                      f"host os.cpu_count()={os.cpu_count()}",
            "seconds": dt, "matches_gpu": ok}


def end_to_end(edges, gen_s, dev_result):
    """The steps either side of the timed path (reported separately, never the
    `value`): on-GPU generation + canonical sort/dedupe of the workload, and the host-buffer
    entry point ghs_mst_host (pageable host arrays: H2D of 12 B/edge + the solve + D2H of the
    m in_mst flags over PCIe) on the same graph, checked against the device-resident solve."""
    from distributed_ghs_implementation_amd.mst import minimum_spanning_forest
    g = edges.to_host()
    minimum_spanning_forest(g)  # warm: device buffers, library state
    t0 = time.perf_counter()
    r = minimum_spanning_forest(g)
    dt = time.perf_counter() - t0
    return {"generation_ms": round(gen_s * 1e3, 1),
            "host_path_ms": round(dt * 1e3, 2), "host_path_edges_per_s": round(g.m / dt, 1),
            "host_path_matches_device": (r.total_weight, r.num_edges) == (dev_result[0], dev_result[1]),
            "note": "ghs_mst_host from pageable numpy arrays (H2D 12 B/edge, solve, D2H m flags); "
                    "generation = GPU R-MAT/grid + canonical radix sort + dedupe, once per graph"}


def networkx_baseline(scale, edgefactor):
    """NetworkX Kruskal (the reference's own verifier, ghs_implementation.py:746 /
    check_mst.py:9; 1 core under the GIL) on R-MAT(scale) from the same generator. Times the
    nx.minimum_spanning_tree call (graph built beforehand, as the GPU timing excludes generation)
    and checks its weight against the oracle's. None when NetworkX is not importable here."""
    try:
        import networkx as nx
    except ImportError:
        return None
    from distributed_ghs_implementation_amd.device import generate_rmat
    from oracle import oracle
    e = generate_rmat(scale, edgefactor, seed=1, wseed=2)
    g = e.to_host()
    del e
    G = nx.Graph()
    G.add_nodes_from(range(g.n))
    G.add_weighted_edges_from(zip(g.u.tolist(), g.v.tolist(), g.w.tolist()))
    t0 = time.perf_counter()
    T = nx.minimum_spanning_tree(G, weight="weight")
    dt = time.perf_counter() - t0
    tw = sum(int(d["weight"]) for _, _, d in T.edges(data=True))
    _, ref_tw, _ = oracle.kruskal_c(g.n, g.u, g.v, g.w)
    return {"value": g.m / dt, "unit": "edges/s", "cores": 1, "kind": "networkx",
            "sample": f"R-MAT scale {scale} edgefactor {edgefactor} ({g.m} canonical edges) through "
                      f"nx.minimum_spanning_tree (networkx {nx.__version__}), graph prebuilt, {dt:.2f} s; "
                      f"weight {'==' if tw == ref_tw else '!='} oracle",
            "seconds": dt, "weight_matches_oracle": tw == ref_tw}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print("run N>1 under torch.distributed.run (one rank per GPU)", file=sys.stderr)
            return 2
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1:
        dist.init_process_group(args.backend)

    from distributed_ghs_implementation_amd.device import DeviceMST, generate_grid, generate_rmat
    from distributed_ghs_implementation_amd.distributed import DistributedMST

    t_gen = time.perf_counter()
    if args.workload == "rmat":
        scale = args.scale if args.scale is not None else min(26, 24 + int(round(math.log2(max(world, 1)))))
        edges = generate_rmat(scale, args.edgefactor, seed=1, wseed=2)
        tag = f"rmat-s{scale}-ef{args.edgefactor}"
        cfg = {"workload": tag, "generator": "R-MAT A,B,C,D=.57,.19,.19,.05, seeds 1/2, self-loops dropped, "
               "deduplicated, unique hashed u32 weights", "scale": scale, "edgefactor": args.edgefactor}
    else:
        k = args.grid_k
        edges = generate_grid(k, 1 if args.workload == "grid-gradient" else 0)
        tag = f"{args.workload}-{k}x{k}"
        cfg = {"workload": tag, "grid_k": k}
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t_gen
    n, m = edges.n, edges.m
    cfg.update({"n": n, "m": m, "partition": f"canonical edge ranges x{world}", "parallelism": f"edges{world}"})

    if world > 1:
        eng = DistributedMST(edges, rank, world)
        step = eng.run
    else:
        eng = DeviceMST(edges)
        step = eng.run

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    all_stats = []
    results = []
    raw_results = []
    for _ in range(args.steps):
        res, stats = step()
        all_stats.append(stats)
        results.append((res.total_weight, res.num_mst_edges, res.rounds, res.ms_total, res.levels))
        raw_results.append(res)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if len(set((r[0], r[1]) for r in results)) != 1:
        raise RuntimeError("non-deterministic MST across steps")
    if world > 1 and args.verify_ranks:
        # every rank must hold the same MSF: (weight, edges, checksum of the chosen eids)
        flags = eng.gather_in_mst()
        chk = int((torch.nonzero(flags).flatten().to(torch.int64) % 1000003).sum().item())
        mine = torch.tensor([results[-1][0], results[-1][1], chk], dtype=torch.int64)
        if args.backend == "nccl":
            mine = mine.cuda()
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        if any(not torch.equal(a.cpu(), allv[0].cpu()) for a in allv):
            raise RuntimeError(f"ranks disagree on the MSF: {[a.tolist() for a in allv]}")
        if rank == 0:
            print(f"ranks agree: weight {results[-1][0]} edges {results[-1][1]} eid checksum {chk}", file=sys.stderr)

    # one more, untimed step with the compacting min-edge launches bracketed by HIP events
    # (GHS_TIME_ROUNDS: ~5.7 us of idle per event, so the timed steps above carry none)
    os.environ["GHS_TIME_ROUNDS"] = "1"
    try:
        _, inst_stats = step()
    finally:
        os.environ.pop("GHS_TIME_ROUNDS", None)
    roof_me = minedge_roofline([inst_stats])
    roof_f = pass_roofline(raw_results, "filter")
    roof_s = pass_roofline(raw_results, "select")
    line = None
    if rank == 0:
        ms_per_step = dt * 1e3 / args.steps
        value = m * args.steps / dt
        kernels = {}
        if roof_f:
            kernels["k_filter"] = roofline_obj(
                roof_f, "k_filter", tag, "dominant kernel of the step: canonical stream (12 B/edge) + giant-bitmap "
                "probe per heavy edge (L2-request bound, DESIGN.md) + level-1/pending writes (16 B/entry)")
        if roof_s:
            kernels["k_select"] = roofline_obj(roof_s, "k_select", tag,
                                               "canonical stream + validation + level-0 split")
        if roof_me:
            kernels["k_minedge"] = roofline_obj(
                roof_me, "k_minedge<false, true>", tag, "min-edge with relabel + compaction, rounds >= 2 "
                "(SURVEY 8(d) stage 1: 24 B per live edge + 16 B per survivor)")
        # the roofline object is the dominant kernel's (largest time per step)
        dom = max(kernels.values(), key=lambda k: k["avg_launch_ms"] * k["launches"]) if kernels else None
        roofline = dom
        s0 = all_stats[-1]
        breakdown = {
            "rounds": results[-1][2],
            "engine_ms_last_step": round(results[-1][3], 3),
            "levels": results[-1][4],
            "per_round": [{"level": s["level"], "level_arcs": s["level_arcs"], "live_arcs": s["live_arcs"],
                           "fragments": s["active_components"], "hooks": s["hooks"],
                           "ms_minedge": round(s["ms_minedge"], 4), "ms_hook": round(s["ms_hook"], 4),
                           "ms_jump": round(s["ms_jump"], 4), "ms_next": round(s["ms_active"], 4)} for s in s0],
        }
        cpu = cpu_nx = cpu_omp = e2e = None
        if world == 1 and not args.no_cpu_baseline:
            e2e = end_to_end(edges, gen_s, results[-1])
            cpu = cpu_baseline(args.cpu_scale, args.edgefactor)
            cpu_omp = omp_baseline(args.omp_scale, args.edgefactor)
            cpu_nx = networkx_baseline(args.nx_scale, args.edgefactor)
        line = {"metric": METRIC, "value": round(value, 1), "unit": "edges/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
                "data": "synthetic (generated on GPU)", "config": cfg, "roofline": roofline,
                "cpu_baseline": cpu_omp, "cpu_baseline_serial": cpu, "cpu_baseline_networkx": cpu_nx, "end_to_end": e2e, "kernels": kernels, "mst": {"total_weight": results[-1][0], "edges": results[-1][1]},
                "breakdown": breakdown}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
