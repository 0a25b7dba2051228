"""Benchmark: MST edges processed/sec on R-MAT (BASELINE.json metric) + % HBM roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scale S] [--workload rmat|grid|grid-gradient]

A step = one full MST of the device-resident canonical edge list (BASELINE.md "Definitions"):
validation, the weight-level plan, every level's pass and all Boruvka rounds -> in_mst flags +
total weight. Inputs are generated on the GPU before the timed region (synthetic R-MAT, Graph500
parameters, unique hashed weights — no dataset download).
  N = 1: R-MAT scale 24 (BASELINE config 3), the headline `value`; the line also carries
         `scaling_base`: R-MAT scale 26 (config 4's graph) solved on this one GPU.
  N > 1 (torch.distributed.run, one rank per GPU, RCCL): strong scaling on R-MAT scale 26 —
         every N solves the same graph, so scaling_base and the N > 1 lines form one curve; a
         step there also gathers the MSF edge ids to rank 0 (the reference's collect_results),
         ms_per_step_solve times the solve alone. "scaling" is "strong" on every line.
Input form (--input, config.input): at N = 1 on graphs with m >= 4n the canonical list is resident in
both forms — CSR row offsets (the north_star's "CSR edge list in HBM", built on the device from the
sorted u before the timed region, config.csr_offsets_build_ms) next to u, v, w: k_select streams
the CSR form, k_filter the COO form; elsewhere COO (u, v, w).
Rank 0 prints ONE JSON line. After the timed steps one extra step runs with every kernel launch
bracketed by HIP events on the solve's stream (libghs_mst.so ghs_profile_enable): `kernels` lists
every kernel's time per step and achieved GB/s under its algorithmic byte model (launch_bytes),
`roofline` is the dominant kernel's (largest time in that step; k_select / k_filter durations are
the event averages inside the timed steps), `stage1_roofline` is BASELINE.md's stage-1 figure
(24 B per live edge over every min-edge round / the min-edge kernels' time). `traffic` comes from
the committed PMC profile (profiles/**/<workload>_pmc.json: rocprofv3 FETCH_SIZE / WRITE_SIZE
passes, tools/gpu/pmc_traffic.sh) when one exists, else null.
CPU baselines, rank 0 at N=1 only: `cpu_baseline` = the all-cores OpenMP Borůvka
(oracle/boruvka_omp.c, kind "port") on the workload's own graph with every CPU the process may
use (affinity / cgroup quota / OMP_NUM_THREADS, reported under host_cpus); `cpu_baseline_serial`
= the oracle's C Kruskal (1 thread) on R-MAT s22; `cpu_baseline_networkx` = NetworkX Kruskal (the
reference's verifier) on R-MAT s16.
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
    ap.add_argument("--input", choices=["auto", "csr", "coo", "both"], default="auto",
                    help="the device-resident input form: CSR (row offsets + v + w, ghs_mst_device_csr, ABI 9), "
                         "COO (u + v + w, ghs_mst_device) or both (offsets + u + v + w: k_select streams the "
                         "CSR form, k_filter the COO form); auto = both at N = 1, COO at N > 1")
    ap.add_argument("--cpu-scale", type=int, default=22, help="R-MAT scale of the serial-Kruskal sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--nx-scale", type=int, default=16, help="R-MAT scale of the NetworkX baseline sample")
    ap.add_argument("--verify", action="store_true", help="check the result against the oracle (slow at s24)")
    ap.add_argument("--stats", action="store_true", help="print per-round stats to stderr")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N>1 (nccl = RCCL; gloo only to rehearse ranks sharing a GPU)")
    ap.add_argument("--verify-ranks", action="store_true", help="N>1: check every rank holds the same MSF")
    ap.add_argument("--no-scaling-base", action="store_true", help="N=1: skip the s26 strong-scaling point")
    ap.add_argument("--options", type=lambda x: int(x, 0), default=0,
                    help="ghs_config_t.options bits for N=1 (A/B of path options; 0 = the default path)")
    ap.add_argument("--level1", type=float, default=None, help="level plan: level-1 edges per vertex (default auto)")
    ap.add_argument("--level-growth", type=float, default=None, help="level plan: growth per level (default auto)")
    ap.add_argument("--dedup-max", type=int, default=None,
                    help="ghs_config_t.dedup_max for N=1 (parallel-edge filter at <= F fragments; A/B)")
    ap.add_argument("--coll-timeout", type=int, default=300,
                    help="N>1: seconds before a torch.distributed collective gives up (then every rank exits)")
    return ap.parse_args()


# Algorithmic bytes per launch of every profiled kernel (DESIGN.md "Kernels"): what the
# algorithm must move, counting a random gather as its element size. `rec` is one profiled launch
# (round / level / host-known items), `st` the solve's round stats, `res` its Result.
def _round_of(rec, stats):
    """The stats entry of a launch's round, or None for a lookahead no-op round (a level's
    trailing rounds reuse the next level's round index with their own, older level)."""
    r = rec["round"]
    if r < len(stats) and stats[r]["level"] == rec["level"]:
        return r
    return None


def _next_live(stats, r):
    return stats[r + 1]["live_arcs"] if r + 1 < len(stats) and stats[r + 1]["level"] == stats[r]["level"] else 0


def _first_round(stats, r):
    return r == 0 or stats[r - 1]["level"] != stats[r]["level"]


# bytes the canonical passes stream per edge and per vertex row: COO u, v, w = 12 B per edge; CSR
# (ABI 9) v, w = 8 B per edge + the u32 row offset of every row (run() sets them from the input
# form; with both forms resident k_select streams the CSR form and k_filter the COO form)
STREAM_BYTES = {"select": (12.0, 0.0), "filter": (12.0, 0.0)}


def _stream_bytes(res, n, kind):
    edge, row = STREAM_BYTES[kind]
    return edge * res.canon_edges + row * (n + 1)


def launch_bytes(rec, stats, res, n, windowed=frozenset()):
    """`windowed`: the rounds whose windowed kernel (k_wmin) did the work — their k_bucket / k_bmin
    launches are the device-side fallback that exited at once (k_select's span flag unset)."""
    k = rec["kernel"]
    if k == "k_select":
        return _stream_bytes(res, n, "select") + 16.0 * res.select_out  # the list in; level-0 edges out
    if k == "k_filter":
        return _stream_bytes(res, n, "filter") + 16.0 * res.filter_out  # stream + level-1 and pending edges out
    if k == "k_resolve":
        return 8.0 * n + n / 8.0  # lab read + write, giant bitmap
    if k == "k_jump_ident":
        return 17.0 * n  # lab 4 + par 4 + best 8 + keep flag 1 per vertex
    r = _round_of(rec, stats)
    if r is None:
        return 0.0
    st = stats[r]
    live, act = st["live_arcs"], st["active_components"]
    if k == "k_level_pass":
        return 16.0 * rec["items"] + 16.0 * st["level_arcs"]  # pending in (+ level edges out)
    if k == "k_seed_runs":
        return 12.0 * live  # a 4 + key 8
    if k == "k_minedge<IDENT>":
        return 16.0 * live  # a 4 + b 4 + key 8 (roots: no gathers)
    if k == "k_minedge<COMPACT>":
        return 24.0 * live + 16.0 * _next_live(stats, r)  # + lab[a], lab[b]; survivors out
    # bucketed rounds: a level's first round buckets its edges, later rounds their compacted
    # survivors; an edge is at least one record (a, b, key: 16 B)
    if k in ("k_bucket", "k_bmin") and r in windowed:
        return 0.0
    if k == "k_wmin" and r not in windowed:
        return 0.0  # exited at once: the fallback bucketed the round
    bucketed_edges = live if _first_round(stats, r) else _next_live(stats, r)
    if k == "k_bucket":
        return 40.0 * bucketed_edges  # pass A a, b (8 B) + pass B edge in (16 B) + record out (16 B)
    if k == "k_bmin":
        return 32.0 * bucketed_edges  # two sweeps over the records
    if k == "k_wmin":
        # level 0's windowed round: every edge read by the windows of its two buckets (a, b, key
        # twice), best + par of every vertex written
        return 32.0 * live + 12.0 * n
    # rounds >= 1 of one rank with >= 1M active fragments launch both CONNECT forms and the
    # device runs one (boruvka.hip k_win / k_hook guards: edge form while the survivors are
    # fewer than 4x the active fragments)
    edge_form = (not _first_round(stats, r)) and act >= (1 << 20) and _next_live(stats, r) < 4 * act
    if k == "k_win":
        if _first_round(stats, r):
            return 32.0 * live  # a, b, key + best[a], best[b]
        return 32.0 * _next_live(stats, r) if edge_form else 0.0
    if k == "k_hook":
        return 0.0 if edge_form else 40.0 * act  # act, best, eu/ev, lab x2, best[other], par
    if k == "k_jump":
        return 21.0 * act  # act, par, lab, best, keep flag
    if k == "k_select_lb":
        return 2.0 * rec["items"]  # keep bytes, two passes
    # the LDS tail (boruvka.hip k_tail_*): 256 blocks, one row of per-fragment minima each
    if k == "k_tail_open":
        # the live edges (a, b, key + lab / dense-id gathers) in, their 12-B records out, the rows
        return 24.0 * live + 12.0 * live + 8.0 * act * TAIL_G
    if k == "k_tail_round":
        return 12.0 * live + 8.0 * act * TAIL_G  # the records, the rows of the round's roots
    if k == "k_tail_hook":
        return 8.0 * act * TAIL_G  # the rows, reduced per root
    return 0.0


TAIL_G = 256  # boruvka.hip TAIL_G: the LDS tail's blocks (rows of block minima)
# every kernel of a min-edge round's stage 1 (the tail's kernels and the bucketed ones also hook)
STAGE1 = ("k_seed_runs", "k_minedge<IDENT>", "k_minedge<COMPACT>", "k_bucket", "k_bmin", "k_wstarts", "k_wmin",
          "k_tail_open", "k_tail_round", "k_tail_hook")


PASS_WINDOWED = 0x4  # ghs_result_t.pass_flags: level 0's round 0 ran windowed (k_select's span flag clear)


def kernel_table(records, stats, res, n):
    """Per kernel: launches, ms per step, algorithmic bytes, achieved GB/s (one profiled step)."""
    tab = {}
    # the windowed round is level 0's round 0; the library reports whether it ran (pass_flags bit 2)
    # or fell back to k_bucket / k_bmin (no longer guessed from the kernels' times)
    windowed = frozenset([0]) if res.pass_flags & PASS_WINDOWED else frozenset()
    for rec in records:
        t = tab.setdefault(rec["kernel"], {"launches": 0, "ms": 0.0, "bytes": 0.0})
        t["launches"] += 1
        t["ms"] += max(rec["ms"], 0.0)
        t["bytes"] += launch_bytes(rec, stats, res, n, windowed)
    for t in tab.values():
        t["achieved_gbs"] = t["bytes"] / (t["ms"] * 1e-3) / 1e9 if t["ms"] > 0 and t["bytes"] > 0 else None
        t["ms"] = round(t["ms"], 4)
    return tab


def stage1_roofline(records, stats):
    """BASELINE.md's stage-1 roofline: 24 B x sum over rounds of the live edges / sum of the
    min-edge time (round 0's IDENT launch + its a-side seeding, and the compacting launches)."""
    live = sum(st["live_arcs"] for st in stats)
    ms = sum(max(r["ms"], 0.0) for r in records if r["kernel"] in STAGE1 and _round_of(r, stats) is not None)
    if ms <= 0 or live == 0:
        return None
    ach = 24.0 * live / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "live_edges": int(live), "ms": round(ms, 4),
            "kernels": list(STAGE1),
            "definition": "24 B x sum of live edges over every min-edge round / sum of stage-1 time (BASELINE.md)"}


# profile name -> the PMC file's kernel-name prefix (rocprofv3 prints every template argument:
# k_minedge<false, true, false>; any later template parameter still matches the prefix)
PMC_NAMES = {"k_minedge<IDENT>": "k_minedge<true, false", "k_minedge<COMPACT>": "k_minedge<false, true",
             "k_bmin": "k_bmin<", "k_wmin": "k_wmin<",
             # the streaming passes' form (<true>: CSR), set from the input the solve streams
             "k_select": "k_select<false", "k_filter": "k_filter<false"}


def _pmc_match(name, key):
    """key (a PMC file's kernel name) is the profile kernel `name`: equal, or a templated name
    whose arguments start with the mapped prefix."""
    want = PMC_NAMES.get(name, name)
    if key == want:
        return True
    if want.endswith("<"):  # any template arguments (k_bmin<13u>, k_bmin<14u>)
        return key.startswith(want)
    return "<" in want and key.startswith(want) and key[len(want):len(want) + 1] in (">", ",")


def load_traffic(workload_tag, kernel):
    """Per-launch HBM bytes of `kernel` from a committed PMC profile (profiles/**/*_pmc.json,
    the newest round's wins). A profile name covering several template instantiations
    (k_minedge<COMPACT>: with and without candidates; k_bmin<..>: the full and the plain form)
    takes their launch-weighted mean."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*_pmc.json"), recursive=True)):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") != workload_tag:
            continue
        hits = [k for key, k in d.get("kernels", {}).items()
                if _pmc_match(kernel, key) and k and k.get("traffic_bytes_per_launch")]
        if hits:
            w = [max(1, int(k.get("launches_fetch_pass", 1))) for k in hits]
            tot = sum(k["traffic_bytes_per_launch"] * wi for k, wi in zip(hits, w))
            best = {"traffic_bytes_per_launch": tot / sum(w), "launches": sum(w), "instantiations": len(hits),
                    "_path": os.path.relpath(p, ROOT)}
    return best


def roofline_obj(kernel, t, tag, note):
    traffic = load_traffic(tag, kernel)
    ach = t["achieved_gbs"] or 0.0
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": (round(traffic["traffic_bytes_per_launch"]) if traffic else None),
            "kernel": kernel, "note": note, "algorithmic_bytes_per_launch": round(t["bytes"] / t["launches"]),
            "avg_launch_ms": round(t["ms"] / t["launches"], 4), "launches": t["launches"],
            "ms_per_step": t["ms"], "timing": t.get("timing", "HIP events around every launch of one profiled step"),
            "traffic_source": traffic["_path"] if traffic else None}


def kernels_obj(ktab, tag):
    """The line's per-kernel table; where a committed PMC profile of the workload has the kernel,
    its measured HBM bytes per launch and their ratio to the algorithmic bytes (traffic well above
    1x = re-reads / write-backs the byte model does not count)."""
    out = {}
    for k, v in sorted(ktab.items(), key=lambda kv: -kv[1]["ms"]):
        e = {"launches": v["launches"], "ms_per_step": v["ms"], "algorithmic_bytes": round(v["bytes"]),
             "achieved_gbs": round(v["achieved_gbs"], 1) if v["achieved_gbs"] else None,
             "frac": round(v["achieved_gbs"] / HBM_PEAK_GBS, 4) if v["achieved_gbs"] else None}
        tr = load_traffic(tag, k)
        if tr and v["bytes"] > 0:
            alg = v["bytes"] / v["launches"]
            e["pmc_bytes_per_launch"] = round(tr["traffic_bytes_per_launch"])
            e["pmc_ratio"] = round(tr["traffic_bytes_per_launch"] / alg, 3)
            e["pmc_source"] = tr["_path"]
        out[k] = e
    return out


def host_cpus():
    """CPUs this process may use: os.cpu_count() (the whole machine), the affinity mask, and the
    cgroup CPU quota (the GPU box grants a share of a large host)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        pass
    usable = min(aff, quota) if quota else aff
    omp = int(os.environ.get("OMP_NUM_THREADS") or 0)
    return {"os_cpu_count": os.cpu_count(), "affinity": aff, "cgroup_quota": quota, "usable": usable,
            "omp_num_threads": omp or None}


def cpu_baseline_serial(scale, edgefactor):
    """Oracle C Kruskal (1 thread) on R-MAT(scale) generated by the same GPU generator."""
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
                      f"{g.m} canonical edges) through oracle/kruskal.c canonical Kruskal, 1 thread, {dt:.2f} s",
            "seconds": dt}


def cpu_baseline_omp(g, gpu_result, tag):
    """The all-cores CPU baseline: oracle/boruvka_omp.c, an OpenMP Boruvka over
    the canonical list (same canonical MSF, parity in tests/test_oracle.py), on the GPU
    workload's own graph `g` (host copy), with every CPU this process may use (affinity and
    cgroup quota; OMP_NUM_THREADS when the box sets it). Checked against the GPU solve."""
    from oracle import oracle
    cpus = host_cpus()
    threads = cpus["omp_num_threads"] or cpus["usable"]
    oracle.boruvka_omp_c(min(g.n, 1024), g.u[:0], g.v[:0], g.w[:0], threads=threads)  # load outside the timing
    t0 = time.perf_counter()
    _, tw, k, rounds = oracle.boruvka_omp_c(g.n, g.u, g.v, g.w, threads=threads)
    dt = time.perf_counter() - t0
    ok = (tw, k) == (gpu_result.total_weight, gpu_result.num_mst_edges)
    return {"value": g.m / dt, "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": f"the GPU workload itself ({tag}, {g.m} canonical edges) through oracle/boruvka_omp.c "
                      f"OpenMP Boruvka, {threads} threads, {rounds} rounds, {dt:.2f} s; weight/edges "
                      f"{'==' if ok else '!='} the GPU solve",
            "seconds": dt, "matches_gpu": ok, "host_cpus": cpus}


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
            "host_path_matches_device": (r.total_weight, r.num_edges) == (dev_result.total_weight,
                                                                          dev_result.num_mst_edges),
            "note": "ghs_mst_host from pageable numpy arrays (H2D 12 B/edge, solve, D2H m flags); "
                    "generation = GPU R-MAT/grid + canonical radix sort + dedupe, once per graph"}, g


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


def input_form(requested, world, n, m):
    """The input form the solve streams: `requested` unless "auto" — both forms (CSR offsets + u)
    at N = 1 when m >= 4n, else COO (reasons at make_workload)."""
    if requested != "auto":
        return requested
    return "both" if world == 1 and m >= 4 * n else "coo"


def set_stream_forms(has_off, has_u, world):
    """The byte model and PMC kernel names of the streaming passes for the resident input: CSR
    offsets -> k_select streams 8 B/edge + 4 B/row (a rank: its share of the rows); k_filter
    streams the CSR form only without u."""
    if not has_off:
        STREAM_BYTES.update(select=(12.0, 0.0), filter=(12.0, 0.0))
        PMC_NAMES.update({"k_select": "k_select<false", "k_filter": "k_filter<false"})
        return
    csr = (8.0, 4.0 / max(1, world))
    STREAM_BYTES.update(select=csr, filter=(12.0, 0.0) if has_u else csr)
    PMC_NAMES.update({"k_select": "k_select<true", "k_filter": f"k_filter<{str(not has_u).lower()}"})


def make_workload(args, world):
    import torch
    from distributed_ghs_implementation_amd.device import generate_grid, generate_rmat
    if args.workload == "rmat":
        # N = 1: the s24 headline (BASELINE config 3); N > 1: strong scaling on s26 (config 4)
        scale = args.scale if args.scale is not None else (24 if world == 1 else 26)
        edges = generate_rmat(scale, args.edgefactor, seed=1, wseed=2)
        tag = f"rmat-s{scale}-ef{args.edgefactor}"
        cfg = {"workload": tag, "generator": "R-MAT A,B,C,D=.57,.19,.19,.05, seeds 1/2, self-loops dropped, "
               "deduplicated, unique hashed u32 weights", "scale": scale, "edgefactor": args.edgefactor}
    else:
        k = args.grid_k
        edges = generate_grid(k, 1 if args.workload == "grid-gradient" else 0)
        tag = f"{args.workload}-{k}x{k}"
        cfg = {"workload": tag, "grid_k": k}
    # auto: at N = 1 the north_star's CSR edge list with u kept resident next to it ("both": k_select
    # streams 8 B/edge from (off, v, w), k_filter 12 from (u, v, w) — 5.15 vs 5.25 ms for COO and 5.19
    # for CSR alone on s24, profiles/r06/both/); at N > 1 COO (the s26 x 8 emulation's slowest-rank
    # kernels were no faster with both, and each rank would validate all n + 1 offsets). Below an
    # average degree of 4 COO too: the CSR pre-pass reads the n + 1 offsets (validation, tile rows)
    # while k_select saves only 4 - 4n/m B per edge — the 16384^2 grids (m/n = 2) ran 0.2-0.3 ms slower
    # with both (profiles/r06/both/grid_ab.txt)
    form = input_form(args.input, world, edges.n, edges.m)
    if form in ("both", "csr"):
        # the offsets' device build, timed for the record (outside the timed region, like generation)
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        edges.with_csr()
        t1.record()
        torch.cuda.synchronize()
        cfg["csr_offsets_build_ms"] = round(t0.elapsed_time(t1), 4)
    if form == "both":
        # both forms resident: row offsets (built on the device from the sorted u, outside the timed
        # region) next to u — the solve streams (off, v, w) in k_select and (u, v, w) in k_filter
        edges = edges.with_csr()
        cfg["input"] = ("CSR + u: n+1 u32 row offsets + u + v + w (u32), the canonical list in both forms "
                        "(ghs_mst_device_csr with d_u)")
    elif form == "csr":
        # the north_star's CSR edge list: row offsets (built on the device from the sorted u, outside
        # the timed region like the generation itself), u released — the solve streams (off, v, w)
        edges = edges.csr_only()
        cfg["input"] = "CSR: n+1 u32 row offsets + v + w (u32), the canonical list with u implied (ghs_mst_device_csr)"
    else:
        cfg["input"] = "COO: u + v + w (u32), the canonical list (ghs_mst_device)"
    return edges, tag, cfg


def mark(rank, msg):
    """A one-line progress mark on stderr per phase (a silent multi-minute phase looks hung)."""
    print(f"[bench rank {rank} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


class PhaseFailed(RuntimeError):
    pass


def agreed(name, fn, rank, world, dist, dev):
    """Run one phase on every rank, then agree on its outcome: a MAX all-reduce of a failure flag at
    the same program point on every rank, so a rank whose phase raised ends EVERY rank with a
    message naming the phase and the failing ranks (non-zero exit) instead of leaving its peers
    waiting in the next collective. The phases' own collectives are bounded by the process group's
    timeout (--coll-timeout)."""
    import torch
    mark(rank, f"{name} ...")
    t0 = time.perf_counter()
    out, err = None, None
    try:
        out = fn()
    except Exception as ex:  # noqa: BLE001 (agreed on below, then raised on every rank)
        import traceback
        traceback.print_exc()
        err = ex
    if world > 1:
        flags = torch.zeros(world, dtype=torch.int32, device=dev)
        flags[rank] = 1 if err is not None else 0
        dist.all_reduce(flags, op=dist.ReduceOp.MAX)
        bad = [r for r in range(world) if int(flags[r].item())]
        if bad:
            raise PhaseFailed(f"phase '{name}' failed on rank(s) {bad}" + (f": {err}" if err is not None else ""))
    elif err is not None:
        raise PhaseFailed(f"phase '{name}' failed: {err}") from err
    mark(rank, f"{name} done ({time.perf_counter() - t0:.1f} s)")
    return out


def dist_engine(edges, rank, world, dist, backend):
    """N > 1: DistributedMST with the library's round loop over its own RCCL communicator; if that
    fails on any rank (setup or the first solve; the ranks agree on it), every rank falls back to
    the torch.distributed loop (run_rounds) and the line names the loop that ran."""
    import torch
    from distributed_ghs_implementation_amd.distributed import DistributedMST
    eng, err = None, None
    try:
        eng = DistributedMST(edges, rank, world)
        eng.run()
    except Exception as ex:  # noqa: BLE001 (reported in the line, then the fallback)
        err = ex
    flag = torch.tensor([1 if err is not None else 0], dtype=torch.int32,
                        device="cuda" if backend == "nccl" else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if not int(flag.item()):
        return eng, "library (ghs_solver_run over its own RCCL communicator)" if eng.native else "run_rounds"
    print(f"rank {rank}: library loop failed ({err or 'on another rank'}); torch.distributed loop instead",
          file=sys.stderr)
    if eng is not None:
        eng.close()
    eng = DistributedMST(edges, rank, world, native=False)
    return eng, f"run_rounds over torch.distributed (the library loop failed: {err or 'on another rank'})"


def time_steps(step, steps, warmup, world, dist):
    import torch
    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = []
    for i in range(steps):
        ts = time.perf_counter()
        out.append(step())
        # a progress mark after a slow step only (N > 1 rehearsals over gloo: a minute per step)
        if world > 1 and time.perf_counter() - ts > 5.0:
            mark(dist.get_rank(), f"step {i + 1}/{steps} done ({time.perf_counter() - t0:.1f} s)")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt, out


def profile_step(step, n):
    """One extra, untimed step with every launch bracketed by HIP events (libghs_mst.so
    ghs_profile_enable): per-kernel durations, the dominant kernel, the stage-1 roofline."""
    from distributed_ghs_implementation_amd import _native
    _native.profile_enable(True)
    try:
        res, stats = step()
        recs = _native.profile_read()
    finally:
        _native.profile_enable(False)
    stats = list(stats)
    return kernel_table(recs, stats, res, n), stage1_roofline(recs, stats), recs


def main():
    args = parse()
    if os.environ.get("GHS_BENCH_STACKS"):  # diagnostic: every rank's Python stacks every N seconds
        import faulthandler
        faulthandler.dump_traceback_later(int(os.environ["GHS_BENCH_STACKS"]), repeat=True)
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
        import datetime
        # every collective of the run ends (with an error, then the phase agreement) instead of
        # waiting for the default 30 minutes behind a peer that died
        dist.init_process_group(args.backend, timeout=datetime.timedelta(seconds=args.coll_timeout))
    dev = "cuda" if world == 1 or args.backend == "nccl" else "cpu"
    try:
        return run(args, world, rank, dist, dev)
    except PhaseFailed as ex:
        mark(rank, f"FAILED: {ex}")
        return 1


def run(args, world, rank, dist, dev):
    import torch

    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, flags_to_eids

    def gen():
        # ranks sharing a GPU (a rehearsal) generate one after another: the radix sort's temporary
        # buffers of N concurrent s26 generations need N x ~30 GB at once
        t0 = time.perf_counter()
        out, err = None, None
        for r in range(world):
            if r == rank:
                try:
                    out = make_workload(args, world)
                    torch.cuda.synchronize()
                    torch.cuda.empty_cache()
                except Exception as ex:  # noqa: BLE001 (after the barriers: every rank reaches them)
                    err = ex
            if world > 1 and torch.cuda.device_count() < world:
                dist.barrier()
        if err is not None:
            raise err
        return out, time.perf_counter() - t0

    (edges, tag, cfg), gen_s = agreed("generate", gen, rank, world, dist, dev)
    n, m = edges.n, edges.m
    set_stream_forms(edges.off is not None, edges.u is not None, world)
    cfg.update({"n": n, "m": m, "partition": f"canonical edge ranges x{world}", "parallelism": f"edges{world}"})

    ref = None
    if world > 1:
        # the parity reference first, while no rank holds its engine: a one-GPU solve of the same
        # resident graph on rank 0 (its ~80 GB s26 workspace freed before the ranks allocate theirs)
        def reference():
            if rank != 0:
                return None
            r1 = DeviceMST(edges)
            rres, _ = r1.run()
            eids = flags_to_eids(r1.in_mst, 0, m, min(m, n)).cpu()
            del r1
            torch.cuda.empty_cache()
            return rres.total_weight, rres.num_mst_edges, eids

        ref = agreed("reference solve (rank 0, one GPU)", reference, rank, world, dist, dev)

    loop = None
    if world > 1:
        eng, loop = agreed("engine setup + first solve", lambda: dist_engine(edges, rank, world, dist, args.backend),
                           rank, world, dist, dev)
    else:
        custom = args.options or args.dedup_max is not None or args.level1 is not None or args.level_growth is not None
        eng = DeviceMST(edges, config=_native.make_config(options=args.options, dedup_max=args.dedup_max,
                                                          level1_edges_per_vertex=args.level1,
                                                          level_growth=args.level_growth)
                        if custom else None)
    step = eng.run
    dt_solve = None
    if world > 1:
        # N > 1: a step ends with the MSF on rank 0, as the reference's MPI run ends with
        # collect_results (ghs_implementation_mpi.py:760-779): each rank's own-range MSF edge ids
        # gathered to rank 0. The solve alone is timed separately (ms_per_step_solve).
        dt_solve, _ = agreed("timed solves", lambda: time_steps(eng.run, args.steps, args.warmup, world, dist),
                             rank, world, dist, dev)

        def step():
            out = eng.run()
            eng.collect_mst(0)
            return out
    dt, outs = agreed("timed steps", lambda: time_steps(step, args.steps, args.warmup, world, dist),
                      rank, world, dist, dev)
    results = [r for r, _ in outs]
    if len(set((r.total_weight, r.num_mst_edges) for r in results)) != 1:
        raise RuntimeError("non-deterministic MST across steps")
    if world > 1 and args.verify_ranks:
        # every rank must hold the same MSF: (weight, edges, checksum of the chosen eids)
        flags = eng.gather_in_mst()
        chk = int((flags_to_eids(flags, 0, flags.numel(), min(flags.numel(), n)) % 1000003).sum().item())
        mine = torch.tensor([results[-1].total_weight, results[-1].num_mst_edges, chk], dtype=torch.int64)
        if args.backend == "nccl":
            mine = mine.cuda()
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        if any(not torch.equal(a.cpu(), allv[0].cpu()) for a in allv):
            raise RuntimeError(f"ranks disagree on the MSF: {[a.tolist() for a in allv]}")
        if rank == 0:
            print(f"ranks agree: weight {results[-1].total_weight} edges {results[-1].num_mst_edges} eid checksum {chk}",
                  file=sys.stderr)

    parity = None
    if world > 1:
        # outside the timed steps: the N-rank MSF (gathered to rank 0) against the one-GPU reference,
        # edge for edge
        def check():
            eids = eng.collect_mst(0)
            if rank != 0:
                return None
            rtw, rk, ref_eids = ref
            got = results[-1]
            p = {"against": "one-GPU solve of the same graph (DeviceMST), edge for edge",
                 "total_weight": got.total_weight, "edges": got.num_mst_edges,
                 "match": bool(rtw == got.total_weight and rk == got.num_mst_edges and torch.equal(ref_eids, eids.cpu()))}
            if not p["match"]:
                print(f"N={world} MSF differs from the one-GPU solve: {p}", file=sys.stderr)
            return p

        parity = agreed("parity vs the one-GPU solve", check, rank, world, dist, dev)

    ktab, s1, _ = agreed("profiled step", lambda: profile_step(eng.run, n), rank, world, dist, dev)
    # the canonical passes are also timed inside the timed steps (two events per pass, no idle
    # between dependent kernels of note): prefer those averages for k_select / k_filter
    for name, attr in (("k_select", "ms_select"), ("k_filter", "ms_filter")):
        ms = [getattr(r, attr) for r in results]
        if name in ktab and ms and min(ms) > 0:
            t = ktab[name]
            t["ms"] = round(sum(ms) / len(ms) * t["launches"], 4)
            t["achieved_gbs"] = t["bytes"] / (t["ms"] * 1e-3) / 1e9
            t["timing"] = "HIP events around the launch inside the timed steps (average)"
    line = None
    if rank == 0:
        ms_per_step = dt * 1e3 / args.steps
        value = m * args.steps / dt
        with_bytes = {k: v for k, v in ktab.items() if v["bytes"] > 0}
        dom = max(ktab, key=lambda k: ktab[k]["ms"])
        if dom not in with_bytes:  # report the largest kernel that has a byte model
            dom = max(with_bytes, key=lambda k: with_bytes[k]["ms"]) if with_bytes else None
        roofline = roofline_obj(dom, ktab[dom], tag, "dominant kernel of the step (largest time in the profiled "
                                "step among every launch; algorithmic bytes per DESIGN.md)") if dom else None
        s0 = outs[-1][1]
        res0 = results[-1]
        breakdown = {
            "rounds": res0.rounds, "engine_ms_last_step": round(res0.ms_total, 3), "levels": res0.levels,
            "pass_flags": res0.pass_flags,
            "per_round": [{"level": st["level"], "level_edges": st["level_arcs"], "live_edges": st["live_arcs"],
                           "fragments": st["active_components"], "hooks": st["hooks"]} for st in s0],
        }
        kernels = kernels_obj(ktab, tag)
        cpu = cpu_omp = cpu_nx = e2e = None
        if world == 1 and not args.no_cpu_baseline:
            e2e, g = end_to_end(edges, gen_s, res0)
            cpu_omp = cpu_baseline_omp(g, res0, tag)
            del g
            cpu = cpu_baseline_serial(args.cpu_scale, args.edgefactor)
            cpu_nx = networkx_baseline(args.nx_scale, args.edgefactor)
        line = {"metric": METRIC, "value": round(value, 1), "unit": "edges/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
                "dtype": "u64", "data": "synthetic (generated on GPU)", "config": cfg, "roofline": roofline,
                "stage1_roofline": s1, "cpu_baseline": cpu_omp, "cpu_baseline_serial": cpu,
                "cpu_baseline_networkx": cpu_nx, "end_to_end": e2e, "kernels": kernels,
                "mst": {"total_weight": res0.total_weight, "edges": res0.num_mst_edges}, "breakdown": breakdown}
        if world > 1:
            line["loop"] = loop
            line["parity"] = parity
            line["ms_per_step_solve"] = round(dt_solve * 1e3 / args.steps, 4)
            line["step"] = "solve + gather of the MSF edge ids to rank 0 (collect_results)"
    del eng
    if world == 1 and args.workload == "rmat" and args.scale is None and not args.no_scaling_base:
        # the strong-scaling reference point: config 4's graph (R-MAT s26) on this one GPU, the
        # graph every N > 1 line of `bench.py --gpus N` solves
        del edges
        torch.cuda.empty_cache()
        sargs = argparse.Namespace(**vars(args))
        sargs.scale = 26
        e26, tag26, _ = make_workload(sargs, 1)
        eng26 = DeviceMST(e26)
        dt26, outs26 = time_steps(eng26.run, max(2, args.steps // 2), 1, 1, dist)
        steps26 = max(2, args.steps // 2)
        if rank == 0:
            line["scaling_base"] = {"workload": tag26, "n_gpus": 1, "m": e26.m, "steps": steps26,
                                    "value": round(e26.m * steps26 / dt26, 1),
                                    "ms_per_step": round(dt26 * 1e3 / steps26, 4),
                                    "note": "bench.py --gpus N > 1 solves this graph (strong scaling); this is its N=1 point"}
        del eng26, e26
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
