"""Sweep the weight-level plan (speed only; results must not change) on one GPU."""
import argparse
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--workload", choices=["rmat", "grid", "grid-gradient"], default="rmat")
    ap.add_argument("--grid-k", type=int, default=16384)
    ap.add_argument("--levels", default="2,3,4,6,8")
    ap.add_argument("--l1", default="0.25,0.5,1.0,2.0")
    ap.add_argument("--growth", default="2,4,8,16")
    args = ap.parse_args()
    import torch
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_grid, generate_rmat
    if args.workload == "rmat":
        e = generate_rmat(args.scale, 16, seed=1, wseed=2)
    else:
        e = generate_grid(args.grid_k, 1 if args.workload == "grid-gradient" else 0)
    fl = lambda s: [float(x) for x in s.split(",")]
    torch.cuda.synchronize()
    ref = None
    for L, l1, gr in itertools.product([int(x) for x in args.levels.split(",")], fl(args.l1), fl(args.growth)):
        if L == 2 and gr != fl(args.growth)[0]:
            continue
        cfg = _native.make_config(max_levels=L, level1_edges_per_vertex=l1, level_growth=gr)
        eng = DeviceMST(e, config=cfg)
        eng.run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            res, stats = eng.run()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        if ref is None:
            ref = res.total_weight
        assert res.total_weight == ref
        print(json.dumps({"levels": L, "l1": l1, "growth": gr, "ms": round(min(ts), 3), "rounds": res.rounds,
                          "planned_levels": res.levels, "ms_select": round(res.ms_select, 3),
                          "ms_filter": round(res.ms_filter, 3), "filter_out": res.filter_out,
                          "edges_per_level": [s["level_arcs"] for s in stats if s["level_arcs"]]}), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
