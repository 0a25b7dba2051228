"""Time the on-GPU graph generation (R-MAT tuples -> sort -> unique -> canonical u/v/w) per scale.

    python tools/gen_time.py [--scales 24 26] [--reps 3]

Prints one JSON line per scale: edges kept, ms per generation (median of reps, device synced).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_ghs_implementation_amd.device import generate_grid, generate_rmat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scales", type=int, nargs="+", default=[24])
    ap.add_argument("--grid", type=int, default=0, help="also time a k x k grid")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    for s in a.scales:
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g = generate_rmat(s, 16, seed=1, wseed=2)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
            m = g.m
            del g
            torch.cuda.empty_cache()
        ts.sort()
        print(json.dumps({"workload": f"rmat-s{s}-ef16", "m": m, "ms": round(ts[len(ts) // 2], 3),
                          "all_ms": [round(t, 3) for t in ts]}), flush=True)
    if a.grid:
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g = generate_grid(a.grid)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
            del g
        ts.sort()
        print(json.dumps({"workload": f"grid-{a.grid}", "ms": round(ts[len(ts) // 2], 3)}), flush=True)


if __name__ == "__main__":
    main()
