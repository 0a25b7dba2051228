"""One profiled solve (every launch bracketed by HIP events): per-round kernel times next to the
round's live edges / active fragments / hooks.

    python tools/round_profile.py [--workload rmat|grid|grid-gradient] [--scale 24] [--grid-k 16384]
                                  [--input auto|coo|csr|both]   (auto: bench.py's N = 1 choice)
"""
import argparse
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="rmat")
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--grid-k", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--input", choices=["auto", "coo", "csr", "both"], default="auto")
    args = ap.parse_args()
    import torch
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_grid, generate_rmat
    if args.workload == "rmat":
        e = generate_rmat(args.scale, 16, seed=1, wseed=2)
    else:
        e = generate_grid(args.grid_k, 1 if args.workload == "grid-gradient" else 0)
    form = args.input if args.input != "auto" else ("both" if e.m >= 4 * e.n else "coo")
    if form == "both":
        e = e.with_csr()
    elif form == "csr":
        e = e.csr_only()
    eng = DeviceMST(e)
    eng.run()
    torch.cuda.synchronize()
    for _ in range(args.reps):
        _native.profile_enable(True)
        res, stats = eng.run()
        recs = _native.profile_read()
        _native.profile_enable(False)
    stats = list(stats)
    per = defaultdict(lambda: defaultdict(float))
    last = {}  # each level's last round with stats
    for i, st in enumerate(stats):
        last[st["level"]] = i
    for r in recs:
        ok = r["round"] < len(stats) and stats[r["round"]]["level"] == r["level"]
        # past a level's rounds: the LDS tail's finishing k_tail_round (the round after the level's
        # last: it applies that round's hooks and writes the level's labels), or a no-op — a tail
        # launch after the finishing one, or a lookahead round of the pipelined loop enqueued before
        # the report that ended the level was read (its kernels exit on the device count)
        fin = not ok and r["round"] == last.get(r["level"], -2) + 1 and r["kernel"] == "k_tail_round"
        key = r["round"] if ok else ("finish" if fin else "noop", r["level"])
        per[key][r["kernel"]] += r["ms"]
    tot = sum(r["ms"] for r in recs)
    print(f"input={form} m={e.m} n={e.n} rounds={res.rounds} levels={res.levels} sum of launches {tot:.3f} ms")
    for i, st in enumerate(stats):
        ks = per.get(i, {})
        print(f"r{i:2d} L{st['level']} live {st['live_arcs']:>11d} frags {st['active_components']:>10d} "
              f"hooks {st['hooks']:>9d} | " + " ".join(f"{k}={v * 1e3:.0f}" for k, v in sorted(ks.items(), key=lambda kv: -kv[1])))
    for k, ks in per.items():
        if isinstance(k, tuple):
            print(k[0], f"L{k[1]}", " ".join(f"{a}={v * 1e3:.0f}" for a, v in ks.items()))


if __name__ == "__main__":
    main()
