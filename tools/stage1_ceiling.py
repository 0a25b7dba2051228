"""Stage-1 ceiling on the R-MAT s24 level-0 edge set.

    python tools/stage1_ceiling.py [--scale 24] [--reps 20] > profiles/r06/stage1_ceiling.json

Builds tools/microbench/stage1_ceiling.hip into a shared library (hipcc, once), generates the
bench's R-MAT graph on the GPU, takes the engine's first weight level (the 0.5 n lightest edges,
as k_plan plans it: w below the 0.5n-th smallest weight) as (a = u, b = v, key = w << 32 | eid),
and times one min-edge round over it per variant (HIP events, best of --reps after a warmup).
Reports each variant's time and its rate under the 24 B-per-live-edge model of BASELINE.md's
stage-1 roofline, as a fraction of the 8 TB/s HBM peak.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KINDS = ["stream", "a_seg", "b_gather", "b_atomic", "ideal", "b_sorted"]


def build():
    src = os.path.join(ROOT, "tools", "microbench", "stage1_ceiling.hip")
    out = os.path.join(ROOT, "tools", "microbench", "libstage1_ceiling.so")
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950", "-o", out, src],
                       check=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--grid", type=int, default=2048)
    args = ap.parse_args()
    import torch  # first: the hipcc-built library then binds to torch's HIP runtime (one runtime)
    lib = ctypes.CDLL(build())
    import torch
    from distributed_ghs_implementation_amd.device import flags_to_eids, generate_rmat
    vp = ctypes.c_void_p
    lib.s1_run.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_uint64, vp, vp, ctypes.c_int, vp]
    e = generate_rmat(args.scale, 16, seed=1, wseed=2)
    n, m = e.n, e.m
    w = e.w.to(torch.int64) & 0xFFFFFFFF
    k0 = int(0.5 * n)  # the engine's level-1 target for m >= 4n (level1_auto): 0.5 n edges
    tau = int(torch.kthvalue(w, k0).values.item())
    sel = flags_to_eids((w <= tau).to(torch.uint8), 0, m, m)  # the library's select (not torch.nonzero)
    a = e.u[sel].contiguous()
    b = e.v[sel].contiguous()
    key = ((w[sel] << 32) | sel).contiguous()
    E = int(sel.numel())
    order = torch.argsort(b.to(torch.int64) * (1 << 32) + a.to(torch.int64))  # the b-grouped copy
    a2, b2, key2 = b[order].contiguous(), a[order].contiguous(), key[order].contiguous()
    del w, order
    best = torch.empty(n, dtype=torch.int64, device="cuda")
    sink = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    rows = {}
    for kind, name in enumerate(KINDS):
        ts = []
        for r in range(args.reps + 2):
            best.fill_(-1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if name == "b_sorted":  # two streams: the a-sorted records (a side), the b-grouped copy (b side)
                e0.record()
                assert lib.s1_run(1, P(a), P(b), P(key), E, P(best), P(sink), args.grid, st) == 0
                assert lib.s1_run(1, P(a2), P(b2), P(key2), E, P(best), P(sink), args.grid, st) == 0
                e1.record()
            else:
                e0.record()
                assert lib.s1_run(kind, P(a), P(b), P(key), E, P(best), P(sink), args.grid, st) == 0
                e1.record()
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(e0.elapsed_time(e1))
        ms = min(ts)
        rows[name] = {"ms": round(ms, 4), "ms_median": round(sorted(ts)[len(ts) // 2], 4),
                      "model_gbs": round(24.0 * E / (ms * 1e-3) / 1e9, 1),
                      "frac_of_8tbs": round(24.0 * E / (ms * 1e-3) / 8e12, 4),
                      "g_edges_per_s": round(E / (ms * 1e-3) / 1e9, 2)}
    # correctness of the minima the two full variants produce (same table both ways)
    best.fill_(-1)
    lib.s1_run(4, P(a), P(b), P(key), E, P(best), P(sink), args.grid, st)
    ref = best.clone()
    best.fill_(-1)
    lib.s1_run(1, P(a), P(b), P(key), E, P(best), P(sink), args.grid, st)
    lib.s1_run(1, P(a2), P(b2), P(key2), E, P(best), P(sink), args.grid, st)
    torch.cuda.synchronize()
    out = {"graph": f"rmat-s{args.scale}-ef16", "n": n, "m": m, "level0_edges": E, "tau": tau,
           "model": "24 B per live edge (BASELINE.md stage-1 roofline) / kernel time, vs 8 TB/s",
           "variants": rows, "minima_agree": bool(torch.equal(ref, best)),
           "ceiling": max(rows[k]["frac_of_8tbs"] for k in ("ideal", "b_sorted"))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
