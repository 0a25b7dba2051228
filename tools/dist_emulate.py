"""Per-rank cost of the multi-GPU decomposition, emulated on ONE GPU (no RCCL).

N edge-range engines (one per emulated rank) step through the level/round loop in one process;
the collectives are emulated with torch.maximum / torch.minimum and are NOT timed. Each rank's
library calls are bracketed by torch.cuda.synchronize(), so per round we get every rank's own
GPU+host time; the projected step time of a real N-GPU run is
    sum over rounds of max over ranks (compute)  +  collectives (payload bytes listed per round)
The result must equal the single-GPU MSF (asserted).

    python tools/dist_emulate.py --scale 26 --world 8
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--no-ref", action="store_true", help="skip the single-GPU reference (profiling)")
    ap.add_argument("--no-inplace", action="store_true",
                    help="pack / int64 MIN / unpack in every round (the gloo loop) instead of the library "
                         "loop's in-place uint64 MIN of a dense level's first round")
    ap.add_argument("--allreduce-hooks", action="store_true",
                    help="a dense level's opening round by all-reduce MIN + owner hooks as int32 MAX (the "
                         "stepwise protocol) instead of the library loop's reduce-scatter + pair all-gather")
    ap.add_argument("--profile", action="store_true",
                    help="per-launch HIP-event profile of the last rep: kernel ms per round of the max rank")
    ap.add_argument("--per-rank", action="store_true", help="with --profile: every rank's kernels in level-opening rounds")
    ap.add_argument("--max-levels", type=int, default=None)
    ap.add_argument("--level-growth", type=float, default=None)
    ap.add_argument("--level1", type=float, default=None, help="level-1 edges per vertex")
    ap.add_argument("--beta", type=float, default=None, help="edge_range's cost slope (device.RANGE_BETA)")
    ap.add_argument("--csr", action="store_true", help="the ranks stream the CSR form (ghs_solver_create_csr)")
    ap.add_argument("--both", action="store_true",
                    help="CSR form with u resident too (k_select streams CSR, k_filter COO)")
    args = ap.parse_args()
    import torch
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, edge_range, generate_rmat
    from distributed_ghs_implementation_amd.distributed import HipStepper

    e = generate_rmat(args.scale, 16, seed=1, wseed=2)
    one_ms, ref_flags, rres = None, None, None
    if not args.no_ref:
        ref = DeviceMST(e)
        rres, _ = ref.run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ref.run()
        torch.cuda.synchronize()
        one_ms = (time.perf_counter() - t0) * 1e3
        ref_flags = ref.in_mst[: e.m].clone()
        del ref
        torch.cuda.empty_cache()

    W = args.world
    cfg = _native.make_config(num_ranks=W, max_levels=args.max_levels, level_growth=args.level_growth,
                              level1_edges_per_vertex=args.level1)
    if args.csr:
        e = e.csr_only()
    elif args.both:
        e = e.with_csr()
    engines = [DeviceMST(e, *edge_range(e.m, r, W, args.beta), config=cfg) for r in range(W)]
    steppers = [HipStepper(x) for x in engines]

    from collections import defaultdict
    kprof = None  # [round][rank] -> {kernel: ms}

    def timed(r, fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) * 1e3
        return out, dt

    for rep in range(args.reps):
        if args.profile and rep == args.reps - 1:
            _native.profile_enable(True)
            kprof = []
        if rep or args.profile:  # a reset also picks up the profile switch
            for s in steppers:
                s.reset()
        rounds = []
        done = False
        carry = [0.0] * W  # a tail's finishing round: counted with the next level's first round
        while not done:
            ms, carry = carry, [0.0] * W
            coll = []
            # a dense level's LDS tail (ABI 10): one entry per tail round (its collectives not timed)
            F = []
            for r, s in enumerate(steppers):
                f, t = timed(r, s.tail_begin)
                F.append(f)
                ms[r] += t
            assert len(set(F)) == 1
            if F[0]:
                bufs = [s.tail_buffers(F[0]) for s in steppers]
                sign = torch.tensor(-(1 << 63), dtype=torch.int64, device=bufs[0][0].device)
                while True:
                    red = bufs[0][0] ^ sign
                    for k, _ in bufs[1:]:
                        red = torch.minimum(red, k ^ sign)
                    red ^= sign
                    for k, _ in bufs:
                        k.copy_(red)
                    for r, s in enumerate(steppers):
                        _, t = timed(r, s.tail_agree)
                        ms[r] += t
                    hmax = bufs[0][1].clone()
                    for _, h in bufs[1:]:
                        hmax = torch.maximum(hmax, h)
                    for _, h in bufs:
                        h.copy_(hmax)
                    coll = [("allreduce_min_u64", F[0] * 8), ("allreduce_max_i32", F[0] * 4)]
                    states = []
                    tr = [0.0] * W
                    for r, s in enumerate(steppers):
                        st, t = timed(r, s.tail_round)
                        states.append(st)
                        tr[r] = t
                    assert len(set(states)) == 1
                    if states[0]:  # the finishing round applies the last hooks and closes the level
                        rounds.append({"max_rank_ms": round(max(ms), 4), "min_rank_ms": round(min(ms), 4),
                                       "collectives": coll, "tail": True})
                        carry = tr
                        break
                    rounds.append({"max_rank_ms": round(max(ms), 4), "min_rank_ms": round(min(ms), 4),
                                   "collectives": coll, "tail": True})
                    ms = tr
                if states[0] == 2:
                    rounds.append({"max_rank_ms": round(max(carry), 4), "min_rank_ms": round(min(carry), 4),
                                   "collectives": [], "tail": True})
                    done = True
                continue
            counts = []
            for r, s in enumerate(steppers):
                c, t = timed(r, s.minedge)
                counts.append(c)
                ms[r] += t
            while counts[0] is None:
                bits = []
                for r, s in enumerate(steppers):
                    b, t = timed(r, lambda: s.flag_bits().clone())
                    bits.append(b)
                    ms[r] += t
                gathered = torch.cat(bits)
                for r, s in enumerate(steppers):
                    _, t = timed(r, lambda: s.merge_flag_bits(gathered, W))
                    ms[r] += t
                coll.append(("allgather_bits", int(bits[0].numel()) * 8))
                counts = []
                for r, s in enumerate(steppers):
                    c, t = timed(r, s.minedge)
                    counts.append(c)
                    ms[r] += t
            assert len(set(counts)) == 1
            rs = [None] if args.allreduce_hooks or not counts[0] else [s.hook_slots(W) for s in steppers]
            if rs[0] is not None:  # the library loop's reduce-scatter protocol (collectives not timed)
                S = int(rs[0].numel())
                per = S // W
                sign = torch.tensor(-(1 << 63), dtype=torch.int64, device=rs[0].device)
                red = rs[0] ^ sign
                for v in rs[1:]:
                    red = torch.minimum(red, v ^ sign)
                red ^= sign
                for v in rs:
                    v.copy_(red)  # (a rank uses only its own slice)
                coll.append(("reducescatter_min_u64", S * 8))
                pairs = torch.empty(S, dtype=torch.int64, device=rs[0].device)
                for r, s in enumerate(steppers):
                    _, t = timed(r, lambda: s.hook_owner(r, per, pairs))
                    ms[r] += t
                coll.append(("allgather_pairs", per * 8))
                partial = []
                for r, s in enumerate(steppers):
                    pt, t = timed(r, lambda: s.apply_hooks(pairs))
                    partial.append(pt)
                    ms[r] += t
                tot = sum(pt.clone() for pt in partial)
                for pt in partial:
                    pt.copy_(tot)
                coll.append(("allreduce_sum_u64", 16))
            elif counts[0]:
                slots = [None] if args.no_inplace else [s.best_slots() for s in steppers]
                if slots[0] is not None:  # the library loop's in-place uint64 MIN (not timed)
                    sign = torch.tensor(-(1 << 63), dtype=torch.int64, device=slots[0].device)
                    red = slots[0] ^ sign
                    for v in slots[1:]:
                        red = torch.minimum(red, v ^ sign)
                    red ^= sign
                    for v in slots:
                        v.copy_(red)
                    coll.append(("allreduce_min_u64", int(red.numel()) * 8))
                else:
                    dense = []
                    for r, s in enumerate(steppers):
                        d, t = timed(r, lambda: s.pack(counts[0]).clone())
                        dense.append(d)
                        ms[r] += t
                    red = dense[0]
                    for d in dense[1:]:
                        red = torch.minimum(red, d)
                    coll.append(("allreduce_min_i64", int(red.numel()) * 8))
                    for r, s in enumerate(steppers):
                        _, t = timed(r, lambda: s.unpack(red))
                        ms[r] += t
                hooks = []
                for r, s in enumerate(steppers):
                    h, t = timed(r, lambda: (lambda x: None if x is None else x.clone())(s.hook_local()))
                    hooks.append(h)
                    ms[r] += t
                if hooks[0] is not None:
                    hmax = hooks[0]
                    for h in hooks[1:]:
                        hmax = torch.maximum(hmax, h)
                    coll.append(("allreduce_max_i32", int(hmax.numel()) * 4))
                    for r, s in enumerate(steppers):
                        _, t = timed(r, lambda: s.unpack_hook(hmax))
                        ms[r] += t
            dones = []
            for r, s in enumerate(steppers):
                d, t = timed(r, s.contract)
                dones.append(d)
                ms[r] += t
            assert len(set(dones)) == 1
            done = dones[0]
            rounds.append({"max_rank_ms": round(max(ms), 4), "min_rank_ms": round(min(ms), 4), "collectives": coll})
        res = [s.finish()[0] for s in steppers]
        if kprof is not None:  # records land at finish; solver tags in creation (= rank) order
            recs = _native.profile_read()
            ids = sorted(set(r["solver"] for r in recs))
            kprof = [[defaultdict(float) for _ in range(W)] for _ in range(len(rounds))]
            for rec in recs:
                rk = ids.index(rec["solver"])
                if rec["round"] < len(rounds):
                    kprof[rec["round"]][rk][rec["kernel"]] += rec["ms"]
        if ref_flags is not None:
            flags = torch.empty_like(ref_flags)
            for x in engines:  # owner-written: each rank's own slice
                flags[x.e_lo:x.e_hi] = x.in_mst[x.e_lo:x.e_hi]
            assert torch.equal(flags, ref_flags), "emulated ranks differ from the single-GPU MSF"
            assert all(r.total_weight == rres.total_weight for r in res)
        compute = sum(r["max_rank_ms"] for r in rounds)
        payload = sum(b for r in rounds for _, b in r["collectives"])
        # ring all-reduce: every rank sends (and receives) 2 (N-1)/N of the buffer; ring
        # reduce-scatter (N-1)/N; all-gather of a b-byte contribution per rank: (N-1) b
        def ring(k, b):
            if k.startswith("allgather"):
                return (W - 1) * b
            return (1.0 if k.startswith("reducescatter") else 2.0) * (W - 1) / W * b
        wire = sum(ring(k, b) for r in rounds for k, b in r["collectives"])
        ncoll = sum(len(r["collectives"]) for r in rounds)
        print(json.dumps({"scale": args.scale, "world": W, "rep": rep, "m": e.m, "n": e.n,
                          "single_gpu_ms": one_ms and round(one_ms, 3), "rounds": len(rounds),
                          "sum_max_rank_compute_ms": round(compute, 3), "collective_bytes": payload,
                          "wire_bytes_per_rank": int(wire), "collectives": ncoll,
                          "projected_ms_busbw_300": round(compute + wire / 300e9 * 1e3 + ncoll * 0.02, 3),
                          "projection_note": "compute + wire bytes per rank / 300 GB/s ring bus bandwidth + "
                                             "20 us latency per collective (assumptions, not measured)",
                          "per_round": rounds}), flush=True)
        if kprof is not None:
            tot = defaultdict(float)
            for i, per_rank in enumerate(kprof):
                worst = max(range(W), key=lambda r: sum(per_rank[r].values()))
                ks = per_rank[worst]
                for k, v in ks.items():
                    tot[k] += v
                print(f"# round {i}: rank {worst} kernels {sum(ks.values()):.3f} ms of {rounds[i]['max_rank_ms']:.3f} | " +
                      " ".join(f"{k}={v:.3f}" for k, v in sorted(ks.items(), key=lambda kv: -kv[1]) if v >= 0.005),
                      file=sys.stderr)
            if args.per_rank:  # every rank's kernels in the rounds that open a level (balance)
                for i, per_rank in enumerate(kprof):
                    if len(rounds[i]["collectives"]) < 2:
                        continue
                    for rk in range(W):
                        ks = per_rank[rk]
                        print(f"#   round {i} rank {rk}: {sum(ks.values()):.3f} ms | " +
                              " ".join(f"{k}={v:.3f}" for k, v in sorted(ks.items(), key=lambda kv: -kv[1])[:6]),
                              file=sys.stderr)
            kmax = sum(max(sum(pr[rk].values()) for rk in range(W)) for pr in kprof)
            print(f"# kernels only: sum over rounds of the max rank's kernel time {kmax:.3f} ms "
                  f"(the stepwise calls' host round trips are the rest of sum_max_rank_compute_ms)", file=sys.stderr)
            print("# per solve (max rank per round): " + " ".join(f"{k}={v:.3f}" for k, v in
                                                                  sorted(tot.items(), key=lambda kv: -kv[1])),
                  file=sys.stderr)
            _native.profile_enable(False)
            kprof = None
    for s in steppers:
        s.close()


if __name__ == "__main__":
    main()
