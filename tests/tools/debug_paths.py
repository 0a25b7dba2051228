"""Which path options give the oracle's MSF on one graph (debug aid): every combination of the
tail and the bucketed rounds, each level plan; prints mismatch counts and the round stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_grid, generate_rmat
    from oracle import oracle
    spec = sys.argv[1] if len(sys.argv) > 1 else "rmat:20:24"
    kind, a, b = (spec.split(":") + ["16"])[:3]
    e = generate_rmat(int(a), int(b), seed=5, wseed=6) if kind == "rmat" else generate_grid(int(a), int(b))
    g = e.to_host()
    ref_in, ref_tw, ref_k = oracle.kruskal_c(g.n, g.u, g.v, g.w)
    ref_in = ref_in.astype(bool)
    opts = {"default": 0, "no_tail": _native.OPT_NO_TAIL, "no_bucketed": _native.OPT_NO_BUCKETED,
            "neither": _native.OPT_NO_TAIL | _native.OPT_NO_BUCKETED, "bucketed": _native.OPT_BUCKETED,
            "bucketed_no_tail": _native.OPT_BUCKETED | _native.OPT_NO_TAIL}
    for levels in [int(x) if x != "None" else None for x in os.environ.get("LEVELS", "None,1,2").split(",")]:
        for name, opt in opts.items():
            kw = {} if levels is None else {"max_levels": levels}
            eng = DeviceMST(e, config=_native.make_config(options=opt, **kw))
            res, stats = eng.run()
            got = eng.in_mst_host()
            bad = int((got != ref_in).sum())
            host_w = int(g.w[got].astype(np.uint64).sum())
            print(f"levels={levels} {name:18s} flags {res.pass_flags:2d} rounds {res.rounds:2d} levels {res.levels} "
                  f"weight_ok {res.total_weight == ref_tw} ({res.total_weight} vs {ref_tw}, flags sum {host_w}) "
                  f"edges {res.num_mst_edges}/{ref_k} mismatched {bad}", flush=True)
            if (bad or res.total_weight != ref_tw) and name in ("default", "neither"):
                for i, st in enumerate(stats):
                    print("   ", i, st)
            del eng


if __name__ == "__main__":
    main()
