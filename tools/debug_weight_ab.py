"""Debug aid: one graph's totals through a given tree's package (A/B of two builds):
python tools/debug_weight_ab.py ROOT SCALE EF"""
import os
import sys


def main():
    root = os.path.abspath(sys.argv[1])
    sys.path.insert(0, root)
    sys.path.insert(1, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # the oracle
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
    from oracle import oracle
    print("package", _native.LIB_PATH, "abi", _native.ABI_VERSION, flush=True)
    sc, ef = int(sys.argv[2]), int(sys.argv[3])
    e = generate_rmat(sc, ef, seed=5, wseed=6)
    g = e.to_host()
    _, ref_tw, ref_k = oracle.kruskal_c(g.n, g.u, g.v, g.w)
    print("oracle", ref_tw, ref_k, flush=True)
    for name, opt in (("default", 0), ("no_bucketed", _native.OPT_NO_BUCKETED), ("bucketed", _native.OPT_BUCKETED)):
        for levels in (None, 2, 3):
            kw = {} if levels is None else {"max_levels": levels}
            a = DeviceMST(e, config=_native.make_config(options=opt, **kw))
            ra, _ = a.run()
            print(name, levels, "levels", ra.levels, ra.total_weight, ra.num_mst_edges, "ok", ra.total_weight == ref_tw,
                  flush=True)


if __name__ == "__main__":
    main()
