"""Debug aid: the totals of one graph through the pipelined one-shot solve and the stepwise API
(synchronous counters), with the level-open diagnostics (GHS_OPT_DEBUG)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from distributed_ghs_implementation_amd import _native
    from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
    from distributed_ghs_implementation_amd.distributed import HipStepper, run_rounds
    from oracle import oracle
    sc, ef = int(sys.argv[1]), int(sys.argv[2])
    e = generate_rmat(sc, ef, seed=5, wseed=6)
    g = e.to_host()
    _, ref_tw, ref_k = oracle.kruskal_c(g.n, g.u, g.v, g.w)
    print("oracle", ref_tw, ref_k, flush=True)
    for opt in (_native.OPT_DEBUG, _native.OPT_DEBUG | _native.OPT_NO_TAIL | _native.OPT_NO_BUCKETED):
        a = DeviceMST(e, config=_native.make_config(options=opt))
        ra, _ = a.run()
        print("one-shot", opt, ra.total_weight, ra.num_mst_edges, flush=True)
        b = DeviceMST(e, config=_native.make_config(options=opt))
        st = HipStepper(b)
        run_rounds(st, lambda t: None)
        rb, _ = st.finish()
        st.close()
        print("stepwise", opt, rb.total_weight, rb.num_mst_edges, flush=True)


if __name__ == "__main__":
    main()
