"""bench.py's per-kernel byte model and stage-1 roofline on synthetic launch records (no GPU):
the windowed level-0 round (k_wmin) against its device-side fallback (k_bucket / k_bmin), and the
PMC kernel-name match of the templated kernels."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402

N = 1 << 20
STATS = [{"level": 0, "live_arcs": 2 * N, "active_components": N, "level_arcs": 2 * N, "hooks": N // 2},
         {"level": 0, "live_arcs": N, "active_components": N // 4, "level_arcs": 0, "hooks": N // 8}]


def _rec(kernel, ms, rnd=0):
    return {"kernel": kernel, "ms": ms, "round": rnd, "level": 0, "items": 0}


class _Res:
    def __init__(self, pass_flags):
        self.pass_flags = pass_flags


def test_windowed_round_charges_k_wmin_only():
    """pass_flags bit 2 (the library's span flag): level 0's round 0 ran windowed —
    even where the fallback launches took longer than k_wmin, the bytes go to k_wmin."""
    recs = [_rec("k_wstarts", 0.01), _rec("k_wmin", 1.0), _rec("k_bucket", 2.0), _rec("k_bmin", 2.0)]
    tab = bench.kernel_table(recs, STATS, _Res(bench.PASS_WINDOWED), N)
    assert tab["k_wmin"]["bytes"] == 32.0 * 2 * N + 12.0 * N
    assert tab["k_bucket"]["bytes"] == 0.0 and tab["k_bmin"]["bytes"] == 0.0


def test_fallback_round_charges_the_bucketed_kernels():
    recs = [_rec("k_wstarts", 0.01), _rec("k_wmin", 0.003), _rec("k_bucket", 0.8), _rec("k_bmin", 0.9)]
    tab = bench.kernel_table(recs, STATS, _Res(0), N)
    assert tab["k_wmin"]["bytes"] == 0.0
    assert tab["k_bucket"]["bytes"] > 0 and tab["k_bmin"]["bytes"] > 0


def test_stage1_counts_the_windowed_kernels():
    recs = [_rec("k_wstarts", 0.01), _rec("k_wmin", 1.0), _rec("k_minedge<COMPACT>", 0.5, 1)]
    s1 = bench.stage1_roofline(recs, STATS)
    assert abs(s1["ms"] - 1.51) < 1e-9
    assert s1["live_edges"] == 3 * N
    assert "k_wmin" in s1["kernels"]


def test_pmc_names_match_templated_kernels():
    assert bench._pmc_match("k_wmin", "k_wmin<14u>")
    assert bench._pmc_match("k_bmin", "k_bmin<13u, false>")
    assert bench._pmc_match("k_minedge<COMPACT>", "k_minedge<false, true, false, true>")
    assert not bench._pmc_match("k_minedge<IDENT>", "k_minedge<false, true, false, true>")


def test_auto_input_form():
    """auto: both forms at N = 1 on graphs with m >= 4n (R-MAT s24: m/n = 15.5), COO on the grids
    (m/n = 2) and at N > 1; an explicit form is kept."""
    assert bench.input_form("auto", 1, 1 << 24, 260383859) == "both"
    assert bench.input_form("auto", 1, 16384 * 16384, 536838144) == "coo"
    assert bench.input_form("auto", 8, 1 << 26, 1051916369) == "coo"
    assert bench.input_form("csr", 8, 10, 5) == "csr"


class _Cnt:
    canon_edges = 1000
    select_out = 10
    filter_out = 20


def test_stream_byte_model_per_form():
    n = 100
    try:
        bench.set_stream_forms(True, True, 1)  # both: CSR select, COO filter
        assert bench._stream_bytes(_Cnt, n, "select") == 8.0 * 1000 + 4.0 * (n + 1)
        assert bench._stream_bytes(_Cnt, n, "filter") == 12.0 * 1000
        assert bench._pmc_match("k_select", "k_select<true>") and bench._pmc_match("k_filter", "k_filter<false>")
        bench.set_stream_forms(True, False, 4)  # CSR alone, a rank of 4: a quarter of the rows
        assert bench._stream_bytes(_Cnt, n, "filter") == 8.0 * 1000 + 1.0 * (n + 1)
        assert bench._pmc_match("k_filter", "k_filter<true>") and not bench._pmc_match("k_filter", "k_filter<false>")
    finally:
        bench.set_stream_forms(False, True, 1)
    assert bench._stream_bytes(_Cnt, n, "select") == 12.0 * 1000
    assert bench._pmc_match("k_select", "k_select<false>") and not bench._pmc_match("k_select", "k_select<true>")
