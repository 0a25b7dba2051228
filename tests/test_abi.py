"""The C-ABI boundary without a GPU: the library loads, exports every symbol include/ghs_mst.h
declares, and the compute entry points fail loudly (no CPU fallback) when no GPU is visible."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from distributed_ghs_implementation_amd import _native

HEADER = os.path.join(ROOT, "include", "ghs_mst.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ghs_[a-z_]+)\s*\(", src)))


def test_header_lists_match_binding():
    assert header_functions() == sorted(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\sT\s(ghs_\w+)", out))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing


def test_library_loads_and_reports_abi():
    L = _native.load()
    assert L.ghs_abi_version() == _native.ABI_VERSION == 10
    assert _native.device_count() >= 0


def test_config_struct_and_no_environment_knobs():
    """ghs_config_t (ABI 5) carries every path option; the default config is the default path,
    and the shipped library names no GHS_* environment variable (A/B launch-shape knobs exist only
    in `make AB=1` builds)."""
    L = _native.load()
    assert ctypes.sizeof(_native.Config) == 40
    c = _native.make_config()
    assert (c.options, c.dedup_max, c.fault_rank, c.fault_round, c.max_levels, c.num_ranks) == (0, 0, 0, 0, 8, 1)
    assert ctypes.sizeof(_native.Result) == 104  # ABI 7: + ms_setup / ms_solve / ms_gather / reused
    blob = open(_native.LIB_PATH, "rb").read()
    for knob in (b"GHS_LOOKAHEAD", b"GHS_HV", b"GHS_DEDUP_MAX", b"GHS_SEED_RUNS", b"GHS_DENSE", b"GHS_SEG_G",
                 b"GHS_MINEDGE_G", b"GHS_DEBUG", b"GHS_DETAIL", b"GHS_TIME_ROUNDS"):
        assert knob not in blob, knob
    del L


def test_sizes_are_sane():
    L = _native.load()
    assert L.ghs_workspace_bytes(1000, 5000, 10000) >= 1000 * 20 + 10000 * 32
    assert L.ghs_rmat_temp_bytes(10, 16) >= 2 * 16 * 1024 * 8


def test_rank_limits_rejected():
    """GHS_MAX_RANKS bounds every multi-rank entry before any device work (the
    reduce-scatter padding lives in 64 spare slots)."""
    L = _native.load()
    h = ctypes.c_void_p(0)
    uid = (ctypes.c_uint8 * _native.GHS_COMM_ID_BYTES)()
    assert L.ghs_comm_init(65, 0, uid, ctypes.byref(h)) == _native.GHS_E_ARG
    assert L.ghs_comm_init(2, 2, uid, ctypes.byref(h)) == _native.GHS_E_ARG
    assert L.ghs_mst_emulated(4, 0, None, None, None, 65, None, None, None, None) == _native.GHS_E_ARG
    assert L.ghs_release_cache() == _native.GHS_OK


def test_slot_retries_diagnostic():
    """ABI 8: the count of round reports re-read for a failed checksum (a process-wide counter: any
    earlier solve in this process may have added to it — ADVICE r05)."""
    assert _native.slot_retries() >= 0
    L = _native.load()
    assert L.ghs_slot_retries(None) == _native.GHS_E_ARG


def test_null_arguments_rejected():
    L = _native.load()
    res = _native.Result()
    rc = L.ghs_mst_host(3, 2, None, None, None, None, ctypes.byref(res), None)
    assert rc == _native.GHS_E_ARG
    assert b"NULL" in L.ghs_last_error()


@pytest.mark.skipif(_native.device_count() > 0, reason="CPU-only behaviour")
def test_no_cpu_fallback_without_gpu():
    from distributed_ghs_implementation_amd import GHSAlgorithm
    with pytest.raises(_native.GHSError) as ei:
        GHSAlgorithm(3, [(0, 1, 1), (0, 2, 2)]).run()
    assert ei.value.code == _native.GHS_E_NODEVICE
    L = _native.load()
    u = np.array([0], np.uint32)
    v = np.array([1], np.uint32)
    w = np.array([1], np.uint32)
    f = np.zeros(1, np.uint8)
    assert L.ghs_mst_host(2, 1, u.ctypes.data, v.ctypes.data, w.ctypes.data, f.ctypes.data, None, None) \
        == _native.GHS_E_NODEVICE


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "distributed_ghs_implementation_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(dirpath, fn)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle\b", text, re.M), fn
                assert "liboracle" not in text, fn
