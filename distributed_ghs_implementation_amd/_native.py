"""ctypes binding of libghs_mst.so (the C-ABI declared in include/ghs_mst.h).

The product path has exactly one implementation of the MST: the gfx950 HIP kernels in this
library. There is no CPU fallback — if the library is missing or no GPU is visible, every
compute entry point raises. (The CPU restatement used to CHECK results lives in oracle/, which
this package never imports.)
"""
import atexit
import collections.abc
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GHS_MST_LIB", os.path.join(_HERE, "lib", "libghs_mst.so"))

GHS_OK = 0
GHS_NEED_EXCHANGE = 1  # positive status of ghs_solver_minedge (several ranks opened a level)
GHS_E_ARG = -1
GHS_E_NONCANON = -2
GHS_E_HIP = -3
GHS_E_ROUNDCAP = -4
GHS_E_NODEVICE = -5
GHS_E_NOMEM = -6
GHS_E_STATE = -7
GHS_MAX_ROUND_STATS = 64

_ERR_NAMES = {
    GHS_E_ARG: "GHS_E_ARG", GHS_E_NONCANON: "GHS_E_NONCANON", GHS_E_HIP: "GHS_E_HIP",
    GHS_E_ROUNDCAP: "GHS_E_ROUNDCAP", GHS_E_NODEVICE: "GHS_E_NODEVICE", GHS_E_NOMEM: "GHS_E_NOMEM",
    GHS_E_STATE: "GHS_E_STATE",
}

# every symbol include/ghs_mst.h declares (tests check the .so exports all of them)
EXPORTED_SYMBOLS = (
    "ghs_abi_version", "ghs_last_error", "ghs_device_count", "ghs_mst_host", "ghs_mst_multi",
    "ghs_default_config", "ghs_workspace_bytes", "ghs_mst_device",
    "ghs_check_canonical",
    "ghs_solver_create", "ghs_solver_minedge", "ghs_solver_exchange_buffer", "ghs_solver_pack_best",
    "ghs_solver_flag_bits", "ghs_solver_merge_flag_bits",
    "ghs_solver_unpack_best", "ghs_solver_best_slots",
    "ghs_solver_contract", "ghs_solver_finish", "ghs_solver_reset", "ghs_solver_cancel", "ghs_solver_destroy",
    "ghs_solver_hook_local", "ghs_solver_unpack_hook",
    "ghs_solver_hook_slots", "ghs_solver_hook_owner", "ghs_solver_apply_hooks", "ghs_solver_tail_begin",
    "ghs_solver_tail_buffers", "ghs_solver_tail_agree", "ghs_solver_tail_round",
    "ghs_rmat_temp_bytes", "ghs_rmat_generate", "ghs_rmat_tuples", "ghs_grid_generate",
    "ghs_profile_enable", "ghs_profile_read", "ghs_kernel_name",
    "ghs_comm_unique_id", "ghs_comm_init", "ghs_comm_destroy", "ghs_solver_run", "ghs_mst_emulated",
    "ghs_release_cache", "ghs_slot_retries", "ghs_flags_to_eids",
    "ghs_mst_device_csr", "ghs_csr_offsets", "ghs_solver_create_csr",
)


class GHSError(RuntimeError):
    """A negative GHS_E_* return code from libghs_mst.so."""

    def __init__(self, code, message):
        super().__init__(f"{_ERR_NAMES.get(code, code)}: {message}")
        self.code = code


class RoundStats(ctypes.Structure):
    _fields_ = [
        ("level", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("level_arcs", ctypes.c_uint64),
        ("live_arcs", ctypes.c_uint64),
        ("active_components", ctypes.c_uint64),
        ("hooks", ctypes.c_uint64),
        ("ms_minedge", ctypes.c_float),
        ("ms_hook", ctypes.c_float),
        ("ms_jump", ctypes.c_float),
        ("ms_active", ctypes.c_float),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}


class RoundStatsList(collections.abc.Sequence):
    """The per-round stats of one solve as a read-only sequence of dicts, converted on access
    (a solve returns up to 64 rounds; building every dict eagerly cost ~27 us per solve)."""

    def __init__(self, arr, n):
        self._arr, self._n = arr, int(n)

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        return self._arr[i].as_dict()

    def __repr__(self):
        return repr(list(self))


ABI_VERSION = 10  # include/ghs_mst.h GHS_MST_ABI_VERSION


class Result(ctypes.Structure):
    _fields_ = [
        ("num_mst_edges", ctypes.c_uint64),
        ("total_weight", ctypes.c_uint64),
        ("rounds", ctypes.c_uint32),
        ("num_stats", ctypes.c_uint32),
        ("levels", ctypes.c_uint32),
        ("pass_flags", ctypes.c_uint32),
        ("ms_total", ctypes.c_double),
        ("ms_select", ctypes.c_float),
        ("ms_filter", ctypes.c_float),
        ("canon_edges", ctypes.c_uint64),
        ("select_out", ctypes.c_uint64),
        ("filter_out", ctypes.c_uint64),
        # ABI 7: the multi-rank drivers' host phases (max over ranks) and cache reuse
        ("ms_setup", ctypes.c_double),
        ("ms_solve", ctypes.c_double),
        ("ms_gather", ctypes.c_double),
        ("reused", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]


class KernelRecord(ctypes.Structure):
    """ghs_kernel_record_t: one profiled launch (ghs_profile_enable / ghs_profile_read)."""
    _fields_ = [
        ("kernel", ctypes.c_uint32),
        ("round", ctypes.c_uint32),
        ("level", ctypes.c_uint32),
        ("solver", ctypes.c_uint32),
        ("items", ctypes.c_uint64),
        ("ms", ctypes.c_float),
        ("reserved2", ctypes.c_float),
    ]


def profile_enable(on=True):
    check(load().ghs_profile_enable(1 if on else 0))


def profile_read():
    """Drain the per-launch profile: [{"kernel": name, "round", "level", "items", "ms"}, ...]."""
    L = load()
    out = []
    while True:
        buf = (KernelRecord * 4096)()
        c = ctypes.c_uint32(0)
        check(L.ghs_profile_read(buf, 4096, ctypes.byref(c)))
        for i in range(c.value):
            r = buf[i]
            out.append({"kernel": L.ghs_kernel_name(r.kernel).decode(), "round": r.round, "level": r.level,
                        "solver": r.solver, "items": r.items, "ms": r.ms})
        if c.value < 4096:
            return out


# ghs_config_t.options bits (include/ghs_mst.h GHS_OPT_*)
OPT_NO_SEED_RUNS = 0x1
OPT_NO_DENSE = 0x2
OPT_BUCKETED = 0x4
OPT_NO_BUCKETED = 0x8
OPT_DEBUG = 0x10
OPT_TIME_ROUNDS = 0x20
OPT_DETAIL = 0x40
OPT_BUCKETED_FIRST = 0x80
OPT_NO_WINDOW = 0x100
OPT_NO_TAIL = 0x200
OPT_CHECK_TOTALS = 0x400  # ABI 8: per level, report totals vs a stream-ordered copy of the counters
OPT_KEEP_CACHE = 0x800    # ABI 8: the multi-rank drivers keep their per-rank state for the next call

# ghs_result_t.pass_flags bits
PASS_BUCKETED = 0x1
PASS_LATTICE = 0x2
PASS_WINDOWED = 0x4
PASS_TAIL = 0x8


class Config(ctypes.Structure):
    """ghs_config_t: the weight-level plan of the filter and the path options (speed only;
    results never change). The library reads no environment variable that changes its path."""
    _fields_ = [
        ("max_levels", ctypes.c_uint32),
        ("num_ranks", ctypes.c_uint32),
        ("level1_edges_per_vertex", ctypes.c_double),
        ("level_growth", ctypes.c_double),
        ("options", ctypes.c_uint32),
        ("dedup_max", ctypes.c_uint32),
        ("fault_rank", ctypes.c_uint32),
        ("fault_round", ctypes.c_uint32),
    ]


def make_config(max_levels=None, level1_edges_per_vertex=None, level_growth=None, num_ranks=None, options=None,
                dedup_max=None, fault_rank=None, fault_round=None):
    c = Config()
    load().ghs_default_config(ctypes.byref(c))
    if options is not None:
        c.options = int(options)
    if dedup_max is not None:
        c.dedup_max = int(dedup_max)
    if fault_rank is not None:
        c.fault_rank = int(fault_rank)
    if fault_round is not None:
        c.fault_round = int(fault_round)
    if num_ranks is not None:
        c.num_ranks = int(num_ranks)
    if max_levels is not None:
        c.max_levels = int(max_levels)
    if level1_edges_per_vertex is not None:
        c.level1_edges_per_vertex = float(level1_edges_per_vertex)
    if level_growth is not None:
        c.level_growth = float(level_growth)
    return c


_lib = None
_lock = threading.Lock()


def load():
    """Load the library once; raise loudly if it is missing (no fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        # Load torch's HIP runtime first when torch is installed: libghs_mst.so then binds to the
        # same libamdhip64.so.7 (same SONAME) instead of bringing up a second runtime, so torch's
        # device pointers and streams are valid in both.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libghs_mst.so not found at {LIB_PATH}; build it with "
                "`make -C distributed_ghs_implementation_amd/csrc` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        u32, u64, i32, sz, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
        P = ctypes.POINTER
        sigs = {
            "ghs_abi_version": (i32, []),
            "ghs_last_error": (ctypes.c_char_p, []),
            "ghs_device_count": (i32, [P(i32)]),
            "ghs_mst_host": (i32, [u32, u64, vp, vp, vp, vp, P(Result), P(RoundStats)]),
            "ghs_mst_multi": (i32, [u32, u64, vp, vp, vp, i32, vp, vp, vp, P(Result), P(RoundStats)]),
            "ghs_default_config": (None, [P(Config)]),
            "ghs_check_canonical": (i32, [u32, u64, vp, vp, vp, P(i32)]),
            "ghs_workspace_bytes": (sz, [u32, u64, u64]),
            "ghs_mst_device": (i32, [u32, u64, vp, vp, vp, P(Config), vp, sz, vp, vp, P(Result), P(RoundStats)]),
            "ghs_solver_create": (i32, [u32, u64, vp, vp, vp, u64, u64, P(Config), vp, sz, vp, vp, P(vp)]),
            "ghs_solver_minedge": (i32, [vp, P(u64)]),
            "ghs_solver_exchange_buffer": (i32, [vp, P(vp), P(u64)]),
            "ghs_solver_flag_bits": (i32, [vp, P(vp), P(u64)]),
            "ghs_solver_merge_flag_bits": (i32, [vp, vp, u32]),
            "ghs_solver_pack_best": (i32, [vp, vp]),
            "ghs_solver_unpack_best": (i32, [vp, vp]),
            "ghs_solver_best_slots": (i32, [vp, P(vp), P(u64)]),
            "ghs_solver_contract": (i32, [vp, P(i32)]),
            "ghs_solver_finish": (i32, [vp, P(Result), P(RoundStats)]),
            "ghs_solver_hook_local": (i32, [vp, vp, P(ctypes.c_uint64)]),
            "ghs_solver_unpack_hook": (i32, [vp, vp]),
            "ghs_solver_hook_slots": (i32, [vp, u32, P(vp), P(u64)]),
            "ghs_solver_hook_owner": (i32, [vp, u32, u64, vp]),
            "ghs_solver_apply_hooks": (i32, [vp, vp, P(vp)]),
            "ghs_solver_tail_begin": (i32, [vp, P(u64)]),
            "ghs_solver_tail_buffers": (i32, [vp, P(vp), P(vp)]),
            "ghs_solver_tail_agree": (i32, [vp]),
            "ghs_solver_tail_round": (i32, [vp, P(i32)]),
            "ghs_solver_reset": (i32, [vp]),
            "ghs_solver_cancel": (i32, [vp]),
            "ghs_solver_destroy": (i32, [vp]),
            "ghs_rmat_temp_bytes": (sz, [u32, u32]),
            "ghs_rmat_generate": (i32, [u32, u32, u64, u64, vp, vp, vp, P(u64), vp, sz, vp]),
            "ghs_rmat_tuples": (i32, [u32, u32, u64, vp, vp]),
            "ghs_profile_enable": (i32, [i32]),
            "ghs_profile_read": (i32, [vp, u32, P(u32)]),
            "ghs_kernel_name": (ctypes.c_char_p, [u32]),
            "ghs_grid_generate": (i32, [u32, u32, u64, vp, vp, vp, vp]),
            "ghs_comm_unique_id": (i32, [vp]),
            "ghs_comm_init": (i32, [i32, i32, vp, P(vp)]),
            "ghs_comm_destroy": (i32, [vp]),
            "ghs_solver_run": (i32, [vp, vp]),
            "ghs_mst_emulated": (i32, [u32, u64, vp, vp, vp, i32, P(Config), vp, P(Result), P(RoundStats)]),
            "ghs_release_cache": (i32, []),
            "ghs_slot_retries": (i32, [P(u64)]),
            "ghs_flags_to_eids": (i32, [vp, u64, u64, vp, u64, P(u64), vp]),
            # ABI 9: the CSR form of the canonical list
            "ghs_mst_device_csr": (i32, [u32, u64, vp, vp, vp, vp, P(Config), vp, sz, vp, vp, P(Result), P(RoundStats)]),
            "ghs_csr_offsets": (i32, [u32, u64, vp, vp, vp]),
            "ghs_solver_create_csr": (i32, [u32, u64, vp, vp, vp, vp, u64, u64, P(Config), vp, sz, vp, vp, P(vp)]),
        }
        for name, (res, args) in sigs.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.ghs_abi_version() != ABI_VERSION:
            raise ImportError(f"libghs_mst.so ABI {L.ghs_abi_version()} != {ABI_VERSION}")
        _lib = L
        # a driver call with OPT_KEEP_CACHE leaves per-rank workspaces (and an RCCL clique) cached:
        # free them before the interpreter tears the HIP runtime down
        atexit.register(_release_at_exit)
        return _lib


def _release_at_exit():
    if _lib is not None:
        try:
            _lib.ghs_release_cache()
        except Exception:
            pass


def check(rc):
    """Raise GHSError for a negative return code (positive statuses are returned)."""
    if rc < GHS_OK:
        msg = load().ghs_last_error()
        raise GHSError(rc, msg.decode() if msg else "")
    return rc


GHS_COMM_ID_BYTES = 128  # include/ghs_mst.h


def comm_unique_id():
    """Rank 0's RCCL unique id (bytes) for ghs_comm_init on every rank."""
    buf = (ctypes.c_uint8 * GHS_COMM_ID_BYTES)()
    check(load().ghs_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """ghs_comm_t: one rank's RCCL communicator for ghs_solver_run (bound to the current device)."""

    def __init__(self, nranks, rank, uid):
        if len(uid) != GHS_COMM_ID_BYTES:
            raise ValueError("the unique id must be GHS_COMM_ID_BYTES bytes")
        buf = (ctypes.c_uint8 * GHS_COMM_ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p(0)
        check(load().ghs_comm_init(int(nranks), int(rank), buf, ctypes.byref(h)))
        self.h = h
        self.nranks, self.rank = int(nranks), int(rank)

    def close(self):
        if self.h:
            load().ghs_comm_destroy(self.h)
            self.h = ctypes.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def release_cache():
    """Free the multi-rank drivers' cached per-rank state (ghs_release_cache)."""
    check(load().ghs_release_cache())


def slot_retries():
    """Round reports the host re-read because their checksum failed (seq landed before a field)."""
    c = ctypes.c_uint64(0)
    check(load().ghs_slot_retries(ctypes.byref(c)))
    return c.value


def device_count():
    c = ctypes.c_int(0)
    check(load().ghs_device_count(ctypes.byref(c)))
    return c.value


def require_gpu():
    """The product path runs only on a GPU: fail loudly, never fall back to the CPU."""
    if device_count() == 0:
        raise GHSError(GHS_E_NODEVICE, "no HIP device visible: the MST engine runs only on MI355X (gfx950)")
