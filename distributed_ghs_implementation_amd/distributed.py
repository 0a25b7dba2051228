"""Multi-GPU MST: one process per GPU, torch.distributed (backend "nccl" == RCCL over xGMI).

Replaces the reference's MPI path (ghs_implementation_mpi.py:884-954: one rank PER VERTEX,
pickled point-to-point messages, bcast/Barrier/gather) with one rank per GPU and ONE collective
per round:

  * partition: rank r owns the contiguous canonical-edge range [r*m/N, (r+1)*m/N) and streams
    only ITS edges through the level passes; the canonical edge list (to resolve a chosen
    edge's endpoints) and the fragment state are replicated;
  * per level: the fragments with a level edge on ANY rank form the identical active list of
    every rank — each rank's n flags packed to a bitmap and all-gathered (OR-ed on the device),
    (n + 1) / 8 bytes per rank (or the n + 1 flag bytes all-reduced with MAX);
    the level then runs in dense labels 0..nact0-1 (boruvka.hip k_dense_open);
  * per round: local min-edge over the rank's level edges -> dense best[] slots of the active
    fragments -> all_reduce(MIN) -> identical hook / pointer-jump / next-list on every rank;
    in a level's first round the hook is owner-computes: each rank hooks the fragments whose
    winning edge it holds and the int32 parent slots are combined with all_reduce(MAX);
  * result: the totals are identical on every rank by construction (same inputs, same
    decisions); every MSF flag is written by the rank that owns its edge, each rank clearing and
    writing only its own range, so the flags are assembled on demand (`gather_in_mst`: an
    all-gather of the ranks' slices, outside the solve) and rank 0 writes the output (the
    reference gathered BRANCH edges to rank 0, ghs_implementation_mpi.py:760-779).

The round loop (`run_rounds`) is written against a small stepper interface so that the same
orchestration can be exercised on CPU with the gloo backend in tests (tests inject a CPU
stepper from oracle/); the product stepper is `HipStepper` (libghs_mst.so).
"""
import ctypes
import hashlib
import threading

import torch
import torch.distributed as dist

from . import _native
from .device import DeviceEdges, DeviceMST, _ptr, _stream, edge_range, flags_to_eids  # noqa: F401


class HipStepper:
    """The stepwise solver of include/ghs_mst.h (ghs_solver_*) over one rank's arcs."""

    def __init__(self, engine):
        self.e = engine
        L = self.L = engine.L
        ed = engine.edges
        h = ctypes.c_void_p(0)
        if getattr(engine, "csr", False):  # ABI 9: the rank streams (off, v, w)
            _native.check(L.ghs_solver_create_csr(ed.n, ed.m, _ptr(ed.off), _ptr(ed.u), _ptr(ed.v), _ptr(ed.w),
                                                  engine.e_lo, engine.e_hi, ctypes.byref(engine.config), _ptr(engine.ws),
                                                  engine.ws_bytes, _ptr(engine.in_mst), _stream(), ctypes.byref(h)))
        else:
            _native.check(L.ghs_solver_create(ed.n, ed.m, _ptr(ed.u), _ptr(ed.v), _ptr(ed.w), engine.e_lo, engine.e_hi,
                                              ctypes.byref(engine.config), _ptr(engine.ws), engine.ws_bytes,
                                              _ptr(engine.in_mst), _stream(), ctypes.byref(h)))
        self.h = h
        self.dense = torch.empty(max(ed.n, 1), dtype=torch.int64, device=ed.device)
        self.dense_hook = torch.empty(max(ed.n, 1), dtype=torch.int32, device=ed.device)

    def minedge(self):
        """Local min-edge of the round; None when a level was opened and its fragment flags must
        be OR-combined across ranks first (exchange_buffer, then minedge again)."""
        c = ctypes.c_uint64(0)
        rc = _native.check(self.L.ghs_solver_minedge(self.h, ctypes.byref(c)))
        if rc == _native.GHS_NEED_EXCHANGE:
            return None
        return int(c.value)

    def exchange_buffer(self):
        """The level's active-fragment flags (uint8, n + 1 with the error byte) as a torch view to
        all-reduce with MAX."""
        p = ctypes.c_void_p(0)
        nb = ctypes.c_uint64(0)
        _native.check(self.L.ghs_solver_exchange_buffer(self.h, ctypes.byref(p), ctypes.byref(nb)))
        return _device_u8_view(p.value, int(nb.value), self.e.edges.device, self.e.ws)

    def flag_bits(self):
        """The same flags packed to int64 bitmap words (a view of the workspace) to all-gather."""
        p = ctypes.c_void_p(0)
        nw = ctypes.c_uint64(0)
        _native.check(self.L.ghs_solver_flag_bits(self.h, ctypes.byref(p), ctypes.byref(nw)))
        return _device_u8_view(p.value, 8 * int(nw.value), self.e.edges.device, self.e.ws).view(torch.int64)

    def merge_flag_bits(self, gathered, nranks):
        """OR the all-gathered bitmaps (rank-major, contiguous) into the level's flags."""
        gathered = gathered.contiguous()
        _native.check(self.L.ghs_solver_merge_flag_bits(self.h, _ptr(gathered), int(nranks)))
        self._keep = gathered  # alive until the stream has consumed it (next call syncs)

    def pack(self, count):
        _native.check(self.L.ghs_solver_pack_best(self.h, _ptr(self.dense)))
        return self.dense[:count]

    def unpack(self, dense):
        _native.check(self.L.ghs_solver_unpack_best(self.h, _ptr(dense)))

    def best_slots(self):
        """A dense level's first round: the solver's own minima as an int64 view of `count` slots
        holding uint64 keys (MIN-reduce them unsigned, in place), or None (use pack / unpack)."""
        p = ctypes.c_void_p(0)
        c = ctypes.c_uint64(0)
        _native.check(self.L.ghs_solver_best_slots(self.h, ctypes.byref(p), ctypes.byref(c)))
        if not p.value:
            return None
        return _device_u8_view(p.value, 8 * int(c.value), self.e.edges.device, self.e.ws).view(torch.int64)

    def hook_local(self):
        """Owner-computes CONNECT of a level's first round: the int32 slots to all-reduce with
        MAX (then unpack_hook), or None when the round hooks inside contract."""
        c = ctypes.c_uint64(0)
        _native.check(self.L.ghs_solver_hook_local(self.h, _ptr(self.dense_hook), ctypes.byref(c)))
        return self.dense_hook[: int(c.value)] if c.value else None

    def unpack_hook(self, dense):
        _native.check(self.L.ghs_solver_unpack_hook(self.h, _ptr(dense)))

    def hook_slots(self, nranks):
        """The reduce-scatter protocol of a dense level's opening round (ABI 6): the best slots,
        padded to a multiple of nranks, as an int64 view holding uint64 keys (MIN-reduce-scatter
        them unsigned, in place), or None (the all-reduce protocol applies)."""
        p = ctypes.c_void_p(0)
        c = ctypes.c_uint64(0)
        _native.check(self.L.ghs_solver_hook_slots(self.h, int(nranks), ctypes.byref(p), ctypes.byref(c)))
        if not c.value:
            return None
        return _device_u8_view(p.value, 8 * int(c.value), self.e.edges.device, self.e.ws).view(torch.int64)

    def hook_owner(self, rank, per, pairs):
        """This rank's hooks (eid << 32 | other fragment) into pairs[rank * per:(rank + 1) * per]."""
        _native.check(self.L.ghs_solver_hook_owner(self.h, int(rank), int(per), _ptr(pairs)))

    def apply_hooks(self, pairs):
        """Every rank's hooks (the all-gathered pairs): par, own-range MSF flags; returns this
        rank's partial totals (an int64 view of 2 words: weight, MSF edges of its own range) to
        SUM-all-reduce in place before contract."""
        p = ctypes.c_void_p(0)
        _native.check(self.L.ghs_solver_apply_hooks(self.h, _ptr(pairs), ctypes.byref(p)))
        return _device_u8_view(p.value, 16, self.e.edges.device, self.e.ws).view(torch.int64)

    def contract(self):
        d = ctypes.c_int(0)
        _native.check(self.L.ghs_solver_contract(self.h, ctypes.byref(d)))
        return bool(d.value)

    # ---- the LDS tail of a dense level (ABI 10, include/ghs_mst.h ghs_solver_tail_*) ----
    def tail_begin(self):
        """0: no tail now (continue with minedge); else F, the tail's fragments: this rank's round-0
        minima are in tail_buffers()[0]."""
        f = ctypes.c_uint64(0)
        _native.check(self.L.ghs_solver_tail_begin(self.h, ctypes.byref(f)))
        return int(f.value)

    def tail_buffers(self, F):
        """(keys: F uint64 as an int64 view — MIN-all-reduce them as UNSIGNED, hooks: F int32 —
        MAX-all-reduce them), device tensors over the solver's workspace."""
        k, h = ctypes.c_void_p(0), ctypes.c_void_p(0)
        _native.check(self.L.ghs_solver_tail_buffers(self.h, ctypes.byref(k), ctypes.byref(h)))
        dev, ws = self.e.edges.device, self.e.ws
        return (_device_u8_view(k.value, 8 * F, dev, ws).view(torch.int64),
                _device_u8_view(h.value, 4 * F, dev, ws).view(torch.int32))

    def tail_agree(self):
        _native.check(self.L.ghs_solver_tail_agree(self.h))

    def tail_round(self):
        """0: the next tail round's minima are in the keys; 1: the level is done; 2: the solve is."""
        st = ctypes.c_int(0)
        _native.check(self.L.ghs_solver_tail_round(self.h, ctypes.byref(st)))
        return int(st.value)

    def run_native(self, comm):
        """The whole round loop in the library (ghs_solver_run): collectives over `comm` (a
        _native.Comm, RCCL on the solver's stream), one host call per solve."""
        _native.check(self.L.ghs_solver_run(self.h, comm.h if comm is not None else None))

    def finish(self):
        res = _native.Result()
        stats = (_native.RoundStats * _native.GHS_MAX_ROUND_STATS)()
        _native.check(self.L.ghs_solver_finish(self.h, ctypes.byref(res), stats))
        return res, _native.RoundStatsList(stats, res.num_stats)

    def reset(self):
        """Start the next solve on the same handle (no new host resources)."""
        _native.check(self.L.ghs_solver_reset(self.h))

    def cancel(self):
        """Thread-safe: end the waits of a ghs_solver_run in progress on another thread (a peer
        rank failed); that call then returns GHS_E_STATE."""
        if self.h:
            self.L.ghs_solver_cancel(self.h)

    def close(self):
        if self.h:
            self.L.ghs_solver_destroy(self.h)
            self.h = ctypes.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def allreduce_min_unsigned(allreduce_min, t):
    """MIN-all-reduce an int64 view of uint64 values as unsigned (the sign bit flipped around a
    signed MIN: order-preserving), in place."""
    sign = torch.tensor(-(1 << 63), dtype=torch.int64, device=t.device)
    t.bitwise_xor_(sign)
    allreduce_min(t)
    t.bitwise_xor_(sign)


def run_rounds(stepper, allreduce_min, max_rounds=4096, allreduce_max=None, allgather=None, rs=None):
    """The level loop shared by every backend: (level open: OR the fragment flags), min-edge,
    all-reduce MIN, (a level's first round: owner-computes hook, all-reduce MAX), contract.

    `rs` (default: allreduce_min.rs when present) enables the library loop's reduce-scatter
    protocol for a level's first round (ABI 6; multi.hip run_loop): hook_slots -> reduce-scatter
    MIN (unsigned) -> hook_owner on this rank's slice -> all-gather of the pairs -> apply_hooks ->
    SUM all-reduce of the partial totals. It needs `rs.world`, `rs.rank`,
    `rs.reduce_scatter_min_u64(t)` (each rank's slice reduced in place), `rs.allgather_slices(t,
    per)` and `rs.allreduce_sum(t)`.

    `allreduce_min(tensor)` / `allreduce_max(tensor)` reduce in place across ranks (identity for
    one rank; allreduce_max defaults to allreduce_min's backend with MAX). `allgather(tensor) ->
    (nranks, tensor)` (default: allreduce_min.gather when present) lets a stepper with bitmap
    flags (flag_bits / merge_flag_bits) exchange (n + 1) / 8 bytes per rank instead of
    all-reducing n + 1 flag bytes. Returns the number of rounds executed (all weight levels).
    Raises RuntimeError past `max_rounds` (hang guard; Boruvka needs at most ceil(log2 n) + 1
    rounds per level)."""
    rounds = 0
    rs = rs or getattr(allreduce_min, "rs", None)
    gather = allgather or getattr(allreduce_min, "gather", None)
    use_bits = gather is not None and hasattr(stepper, "flag_bits")
    tail_begin = getattr(stepper, "tail_begin", None)
    while True:
        # a dense level's LDS tail (ABI 10): per round a MIN of F keys and a MAX of F hooks
        F = tail_begin() if tail_begin is not None else 0
        if F:
            keys, hooks = stepper.tail_buffers(F)
            while True:
                allreduce_min_unsigned(allreduce_min, keys)
                stepper.tail_agree()
                (allreduce_max or allreduce_min.max)(hooks)
                state = stepper.tail_round()
                rounds += 1
                if state:
                    break
            if state == 2:
                return rounds
            continue
        count = stepper.minedge()
        while count is None:  # a level opened: its active fragments = flagged on ANY rank
            if use_bits:
                nranks, gathered = gather(stepper.flag_bits())
                stepper.merge_flag_bits(gathered, nranks)
            else:
                (allreduce_max or allreduce_min.max)(stepper.exchange_buffer())
            count = stepper.minedge()
        slots = None
        if count and rs is not None and getattr(stepper, "hook_slots", None) is not None:
            slots = stepper.hook_slots(rs.world)
        if slots is not None:  # reduce-scatter CONNECT: S * 8 (N - 1) / N wire bytes per rank
            per = slots.numel() // rs.world
            rs.reduce_scatter_min_u64(slots)
            pairs = torch.empty(slots.numel(), dtype=torch.int64, device=slots.device)
            stepper.hook_owner(rs.rank, per, pairs)
            rs.allgather_slices(pairs, per)
            rs.allreduce_sum(stepper.apply_hooks(pairs))
        elif count:
            dense = stepper.pack(count)
            allreduce_min(dense)
            stepper.unpack(dense)
            hook = getattr(stepper, "hook_local", None)
            hooks = hook() if hook is not None else None
            if hooks is not None:  # each winning edge lives on one rank: MAX gathers the hooks
                (allreduce_max or allreduce_min.max)(hooks)
                stepper.unpack_hook(hooks)
        done = stepper.contract()
        rounds += 1
        if done:
            return rounds
        if rounds >= max_rounds:
            raise RuntimeError("round cap exceeded")


def _torch_allreduce(op, group=None):
    def fn(t):
        if dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(t, op=op, group=group)
    return fn


def _torch_allgather(group=None):
    def fn(t):
        if not (dist.is_initialized() and dist.get_world_size(group) > 1):
            return 1, t
        world = dist.get_world_size(group)
        out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
        if dist.get_backend(group) == "nccl":
            dist.all_gather_into_tensor(out, t, group=group)
        else:
            dist.all_gather(list(out.chunk(world)), t, group=group)
        return world, out
    return fn


class TorchRs:
    """The reduce-scatter protocol's collectives over a torch.distributed group (see run_rounds).
    uint64 keys travel as int64 with the sign bit flipped, so a signed MIN orders them unsigned;
    nccl reduce-scatters into this rank's slice and all-gathers the slices, gloo (no
    reduce-scatter) all-reduces the whole buffer and all-gathers through per-rank chunks."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.nccl = dist.get_backend(group) == "nccl"

    def reduce_scatter_min_u64(self, t):
        sign = torch.tensor(-(1 << 63), dtype=torch.int64, device=t.device)
        t.bitwise_xor_(sign)
        if self.nccl:  # (a separate output: no aliasing between the collective's buffers)
            per = t.numel() // self.world
            out = torch.empty(per, dtype=t.dtype, device=t.device)
            dist.reduce_scatter_tensor(out, t, op=dist.ReduceOp.MIN, group=self.group)
            t[self.rank * per:(self.rank + 1) * per].copy_(out)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        t.bitwise_xor_(sign)

    def allgather_slices(self, t, per):
        mine = t[self.rank * per:(self.rank + 1) * per]
        if self.nccl:
            dist.all_gather_into_tensor(t, mine.clone(), group=self.group)
        else:
            parts = [torch.empty_like(mine) for _ in range(self.world)]
            dist.all_gather(parts, mine.clone(), group=self.group)
            t.copy_(torch.cat(parts))

    def allreduce_sum(self, t):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)


def torch_allreduce_min(group=None, rs=True):
    fn = _torch_allreduce(dist.ReduceOp.MIN, group)
    fn.max = _torch_allreduce(dist.ReduceOp.MAX, group)
    fn.gather = _torch_allgather(group)
    fn.rs = TorchRs(group) if rs and dist.is_initialized() and dist.get_world_size(group) > 1 else None
    return fn


class _FailureWatch:
    """A daemon thread polling `key` in a torch.distributed store; when any rank sets it, the
    stepper's solve in progress is cancelled (see DistributedMST._watchdog)."""

    def __init__(self, store, key, stepper, period=0.02):
        self.store, self.key, self.stepper = store, key, stepper
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, args=(period,), daemon=True)
        self._t.start()

    def _run(self, period):
        while not self._stop.wait(period):
            try:
                if self.store.check([self.key]):
                    self.stepper.cancel()
                    return
            except Exception:  # noqa: BLE001 (store gone: the process group is shutting down)
                return

    def report(self):
        try:
            self.store.set(self.key, b"1")
        except Exception:  # noqa: BLE001
            pass

    def stop(self):
        self._stop.set()
        self._t.join()


def _device_u8_view(ptr, nbytes, device, owner):
    """A torch uint8 tensor over nbytes of device memory inside `owner`'s storage (the solver's
    workspace) — no copy, so the all-reduce combines the engine's own flag array."""
    base = owner.data_ptr()
    off = ptr - base
    if off < 0 or off + nbytes > owner.numel() * owner.element_size():
        raise RuntimeError("exchange buffer outside the workspace")
    return owner.view(torch.uint8)[off:off + nbytes]


class DistributedMST:
    """One rank's share of a multi-GPU MST over a replicated DeviceEdges graph.

    native (default: on when the process group's backend is nccl and world > 1): the round loop
    runs inside the library (ghs_solver_run) over the library's own RCCL communicator — created
    once from a unique id that rank 0 broadcasts through the process group — with the collectives
    on the solver's stream: one host call per solve. Off: `run_rounds` drives the same protocol
    from Python through torch.distributed (any backend)."""

    def __init__(self, edges, rank=None, world=None, group=None, config=None, native=None):
        self.rank = dist.get_rank(group) if rank is None else rank
        self.world = dist.get_world_size(group) if world is None else world
        self.group = group
        lo, hi = edge_range(edges.m, self.rank, self.world)
        if config is None:
            config = _native.make_config(num_ranks=self.world)
        config.num_ranks = self.world
        self.edges = edges
        self.stepper = None
        self._solves = 0
        # setup agreement before the first collective: a rank whose workspace allocation fails
        # raises on EVERY rank instead of leaving the others blocked in the next collective
        err = None
        try:
            if config.fault_rank == self.rank + 1 and config.fault_round == 0:  # test hook (ghs_config_t.fault_rank)
                raise _native.GHSError(_native.GHS_E_NOMEM, "injected setup failure (fault_rank)")
            self.engine = DeviceMST(edges, lo, hi, config)
        except Exception as ex:  # noqa: BLE001 (re-raised below, after the agreement)
            err = ex
        if self.world > 1 and dist.is_initialized():
            dev = edges.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
            flag = torch.tensor([1 if err is not None else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
            if err is None and int(flag.item()):
                raise _native.GHSError(_native.GHS_E_STATE, "another rank failed during setup")
        if err is not None:
            raise err
        if native is None:
            native = self.world > 1 and dist.is_initialized() and dist.get_backend(group) == "nccl"
        self.native = bool(native)
        # the failure watchdog's store keys carry a value every rank of THIS instance shares and no
        # other instance does (its RCCL unique id, broadcast by rank 0): a key left by a failed solve
        # of an earlier instance — a retry, another group on the same store — never cancels this one
        self._nonce = None
        self.comm = self._make_comm() if self.native and self.world > 1 else None

    def _make_comm(self):
        """The library's RCCL communicator: rank 0's unique id broadcast over the process group."""
        uid = torch.zeros(_native.GHS_COMM_ID_BYTES, dtype=torch.uint8, device=self.edges.device)
        if self.rank == 0:
            uid.copy_(torch.frombuffer(bytearray(_native.comm_unique_id()), dtype=torch.uint8))
        src = dist.get_global_rank(self.group, 0) if self.group is not None else 0
        dist.broadcast(uid, src=src, group=self.group)
        self._nonce = hashlib.sha1(uid.cpu().numpy().tobytes()).hexdigest()[:16]
        # the communicator binds to the device current at ghs_comm_init: the edges' device
        with torch.cuda.device(self.edges.device):
            return _native.Comm(self.world, self.rank, bytes(uid.cpu().numpy().tobytes()))

    def run(self):
        """The level/round loop over the owned edge range. Returns (Result, stats). The solver
        handle is created once and reset for every later solve."""
        if self.stepper is None:
            self.stepper = HipStepper(self.engine)
        else:
            self.stepper.reset()
        self._solves += 1
        watch = self._watchdog() if self.native and self.world > 1 else None
        try:
            if self.native:
                self.stepper.run_native(self.comm)
            else:
                run_rounds(self.stepper, torch_allreduce_min(self.group))
            return self.stepper.finish()
        except BaseException:
            if watch is not None:
                watch.report()  # the peers' waits end (their ghs_solver_run returns an error)
                watch.stop()    # before the handle goes away under the watchdog thread
                watch = None
            self.close()
            raise
        finally:
            if watch is not None:
                watch.stop()

    def _watchdog(self):
        """Failure agreement during a native solve: a rank that fails sets a key in the process
        group's store; every rank's watchdog thread polls it and cancels its own solver, whose
        waits then end (ghs_solver_cancel) instead of blocking behind the failed rank's missing
        collective. None when the store is not reachable."""
        try:
            store = dist.distributed_c10d._get_default_store()
        except Exception:  # noqa: BLE001
            return None
        return _FailureWatch(store, self._failure_key(), self.stepper)

    def _failure_key(self):
        """The store key of this instance's current solve: instance nonce + solve index (a new
        instance, or the same one's next solve, never sees an older failure)."""
        return f"ghs_failed/{self._nonce}/{self._solves}"

    def close(self):
        if self.stepper is not None:
            self.stepper.close()
            self.stepper = None
        if self.comm is not None:
            self.comm.close()
            self.comm = None

    def gather_in_mst(self):
        """Assemble the MSF flags from every rank's own slice [e_lo, e_hi) (collective: every rank
        calls it; an all-gather of equal-size padded slices). Returns the device flags (m)."""
        m = self.edges.m
        flags = self.engine.in_mst[:m]
        if not (dist.is_initialized() and dist.get_world_size(self.group) > 1):
            return flags
        world = dist.get_world_size(self.group)
        ranges = [edge_range(m, r, world) for r in range(world)]
        width = max(hi - lo for lo, hi in ranges)
        dev = flags.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        mine = torch.zeros(width, dtype=torch.uint8, device=dev)
        lo, hi = ranges[self.rank]
        mine[: hi - lo] = flags[lo:hi].to(dev)
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine, group=self.group)
        out = torch.empty(m, dtype=torch.uint8, device=flags.device)
        for (plo, phi), part in zip(ranges, parts):
            out[plo:phi] = part[: phi - plo].to(flags.device)
        return out

    def collect_mst(self, dst=0):
        """The reference's `collect_results` (ghs_implementation_mpi.py:760-779: every rank sends
        its BRANCH edges to rank 0): each rank compacts its own range's MSF flags to global edge
        ids and `dst` gathers them (collective). Returns the sorted int64 eids of the whole MSF on
        `dst` (the ranks' ranges ascend, so the concatenation is sorted), None elsewhere."""
        m = self.edges.m
        lo, hi = edge_range(m, self.rank, self.world)
        # the MSF has < n edges: a range's ids fit min(hi - lo, n) slots
        mine = flags_to_eids(self.engine.in_mst, lo, hi, min(hi - lo, self.edges.n))
        if not (dist.is_initialized() and dist.get_world_size(self.group) > 1):
            return mine
        world = dist.get_world_size(self.group)
        dev = mine.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        cnt = torch.tensor([mine.numel()], dtype=torch.int64, device=dev)
        counts = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(counts, cnt, group=self.group)
        counts = [int(c.item()) for c in counts]
        width = max(max(counts), 1)
        pad = torch.full((width,), -1, dtype=torch.int64, device=dev)
        pad[: mine.numel()] = mine.to(dev)
        gdst = dist.get_global_rank(self.group, dst) if self.group is not None else dst
        parts = [torch.empty_like(pad) for _ in range(world)] if self.rank == dst else None
        dist.gather(pad, parts, dst=gdst, group=self.group)
        if self.rank != dst:
            return None
        return torch.cat([p[:c] for p, c in zip(parts, counts)]).to(mine.device)

    def in_mst_host(self):
        """The MSF flags as a host bool array (collective, see gather_in_mst)."""
        return self.gather_in_mst().cpu().numpy().astype(bool)
