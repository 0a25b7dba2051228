/*
 * ghs_mst.h — C-ABI of the MI355X-native MST engine (libghs_mst.so).
 *
 * The reference (Trisanu-007/Distributed_GHS_Implementation) computes an MST with the GHS
 * message protocol: one Python thread (ghs_implementation.py:46-413) or one MPI rank
 * (ghs_implementation_mpi.py:37-757) per vertex exchanging CONNECT/INITIATE/TEST/ACCEPT/
 * REJECT/REPORT/CHANGEROOT. It has no FFI; its path sits behind two call surfaces:
 *   (1) GHSAlgorithm(num_nodes, edges).run(timeout) -> [(u, v)]   ghs_implementation.py:417-490
 *   (2) MPINode(...).run() + collect_results() -> [(u, v, w)]       ghs_implementation_mpi.py:673-779
 * This library replaces the protocol with a level-synchronous Boruvka fragment contraction
 * (one GHS level == one Boruvka round) in hand-written gfx950 HIP kernels. Every entry point
 * below names the reference interface it stands in for. Conventions:
 *   - all functions return GHS_OK (0) or a negative GHS_E_* code and never abort;
 *     ghs_last_error() returns a thread-local message for the last failure;
 *   - "canonical edge list": u[e] < v[e] < n, strictly ascending (u, v), no duplicates;
 *     eid = e. Size limits: m < 2^31 (edge ids are 32-bit inside the 64-bit keys and the
 *     kernels' byte offsets) and n <= 2^32 - 1 (ids < n, so 0xffffffff never names a vertex
 *     and marks dead entries); every entry point that takes m returns GHS_E_ARG past the cap. Ties resolve under the strict key (w, u, v) == (w, eid) — the order in which
 *     NetworkX Kruskal (the reference's verifier, ghs_implementation.py:746) visits edges on a
 *     canonically built graph. The result is a minimum spanning FOREST.
 *   - d_* pointers are device pointers (HIP / torch device memory) on the current device;
 *     `stream` is a hipStream_t passed as void* (NULL = default stream);
 *   - 64-bit keys: key = (uint64)w << 32 | eid; UINT64_MAX = "no outgoing edge" (the
 *     reference's best_weight = float('inf'), ghs_implementation.py:61).
 */
#ifndef GHS_MST_H
#define GHS_MST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GHS_MST_ABI_VERSION 10

#define GHS_OK 0
#define GHS_NEED_EXCHANGE 1   /* ghs_solver_minedge on a multi-rank solver opened a level: OR-combine
                                 the level's fragment flags across ranks, then call it again */
#define GHS_E_ARG (-1)        /* bad argument (null pointer, size, alignment) */
#define GHS_E_NONCANON (-2)   /* input edge list is not canonical */
#define GHS_E_HIP (-3)        /* HIP runtime error */
#define GHS_E_ROUNDCAP (-4)   /* round cap exceeded (never expected: hang guard) */
#define GHS_E_NODEVICE (-5)   /* no usable gfx950 device */
#define GHS_E_NOMEM (-6)      /* workspace too small / allocation failed */
#define GHS_E_STATE (-7)      /* solver handle used out of order */

#define GHS_MAX_ROUND_STATS 64
#define GHS_MAX_RANKS 64       /* ranks of one multi-rank solve (ghs_config_t.num_ranks, communicators) */

/* Per-round record (one Boruvka round == one GHS level of the reference). */
typedef struct ghs_round_stats {
  uint32_t level;             /* weight level this round belongs to */
  uint32_t reserved;
  uint64_t level_arcs;        /* first round of a level: arcs built for the level, else 0 */
  uint64_t live_arcs;         /* arcs scanned by the min-edge kernel this round */
  uint64_t active_components; /* fragments that searched for an outgoing edge */
  uint64_t hooks;             /* fragments that merged (== MST edges added) */
  float ms_minedge;           /* min-outgoing-edge (+ fused compaction) kernel */
  float ms_hook;              /* hook (CONNECT) kernel */
  float ms_jump;              /* pointer-jump relabel (INITIATE) kernel */
  float ms_active;            /* next-fragment-list compaction */
} ghs_round_stats_t;

typedef struct ghs_result {
  uint64_t num_mst_edges;     /* n - (#components) */
  uint64_t total_weight;      /* sum of w over MST edges */
  uint32_t rounds;            /* Boruvka rounds executed (all levels) */
  uint32_t num_stats;         /* entries filled in the stats array (<= GHS_MAX_ROUND_STATS) */
  uint32_t levels;            /* weight levels planned */
  uint32_t pass_flags;        /* bit 0: the solve ran bucketed rounds (k_bucket / k_bmin);
                                 bit 1: the plan's span sample found the graph lattice-like;
                                 bit 2: level 0's round 0 ran windowed (k_wmin over the edge list;
                                 unset when k_select's span flag sent it to k_bucket / k_bmin);
                                 bit 3: a level finished in the LDS tail (k_tail_*) */
  double ms_total;            /* host wall time of the solve (device-resident input -> flags) */
  /* The two full streams over the canonical list (HIP events on the solve's stream). */
  float ms_select;            /* k_select: validation + level-0 split */
  float ms_filter;            /* k_filter: giant-bitmap filter + level-1 split (0 if not run) */
  uint64_t canon_edges;       /* canonical edges each pass streams (the solver's range) */
  uint64_t select_out;        /* entries k_select wrote (level-0 edges, incl. region padding) */
  uint64_t filter_out;        /* entries k_filter wrote (level-1 + pending edges, incl. padding) */
  /* ABI 7: host-side phases of the multi-rank drivers (ghs_mst_multi / ghs_mst_emulated; 0
     elsewhere), the maximum over the ranks: setup (stream, workspace, H2D copy, solver creation,
     agreement), the ghs_solver_run loop, the flags' D2H gather. reused = 1 when the call ran on
     the rank state cached by an earlier call of the same shape (no hipMalloc, no RCCL init). */
  double ms_setup;
  double ms_solve;
  double ms_gather;
  uint32_t reused;
  uint32_t reserved;
} ghs_result_t;

/* Weight-level plan of the filter. Level 1 holds roughly the
 * level1_edges_per_vertex * n lightest edges, each further level level_growth times more, the
 * last level the rest; max_levels = 1 runs plain Boruvka over every edge at once. Thresholds
 * are weight quantiles of a fixed sample of the canonical list, so every rank plans the same
 * levels. level1_edges_per_vertex <= 0 (the default) = auto: 0.5 when m >= 4n, else 1.2.
 * Results do not depend on the plan (only speed does).
 * ABI 5: every path option lives here (the library reads no environment variable that changes the
 * algorithm or a launch shape); options = 0 and dedup_max = 0 select the default path. */
#define GHS_OPT_NO_SEED_RUNS 0x1u  /* level 0, round 0: a-side minima through the min-edge kernel
                                      instead of the single-writer run seeding */
#define GHS_OPT_NO_DENSE 0x2u      /* several ranks: levels in vertex labels, not dense labels */
#define GHS_OPT_BUCKETED 0x4u      /* one rank: every round bucketed, whatever the graph (default:
                                      a lattice-like graph's level-0 rounds with >= 2^23 active
                                      fragments, another graph's first round of every level —
                                      decided from the plan's span sample; tests force it) */
#define GHS_OPT_NO_BUCKETED 0x8u   /* one rank: never bucketed rounds */
#define GHS_OPT_DEBUG 0x10u        /* per-level sizes on stderr (diagnostic) */
#define GHS_OPT_TIME_ROUNDS 0x20u  /* HIP events around the compacting min-edge launches
                                      (ghs_round_stats_t.ms_minedge; idles the GPU ~6 us each) */
#define GHS_OPT_DETAIL 0x40u       /* HIP events around every stage of every round (diagnostic) */
#define GHS_OPT_NO_WINDOW 0x100u   /* one rank, lattice-like: level 0 round 0 through k_bucket / k_bmin
                                      records instead of the windowed k_wmin over the edge list */
#define GHS_OPT_BUCKETED_FIRST 0x80u /* one rank: bucketed first rounds of every level (whatever the
                                        graph), the other rounds unbucketed */
#define GHS_OPT_NO_TAIL 0x200u     /* one rank: no LDS tail — every round of a level through the
                                      per-round kernels (default: once a level's active fragments fit
                                      the tail's LDS, its remaining rounds run in k_tail_*) */
/* ABI 8 */
#define GHS_OPT_CHECK_TOTALS 0x400u /* one rank: at the end of every level the device counters are copied
                                       behind the level's last kernel (stream-ordered) and compared with
                                       the totals of the level's last round report (GHS_E_STATE if they
                                       differ); the solve's totals then come from that copy (test /
                                       diagnostic: one host sync per level) */
#define GHS_OPT_KEEP_CACHE 0x800u  /* ghs_mst_multi / ghs_mst_emulated: keep the per-rank state for the
                                      next call of the same shape (default: freed when the call returns;
                                      see ghs_release_cache) */
typedef struct ghs_config {
  uint32_t max_levels;
  uint32_t num_ranks;         /* ranks sharing the solve (1 = single GPU; >1: identical rounds on
                                 every rank, so empty levels are not skipped) */
  double level1_edges_per_vertex;
  double level_growth;
  uint32_t options;           /* GHS_OPT_* bits (0 = default path) */
  uint32_t dedup_max;         /* cross-component parallel-edge filter in the compacting rounds once
                                 at most this many fragments are active (0 = off, the default) */
  uint32_t fault_rank;        /* test hook of the multi-rank drivers: 1 + the rank whose setup is
                                 made to fail (ghs_mst_multi / ghs_mst_emulated); 0 = none */
  uint32_t fault_round;       /* ABI 7 test hook: with fault_rank set, that rank fails in the round
                                 loop (ghs_solver_run) once it has completed this many rounds instead
                                 of at setup; 0 = the setup failure above. ABI 8: GHS_E_ARG with
                                 num_ranks == 1 (a one-rank loop has no exchange to fail in) */
} ghs_config_t;

/* ---- library / device ------------------------------------------------------------------- */
int ghs_abi_version(void);
const char *ghs_last_error(void);
/* number of visible HIP devices (0 on a host without GPU; never an error) */
int ghs_device_count(int *count);

/* ---- host-buffer convenience -------------------------------------------------------------
 * Replaces GHSAlgorithm.run (ghs_implementation.py:442-490: starts n threads, polls
 * termination, sweeps BRANCH edges) and MPINode.run + collect_results
 * (ghs_implementation_mpi.py:673-779). Input: canonical edge list on the HOST. Output:
 * in_mst[e] = 1 iff canonical edge e is in the MSF (m bytes, host). Copies in/out, runs on the
 * current device, serialised per process. stats may be NULL (else GHS_MAX_ROUND_STATS entries). */
int ghs_mst_host(uint32_t n, uint64_t m, const uint32_t *u, const uint32_t *v, const uint32_t *w,
                 uint8_t *in_mst, ghs_result_t *result, ghs_round_stats_t *stats);

/* ---- one process, several GPUs ------------------------------------------------------------
 * Replaces the MPI path as ONE call (ghs_implementation_mpi.py:884-954: mpiexec with one rank per
 * vertex, pickled p2p messages, Barrier, gather of the BRANCH edges to rank 0 at :760-779):
 * num_gpus devices of this node (devices: their HIP ids, NULL = 0..num_gpus-1, distinct) form an
 * RCCL clique (ncclCommInitAll); one host thread per device copies the canonical list (host
 * arrays, as ghs_mst_host) to its device and runs the stepwise solver below over its own edge
 * range [r*m/N, (r+1)*m/N) (4-aligned), with the round's collectives over RCCL (all-gather of the
 * level-flag bitmaps, int64 MIN of the best keys, int32 MAX of the owner-computed hooks). in_mst
 * (host, m bytes) = the devices' own-range flags; result/stats are device 0's (the totals are
 * checked equal on every device). cfg may be NULL (defaults; num_ranks is set to num_gpus).
 * An input error (non-canonical list) fails the call on every device together (the error byte
 * of the flag exchange); a device fault (GHS_E_HIP) is not recoverable. */
int ghs_mst_multi(uint32_t n, uint64_t m, const uint32_t *u, const uint32_t *v, const uint32_t *w,
                  int num_gpus, const int *devices, const ghs_config_t *cfg, uint8_t *in_mst,
                  ghs_result_t *result, ghs_round_stats_t *stats);
/* ABI 7/8: with GHS_OPT_KEEP_CACHE the multi-rank drivers (ghs_mst_multi, ghs_mst_emulated) keep
 * their per-rank state — streams, workspaces, replicated canonical copies, pinned report rings,
 * collective scratch, and ghs_mst_multi's RCCL clique — in one process-wide cache keyed by (driver,
 * devices, ranks, n, m); a later call of the same shape allocates nothing (ghs_result_t.reused = 1),
 * a call of another shape or a failed call frees it first. Without the option (ABI 8 default) a
 * call frees its state before returning. ghs_release_cache frees it now (device memory back to the
 * caller; safe to call at any time outside a driver call), and (ABI 9) ghs_flags_to_eids' cached
 * temporary storage with it. */
int ghs_release_cache(void);
/* ABI 8: the MSF edge ids of the flag range [lo, hi) in order — d_eids[k] = the k-th e with
 * d_in_mst[e] != 0 (uint32; room for `capacity` ids), *count (host) = how many — on the device
 * (a flagged select), the form a rank's own-range MSF is gathered in (the reference's
 * collect_results, ghs_implementation_mpi.py:760-779). Returns once *count is known (one stream
 * sync); GHS_E_NOMEM without writing when more than `capacity` edges are flagged. hi < 2^32. */
int ghs_flags_to_eids(const uint8_t *d_in_mst, uint64_t lo, uint64_t hi, uint32_t *d_eids, uint64_t capacity,
                      uint64_t *count, void *stream);

/* ---- device-resident API -----------------------------------------------------------------
 * Input: the canonical edge list in HBM (d_u, d_v, d_w: m uint32 each, 16-byte aligned) — the
 * device form of the reference's per-node neighbour files node_<id>.json
 * (create_graph_files.py:56-74), each edge once, key = w<<32 | eid. Each weight level's edges
 * are streamed out of it (edge-centric: every edge is a candidate for both of its fragments). */
void ghs_default_config(ghs_config_t *cfg);

/* workspace bytes for ghs_mst_device / a solver handle owning local_edges canonical edges */
size_t ghs_workspace_bytes(uint32_t n, uint64_t m, uint64_t local_edges);

/* Whole MST on one device: canonical edges -> d_in_mst (m bytes, 1 = in the MSF) + totals.
 * cfg may be NULL (defaults). Returns once *result is final (the host polls the rounds'
 * reports; one sync for the level plan). d_in_mst is written by work enqueued on `stream`:
 * complete once the stream is synchronized (a trailing no-op round may still run on return).
 * Reference: GHSAlgorithm.run, ghs_implementation.py:442-490. */
int ghs_mst_device(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                   const ghs_config_t *cfg, void *d_workspace, size_t workspace_bytes, uint8_t *d_in_mst,
                   void *stream, ghs_result_t *result, ghs_round_stats_t *stats);

/* ABI 9: the same canonical list in CSR form — the north_star's "CSR edge list in HBM" and the
 * reference's per-node neighbour files (create_graph_files.py:56-74: node u lists its neighbours)
 * with each edge stored once at its smaller end: d_off = n + 1 uint32 row offsets (d_off[0] = 0,
 * nondecreasing, d_off[n] = m), edge e of row u (d_off[u] <= e < d_off[u + 1]) joins u and d_v[e]
 * with weight d_w[e]; d_v strictly ascending inside a row, u < d_v[e] < n. eid = e as in the COO
 * form (same keys, same MSF flags). The streaming passes read 8 B per edge (+ 4 B per row) instead
 * of 12. d_u may be NULL, or the caller's expanded u (16-byte aligned): then gathers of u by edge
 * id read it instead of searching d_off, and the level-opening filter pass streams (u, v, w) — the
 * faster form for that pass — while the first pass streams the CSR form. The offsets are validated
 * with the rest (GHS_E_NONCANON). */
int ghs_mst_device_csr(uint32_t n, uint64_t m, const uint32_t *d_off, const uint32_t *d_u, const uint32_t *d_v,
                       const uint32_t *d_w, const ghs_config_t *cfg, void *d_workspace, size_t workspace_bytes,
                       uint8_t *d_in_mst, void *stream, ghs_result_t *result, ghs_round_stats_t *stats);
/* d_off (n + 1 uint32) from a canonical COO list's d_u (u ascending), on the device */
int ghs_csr_offsets(uint32_t n, uint64_t m, const uint32_t *d_u, uint32_t *d_off, void *stream);

/* device-side canonicity check: *ok = 1 iff u < v < n and (u, v) strictly ascending */
int ghs_check_canonical(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, void *stream, int *ok);

/* ---- stepwise solver (multi-GPU: one process per GPU, RCCL all-reduce between steps) ------
 * Replaces the per-rank protocol loop of ghs_implementation_mpi.py:673-748 and its
 * collectives (:907 bcast, :929 Barrier, :766 gather). Every rank holds the replicated
 * canonical list and owns the contiguous edge range [e_lo, e_hi); per round it scans the arcs of
 * ITS edges and the per-fragment best keys are combined with an all-reduce MIN by the caller:
 *   h = ghs_solver_create(...)
 *   loop: rc = ghs_solver_minedge(h, &C)       local min-edge per fragment (opens levels)
 *         while rc == GHS_NEED_EXCHANGE:       a level was opened (several ranks): its active
 *           <caller: all_reduce(flags, MAX)>     fragments = those with a level edge on ANY rank
 *           rc = ghs_solver_minedge(h, &C)       (ghs_solver_exchange_buffer: n uint8 flags)
 *         ghs_solver_pack_best(h, d_dense)     C int64 slots, order-preserving (key ^ 2^63)
 *         <caller: all_reduce(d_dense[0:C], MIN)>
 *         ghs_solver_unpack_best(h, d_dense)
 *         ghs_solver_contract(h, &done)        hook + pointer-jump + next fragment list
 *   ghs_solver_finish(h, result, stats); ghs_solver_destroy(h)
 * Identical inputs on every rank => identical hook decisions => identical totals (ghs_solver_finish)
 * on every rank. MSF flags are owner-written: a solver clears and writes d_in_mst[e] only for its
 * own range e in [e_lo, e_hi) and never touches the rest, so the MSF is the concatenation of the
 * ranks' slices (an all-gather of [e_lo, e_hi) from every rank; the reference gathered BRANCH
 * edges to rank 0, ghs_implementation_mpi.py:760-779).
 * Errors: a rank that finds its edge range non-canonical records it in the exchanged flag
 * buffer (its last byte), so after the caller's MAX every rank returns GHS_E_NONCANON from the
 * same ghs_solver_minedge call — no rank is left waiting in a collective. */
typedef struct ghs_solver ghs_solver_t;
int ghs_solver_create(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                      uint64_t e_lo, uint64_t e_hi, const ghs_config_t *cfg, void *d_workspace,
                      size_t workspace_bytes, uint8_t *d_in_mst, void *stream, ghs_solver_t **out);
/* ABI 9: a rank of the same loop over the CSR form (d_off, optional d_u; see ghs_mst_device_csr) */
int ghs_solver_create_csr(uint32_t n, uint64_t m, const uint32_t *d_off, const uint32_t *d_u, const uint32_t *d_v,
                          const uint32_t *d_w, uint64_t e_lo, uint64_t e_hi, const ghs_config_t *cfg, void *d_workspace,
                          size_t workspace_bytes, uint8_t *d_in_mst, void *stream, ghs_solver_t **out);
/* runs the min-edge kernel; *num_active = fragments whose best slot must be all-reduced */
int ghs_solver_minedge(ghs_solver_t *h, uint64_t *num_active);
/* the flag array to OR-combine (uint8 MAX all-reduce) after GHS_NEED_EXCHANGE: n fragment flags
 * + 1 error byte (*bytes = n + 1) */
int ghs_solver_exchange_buffer(ghs_solver_t *h, uint8_t **d_flags, uint64_t *bytes);
/* the same exchange as bitmaps (half the wire bytes of the MAX all-reduce per rank): flag_bits
 * packs the n + 1 flags into *words uint64 words; the caller all-gathers every rank's words
 * (rank-major, nranks x words) and hands the gathered buffer to merge_flag_bits (OR), then calls
 * ghs_solver_minedge again — instead of exchange_buffer + MAX all-reduce */
int ghs_solver_flag_bits(ghs_solver_t *h, uint64_t **d_bits, uint64_t *words);
int ghs_solver_merge_flag_bits(ghs_solver_t *h, const uint64_t *d_all, uint32_t nranks);
int ghs_solver_pack_best(ghs_solver_t *h, int64_t *d_dense);
int ghs_solver_unpack_best(ghs_solver_t *h, const int64_t *d_dense);
/* optional, instead of pack_best / int64 MIN / unpack_best: a dense level's first round keeps its
 * *count slots contiguous in the solver's own minima (identity order), so the caller may MIN
 * all-reduce *d_slots in place as UNSIGNED 64-bit (ncclUint64 + ncclMin). *d_slots = NULL: this
 * round needs pack / unpack. (ghs_solver_run uses it; ABI 4 addition) */
int ghs_solver_best_slots(ghs_solver_t *h, uint64_t **d_slots, uint64_t *count);
/* optional, after unpack_best (a level's first round, several ranks): owner-computes CONNECT.
 * Each rank hooks the fragments whose winning edge it holds and fills *count int32 slots
 * (par ^ fragment, 0 where another rank owns the winner); the caller all-reduces them with MAX
 * and hands them to unpack_hook, after which contract skips its own hook. *count = 0: not
 * applicable this round (contract hooks in fragment form, as without the call). Replaces the
 * per-fragment gathers of the fragment-form hook with 4 bytes per active fragment on the wire.
 * The MSF flag of such a hook is set only on the rank that owns the edge (as every flag: see
 * above); the totals of ghs_solver_finish are complete on every rank. */
int ghs_solver_hook_local(ghs_solver_t *h, int32_t *d_dense, uint64_t *count);
int ghs_solver_unpack_hook(ghs_solver_t *h, const int32_t *d_dense);
/* optional (ABI 6), a dense level's opening round instead of best_slots / MIN all-reduce /
 * hook_local / MAX all-reduce / unpack_hook — half the wire of a ring all-reduce per slot, the
 * reference's collect of the CONNECT decisions (ghs_implementation_mpi.py:582-671) as 16 bytes:
 *   hook_slots(h, N, &slots, &S)      S = 0: not applicable this round (use the calls above);
 *                                     else `slots` = S uint64 (a multiple of N, padding = UINT64_MAX)
 *   <caller: reduce-scatter MIN (uint64, in place): rank r keeps slots[r*S/N, (r+1)*S/N)>
 *   hook_owner(h, r, S/N, pairs)      pairs[c] for the rank's slots: eid << 32 | the other dense
 *                                     fragment of c's minimum edge (UINT64_MAX: no edge); the ends
 *                                     come from the replicated canonical list
 *   <caller: all-gather the S/N-slot slices (in place into pairs, S uint64)>
 *   apply_hooks(h, pairs, &partial)   par for every fragment (a mutual pair stays a 2-cycle that the
 *                                     jump resolves: its smaller fragment keeps the root), the MSF
 *                                     flags of the rank's own edge range, and in `partial` (2 uint64,
 *                                     device) the weight and count of those own-range MSF edges
 *   <caller: all-reduce SUM (uint64) of partial, in place>
 * then contract as usual (it adds the summed partial totals to the solve's totals). (Replaces
 * 2(N-1)/N x 12 bytes per slot with (N-1)/N x 16, + 16 bytes.) */
int ghs_solver_hook_slots(ghs_solver_t *h, uint32_t nranks, uint64_t **d_slots, uint64_t *padded);
int ghs_solver_hook_owner(ghs_solver_t *h, uint32_t rank, uint64_t per_rank, uint64_t *d_pairs);
int ghs_solver_apply_hooks(ghs_solver_t *h, const uint64_t *d_pairs, uint64_t **d_partial);
/* optional (ABI 10), at the top of the loop (before minedge), several ranks: the LDS tail of a
 * dense level — its last rounds (ghs_implementation_mpi.py:673-748 once few fragments remain, the
 * REPORT / CHANGEROOT convergecasts of ghs_implementation.py:235-387) with the fragments renumbered
 * 0..F-1 and each round's minima kept in LDS, so a round moves 12 bytes per fragment on the wire
 * instead of a min-edge + hook over n-sized arrays:
 *   tail_begin(h, &F)              F = 0: not applicable now (call minedge as usual); else the tail
 *                                  opened and this rank's minima of its round 0 are in `keys`
 *   loop: tail_buffers(h, &keys, &hooks)    F uint64 keys, F int32 CONNECT targets (device)
 *     <caller: all-reduce MIN (UNSIGNED 64-bit) of keys[0:F], in place>
 *     tail_agree(h)                the owner of each minimum keeps its target and writes the MSF
 *                                  flag of its own edge; the other ranks withdraw theirs (-1)
 *     <caller: all-reduce MAX (int32) of hooks[0:F], in place>
 *     tail_round(h, &state)        the hooks applied, the next round streamed (one host sync);
 *                                  state 0: the next round's minima are in keys (loop); 1: the level
 *                                  is complete (continue with minedge); 2: so is the solve (finish)
 * Every rank takes the same branch (the counts are identical on every rank). ghs_solver_run runs the
 * same tail with its own collectives (several rounds per host sync). */
int ghs_solver_tail_begin(ghs_solver_t *h, uint64_t *num_fragments);
int ghs_solver_tail_buffers(ghs_solver_t *h, uint64_t **d_keys, int32_t **d_hooks);
int ghs_solver_tail_agree(ghs_solver_t *h);
int ghs_solver_tail_round(ghs_solver_t *h, int *state);
/* hook + jump + next list; *done = 1 when every level is complete */
int ghs_solver_contract(ghs_solver_t *h, int *done);
int ghs_solver_finish(ghs_solver_t *h, ghs_result_t *result, ghs_round_stats_t *stats);
/* start the next solve of the same inputs on the same handle (keeps the workspace layout and the
 * pinned host resources: a multi-GPU caller's per-solve create/destroy becomes one reset) */
int ghs_solver_reset(ghs_solver_t *h);
/* thread-safe, callable while another thread is inside ghs_solver_run (ABI 5): a rank whose peer
 * failed ends its waits — the call in progress returns GHS_E_STATE instead of waiting forever
 * behind a collective the peer never joins (DistributedMST: a watchdog thread calls it when
 * another rank reports a failure). The handle is then only good for reset or destroy. */
int ghs_solver_cancel(ghs_solver_t *h);
int ghs_solver_destroy(ghs_solver_t *h);

/* ---- the round loop in the library --------------------------------------------------------
 * ghs_solver_run drives the loop above to completion on the solver's stream — minedge, the
 * level-flag bitmap all-gather, pack / int64 MIN / unpack, the owner-computed hooks' int32 MAX,
 * contract — with the collectives of `comm` enqueued on that same stream (RCCL): one host call
 * per solve instead of ~6 library calls + 2-3 collective launches per round from the caller.
 * comm: one per rank from ghs_comm_init, after rank 0's ghs_comm_unique_id has reached every
 * rank (torch.distributed / MPI broadcast of GHS_COMM_ID_BYTES bytes); NULL for a single-rank
 * solver. Collective: every rank calls it; then ghs_solver_finish as usual. The communicator is
 * bound to the device current at ghs_comm_init and keeps its own device scratch (grown on demand,
 * n-sized). */
#define GHS_COMM_ID_BYTES 128
typedef struct ghs_comm ghs_comm_t;
int ghs_comm_unique_id(uint8_t *id);
int ghs_comm_init(int nranks, int rank, const uint8_t *id, ghs_comm_t **out);
int ghs_comm_destroy(ghs_comm_t *comm);
int ghs_solver_run(ghs_solver_t *h, ghs_comm_t *comm);
/* Test / diagnostic entry: the ghs_solver_run loop of a num_ranks-GPU solve, every rank on the
 * CURRENT device (one host thread and stream per rank, in-process collectives with the same
 * semantics as RCCL's) — exercises the exact multi-rank loop on one GPU. Device pointers; every
 * rank writes its own range of d_in_mst (m flags). result/stats: rank 0's (checked equal on every
 * rank). */
int ghs_mst_emulated(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                     int num_ranks, const ghs_config_t *cfg, uint8_t *d_in_mst, ghs_result_t *result,
                     ghs_round_stats_t *stats);

/* ABI 8 diagnostic: round reports whose sequence number the host read before every field had
 * landed (the checksum of the report failed and the host polled again), since the process started */
int ghs_slot_retries(uint64_t *count);

/* ---- per-launch profile ------------------------------------------------------------------
 * The reference measured only wall time (time.time(), ghs_implementation.py:453-464,
 * ghs_implementation_mpi.py:920-933). With profiling on, every kernel launch of later solves is
 * bracketed by two HIP events on the solve's stream and its duration lands in a process-wide
 * list (read and drained by ghs_profile_read). The events idle the GPU ~6 us each between
 * launches: profile a separate solve, not the timed ones. */
enum ghs_kernel_id {
  GHS_K_SELECT = 0, GHS_K_FILTER, GHS_K_LEVEL_PASS, GHS_K_SEED_RUNS, GHS_K_MINEDGE_IDENT, GHS_K_MINEDGE_COMPACT,
  GHS_K_WIN, GHS_K_HOOK, GHS_K_JUMP_IDENT, GHS_K_JUMP, GHS_K_SELECT_LB, GHS_K_RESOLVE, GHS_K_GIANT, GHS_K_SCAN,
  GHS_K_PLAN, GHS_K_INIT, GHS_K_PACK, GHS_K_UNPACK, GHS_K_ROUND_REPORT, GHS_K_PACK_HOOK, GHS_K_UNPACK_HOOK,
  GHS_K_DENSE, GHS_K_FLAG_BITS, GHS_K_BUCKET, GHS_K_BMIN, GHS_K_WSTARTS, GHS_K_WMIN, GHS_K_HOT_HOOK,
  GHS_K_TAIL_OPEN, GHS_K_TAIL_ROUND, GHS_K_TAIL_HOOK, GHS_K_CSR_TROW /* ABI 9 */, GHS_K_COUNT
};
typedef struct ghs_kernel_record {
  uint32_t kernel;  /* ghs_kernel_id */
  uint32_t round;   /* round index (all levels) when launched; a lookahead no-op round past a
                       level's end reuses the next level's index with its own (older) level */
  uint32_t level;   /* weight level when launched */
  uint32_t solver;  /* the launching solver handle (creation order in the process) */
  uint64_t items;   /* host-known work count at launch (edges / vertices / fragments), 0 = unknown */
  float ms;         /* event-to-event duration */
  float reserved2;
} ghs_kernel_record_t;
int ghs_profile_enable(int on);  /* also clears the list */
int ghs_profile_read(ghs_kernel_record_t *out, uint32_t capacity, uint32_t *count);
const char *ghs_kernel_name(uint32_t kernel);

/* ---- synthetic graph generators (device; BASELINE.json configs 3-5) ----------------------
 * R-MAT (Graph500 A,B,C,D = .57,.19,.19,.05, edgefactor ef, 2^scale vertices, seeded vertex
 * permutation), self-loops dropped, duplicates removed, canonical order, unique weights
 * w = bijective_hash32(eid ^ wseed) (distinct by construction). d_u/d_v/d_w must hold
 * edgefactor * 2^scale entries (the tuple count, an upper bound); *m_out = canonical edge count.
 * d_temp: ghs_rmat_temp_bytes(scale, edgefactor) bytes. */
size_t ghs_rmat_temp_bytes(uint32_t scale, uint32_t edgefactor);
int ghs_rmat_generate(uint32_t scale, uint32_t edgefactor, uint64_t seed, uint64_t wseed,
                      uint32_t *d_u, uint32_t *d_v, uint32_t *d_w, uint64_t *m_out,
                      void *d_temp, size_t temp_bytes, void *stream);
/* The raw R-MAT tuples of ghs_rmat_generate before its canonical sort/dedupe (generator parity
 * tests): d_keys[t] = min << scale | max of tuple t, or 2^(2 scale) - 1 for a self-loop;
 * edgefactor * 2^scale entries. */
int ghs_rmat_tuples(uint32_t scale, uint32_t edgefactor, uint64_t seed, uint64_t *d_keys, void *stream);
/* k x k grid, vertex r*k+c, right + down edges (m = 2k(k-1)), canonical order.
 * mode 0: unique hashed weights; mode 1: "road-like" gradient weights w = eid (unique, forces
 * long hook chains). */
int ghs_grid_generate(uint32_t k, uint32_t mode, uint64_t wseed, uint32_t *d_u, uint32_t *d_v, uint32_t *d_w,
                      void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GHS_MST_H */
