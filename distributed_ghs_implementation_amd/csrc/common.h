// Shared definitions for libghs_mst.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/ghs_mst.h"

namespace ghs {

constexpr uint64_t KEY_NONE = ~0ull;       // "no outgoing edge" (reference: best_weight = inf)
constexpr uint32_t LABEL_NONE = 0xffffffffu;
constexpr int WAVE = 64;                   // CDNA wavefront
constexpr int BLOCK = 256;                 // 4 waves
constexpr int ARCS_PER_THREAD = 4;         // one 16-B load of src / dst per lane
constexpr int ARCS_PER_BLOCK = BLOCK * ARCS_PER_THREAD;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

void set_error(const std::string &msg);

// Attributes of every fixed-grid streaming kernel (grid = 8 blocks per CU x 256 CUs). gfx950
// admits 8 resident 256-thread blocks per CU only while .sgpr_count <= 80 (MI355X_MICROARCH.md,
// "Residency"); at 82-96 it admits 7 and a 2048-block grid runs a second, nearly empty wave of
// blocks — half the throughput of an equal-work grid. The cap keeps these kernels at 8.
// VGPRs are NOT capped: k_filter / k_level_pass / k_minedge use 75-80 (6 waves per SIMD), and
// forcing 8 waves (GHS_STREAM_WAVES=8, <= 64 VGPRs) spills 8-14 of them to scratch and measured
// slower (R-MAT s24: 7.41 vs 7.00 ms per step); a grid sized to 6 blocks per CU (GHS_SEG_G=1536)
// measured the same as 2048 (7.04-7.12 ms). Second argument: min waves per SIMD.
#ifndef GHS_STREAM_WAVES
#define GHS_STREAM_WAVES 1
#endif
#define GHS_STREAM_KERNEL \
  __global__ __launch_bounds__(BLOCK, GHS_STREAM_WAVES) __attribute__((amdgpu_num_sgpr(72)))
// Streaming kernels whose VGPR count (> 64) already limits them to 6 waves per SIMD: no SGPR cap
// (6 waves leave ~128 SGPRs each) but a 6-wave bound (<= 80 VGPRs). An SGPR cap there only
// spills SGPRs into VGPR lanes — k_filter's loop spent 112 of its 432 VALU instructions on
// v_readlane/v_writelane under a cap of 72 — and without the wave bound the freed SGPRs turn
// into VGPRs (k_filter 83, k_level_pass 91: 5 waves, measured slower). k_filter itself stays
// under the cap: uncapped (106 SGPRs, 75 VGPRs, 20 spills instead of 44) it measured ~3% slower.
#define GHS_STREAM_KERNEL_6 __global__ __launch_bounds__(BLOCK, 6)

// bijective 32-bit mixer (xorshift-multiply; every step is invertible on u32)
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

}  // namespace ghs

// solver fields for the round loop of multi.hip (defined in boruvka.hip)
hipStream_t ghs_solver_stream_of(const ghs_solver *s);
uint32_t ghs_solver_n_of(const ghs_solver *s);
uint32_t ghs_solver_ranks_of(const ghs_solver *s);
uint64_t *ghs_solver_best_slots_of(ghs_solver *s);
int ghs_solver_flag_bits_async(ghs_solver *s, uint64_t **d_bits, uint64_t *words);
// a multi-rank driver's shared failure flag: the solver's waits end once it is set
void ghs_solver_set_group_cancel(ghs_solver *s, const int *flag);
bool ghs_solver_cancelled_of(const ghs_solver *s);
// the multi-rank round loop's contract: rounds >= 2 of a level pipelined (no host sync)
int ghs_solver_contract_async(ghs_solver *s, int *done);
// the multi-rank loop's LDS tail: the collectives it needs, enqueued on the solver's stream
struct GhsTailColl {
  void *ctx;
  int (*min_u64)(void *ctx, uint64_t *buf, size_t count, hipStream_t st);  // in place, MIN
  int (*max_i32)(void *ctx, int32_t *buf, size_t count, hipStream_t st);   // in place, MAX
};
// 0: not applicable (run the round as usual); 1: the level finished; 2: so did the solve; < 0: error
int ghs_solver_tail_multi(ghs_solver *s, const GhsTailColl *coll);
const ghs_config_t *ghs_solver_cfg_of(const ghs_solver *s);
uint32_t ghs_solver_round_of(const ghs_solver *s);
// pinned host resources of a solver (report ring, counters mirror, events), kept across solves by
// the multi-rank drivers' cache: solver creation over them allocates nothing on the host
void *ghs_hostres_new(int *rc);
void ghs_hostres_delete(void *res);
int ghs_solver_create_pooled(uint32_t n, uint64_t m, const uint32_t *d_u, const uint32_t *d_v, const uint32_t *d_w,
                             uint64_t e_lo, uint64_t e_hi, const ghs_config_t *cfg, void *d_workspace,
                             size_t workspace_bytes, uint8_t *d_in_mst, void *stream, void *hostres,
                             ghs_solver_t **out);

// ghs_flags_to_eids' cached temporaries (ingest.hip), freed by ghs_release_cache (multi.hip)
void ghs_release_eid_temps();

#define GHS_HIP_CHECK(expr)                                                                     \
  do {                                                                                          \
    hipError_t _e = (expr);                                                                     \
    if (_e != hipSuccess) {                                                                     \
      ::ghs::set_error(std::string(#expr) + ": " + hipGetErrorString(_e) + " (" __FILE__ ":" + \
                       std::to_string(__LINE__) + ")");                                         \
      return GHS_E_HIP;                                                                         \
    }                                                                                           \
  } while (0)

#define GHS_FAIL(code, msg)          \
  do {                               \
    ::ghs::set_error(msg);           \
    return (code);                   \
  } while (0)
