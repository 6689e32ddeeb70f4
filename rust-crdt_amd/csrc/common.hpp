// Internal shared definitions for libcrdt_gpu (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "crdt_gpu.h"
#include "shard_host.hpp"

namespace crdt {

using u64 = unsigned long long;
using u64x2 = unsigned long long __attribute__((ext_vector_type(2)));

// One wave is 64 lanes on gfx950; every block size below is a multiple of it.
constexpr int kWave = 64;

// Waves per SIMD asked of the A > 64 map_apply_kernel instances (0: the compiler's choice).  The
// A <= 64 instance asks for 7 (map_apply.hip).  Round 1 blamed a miscompute of a forced-7 build
// on spilling; the cause was a readlane of a spilled VGPR inside a one-lane branch (only the
// active lane's copy is reloaded), fixed in map_apply.hip, and the forced build now passes
// tests/test_gpu_map_apply.py (profiles/r02_map_apply_wpe7_tests.log).
#ifndef CRDT_APPLY_WPE
#define CRDT_APPLY_WPE 0
#endif
#if CRDT_APPLY_WPE
#define CRDT_APPLY_ATTR __attribute__((amdgpu_waves_per_eu(CRDT_APPLY_WPE)))
#else
#define CRDT_APPLY_ATTR
#endif
constexpr int kBlock = 256;

struct KernelTimer {
  double total_ms = 0.0;
  uint64_t launches = 0;
};

// Launch-geometry knobs (defaults chosen by measurement).  Overridable for
// tuning runs through the environment variable CRDT_TUNE="key=value,..." read at ctx create.
struct Tune {
  int lub_blocks_per_cu = 1;
  int lub_grid = 0;  // >0: total workgroups target (overrides lub_blocks_per_cu)
  int lub_min_steps = 16;
  int lub_interleave = 0;
  int lub_unroll = 8;
  int lub_nt = 1;
  int orswot_blocks_per_cu = 2;
  int orswot_unroll = 1;
  int orswot_mpt = 4;  // member rows per thread of the join (4, 8, 16)
  int merge_blocks_per_cu = 2;
  int merge_rows = 1;  // merge_batch of 16-byte rows by LR-lane row groups (0: merge_pairs_kernel)
  int map_glds = 1;    // Map fold: LDS-DMA staging where the shape allows it
  int map_chunk = 16;  // ... replicas per LDS chunk slot (8 or 16)
  int map_ring = 2;    // ... chunk slots in the ring (2-4)
  int map_spec = 1;    // ... speculative no-op scan
  int map_nt = 0;      // ... non-temporal policy on the LDS-DMA step images
  int map_scan2 = 0;   // ... scan two actors per 16-byte LDS read (even A; measured no faster)
  int map_scan3 = 1;   // ... scan from per-actor thresholds with every LDS read issued first
  int map_rs = 1;      // ... register-staged whole-chunk skip (A <= 32 on the LDS-DMA shapes)
  int map_batch = 1;   // ... RS path: chunk-test compares batched ahead of their scalar ANDs
  int map_sh = 0;      // ... RS path at A = 32, V = 2, K % 4 == 0: four key waves share each chunk's clock
                       //     rows (less traffic, but slower: the coupled waves; opt-in)
  int map_lazyv = 1;   // ... RS path: values fetched only for chunks the exact loop runs (not streamed)
  int map_st = 0;      // ... RS path at A = 32, V = 2: two waves per key, each testing 8 steps of a chunk (ST)
  int shagree = 0;     // sharded calls: 1 = the validation-header exchange on every call (no agreed-plan path)
  int map_diag = 0;    // ... timing probes only, results WRONG (bit0: no clock-max piece, bit1: 3 fewer step pieces)
  int rows_blocks_per_cu = 0;  // row-pair / row-reduction kernels (causal.hip); 0 = per-kernel default
  int apply_hot_slots = 8;     // Orswot apply: deferred slots kept in LDS per state (the rest in HBM)
  int map_apply_hot = 1 << 20;  // Map apply: cap on the deferred slots kept in LDS (default: all that fit)
  int map_forget_vec2 = 1;     // Map forget: 16-byte pieces per lane where the shape allows it
  int map_pair_reg = 1;        // Map merge_batch, V <= 4: 1 sub-wave register kernel, 2 whole-wave one, 0 generic
  int pair_rows = 256;         // Orswot merge_batch: member rows per workgroup (64, 128, 256)
  int pair_ur = 8;             // ... member rows per thread in flight (2, 4 at 128 rows; 8)
  int pair_occ = 1;            // ... cap on workgroups per CU (LDS padding; 0 = none): one workgroup
                               //     per CU keeps fewer HBM requests in flight, 69% -> 74-75% of 8 TB/s
  int map_forget_bpc = 1;      // Map forget, 16-byte kernel: workgroups per CU (1: 67% of 8 TB/s vs 64% at 4)
  int map_pair_pf = 0;         // Map merge_batch sub-wave key pass: the next keys' rows loaded before the merge
                               //     (opt-in: 5.86 vs 5.81 ms at 4 waves/SIMD, profiles/r04_map_pair_pf_ab.log)
  int map_pair_nt = 1;         // ... sub-wave key pass: key rows loaded / stored non-temporal (5.14 -> 5.00 ms,
                               //     profiles/r04_map_pair_nt_ab.log)
  int map_pair_bpc = 64;       // Map merge_batch key pass: workgroups per CU (grid-stride over keys;
                               //     latency-bound: 16 -> 64 is 64% -> 67-69% of 8 TB/s)
  int merge_flat = 1;          // lattice merge_batch of packed rows: workgroups per CU of the flat
                               //     stream (0: the row-group kernels)
  int merge_flat_u = 2;        // ... 16-byte pieces per lane in flight before the first store (1, 2, 4)
  int merge_ppl = 8;           // lattice merge_batch rows: 16-byte pieces per lane per row
  int stage_kb = 262144;       // CRDT_MEM_HOST: bytes per device chunk buffer (KiB; two buffers)
  int wire_walk = 1;           // Map ingest: walk + batched parse (0: one dependent chain per state)
  int wire_fill = 1;           // Orswot ingest: rows zeroed by filler waves beside the walk (0: a fill pass first)
  int host_stream = 1;         // CRDT_MEM_HOST Orswot / Map lub_many: stream replica chunks (0: stage whole)
  int apply_lane = 1;          // Orswot apply at A <= 64: 16 lanes per state (0: one wave per state)
  int apply_fence = 0;         // Orswot / Map apply: a workgroup fence after every op's stores (round-2 form)
  int orswot_apply_pf = 0;     // Orswot apply (16-lane groups): an Rm's clock row loaded during the op before
                               //     (opt-in: 4 VGPRs spill, 990 vs 918 us, profiles/r04_orswot_apply_pf_ab.log)
  int orswot_apply_stg = 0;    // Orswot apply (16-lane groups): a batch's first 2 Rm clock rows staged in LDS by LDS-DMA
                               //     (opt-in: 872 vs 854 us, profiles/r05_oapply_stg_ab.log)
  int orswot_apply_l2pf = 0;   // Orswot apply (16-lane groups): a one-member Rm's entry row touched with the batch header
                               // (lines pulled toward L2 while the header's other loads are in flight; CRDT_TUNE oal2=1)
  int orswot_apply_meta = 1;   // Orswot apply (16-lane groups): per-slot member blooms in LDS (oameta)
  int orswot_apply_hpf = 0;    // Orswot apply (16-lane groups): the next op batch's fields / first members loaded
                               //     while the current batch runs (opt-in: 2 VGPRs spill, 878 vs 856 us, profiles/r04_oapply_hpf_ab.log)
  int map_counter_dma = 0;     // Map<K, counter> fold: LDS-DMA ring slots (8 or 16; 0: register ring, 8.7 vs 9.1 ms)
  int map_counter_depth = 8;   // Map<K, counter> fold: register-ring depth at A <= 64 (4, 8, 16; 16: 4.86 vs 4.33 ms)
  int map_counter_kpw = 0;     // Map<K, counter> fold: keys per wave (1, 2, 4; A <= 64 / KPW; 0: automatic)
  int map_counter_cs = 1;      // Map<K, counter> fold: whole-chunk skip (A = 8, 16, 32; one key per wave)
  int map_counter_cl = 0;      // ... its chunks staged in LDS by LDS-DMA (opt-in: 2.24 vs 2.07 ms in registers,
                               //     profiles/r05_map_counter_cl_ab.log; the fold is issue-bound per wave)
  int map_orswot_cs = 0;       // Map<K, Orswot> fold: whole-chunk skip (A = 8, 16, 32; M <= 4; opt-in: the kernel
                               //     takes as long as its slowest key, and on the config-4 generator's replicas
                               //     some keys change in most chunks, profiles/r05_map_orswot_chunk_ab.log)
  int map_orswot_wide = 0;     // Map<K, Orswot> fold: the wide kernel at every shape (it is used past A = 64 / M = 32)
  int map_nested_lds = 1;      // Map<K, Map<K2, MVReg>> fold: inner state in LDS + staged replica rows, where they fit
  int map_apply_meta = 1;      // Map apply (16-lane groups, with mapf): per-slot key blooms in LDS (mameta)
  int map_apply_pf = 1;        // Map apply (16-lane groups): the next op's entry-clock row prefetched with its
                               //     Put / rm clock; absent keys skip their value rows (0: round-3 form;
                               //     1.28 vs 1.81 ms, profiles/r04_map_apply_pf_ab.log)
};

struct PendingTiming {
  std::string name;
  hipEvent_t start, stop;
};

}  // namespace crdt

struct crdt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int cu_count = 256;
  bool timing = false;
  crdt::Tune tune;
  std::string last_error;
  // Device scratch (grown on demand, never shrunk; freed in destroy).
  void *scratch = nullptr;
  size_t scratch_bytes = 0;
  // Second region for the Orswot deferred-remove bookkeeping (used after the join).
  void *dscratch = nullptr;
  size_t dscratch_bytes = 0;
  // Arrival counters of the last-arriver combines: a dedicated region that is zero between
  // calls (kernels reset every counter they use), never shared with scratch.
  unsigned *counters = nullptr;
  size_t counters_n = 0;
  // Pinned host staging for small host->device copies of caller arrays (crdt_orswot_lub_many
  // def_off): the caller's memory is not read after return.
  void *pinned = nullptr;
  size_t pinned_bytes = 0;
  hipEvent_t pinned_done = nullptr;
  std::map<std::string, crdt::KernelTimer> timers;
  std::vector<crdt::PendingTiming> pending;
  std::vector<hipEvent_t> free_events;
  // Multi-GPU (csrc/shard.hip): this rank's RCCL communicator and the buffers of the exchange
  // (partials, gathered partials, deferred pools), owned by the ctx and reused.
  void *comm = nullptr;
  int nranks = 1, rank = 0;
  void (*comm_destroy)(void *) = nullptr;
  void *sbuf[8] = {};
  size_t sbuf_bytes[8] = {};
  // ... or the caller's own collectives (crdt_ctx_comm_init_ops) instead of RCCL
  bool has_ops = false;
  crdt_comm_ops ops{};
  // validation agreement before the first data collective of every sharded call: a side stream
  // (so the agreement overlaps the local fold), its events, a device and a pinned host header
  // buffer of nranks rows; released by comm_release (shard.hip)
  hipStream_t astream = nullptr;
  hipEvent_t a_main = nullptr, a_done = nullptr;
  void *a_dev = nullptr, *a_host = nullptr;
  size_t a_rows = 0;
  std::string comm_note;  // e.g. an RCCL runtime / header version mismatch found at init
  void (*comm_release)(crdt_ctx *) = nullptr;
  // agreed plans (shard_host::PlanCache keys) and the pending check of the last cached-path call:
  // 3 device words all-reduced beside the data, their pinned host copy [send 3 | reduced 3] and the
  // event after the copy back (shard.hip)
  crdt::shard_host::PlanCache plans;
  bool chk_pending = false;
  uint64_t chk_key = 0;
  void *chk_dev = nullptr;
  uint64_t *chk_host = nullptr;
  hipEvent_t chk_ev = nullptr;
  int (*comm_check)(crdt_ctx *) = nullptr;  // the pending check (crdt_ctx_synchronize runs it)
  // Host-memory mode (csrc/host_stage.hip): CRDT_MEM_DEVICE / CRDT_MEM_HOST, the copy stream, two
  // device chunk buffers with their copied / free events, and the device accumulator.
  int mem_kind = CRDT_MEM_DEVICE;
  hipStream_t hstream = nullptr;
  void *hbuf[2] = {};
  size_t hbuf_bytes = 0;
  void *hacc = nullptr;
  size_t hacc_bytes = 0;
  hipEvent_t hcopied[2] = {}, hfree[2] = {};
};

namespace crdt {

int fail(crdt_ctx *ctx, int code, const char *fmt, ...);
int hip_fail(crdt_ctx *ctx, hipError_t e, const char *what);
// Ensure ctx->scratch holds at least `bytes`; returns CRDT_OK or CRDT_ENOMEM.
int ensure_scratch(crdt_ctx *ctx, size_t bytes);
int ensure_dscratch(crdt_ctx *ctx, size_t bytes);
// Ensure ctx->counters holds at least n zeroed counters.
int ensure_counters(crdt_ctx *ctx, size_t n);
// Copy `bytes` of host memory to device memory `dst` on the ctx stream; `src` is read before
// return (through a pinned staging buffer), so the caller may free it immediately.
int stage_h2d(crdt_ctx *ctx, void *dst, const void *src, size_t bytes);
// Fill `bytes` of device memory with `byte` by a kernel on the ctx stream.
int device_fill(crdt_ctx *ctx, void *dst, size_t bytes, unsigned char byte);
// Bracket the dominant kernel of a call with events when timing is on.
void timing_begin(crdt_ctx *ctx, const char *name);
void timing_end(crdt_ctx *ctx);
// Host wall time of a host-synchronous step (e.g. the sharded calls' header agreement), recorded
// under `name` like a kernel timing when timing is on.
void timing_add_host(crdt_ctx *ctx, const char *name, double ms);

// Pooled deferred-remove list of a batch (Orswot members / Map keys): survival !(rm <= final
// clock), optional ceiling forget on the joined entries, representative + set union of
// survivors with identical rm clocks (orswot.rs:240-249, map.rs:336-345).
struct DefPlan {
  const size_t *def_off;  // device copy, G+1 (set by launch_deferred)
  unsigned long long G, D, M, A, Mw;
  const u64 *def_clock, *def_members;
  const u64 *out_clock;
  u64 *out_entries;   // joined entries [G][M][A] (ceiling target when apply_ceiling)
  int apply_ceiling;
  u64 *hash;          // [D]
  unsigned *surv;     // [D] compacted survivor list
  unsigned *nsurv;    // counter
  uint8_t *out_keep;
  u64 *out_members;
  u64 *tkey;          // dedup table: keys (0 = empty) [tmask+1]
  unsigned *trep;     // ... min survivor index per key
  unsigned long long tmask;
};
// The pool's CSR offsets come from the host (staged) or, with dev_def_off, from device memory
// (checked and clamped on the device by stage_def_off_dev below; no host sync).
int launch_deferred(crdt_ctx *ctx, const size_t *host_def_off, DefPlan q, const u64 *dev_def_off = nullptr,
                    unsigned *status = nullptr);
// dst[i] = src[i] clamped to [0, D] (dst[0] = 0, dst[G] = D), so every kernel that walks the
// offsets stays inside the pool; an invalid entry i (i = 0: != 0, i = G: != D, else > D or below
// entry i-1) ORs bit 0 into *status and bit 1 into flags[i-1] / flags[i] (each may be NULL).
int stage_def_off_dev(crdt_ctx *ctx, const u64 *src, size_t *dst, size_t G, size_t D, unsigned *status,
                      unsigned *flags);

// Max / OR join on u64 lanes.
enum class Op : int { Max = 0, Or = 1 };

template <Op OP>
__device__ __forceinline__ u64 join(u64 a, u64 b) {
  if constexpr (OP == Op::Max) return a > b ? a : b;
  else return a | b;
}
template <Op OP>
__device__ __forceinline__ u64x2 join2(u64x2 a, u64x2 b) {
  u64x2 r;
  r.x = join<OP>(a.x, b.x);
  r.y = join<OP>(a.y, b.y);
  return r;
}

// Host entry for the lattice (max / or) lub used by vclock, gcounter, pncounter and gset.
int lattice_lub_many(crdt_ctx *ctx, Op op, const u64 *in, size_t G, size_t R, size_t W,
                     size_t row_stride, size_t group_stride, u64 *out, size_t out_stride,
                     unsigned flags);
int lattice_merge_batch(crdt_ctx *ctx, Op op, u64 *self, const u64 *other, size_t N, size_t W,
                        size_t self_stride, size_t other_stride);
// One lattice lub of a multi-segment call (crdt_lub_many_multi): W = words per replica row.
struct LubReq {
  Op op;
  const u64 *in;
  size_t G, R, W, row_stride, group_stride;
  u64 *out;
  size_t out_stride;
  unsigned flags;
};
int lattice_lub_many_multi(crdt_ctx *ctx, const LubReq *reqs, size_t n);
int lub_reqs_from_segments(crdt_ctx *ctx, const crdt_lub_segment *segs, size_t nseg, std::vector<LubReq> &reqs);

// Host-memory mode (host_stage.hip): the same entry points over host pointers, staged in chunks.
int lattice_lub_many_host(crdt_ctx *ctx, Op op, const u64 *in, size_t G, size_t R, size_t W,
                          size_t row_stride, size_t group_stride, u64 *out, size_t out_stride,
                          unsigned flags);
int lattice_merge_batch_host(crdt_ctx *ctx, Op op, u64 *self, const u64 *other, size_t N, size_t W,
                             size_t self_stride, size_t other_stride);
int lww_lub_many_dev(crdt_ctx *ctx, const u64 *marker, const u64 *val, size_t G, size_t R, size_t group_stride,
                     u64 *out_marker, u64 *out_val, u64 *first_conflict, unsigned flags);
int lww_merge_batch_dev(crdt_ctx *ctx, u64 *sm, u64 *sv, const u64 *om, const u64 *ov, size_t N, uint8_t *conflict);
int lww_lub_many_host(crdt_ctx *ctx, const u64 *marker, const u64 *val, size_t G, size_t R, size_t group_stride,
                      u64 *out_marker, u64 *out_val, u64 *first_conflict, unsigned flags);
int lww_merge_batch_host(crdt_ctx *ctx, u64 *sm, u64 *sv, const u64 *om, const u64 *ov, size_t N, uint8_t *conflict);
int orswot_lub_many_host(crdt_ctx *ctx, const crdt_orswot_batch *in, crdt_orswot_out *out);
// Device-mode Orswot lub_many with a fold start (the left fold continues from init instead of the
// empty Orswot; device [G][A] / [G][M][A] packed, or NULL) and per-group flags (device u32 [G],
// zeroed by the call, bit 0 = some input cell had E > C; or NULL).  Used by the sharded fold.
struct OrswotJoinExtra {
  const u64 *init_clock = nullptr, *init_entries = nullptr;
  unsigned *viol = nullptr;
};
int orswot_lub_many_ex(crdt_ctx *ctx, const crdt_orswot_batch *in, crdt_orswot_out *out, const OrswotJoinExtra &ex);
int orswot_merge_batch_host(crdt_ctx *ctx, const crdt_orswot_states *self, const crdt_orswot_states *other,
                            uint32_t *status);
int map_lub_many_host(crdt_ctx *ctx, const crdt_map_batch *in, crdt_map_out *out);
int map_counter_lub_many_host(crdt_ctx *ctx, const crdt_map_counter_batch *in, crdt_map_counter_out *out);
int map_orswot_lub_many_host(crdt_ctx *ctx, const crdt_map_orswot_batch *in, crdt_map_orswot_out *out);
int map_nested_lub_many_host(crdt_ctx *ctx, const crdt_map_nested_batch *in, crdt_map_nested_out *out);
// The workgroup-per-key Map fold for A > 256 or V > 8 (map_wide.hip): def_off_dev = the device copy
// of the deferred offsets (or NULL); outputs and flags as crdt_map_lub_many (flags zeroed by the caller).
int map_lub_wide(crdt_ctx *ctx, const crdt_map_batch *in, const size_t *def_off_dev, crdt_map_out *out);
int map_merge_batch_host(crdt_ctx *ctx, const crdt_map_states *self, const crdt_map_deferred *self_def,
                         const crdt_map_states *other, const crdt_map_deferred *other_def, uint32_t *status);
void free_stage(crdt_ctx *ctx);

// Wave-uniform row-group loop: every lane runs the same iterations (rows past N are masked),
// so group-wide votes and shuffles see the whole wave.
#define ROW_GROUP_LOOP(N, lr_log)                                                                  \
  const int lane = threadIdx.x % kWave;                                                             \
  const int LR = 1 << (lr_log);                                                                     \
  const int gl = lane & (LR - 1);                                                                   \
  const unsigned long long RW = kWave >> (lr_log);                                                  \
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;   \
  const unsigned long long nw = (unsigned long long)gridDim.x * (kBlock / kWave);                   \
  for (unsigned long long rb = w0 * RW; rb < (N); rb += nw * RW)

// LR lanes per row (power of two, <= 64) so that each lane moves about 8 pieces of its row.
inline int row_lr_log(unsigned long long pieces, unsigned long long ppl = 8) {
  int lg = 0;
  while (lg < 6 && (pieces + (1ull << lg) - 1) >> lg > ppl) ++lg;
  return lg;
}

}  // namespace crdt

#define CRDT_CHECK_CTX(ctx)                   \
  do {                                        \
    if (!(ctx)) return CRDT_EINVAL;           \
  } while (0)

#define CRDT_HIP(ctx, expr)                            \
  do {                                                 \
    hipError_t _e = (expr);                            \
    if (_e != hipSuccess) return crdt::hip_fail((ctx), _e, #expr); \
  } while (0)

// Entry points without a host-memory path: refuse CRDT_MEM_HOST instead of reading host
// pointers as device memory (host_stage.hip lists the ones that have one).
#define CRDT_DEVICE_MEM_ONLY(ctx)                                                              \
  do {                                                                                         \
    if ((ctx) && (ctx)->mem_kind != CRDT_MEM_DEVICE)                                            \
      return crdt::fail((ctx), CRDT_EUNSUPPORTED, "%s: device pointers only (CRDT_MEM_HOST is " \
                        "supported by the lattice and lwwreg lub_many / merge_batch)", __func__); \
  } while (0)
