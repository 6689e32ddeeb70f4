/*
 * crdt_gpu.h — C ABI of the MI355X batched CvRDT merge engine (libcrdt_gpu.so).
 *
 * Drop-in boundary for the `crdts` 3.0.0 (rust-crdt) state-merge path.  The reference
 * exposes one merge per pair of states:
 *
 *     CvRDT::merge(&mut self, other: Self)                      traits.rs:4-7
 *     FunkyCvRDT::merge(&mut self, other) -> Result<(), Error>  traits.rs:49-55 (LWWReg)
 *
 * and users fold it over replicas (`acc.merge(r)` loops, test/orswot.rs:50-53,
 * pncounter.rs:151-154).  This library adds the batched forms a `gpu` module of the
 * crate binds through `extern "C"` (see INTEGRATION.md for the Rust / ctypes stubs):
 *
 *     *_lub_many    — G independent left folds, each over R replicas  (acc = T::new(); for r: acc.merge(r))
 *     *_merge_batch — N independent pairwise merges, self[i].merge(other[i]), in place
 *
 * States are dense structure-of-arrays in device memory (HBM): actors/members are interned
 * to dense indices by the caller, an absent actor is a 0 counter (exact: VClock::apply_dot
 * never stores 0, vclock.rs:155-159).  All pointers are DEVICE pointers unless stated or the
 * ctx is in CRDT_MEM_HOST mode (crdt_ctx_set_mem_kind below).
 * Every stride is in 64-bit words.  Results are bit-exact against the reference fold.
 *
 * Conventions
 *   - Return value: CRDT_OK (0) or a negative status; crdt_last_error() has the text.
 *     No C++ exception crosses this ABI.  LWW marker conflicts are DATA, not a status.
 *   - Calls are stream-ordered on the ctx's stream and asynchronous unless stated.
 *     The caller owns every buffer; the library keeps no pointer past return.
 *   - One ctx per host thread; a ctx is bound to one device.
 */
#ifndef CRDT_GPU_H
#define CRDT_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------ */
#define CRDT_OK 0
#define CRDT_EINVAL -1       /* bad argument (null pointer, zero dim, stride < width, ...) */
#define CRDT_EHIP -2         /* a HIP runtime call failed                                   */
#define CRDT_ENOMEM -3       /* device scratch allocation failed                            */
#define CRDT_EUNSUPPORTED -4 /* shape the kernels do not handle                             */
#define CRDT_ECOMM -5        /* an RCCL call failed (sharded entry points)                  */

/* ---- flags for *_lub_many ---------------------------------------------------------- */
/* out := out ⊔ fold(in) instead of out := fold(in): i.e. `self.merge(r)` for every r,
 * starting from the caller's current state rather than from T::new(). */
#define CRDT_ACCUMULATE 0x1u

typedef struct crdt_ctx crdt_ctx;

/* ---- context ------------------------------------------------------------------------- */
/* Create a ctx bound to HIP device `device` (>= 0).  Scratch is owned by the ctx. */
int crdt_ctx_create(int device, crdt_ctx **out);
int crdt_ctx_destroy(crdt_ctx *ctx);
/* Launch on `hip_stream` (a hipStream_t; NULL = the device's null stream). */
int crdt_ctx_set_stream(crdt_ctx *ctx, void *hip_stream);
/* Block until all work issued through ctx has finished. */
int crdt_ctx_synchronize(crdt_ctx *ctx);
/* Text of the last failure on this ctx (static storage owned by ctx). ctx may be NULL. */
const char *crdt_last_error(const crdt_ctx *ctx);
/* Library version, e.g. "0.6.0"; and the gfx target the code objects were built for. */
const char *crdt_version(void);
/* ABI revision of this header: bumped whenever a struct or signature changes incompatibly (round 5
 * appended `size_t Dv` to crdt_map_orswot_batch: revision 5 -> 6; round 6 appended `size_t Vd` to
 * crdt_map_orswot_states / crdt_map_orswot_out and `size_t Id` to crdt_map_nested_states /
 * crdt_map_nested_out: 7 -> 8).  A caller checks
 * crdt_abi_version() == CRDT_ABI_VERSION of the header it was built against before any other call,
 * so a mismatched library fails clearly instead of reading a shorter struct. */
#define CRDT_ABI_VERSION 8
int crdt_abi_version(void);
const char *crdt_build_target(void);

/* Per-kernel timing with HIP events recorded on the ctx stream around the DOMINANT kernel of
 * each call (the replica stream pass).  Enabling costs two event records per call. */
int crdt_ctx_set_timing(crdt_ctx *ctx, int enable);
/* Sum of elapsed ms and launch count for kernel class `name` ("lub_stream", "orswot_join",
 * "lww_reduce", ...) since the last reset.  Synchronises the ctx stream. */
int crdt_ctx_timing(crdt_ctx *ctx, const char *name, double *total_ms, uint64_t *launches);
int crdt_ctx_timing_reset(crdt_ctx *ctx);
/* Override launch-geometry knobs ("key=value,...", the CRDT_TUNE syntax read at create; see
 * DESIGN.md §3).  Results never depend on them; tests use it to exercise every staging path. */
int crdt_ctx_tune(crdt_ctx *ctx, const char *spec);

/* ---- memory kind (crdt_mem_kind) ---------------------------------------------------------
 * CRDT_MEM_DEVICE (default): every buffer pointer is a device pointer and calls are
 * asynchronous on the ctx stream.  CRDT_MEM_HOST: the buffers of
 *     crdt_{vclock,gcounter,pncounter,gset}_lub_many / _merge_batch,
 *     crdt_lwwreg_lub_many / _merge_batch,
 *     crdt_orswot_lub_many / _merge_batch, crdt_map_lub_many / _merge_batch (every pointer in
 *     the structs; def_off stays host)
 * are HOST pointers (pageable, or pinned by crdt_host_alloc for direct DMA).  The lub_many forms
 * stream them through two ctx-owned device chunk buffers (tune key stage_kb, default 256 MiB
 * each), overlapping the H2D copy of chunk k+1 with the fold of chunk k: lattice / LWW folds
 * accumulate; Orswot joins each chunk into a running join kept in HBM and settles the deferred
 * removes once at the end; Map folds each chunk behind the running fold as its replica 0 (its
 * surviving removes carried along), falling back to whole-batch staging when a key needs more than
 * 8 value slots mid-fold.  merge_batch of Orswot / Map stages the whole batch.  The call returns when
 * the results are in host memory.  Results are identical to the device-pointer call.  In host mode
 * crdt_lwwreg_lub_many needs out_marker and out_val; a device pointer is rejected (CRDT_EINVAL);
 * every other entry point returns CRDT_EUNSUPPORTED. */
#define CRDT_MEM_DEVICE 0
#define CRDT_MEM_HOST 1
int crdt_ctx_set_mem_kind(crdt_ctx *ctx, int kind);
/* The ctx's current kind, or CRDT_EINVAL for a NULL ctx. */
int crdt_ctx_mem_kind(const crdt_ctx *ctx);
/* Page-locked host memory (hipHostMalloc): host-mode inputs in it are copied by DMA at the full
 * link rate.  Free with crdt_host_free. */
int crdt_host_alloc(size_t bytes, void **out);
int crdt_host_free(void *p);
/* Device memory on the ctx's GPU in one physically contiguous block (hipExtMallocWithFlags with
 * hipDeviceMallocContiguous), for the large replica batches a fold streams once: a batch in fewer,
 * larger page fragments is walked with fewer translation misses (config 3's 128 GiB Orswot input
 * folds in 20.4 ms from such a block against 21.4-22.9 ms from a torch allocator block on the same
 * box).  CRDT_ENOMEM when no such block is free (callers fall back to any device
 * memory).  Free with crdt_device_free (its ctx may be NULL). */
int crdt_device_alloc(crdt_ctx *ctx, size_t bytes, void **out);
int crdt_device_free(crdt_ctx *ctx, void *p);

/* ---- VClock / GCounter: elementwise-max lub ----------------------------------------------
 * Replaces VClock::merge (vclock.rs:130-136, via apply_dot :155-159) and GCounter::merge
 * (gcounter.rs:44-48) folded over replicas.
 * Replica (g, r) row = in + g*group_stride + r*row_stride, A counters contiguous.
 * Output row g = out + g*out_stride.                                                    */
int crdt_vclock_lub_many(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                         size_t row_stride, size_t group_stride, uint64_t *out,
                         size_t out_stride, unsigned flags);
/* self[i] := self[i] ⊔ other[i] for i < N (rows of A counters). */
int crdt_vclock_merge_batch(crdt_ctx *ctx, uint64_t *self, const uint64_t *other, size_t N,
                            size_t A, size_t self_stride, size_t other_stride);
int crdt_gcounter_lub_many(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                           size_t row_stride, size_t group_stride, uint64_t *out,
                           size_t out_stride, unsigned flags);
int crdt_gcounter_merge_batch(crdt_ctx *ctx, uint64_t *self, const uint64_t *other, size_t N,
                              size_t A, size_t self_stride, size_t other_stride);

/* ---- PNCounter: dual max ---------------------------------------------------------------
 * Replaces PNCounter::merge (pncounter.rs:70-75).  A replica row holds 2*A words:
 * P counters in [0, A), N counters in [A, 2A).  Strides as for VClock (row_stride >= 2A). */
int crdt_pncounter_lub_many(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                            size_t row_stride, size_t group_stride, uint64_t *out,
                            size_t out_stride, unsigned flags);
int crdt_pncounter_merge_batch(crdt_ctx *ctx, uint64_t *self, const uint64_t *other,
                               size_t N, size_t A, size_t self_stride, size_t other_stride);

/* ---- GSet: bitmap union ----------------------------------------------------------------
 * Replaces GSet::merge (gset.rs:38-40 → insert :69-71).  Elements are interned to bit
 * positions; a replica row is `words` u64 words (bit u of word u/64 = element u present). */
int crdt_gset_lub_many(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t words,
                       size_t row_stride, size_t group_stride, uint64_t *out,
                       size_t out_stride, unsigned flags);
int crdt_gset_merge_batch(crdt_ctx *ctx, uint64_t *self, const uint64_t *other, size_t N,
                          size_t words, size_t self_stride, size_t other_stride);

/* ---- several lattice lubs in one launch ------------------------------------------------------
 * Each segment is one crdt_{vclock,gcounter,pncounter,gset}_lub_many call (same dims, strides,
 * flags and result); segments of the same join (max: VClock / GCounter / PNCounter; or: GSet)
 * run in ONE launch (up to 8 per launch), so a batch of CRDT states of several types pays one
 * launch ramp and tail.  A = counters per replica (PNCounter: per half) or words (GSet). */
#define CRDT_KIND_VCLOCK 1
#define CRDT_KIND_GCOUNTER 2
#define CRDT_KIND_PNCOUNTER 3
#define CRDT_KIND_GSET 4
typedef struct crdt_lub_segment {
  int kind; /* CRDT_KIND_* */
  const uint64_t *in;
  size_t G, R, A, row_stride, group_stride;
  uint64_t *out;
  size_t out_stride;
  unsigned flags;
} crdt_lub_segment;
int crdt_lub_many_multi(crdt_ctx *ctx, const crdt_lub_segment *segs, size_t nseg);

/* ---- LWWReg<u64 val, u64 marker> -------------------------------------------------------
 * Replaces FunkyCvRDT::merge for LWWReg (lwwreg.rs:43-45 → update :84-98).
 * lub_many folds group g as acc = replica[g][0]; for r in 1..R: acc.merge(replica[g][r]),
 * where an erroring merge leaves acc unchanged (exactly what update does on Err).
 * Outputs: out_marker[g], out_val[g] = the folded state (max marker, val of the FIRST
 * replica holding it); first_conflict[g] = index r of the first merge that returns
 * Err(ConflictingMarker) in that fold, or UINT64_MAX if none.  Any of the three outputs
 * may be NULL.  Inputs: marker/val at [g*group_stride + r].
 * flags = CRDT_ACCUMULATE: acc starts at the caller's state (out_marker[g], out_val[g], both
 * required) and every replica 0..R-1 is merged into it (R may then be 0). */
int crdt_lwwreg_lub_many(crdt_ctx *ctx, const uint64_t *marker, const uint64_t *val, size_t G,
                         size_t R, size_t group_stride, uint64_t *out_marker,
                         uint64_t *out_val, uint64_t *first_conflict, unsigned flags);
/* self[i].merge(other[i]) for i < N; conflict[i] = 1 where it returns Err (state then
 * unchanged), else 0.  conflict may be NULL. */
int crdt_lwwreg_merge_batch(crdt_ctx *ctx, uint64_t *self_marker, uint64_t *self_val,
                            const uint64_t *other_marker, const uint64_t *other_val,
                            size_t N, uint8_t *conflict);

/* ---- Orswot<member, actor> ---------------------------------------------------------------
 * Replaces Orswot::merge (orswot.rs:81-149) incl. apply_rm (:230-250) and apply_deferred
 * (:281-286).
 * Exact for ANY input states: the result is the left fold acc = Orswot::new(); for r in replicas
 * { acc.merge(r) }, removes included.  On the reference's own invariants (entry dots covered by
 * their replica's clock, E <= C, as every state its API builds) the per-cell join is associative
 * and the kernels fold replica slices in any grouping; where an input cell has E > C (e.g. a
 * deserialized state) the unit holding it is re-folded in replica order inside the same launch,
 * and applying the deferred removes after the in-order join equals applying them at their own
 * step.  The host-memory mode continues the fold chunk by chunk, the sharded form
 * folds the ranks in rank order when any shard holds such a cell (below).
 * Dense layout per replica (g, r):
 *   clock   C[g][r][a]      at clock   + g*clock_gstride + r*clock_rstride + a
 *   entries E[g][r][m][a]   at entries + g*entry_gstride + r*entry_rstride + m*entry_mstride + a
 *                            (E = the member's dot clock; member absent <=> row all 0)
 *   deferred removes, pooled per group (CSR): group g owns d in [def_off[g], def_off[g+1]);
 *     rm clock  def_clock[d*A + a], member set bitmap def_members[d*Mw + w], Mw = ceil(M/64).
 *     def_off is a HOST array of G+1 entries (crdt_orswot_lub_many_doff below: a device one).
 * Output per group g: out_clock[g*A + a], out_entries[g*M*A + m*A + a] (packed), and for the
 * deferred pool: out_def_keep[d] = 1 iff d is the representative of a surviving deferred
 * remove (¬(rm ≤ final clock), first of its group with that exact clock), and
 * out_def_members[d*Mw + w] = union of the member sets of every surviving deferred of the
 * group with the same clock (only meaningful where out_def_keep[d] = 1). */
typedef struct crdt_orswot_batch {
  size_t G, R, M, A;
  const uint64_t *clock;
  size_t clock_rstride, clock_gstride;
  const uint64_t *entries;
  size_t entry_mstride, entry_rstride, entry_gstride;
  const size_t *def_off; /* host, G+1 entries; NULL or all-zero = no deferred removes */
  const uint64_t *def_clock;
  const uint64_t *def_members;
} crdt_orswot_batch;

typedef struct crdt_orswot_out {
  uint64_t *clock;       /* [G][A]    */
  uint64_t *entries;     /* [G][M][A] */
  uint8_t *def_keep;     /* [D]       */
  uint64_t *def_members; /* [D][Mw]   */
} crdt_orswot_out;

int crdt_orswot_lub_many(crdt_ctx *ctx, const crdt_orswot_batch *in, crdt_orswot_out *out);
/* crdt_orswot_lub_many with the deferred pool's CSR offsets in DEVICE memory (a pool built on the
 * GPU, e.g. by crdt_orswot_ingest, needs no host round trip): in->def_off must be NULL; def_off
 * (device u64 [G+1], or NULL = no deferred removes) with def_off[G] == D, the pool length (the rows
 * of def_clock / def_members, known to the caller from its own allocation).  The offsets are checked
 * on the device: def_off[0] != 0, def_off[G] != D, an entry > D or a decreasing step set bit 0 of
 * *status (device u32, written for every call; may be NULL) and the kernels then read the offsets
 * clamped to [0, D] (in bounds; the results are unreliable).  Device-memory contexts only
 * (CRDT_EUNSUPPORTED otherwise). */
int crdt_orswot_lub_many_doff(crdt_ctx *ctx, const crdt_orswot_batch *in, const uint64_t *def_off, size_t D,
                              crdt_orswot_out *out, uint32_t *status);

/* Batched Orswot CmRDT::apply (orswot.rs:55-79 with apply_rm :230-250 and apply_deferred
 * :281-286): state s < N applies its ops [op_off[s], op_off[s+1]) in order, in place.
 * State layout (device): clock C[s][a] at clock + s*clock_stride + a; entries E[s][m][a] at
 * entries + s*entry_sstride + m*entry_mstride + a (member absent <=> row all 0); the deferred
 * list of state s has def_count[s] <= Dcap slots, slot d holding the rm clock
 * def_clock[(s*Dcap + d)*A + a] and the member bitmap def_members[(s*Dcap + d)*Mw + w],
 * Mw = ceil(M/64), clocks pairwise distinct (the reference's HashMap<VClock, HashSet<M>>).
 * Ops (device): kind[o] 0 = Op::Add { dot: (actor[o], counter[o]), members },
 * 1 = Op::Rm { clock: rm_clock[rm_row[o]*A ..], members }; members of op o are
 * mem[mem_off[o] .. mem_off[o+1]) (u32 member indices, duplicates allowed).  op_off has N+1
 * entries, mem_off n_ops+1.  actor/counter may be NULL if no op is an Add, rm_row/rm_clock if
 * none is an Rm (n_rm_rows = rows of rm_clock).
 * status[s] (device u32, written for every s): bit 0 = the deferred list needed more than Dcap
 * slots (the state is incomplete: retry with a larger Dcap), bit 1 = an op named an actor,
 * member or rm row out of range or a bad kind / member range (reversed, or ending past n_mem)
 * (that op, or its bad members, were skipped), bit 2 = def_count[s] > Dcap on input, bit 3 = op_off[s..s+1] invalid (bits 2 and 3:
 * state left untouched).  Limits: A <= 1024 (1, 4 or 16 clock words per lane; the first slots of
 * the deferred list are kept in LDS, as many as 64 KiB holds; the rest stay in the state's own
 * slots, so Dcap is not bounded). */
typedef struct crdt_orswot_states {
  size_t N, M, A, Dcap;
  uint64_t *clock;
  size_t clock_stride;
  uint64_t *entries;
  size_t entry_mstride, entry_sstride;
  uint64_t *def_clock;   /* [N][Dcap][A]  */
  uint64_t *def_members; /* [N][Dcap][Mw] */
  uint32_t *def_count;   /* [N]           */
} crdt_orswot_states;

typedef struct crdt_orswot_ops {
  size_t n_ops;
  const uint64_t *op_off; /* [N+1]     */
  const uint8_t *kind;    /* [n_ops]   */
  const uint32_t *actor;  /* [n_ops]   */
  const uint64_t *counter; /* [n_ops]  */
  const uint32_t *rm_row; /* [n_ops]   */
  const uint64_t *rm_clock; /* [n_rm_rows][A] */
  size_t n_rm_rows;
  const uint64_t *mem_off; /* [n_ops+1] */
  const uint32_t *mem;      /* [n_mem]   */
  size_t n_mem;             /* entries of mem: a member range ending past it is malformed */
} crdt_orswot_ops;

int crdt_orswot_apply_batch(crdt_ctx *ctx, const crdt_orswot_states *states, const crdt_orswot_ops *ops,
                            uint32_t *status);

/* Pairwise in-place Orswot merge (the batched form of CvRDT::merge, traits.rs:4-7 ->
 * Orswot::merge orswot.rs:81-149 with apply_rm :230-250 and apply_deferred :281-286):
 * self[i].merge(other[i]) for i < N, exact for ANY pair of states.  Both sides use the
 * crdt_orswot_states layout (the apply layout: per-state deferred slots, clocks pairwise distinct
 * within a state); N, M and A must match, Dcap may differ.  self's clock, entries, deferred slots
 * and def_count are rewritten; other is read only (its def_count may be NULL when its Dcap is 0).
 * The surviving deferred removes (!(rm <= merged clock)) of both sides are compacted into self's
 * slots (self's survivors first, in slot order, then other's; identical clocks merge their member
 * sets, as the reference's HashMap<VClock, HashSet<M>> does).
 * status[s] (device u32): bit 0 = more survivors than self's Dcap (state incomplete), bit 2 =
 * def_count above Dcap on input (state untouched).  Dcap is not bounded: a pair with more than
 * 512 removes is forgotten in further passes of 512 (forgets compose and commute). */
int crdt_orswot_merge_batch(crdt_ctx *ctx, const crdt_orswot_states *self, const crdt_orswot_states *other,
                            uint32_t *status);

/* ---- batched Causal::forget of whole states -----------------------------------
 * State s forgets the clock y + s*y_stride (y_stride = 0: one clock for every state), in place.
 * Orswot::forget (orswot.rs:150-183): clock, entry clocks (an emptied entry = all-zero row =
 *     dropped) and deferred rm clocks.  Deferred removes are a pool of D rows: row d belongs to
 *     state def_state[d] (device u32); def_keep[d] = 0 iff its rm clock emptied (dropped by the
 *     reference, :168-180); member sets are untouched.  When two surviving rm clocks of one state
 *     become equal the reference's HashMap collect keeps ONE of them with its own member set,
 *     chosen by hash iteration order (unspecified); both rows are kept here.  Rows with
 *     def_state[d] >= N are left untouched (def_keep[d] = 1).
 * Map::forget (map.rs:85-114) with V = MVReg: entry clocks, every value clock (MVReg::forget
 *     mvreg.rs:88-104: an emptied value is dropped: slot clock all 0, value 0), an entry whose own
 *     clock empties is dropped with its values, deferred rm clocks as for Orswot, the map clock.
 *     Layout (device, per state s): clock + s*clock_stride; ec + s*ec_stride + k*A;
 *     vclk + s*vclk_stride + (k*V + j)*A; vval + s*vval_stride + k*V + j (the crdt_map_lub_many
 *     slot convention: empty slot <=> all-zero clock row, skipped on egress). */
int crdt_orswot_forget_batch(crdt_ctx *ctx, uint64_t *clock, size_t clock_stride, uint64_t *entries,
                             size_t entry_mstride, size_t entry_sstride, size_t N, size_t M, size_t A,
                             const uint64_t *y, size_t y_stride, uint64_t *def_clock,
                             const uint32_t *def_state, size_t D, uint8_t *def_keep);

typedef struct crdt_map_states {
  size_t N, K, A, V;
  uint64_t *clock;
  size_t clock_stride;
  uint64_t *ec;
  size_t ec_stride;
  uint64_t *vclk;
  size_t vclk_stride;
  uint64_t *vval;
  size_t vval_stride;
} crdt_map_states;

int crdt_map_forget_batch(crdt_ctx *ctx, const crdt_map_states *states, const uint64_t *y, size_t y_stride,
                          uint64_t *def_clock, const uint32_t *def_state, size_t D, uint8_t *def_keep);

/* Map::forget (map.rs:85-114) of whole value-typed Map states (round 5), in place, arguments as
 * crdt_map_forget_batch (one forget clock per state, the Map-level deferred rm clocks as a pool of
 * D rows with their states, def_keep[d] = 0 where one emptied):
 *  - Map<K, GCounter / PNCounter>: the crdt_map_counter_lub_many output layout per state s:
 *    clock + s*clock_stride, ec + s*ec_stride + k*A, val + s*val_stride + (k*W + w)*A; a dropped
 *    entry has all-zero rows; the counter rows forget word by word (gcounter.rs:51-53,
 *    pncounter.rs:78-81).
 *  - Map<K, Orswot<M>>: the crdt_map_orswot_lub_many output layout (packed; N states), the Orswot
 *    clock, member rows and nested deferred removes forgotten (orswot.rs:150-183): an emptied member
 *    row is absent, an emptied nested rm clock dropped, two that become equal keep one entry with the
 *    later one's members at the earlier one's place (the fold's rule; the reference's HashMap order is
 *    unspecified), and a dropped entry drops its nested removes (vd_n = 0).  A <= 1,024. */
typedef struct crdt_map_counter_states {
  size_t N, K, A, W;
  uint64_t *clock;
  size_t clock_stride;
  uint64_t *ec;
  size_t ec_stride;
  uint64_t *val;
  size_t val_stride;
} crdt_map_counter_states;

int crdt_map_counter_forget_batch(crdt_ctx *ctx, const crdt_map_counter_states *states, const uint64_t *y,
                                  size_t y_stride, uint64_t *def_clock, const uint32_t *def_state, size_t D,
                                  uint8_t *def_keep);

/* Batched Map<K, GCounter / PNCounter> CmRDT::apply (round 5; map.rs:119-137 with gcounter.rs:36-42 /
 * pncounter.rs:59-68, apply_keyset_rm :318-348, apply_deferred :311-316): state s applies its ops
 * [op_off[s], op_off[s+1]) in order, in place, on the crdt_map_counter_states layout; deferred
 * removes as crdt_map_apply_batch (def_count[s] <= Dcap slots, rm clock def_clock[(s*Dcap + d)*A + a],
 * key bitmap def_keys[(s*Dcap + d)*Kw + w]).  Ops: kind 0 = Op::Up { dot: (actor, counter), key,
 * op: the counter's op (vactor, vcounter) — a Dot — with vdir 0 = P (GCounter: always 0), 1 = N
 * (vdir may be NULL: all P) }, kind 1 = Op::Rm { clock: clk_pool[clk_row*A ..], keyset: keys[key_off[o]
 * .. key_off[o+1]) }.  status[s]: bit 0 = deferred slots exhausted, bit 1 = a malformed op / key
 * skipped, bits 2-3 = invalid input (state untouched).  Limits: A <= 512.  Dcap is not bounded:
 * during the stream the first min(Dcap, 16) slots live in LDS and the rest are used in place in
 * def_clock / def_keys (round 6: exact up to Dcap; bit 0 only past Dcap).  Slots the list vacates
 * during a call (a remove that became dominated) are written zero, so a state whose slots past
 * def_count were zero keeps them zero (the wire ingest's form); the same holds for the Orswot and
 * nested Map apply below. */
typedef struct crdt_map_counter_ops {
  size_t n_ops;
  const uint64_t *op_off;    /* [N+1]       */
  const uint8_t *kind;       /* [n_ops]     */
  const uint32_t *actor;     /* [n_ops] Up: the Map's dot */
  const uint64_t *counter;   /* [n_ops] Up  */
  const uint32_t *key;       /* [n_ops] Up  */
  const uint32_t *vactor;    /* [n_ops] Up: the counter's dot */
  const uint64_t *vcounter;  /* [n_ops] Up  */
  const uint8_t *vdir;       /* [n_ops] Up: 0 P, 1 N (or NULL) */
  const uint32_t *clk_row;   /* [n_ops] Rm  */
  const uint64_t *clk_pool;  /* [n_clk_rows][A] */
  size_t n_clk_rows;
  const uint64_t *key_off;   /* [n_ops+1] Rm */
  const uint32_t *keys;      /* [n_keys]    */
  size_t n_keys;
} crdt_map_counter_ops;

int crdt_map_counter_apply_batch(crdt_ctx *ctx, const crdt_map_counter_states *states, uint64_t *def_clock,
                                 uint64_t *def_keys, uint32_t *def_count, size_t Dcap,
                                 const crdt_map_counter_ops *ops, uint32_t *status);

typedef struct crdt_map_orswot_states {
  size_t N, K, M, A;
  uint64_t *clock;    /* [N][A]            */
  uint64_t *ec;       /* [N][K][A]         */
  uint64_t *oc;       /* [N][K][A]         */
  uint64_t *ent;      /* [N][K][M][A]      */
  uint32_t *vd_n;     /* [N][K]            */
  uint64_t *vd_clock; /* [N][K][Vd][A]     */
  uint64_t *vd_mem;   /* [N][K][Vd][Mw]    */
  size_t Vd;          /* nested deferred slots per key (round 6, ABI 8; 0 = 16) */
} crdt_map_orswot_states;

int crdt_map_orswot_forget_batch(crdt_ctx *ctx, const crdt_map_orswot_states *states, const uint64_t *y,
                                 size_t y_stride, uint64_t *def_clock, const uint32_t *def_state, size_t D,
                                 uint8_t *def_keep);

/* Batched Map<K, Orswot<M>> CmRDT::apply (round 5; map.rs:119-137 with Orswot::apply orswot.rs:55-79,
 * apply_rm :230-250 and apply_deferred :281-286 inside, the Map's apply_keyset_rm :318-348 with
 * Orswot::forget :150-183 and apply_deferred :311-316): state s applies its ops [op_off[s],
 * op_off[s+1]) in order, in place, on the crdt_map_orswot_states layout (nested deferred lists of
 * <= 16 per key); the Map's deferred removes as crdt_map_counter_apply_batch.  Ops: kind 0 = Op::Up
 * { dot: (actor, counter), key, op } with vkind 0 = Orswot Add { dot: (vactor, vcounter), members }
 * or 1 = Orswot Rm { clock: clk_pool[clk_row*A ..], members }, the members mems[mem_off[o] ..
 * mem_off[o+1]); kind 1 = Op::Rm { clock: clk_pool[clk_row*A ..], keyset: keys[key_off[o] ..
 * key_off[o+1]) } (key_off may be NULL when no op is a Map Rm).  status[s]: bit 0 = a deferred list
 * (the Map's or a nested one) exhausted, bit 1 = a malformed op / key / member skipped, bits 2-3 =
 * invalid input (state untouched).  Nested removes whose clocks become equal under a Map-level
 * forget keep one entry, the later one's members (the fold's rule).  Limits: A <= 512, M <= 1,024;
 * Dcap is not bounded (the Map's first min(Dcap, 16) slots in LDS, the rest in place, round 6). */
typedef struct crdt_map_orswot_ops {
  size_t n_ops;
  const uint64_t *op_off;    /* [N+1]       */
  const uint8_t *kind;       /* [n_ops]     */
  const uint32_t *actor;     /* [n_ops] Up: the Map's dot */
  const uint64_t *counter;   /* [n_ops] Up  */
  const uint32_t *key;       /* [n_ops] Up  */
  const uint8_t *vkind;      /* [n_ops] Up: 0 Orswot Add, 1 Orswot Rm */
  const uint32_t *vactor;    /* [n_ops] Up / Add: the Orswot's dot */
  const uint64_t *vcounter;  /* [n_ops] Up / Add */
  const uint32_t *clk_row;   /* [n_ops] Up / Rm and Map Rm: row of clk_pool */
  const uint64_t *clk_pool;  /* [n_clk_rows][A] */
  size_t n_clk_rows;
  const uint64_t *key_off;   /* [n_ops+1] Map Rm keysets */
  const uint32_t *keys;      /* [n_keys]    */
  size_t n_keys;
  const uint64_t *mem_off;   /* [n_ops+1] Up: the Orswot op's members */
  const uint32_t *mems;      /* [n_mems]    */
  size_t n_mems;
} crdt_map_orswot_ops;

int crdt_map_orswot_apply_batch(crdt_ctx *ctx, const crdt_map_orswot_states *states, uint64_t *def_clock,
                                uint64_t *def_keys, uint32_t *def_count, size_t Dcap,
                                const crdt_map_orswot_ops *ops, uint32_t *status);

/* Batched Map<K, MVReg<u64>> CmRDT::apply (map.rs:119-137, apply_keyset_rm :318-348,
 * apply_deferred :311-316, MVReg::apply mvreg.rs:130-166): state s applies its ops
 * [op_off[s], op_off[s+1]) in order, in place, on the crdt_map_states layout (value slots in Vec
 * order, empty slot <=> all-zero clock; an append goes after the last used slot, compacting the
 * slots when that one is the last).  Deferred removes: def_count[s] <= Dcap slots, rm clock
 * def_clock[(s*Dcap + d)*A + a], key bitmap def_keys[(s*Dcap + d)*Kw + w], Kw = ceil(K/64).
 * Ops: kind 0 = Op::Up { dot: (actor, counter), key, op: Put { clock: clk_pool[clk_row*A ..],
 * val } }, kind 1 = Op::Rm { clock: clk_pool[clk_row*A ..], keyset: keys[key_off[o] ..
 * key_off[o+1]) } (key_off: n_ops+1 entries, may be NULL when no op is an Rm).
 * status[s]: bit 0 = deferred slots exhausted, bit 1 = an out-of-range op / key skipped (incl. a
 * key range reversed or ending past n_keys),
 * bits 2-3 = invalid input (state untouched), bit 4 = a register needed more than V values (the
 * state is incomplete: retry with more slots), bit 5 = internal slot invariant violated (never
 * expected; the value was not written).  Limits: A <= 1024, V >= 1 (the value slots are walked in
 * HBM, so V is not bounded; the first deferred slots are kept in LDS, as many as 64 KiB holds; the
 * rest stay in the state's own slots). */
typedef struct crdt_map_ops {
  size_t n_ops;
  const uint64_t *op_off;   /* [N+1]       */
  const uint8_t *kind;      /* [n_ops]     */
  const uint32_t *actor;    /* [n_ops] Up  */
  const uint64_t *counter;  /* [n_ops] Up  */
  const uint32_t *key;      /* [n_ops] Up  */
  const uint64_t *val;      /* [n_ops] Up  */
  const uint32_t *clk_row;  /* [n_ops]     */
  const uint64_t *clk_pool; /* [n_clk_rows][A] */
  size_t n_clk_rows;
  const uint64_t *key_off;  /* [n_ops+1] Rm */
  const uint32_t *keys;     /* [n_keys]    */
  size_t n_keys;            /* entries of keys: a key range ending past it is malformed */
} crdt_map_ops;

int crdt_map_apply_batch(crdt_ctx *ctx, const crdt_map_states *states, uint64_t *def_clock, uint64_t *def_keys,
                         uint32_t *def_count, size_t Dcap, const crdt_map_ops *ops, uint32_t *status);

/* Deferred-remove slots of N Map states (the crdt_map_apply_batch convention): state s holds
 * count[s] <= Dcap removes, rm clock clock[(s*Dcap + d)*A + a], key bitmap keys[(s*Dcap + d)*Kw + w]. */
typedef struct crdt_map_deferred {
  uint64_t *clock;
  uint64_t *keys;
  uint32_t *count;
  size_t Dcap;
} crdt_map_deferred;

/* Pairwise in-place Map<K, MVReg<u64>> merge: self[i].merge(other[i]) for i < N (Map::merge
 * map.rs:140-220, MVReg::merge mvreg.rs:112-128, MVReg::forget :88-104, apply_keyset_rm
 * map.rs:318-348), exact for ANY pair of states, on the crdt_map_states layout (N, K, A equal on
 * both sides; V may differ; value slots in Vec order: self's kept values then other's added ones,
 * written from slot 0, empty slots zeroed).  Deferred removes as crdt_orswot_merge_batch over key
 * bitmaps.  status[s]: bit 0 = deferred slots exhausted, bit 2 = invalid def_count (untouched),
 * bit 4 = some register needed more than self's V slots (that key is incomplete).
 * Limits: A <= 1024, 1 <= V <= 32 on each side (Dcap is not bounded). */
int crdt_map_merge_batch(crdt_ctx *ctx, const crdt_map_states *self, const crdt_map_deferred *self_def,
                         const crdt_map_states *other, const crdt_map_deferred *other_def, uint32_t *status);

/* ---- multi-GPU: replica-sharded lub over RCCL ----------------------------
 * One process (one ctx) per GPU.  Rank 0 calls crdt_comm_unique_id and sends the 128 bytes to
 * every rank over the caller's own channel; every rank then calls crdt_ctx_comm_init (collective:
 * all ranks must call it).  The *_sharded calls are collective too: rank k passes its own replica
 * shard (same G and row width on every rank, any R_k >= 0) and every rank receives the global
 * lub, equal to lub_many over the concatenation of the shards.
 *   vclock / gcounter / pncounter: local lub_many + one ncclAllReduce(ncclUint64, ncclMax) of the
 *       packed G x W partials (W = A, 2A for PNCounter) — out is packed [G][W]
 *   gset: local lub_many + ncclAllGather of the partial bitmaps + OR-fold of the world partials
 *   orswot: local join without deferred removes, ncclAllGather of the partial (clock, entries),
 *       all ranks' deferred removes gathered and pooled per group (rank order, then local order),
 *       re-merge of the world partials with every deferred remove (orswot.rs:141-147).  If any
 *       rank's shard holds an entry cell with E > C (flags gathered with the deferred counts), the
 *       partials are not joined as a tree: rank k re-folds its shard starting from rank k-1's state,
 *       one all-gather per step (W-1 extra exchanges), and the re-merge reads the last rank's state —
 *       the left fold over the concatenated shards for any input.  Output:
 *       clock [G][A], entries [G][M][A], and the surviving deferred removes compacted: *ndef (host)
 *       = their number; the first min(*ndef, def_cap) are written as def_clock[d*A + a],
 *       def_members[d*Mw + w] (union over the survivors with that exact clock in the group) and
 *       def_group[d] (device u32), in group order.
 * The replaced reference operation is the same CvRDT::merge fold (traits.rs:4-7), split over
 * processes: a Rust caller would distribute the id over its own transport.
 *
 * Agreement: every *_sharded call first exchanges a small header (this rank's validation status
 * and the call's rank-uniform dims: G, row width, M / K, A, D ...) and only runs its data
 * collectives when every rank validated and the dims agree; otherwise EVERY rank returns an error
 * (CRDT_EINVAL: its own validation failed, or the ranks disagree; CRDT_ECOMM with "another rank"
 * in crdt_last_error: a peer's failed), so a bad argument on one rank never leaves the others
 * blocked in a collective.  The header exchange runs on a side stream while the local fold runs.
 *
 * The caller's own collectives instead of RCCL (crdt_ctx_comm_init_ops): every *_sharded call then
 * runs its exchange through these HOST callbacks on host buffers (the library copies device data
 * to host memory and back around each call, after draining its stream).  A transport seam for
 * callers with their own channel (MPI, TCP, a test harness) and for running the multi-rank code of
 * this file with several ranks on one GPU.  Callbacks return 0 on success; any other value makes
 * the sharded call return CRDT_ECOMM.
 *   allgather:     recv[r*bytes .. (r+1)*bytes) = rank r's `send` bytes, for every rank r
 *   allreduce_u64: buf[i] = op over the ranks of buf[i] (unsigned 64-bit; CRDT_RED_*) */
#define CRDT_UNIQUE_ID_BYTES 128
#define CRDT_RED_MAX 0
#define CRDT_RED_MIN 1
#define CRDT_RED_SUM 2
typedef struct crdt_comm_ops {
  void *user;
  int (*allgather)(void *user, const void *send, void *recv, size_t bytes);
  int (*allreduce_u64)(void *user, uint64_t *buf, size_t n, int op);
} crdt_comm_ops;
int crdt_comm_unique_id(uint8_t *id /* [CRDT_UNIQUE_ID_BYTES] */);
/* Collective.  RCCL is bound at run time (dlopen + dlsym, csrc/shard.hip), from ONE librccl.so.1:
 * $CRDT_RCCL_LIB when set, else the copy the process already has loaded (torch's own RCCL inside
 * a torch process, so the library and torch.distributed share one RCCL), else librccl.so.1 through
 * the library's RUNPATH (/opt/rocm/lib).  CRDT_ECOMM if none loads or it is older than 2.18. */
int crdt_ctx_comm_init(crdt_ctx *ctx, const uint8_t *id, int nranks, int rank);
/* Not collective (the callbacks are the caller's); ops is copied, its user pointer must stay
 * valid until crdt_ctx_comm_destroy. */
int crdt_ctx_comm_init_ops(crdt_ctx *ctx, const crdt_comm_ops *ops, int nranks, int rank);
int crdt_ctx_comm_destroy(crdt_ctx *ctx);
int crdt_ctx_comm_info(const crdt_ctx *ctx, int *nranks, int *rank);
/* The RCCL the ctx's communicator runs on, noted at comm init ("" before it / for caller ops), e.g.
 * "RCCL 2.26.6 (22606) at /.../librccl.so.1, already loaded by the process ..."; storage owned by
 * ctx.  *runtime = the bound RCCL's version code (0 if none binds), *header = the rccl.h version
 * the types were taken from (may be NULL). */
const char *crdt_ctx_comm_note(const crdt_ctx *ctx, int *runtime, int *header);
int crdt_vclock_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                                 size_t row_stride, size_t group_stride, uint64_t *out);
int crdt_gcounter_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                                   size_t row_stride, size_t group_stride, uint64_t *out);
int crdt_pncounter_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                                    size_t row_stride, size_t group_stride, uint64_t *out);
int crdt_gset_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t words,
                               size_t row_stride, size_t group_stride, uint64_t *out);

typedef struct crdt_orswot_sharded_out {
  uint64_t *clock;       /* [G][A]      */
  uint64_t *entries;     /* [G][M][A]   */
  size_t def_cap;        /* rows available below */
  uint64_t *def_clock;   /* [def_cap][A]  */
  uint64_t *def_members; /* [def_cap][Mw] */
  uint32_t *def_group;   /* [def_cap]     */
  size_t *ndef;          /* host: number of surviving deferred removes */
} crdt_orswot_sharded_out;

int crdt_orswot_lub_many_sharded(crdt_ctx *ctx, const crdt_orswot_batch *in, crdt_orswot_sharded_out *out);
/* crdt_orswot_lub_many_sharded with this rank's deferred-pool offsets in DEVICE memory (round 4):
 * in->def_off NULL, def_off device u64 [G+1] (or NULL when D == 0) with def_off[G] == D, D the
 * rank's pool length.  The per-group counts are taken on the device and travel in the exchange's
 * count row, so no host sync is added: the offsets are checked there too (def_off[0] == 0,
 * def_off[G] == D, non-decreasing), and an invalid entry on ANY rank makes every rank return
 * before a deferred row moves (CRDT_EINVAL on that rank, CRDT_ECOMM on the others). */
int crdt_orswot_lub_many_sharded_doff(crdt_ctx *ctx, const crdt_orswot_batch *in, const uint64_t *def_off, size_t D,
                                      crdt_orswot_sharded_out *out);
/* crdt_lub_many_multi over replica shards: one fused local launch, then ONE grouped RCCL call
 * (an in-place ncclMax all-reduce per max segment; GSet segments as crdt_gset_lub_many_sharded).
 * Outputs must be contiguous (out_stride == row words, or G == 1). */
int crdt_lub_many_multi_sharded(crdt_ctx *ctx, const crdt_lub_segment *segs, size_t nseg);

/* LWWReg (lwwreg.rs:43-45 -> update :84-98), replicas split in rank order: rank k holds replicas
 * [base_k, base_k + R_k) of every group (marker / val at [g*group_stride + r], R_k may be 0) and
 * passes its base_k.  Every rank receives the state of the GLOBAL left fold (out_marker[g],
 * out_val[g]) and first_conflict[g] = the global index of its first erroring merge (UINT64_MAX if
 * none; may be NULL): each rank continues the fold from the fold of the lower ranks' states, then a
 * MIN all-reduce.  Exchange: ncclAllGather of (G markers, G vals, R_k) + ncclAllReduce(ncclMin). */
int crdt_lwwreg_lub_many_sharded(crdt_ctx *ctx, const uint64_t *marker, const uint64_t *val, size_t G, size_t R,
                                 size_t group_stride, uint64_t base, uint64_t *out_marker, uint64_t *out_val,
                                 uint64_t *first_conflict);

/* ---- Map<K, MVReg<u64, A>, A> --------------------------------------------------------------
 * Replaces Map::merge (map.rs:140-220) with V = MVReg (MVReg::merge mvreg.rs:112-128,
 * MVReg::forget :88-104), incl. apply_keyset_rm (map.rs:318-348) and apply_deferred (:311-316),
 * folded as acc = Map::new(); for r in 0..R: acc.merge(replica[g][r]).  Exact for any input
 * (no associativity is assumed: each key is folded in replica order).
 * Dense layout per replica (g, r) — keys, actors and MVReg values interned by the caller:
 *   clock C[a]            at clock + g*clock_gstride + r*clock_rstride + a
 *   entry clocks EC[k][a] at ec    + g*ec_gstride    + r*ec_rstride    + k*A + a
 *                          (key absent <=> row all 0)
 *   value clocks VC[k][s][a] at vclk + g*vclk_gstride + r*vclk_rstride + (k*V + s)*A + a and
 *   values VV[k][s]         at vval + g*vval_gstride + r*vval_rstride + k*V + s, for the
 *                          s < V value slots of the key's MVReg in Vec order (slot empty <=>
 *                          clock row all 0; empty slots are skipped)
 *   deferred removes pooled per group (CSR): group g owns d in [def_off[g], def_off[g+1])
 *     (def_off a HOST array of G+1 entries; crdt_map_lub_many_doff: device), held by replica
 *     def_row[d] of the group (device u32, non-decreasing within the group, < R), rm clock
 *     def_clock[d*A + a], key bitmap
 *     def_keys[d*Kw + w], Kw = ceil(K/64).
 * Output per group g (packed): clock[g*A + a], ec[(g*K + k)*A + a], value slots s < Vout:
 * vclk[((g*K + k)*Vout + s)*A + a], vval[(g*K + k)*Vout + s]; nval[g*K + k] = number of values
 * (may be NULL); flags[g] (required): bit 0 = some key folded to more than Vout values (its
 * slots are then incomplete: retry with a larger Vout), bit 1 = def_row not non-decreasing or
 * >= R, bit 2 = the fold state of some key needed more values than it holds (results of the
 * group incomplete: retry with Vstate = 8), bit 3 = internal: a key wave waited past its bound
 * for the workgroup's shared clock-row ring (results of the group unreliable; never expected —
 * report it).  The state holds VO = 2*pow2(V') values, V' the
 * smallest power of two with V' >= V and 2V' >= min(8, max(Vout, Vstate)); VO <= 8.
 * Deferred output as for Orswot (def_keep / def_keys over keys).
 * Limits: A <= 1024, V <= 16, Vout <= 64; the fold state holds up to 16 values per key (bit 2 of
 * flags when a key needs more).  A > 256 or V > 8 runs the workgroup-per-key fold (csrc/map_wide.hip:
 * the same exact left fold, no speculative scan — a correctness path, not a tuned one). */
typedef struct crdt_map_batch {
  size_t G, R, K, A, V;
  const uint64_t *clock;
  size_t clock_rstride, clock_gstride;
  const uint64_t *ec;
  size_t ec_rstride, ec_gstride;
  const uint64_t *vclk;
  size_t vclk_rstride, vclk_gstride;
  const uint64_t *vval;
  size_t vval_rstride, vval_gstride;
  const size_t *def_off; /* host, G+1 entries; NULL or all-zero = no deferred removes */
  const uint32_t *def_row;
  const uint64_t *def_clock;
  const uint64_t *def_keys;
} crdt_map_batch;

typedef struct crdt_map_out {
  size_t Vout;
  size_t Vstate; /* value capacity hint for the fold state (0 = from Vout and V) */
  uint64_t *clock; /* [G][A]          */
  uint64_t *ec;    /* [G][K][A]       */
  uint64_t *vclk;  /* [G][K][Vout][A] */
  uint64_t *vval;  /* [G][K][Vout]    */
  uint32_t *nval;  /* [G][K] or NULL  */
  uint32_t *flags; /* [G]             */
  uint8_t *def_keep; /* [D]     */
  uint64_t *def_keys; /* [D][Kw] */
} crdt_map_out;

int crdt_map_lub_many(crdt_ctx *ctx, const crdt_map_batch *in, crdt_map_out *out);
/* crdt_map_lub_many with the deferred pool's CSR offsets in DEVICE memory, as for
 * crdt_orswot_lub_many_doff: in->def_off NULL, def_off device u64 [G+1] (or NULL) with
 * def_off[G] == D.  An invalid entry i (checked on the device, as there) sets bit 1 of flags[i-1]
 * and flags[i] (the groups whose range it bounds); the fold then reads the offsets clamped to
 * [0, D].  Device-memory contexts only. */
int crdt_map_lub_many_doff(crdt_ctx *ctx, const crdt_map_batch *in, const uint64_t *def_off, size_t D,
                           crdt_map_out *out);

/* Map<K, MVReg> sharded by KEYS: rank k holds keys [k0, k0 + in->K) of every
 * replica (the crdt_map_batch layout with K = its key count), every replica's clock and the group's
 * whole deferred list with key bitmaps over all K keys (def_keys [D][ceil(K/64)]).  Keys are
 * independent given the clocks and the deferred list, so each rank's fold of its keys is the exact
 * left fold (no data-path collective); out holds the rank's keys, except out->def_keys
 * [D][ceil(K/64)]: the surviving removes' key sets over ALL keys, assembled by one
 * ncclAllReduce(ncclSum) (disjoint ranges: sum = union).  def_keep is the same on every rank. */
int crdt_map_lub_many_sharded(crdt_ctx *ctx, const crdt_map_batch *in, size_t k0, size_t K, crdt_map_out *out);
/* crdt_map_lub_many_sharded with the deferred pool's offsets in DEVICE memory (round 4), as for
 * crdt_map_lub_many_doff: in->def_off NULL, def_off device u64 [G+1] (or NULL when D == 0),
 * def_off[G] == D.  Checked on the device (an invalid entry sets bit 1 of the flags of the groups
 * it bounds, ORed over the ranks); instead of the host offsets' hash in the agreed header, a
 * device hash of the offsets travels in the flags exchange and ranks holding different offsets
 * all return CRDT_EINVAL before the key sets are exchanged. */
int crdt_map_lub_many_sharded_doff(crdt_ctx *ctx, const crdt_map_batch *in, const uint64_t *def_off, size_t D,
                                   size_t k0, size_t K, crdt_map_out *out);

/* ---- Map<K, GCounter<A>, A> and Map<K, PNCounter<A>, A> (round 4) ----------------------------
 * Map::merge (map.rs:140-220) with a counter value: GCounter (gcounter.rs:44-54: merge = the VClock
 * max, Causal::forget = VClock::forget) or PNCounter (pncounter.rs:70-82: P and N each), folded as
 * acc = Map::new(); for r: acc.merge(replica[g][r]) — exact for any input (each key folded in
 * replica order: the fold is not associative for these values either).  Layout as crdt_map_batch,
 * with the value of key k a block of W counter rows (W = 1 GCounter, W = 2 PNCounter: P then N):
 *   val + g*val_gstride + r*val_rstride + (k*W + w)*A + a   (an absent key: its rows all 0)
 * deferred removes pooled per group as for Map<K, MVReg>: def_off a HOST array of G+1 entries,
 * def_row device u32 non-decreasing within the group and < R, def_clock [D][A], def_keys [D][Kw].
 * Output per group g (packed): clock[g*A + a], ec[(g*K + k)*A + a], val[((g*K + k)*W + w)*A + a],
 * flags[g] (required): bit 1 = def_row not non-decreasing or >= R, bit 3 = more than 512 live
 * removes named one key (results of the group unreliable); def_keep / def_keys as crdt_map_out.
 * Limits: A <= 512.  Device and host memory (crdt_mem_kind; round 5). */
typedef struct crdt_map_counter_batch {
  size_t G, R, K, A, W;
  const uint64_t *clock;
  size_t clock_rstride, clock_gstride;
  const uint64_t *ec;
  size_t ec_rstride, ec_gstride;
  const uint64_t *val;
  size_t val_rstride, val_gstride;
  const size_t *def_off; /* host, G+1 entries; NULL = no deferred removes */
  const uint32_t *def_row;
  const uint64_t *def_clock;
  const uint64_t *def_keys;
} crdt_map_counter_batch;

typedef struct crdt_map_counter_out {
  uint64_t *clock;    /* [G][A]       */
  uint64_t *ec;       /* [G][K][A]    */
  uint64_t *val;      /* [G][K][W][A] */
  uint32_t *flags;    /* [G]          */
  uint8_t *def_keep;  /* [D]          */
  uint64_t *def_keys; /* [D][Kw]      */
} crdt_map_counter_out;

int crdt_map_counter_lub_many(crdt_ctx *ctx, const crdt_map_counter_batch *in, crdt_map_counter_out *out);
/* Map<K, GCounter / PNCounter> sharded by KEYS (round 5), as crdt_map_lub_many_sharded: rank k holds keys
 * [k0, k0 + in->K) of every replica (the layout above with K = its key count), every replica's
 * clock and the group's whole deferred list with key bitmaps over all K keys (def_keys
 * [D][ceil(K/64)]); its fold of its keys is the exact left fold (no data-path collective).  out holds
 * the rank's keys, flags ORed over the ranks, and out->def_keys [D][ceil(K/64)] the surviving removes'
 * key sets over ALL keys (one ncclAllReduce(ncclSum): disjoint ranges).  Device memory only. */
int crdt_map_counter_lub_many_sharded(crdt_ctx *ctx, const crdt_map_counter_batch *in, size_t k0, size_t K,
                                      crdt_map_counter_out *out);

/* ---- Map<K, Orswot<M, A>, A> (round 4) ----------------------------------------------------------
 * Map::merge (map.rs:140-220) with a nested Orswot value (orswot.rs:81-149 merge, :150-183 forget)
 * — the value type of the reference's merge_error KAT (map.rs:435-494) — folded as
 * acc = Map::new(); for r: acc.merge(replica[g][r]), exact for any input (each key in replica
 * order).  Contiguous layouts (no strides):
 *   clock [G][R][A], ec [G][R][K][A] the entry clocks, oc [G][R][K][A] the nested Orswot clocks,
 *   ent [G][R][K][M][A] its member dots (a member absent: its row 0; a key absent: ec row 0),
 *   the nested deferred removes as a device CSR over (g, r, k): vd_off u64 [G*R*K + 1],
 *   vd_clock [Dv][A], vd_mem [Dv][Mw] member bitmasks, Mw = ceil(M / 64) words (1 for M <= 64: [Dv])
 *   (an equal clock twice in one list: unioned);
 *   the Map's own deferred removes as for the counter Map: def_off HOST, G+1 entries.
 * Output per group g (packed): clock[g*A + a], ec / oc [(g*K + k)*A + a], ent [((g*K + k)*M + m)*A
 * + a], nested deferred vd_n[g*K + k] (<= Vd) with vd_clock [((g*K + k)*Vd + i)*A + a] and
 * vd_mem [((g*K + k)*Vd + i)*Mw + w] (Vd = out->Vd, 0 meaning 16; round 6: the fold keeps 16 slots per
 * key in LDS and re-folds, exactly, the keys whose list passed 16 with all Vd — a second launch of one
 * wave per marked key, its Vd member masks in LDS: Vd * Mw * 8 + 6 KiB <= 160 KiB); flags[g]: bit 1 =
 * def_row not non-decreasing or >= R, bit 3 = more live Map removes named one key than the deep pass
 * holds (256 in the first pass; the deep pass takes the largest group's whole list, ~80,000 in its
 * LDS), bit 4 = a key's Orswot held more than Vd deferred removes, bit 5 = vd_off invalid (checked on the device: vd_off[0] == 0, non-decreasing,
 * vd_off[G*R*K] == Dv; the fold reads only rows [0, Dv) whatever it holds) — results of the
 * group unreliable; def_keep / def_keys as crdt_map_out.
 * Orswot::forget collects its deferred removes into a new map: two whose clocks become equal keep
 * one entry with the later one's members (the oracle's dict order).
 * Limits: A <= 1,024, M <= 1,024 (round 5: past A = 64 or M = 32 a wide kernel, lane = 64 actors
 * apart, the key's member rows in its own output rows; CRDT_TUNE mowide=1 runs it at every shape).
 * Device and host memory (crdt_mem_kind). */
typedef struct crdt_map_orswot_batch {
  size_t G, R, K, M, A;
  const uint64_t *clock, *ec, *oc, *ent;
  const uint64_t *vd_off;   /* device, G*R*K + 1 */
  const uint64_t *vd_clock; /* [Dv][A] */
  const uint64_t *vd_mem;   /* [Dv][Mw] */
  const size_t *def_off;    /* host, G+1 entries; NULL = no Map-level deferred removes */
  const uint32_t *def_row;
  const uint64_t *def_clock;
  const uint64_t *def_keys;
  size_t Dv;                /* rows of vd_clock / vd_mem (= vd_off[G*R*K]) */
} crdt_map_orswot_batch;

typedef struct crdt_map_orswot_out {
  uint64_t *clock;    /* [G][A]          */
  uint64_t *ec;       /* [G][K][A]       */
  uint64_t *oc;       /* [G][K][A]       */
  uint64_t *ent;      /* [G][K][M][A]    */
  uint32_t *vd_n;     /* [G][K]          */
  uint64_t *vd_clock; /* [G][K][Vd][A]   */
  uint64_t *vd_mem;   /* [G][K][Vd][Mw]  */
  uint32_t *flags;    /* [G]             */
  uint8_t *def_keep;  /* [D]             */
  uint64_t *def_keys; /* [D][Kw]         */
  size_t Vd;          /* nested deferred slots per key (round 6, ABI 8; 0 = 16) */
} crdt_map_orswot_out;

int crdt_map_orswot_lub_many(crdt_ctx *ctx, const crdt_map_orswot_batch *in, crdt_map_orswot_out *out);
/* Map<K, Orswot> sharded by KEYS (round 5), as crdt_map_lub_many_sharded: rank k holds keys
 * [k0, k0 + in->K) of every replica (the layout above with K = its key count; the nested removes' CSR over the rank's (g, r, k)), every replica's
 * clock and the group's whole deferred list with key bitmaps over all K keys (def_keys
 * [D][ceil(K/64)]); its fold of its keys is the exact left fold (no data-path collective).  out holds
 * the rank's keys, flags ORed over the ranks, and out->def_keys [D][ceil(K/64)] the surviving removes'
 * key sets over ALL keys (one ncclAllReduce(ncclSum): disjoint ranges).  Device memory only. */
int crdt_map_orswot_lub_many_sharded(crdt_ctx *ctx, const crdt_map_orswot_batch *in, size_t k0, size_t K,
                                     crdt_map_orswot_out *out);

/* ---- Map<K, Map<K2, MVReg<u64, A>, A>, A> (round 5) -----------------------------------------------
 * The nested type of the reference's own Map tests (TMap, test/map.rs:10; TestMap, map.rs:359):
 * Map::merge (map.rs:140-220) whose value is a Map<K2, MVReg> — merged by Map::merge again with
 * MVReg::merge (mvreg.rs:112-128) innermost, and forgotten by Map's Causal::forget (map.rs:85-114) —
 * folded as acc = Map::new(); for r: acc.merge(replica[g][r]), exact for any input (each outer key in
 * replica order).  Contiguous layouts (no strides), per replica r of group g:
 *   clock [G][R][A]; ec [G][R][K][A] outer entry clocks (key absent: row 0); ic [G][R][K][A] the
 *   inner Map clocks; iec [G][R][K][K2][A] inner entry clocks; ivc [G][R][K][K2][V][A] / ivv
 *   [G][R][K][K2][V] the inner MVReg slots in Vec order (an empty slot: clock row 0); the inner
 *   deferred removes as a device CSR over (g, r, k): id_off u64 [G*R*K + 1], id_clock [Di][A],
 *   id_keys [Di][K2w] inner-key bitmasks (K2w = 1 up to K2 = 64, else ceil(K2/64) words, round 6);
 *   the outer deferred removes as for the MVReg Map: def_off HOST
 *   (G+1), def_row, def_clock [D][A], def_keys [D][Kw].
 * Output per (g, k) (packed): clock [g*A + a], ec / ic [(g*K + k)*A + a], iec [((g*K + k)*K2 + j)*A +
 *   a], Vs slots per inner key (out->Vs, 0 meaning 8, at most 64) ivc [(((g*K + k)*K2 + j)*Vs + s)*A +
 *   a], ivv [((g*K + k)*K2 + j)*Vs + s] with nval [(g*K + k)*K2 + j] used (unused slots 0; round 6: a
 *   key past 8 values re-folds in the deep pass, which also takes inputs with V up to 64), inner deferred id_n [g*K + k] (<= Id = out->Id,
 *   0 meaning 16), id_clock [((g*K + k)*Id + i)*A + a], id_keys [((g*K + k)*Id + i)*K2w + w] (round 6:
 *   the fold keeps 16 in LDS and re-folds, exactly, the keys whose inner list passed 16 with all Id —
 *   a second launch of one wave per marked key); flags[g]: bit 1 = def_row not non-decreasing or >= R,
 *   bit 3 = more live outer removes named one key than the deep pass holds (256 in the first pass,
 *   the largest group's whole list in the deep pass), bit 4 = an inner Map held more than Id deferred
 *   removes, bit 5 = id_off invalid (checked on the device: starts at
 *   0, non-decreasing, ends at Di; the fold never reads past Di), bit 6 = an inner key held more than
 *   Vs values — results of the group unreliable; def_keep / def_keys as crdt_map_out.
 * Map::forget collects the inner deferred removes into a new map: two whose clocks become equal keep
 * one entry with the later one's keys (the oracle's dict order; the reference's is unspecified).
 * Limits: A <= 256 and K2 <= 256 (round 6: lane l holds actors l + 64 j; K2w key-set words), V <= 8.
 * Device and host memory
 * (crdt_mem_kind). */
typedef struct crdt_map_nested_batch {
  size_t G, R, K, K2, V, A;
  const uint64_t *clock, *ec, *ic, *iec, *ivc, *ivv;
  const uint64_t *id_off;   /* device, G*R*K + 1 */
  const uint64_t *id_clock; /* [Di][A] */
  const uint64_t *id_keys;  /* [Di][K2w] */
  size_t Di;
  const size_t *def_off;    /* host, G+1 entries; NULL = no outer deferred removes */
  const uint32_t *def_row;
  const uint64_t *def_clock;
  const uint64_t *def_keys;
} crdt_map_nested_batch;

typedef struct crdt_map_nested_out {
  uint64_t *clock;    /* [G][A]            */
  uint64_t *ec;       /* [G][K][A]         */
  uint64_t *ic;       /* [G][K][A]         */
  uint64_t *iec;      /* [G][K][K2][A]     */
  uint64_t *ivc;      /* [G][K][K2][Vs][A] */
  uint64_t *ivv;      /* [G][K][K2][Vs]    */
  uint32_t *nval;     /* [G][K][K2]        */
  uint32_t *id_n;     /* [G][K]            */
  uint64_t *id_clock; /* [G][K][Id][A]     */
  uint64_t *id_keys;  /* [G][K][Id][K2w]   */
  uint32_t *flags;    /* [G]               */
  uint8_t *def_keep;  /* [D]               */
  uint64_t *def_keys; /* [D][Kw]           */
  size_t Id;          /* inner deferred slots per key (round 6, ABI 8; 0 = 16) */
  size_t Vs;          /* MVReg slots per inner key (round 6, ABI 8; 0 = 8, at most 64) */
} crdt_map_nested_out;

int crdt_map_nested_lub_many(crdt_ctx *ctx, const crdt_map_nested_batch *in, crdt_map_nested_out *out);
/* Map<K, Map<K2, MVReg>> sharded by KEYS (round 5), as crdt_map_lub_many_sharded: rank k holds keys
 * [k0, k0 + in->K) of every replica (the layout above with K = its key count; the inner removes' CSR over the rank's (g, r, k)), every replica's
 * clock and the group's whole deferred list with key bitmaps over all K keys (def_keys
 * [D][ceil(K/64)]); its fold of its keys is the exact left fold (no data-path collective).  out holds
 * the rank's keys, flags ORed over the ranks, and out->def_keys [D][ceil(K/64)] the surviving removes'
 * key sets over ALL keys (one ncclAllReduce(ncclSum): disjoint ranges).  Device memory only. */
int crdt_map_nested_lub_many_sharded(crdt_ctx *ctx, const crdt_map_nested_batch *in, size_t k0, size_t K,
                                     crdt_map_nested_out *out);

/* Map<K, Map<K2, MVReg<u64>>> states in place (round 5), on the crdt_map_nested_lub_many output layout
 * with N states (packed; Vs MVReg slots per inner key in Vec order (states->Vs, 0 = 8), nval used, the rest zero; Id inner
 * deferred slots per key (states->Id, 0 = 16) with a K2w-word inner-key mask each, K2w = 1 up to K2 = 64):
 *   crdt_map_nested_apply_batch — CmRDT::apply (map.rs:119-137, apply_keyset_rm :318-348,
 *     apply_deferred :311-316) with the inner Map's apply one level down and MVReg::apply
 *     (mvreg.rs:130-166) innermost: state s applies ops [op_off[s], op_off[s+1]) in order; the outer
 *     deferred removes as crdt_map_counter_apply_batch (def_count[s] <= Dcap slots); an inner list past
 *     Id sets bit 0.  Ops: kind 0 =
 *     Op::Up { dot: (actor, counter), key, op } with ikind 0 = inner Op::Up { dot: (iactor, icounter),
 *     key: ikey, op: Put { clock: clk_pool[clk_row*A ..], val } } or 1 = inner Op::Rm { clock:
 *     clk_pool[clk_row*A ..], keyset: the inner-key mask ikeys [n_ops][K2w] }; kind 1 = Op::Rm { clock:
 *     clk_pool[clk_row*A ..], keyset: keys[key_off[o] .. key_off[o+1]) } (key_off may be NULL when no
 *     op is an outer Rm).  status[s]: bit 0 = a deferred list (outer Dcap or an inner one's Id)
 *     exhausted, bit 1 = a malformed op skipped whole, bits 2-3 = invalid input (state untouched),
 *     bit 4 = a register needed more than Vs values (that value was not added).
 *   crdt_map_nested_forget_batch — Causal::forget (map.rs:85-114) of the whole state by y[s] (y_stride
 *     0: one row for all): entry clocks, the inner Maps (their entries, registers — MVReg::forget
 *     mvreg.rs:88-104, emptied values dropped, order kept —, deferred removes, clocks), an emptied
 *     entry dropped; the outer deferred pool and the map clock as crdt_map_forget_batch.  Inner removes
 *     whose clocks become equal keep one entry with the later one's keys (the fold's rule).
 * Limits: A <= 512, K2 <= 256 (round 6; a key bit past K2 makes the op malformed); the outer Dcap is not bounded (its first min(Dcap, 16) slots in LDS during
 * an apply stream, the rest used in place, round 6).  Device memory only. */
typedef struct crdt_map_nested_states {
  size_t N, K, K2, A;
  uint64_t *clock;    /* [N][A]           */
  uint64_t *ec;       /* [N][K][A]        */
  uint64_t *ic;       /* [N][K][A]        */
  uint64_t *iec;      /* [N][K][K2][A]    */
  uint64_t *ivc;      /* [N][K][K2][Vs][A] */
  uint64_t *ivv;      /* [N][K][K2][Vs]   */
  uint32_t *nval;     /* [N][K][K2]       */
  uint32_t *id_n;     /* [N][K]           */
  uint64_t *id_clock; /* [N][K][Id][A]    */
  uint64_t *id_keys;  /* [N][K][Id][K2w]  */
  size_t Id;          /* inner deferred slots per key (round 6, ABI 8; 0 = 16) */
  size_t Vs;          /* MVReg slots per inner key (round 6, ABI 8; 0 = 8, at most 64) */
} crdt_map_nested_states;

typedef struct crdt_map_nested_ops {
  size_t n_ops;
  const uint64_t *op_off;    /* [N+1]       */
  const uint8_t *kind;       /* [n_ops] 0 = Op::Up, 1 = Op::Rm */
  const uint32_t *actor;     /* [n_ops] Up: the outer dot */
  const uint64_t *counter;   /* [n_ops] Up  */
  const uint32_t *key;       /* [n_ops] Up  */
  const uint8_t *ikind;      /* [n_ops] Up: 0 inner Up (Put), 1 inner Rm */
  const uint32_t *iactor;    /* [n_ops] inner Up: its dot */
  const uint64_t *icounter;  /* [n_ops] inner Up */
  const uint32_t *ikey;      /* [n_ops] inner Up: the inner key */
  const uint64_t *val;       /* [n_ops] inner Up: the Put's value */
  const uint64_t *ikeys;     /* [n_ops][K2w] inner Rm: inner-key mask */
  const uint32_t *clk_row;   /* [n_ops] the Put clock / an rm clock: row of clk_pool */
  const uint64_t *clk_pool;  /* [n_clk_rows][A] */
  size_t n_clk_rows;
  const uint64_t *key_off;   /* [n_ops+1] outer Rm keysets */
  const uint32_t *keys;      /* [n_keys]    */
  size_t n_keys;
} crdt_map_nested_ops;

int crdt_map_nested_apply_batch(crdt_ctx *ctx, const crdt_map_nested_states *states, uint64_t *def_clock,
                                uint64_t *def_keys, uint32_t *def_count, size_t Dcap,
                                const crdt_map_nested_ops *ops, uint32_t *status);
int crdt_map_nested_forget_batch(crdt_ctx *ctx, const crdt_map_nested_states *states, const uint64_t *y,
                                 size_t y_stride, uint64_t *def_clock, const uint32_t *def_state, size_t D,
                                 uint8_t *def_keep);

/* Pairwise in-place merge of value-typed Map states (round 6): self[i].merge(other[i]) for i < N
 * (Map::merge map.rs:140-220 with the value's merge / forget: gcounter.rs:44-54 / pncounter.rs:70-82,
 * orswot.rs:81-183, or the inner Map's map.rs:85-220 with mvreg.rs:88-128), on the apply layouts
 * (crdt_map_counter_states / crdt_map_orswot_states / crdt_map_nested_states, N, K, A and W / M / K2
 * equal on both sides) with each side's Map-level deferred removes as crdt_map_deferred slots (the
 * counts may differ in Dcap).  Each pair is one group of the exact left fold above with R = 2
 * (Map::new() merged with self, then other): self.merge(other) on every state apply, merge, forget or
 * ingest leaves (deferred removes applied and not dominated by the clock).  self is rewritten: its
 * rows, its nested lists, and its slots with the surviving removes (their merged key sets) in pool
 * order, vacated slots zeroed; other is read only.  status[i]: bit 0 = more surviving removes than
 * self's Dcap (the first Dcap kept), bit 3 = the fold reported a capacity for the pair (more than
 * 256 / 512 live removes naming one key, more than self's Vd / Id nested deferred removes on a key,
 * more than 8 values on an inner key: that pair's state is incomplete).  A def_count above its Dcap or
 * a nested count above its side's Vd / Id fails the call (CRDT_EINVAL) before anything is written.  The call reads the slot
 * counts on the host (one stream synchronisation).  Device memory only. */
int crdt_map_counter_merge_batch(crdt_ctx *ctx, const crdt_map_counter_states *self, const crdt_map_deferred *self_def,
                                 const crdt_map_counter_states *other, const crdt_map_deferred *other_def,
                                 uint32_t *status);
int crdt_map_orswot_merge_batch(crdt_ctx *ctx, const crdt_map_orswot_states *self, const crdt_map_deferred *self_def,
                                const crdt_map_orswot_states *other, const crdt_map_deferred *other_def,
                                uint32_t *status);
int crdt_map_nested_merge_batch(crdt_ctx *ctx, const crdt_map_nested_states *self, const crdt_map_deferred *self_def,
                                const crdt_map_nested_states *other, const crdt_map_deferred *other_def,
                                uint32_t *status);

/* ---- MVReg<u64, A> on its own (outside a Map) ------------------------------------------------
 * Replaces MVReg::merge (mvreg.rs:112-128) and MVReg::apply (mvreg.rs:130-166) for registers in the
 * dense layout the Map entry points use for their values: slots in Vec order, slot s of register i
 * = (clock vclk[i*vclk_stride + s*A + a], value vval[i*vval_stride + s]); an empty slot is an
 * all-zero clock row (skipped; results are written from slot 0, empty slots zeroed).  Values are
 * u64 ids interned by the caller (merge and apply compare clocks only, never values).  Exact for
 * any input: each register is folded / applied in order.
 *   lub_many:    acc = MVReg::new(); for r in 0..R: acc.merge(replica[g][r]) per group g; replica
 *                (g, r) at vclk + g*vclk_gstride + r*vclk_rstride (vval likewise).  out: Vout slots
 *                per group (packed [G][Vout][A] / [G][Vout]), nval[g] (may be NULL), flags[g]: bit 0
 *                = more than Vout values (slots incomplete: retry with a larger Vout), bit 2 = the
 *                fold state overflowed (retry with Vstate = 16; past 16 values it is reported).
 *   merge_batch: self[i].merge(other[i]), in place in self's V slots (own kept values, then other's
 *                added ones); status[i] bit 4 = more than self's V values (register incomplete).
 *   apply_batch: register i applies ops [op_off[i], op_off[i+1]) in order, Op::Put { clock:
 *                clk_pool[clk_row[o]*A ..], val: val[o] }; status[i] bit 1 = an op's clk_row out
 *                of range (skipped), bit 3 = op_off invalid (register untouched), bit 4 = more than
 *                V values.
 * Limits: A <= 1024, 1 <= V <= 16 (lub_many: Vout <= 16); A > 256 or V > 8 run one workgroup of
 * ceil(A / 64) waves per register. */
typedef struct crdt_mvreg_states {
  size_t N, A, V;
  uint64_t *vclk;
  size_t vclk_stride;
  uint64_t *vval;
  size_t vval_stride;
} crdt_mvreg_states;

typedef struct crdt_mvreg_batch {
  size_t G, R, A, V;
  const uint64_t *vclk;
  size_t vclk_rstride, vclk_gstride;
  const uint64_t *vval;
  size_t vval_rstride, vval_gstride;
} crdt_mvreg_batch;

typedef struct crdt_mvreg_out {
  size_t Vout;
  size_t Vstate;   /* value capacity hint for the fold state (0 = from Vout and V) */
  uint64_t *vclk;  /* [G][Vout][A] */
  uint64_t *vval;  /* [G][Vout]    */
  uint32_t *nval;  /* [G] or NULL  */
  uint32_t *flags; /* [G]          */
} crdt_mvreg_out;

typedef struct crdt_mvreg_ops {
  size_t n_ops;
  const uint64_t *op_off;   /* [N+1]           */
  const uint32_t *clk_row;  /* [n_ops]         */
  const uint64_t *clk_pool; /* [n_clk_rows][A] */
  size_t n_clk_rows;
  const uint64_t *val;      /* [n_ops]         */
} crdt_mvreg_ops;

int crdt_mvreg_lub_many(crdt_ctx *ctx, const crdt_mvreg_batch *in, crdt_mvreg_out *out);
int crdt_mvreg_merge_batch(crdt_ctx *ctx, const crdt_mvreg_states *self, const crdt_mvreg_states *other,
                           uint32_t *status);
int crdt_mvreg_apply_batch(crdt_ctx *ctx, const crdt_mvreg_states *states, const crdt_mvreg_ops *ops,
                           uint32_t *status);

/* ---- causal helpers on dense clock rows -----------------------------------
 * Row-pair ops over N pairs (x_i, y_i) of A-word rows (VClock, GCounter inner, or a PNCounter
 * P‖N row with A = 2·actors):
 *   CRDT_PAIR_GLB     out_i = x_i.glb(y_i): pointwise min, a 0 drops the actor   vclock.rs:246-259
 *   CRDT_PAIR_FORGET  out_i = x_i.forget(y_i): keep x[a] iff x[a] > y[a]         vclock.rs:95-105
 *                     (GCounter::forget gcounter.rs:51-53, PNCounter::forget pncounter.rs:78-81
 *                     are the same op on their rows)
 *   CRDT_PAIR_INTERSECTION  out_i = VClock::intersection(x_i, y_i): keep x[a] iff
 *                     y[a] == x[a] (the common dots)                            vclock.rs:218-227
 * `out` may alias `x` (in place, like the reference's &mut self). */
#define CRDT_PAIR_GLB 1
#define CRDT_PAIR_FORGET 2
#define CRDT_PAIR_INTERSECTION 3
int crdt_vclock_pair_op(crdt_ctx *ctx, int op, uint64_t *out, const uint64_t *x, const uint64_t *y,
                        size_t N, size_t A, size_t out_stride, size_t x_stride, size_t y_stride);

/* VClock::partial_cmp (vclock.rs:68-80) of N row pairs: out[i] = 0 Equal, 1 Greater (x ≥ y),
 * -1 Less, 2 None (concurrent). */
int crdt_vclock_partial_cmp(crdt_ctx *ctx, const uint64_t *x, const uint64_t *y, size_t N, size_t A,
                            size_t x_stride, size_t y_stride, int8_t *out);

/* All-pairs partial_cmp of N clocks (the dominance / concurrency matrix): out[i*N + j] =
 * partial_cmp(x_i, x_j) coded as above.  N <= 4,194,240. */
int crdt_vclock_cmp_matrix(crdt_ctx *ctx, const uint64_t *x, size_t N, size_t A, size_t x_stride,
                           int8_t *out);

/* read() of N counters, exact: out[2i] + 2^64·out[2i+1] is
 *   GCounter::read  (gcounter.rs:70-72, BigUint sum of the A counters of row i), or
 *   PNCounter::read (pncounter.rs:110-115, BigInt P − N of row i = P[0..A) ‖ N[A..2A)) as a
 *                   two's-complement 128-bit integer.
 * Exact for A < 2^62 (the reference's num-bigint is unbounded; no sum of u64 counters of one
 * row reaches 2^126). */
int crdt_gcounter_read(crdt_ctx *ctx, const uint64_t *in, size_t N, size_t A, size_t row_stride,
                       uint64_t *out);
int crdt_pncounter_read(crdt_ctx *ctx, const uint64_t *in, size_t N, size_t A, size_t row_stride,
                        uint64_t *out);

/* ---- batched CmRDT::apply ---------------------------------------------------
 * Apply n_ops ops to N dense states; op i targets state state_idx[i] (row at
 * states + state_idx[i]*row_stride).  The ops of these types are per-cell joins, so they commute:
 * the batch equals applying them one by one in any order, as the reference's apply does.
 *   VClock::apply / apply_dot (vclock.rs:125-127, :155-159), GCounter::apply (gcounter.rs:39-41):
 *       row[actor[i]] = max(row[actor[i]], counter[i])                       (A-word rows)
 *   PNCounter::apply (pncounter.rs:62-67): dir[i] == 0 (Dir::Pos) -> P column actor[i],
 *       1 (Dir::Neg) -> N column A + actor[i]                                 (2A-word rows P ‖ N)
 *   GSet::apply / insert (gset.rs:46-48, :69-71): set bit element[i] of a ceil(U/64)-word bitmap
 * state_idx / actor / element are device u32, counter device u64, dir device u8.  Ops with
 * state_idx >= N or actor >= A (element >= U) are skipped and counted into *bad (device u32,
 * added to; may be NULL). */
int crdt_vclock_apply_batch(crdt_ctx *ctx, uint64_t *states, size_t N, size_t A, size_t row_stride,
                            const uint32_t *state_idx, const uint32_t *actor, const uint64_t *counter,
                            size_t n_ops, uint32_t *bad);
int crdt_gcounter_apply_batch(crdt_ctx *ctx, uint64_t *states, size_t N, size_t A, size_t row_stride,
                              const uint32_t *state_idx, const uint32_t *actor, const uint64_t *counter,
                              size_t n_ops, uint32_t *bad);
int crdt_pncounter_apply_batch(crdt_ctx *ctx, uint64_t *states, size_t N, size_t A, size_t row_stride,
                               const uint32_t *state_idx, const uint32_t *actor, const uint64_t *counter,
                               const uint8_t *dir, size_t n_ops, uint32_t *bad);
int crdt_gset_apply_batch(crdt_ctx *ctx, uint64_t *states, size_t N, size_t U, size_t row_stride,
                          const uint32_t *state_idx, const uint32_t *element, size_t n_ops, uint32_t *bad);

/* ---- serde wire format ingest / egress -------------------------------------
 * Replicas ship whole states serialized through the serde derives of the reference types
 * (vclock.rs:56, gcounter.rs:25, pncounter.rs:28, gset.rs:7, lwwreg.rs:13, orswot.rs:20).  These
 * entry points read / write the bytes `bincode::serialize` (bincode 1.x default options) produces:
 * little-endian fixed-width integers, a struct = its fields in order, a map / set / Vec = u64 length
 * then its entries (key, value).  Instantiations: actors u32, members / set elements u64:
 *   VClock<u32> = GCounter<u32>: u64 n, n x (u32 actor, u64 counter)        (actors ascending)
 *   PNCounter<u32>: GCounter p then GCounter n
 *   GSet<u64>: u64 n, n x u64 (ascending);  LWWReg<u64, u64>: u64 val, u64 marker
 *   Orswot<u64, u32>: VClock clock; u64 n, n x (u64 member, VClock); u64 d, d x (VClock rm,
 *       u64 k, k x u64 member)                     (HashMap / HashSet: any order on input)
 * Frames (device): state s is bytes[frame_off[s] .. frame_off[s+1]), offsets 4-byte aligned.
 * Dictionaries (device, ascending, unique): the dense column / bit / row of an id is its position.
 * status[s] (device u32): bit 0 = malformed frame (truncated, trailing bytes, misaligned), bit 1 = an
 * id missing from its dictionary (skipped), bit 2 = more deferred removes than def_cap.
 * Egress writes the same format (maps in ascending dictionary order) and the frame offsets
 * (device, N+1); it always returns the byte total in *total (host, synchronises) and writes the
 * bytes only when `bytes` is non-NULL and cap >= *total (call once with NULL to size a buffer).
 * Limits: A <= 4096 (VClock family), ceil(U/64) <= 4096, A + ceil(M/64) <= 4096 (Orswot). */
int crdt_vclock_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, size_t N,
                       const uint32_t *actors, size_t A, uint64_t *out, size_t row_stride, uint32_t *status);
int crdt_pncounter_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, size_t N,
                          const uint32_t *actors, size_t A, uint64_t *out, size_t row_stride, uint32_t *status);
int crdt_gset_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, size_t N,
                     const uint64_t *elems, size_t U, uint64_t *out, size_t row_stride, uint32_t *status);
int crdt_lwwreg_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, size_t N,
                       uint64_t *marker, uint64_t *val, uint32_t *status);
/* Orswot: clock [N][A], entries [N][M][A] (zero-filled, then the present members' rows), the
 * deferred removes pooled in state order: def_off [N+1] (device, written), rows d < def_cap of
 * def_clock [D][A] / def_members [D][ceil(M/64)], *n_def = D (host). */
int crdt_orswot_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, size_t N,
                       const uint32_t *actors, size_t A, const uint64_t *members, size_t M, uint64_t *clock,
                       uint64_t *entries, uint64_t *def_off, uint64_t *def_clock, uint64_t *def_members,
                       size_t def_cap, size_t *n_def, uint32_t *status);
int crdt_vclock_egress(crdt_ctx *ctx, const uint64_t *rows, size_t N, size_t A, size_t row_stride,
                       const uint32_t *actors, uint64_t *frame_off, uint8_t *bytes, size_t cap, size_t *total);
int crdt_pncounter_egress(crdt_ctx *ctx, const uint64_t *rows, size_t N, size_t A, size_t row_stride,
                          const uint32_t *actors, uint64_t *frame_off, uint8_t *bytes, size_t cap, size_t *total);
int crdt_gset_egress(crdt_ctx *ctx, const uint64_t *rows, size_t N, size_t U, size_t row_stride,
                     const uint64_t *elems, uint64_t *frame_off, uint8_t *bytes, size_t cap, size_t *total);
/* 16 bytes per state at bytes + 16*s (val, marker). */
int crdt_lwwreg_egress(crdt_ctx *ctx, const uint64_t *marker, const uint64_t *val, size_t N, uint8_t *bytes);
/* Orswot states (clock [N][A], entries [N][M][A] packed) and their deferred removes pooled by state
 * (def_off device [N+1] or NULL = none; def_keep [D] or NULL = all kept): the lub_many output
 * shape with def_off as a device array. */
int crdt_orswot_egress(crdt_ctx *ctx, const uint64_t *clock, const uint64_t *entries, size_t N, size_t M, size_t A,
                       const uint32_t *actors, const uint64_t *members, const uint64_t *def_off,
                       const uint64_t *def_clock, const uint64_t *def_members, const uint8_t *def_keep,
                       uint64_t *frame_off, uint8_t *bytes, size_t cap, size_t *total);
/* Map<u32, MVReg<u64, u32>, u32> (BASELINE config 4's type; map.rs:31-47, mvreg.rs:32-35) frames
 * <-> packed crdt_map_states: clock_stride A, ec_stride K*A, vclk_stride K*V*A, vval_stride K*V;
 * key k = position of its u32 id in the sorted `keys` dictionary, MVReg values in Vec order in
 * slots 0.., and per-state deferred slots of a crdt_map_deferred.  Ingest status bits as above
 * (4 = a key had more than V values or a state more than Dcap removes: the excess was dropped).
 * Egress writes present keys ascending, occupied value slots in slot order, count[s] removes. */
int crdt_map_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, const uint32_t *actors,
                    const uint32_t *keys, const crdt_map_states *out, const crdt_map_deferred *out_def,
                    uint32_t *status);
int crdt_map_egress(crdt_ctx *ctx, const crdt_map_states *states, const crdt_map_deferred *def, const uint32_t *actors,
                    const uint32_t *keys, uint64_t *frame_off, uint8_t *bytes, size_t cap, size_t *total);
/* The value-typed Maps (round 5): Map<u32, GCounter<u32>, u32> / Map<u32, PNCounter<u32>, u32>
 * (W = 1 / 2) frames <-> packed crdt_map_counter_states: clock_stride A, ec_stride K*A, val_stride
 * K*W*A; and Map<u32, Orswot<u64, u32>, u32> frames <-> crdt_map_orswot_states: the nested Orswot's
 * clock oc, member dots ent by the sorted u64 `members` dictionary, its deferred removes in slots
 * 0 .. vd_n[s][k] < Vd with member bitmaps vd_mem [N][K][Vd][ceil(M/64)]; the Map's deferred removes
 * in per-state slots, a crdt_map_deferred.  Value encodings: GCounter = VClock, PNCounter = VClock p,
 * VClock n, Orswot as crdt_orswot_ingest.  Ingest status bits as above (4 = a state held more than
 * Dcap Map removes or a key's Orswot more than Vd: the excess was dropped).  Egress writes present
 * keys ascending (entry clock nonzero), present members ascending (dot row nonzero), vd_n nested
 * removes and count[s] Map removes with their ids ascending. */
int crdt_map_counter_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, const uint32_t *actors,
                            const uint32_t *keys, const crdt_map_counter_states *out, const crdt_map_deferred *out_def,
                            uint32_t *status);
int crdt_map_counter_egress(crdt_ctx *ctx, const crdt_map_counter_states *states, const crdt_map_deferred *def,
                            const uint32_t *actors, const uint32_t *keys, uint64_t *frame_off, uint8_t *bytes,
                            size_t cap, size_t *total);
int crdt_map_orswot_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, const uint32_t *actors,
                           const uint32_t *keys, const uint64_t *members, const crdt_map_orswot_states *out,
                           const crdt_map_deferred *out_def, uint32_t *status);
int crdt_map_orswot_egress(crdt_ctx *ctx, const crdt_map_orswot_states *states, const crdt_map_deferred *def,
                           const uint32_t *actors, const uint32_t *keys, const uint64_t *members, uint64_t *frame_off,
                           uint8_t *bytes, size_t cap, size_t *total);
/* Map<u32, Map<u32, MVReg<u64, u32>, u32>, u32> (the reference's own Map test type, test/map.rs:10)
 * frames <-> crdt_map_nested_states: the inner Map's clock ic, its entries by the sorted u32 inner-key
 * dictionary `ikeys` (K2 <= 256, round 6) with their MVReg values in slots 0 .. nval < 8 (Vec order), its
 * deferred removes in slots 0 .. id_n < 16 with a K2w-word inner-key mask each; the outer Map's removes in
 * per-state slots.  Status bit 4: a register past 8 values, an inner list past 16 or an outer one
 * past Dcap (the excess dropped). */
int crdt_map_nested_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, const uint32_t *actors,
                           const uint32_t *keys, const uint32_t *ikeys, const crdt_map_nested_states *out,
                           const crdt_map_deferred *out_def, uint32_t *status);
int crdt_map_nested_egress(crdt_ctx *ctx, const crdt_map_nested_states *states, const crdt_map_deferred *def,
                           const uint32_t *actors, const uint32_t *keys, const uint32_t *ikeys, uint64_t *frame_off,
                           uint8_t *bytes, size_t cap, size_t *total);

/* ---- synthetic inputs (bench / test data, generated in HBM) --------------------------------
 * Counter-based and reproducible on the CPU (oracle/oracle.py synth_* restates them; small
 * fixtures of both are pinned by tests/golden/make_golden.py -> tests/golden/synth.json).
 * kind 0 = clock/counter cells, 1 = GSet bitmap words, 2 = LWW markers, 3 = LWW vals.
 * Row r < rows of the output is row (first_row + r) of the global synthetic matrix: cell
 * (first_row + r, i) gets synth(seed, (first_row + r)*width + i), stored at out[r*row_stride + i].
 * (first_row lets every rank generate its own replica shard of one global input.) */
int crdt_synth_fill(crdt_ctx *ctx, uint64_t *out, size_t rows, size_t width, size_t row_stride,
                    size_t first_row, uint64_t seed, int kind);

/* Well-formed synthetic Orswot replicas, packed clock[R][A] and entries[R][M][A] (replica r is
 * global replica first_row + r).  clock[r][a] = synth(seed, r*A + a) % (kmax + 1); actor a's
 * k-th add targets member (a*P + k) mod M (P = 0x9E3779B1 mod M), so a dot is unique and
 * entries[r][m][a] = k <= clock[r][a] or 0: a quarter of the dots are removed, and a replica has
 * observed (zeroed) a removed dot once clock[r][a] >= k + 1 + delta(m, a), delta in 0..7.
 * Requires kmax < M.  Restated on the CPU by oracle.synth_orswot. */
int crdt_synth_orswot(crdt_ctx *ctx, uint64_t *clock, uint64_t *entries, size_t R, size_t M,
                      size_t A, size_t first_row, uint64_t seed, uint64_t kmax);
/* For each deferred remove d held by replica def_row[d] (rm clock def_clock[d*A..], member
 * bitmap def_members[d*Mw..]): forget(rm) on those members of that replica's entries — the
 * state apply_rm (orswot.rs:230-238) leaves behind.  Used to build consistent inputs. */
int crdt_synth_orswot_rm(crdt_ctx *ctx, uint64_t *entries, size_t M, size_t A, size_t D,
                         const uint32_t *def_row, const uint64_t *def_clock,
                         const uint64_t *def_members);

/* Well-formed synthetic Map<K, MVReg<u64>> replicas (config 4), packed clock[R][A],
 * ec[R][K][A], vclk[R][K][V][A], vval[R][K][V] for global replicas first_row + r; model in
 * csrc/synth.hip, restated on the CPU by oracle.synth_map.  def_off (device, R+1 local
 * offsets, may be NULL), def_clock[D][A], def_keys[D][Kw]: the replicas' own deferred removes,
 * pre-applied (apply_keyset_rm, map.rs:318-333). */
int crdt_synth_map(crdt_ctx *ctx, uint64_t *clock, uint64_t *ec, uint64_t *vclk, uint64_t *vval,
                   size_t R, size_t K, size_t A, size_t V, size_t first_row, uint64_t seed,
                   uint64_t kmax, const uint64_t *def_off, const uint64_t *def_clock,
                   const uint64_t *def_keys);

#ifdef __cplusplus
}
#endif
#endif /* CRDT_GPU_H */
