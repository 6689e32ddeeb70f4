// Batched Map<K, MVReg<u64>> CmRDT::apply: N independent states, each with its own ordered op
// stream.  Reference (map.rs:119-137, apply_keyset_rm :318-348,
// apply_deferred :311-316; MVReg::apply mvreg.rs:130-166, MVReg::forget :88-104), restated on
// the dense layout of crdt_map_lub_many (entry clock EC[k][a], value slots VC[k][j][a] / VV[k][j]
// in Vec order with empty slots skipped, deferred (rm clock, key set) slots):
//   Op::Up { dot (a, k), key, op: Put { clock pc, val } }:
//       if C[a] >= k: seen, no-op                                              (:123-126)
//       EC[key][a] = max(EC[key][a], k)                      (entry().or_default(), clock.apply)
//       MVReg::apply: if pc is empty: nothing; else drop every value whose clock is <= pc
//           (partial_cmp not in {None, Greater}); append (pc, val) unless a remaining value's
//           clock is > pc                                                 (mvreg.rs:130-166)
//       C[a] = k; apply_deferred()                                              (:133-134)
//   Op::Rm { clock rm, keyset }: apply_keyset_rm                                (:121, :318-348)
//       for key in keyset: EC[key] = EC[key].forget(rm); if it empties the entry is dropped
//           (values too), else every value clock forgets rm and an emptied value is dropped
//       if !(rm <= C) (C.partial_cmp(rm) in {None, Less}): defer (rm, keyset), OR-ing the keys
//           into an existing deferred with the identical clock
// One wave per state (lanes = actors, A <= 1,024 with 1-16 clock words per lane; V unbounded: the
// value slots are walked in HBM; the state's clock in registers, its deferred list
// in LDS for the whole stream, entries and values in HBM), as orswot_apply.hip.
#include "common.hpp"
#include "group.hpp"

namespace crdt {

constexpr int kMA = 4;      // clock words per lane of the fast instances (A <= 256)
constexpr int kMAWide = 16;  // ... of the widest instance (A <= 1,024; round 4: the reference is unbounded)

struct MapApplyPlan {
  u64 *clock;
  unsigned long long clock_s;
  u64 *ec;
  unsigned long long ec_s;
  u64 *vclk;
  unsigned long long vclk_s;
  u64 *vval;
  unsigned long long vval_s;
  u64 *def_clock, *def_keys;
  uint32_t *def_count;
  unsigned long long N, K, A, V, Kw, Dcap;
  const u64 *op_off;
  const uint8_t *kind;
  const uint32_t *actor;
  const u64 *counter;
  const uint32_t *key;
  const u64 *val;
  const uint32_t *clk_row;
  const u64 *clk_pool;
  unsigned long long n_clk_rows;
  const u64 *key_off;
  const uint32_t *keys;
  unsigned long long n_keys;
  unsigned long long n_ops;
  uint32_t *status;
  int wpb;
  unsigned long long Dh;  // deferred slots kept in LDS (the rest in the state's own HBM slots)
  int fence;              // 1: a workgroup fence after each op's stores (CRDT_TUNE afence=1, the round-2 form)
};

// W clock words per lane: 1 for A <= 64 (fewer VGPRs, more waves per SIMD), 2 to A = 128, 4 to 256
template <int W>
struct RowT {
  u64 w[W];
};

template <int W>
__device__ __forceinline__ RowT<W> load_row(const u64 *p, int lane, unsigned long long A) {
  RowT<W> r;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const unsigned long long a = lane + j * kWave;
    r.w[j] = a < A ? p[a] : 0ull;
  }
  return r;
}
template <int W>
__device__ __forceinline__ void store_row(u64 *p, const RowT<W> &r, int lane, unsigned long long A) {
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const unsigned long long a = lane + j * kWave;
    if (a < A) p[a] = r.w[j];
  }
}
template <int W>
__device__ __forceinline__ bool any_nz(const RowT<W> &r) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < W; ++j) b |= r.w[j] != 0;
  return __ballot(b) != 0;
}
// x <= y on every actor (padding lanes hold 0 on both sides)
template <int W>
__device__ __forceinline__ bool all_le(const RowT<W> &x, const RowT<W> &y) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < W; ++j) b |= x.w[j] > y.w[j];
  return __ballot(b) == 0;
}
template <int W>
__device__ __forceinline__ bool rows_eq(const RowT<W> &x, const RowT<W> &y) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < W; ++j) b |= x.w[j] != y.w[j];
  return __ballot(b) == 0;
}
template <int W>
__device__ __forceinline__ RowT<W> forget_row(const RowT<W> &x, const RowT<W> &y) {  // vclock.rs:95-105
  RowT<W> r;
#pragma unroll
  for (int j = 0; j < W; ++j) r.w[j] = x.w[j] > y.w[j] ? x.w[j] : 0ull;
  return r;
}
template <int W>
__device__ __forceinline__ RowT<W> zero_row() {
  RowT<W> r;
#pragma unroll
  for (int j = 0; j < W; ++j) r.w[j] = 0;
  return r;
}
__device__ __forceinline__ unsigned rl32m(unsigned x, int l) { return (unsigned)__builtin_amdgcn_readlane((int)x, l); }
__device__ __forceinline__ u64 rl64m(u64 x, int l) {
  return ((u64)rl32m((unsigned)(x >> 32), l) << 32) | rl32m((unsigned)x, l);
}
__device__ __forceinline__ void wave_fence_m() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup"); }

struct KeyRefs {
  u64 *ec, *vc, *vv;
};
__device__ __forceinline__ KeyRefs key_refs(const MapApplyPlan &p, unsigned long long s, unsigned long long k) {
  return KeyRefs{p.ec + s * p.ec_s + k * p.A, p.vclk + s * p.vclk_s + k * p.V * p.A, p.vval + s * p.vval_s + k * p.V};
}

// apply_keyset_rm's body for one key (map.rs:320-333)
template <int W>
__device__ void key_rm(const MapApplyPlan &p, unsigned long long s, unsigned long long k, const RowT<W> &rm, int lane) {
  const KeyRefs q = key_refs(p, s, k);
  const RowT<W> e = load_row<W>(q.ec, lane, p.A);
  if (!any_nz(e)) return;  // no entry for this key
  const RowT<W> e2 = forget_row(e, rm);
  const bool alive = any_nz(e2);
  store_row(q.ec, e2, lane, p.A);
  for (unsigned long long j = 0; j < p.V; ++j) {
    u64 *vr = q.vc + j * p.A;
    const RowT<W> v = load_row<W>(vr, lane, p.A);
    if (!any_nz(v)) continue;
    const RowT<W> v2 = alive ? forget_row(v, rm) : zero_row<W>();  // MVReg::forget mvreg.rs:88-104
    store_row(vr, v2, lane, p.A);
    if (!any_nz(v2) && lane == 0) q.vv[j] = 0;
  }
}

// forget every key of an LDS bitmap
template <int W>
__device__ void keyset_rm(const MapApplyPlan &p, unsigned long long s, const u64 *bits, const RowT<W> &rm, int lane) {
  for (unsigned long long w0 = 0; w0 < p.Kw; w0 += kWave) {
    const u64 word = (w0 + lane < p.Kw) ? bits[w0 + lane] : 0ull;
    u64 nz = __ballot(word != 0);
    while (nz) {
      const int l = __builtin_ctzll(nz);
      nz &= nz - 1;
      u64 wv = rl64m(word, l);
      while (wv) {
        const unsigned long long k = (w0 + l) * 64 + __builtin_ctzll(wv);
        wv &= wv - 1;
        if (k < p.K) key_rm(p, s, k, rm, lane);
      }
    }
  }
}

template <int W>
__device__ __forceinline__ bool any_gt(const RowT<W> &r, const RowT<W> &c) {  // !(r <= c)
  return !all_le(r, c);
}

// SP: some deferred slots live in HBM (Dh < Dcap); without it every slot pointer is a known LDS
// address (ds_read/ds_write, not flat accesses)
template <int W, bool SP>
__device__ __forceinline__ void map_apply_body(const MapApplyPlan &p) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x % kWave;
  const int wib = threadIdx.x / kWave;
  const unsigned long long A = p.A;
  const unsigned long long per_wave = p.Dh * (A + p.Kw);
  u64 *dcl = lds + wib * per_wave;  // [Dh][A]
  u64 *dkb = dcl + p.Dh * A;        // [Dh][Kw]

  for (unsigned long long s = (unsigned long long)blockIdx.x * p.wpb + wib; s < p.N;
       s += (unsigned long long)gridDim.x * p.wpb) {
    unsigned st = 0;
    const unsigned long long ob = p.op_off[s], oe = p.op_off[s + 1];
    unsigned dcnt = p.def_count[s];
    if (dcnt > p.Dcap || oe < ob || oe > p.n_ops) {
      if (lane == 0) p.status[s] = (dcnt > p.Dcap ? 4u : 0u) | (oe < ob || oe > p.n_ops ? 8u : 0u);
      continue;
    }
    u64 *Cg = p.clock + s * p.clock_s;
    RowT<W> C = load_row<W>(Cg, lane, A);
    const u64 *gdc = p.def_clock + s * p.Dcap * A;
    const u64 *gdk = p.def_keys + s * p.Dcap * p.Kw;
    const unsigned long long dhot = SP && dcnt > p.Dh ? p.Dh : dcnt;
    for (unsigned long long i = lane; i < dhot * A; i += kWave) dcl[i] = gdc[i];
    for (unsigned long long i = lane; i < dhot * p.Kw; i += kWave) dkb[i] = gdk[i];
    // slot d: LDS for d < Dh, else the state's own HBM slot (SP only; generic pointers)
    auto SC = [&](unsigned long long d) -> u64 * {
      return !SP || d < p.Dh ? dcl + d * A : p.def_clock + (s * p.Dcap + d) * A;
    };
    auto SK = [&](unsigned long long d) -> u64 * {
      return !SP || d < p.Dh ? dkb + d * p.Kw : p.def_keys + (s * p.Dcap + d) * p.Kw;
    };
    wave_fence_m();
    // apply_deferred re-forgets every key of every deferred slot (map.rs:311-316).  After one full
    // pass each slot's keys are forgotten by its clock; later ops keep that (an Rm only forgets more,
    // and forgets commute; a new slot's keys were just forgotten by it), and an Up changes only its
    // own key's rows, so every later pass re-forgets key k alone — the same rows as the full pass,
    // since forgetting is idempotent.  The first pass stays full: the input state need not hold
    // the invariant.
    bool full = true;

    for (unsigned long long base = ob; base < oe; base += kWave) {
      const unsigned long long o = base + lane;
      const bool ov = o < oe;
      const unsigned h_kind = ov ? p.kind[o] : 0u;
      const unsigned h_actor = ov && p.actor ? p.actor[o] : 0u;
      const u64 h_counter = ov && p.counter ? p.counter[o] : 0ull;
      const unsigned h_key = ov && p.key ? p.key[o] : 0u;
      const u64 h_val = ov && p.val ? p.val[o] : 0ull;
      const unsigned h_row = ov && p.clk_row ? p.clk_row[o] : 0u;
      const u64 h_kb = ov && p.key_off ? p.key_off[o] : 0ull;
      const u64 h_ke = ov && p.key_off ? p.key_off[o + 1] : 0ull;
      const int nb = (int)((oe - base) < (unsigned long long)kWave ? (oe - base) : kWave);
      // op i's clock row is loaded while op i-1 runs (the pool is read-only): one dependent
      // round trip less per op
      auto pool_row = [&](int j) -> RowT<W> {
        const unsigned r = rl32m(h_row, j);
        return load_row<W>(p.clk_pool + (unsigned long long)(r < p.n_clk_rows ? r : 0u) * A, lane, A);
      };
      RowT<W> ocn = p.n_clk_rows ? pool_row(0) : zero_row<W>();
      for (int i = 0; i < nb; ++i) {
        const RowT<W> oc = ocn;
        if (i + 1 < nb && p.n_clk_rows) ocn = pool_row(i + 1);
        const unsigned kind = rl32m(h_kind, i);
        const unsigned rr = rl32m(h_row, i);
        if (kind > 1 || rr >= p.n_clk_rows) {
          st |= 2u;
          continue;
        }
        if (kind == 0) {  // ---- Op::Up
          const unsigned long long a = rl32m(h_actor, i), k = rl32m(h_key, i);
          const u64 kc = rl64m(h_counter, i);
          if (a >= A || k >= p.K) {
            st |= 2u;
            continue;
          }
          const int ja = (int)(a / kWave), la = (int)(a % kWave);
          u64 cj = C.w[0];
#pragma unroll
          for (int j = 1; j < W; ++j)
            if (j == ja) cj = C.w[j];
          if (rl64m(cj, la) >= kc) continue;  // seen (:123-126)
          const KeyRefs q = key_refs(p, s, k);
          // the register's first kVB value rows in one batch of loads (clamped, unconditional, so
          // they issue together and under the entry cell's round trip), the rest one at a time
          constexpr int kVB = 4;
          RowT<W> vb[kVB];
#pragma unroll
          for (int j = 0; j < kVB; ++j)
            vb[j] = load_row<W>(q.vc + ((unsigned long long)j < p.V ? j : 0) * A, lane, A);
          if (lane == la) {  // entry clock apply(dot) (:130)
            u64 *cell = q.ec + a;
            if (*cell < kc) *cell = kc;
          }
          if (any_nz(oc)) {  // MVReg::apply (mvreg.rs:130-166)
            bool should_add = true;
            int last = -1, used = 0;
            for (unsigned long long j = 0; j < p.V; ++j) {
              u64 *vr = q.vc + j * A;
              RowT<W> v;
              if (j < (unsigned long long)kVB) {
                v = vb[0];
#pragma unroll
                for (int t = 1; t < kVB; ++t)
                  if ((unsigned long long)t == j) v = vb[t];
              } else {
                v = load_row<W>(vr, lane, A);
              }
              if (!any_nz(v)) continue;
              if (all_le(v, oc)) {  // partial_cmp in {Less, Equal}: dropped
                store_row(vr, zero_row<W>(), lane, A);
                if (lane == 0) q.vv[j] = 0;
                continue;
              }
              if (all_le(oc, v)) should_add = false;  // v > pc (Greater)
              last = (int)j;
              ++used;
            }
            if (should_add) {
              int slot = last + 1;
              if (slot >= (int)p.V) {
                if (used >= (int)p.V) {
                  st |= 16u;  // more values than slots: the state is incomplete
                  slot = -1;
                } else {  // compact the used slots in order, then append
                  if (p.fence) wave_fence_m();
                  int w = 0;
                  for (unsigned long long j = 0; j < p.V; ++j) {
                    const RowT<W> v = load_row<W>(q.vc + j * A, lane, A);
                    if (!any_nz(v)) continue;
                    if ((unsigned long long)w != j) {
                      const u64 x = q.vv[j];
                      if (p.fence) wave_fence_m();
                      store_row(q.vc + (unsigned long long)w * A, v, lane, A);
                      store_row(q.vc + j * A, zero_row<W>(), lane, A);
                      if (lane == 0) {
                        q.vv[w] = x;
                        q.vv[j] = 0;
                      }
                      if (p.fence) wave_fence_m();
                    }
                    ++w;
                  }
                  slot = w;
                }
              }
              // readlane with every lane active: inside `if (lane == 0)` only lane 0 of a
              // spilled h_val would be reloaded and lane i's copy would be stale
              const u64 pv = rl64m(h_val, i);
              if (slot >= (int)p.V) {  // unreachable by construction; reported, never written
                st |= 32u;
                slot = -1;
              }
              if (slot >= 0) {
                store_row(q.vc + (unsigned long long)slot * A, oc, lane, A);
                if (lane == 0) q.vv[slot] = pv;
              }
            }
          }
#pragma unroll
          for (int j = 0; j < W; ++j)
            if (j == ja && lane == la) C.w[j] = kc;  // self.clock.apply(dot) (:133)
          if (p.fence) wave_fence_m();
          unsigned nk = 0;  // apply_deferred (:134, :311-316)
          for (unsigned d = 0; d < dcnt; ++d) {
            const RowT<W> rm = load_row<W>(SC(d), lane, A);
            if (full) {
              keyset_rm(p, s, SK(d), rm, lane);
            } else if ((rl64m(SK(d)[k / 64], 0) >> (k % 64)) & 1ull) {
              key_rm(p, s, k, rm, lane);  // only key k changed since the last full pass
            }
            if (p.fence) wave_fence_m();
            if (any_gt(rm, C)) {
              if (nk != d) {
                u64 *dc = SC(nk), *dk = SK(nk);
                const u64 *sc = SC(d), *sk = SK(d);
                for (unsigned long long t = lane; t < A; t += kWave) dc[t] = sc[t];
                for (unsigned long long t = lane; t < p.Kw; t += kWave) dk[t] = sk[t];
              }
              ++nk;
            }
          }
          dcnt = nk;
          full = false;
          if (p.fence) wave_fence_m();
        } else {  // ---- Op::Rm -> apply_keyset_rm (:318-348)
          const u64 kb = rl64m(h_kb, i), ke = rl64m(h_ke, i);
          if (ke < kb || ke > p.n_keys) {  // reversed, or runs past the keys buffer
            st |= 2u;
            continue;
          }
          for (u64 jb = kb; jb < ke; jb += kWave) {
            const unsigned kk = jb + lane < ke ? p.keys[jb + lane] : 0u;
            const int n = (int)((ke - jb) < (u64)kWave ? (ke - jb) : kWave);
            for (int t = 0; t < n; ++t) {
              const unsigned long long k = rl32m(kk, t);
              if (k >= p.K) {
                st |= 2u;
                continue;
              }
              key_rm(p, s, k, oc, lane);
              if (p.fence) wave_fence_m();
            }
          }
          if (!any_gt(oc, C)) continue;  // rm <= clock: not deferred (:336-345)
          int slot = -1;
          for (unsigned d = 0; d < dcnt; ++d)
            if (rows_eq(load_row<W>(SC(d), lane, A), oc)) {
              slot = (int)d;
              break;
            }
          if (slot < 0) {
            if (dcnt >= p.Dcap) {
              st |= 1u;
              continue;
            }
            slot = (int)dcnt++;
            store_row(SC((unsigned long long)slot), oc, lane, A);
            u64 *nb = SK((unsigned long long)slot);
            for (unsigned long long t = lane; t < p.Kw; t += kWave) nb[t] = 0;
            if (p.fence) wave_fence_m();
          }
          u64 *bits = SK((unsigned long long)slot);
          if (!SP || (unsigned long long)slot < p.Dh) {  // LDS: lanes OR their keys in at once
            for (u64 jk = kb + lane; jk < ke; jk += kWave) {
              const unsigned long long k = p.keys[jk];
              if (k < p.K) atomicOr(bits + k / 64, 1ull << (k % 64));
            }
          } else {  // an HBM slot: plain read-modify-writes, one key at a time (no L2 atomics that
                    // this wave's later plain loads could miss through its L1)
            for (u64 jb = kb; jb < ke; jb += kWave) {
              const unsigned kk = jb + lane < ke ? p.keys[jb + lane] : 0u;
              const int n = (int)((ke - jb) < (u64)kWave ? (ke - jb) : kWave);
              for (int t = 0; t < n; ++t) {
                const unsigned long long k = (unsigned)__builtin_amdgcn_readlane((int)kk, t);
                if (k < p.K && lane == 0) bits[k / 64] |= 1ull << (k % 64);
                if (p.fence) wave_fence_m();
              }
            }
          }
          if (p.fence) wave_fence_m();
        }
      }
    }
    store_row(Cg, C, lane, A);
    const unsigned long long dout = SP && dcnt > p.Dh ? p.Dh : dcnt;  // slots >= Dh are already in HBM
    u64 *wdc = p.def_clock + s * p.Dcap * A;
    u64 *wdk = p.def_keys + s * p.Dcap * p.Kw;
    for (unsigned long long i = lane; i < dout * A; i += kWave) wdc[i] = dcl[i];
    for (unsigned long long i = lane; i < dout * p.Kw; i += kWave) wdk[i] = dkb[i];
    if (lane == 0) {
      p.def_count[s] = dcnt;
      p.status[s] = st;
    }
    wave_fence_m();
  }
}

// A <= 64: asking for 7 waves per SIMD (72 VGPRs, 28 B/lane of spills) is 7% faster than the
// compiler's 6 (3.29 vs 3.53 ms, profiles/r02_map_apply_wpe7_ab.log).  Round 1's miscompute at
// that occupancy was a readlane of a spilled VGPR inside `if (lane == 0)` (fixed above), not the
// spilling itself; the wider instances keep the compiler's choice (they would spill 44-116 B/lane).
template <bool SP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(7))) void map_apply_kernel_w1(MapApplyPlan p) {
  map_apply_body<1, SP>(p);
}
template <int W, bool SP>
__global__ __launch_bounds__(kBlock) CRDT_APPLY_ATTR void map_apply_kernel(MapApplyPlan p) {
  map_apply_body<W, SP>(p);
}

// ---- 16 lanes per state (A <= 64) ----------------------------------------------------------------
// The structure of the Orswot group kernel (orswot_apply.hip, group.hpp) for Map<K, MVReg>: a group
// of 16 lanes runs one state (4 states per wave; lane g holds actors g + 16j, the clock in
// registers), op headers come 16 at a time through LDS, a row operation (entry clock, value clock,
// Put / rm clock) costs each lane KJ words read 128 contiguous bytes per group.  apply_deferred
// (map.rs:311-316) without rescanning every slot on every Up: each slot keeps a WITNESS, the first
// actor with rm[a] > C[a] (C only grows: the witness only moves forward; an Up to actor a re-examines
// the slots whose witness is a, W a 64-bit mask of witness actors), the re-forget after the first
// full pass touches the Up's own key only (its rows are all the Up changed) and only when its key may
// be in a slot (bloom of the slots' key-bitmap words), and a Rm compares its clock in full only
// with slots of the same witness.  Exact for any input state.
// Forget rm on key k whose entry-clock row is already in e (filtered in place).
template <int KJ>
__device__ void gkey_rm_row(const MapApplyPlan &p, const KeyRefs &q, u64 (&e)[KJ], const u64 (&rm)[KJ], int g,
                            int lane) {
  if (!grp::any_nz<KJ>(e, lane)) return;  // no entry for this key
#pragma unroll
  for (int j = 0; j < KJ; ++j) e[j] = e[j] > rm[j] ? e[j] : 0ull;
  const bool alive = grp::any_nz<KJ>(e, lane);
  grp::store_row<KJ>(q.ec, e, g, p.A);
  for (unsigned long long jv = 0; jv < p.V; ++jv) {
    u64 v[KJ];
    grp::load_row<KJ>(v, q.vc + jv * p.A, g, p.A);
    if (!grp::any_nz<KJ>(v, lane)) continue;
#pragma unroll
    for (int j = 0; j < KJ; ++j) v[j] = alive && v[j] > rm[j] ? v[j] : 0ull;  // MVReg::forget mvreg.rs:88-104
    grp::store_row<KJ>(q.vc + jv * p.A, v, g, p.A);
    if (!grp::any_nz<KJ>(v, lane) && g == 0) q.vv[jv] = 0;
  }
}
template <int KJ>
__device__ void gkey_rm(const MapApplyPlan &p, unsigned long long s, unsigned long long k, const u64 (&rm)[KJ],
                        int g, int lane) {
  const KeyRefs q = key_refs(p, s, k);
  u64 e[KJ];
  grp::load_row<KJ>(e, q.ec, g, p.A);
  gkey_rm_row<KJ>(p, q, e, rm, g, lane);
}

// PF (round 4): the entry-clock row of op i+1's key (an Up's key, an Rm's first key — carried in the
// header) is loaded with its Put / rm clock while op i runs; op i marks it stale when it writes that
// key's rows (same key, or a full apply_deferred pass) and op i+1 then reloads it.  The entry cell
// of an Up is updated from that row (no dependent read), and an Up of an absent key (entry clock
// all 0 <=> key absent, whose value rows are all 0 by the layout) writes its value to slot 0
// without reading the value rows: ~90% of the Ups at the apply benchmark's shape.
// MT (round 5, default with PF while Dcap <= kMapMetaSlots): per slot, next to its witness byte, the
// OR of the slot's key-bitmap words in LDS — the bloom is rebuilt from LDS alone after a slot is
// dropped, and an Up's re-forget tests a slot's LDS word before reading its key word (as the Orswot
// kernel's MT, orswot_apply.hip).
constexpr unsigned long long kMapMetaSlots = 64;
template <int KJ, bool PF, bool MT = false>
#ifndef CRDT_MAPGRP_WPE
#define CRDT_MAPGRP_WPE 4  // waves per SIMD of the KJ <= 2 instances (build option)
#endif
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KJ <= 2 ? CRDT_MAPGRP_WPE : 1))) void map_apply_grp_kernel(MapApplyPlan p) {
  extern __shared__ u64 lds[];
  constexpr int kG = grp::kG;
  constexpr int kVB = 4;  // value rows of an Up loaded in one batch
  const int lane = (int)(threadIdx.x % kWave), g = lane & (kG - 1);
  const bool lead = g == 0;
  const unsigned long long s = ((unsigned long long)blockIdx.x * kBlock + threadIdx.x) / kG;
  if (s >= p.N) return;  // (whole groups)
  const unsigned long long A = p.A, K = p.K, V = p.V, Kw = p.Kw, Dcap = p.Dcap;
  // LDS: per group the op headers of the current batch (48 bytes each), then the slot witnesses
  u64 *hdr = lds + (threadIdx.x / kG) * (6 * kG);
  uint8_t *wit = reinterpret_cast<uint8_t *>(lds + (kBlock / kG) * 6 * kG) + (threadIdx.x / kG) * Dcap;
  u64 *sbl = lds + (kBlock / kG) * 6 * kG + ((kBlock / kG) * Dcap + 7) / 8 + (threadIdx.x / kG) * Dcap;  // (MT)

  const unsigned long long ob = p.op_off[s], oe = p.op_off[s + 1];
  unsigned dcnt = p.def_count[s];
  if (dcnt > Dcap || oe < ob || oe > p.n_ops) {
    if (lead) p.status[s] = (dcnt > Dcap ? 4u : 0u) | (oe < ob || oe > p.n_ops ? 8u : 0u);
    return;  // state left untouched
  }
  unsigned st = 0;
  u64 *Cg = p.clock + s * p.clock_s;
  u64 *DC = p.def_clock + s * Dcap * A;
  u64 *DK = p.def_keys + s * Dcap * Kw;
  u64 c[KJ];
  grp::load_row<KJ>(c, Cg, g, A);

  u64 W = 0, bloom = 0;
  auto rebuild = [&]() {  // witness mask and key bloom from the slots (the same in the group's lanes)
    W = 0;
    u64 b = 0;
    for (unsigned d = 0; d < dcnt; ++d) {
      const unsigned w = wit[d];
      if (w != grp::kNone) W |= 1ull << w;
      if (MT) b |= sbl[d];
      else
        for (unsigned long long x = g; x < Kw; x += kG) b |= DK[d * Kw + x];
    }
    bloom = MT ? b : grp::orx(b);
  };
  for (unsigned d = 0; d < dcnt; ++d) {  // the input slots' witnesses at the input clock
    u64 x[KJ];
    grp::load_row<KJ>(x, DC + d * A, g, A);
    const unsigned w = grp::witness<KJ>(x, c, g, 0, A);
    if (lead) wit[d] = (uint8_t)w;
    if (MT) {
      u64 b = 0;
      for (unsigned long long y = g; y < Kw; y += kG) b |= DK[d * Kw + y];
      b = grp::orx(b);
      if (lead) sbl[d] = b;
    }
  }
  rebuild();
  bool full = true;  // no Up yet: the input slots' keys are re-forgotten in full at the first
  auto drop = [&](unsigned d) {  // the last slot moves over slot d
    const unsigned last = dcnt - 1;
    if (d != last) {
#pragma unroll
      for (int j = 0; j < KJ; ++j) {
        const unsigned a = g + kG * j;
        if (a < A) DC[d * A + a] = DC[last * A + a];
      }
      for (unsigned long long x = g; x < Kw; x += kG) DK[d * Kw + x] = DK[last * Kw + x];
      if (lead) wit[d] = wit[last];
      if (MT && lead) sbl[d] = sbl[last];
    }
    dcnt = last;
  };

  for (unsigned long long base = ob; base < oe; base += kG) {
    // op headers, lane g = op base + g: kind (0 Up, 1 Rm, 2 malformed) | actor, key | pool row,
    // counter, value, key range
    {
      const unsigned long long o = base + g;
      u64 w0 = 2, w1 = 0xFFFFFFFFull, w2 = 0, w3 = 0, w4 = 0, w5 = 0;
      if (o < oe) {
        const unsigned kind = p.kind[o];
        const unsigned rr = p.clk_row ? p.clk_row[o] : 0u;
        if (kind == 0 && rr < p.n_clk_rows) {
          const unsigned a = p.actor ? p.actor[o] : 0u, k = p.key ? p.key[o] : 0u;
          if (a < A && k < K) {
            w0 = (u64)a << 32;
            w1 = ((u64)rr << 32) | k;
            w2 = p.counter ? p.counter[o] : 0ull;
            w3 = p.val ? p.val[o] : 0ull;
          }
        } else if (kind == 1 && rr < p.n_clk_rows) {
          const u64 kb = p.key_off ? p.key_off[o] : 0ull, ke = p.key_off ? p.key_off[o + 1] : 0ull;
          if (ke >= kb && ke <= p.n_keys) {  // (reversed, or past the keys buffer: malformed)
            w0 = 1;
            w1 = ((u64)rr << 32) | (PF && kb < ke ? (u64)p.keys[kb] : 0xFFFFFFFFull);
            w4 = kb;
            w5 = ke;
          }
        }
      }
      *reinterpret_cast<u64x2 *>(hdr + 6 * g) = u64x2{w0, w1};
      *reinterpret_cast<u64x2 *>(hdr + 6 * g + 2) = u64x2{w2, w3};
      *reinterpret_cast<u64x2 *>(hdr + 6 * g + 4) = u64x2{w4, w5};
    }
    const int nb = (int)((oe - base) < (unsigned long long)kG ? (oe - base) : kG);
    // the Put / rm clock of op i+1 is loaded while op i runs (the pool is read-only)
    auto pool_row = [&](int i, u64 (&x)[KJ]) {
      const u64 h1 = hdr[6 * i + 1];
      grp::load_row<KJ>(x, p.clk_pool + (h1 >> 32) * A, g, A);
    };
    // PF: the entry-clock row of op i's key (the low word of header word 1; >= K: none)
    auto hkey = [&](int i) -> unsigned { return (unsigned)hdr[6 * i + 1]; };
    auto ec_row = [&](unsigned k, u64 (&x)[KJ]) {
      if (k < K) {
        grp::load_row<KJ>(x, p.ec + s * p.ec_s + (unsigned long long)k * A, g, A);
      } else {
#pragma unroll
        for (int j = 0; j < KJ; ++j) x[j] = 0;
      }
    };
    u64 ocn[KJ], ecn[KJ];
    unsigned kn = 0xFFFFFFFFu;  // key of the row in ecn
    bool ndirty = false;        // ecn stale: the op in flight wrote key kn's rows
    auto touch = [&](unsigned long long k) {
      if (PF && k == kn) ndirty = true;
    };
    pool_row(0, ocn);
    if (PF) {
      kn = hkey(0);
      ec_row(kn, ecn);
    }
    for (int i = 0; i < nb; ++i) {
      u64 oc[KJ], e[KJ];
#pragma unroll
      for (int j = 0; j < KJ; ++j) {
        oc[j] = ocn[j];
        e[j] = PF ? ecn[j] : 0ull;
      }
      const unsigned kcur = kn;
      const bool stale = ndirty;
      ndirty = false;
      if (i + 1 < nb) {
        pool_row(i + 1, ocn);
        if (PF) {
          kn = hkey(i + 1);
          ec_row(kn, ecn);
        }
      } else {
        kn = 0xFFFFFFFFu;
      }
      const u64x2 h0 = *reinterpret_cast<const u64x2 *>(hdr + 6 * i);
      const unsigned kind = (unsigned)h0[0];
      if (kind > 1) {
        st |= 2u;
        continue;
      }
      if (kind == 0) {  // ---- Op::Up (map.rs:119-137)
        const unsigned a = (unsigned)(h0[0] >> 32);
        const unsigned long long k = (unsigned)h0[1];
        const u64x2 h1 = *reinterpret_cast<const u64x2 *>(hdr + 6 * i + 2);
        const u64 kc = h1[0];
        if (grp::clock_at<KJ>(c, a, lane) >= kc) continue;  // seen (:123-126)
        const KeyRefs q = key_refs(p, s, k);
        u64 vb[kVB][KJ];
        bool vals = true;  // the key's value rows are read
        if (PF) {
          if (stale) grp::load_row<KJ>(e, q.ec, g, A);
          vals = grp::any_nz<KJ>(e, lane);  // an absent key holds no values
          if ((unsigned)g == a % kG) {      // entry clock apply(dot) (:130), from the row in registers
            u64 ea = e[0];
#pragma unroll
            for (int j = 1; j < KJ; ++j)
              if ((unsigned)j == a / kG) ea = e[j];
            if (ea < kc) q.ec[a] = kc;
          }
          touch(k);
          if (vals)
#pragma unroll
            for (int t = 0; t < kVB; ++t)
              grp::load_row<KJ>(vb[t], q.vc + ((unsigned long long)t < V ? t : 0) * A, g, A);
        } else {
#pragma unroll
          for (int t = 0; t < kVB; ++t)
            grp::load_row<KJ>(vb[t], q.vc + ((unsigned long long)t < V ? t : 0) * A, g, A);
          if ((unsigned)g == a % kG) {  // entry clock apply(dot) (:130)
            u64 *cell = q.ec + a;
            if (*cell < kc) *cell = kc;
          }
        }
        if (!vals && grp::any_nz<KJ>(oc, lane)) {  // MVReg::apply on no values: slot 0
          grp::store_row<KJ>(q.vc, oc, g, A);
          if (lead) q.vv[0] = h1[1];
        } else if (grp::any_nz<KJ>(oc, lane)) {  // MVReg::apply (mvreg.rs:130-166)
          bool should_add = true;
          int last = -1, used = 0;
          for (unsigned long long j = 0; j < V; ++j) {
            u64 v[KJ];
            if (j < (unsigned long long)kVB) {
#pragma unroll
              for (int t = 0; t < KJ; ++t) v[t] = vb[0][t];
#pragma unroll
              for (int u = 1; u < kVB; ++u)
                if ((unsigned long long)u == j)
#pragma unroll
                  for (int t = 0; t < KJ; ++t) v[t] = vb[u][t];
            } else {
              grp::load_row<KJ>(v, q.vc + j * A, g, A);
            }
            if (!grp::any_nz<KJ>(v, lane)) continue;
            if (grp::all_le<KJ>(v, oc, lane)) {  // partial_cmp in {Less, Equal}: dropped
              u64 z[KJ] = {};
              grp::store_row<KJ>(q.vc + j * A, z, g, A);
              if (lead) q.vv[j] = 0;
              continue;
            }
            if (grp::all_le<KJ>(oc, v, lane)) should_add = false;  // v > pc (Greater)
            last = (int)j;
            ++used;
          }
          if (should_add) {
            int slot = last + 1;
            if (slot >= (int)V) {
              if (used >= (int)V) {
                st |= 16u;  // more values than slots: the state is incomplete
                slot = -1;
              } else {  // compact the used slots in order, then append
                int w = 0;
                for (unsigned long long j = 0; j < V; ++j) {
                  u64 v[KJ];
                  grp::load_row<KJ>(v, q.vc + j * A, g, A);
                  if (!grp::any_nz<KJ>(v, lane)) continue;
                  if ((unsigned long long)w != j) {
                    const u64 x = q.vv[j];
                    u64 z[KJ] = {};
                    grp::store_row<KJ>(q.vc + (unsigned long long)w * A, v, g, A);
                    grp::store_row<KJ>(q.vc + j * A, z, g, A);
                    if (lead) {
                      q.vv[w] = x;
                      q.vv[j] = 0;
                    }
                  }
                  ++w;
                }
                slot = w;
              }
            }
            if (slot >= (int)V) {  // unreachable by construction; reported, never written
              st |= 32u;
              slot = -1;
            }
            if (slot >= 0) {
              grp::store_row<KJ>(q.vc + (unsigned long long)slot * A, oc, g, A);
              if (lead) q.vv[slot] = h1[1];
            }
          }
        }
        grp::clock_set<KJ>(c, a, kc, g);  // self.clock.apply(dot) (:133)
        // apply_deferred (:134, :311-316)
        if (full) {  // every slot's keys forgotten in full, every witness recomputed
          full = false;
          if (PF) ndirty = true;
          for (unsigned d = 0; d < dcnt;) {
            u64 rm[KJ];
            grp::load_row<KJ>(rm, DC + d * A, g, A);
            for (unsigned long long x = 0; x < Kw; ++x) {
              u64 kbits = DK[d * Kw + x];
              while (kbits) {
                const unsigned long long kk = x * 64 + __builtin_ctzll(kbits);
                kbits &= kbits - 1;
                if (kk < K) gkey_rm<KJ>(p, s, kk, rm, g, lane);
              }
            }
            const unsigned w = grp::witness<KJ>(rm, c, g, 0, A);
            if (w == grp::kNone) {
              drop(d);
            } else {
              if (lead) wit[d] = (uint8_t)w;
              ++d;
            }
          }
          rebuild();
          continue;
        }
        // key k re-forgotten by every slot naming it (only its rows changed)
        if (dcnt > 0 && ((bloom >> (k % 64)) & 1ull)) {
          for (unsigned d = 0; d < dcnt; ++d)
            if ((!MT || ((sbl[d] >> (k % 64)) & 1ull)) && ((DK[d * Kw + k / 64] >> (k % 64)) & 1ull)) {
              u64 rm[KJ];
              grp::load_row<KJ>(rm, DC + d * A, g, A);
              gkey_rm<KJ>(p, s, k, rm, g, lane);
            }
        }
        // the slots whose witness was actor a: move the witness on, drop a slot left without one
        if ((W >> a) & 1ull) {
          bool dropped = false;
          for (unsigned d = 0; d < dcnt;) {
            if (wit[d] == a && DC[d * A + a] <= kc) {
              u64 x[KJ];
              grp::load_row<KJ>(x, DC + d * A, g, A);
              const unsigned w = grp::witness<KJ>(x, c, g, a + 1, A);
              if (w == grp::kNone) {
                drop(d);
                dropped = true;
                continue;
              }
              if (lead) wit[d] = (uint8_t)w;
            }
            ++d;
          }
          if (dropped) {
            rebuild();
          } else {
            W = 0;
            for (unsigned d = 0; d < dcnt; ++d) {
              const unsigned w = wit[d];
              if (w != grp::kNone) W |= 1ull << w;
            }
          }
        }
      } else {  // ---- Op::Rm -> apply_keyset_rm (:318-348)
        const u64x2 h2 = *reinterpret_cast<const u64x2 *>(hdr + 6 * i + 4);
        const u64 kb = h2[0], ke = h2[1];
        for (u64 jk = kb; jk < ke; ++jk) {
          const unsigned long long kk = PF && jk == kb ? kcur : p.keys[jk];
          if (kk >= K) {
            st |= 2u;
            continue;
          }
          if (PF && jk == kb) {  // the first key's entry row came with the header
            const KeyRefs q = key_refs(p, s, kk);
            if (stale) grp::load_row<KJ>(e, q.ec, g, A);
            gkey_rm_row<KJ>(p, q, e, oc, g, lane);
          } else {
            gkey_rm<KJ>(p, s, kk, oc, g, lane);
          }
          touch(kk);
        }
        const unsigned wr = grp::witness<KJ>(oc, c, g, 0, A);
        if (wr == grp::kNone) continue;  // rm <= clock: not deferred (:336-345)
        int slot = -1;
        for (unsigned d = 0; d < dcnt; ++d) {
          if (wit[d] != wr) continue;
          u64 x[KJ];
          grp::load_row<KJ>(x, DC + d * A, g, A);
          if (grp::rows_eq<KJ>(x, oc, lane)) {
            slot = (int)d;
            break;
          }
        }
        if (slot < 0) {
          if (dcnt >= Dcap) {
            st |= 1u;
            continue;
          }
          slot = (int)dcnt++;
          grp::store_row<KJ>(DC + (unsigned long long)slot * A, oc, g, A);
          // a one-key Rm's bit goes in with the zeros (no read-modify-write behind the stores)
          const unsigned long long k1 = ke == kb + 1 ? (PF ? (unsigned long long)kcur : p.keys[kb]) : ~0ull;
          const unsigned long long wk = k1 < K ? k1 / 64 : ~0ull;
          for (unsigned long long x = g; x < Kw; x += kG) DK[slot * Kw + x] = x == wk ? 1ull << (k1 % 64) : 0ull;
          if (lead) wit[slot] = (uint8_t)wr;
          if (MT && lead) sbl[slot] = k1 < K ? 1ull << (k1 % 64) : 0ull;
          W |= 1ull << wr;
          if (ke == kb + 1) {
            if (k1 < K) bloom |= 1ull << (k1 % 64);
            continue;
          }
        }
        for (u64 jk = kb; jk < ke; ++jk) {
          const unsigned long long kk = PF && jk == kb ? kcur : p.keys[jk];
          if (kk >= K) continue;
          if (lead) DK[slot * Kw + kk / 64] |= 1ull << (kk % 64);
          if (MT && lead) sbl[slot] |= 1ull << (kk % 64);
          bloom |= 1ull << (kk % 64);
        }
      }
    }
  }
  grp::store_row<KJ>(Cg, c, g, A);
  if (lead) {
    p.def_count[s] = dcnt;
    p.status[s] = st;
  }
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_map_apply_batch(crdt_ctx *ctx, const crdt_map_states *m, uint64_t *def_clock, uint64_t *def_keys,
                                    uint32_t *def_count, size_t Dcap, const crdt_map_ops *ops, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!m || !ops || !status) return fail(ctx, CRDT_EINVAL, "map_apply_batch: NULL argument");
  const size_t N = m->N, K = m->K, A = m->A, V = m->V;
  if (N == 0) return CRDT_OK;
  if (A == 0 || V == 0 || K == 0) return fail(ctx, CRDT_EINVAL, "map_apply_batch: need A, V, K >= 1");
  if (A > (size_t)(kMAWide * kWave))
    return fail(ctx, CRDT_EUNSUPPORTED, "map_apply_batch: A = %zu > %d actors", A, kMAWide * kWave);
  if (!m->clock || !m->ec || !m->vclk || !m->vval || !def_count || !ops->op_off)
    return fail(ctx, CRDT_EINVAL, "map_apply_batch: NULL buffer");
  if (Dcap && (!def_clock || !def_keys)) return fail(ctx, CRDT_EINVAL, "map_apply_batch: NULL deferred buffers");
  if (ops->n_ops && (!ops->kind || !ops->clk_row || !ops->clk_pool))
    return fail(ctx, CRDT_EINVAL, "map_apply_batch: NULL op buffer");
  if (m->clock_stride < A || m->ec_stride < K * A || m->vclk_stride < K * V * A || m->vval_stride < K * V)
    return fail(ctx, CRDT_EINVAL, "map_apply_batch: stride smaller than the rows it holds");
  const size_t Kw = (K + 63) / 64;
  // deferred slots in LDS: all of them when they fit (tune mhot caps them), else as many as 64 KiB
  // holds, down to none; the rest stay in the state's own HBM slots
  const size_t lds_cap = 64 * 1024;
  const size_t slot_b = (A + Kw) * 8;
  size_t Dh = Dcap < (size_t)ctx->tune.map_apply_hot ? Dcap : (size_t)ctx->tune.map_apply_hot;
  if (Dh * slot_b > lds_cap) Dh = lds_cap / slot_b;
  const size_t per_wave = Dh * slot_b;
  int wpb = kBlock / kWave;
  while (wpb > 1 && per_wave * wpb > lds_cap) --wpb;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  MapApplyPlan p{(u64 *)m->clock, m->clock_stride, (u64 *)m->ec, m->ec_stride, (u64 *)m->vclk, m->vclk_stride,
                 (u64 *)m->vval, m->vval_stride, (u64 *)def_clock, (u64 *)def_keys, def_count, N, K, A, V, Kw, Dcap,
                 (const u64 *)ops->op_off, ops->kind, ops->actor, (const u64 *)ops->counter, ops->key,
                 (const u64 *)ops->val, ops->clk_row, (const u64 *)ops->clk_pool, ops->n_clk_rows,
                 (const u64 *)ops->key_off, ops->keys, ops->keys ? ops->n_keys : 0, ops->n_ops, status, wpb, Dh,
                 ctx->tune.apply_fence};
  if (ctx->tune.apply_lane && A <= (size_t)kWave && Dcap <= 2048) {
    // 16 lanes per state: kBlock / 16 states per block (KJ = ceil(A / 16) clock words per lane)
    const size_t per_block = kBlock / grp::kG;
    const dim3 g2((unsigned)((N + per_block - 1) / per_block)), b2(kBlock);
    const bool pf = ctx->tune.map_apply_pf;
    // MT: the slots' key blooms in LDS (with PF; CRDT_TUNE mameta=0: the round-4 form, HBM only)
    const bool mt = pf && ctx->tune.map_apply_meta && Dcap <= kMapMetaSlots;
    const size_t lds2 = per_block * 6 * grp::kG * 8 + (per_block * Dcap + 7) / 8 * 8 + (mt ? per_block * Dcap * 8 : 0);
    timing_begin(ctx, "map_apply");
    auto pick = [&](auto m, auto mf, auto nf) { return mt ? m : pf ? mf : nf; };
    if (A <= 16)
      hipLaunchKernelGGL(pick(map_apply_grp_kernel<1, true, true>, map_apply_grp_kernel<1, true, false>,
                              map_apply_grp_kernel<1, false, false>), g2, b2, lds2, ctx->stream, p);
    else if (A <= 32)
      hipLaunchKernelGGL(pick(map_apply_grp_kernel<2, true, true>, map_apply_grp_kernel<2, true, false>,
                              map_apply_grp_kernel<2, false, false>), g2, b2, lds2, ctx->stream, p);
    else
      hipLaunchKernelGGL(pick(map_apply_grp_kernel<4, true, true>, map_apply_grp_kernel<4, true, false>,
                              map_apply_grp_kernel<4, false, false>), g2, b2, lds2, ctx->stream, p);
    timing_end(ctx);
    CRDT_HIP(ctx, hipGetLastError());
    return CRDT_OK;
  }
  const unsigned long long want = (N + wpb - 1) / wpb;
  const unsigned long long cap = (unsigned long long)ctx->cu_count * 64;
  timing_begin(ctx, "map_apply");
  const dim3 grid((unsigned)(want < cap ? want : cap)), block(wpb * kWave);
  const bool sp = Dh < Dcap;
  if (A <= (size_t)kWave)
    hipLaunchKernelGGL((sp ? map_apply_kernel_w1<true> : map_apply_kernel_w1<false>), grid, block, per_wave * wpb,
                       ctx->stream, p);
  else if (A <= (size_t)(2 * kWave))
    hipLaunchKernelGGL((sp ? map_apply_kernel<2, true> : map_apply_kernel<2, false>), grid, block, per_wave * wpb,
                       ctx->stream, p);
  else if (A <= (size_t)(kMA * kWave))
    hipLaunchKernelGGL((sp ? map_apply_kernel<kMA, true> : map_apply_kernel<kMA, false>), grid, block,
                       per_wave * wpb, ctx->stream, p);
  else if (A <= (size_t)(8 * kWave))  // wide states: more clock words per lane (a correctness path)
    hipLaunchKernelGGL((sp ? map_apply_kernel<8, true> : map_apply_kernel<8, false>), grid, block, per_wave * wpb,
                       ctx->stream, p);
  else
    hipLaunchKernelGGL((sp ? map_apply_kernel<kMAWide, true> : map_apply_kernel<kMAWide, false>), grid, block,
                       per_wave * wpb, ctx->stream, p);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}
