// Map<K, GCounter> / Map<K, PNCounter> lub_many (round 4): Map::merge (map.rs:140-220) with a
// counter value — GCounter (gcounter.rs:44-54: merge = the VClock max, forget = VClock::forget) or
// PNCounter (pncounter.rs:70-82: P and N each).  The fold acc = Map::new(); for r: acc.merge(r) is
// not associative for these values either (tree vs left fold differ on op-replay histories, as for
// MVReg), so, as map.hip does, each key is folded in replica order — exact for ANY
// input.  Keys are independent given the prefix max of the replica clocks C and the deferred
// removes, so one wave folds one (group, key), lane = actor (APL actors per lane), and the votes
// the reference makes over a whole clock (dominance, emptiness, rm <= C) are ballots.
//
// Step r (replica r of the group: clock c2, entry clock e2, value rows v2) on the key's state
// (C, e, v):  the entry join of map.rs:142-210, then the forgets of apply_keyset_rm /
// apply_deferred (map.rs:213-219, :311-348) — replica r's own removes naming the key, and every
// earlier remove naming it that was still deferred after step r-1 — then C |= c2, and a remove
// stays deferred while !(rm <= C).  Forgets commute and compose by max, so the step applies one
// forget by the max of those removes; the entry is dropped (clock and value 0) when its clock
// empties.  Replica rows are loaded DEPTH steps ahead into a register ring; the removes naming the
// key are gathered from the group's pool into LDS in replica order, and the live ones keep their rm
// rows in LDS (beyond that, re-read from HBM: correct, slower).
#include "common.hpp"

namespace crdt {

constexpr int kMcWaves = 4;    // key waves per workgroup
constexpr int kMcList = 256;   // removes naming the key, gathered per window (row << 32 | index)
constexpr int kMcLive = 512;   // live removes (pool index) per key
constexpr int kMcRowsB = 8192; // bytes of live rm rows cached in LDS per wave

struct MapCounterPlan {
  const u64 *clock, *ec, *val;
  unsigned long long c_rs, c_gs, e_rs, e_gs, v_rs, v_gs;
  unsigned long long G, R, K, A, Kw;
  const size_t *def_off;  // device copy (G+1), or null: no removes
  const uint32_t *def_row;
  const u64 *def_clock, *def_keys;
  u64 *o_clock, *o_ec, *o_val;
  unsigned *o_flags;
};

template <int APL>
__device__ __forceinline__ bool mc_any(const u64 (&x)[APL], const u64 (&y)[APL]) {  // some x[a] > y[a]
  bool b = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) b |= x[j] > y[j];
  return __ballot(b) != 0;
}
template <int APL>
__device__ __forceinline__ bool mc_nz(const u64 (&x)[APL]) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) b |= x[j] != 0;
  return __ballot(b) != 0;
}

template <int APL, int W>
__global__ __launch_bounds__(kMcWaves * kWave) void map_counter_fold_kernel(MapCounterPlan p) {
  constexpr int DEPTH = APL >= 8 ? 1 : 8 / APL;    // replica steps in flight (16 at APL 1 ran slower:
                                                   // 20.0 vs 12.9 ms, probably the unrolled body's size)
  constexpr int NROW = kMcRowsB / (8 * kWave * APL);  // live rm rows cached in LDS
  extern __shared__ u64 lds[];
  const int lane = (int)(threadIdx.x % kWave), wv = (int)(threadIdx.x / kWave);
  const unsigned long long gk = (unsigned long long)blockIdx.x * kMcWaves + wv;
  if (gk >= p.G * p.K) return;  // (whole waves; nothing below synchronises the workgroup)
  const unsigned long long g = gk / p.K, k = gk % p.K, A = p.A, R = p.R;
  u64 *lst = lds + (unsigned long long)wv * (kMcList + kMcLive / 2 + NROW * kWave * APL);
  uint32_t *live = reinterpret_cast<uint32_t *>(lst + kMcList);
  u64 *rows = lst + kMcList + kMcLive / 2;  // [NROW][APL][64]

  // Loads are never EXEC-masked: lanes past A read the row's last word and zero it after (a masked
  // load puts the wait counter's bookkeeping on branches, and the compiler then drains every
  // outstanding load — the replica ring's prefetch included — at the join).
  auto ld_row = [&](u64 (&x)[APL], const u64 *src) {
#pragma unroll
    for (int j = 0; j < APL; ++j) {
      const unsigned long long a = (unsigned long long)lane + (unsigned long long)kWave * j;
      const u64 t = src[a < A ? a : A - 1];
      x[j] = a < A ? t : 0ull;
    }
  };

  // ---- the removes naming key k, in replica order (windows of kMcList)
  const unsigned long long d0 = p.def_off ? p.def_off[g] : 0, d1 = p.def_off ? p.def_off[g + 1] : 0;
  unsigned long long dc = d0;  // next pool entry to scan
  int nl = 0, li = 0;          // window length / next entry
  bool bad = false;            // def_row not non-decreasing or >= R (flags bit 1)
  u64 last_row = 0;
  auto refill = [&]() {
    nl = 0;
    li = 0;
    while (dc < d1 && nl + kWave <= kMcList) {
      const unsigned long long d = dc + lane;
      bool hit = false;
      u64 row = 0;
      if (d < d1) {
        row = p.def_row[d];
        hit = (p.def_keys[d * p.Kw + k / 64] >> (k % 64)) & 1ull;
      }
      const u64 prev = __shfl_up(row, 1);
      bool b = d < d1 && (row >= R || (lane == 0 ? row < last_row : row < prev));
      if (__ballot(b)) bad = true;
      const unsigned long long n = d1 - dc < (unsigned long long)kWave ? d1 - dc : kWave;
      last_row = __shfl(row, (int)n - 1);
      const u64 m = __ballot(hit);
      if (hit) lst[nl + __popcll(m & ((1ull << lane) - 1))] = (row << 32) | (u64)(d - d0);
      nl += __popcll(m);
      dc += n;
    }
  };
  u64 nxt = ~0ull;  // replica row of lst[li], the next remove naming k (~0: none left)
  auto advance = [&]() {
    for (;;) {
      if (li < nl) {
        nxt = lst[li] >> 32;
        return;
      }
      if (dc >= d1) {
        nxt = ~0ull;
        return;
      }
      refill();
    }
  };
  refill();
  advance();
  bool full = false;  // more than kMcLive live removes on the key (flags bit 3)

  // ---- the live removes (pool indices; the first NROW rows cached in LDS)
  int na = 0;
  auto live_row = [&](int i, u64 (&x)[APL]) {
    if (i < NROW) {
#pragma unroll
      for (int j = 0; j < APL; ++j) x[j] = rows[((unsigned long long)i * APL + j) * kWave + lane];
    } else {
      ld_row(x, p.def_clock + (d0 + live[i]) * A);
    }
  };
  auto put_row = [&](int i, const u64 (&x)[APL]) {
    if (i < NROW) {
#pragma unroll
      for (int j = 0; j < APL; ++j) rows[((unsigned long long)i * APL + j) * kWave + lane] = x[j];
    }
  };
  u64 rk[APL];  // max of the live removes' clocks (the forget every later step applies)
#pragma unroll
  for (int j = 0; j < APL; ++j) rk[j] = 0;

  u64 C[APL], e[APL], v[W][APL];
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    C[j] = 0;
    e[j] = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) v[w][j] = 0;
  }

  // ---- replica rows, DEPTH steps ahead
  u64 c2r[DEPTH][APL], e2r[DEPTH][APL], v2r[DEPTH][W][APL];
  // the lane's word of each row, advanced by one replica stride per step (no per-step multiplies);
  // past the last replica the pointers stay on it (loaded, never used)
  const u64 *pc = p.clock + g * p.c_gs, *pe = p.ec + g * p.e_gs + k * A, *pv = p.val + g * p.v_gs + k * W * A;
  unsigned long long nload = 0;  // replica of the next load_step
  unsigned aj[APL];              // the lane's actor per word, clamped to the row (see ld_row)
  bool inj[APL];
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = (unsigned long long)lane + (unsigned long long)kWave * j;
    inj[j] = a < A;
    aj[j] = (unsigned)(a < A ? a : A - 1);
  }
  auto load_step = [&](int s) {
#pragma unroll
    for (int j = 0; j < APL; ++j) {
      const u64 tc = pc[aj[j]], te = pe[aj[j]];
      c2r[s][j] = inj[j] ? tc : 0ull;
      e2r[s][j] = inj[j] ? te : 0ull;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const u64 tv = pv[w * A + aj[j]];
        v2r[s][w][j] = inj[j] ? tv : 0ull;
      }
    }
    if (++nload < R) {
      pc += p.c_rs;
      pe += p.e_rs;
      pv += p.v_rs;
    }
  };
#pragma unroll
  for (int s = 0; s < DEPTH; ++s) load_step(s);

  for (unsigned long long r0 = 0; r0 < R; r0 += DEPTH) {
#pragma unroll
    for (int s = 0; s < DEPTH; ++s) {
      const unsigned long long r = r0 + s;
      if (r >= R) break;
      const u64(&c2)[APL] = c2r[s];
      const u64(&e2)[APL] = e2r[s];
      // 1. entry join (map.rs:142-210) against the state before this step (clock C)
      const bool p1 = mc_nz<APL>(e), p2 = mc_nz<APL>(e2);
      if (p1 && !p2) {  // :146-161
        if (!mc_any<APL>(e, c2)) {  // other.clock >= entry.clock: dropped
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            e[j] = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) v[w][j] = 0;
          }
        } else {
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            e[j] = e[j] > c2[j] ? e[j] : 0;                 // entry.clock.forget(other.clock)
            const u64 ri = c2[j] > e[j] ? c2[j] : 0;        // removed_information
#pragma unroll
            for (int w = 0; w < W; ++w) v[w][j] = v[w][j] > ri ? v[w][j] : 0;
          }
        }
      } else if (!p1 && p2) {  // :193-208
        if (mc_any<APL>(e2, C)) {  // else self.clock >= entry.clock: not added
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            e[j] = e2[j] > C[j] ? e2[j] : 0;                // entry.clock.forget(self.clock)
            const u64 wd = C[j] > e[j] ? C[j] : 0;          // we_deleted
#pragma unroll
            for (int w = 0; w < W; ++w) v[w][j] = v2r[s][w][j] > wd ? v2r[s][w][j] : 0;
          }
        }
      } else if (p1 && p2) {  // :170-192
        u64 cm[APL];
        bool nz = false;
#pragma unroll
        for (int j = 0; j < APL; ++j) {
          const u64 t0 = e[j] == e2[j] ? e[j] : 0, t1 = e2[j] > C[j] ? e2[j] : 0, t2 = e[j] > c2[j] ? e[j] : 0;
          const u64 t = t0 > t1 ? t0 : t1;
          cm[j] = t > t2 ? t : t2;
          nz |= cm[j] != 0;
        }
        if (!__ballot(nz)) {  // common empty: the key is dropped
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            e[j] = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) v[w][j] = 0;
          }
        } else {
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            const u64 mx = e[j] > e2[j] ? e[j] : e2[j];
            const u64 del = mx > cm[j] ? mx : 0;            // (e1 + e2).forget(common)
#pragma unroll
            for (int w = 0; w < W; ++w) {
              const u64 m = v[w][j] > v2r[s][w][j] ? v[w][j] : v2r[s][w][j];  // val.merge
              v[w][j] = m > del ? m : 0;                                      // val.forget(deleted)
            }
            e[j] = cm[j];
          }
        }
      }
      // 2. this step's forget: replica r's removes naming k (apply_keyset_rm, unconditional) and the
      //    removes still deferred after step r-1 (apply_deferred)
      u64 f[APL];
#pragma unroll
      for (int j = 0; j < APL; ++j) f[j] = rk[j];
      int nnew = 0;
      while (nxt <= r) {  // (a row below r only when def_row is unsorted: flagged)
        const unsigned idx = (unsigned)lst[li];
        u64 rm[APL];
        ld_row(rm, p.def_clock + (d0 + idx) * A);
#pragma unroll
        for (int j = 0; j < APL; ++j) f[j] = f[j] > rm[j] ? f[j] : rm[j];
        if (na < kMcLive) {  // a candidate for the live set (checked against C below)
          if (lane == 0) live[na] = idx;
          put_row(na, rm);
          ++na;
          ++nnew;
        } else {
          full = true;  // (more than kMcLive live removes on one key: reported, never silent)
        }
        ++li;
        advance();
      }
#pragma unroll
      for (int j = 0; j < APL; ++j) {
        e[j] = e[j] > f[j] ? e[j] : 0;
#pragma unroll
        for (int w = 0; w < W; ++w) v[w][j] = v[w][j] > f[j] ? v[w][j] : 0;
      }
      if (!mc_nz<APL>(e)) {  // an entry whose clock emptied is dropped with its value
#pragma unroll
        for (int j = 0; j < APL; ++j)
#pragma unroll
          for (int w = 0; w < W; ++w) v[w][j] = 0;
      }
      // 3. self.clock.merge(other.clock) (:217), then a remove stays deferred while !(rm <= C)
#pragma unroll
      for (int j = 0; j < APL; ++j) C[j] = C[j] > c2[j] ? C[j] : c2[j];
      if (na > 0) {
        bool changed = nnew > 0;
        for (int i = 0; i < na;) {
          u64 rm[APL];
          live_row(i, rm);
          if (mc_any<APL>(rm, C)) {
            ++i;
            continue;
          }
          changed = true;  // dominated: no longer deferred; the last entry moves over it
          const int lastp = na - 1;
          if (i != lastp) {
            u64 x[APL];
            live_row(lastp, x);
            put_row(i, x);
            const unsigned li_last = live[lastp];
            if (lane == 0) live[i] = li_last;
          }
          --na;
        }
        if (changed) {
#pragma unroll
          for (int j = 0; j < APL; ++j) rk[j] = 0;
          for (int i = 0; i < na; ++i) {
            u64 rm[APL];
            live_row(i, rm);
#pragma unroll
            for (int j = 0; j < APL; ++j) rk[j] = rk[j] > rm[j] ? rk[j] : rm[j];
          }
        }
      }
      load_step(s);
    }
  }
  // ---- the key's folded entry, the group's clock (key 0's wave)
  u64 *oe = p.o_ec + gk * A;
  u64 *ov = p.o_val + gk * W * A;
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = (unsigned long long)lane + (unsigned long long)kWave * j;
    if (a < A) {
      oe[a] = e[j];
#pragma unroll
      for (int w = 0; w < W; ++w) ov[w * A + a] = v[w][j];
      if (k == 0) p.o_clock[g * A + a] = C[j];
    }
  }
  if ((bad || full) && lane == 0) atomicOr(p.o_flags + g, (bad ? 2u : 0u) | (full ? 8u : 0u));
}

template <int APL, int W>
static size_t mc_lds() {
  return (size_t)kMcWaves * (kMcList * 8 + kMcLive * 4 + (kMcRowsB / (8 * kWave * APL)) * kWave * APL * 8);
}

template <int APL, int W>
static hipError_t launch_mc(const MapCounterPlan &p, hipStream_t s) {
  const unsigned long long blocks = (p.G * p.K + kMcWaves - 1) / kMcWaves;
  const size_t lds = mc_lds<APL, W>();
  hipLaunchKernelGGL((map_counter_fold_kernel<APL, W>), dim3((unsigned)blocks), dim3(kMcWaves * kWave), lds, s, p);
  return hipGetLastError();
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_map_counter_lub_many(crdt_ctx *ctx, const crdt_map_counter_batch *in,
                                         crdt_map_counter_out *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: NULL batch/out");
  const size_t G = in->G, R = in->R, K = in->K, A = in->A, W = in->W;
  if (W != 1 && W != 2) return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: W = %zu (1 GCounter, 2 PNCounter)", W);
  if (G == 0 || K == 0 || A == 0) return CRDT_OK;
  if (A > 8 * (size_t)kWave) return fail(ctx, CRDT_EUNSUPPORTED, "map_counter_lub_many: A = %zu > %d", A, 8 * kWave);
  if (!out->clock || !out->ec || !out->val || !out->flags)
    return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: NULL output");
  if (R > 0 && (!in->clock || !in->ec || !in->val)) return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: NULL input");
  if (G * K > 0x7fffffffULL * (size_t)kMcWaves || R > 0xfffffffeULL)
    return fail(ctx, CRDT_EUNSUPPORTED, "map_counter_lub_many: G*K or R too large");
  if (in->def_off && in->def_off[0] != 0) return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: def_off[0] must be 0");
  const size_t D = (in->def_off && G > 0) ? in->def_off[G] : 0;
  for (size_t i = 0; in->def_off && i < G; ++i)
    if (in->def_off[i + 1] < in->def_off[i])
      return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: def_off not non-decreasing");
  if (D > 0 && (!in->def_row || !in->def_clock || !in->def_keys || !out->def_keep || !out->def_keys))
    return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: deferred buffers missing");
  if (D > 0xffffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_counter_lub_many: too many deferred");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const size_t Kw = (K + 63) / 64;
  MapCounterPlan p{(const u64 *)in->clock, (const u64 *)in->ec, (const u64 *)in->val, in->clock_rstride,
                   in->clock_gstride, in->ec_rstride, in->ec_gstride, in->val_rstride, in->val_gstride, G, R, K, A,
                   Kw, nullptr, in->def_row, (const u64 *)in->def_clock, (const u64 *)in->def_keys,
                   (u64 *)out->clock, (u64 *)out->ec, (u64 *)out->val, out->flags};
  if (int rc = device_fill(ctx, out->flags, G * sizeof(unsigned), 0)) return rc;
  if (R == 0) {  // fold of nothing: Map::new()
    if (int rc = device_fill(ctx, out->clock, G * A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, out->ec, G * K * A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, out->val, G * K * W * A * 8, 0)) return rc;
  } else {
    if (D > 0) {
      if (int rc = ensure_scratch(ctx, (G + 1) * sizeof(size_t))) return rc;
      if (int rc = stage_h2d(ctx, ctx->scratch, in->def_off, (G + 1) * sizeof(size_t))) return rc;
      p.def_off = reinterpret_cast<const size_t *>(ctx->scratch);
    }
    timing_begin(ctx, "map_counter_fold");
    hipError_t he;
    if (A <= (size_t)kWave) he = W == 1 ? launch_mc<1, 1>(p, ctx->stream) : launch_mc<1, 2>(p, ctx->stream);
    else if (A <= 2 * (size_t)kWave) he = W == 1 ? launch_mc<2, 1>(p, ctx->stream) : launch_mc<2, 2>(p, ctx->stream);
    else if (A <= 4 * (size_t)kWave) he = W == 1 ? launch_mc<4, 1>(p, ctx->stream) : launch_mc<4, 2>(p, ctx->stream);
    else he = W == 1 ? launch_mc<8, 1>(p, ctx->stream) : launch_mc<8, 2>(p, ctx->stream);
    timing_end(ctx);
    if (he != hipSuccess) return hip_fail(ctx, he, "map_counter_fold_kernel launch");
  }
  if (D == 0) return CRDT_OK;
  DefPlan q{};  // survivors (!(rm <= C_final)), identical rm clocks merged: as for crdt_map_lub_many
  q.G = G;
  q.D = D;
  q.M = K;
  q.A = A;
  q.Mw = Kw;
  q.def_clock = (const u64 *)in->def_clock;
  q.def_members = (const u64 *)in->def_keys;
  q.out_clock = (const u64 *)out->clock;
  q.out_entries = nullptr;
  q.apply_ceiling = 0;  // the fold kernel applied every remove at the right step
  q.out_keep = out->def_keep;
  q.out_members = (u64 *)out->def_keys;
  return launch_deferred(ctx, in->def_off, q);
}
