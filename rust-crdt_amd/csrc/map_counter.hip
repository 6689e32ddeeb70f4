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
  // Keys per wave > 1 share one live-remove list of kMcLive entries, so a wave can run out of room
  // while each of its keys holds <= kMcLive live removes.  With rerun_out set, such a
  // wave marks its group in rerun_out instead of flags bit 3; a second launch with one key per wave
  // and rerun_in = that array re-folds exactly the marked groups (every other wave returns at once),
  // so the documented per-key capacity holds whatever the automatic keys-per-wave choice.
  const unsigned *rerun_in;
  unsigned *rerun_out;
};

// MC_AUX (build option): the cache-policy bits of the step-image LDS-DMA (0 default; 2 = nt, as the
// MVReg Map fold's step images since round 6)
#ifndef MC_AUX
#define MC_AUX 0
#endif
__device__ __forceinline__ void glds16_mc(const void *g, u64 *lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)lds, 16, 0, MC_AUX);
}

// votes over the lanes of the caller's key (hm: its lanes' bits; ~0 with one key per wave)
template <int APL>
__device__ __forceinline__ bool mc_any(const u64 (&x)[APL], const u64 (&y)[APL], u64 hm) {  // some x[a] > y[a]
  bool b = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) b |= x[j] > y[j];
  return (__ballot(b) & hm) != 0;
}
template <int APL>
__device__ __forceinline__ bool mc_nz(const u64 (&x)[APL], u64 hm) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) b |= x[j] != 0;
  return (__ballot(b) & hm) != 0;
}

// DMA (APL = 1, (2+W)*A <= 128 words, A even, 16-byte aligned rows): the replica rows of a step
// arrive as ONE 1-KiB LDS-DMA piece (lane l moves words 2l, 2l+1 of the step image [ec | val rows |
// clock]) into a ring of RING slots (8 or 16), waited on with an explicit vmcnt; otherwise
// (RING = 0) a register ring.  (The register ring's loads are register values, and the compiler
// drains them all at the loop's back edge — one memory latency every DEPTH steps; LDS-DMA loads
// it leaves to us.)
// KPW keys per wave (APL = 1, register ring, A <= 64 / KPW): lanes [h*64/KPW, (h+1)*64/KPW) fold
// key kb + h of the group, so a 32-actor key no longer leaves half the wave idle.  The group's
// clock C and a remove's liveness (!(rm <= C)) are the same for every key of the group, so the
// keys share one walk of the remove pool; each entry carries which of the wave's keys it names.
// LDS-staged chunk skip (SPL > 0, CL): chunks of kMcClS steps, each step an image [ec | val_0..W-1 |
// clock] of (2 + W) * A words, moved by 1-KiB global_load_lds pieces into kMcClNB slots per wave.
constexpr int kMcClS = 8, kMcClNB = 4;
template <int W, int SPL>
__host__ __device__ constexpr int mc_cl_pieces() {
  return SPL > 0 ? (kMcClS * (2 + W) * (kWave / (SPL > 0 ? SPL : 1)) + 127) / 128 : 0;
}
template <int W, int SPL>
__host__ __device__ constexpr unsigned long long mc_cl_words() {
  return (unsigned long long)kMcClNB * mc_cl_pieces<W, SPL>() * 128;
}

// SPL > 0 (A == 64 / SPL: 32, 16 or 8 actors; one key per wave, register rows): the whole-chunk
// skip below, with lane l holding actor l % A in every register of the key's state.
template <int APL, int W, int RING, int KPW, int DEP = 8, int SPL = 0, int CL = 0>
__global__ __launch_bounds__(kMcWaves * kWave) void map_counter_fold_kernel(MapCounterPlan p) {
  constexpr bool DMA = RING > 0;
  constexpr int kMcRing = DMA ? RING : 1;
  constexpr int DEPTH = DMA ? 1 : (APL >= 8 ? 1 : DEP / APL);  // register ring: steps in flight (16 at
                                                   // APL 1 ran slower: 20.0 vs 12.9 ms, probably the
                                                   // unrolled body's size)
  static_assert(KPW == 1 || (APL == 1 && !DMA), "several keys per wave: APL 1, register ring");
  static_assert(SPL == 0 || (APL == 1 && KPW == 1 && !DMA), "chunk skip: one key per wave, APL 1, register rows");
  // live rm rows cached in LDS (the LDS-staged chunk skip keeps 4: its chunk slots take the room)
  constexpr int NROW = (SPL > 0 && CL) ? 4 : kMcRowsB / (8 * kWave * APL);
  constexpr int HL = kWave / KPW;                     // lanes per key
  extern __shared__ u64 lds[];
  const int lane = (int)(threadIdx.x % kWave), wv = (int)(threadIdx.x / kWave);
  const int h = lane / HL, al = lane % HL;  // the lane's key of the wave / actor lane
  const u64 hm = KPW == 1 ? ~0ull : (((1ull << HL) - 1) << (h * HL));
  const unsigned long long KW = (p.K + KPW - 1) / KPW;  // waves per group
  const unsigned long long wk = (unsigned long long)blockIdx.x * kMcWaves + wv;
  if (wk >= p.G * KW) return;  // (whole waves; nothing below synchronises the workgroup)
  const unsigned long long g = wk / KW, kb = (wk % KW) * KPW, A = p.A, R = p.R;
  if (p.rerun_in && p.rerun_in[g] == 0) return;  // (the re-fold launch: only the marked groups)
  const unsigned long long k = kb + h;  // the lane's key (past K: a copy of key K-1, not written)
  const bool kval = k < p.K;
  const unsigned long long kc = kval ? k : p.K - 1;
  const unsigned kbits = (unsigned)(p.K - kb < (unsigned long long)KPW ? (1u << (p.K - kb)) - 1 : (1u << KPW) - 1);
  constexpr unsigned long long WQ = kMcList + kMcLive / 2 + NROW * kWave * APL + (DMA ? kMcRing * 128 : 0);
  u64 *lst = lds + (unsigned long long)wv * WQ;
  uint32_t *live = reinterpret_cast<uint32_t *>(lst + kMcList);
  u64 *rows = lst + kMcList + kMcLive / 2;  // [NROW][APL][64]
  u64 *ring = rows + NROW * kWave * APL;    // DMA: [kMcRing][128] step images
  // which of the wave's keys each gathered / live remove names (bit h)
  uint8_t *lmask = reinterpret_cast<uint8_t *>(lds + kMcWaves * WQ) + wv * (kMcList + kMcLive);
  uint8_t *lvm = lmask + kMcList;
  // (SPL > 0, CL: the wave's LDS chunk slots, after every wave's lists; 16-byte aligned)
  u64 *cslots = lds + kMcWaves * WQ + (kMcWaves * (kMcList + kMcLive)) / 8 + (unsigned long long)wv * mc_cl_words<W, SPL>();

  // Loads are never EXEC-masked: lanes past A read the row's last word (a masked load puts the wait
  // counter's bookkeeping on branches, and the compiler then drains every outstanding load — the
  // replica ring's prefetch included — at the join).  Every row a lane holds, remove rows included,
  // is a copy of actor A-1 past A, so those lanes evolve exactly as actor A-1 and never change a vote.
  // (SPL > 0: lane l reads actor l % A, A == 64 / SPL, so every lane holds a real actor)
  auto ld_row = [&](u64 (&x)[APL], const u64 *src) {
#pragma unroll
    for (int j = 0; j < APL; ++j) {
      const unsigned long long a = SPL > 0 ? (unsigned long long)(lane & (kWave / (SPL > 0 ? SPL : 1) - 1))
                                           : (unsigned long long)al + (unsigned long long)HL * j;
      x[j] = src[a < A ? a : A - 1];
    }
  };

  // ---- the removes naming the wave's keys, in replica order (windows of kMcList)
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
      unsigned bits = 0;  // (the wave's keys share one def_keys word: KPW divides 64)
      u64 row = 0;
      if (d < d1) {
        row = p.def_row[d];
        bits = (unsigned)(p.def_keys[d * p.Kw + kb / 64] >> (kb % 64)) & kbits;
      }
      const bool hit = bits != 0;
      const u64 prev = __shfl_up(row, 1);
      bool b = d < d1 && (row >= R || (lane == 0 ? row < last_row : row < prev));
      if (__ballot(b)) bad = true;
      const unsigned long long n = d1 - dc < (unsigned long long)kWave ? d1 - dc : kWave;
      last_row = __shfl(row, (int)n - 1);
      const u64 m = __ballot(hit);
      if (hit) {
        const int at = nl + __popcll(m & ((1ull << lane) - 1));
        lst[at] = (row << 32) | (u64)(d - d0);
        lmask[at] = (uint8_t)bits;
      }
      nl += __popcll(m);
      dc += n;
    }
  };
  unsigned nxt = ~0u;  // replica row of lst[li], the next remove naming one of the keys (~0: none
                       // left; rows < R <= 0xfffffffe)
  auto advance = [&]() {
    for (;;) {
      if (li < nl) {  // (uniform: a scalar, so the per-step test is a scalar compare)
        const u64 x = lst[li] >> 32;
        nxt = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)x);
        return;
      }
      if (dc >= d1) {
        nxt = ~0u;
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
      for (int j = 0; j < APL; ++j) x[j] = rows[((unsigned long long)i * APL + j) * kWave + lane];  // (KPW > 1: each key's lanes hold a copy)
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
  u64 T[APL];   // witness thresholds (see step 3)
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    rk[j] = 0;
    T[j] = ~0ull;
  }

  u64 C[APL], e[APL], v[W][APL];
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    C[j] = 0;
    e[j] = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) v[w][j] = 0;
  }

  // ---- replica rows
  unsigned aj[APL];  // the lane's actor per word, clamped to the row (see ld_row)
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = SPL > 0 ? (unsigned long long)(lane & (kWave / (SPL > 0 ? SPL : 1) - 1))
                                         : (unsigned long long)al + (unsigned long long)HL * j;
    aj[j] = (unsigned)(a < A ? a : A - 1);
  }
  // Each live remove keeps a witness: an actor whose rm word is still above C.  T holds, per lane
  // word, the least rm word among the removes witnessed there; while no C word reached its T, no
  // live remove can have become dominated (C only grows), and the scan is skipped.  (chg: removes
  // joined the live set this step.)
  auto liveness = [&](bool chg) {
    {
      bool b = false;  // (no live removes: every T word is ~0, no vote)
#pragma unroll
      for (int j = 0; j < APL; ++j) b |= C[j] >= T[j];
      if (chg || __ballot(b) != 0) {
        bool changed = chg;
#pragma unroll
        for (int j = 0; j < APL; ++j) T[j] = ~0ull;
        for (int i = 0; i < na;) {
          u64 rm[APL];
          live_row(i, rm);
          bool wit = false;  // (every key's lanes hold rm and C: one vote)
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            const u64 m = __ballot(rm[j] > C[j]);
            if (m && !wit) {
              wit = true;
              const int wl = __builtin_ctzll(m);
              T[j] = lane == wl && rm[j] < T[j] ? rm[j] : T[j];
            }
          }
          if (wit) {
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
            const uint8_t lm_last = lvm[lastp];
            if (lane == 0) {
              live[i] = li_last;
              lvm[i] = lm_last;
            }
          }
          --na;
        }
        if (changed) {
#pragma unroll
          for (int j = 0; j < APL; ++j) rk[j] = 0;
          for (int i = 0; i < na; ++i) {
            u64 rm[APL];
            live_row(i, rm);
            const bool named = (lvm[i] >> h) & 1u;
#pragma unroll
            for (int j = 0; j < APL; ++j) rk[j] = named && rm[j] > rk[j] ? rm[j] : rk[j];
          }
        }
      }
    }
  };
  // one replica step on the key's state.  Lanes past A hold copies of actor A-1 (clamped loads;
  // every operation is lane-local), so they never change a vote and need no masking.
  //
  // The entry join is branch-free.  With forget(x, c)[a] = x[a] > c[a] ? x[a] : 0, the joined
  // entry clock is, in all four presence cases (map.rs:146-161, :170-192, :193-208, absent both),
  //     e' = max(e == e2 ? e : 0, forget(e2, C), forget(e, c2))
  // (the "common" clock of :174-178 — it reduces to forget(e, c2) when the replica has no entry,
  // to forget(e2, C) when we have none, and is empty exactly when the reference drops the key),
  // and the value is forget(max(v, v2), forget(Y, e')) with Y = c2 (removed_information, :151),
  // C (we_deleted, :200) or max(e, e2) (deleted, :185) by case.  An entry whose clock is empty
  // keeps a stale value row, ignored (read as 0) from then on: the next step masks v by the same
  // presence vote it needs anyway, and the final rows are masked once.  Two votes per step, both
  // on the step's inputs.
  auto step = [&](unsigned long long r, const u64 (&c2)[APL], const u64 (&e2)[APL], const u64 (&v2)[W][APL]) {
    // 1. entry join (map.rs:142-210) against the state before this step (clock C)
    const bool p1 = mc_nz<APL>(e, hm), p2 = mc_nz<APL>(e2, hm);
#pragma unroll
    for (int j = 0; j < APL; ++j) {
      // (where e == e2 the common clock is e itself: the two forgets are at most e there)
      const u64 t1 = e2[j] > C[j] ? e2[j] : 0, t2 = e[j] > c2[j] ? e[j] : 0;
      const u64 en = e[j] == e2[j] ? e[j] : (t1 > t2 ? t1 : t2);
      const u64 mx = e[j] > e2[j] ? e[j] : e2[j];
      const u64 y = p1 ? (p2 ? mx : c2[j]) : C[j];
      const u64 x = y > en ? y : 0;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const u64 a1 = p1 ? v[w][j] : 0, a2 = p2 ? v2[w][j] : 0;
        const u64 m = a1 > a2 ? a1 : a2;  // val.merge
        v[w][j] = m > x ? m : 0;          // val.forget
      }
      e[j] = en;
    }
    // 2. this step's forget: replica r's removes naming k (apply_keyset_rm, unconditional) and the
    //    removes still deferred after step r-1 (apply_deferred, rk: 0 when there are none, so the
    //    common step applies it without a branch)
    bool chg = false;  // removes joined the live set this step
    u64 f[APL];
#pragma unroll
    for (int j = 0; j < APL; ++j) f[j] = rk[j];
    const unsigned r32 = (unsigned)r;
    if (nxt <= r32) {  // (a row below r only when def_row is unsorted: flagged)
      do {
        const unsigned idx = (unsigned)lst[li];
        const unsigned bits = lmask[li];
        const bool named = (bits >> h) & 1u;
        u64 rm[APL];
        ld_row(rm, p.def_clock + (d0 + idx) * A);
#pragma unroll
        for (int j = 0; j < APL; ++j) f[j] = named && rm[j] > f[j] ? rm[j] : f[j];
        if (na < kMcLive) {  // a candidate for the live set (checked against C below)
          if (lane == 0) {
            live[na] = idx;
            lvm[na] = (uint8_t)bits;
          }
          put_row(na, rm);
          ++na;
          chg = true;
        } else {
          full = true;  // (more than kMcLive live removes on one key: reported, never silent)
        }
        ++li;
        advance();
      } while (nxt <= r32);
    }
#pragma unroll
    for (int j = 0; j < APL; ++j) {
      e[j] = e[j] > f[j] ? e[j] : 0;
#pragma unroll
      for (int w = 0; w < W; ++w) v[w][j] = v[w][j] > f[j] ? v[w][j] : 0;
    }
    // 3. self.clock.merge(other.clock) (:217), then a remove stays deferred while !(rm <= C)
#pragma unroll
    for (int j = 0; j < APL; ++j) C[j] = C[j] > c2[j] ? C[j] : c2[j];
    liveness(chg);
  };
  if constexpr (SPL > 0 && CL) {
    // ---- whole-chunk skip, LDS-staged (round 5, opt-in: CRDT_TUNE mccl=1).  The test and the
    // per-step verdicts are the register path's below; the chunks come by LDS-DMA instead of into
    // registers.  A register still pending at the chunk loop's back-edge makes the compiler drain
    // every load there (vmcnt(0)), so the register path keeps about one chunk in flight; LDS-DMA
    // writes no register, and the fold waits for a chunk with a counted vmcnt, keeping
    // kMcClNB - 1 chunks in flight.  Measured slower all the same (profiles/r05_map_counter_cl_ab.log).
    constexpr int S = kMcClS, NE = S / SPL, NB = kMcClNB, P = mc_cl_pieces<W, SPL>();
    constexpr unsigned long long AA = kWave / SPL;      // == A
    constexpr unsigned long long IMG = (2 + W) * AA;    // words per step image
    const int hh = lane / (int)AA;
    const unsigned a = (unsigned)lane & (unsigned)(AA - 1);
    const unsigned long long nch = (R + S - 1) / S;
    // lane l's 16-byte piece j: image word o = j*128 + 2l of the chunk, i.e. step o / IMG, row
    // (o % IMG) / A (0: ec, 1..W: val, 1+W: clock), actors (o % A, +1); source row bases as values
    // (a per-lane choice between struct fields would be lowered as a dynamic-offset load)
    const unsigned long long be = (unsigned long long)(p.ec + g * p.e_gs + k * AA),
                             bv = (unsigned long long)(p.val + g * p.v_gs + k * W * AA),
                             bcl = (unsigned long long)(p.clock + g * p.c_gs);
    const unsigned long long se = (unsigned long long)p.e_rs * 8, sv = (unsigned long long)p.v_rs * 8,
                             sc = (unsigned long long)p.c_rs * 8;
    unsigned long long pb[P], ps[P];
    unsigned pst[P];
    bool pon[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const unsigned long long o = (unsigned long long)j * 128 + 2ull * lane;
      const unsigned long long st = o / IMG, q = o % IMG, row = q / AA, col = q % AA;
      pon[j] = o < (unsigned long long)S * IMG;
      pst[j] = (unsigned)st;
      pb[j] = row == 0 ? be + col * 8 : (row <= W ? bv + ((row - 1) * AA + col) * 8 : bcl + col * 8);
      ps[j] = row == 0 ? se : (row <= W ? sv : sc);
    }
    auto issue = [&](auto B, unsigned long long c) {  // chunk c into slot B (past R: row R-1 again)
      constexpr int b = decltype(B)::value;
      u64 *slot = cslots + (unsigned long long)b * P * 128;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        unsigned long long rr = c * S + pst[j];
        rr = rr < R ? rr : R - 1;
        if (pon[j]) glds16_mc(reinterpret_cast<const void *>(pb[j] + rr * ps[j]), slot + j * 128);
      }
    };
    auto wait_chunk = [&](unsigned long long c) {  // chunk c has landed: later chunks may be in flight
      const unsigned long long later = nch - 1 - c < (unsigned long long)(NB - 1) ? nch - 1 - c : NB - 1;
      if (later >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * P > 63 ? 63 : 3 * P) : "memory");
      else if (later == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P) : "memory");
      else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    auto test_chunk = [&](const u64 *slot) -> bool {
      // (every element read first, then one branch-free test: a read inside a short-circuit would
      // put each on its own EXEC-masked branch with its own wait)
      u64 qe[NE], qc[NE], qv[W][NE];
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const u64 *img = slot + (i * SPL + hh) * IMG;
        qe[i] = img[a];
        qc[i] = img[(1 + W) * AA + a];
#pragma unroll
        for (int w = 0; w < W; ++w) qv[w][i] = img[(1 + w) * AA + a];
      }
      const u64 e0 = e[0], C0 = C[0];
      if (!mc_nz<1>(e, ~0ull)) {
        u64 okm = ~0ull;
#pragma unroll
        for (int i = 0; i < NE; ++i) okm &= __ballot(qe[i] <= C0);
        return okm == ~0ull;
      }
      const u64 em1 = e0 ? e0 - 1 : 0;
      const u64 TE = e0 ? em1 : ~0ull, TB = C0 > em1 ? C0 : em1;
      u64 TV = ~0ull;
      bool vz[W];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const u64 vw = v[w][0];
        vz[w] = vw == 0;
        const u64 t = vz[w] ? ~0ull : (e0 > vw - 1 ? e0 : vw - 1);
        TV = t < TV ? t : TV;
      }
      const u64 TN = TE < TV ? TE : TV;
      u64 fail = 0;
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const u64 e2 = qe[i], c2 = qc[i];
        const u64 x = e2 > e0 ? e2 : 0;
        bool cb = ((e2 == e0) | ((c2 <= TE) & (e2 <= TB))) & (e2 <= TV);
#pragma unroll
        for (int w = 0; w < W; ++w) cb = cb & (qv[w][i] <= (vz[w] ? x : v[w][0]));
        const u64 mN = __ballot(e2 != 0), mB = __ballot(cb), mO = __ballot(c2 <= TN);
#pragma unroll
        for (int s2 = 0; s2 < SPL; ++s2) {
          const u64 M = (AA == 64 ? ~0ull : ((1ull << AA) - 1)) << (s2 * AA);
          const u64 sel = (mN & M) ? mB : mO;
          fail |= ~sel & M;
        }
      }
      return fail == 0;
    };
    auto body = [&](auto B, unsigned long long c) {
      constexpr int b = decltype(B)::value;
      if (c >= nch) return;
      if (c + NB - 1 < nch) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // chunk c-1's slot is read: refill it
        issue(std::integral_constant<int, (b + NB - 1) % NB>{}, c + NB - 1);
      }
      wait_chunk(c);
      const u64 *slot = cslots + (unsigned long long)b * P * 128;
      const unsigned long long r0 = c * S;
      const unsigned long long n = R - r0 < (unsigned long long)S ? R - r0 : S;
      if (n == S && (unsigned long long)nxt >= r0 + S && test_chunk(slot)) {
        u64 cm = 0;
#pragma unroll
        for (int i = 0; i < NE; ++i) {
          const u64 c2 = slot[(i * SPL + hh) * IMG + (1 + W) * AA + a];
          cm = c2 > cm ? c2 : cm;
        }
#pragma unroll
        for (int off = (int)AA; off < kWave; off <<= 1) {
          const u64 o = __shfl_xor(cm, off);
          cm = o > cm ? o : cm;
        }
        C[0] = C[0] > cm ? C[0] : cm;
        liveness(false);
        return;
      }
      for (int s2 = 0; s2 < (int)n; ++s2) {  // the chunk's steps, exactly (lane = actor a: its words)
        const u64 *img = slot + (unsigned long long)s2 * IMG;
        u64 c2[1], e2[1], v2[W][1];
        e2[0] = img[a];
        c2[0] = img[(1 + W) * AA + a];
#pragma unroll
        for (int w = 0; w < W; ++w) v2[w][0] = img[(1 + w) * AA + a];
        step(r0 + s2, c2, e2, v2);
      }
    };
#pragma unroll
    for (int b = 0; b + 1 < NB; ++b)
      if ((unsigned long long)b < nch) {
        if (b == 0) issue(std::integral_constant<int, 0>{}, 0);
        if (b == 1) issue(std::integral_constant<int, 1>{}, 1);
        if (b == 2) issue(std::integral_constant<int, 2>{}, 2);
      }
    for (unsigned long long c = 0; c < nch; c += NB) {
      body(std::integral_constant<int, 0>{}, c);
      body(std::integral_constant<int, 1>{}, c + 1);
      body(std::integral_constant<int, 2>{}, c + 2);
      body(std::integral_constant<int, 3>{}, c + 3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (no piece lands after the wave ends)
  } else if constexpr (SPL > 0) {
    // ---- whole-chunk skip (round 5).  Almost every replica step of a long fold leaves the key's
    // (entry clock, value) unchanged (config-4 shape: ~7 of 16,384 steps change it), and a step's
    // no-change test needs only the state, not the steps before it, once the state is assumed
    // unchanged.  Chunks of S = 16 steps come into registers in a transposed layout — lane
    // (hh, a) = (lane / A, lane % A) holds, in element i, actor a of step i*SPL + hh, so a 32-actor
    // key uses all 64 lanes (two steps per instruction) — and are tested against the state at the
    // chunk's start.  By induction every step of a chunk that passes leaves the state unchanged, so
    // the chunk only merges its clocks (C |= its clock max) and re-tests the live removes once at
    // its end (liveness only shrinks the forget rk, whose re-application is the identity on a state
    // already forgotten by it).  A chunk holding a remove that names the key, a partial last chunk
    // or a failed test runs its steps exactly.
    //
    // The per-element test, with the state (e, v_w, C0 = C at the chunk's start) and the step's
    // (c2, e2, v2_w), derived from the exact join above (en == e and the value unchanged):
    //   the acc holds the key (p1) and the step's replica too (p2):
    //     (e2 == e || (c2 <= TE && e2 <= TB)) && e2 <= TV && v2_w <= (v_w ? v_w : x)   for every w
    //     with TE = e ? e-1 : MAX (e == 0 or c2 < e), TB = max(C0, e ? e-1 : 0) (e2 < e or e2 <= C),
    //     x = e2 > e ? e2 : 0 (the case's forget word) and TV = min_w (v_w ? max(e, v_w - 1) : MAX)
    //     (the kept value survives x);
    //   p1 without p2:  c2 <= min(TE, TV)  (the entry survives forget(e, c2); the value forget(.., x = c2 > e ? c2 : 0));
    //   no p1:          e2 <= C0 (the replica's entry is not added: forget(e2, C) is empty).
    // C only grows, so testing against C0 is sound; tests/test_map_counter_chunk_model.py checks the
    // test against the exact join on op-replay, arbitrary and synthetic states.
    constexpr int S = 16, NE = S / SPL, NB = W == 1 ? 4 : 3;
    constexpr unsigned long long AA = kWave / SPL;  // == A
    const int hh = lane / (int)AA;
    const unsigned a = (unsigned)lane & (unsigned)(AA - 1);
    const u64 *bc = p.clock + g * p.c_gs + a, *be = p.ec + g * p.e_gs + k * AA + a,
              *bv = p.val + g * p.v_gs + k * W * AA + a;
    const unsigned long long nch = (R + S - 1) / S;
    u64 qc[NB][NE], qe[NB][NE], qv[NB][W][NE];
    auto load_chunk = [&](auto B, unsigned long long c) {
      constexpr int b = decltype(B)::value;
      const unsigned long long r0 = c * S;
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        unsigned long long rr = r0 + (unsigned long long)(i * SPL + hh);
        rr = rr < R ? rr : R - 1;  // (past the last replica: its row again, never used)
        qc[b][i] = bc[rr * p.c_rs];
        qe[b][i] = be[rr * p.e_rs];
#pragma unroll
        for (int w = 0; w < W; ++w) qv[b][w][i] = bv[rr * p.v_rs + w * AA];
      }
    };
    auto test_chunk = [&](auto B) -> bool {
      constexpr int b = decltype(B)::value;
      const u64 e0 = e[0], C0 = C[0];
      if (!mc_nz<1>(e, ~0ull)) {  // the acc lacks the key: no replica of the chunk may add it
        u64 okm = ~0ull;
#pragma unroll
        for (int i = 0; i < NE; ++i) okm &= __ballot(qe[b][i] <= C0);
        return okm == ~0ull;
      }
      const u64 em1 = e0 ? e0 - 1 : 0;
      const u64 TE = e0 ? em1 : ~0ull, TB = C0 > em1 ? C0 : em1;
      u64 TV = ~0ull;
      bool vz[W];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const u64 vw = v[w][0];
        vz[w] = vw == 0;
        const u64 t = vz[w] ? ~0ull : (e0 > vw - 1 ? e0 : vw - 1);
        TV = t < TV ? t : TV;
      }
      const u64 TN = TE < TV ? TE : TV;
      u64 fail = 0;
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const u64 e2 = qe[b][i], c2 = qc[b][i];
        const u64 x = e2 > e0 ? e2 : 0;
        bool cb = (e2 == e0 || (c2 <= TE && e2 <= TB)) && e2 <= TV;
#pragma unroll
        for (int w = 0; w < W; ++w) cb = cb && qv[b][w][i] <= (vz[w] ? x : v[w][0]);
        const u64 mN = __ballot(e2 != 0), mB = __ballot(cb), mO = __ballot(c2 <= TN);
#pragma unroll
        for (int s2 = 0; s2 < SPL; ++s2) {
          const u64 M = (AA == 64 ? ~0ull : ((1ull << AA) - 1)) << (s2 * AA);
          const u64 sel = (mN & M) ? mB : mO;
          fail |= ~sel & M;
        }
      }
      return fail == 0;
    };
    auto body = [&](auto B, unsigned long long c) {
      constexpr int b = decltype(B)::value;
      if (c >= nch) return;
      if (c + NB - 1 < nch) load_chunk(std::integral_constant<int, (b + NB - 1) % NB>{}, c + NB - 1);
      const unsigned long long r0 = c * S;
      const unsigned long long n = R - r0 < (unsigned long long)S ? R - r0 : S;
      const bool skip = n == S && (unsigned long long)nxt >= r0 + S && test_chunk(B);
      if (skip) {
        u64 cm = 0;
#pragma unroll
        for (int i = 0; i < NE; ++i) cm = qc[b][i] > cm ? qc[b][i] : cm;
#pragma unroll
        for (int off = (int)AA; off < kWave; off <<= 1) {
          const u64 o = __shfl_xor(cm, off);
          cm = o > cm ? o : cm;
        }
        C[0] = C[0] > cm ? C[0] : cm;
        liveness(false);
        return;
      }
      for (int s2 = 0; s2 < (int)n; ++s2) {  // the chunk's steps, exactly (a step's rows moved into
        const int i = s2 / SPL, src = (s2 % SPL) * (int)AA + (int)a;  // the lane = actor layout)
        u64 c2[1] = {0}, e2[1] = {0}, v2[W][1];
#pragma unroll
        for (int w = 0; w < W; ++w) v2[w][0] = 0;
#pragma unroll
        for (int ii = 0; ii < NE; ++ii) {
          if (ii == i) {
            c2[0] = qc[b][ii];
            e2[0] = qe[b][ii];
#pragma unroll
            for (int w = 0; w < W; ++w) v2[w][0] = qv[b][w][ii];
          }
        }
        c2[0] = __shfl(c2[0], src);
        e2[0] = __shfl(e2[0], src);
#pragma unroll
        for (int w = 0; w < W; ++w) v2[w][0] = __shfl(v2[w][0], src);
        step(r0 + s2, c2, e2, v2);
      }
    };
#pragma unroll
    for (int b = 0; b + 1 < NB; ++b)
      if ((unsigned long long)b < nch) {
        if (b == 0) load_chunk(std::integral_constant<int, 0>{}, 0);
        if (b == 1) load_chunk(std::integral_constant<int, 1>{}, 1);
        if (b == 2) load_chunk(std::integral_constant<int, 2>{}, 2);
      }
    for (unsigned long long c = 0; c < nch; c += NB) {
      body(std::integral_constant<int, 0>{}, c);
      body(std::integral_constant<int, 1>{}, c + 1);
      body(std::integral_constant<int, 2>{}, c + 2);
      if constexpr (NB > 3) body(std::integral_constant<int, (NB > 3 ? 3 : 0)>{}, c + 3);
    }
  } else if constexpr (DMA) {
    // lane l's 16-byte piece of the step image and its source row (advanced by the row stride)
    const unsigned long long o = 2ull * lane, I = (2 + W) * A;
    const bool on = o < I;
    const u64 *src0 = o < A ? p.ec + g * p.e_gs + k * A + o
                            : (o < (1 + W) * A ? p.val + g * p.v_gs + k * W * A + (o - A)
                                               : p.clock + g * p.c_gs + (o < I ? o - (1 + W) * A : 0));
    const unsigned long long st = o < A ? p.e_rs : (o < (1 + W) * A ? p.v_rs : p.c_rs);
    auto issue = [&](unsigned long long r) {  // step r's image into its slot (past R: row R-1 again)
      const unsigned long long rr = r < R ? r : R - 1;
      if (on) glds16_mc(src0 + rr * st, ring + (r % kMcRing) * 128);
    };
    for (int s = 0; s < kMcRing; ++s) issue((unsigned long long)s);
    for (unsigned long long r = 0; r < R; ++r) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kMcRing - 1) : "memory");  // step r's piece has landed
      const u64 *img = ring + (r % kMcRing) * 128;
      u64 c2[APL], e2[APL], v2[W][APL];
      const unsigned a0 = aj[0];
      e2[0] = img[a0];
      c2[0] = img[(1 + W) * A + a0];
#pragma unroll
      for (int w = 0; w < W; ++w) v2[w][0] = img[(1 + w) * A + a0];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is read: refill it
      issue(r + kMcRing);
      step(r, c2, e2, v2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (no piece lands after the wave ends)
  } else {
    u64 c2r[DEPTH][APL], e2r[DEPTH][APL], v2r[DEPTH][W][APL];
    // the lane's word of each row, advanced by one replica stride per step (no per-step
    // multiplies); past the last replica the pointers stay on it (loaded, never used)
    const u64 *pc = p.clock + g * p.c_gs, *pe = p.ec + g * p.e_gs + kc * A, *pv = p.val + g * p.v_gs + kc * W * A;
    unsigned long long nload = 0;  // replica of the next load_step
    // (the ring holds the raw words, lanes past A copies of actor A-1, used as they are: a select
    // right behind a load would make the wave wait for it at once)
    auto load_step = [&](int s, bool last_check) {
#pragma unroll
      for (int j = 0; j < APL; ++j) {
        c2r[s][j] = pc[aj[j]];
        e2r[s][j] = pe[aj[j]];
#pragma unroll
        for (int w = 0; w < W; ++w) v2r[s][w][j] = pv[w * A + aj[j]];
      }
      if (!last_check || nload + 1 < R) {
        pc += p.c_rs;
        pe += p.e_rs;
        pv += p.v_rs;
      }
      ++nload;
    };
#pragma unroll
    for (int s = 0; s < DEPTH; ++s) load_step(s, true);
    unsigned long long r0 = 0;
    // blocks whose loads (rows r0 + DEPTH .. r0 + 2 DEPTH - 1) all have a next row: no clamp
    for (; r0 + 2 * DEPTH < R; r0 += DEPTH) {
#pragma unroll
      for (int s = 0; s < DEPTH; ++s) {
        step(r0 + s, c2r[s], e2r[s], v2r[s]);
        load_step(s, false);
      }
    }
    for (; r0 < R; r0 += DEPTH) {
#pragma unroll
      for (int s = 0; s < DEPTH; ++s) {
        const unsigned long long r = r0 + s;
        if (r >= R) break;
        step(r, c2r[s], e2r[s], v2r[s]);
        load_step(s, true);
      }
    }
  }
  // ---- the key's folded entry (a stale value behind an empty clock reads 0), the group's clock
  //      (key 0's lanes)
  const bool pf = mc_nz<APL>(e, hm);
  u64 *oe = p.o_ec + (g * p.K + kc) * A;
  u64 *ov = p.o_val + (g * p.K + kc) * W * A;
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = (unsigned long long)al + (unsigned long long)HL * j;
    if (kval && a < A) {
      oe[a] = e[j];
#pragma unroll
      for (int w = 0; w < W; ++w) ov[w * A + a] = pf ? v[w][j] : 0ull;
      if (k == 0) p.o_clock[g * A + a] = C[j];
    }
  }
  if (full && p.rerun_out) {  // the shared list overflowed: the group is re-folded one key per wave
    if (lane == 0) atomicOr(p.rerun_out + g, 1u);
    full = false;
  }
  if ((bad || full) && lane == 0) atomicOr(p.o_flags + g, (bad ? 2u : 0u) | (full ? 8u : 0u));
}

template <int APL, int RING, int W = 1, int SPL = 0, int CL = 0>
static size_t mc_lds() {
  const size_t nrow = (SPL > 0 && CL) ? 4 : kMcRowsB / (8 * kWave * APL);
  return (size_t)kMcWaves * (kMcList * 8 + kMcLive * 4 + nrow * kWave * APL * 8 + RING * 128 * 8 + kMcList + kMcLive +
                             ((SPL > 0 && CL) ? mc_cl_words<W, SPL>() * 8 : 0));
}

template <int APL, int W, int RING = 0, int KPW = 1, int DEP = 8, int SPL = 0, int CL = 0>
static hipError_t launch_mc(const MapCounterPlan &p, hipStream_t s) {
  const unsigned long long blocks = (p.G * ((p.K + KPW - 1) / KPW) + kMcWaves - 1) / kMcWaves;
  const size_t lds = mc_lds<APL, RING, W, SPL, CL>();
  auto *fn = &map_counter_fold_kernel<APL, W, RING, KPW, DEP, SPL, CL>;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(kMcWaves * kWave), lds, s, p);
  return hipGetLastError();
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_map_counter_lub_many(crdt_ctx *ctx, const crdt_map_counter_batch *in,
                                         crdt_map_counter_out *out) {
  if (ctx && ctx->mem_kind == CRDT_MEM_HOST) return crdt::map_counter_lub_many_host(ctx, in, out);
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
                   (u64 *)out->clock, (u64 *)out->ec, (u64 *)out->val, out->flags, nullptr, nullptr};
  if (int rc = device_fill(ctx, out->flags, G * sizeof(unsigned), 0)) return rc;
  if (R == 0) {  // fold of nothing: Map::new()
    if (int rc = device_fill(ctx, out->clock, G * A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, out->ec, G * K * A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, out->val, G * K * W * A * 8, 0)) return rc;
  } else {
    // keys per wave: explicit (mckpw=1/2/4), or automatic (0): pair keys in a wave only while the
    // paired grid still has 2,048+ waves (2 per SIMD) — at 4,096 keys x 4,096 replicas two keys per
    // wave ran 1.60 vs 2.52 ms, at 1,024 keys (one wave per SIMD) 5.33 vs 5.03 ms
    int kpw = ctx->tune.map_counter_kpw;
    const bool auto_kpw = kpw == 0;
    // the whole-chunk skip (one key per wave, A = 32 / 16 / 8, register rows) wins over pairing keys
    const bool al16 = ((p.c_rs | p.c_gs | p.e_rs | p.e_gs | p.v_rs | p.v_gs) & 1) == 0 &&
                      ((uintptr_t)in->clock & 15) == 0 && ((uintptr_t)in->ec & 15) == 0 &&
                      ((uintptr_t)in->val & 15) == 0;
    const int ring0 = A % 2 == 0 && (2 + W) * A <= 128 && al16 ? ctx->tune.map_counter_dma : 0;
    const int spl = ctx->tune.map_counter_cs && !ring0 && ctx->tune.map_counter_depth == 8 && (auto_kpw || kpw == 1)
                        ? (A == 32 ? 2 : (A == 16 ? 4 : (A == 8 ? 8 : 0)))
                        : 0;
    if (spl) kpw = 1;
    if (auto_kpw && !spl) {
      const size_t waves_per_simd2 = 2048;
      kpw = A <= (size_t)kWave / 4 && G * ((K + 3) / 4) >= waves_per_simd2   ? 4
            : A <= (size_t)kWave / 2 && G * ((K + 1) / 2) >= waves_per_simd2 ? 2
                                                                                : 1;
    }
    // scratch: [def_off (G+1) size_t | rerun marks (G) unsigned, automatic keys per wave > 1 only]
    const size_t off_bytes = (G + 1) * sizeof(size_t);
    const bool rerun = D > 0 && auto_kpw && kpw > 1;
    if (D > 0) {
      if (int rc = ensure_scratch(ctx, off_bytes + (rerun ? G * sizeof(unsigned) : 0))) return rc;
      if (int rc = stage_h2d(ctx, ctx->scratch, in->def_off, off_bytes)) return rc;
      p.def_off = reinterpret_cast<const size_t *>(ctx->scratch);
      if (rerun) {
        p.rerun_out = reinterpret_cast<unsigned *>(static_cast<char *>(ctx->scratch) + off_bytes);
        if (int rc = device_fill(ctx, p.rerun_out, G * sizeof(unsigned), 0)) return rc;
      }
    }
    timing_begin(ctx, "map_counter_fold");
    hipError_t he;
    const bool al = ((p.c_rs | p.c_gs | p.e_rs | p.e_gs | p.v_rs | p.v_gs) & 1) == 0 &&
                    ((uintptr_t)in->clock & 15) == 0 && ((uintptr_t)in->ec & 15) == 0 && ((uintptr_t)in->val & 15) == 0;
    const int ring = A % 2 == 0 && (2 + W) * A <= 128 && al ? ctx->tune.map_counter_dma : 0;
    // the LDS-staged chunk skip (opt-in, CRDT_TUNE mccl=1) needs 16-byte aligned rows
    const bool cl = spl && al && ctx->tune.map_counter_cl;
    if (cl && spl == 2) he = W == 1 ? launch_mc<1, 1, 0, 1, 8, 2, 1>(p, ctx->stream) : launch_mc<1, 2, 0, 1, 8, 2, 1>(p, ctx->stream);
    else if (cl && spl == 4) he = W == 1 ? launch_mc<1, 1, 0, 1, 8, 4, 1>(p, ctx->stream) : launch_mc<1, 2, 0, 1, 8, 4, 1>(p, ctx->stream);
    else if (cl && spl == 8) he = W == 1 ? launch_mc<1, 1, 0, 1, 8, 8, 1>(p, ctx->stream) : launch_mc<1, 2, 0, 1, 8, 8, 1>(p, ctx->stream);
    else if (spl == 2) he = W == 1 ? launch_mc<1, 1, 0, 1, 8, 2>(p, ctx->stream) : launch_mc<1, 2, 0, 1, 8, 2>(p, ctx->stream);
    else if (spl == 4) he = W == 1 ? launch_mc<1, 1, 0, 1, 8, 4>(p, ctx->stream) : launch_mc<1, 2, 0, 1, 8, 4>(p, ctx->stream);
    else if (spl == 8) he = W == 1 ? launch_mc<1, 1, 0, 1, 8, 8>(p, ctx->stream) : launch_mc<1, 2, 0, 1, 8, 8>(p, ctx->stream);
    else if (!ring && kpw >= 4 && A <= (size_t)kWave / 4)
      he = W == 1 ? launch_mc<1, 1, 0, 4>(p, ctx->stream) : launch_mc<1, 2, 0, 4>(p, ctx->stream);
    else if (!ring && kpw >= 2 && A <= (size_t)kWave / 2)
      he = W == 1 ? launch_mc<1, 1, 0, 2>(p, ctx->stream) : launch_mc<1, 2, 0, 2>(p, ctx->stream);
    else if (ring == 16) he = W == 1 ? launch_mc<1, 1, 16>(p, ctx->stream) : launch_mc<1, 2, 16>(p, ctx->stream);
    else if (ring) he = W == 1 ? launch_mc<1, 1, 8>(p, ctx->stream) : launch_mc<1, 2, 8>(p, ctx->stream);
    else if (A <= (size_t)kWave && ctx->tune.map_counter_depth == 16)
      he = W == 1 ? launch_mc<1, 1, 0, 1, 16>(p, ctx->stream) : launch_mc<1, 2, 0, 1, 16>(p, ctx->stream);
    else if (A <= (size_t)kWave && ctx->tune.map_counter_depth == 4)
      he = W == 1 ? launch_mc<1, 1, 0, 1, 4>(p, ctx->stream) : launch_mc<1, 2, 0, 1, 4>(p, ctx->stream);
    else if (A <= (size_t)kWave) he = W == 1 ? launch_mc<1, 1>(p, ctx->stream) : launch_mc<1, 2>(p, ctx->stream);
    else if (A <= 2 * (size_t)kWave) he = W == 1 ? launch_mc<2, 1>(p, ctx->stream) : launch_mc<2, 2>(p, ctx->stream);
    else if (A <= 4 * (size_t)kWave) he = W == 1 ? launch_mc<4, 1>(p, ctx->stream) : launch_mc<4, 2>(p, ctx->stream);
    else he = W == 1 ? launch_mc<8, 1>(p, ctx->stream) : launch_mc<8, 2>(p, ctx->stream);
    if (he == hipSuccess && rerun && p.rerun_out) {  // re-fold the groups whose shared list overflowed
      MapCounterPlan q = p;
      q.rerun_in = p.rerun_out;
      q.rerun_out = nullptr;
      he = W == 1 ? launch_mc<1, 1>(q, ctx->stream) : launch_mc<1, 2>(q, ctx->stream);
    }
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
