// Map<K, Orswot<M>> lub_many (round 4): Map::merge (map.rs:140-220) with a nested Orswot value —
// the value type of the reference's own full Map KAT (map.rs:435-494, merge_error).  The value's
// merge is Orswot::merge (orswot.rs:81-149) and its forget Orswot's Causal::forget
// (orswot.rs:150-183).  As for every Map value type the fold acc = Map::new(); for r: acc.merge(r)
// is not associative, so each key is folded in replica order (exact for any input), one wave per
// (group, key), lane = actor (A <= 64), the member rows of the key's Orswot in registers (M <= 32).
//
// Step r on the key's state (map clock C, entry clock e, Orswot clock oc, member rows E[m], nested
// deferred removes D in LDS) with replica r's (c2, e2, oc2, E2[m], D2):
//  - entry clock: the branch-free join of map_counter.hip (the "common" clock covers all four
//    presence cases) and the case's forget clock X (removed_information / we_deleted / deleted);
//  - value, both present (:183): Orswot::merge — per member the dot-survival join
//    max(E == E2 ? E : 0, forget(E2, oc), forget(E, oc2)) (:84-138: elementwise, and empty exactly
//    when the reference drops the member), then every remove of D and D2 forgets its members
//    (apply_rm of other.deferred :141-143 and apply_deferred :147; forgets commute), D2 joins D
//    (an equal clock unions its members, apply_rm :242-246), oc |= oc2, and D keeps the removes
//    with !(rm <= oc) (the re-test of apply_deferred);  only the replica's entry (:193-208): the
//    value is the replica's;  then the value forgets X (:160, :188, :205);
//  - the Map's own removes naming the key (apply_keyset_rm / apply_deferred, :213-219, :318-348),
//    one forget by their max: the entry clock, and the value while the entry stays;
//  - C |= c2 and the Map-level deferral test (witness thresholds, as in map_counter.hip).
// Orswot::forget rebuilds its deferred map with collect(): two removes whose clocks become equal
// keep one entry, the later one's members (HashMap insert order; the reference's own iteration
// order is unspecified, this is the oracle's dict order) at the earlier one's place.
// Lanes past A hold copies of actor A-1 (clamped loads), so they never change a vote.
#include "common.hpp"

namespace crdt {

constexpr int kMoWaves = 4;   // key waves per workgroup
constexpr int kMoList = 256;  // Map removes naming the key, gathered per window (row << 32 | index)
constexpr int kMoLive = 256;  // live Map removes per key
constexpr int kMoRows = 8;    // live Map-remove rows cached in LDS
constexpr int kMoVd = 16;     // nested deferred removes per key state (flags bit 4 past it)
constexpr size_t kMoShallowWaves = 2048;  // key waves from which the 4-step ring (2 waves per SIMD) runs
constexpr unsigned long long kMoRingSpan = 2048;  // chunk-skip mode: register-ring steps run after a
                                                  // window of chunks that rarely skipped (multiple of 8)

struct MapOrswotPlan {
  const u64 *clock, *ec, *oc, *ent;   // (G,R,A), (G,R,K,A), (G,R,K,A), (G,R,K,M,A)
  const u64 *vd_off;                  // nested deferred CSR over (g, r, k): G*R*K + 1 (device)
  const u64 *vd_clock, *vd_mem;       // (Dv, A), (Dv) member bitmasks
  unsigned long long Dv;              // (a step reads rows [min(lo, hi'), hi') with hi' = min(hi, Dv))
  unsigned long long G, R, K, M, A, Kw;
  unsigned long long Mw;  // u64 words per member bitmask: (M + 63) / 64 (1 for M <= 64)
  const size_t *def_off;  // device copy (G+1), or null: no Map-level removes
  const uint32_t *def_row;
  const u64 *def_clock, *def_keys;
  u64 *o_clock, *o_ec, *o_oc, *o_ent, *o_vd_clock, *o_vd_mem;
  unsigned *o_vd_n, *o_flags;
  // round 6: the output's nested slots per key (>= kMoVd; the first kMoVd in LDS during the fold), and
  // when Vd > kMoVd a per-(g, k) marker: the key's list passed kMoVd, re-fold it deep (pass 2)
  unsigned long long Vd;
  uint8_t *ovf;
  unsigned long long Lc;  // the deep pass's live Map-remove capacity per key (>= kMoLive)
};

__device__ __forceinline__ bool mo_nz(u64 x) { return __ballot(x != 0) != 0; }
__device__ __forceinline__ u64 mo_fg(u64 x, u64 c) { return x > c ? x : 0; }  // VClock::forget, per actor
__device__ __forceinline__ u64 mo_max(u64 x, u64 y) { return x > y ? x : y; }

// SPL > 0 (A == 64 / SPL: 32, 16 or 8 actors): the whole-chunk skip below, lane l holding actor
// l % A in every register of the key's state.  SHALLOW (M <= 4): a ring of 4 steps instead of 8, which
// fits two waves per SIMD — chosen where the launch has at least two key waves per SIMD (G*K >= 2,048):
// the config-4-scale causal fold cut into 2 groups of 8,192 replicas ran 6.4-6.7 ms against 11.4 ms for
// the deep ring at 1 wave per SIMD (profiles/r06_mo_split.log).
template <int MT, int SPL = 0, bool SHALLOW = false>
__global__ __launch_bounds__(kMoWaves * kWave) void map_orswot_fold_kernel(MapOrswotPlan p) {
#ifndef MO_RING_DEPTH4
#define MO_RING_DEPTH4 8
#endif
  // replica steps in flight (register ring); the chunk-skip mode's ring phase runs half as deep
  constexpr int DEPTH = SPL > 0 ? (MT <= 4 ? 4 : 2) : (MT <= 4 ? (SHALLOW ? 4 : MO_RING_DEPTH4) : (MT <= 8 ? 4 : 2));
  extern __shared__ u64 lds[];
  const int lane = (int)(threadIdx.x % kWave), wv = (int)(threadIdx.x / kWave);
  const unsigned long long gk = (unsigned long long)blockIdx.x * kMoWaves + wv;
  if (gk >= p.G * p.K) return;  // (whole waves; nothing below synchronises the workgroup)
  const unsigned long long g = gk / p.K, k = gk % p.K, A = p.A, R = p.R, K = p.K, M = p.M;
  constexpr unsigned long long WQ = kMoList + kMoLive / 2 + kMoRows * kWave + kMoVd * kWave + kMoVd;
  u64 *lst = lds + (unsigned long long)wv * WQ;
  uint32_t *live = reinterpret_cast<uint32_t *>(lst + kMoList);
  u64 *rows = lst + kMoList + kMoLive / 2;  // [kMoRows][64] live Map-remove rows
  u64 *vrow = rows + kMoRows * kWave;       // [kMoVd][64] nested deferred rm rows
  u64 *vmsk = vrow + kMoVd * kWave;         // [kMoVd] their member masks
  const unsigned la = SPL > 0 ? (unsigned)lane & (unsigned)(kWave / (SPL > 0 ? SPL : 1) - 1)  // the lane's actor
                              : (unsigned)((unsigned long long)lane < A ? lane : A - 1);
  auto ld = [&](const u64 *row) { return row[la]; };

  // ---- the Map's removes naming key k, in replica order (map_counter.hip's walk, one key)
  const unsigned long long d0 = p.def_off ? p.def_off[g] : 0, d1 = p.def_off ? p.def_off[g + 1] : 0;
  unsigned long long dc = d0;
  int nl = 0, li = 0;
  bool bad = false;  // def_row not non-decreasing or >= R (flags bit 1)
  u64 last_row = 0;
  auto refill = [&]() {
    nl = 0;
    li = 0;
    while (dc < d1 && nl + kWave <= kMoList) {
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
  unsigned nxt = ~0u;  // replica row of the next remove naming k (~0: none left)
  auto advance = [&]() {
    for (;;) {
      if (li < nl) {
        nxt = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(lst[li] >> 32));
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
  bool full = false;   // more than kMoLive live Map removes on the key (flags bit 3)
  bool vfull = false;  // more than kMoVd nested deferred removes (flags bit 4)
  int na = 0;
  auto live_row = [&](int i) -> u64 {
    return i < kMoRows ? rows[(unsigned long long)i * kWave + lane] : ld(p.def_clock + (d0 + live[i]) * A);
  };
  auto put_row = [&](int i, u64 x) {
    if (i < kMoRows) rows[(unsigned long long)i * kWave + lane] = x;
  };
  u64 rk = 0, T = ~0ull;  // max of the live Map removes / witness thresholds

  // ---- the key's state
  u64 C = 0, e = 0, oc = 0, E[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) E[m] = 0;
  int nd = 0;  // nested deferred removes in vrow / vmsk (uniform)
  // the member rows are forgotten by every held nested remove (true after a both-present merge, which
  // re-applies them all, and kept by forgets; false after the replica's Orswot was taken as it came,
  // whose own removes need not have been applied to its rows): a precondition of the chunk skip
  bool vnorm = true;

  // nested deferred helpers (LDS rows, uniform control flow)
  auto forget_members = [&](u64 rm, u64 msk) {  // Orswot::apply_rm's member forget (orswot.rs:231-238)
#pragma unroll
    for (int m = 0; m < MT; ++m)
      if ((msk >> m) & 1ull) E[m] = mo_fg(E[m], rm);
  };
  auto vd_add = [&](u64 rm, u64 msk) {  // deferred.entry(clock) extend / insert (orswot.rs:242-246)
    for (int i = 0; i < nd; ++i) {
      if (!__ballot(vrow[(unsigned long long)i * kWave + lane] != rm)) {
        const u64 mm = vmsk[i] | msk;
        if (lane == 0) vmsk[i] = mm;
        return;
      }
    }
    if (nd < kMoVd) {
      vrow[(unsigned long long)nd * kWave + lane] = rm;
      if (lane == 0) vmsk[nd] = msk;
      ++nd;
    } else {
      vfull = true;
    }
  };
  auto vd_keep_live = [&]() {  // apply_deferred's re-test: keep !(rm <= oc), in order
    int o = 0;
    for (int i = 0; i < nd; ++i) {
      const u64 x = vrow[(unsigned long long)i * kWave + lane];
      const u64 mi = vmsk[i];
      if (__ballot(x > oc)) {
        if (o != i) {
          vrow[(unsigned long long)o * kWave + lane] = x;
          if (lane == 0) vmsk[o] = mi;
        }
        ++o;
      }
    }
    nd = o;
  };
  auto value_forget = [&](u64 X) {  // Orswot's Causal::forget (orswot.rs:150-183)
    oc = mo_fg(oc, X);
#pragma unroll
    for (int m = 0; m < MT; ++m) E[m] = mo_fg(E[m], X);
    int o = 0;
    for (int i = 0; i < nd; ++i) {
      const u64 x = mo_fg(vrow[(unsigned long long)i * kWave + lane], X);
      const u64 mi = vmsk[i];
      if (!__ballot(x != 0)) continue;  // forgotten
      int j = 0;
      for (; j < o; ++j)  // equal to a kept one: the later members at the earlier place (collect())
        if (!__ballot(vrow[(unsigned long long)j * kWave + lane] != x)) break;
      if (j < o) {
        if (lane == 0) vmsk[j] = mi;
        continue;
      }
      vrow[(unsigned long long)o * kWave + lane] = x;
      if (lane == 0) vmsk[o] = mi;
      ++o;
    }
    nd = o;
  };

  // the Map-level live set re-test (witness thresholds; chg: removes joined the live set)
  auto liveness = [&](bool chg) {
    if (na > 0 && (chg || __ballot(C >= T))) {
      bool changed = chg;
      T = ~0ull;
      for (int i = 0; i < na;) {
        const u64 rm = live_row(i);
        const u64 m = __ballot(rm > C);
        if (m) {
          const int wl = __builtin_ctzll(m);
          T = lane == wl && rm < T ? rm : T;
          ++i;
          continue;
        }
        changed = true;
        const int lastp = na - 1;
        if (i != lastp) {
          put_row(i, live_row(lastp));
          const unsigned li_last = live[lastp];
          if (lane == 0) live[i] = li_last;
        }
        --na;
      }
      if (changed) {
        rk = 0;
        for (int i = 0; i < na; ++i) rk = mo_max(rk, live_row(i));
      }
    }
  };

  // one replica step
  auto step = [&](unsigned long long r, u64 c2, u64 e2, u64 o2, const u64 (&E2)[MT], u64 vlo, u64 vhi) {
    const bool p1 = mo_nz(e), p2 = mo_nz(e2);
    const u64 en = e == e2 ? e : mo_max(mo_fg(e2, C), mo_fg(e, c2));  // (the forgets are <= e where e == e2)
    const u64 y = p1 ? (p2 ? mo_max(e, e2) : c2) : C;
    const u64 X = mo_fg(y, en);
    // An empty joined clock drops the entry without touching its value (map.rs:178-180, :191-192:
    // no val.merge), so the value work runs only while the entry stays; a dropped entry's stale rows
    // are never read again (p1 is false until the key is re-added, which overwrites them).
    const bool stays = mo_nz(en);
    if (p1 && p2 && stays) {  // our_entry.val.merge(entry.val) (map.rs:183) = Orswot::merge
#pragma unroll
      for (int m = 0; m < MT; ++m)
        E[m] = E[m] == E2[m] ? E[m] : mo_max(mo_fg(E2[m], oc), mo_fg(E[m], o2));
      // apply_rm of each of the replica's removes against the clock BEFORE oc |= oc2 (orswot.rs:
      // 141-143, :230-238): its members are forgotten, and it is deferred only if !(rm <= oc)
      for (u64 d = vlo; d < vhi; ++d) {
        const u64 rm = ld(p.vd_clock + d * A), msk = p.vd_mem[d];
        forget_members(rm, msk);
        if (__ballot(rm > oc)) vd_add(rm, msk);
      }
      // apply_deferred (:147, :281-286): every remove still held forgets its members again with
      // the merged clock, and stays while !(rm <= oc)
      oc = mo_max(oc, o2);
      for (int i = 0; i < nd; ++i) forget_members(vrow[(unsigned long long)i * kWave + lane], vmsk[i]);
      vd_keep_live();
      vnorm = true;
    } else if (p2 && !p1 && stays) {  // the replica's entry (map.rs:193-208)
#pragma unroll
      for (int m = 0; m < MT; ++m) E[m] = E2[m];
      oc = o2;
      nd = 0;
      for (u64 d = vlo; d < vhi; ++d) {
        const u64 rm = ld(p.vd_clock + d * A), msk = p.vd_mem[d];
        vd_add(rm, msk);
      }
      vnorm = nd == 0;
    }
    if (stays && (p1 || p2)) value_forget(X);
    e = en;
    // the Map's removes: replica r's own (apply_keyset_rm) and the live ones (apply_deferred)
    bool chg = false;
    u64 f = rk;
    const unsigned r32 = (unsigned)r;
    if (nxt <= r32) {
      do {
        const unsigned idx = (unsigned)lst[li];
        const u64 rm = ld(p.def_clock + (d0 + idx) * A);
        f = mo_max(f, rm);
        if (na < kMoLive) {
          if (lane == 0) live[na] = idx;
          put_row(na, rm);
          ++na;
          chg = true;
        } else {
          full = true;
        }
        ++li;
        advance();
      } while (nxt <= r32);
    }
    if (na > 0) {  // (f = 0 otherwise: nothing to forget)
      e = mo_fg(e, f);
      if (mo_nz(e)) value_forget(f);  // entry.val.forget only while the entry stays (map.rs:321-330)
    }
    C = mo_max(C, c2);
    liveness(chg);
  };

  // ---- replica rows [rs, re) through a register ring (DEPTH steps ahead; clamped at row re - 1)
  auto ring_phase = [&](unsigned long long rs, unsigned long long re) {
    const u64 *pc = p.clock + (g * R + rs) * A, *pe = p.ec + ((g * R + rs) * K + k) * A,
              *po = p.oc + ((g * R + rs) * K + k) * A;
    const u64 *pm = p.ent + ((g * R + rs) * K + k) * M * A;
    const u64 *pvo = p.vd_off + (g * R + rs) * K + k;
    const unsigned long long rsK = K * A, rsM = K * M * A;
    u64 c2r[DEPTH], e2r[DEPTH], o2r[DEPTH], E2r[DEPTH][MT], vlr[DEPTH], vhr[DEPTH];
    unsigned long long nload = rs;
    auto load_step = [&](int s, bool last_check) {
      c2r[s] = ld(pc);
      e2r[s] = ld(pe);
      o2r[s] = ld(po);
#pragma unroll
      for (int m = 0; m < MT; ++m) E2r[s][m] = (unsigned long long)m < M ? ld(pm + m * A) : 0ull;
      vlr[s] = pvo[0];
      vhr[s] = pvo[1];
      if (!last_check || nload + 1 < re) {
        pc += A;
        pe += rsK;
        po += rsK;
        pm += rsM;
        pvo += K;
      }
      ++nload;
    };
    auto run = [&](unsigned long long r, int s, bool last_check) {
      const u64 vlo = __builtin_amdgcn_readfirstlane((unsigned)vlr[s]) |
                      ((u64)__builtin_amdgcn_readfirstlane((unsigned)(vlr[s] >> 32)) << 32);
      u64 vhi = __builtin_amdgcn_readfirstlane((unsigned)vhr[s]) |
                ((u64)__builtin_amdgcn_readfirstlane((unsigned)(vhr[s] >> 32)) << 32);
      vhi = vhi < p.Dv ? vhi : p.Dv;  // (a malformed vd_off never reads past the rows: flags bit 5)
      step(r, c2r[s], e2r[s], o2r[s], E2r[s], vlo < vhi ? vlo : vhi, vhi);
      load_step(s, last_check);
    };
#pragma unroll
    for (int s = 0; s < DEPTH; ++s) load_step(s, true);
    unsigned long long r0 = rs;
    // blocks whose loads (rows r0 + DEPTH .. r0 + 2 DEPTH - 1) all have a next row: no clamp
    for (; r0 + 2 * DEPTH < re; r0 += DEPTH) {
#pragma unroll
      for (int s = 0; s < DEPTH; ++s) run(r0 + s, s, false);
    }
    for (; r0 < re; r0 += DEPTH) {
#pragma unroll
      for (int s = 0; s < DEPTH; ++s) {
        if (r0 + s >= re) break;
        run(r0 + s, s, true);
      }
    }
  };

  if constexpr (SPL > 0) {
    // ---- whole-chunk skip (round 5), the counter Map's (map_counter.hip) with the nested Orswot:
    // chunks of S = 8 steps in the transposed layout (lane (hh, a): actor a of step i*SPL + hh),
    // tested against the state at the chunk's start; a chunk all of whose steps leave (entry clock,
    // Orswot clock, member dots, nested deferred removes) unchanged only merges its clocks.  With
    // the acc holding the key (p1), per word, besides the entry tests of map_counter.hip:
    //   the replica holds it too (p2):  o2 <= oc (the Orswot clock does not grow), and for every
    //     member E2 == E || (E2 <= oc && o2 <= TE_m), TE_m = E ? E-1 : MAX (the dot-survival join
    //     keeps E: forget(E2, oc) is empty and forget(E, o2) is E), no nested removes in the step,
    //     and e2 <= TX, TX = min over oc, every E and every held nested rm word v of
    //     (v ? max(e, v-1) : MAX) (the value forget by x = e2 > e ? e2 : 0 keeps every word);
    //   only the acc holds it:  c2 <= min(TE, TX) (entry and value survive forget by c2);
    //   no p1:  e2 <= C0.
    // The held nested removes and the Map's live removes were applied when they joined (forgets
    // are idempotent), so an unchanged state stays unchanged under their re-application.
    constexpr int S = 8, NE = S / SPL, NB = 3;
    constexpr unsigned long long AA = kWave / SPL;  // == A
    const int hh = lane / (int)AA;
    const unsigned a = (unsigned)lane & (unsigned)(AA - 1);
    const unsigned long long rsK = K * AA, rsM = K * M * AA;
    const u64 *bc = p.clock + g * R * AA + a, *be = p.ec + (g * R * K + k) * AA + a,
              *bo = p.oc + (g * R * K + k) * AA + a, *bm = p.ent + (g * R * K + k) * M * AA + a;
    const u64 *pvo0 = p.vd_off + g * R * K + k;
    const unsigned long long nch = (R + S - 1) / S;
    u64 qc[NB][NE], qe[NB][NE], qo[NB][NE], qm[NB][MT][NE], qlo[NB], qhi[NB];
    auto load_chunk = [&](auto B, unsigned long long c) {
      constexpr int b = decltype(B)::value;
      const unsigned long long r0 = c * S;
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        unsigned long long rr = r0 + (unsigned long long)(i * SPL + hh);
        rr = rr < R ? rr : R - 1;  // (past the last replica: its row again, never used)
        qc[b][i] = bc[rr * AA];
        qe[b][i] = be[rr * rsK];
        qo[b][i] = bo[rr * rsK];
        // (every load unconditional, so that no load sits in a branch and none is waited for at
        // once: a member past M reads member 0's row, which the test ignores)
#pragma unroll
        for (int m = 0; m < MT; ++m) qm[b][m][i] = bm[rr * rsM + ((unsigned long long)m < M ? m : 0) * AA];
      }
      unsigned long long rs = r0 + (unsigned long long)(lane & (S - 1));
      rs = rs < R ? rs : R - 1;
      qlo[b] = pvo0[rs * K];  // lane s (mod S): step r0 + s's nested remove range
      qhi[b] = pvo0[rs * K + 1];
    };
#ifdef MO_STATS
    unsigned st[7] = {0, 0, 0, 0, 0, 0, 0};  // skipped, nested rm, !vnorm, held dead, no p1, test, other
#define MO_ST(i) (++st[i])
#else
#define MO_ST(i) ((void)0)
#endif
    auto test_chunk = [&](auto B) -> bool {
      constexpr int b = decltype(B)::value;
      if (__ballot(qhi[b] != qlo[b])) return MO_ST(1), false;  // a step carries nested removes: exact
      // the held nested removes must already be applied to the rows and live (!(rm <= oc)): a
      // both-present step re-applies them and re-tests their liveness
      if (!vnorm) return MO_ST(2), false;
      for (int i = 0; i < nd; ++i)
        if (!__ballot(vrow[(unsigned long long)i * kWave + lane] > oc)) return MO_ST(3), false;
      const u64 e0 = e, C0 = C;
      if (!mo_nz(e0)) {  // the acc lacks the key: no replica of the chunk may add it
        u64 okm = ~0ull;
#pragma unroll
        for (int i = 0; i < NE; ++i) okm &= __ballot(qe[b][i] <= C0);
        if (okm != ~0ull) MO_ST(4);
        return okm == ~0ull;
      }
      const u64 em1 = e0 ? e0 - 1 : 0;
      const u64 TE = e0 ? em1 : ~0ull, TB = C0 > em1 ? C0 : em1;
      auto tv = [&](u64 v) -> u64 { return v == 0 ? ~0ull : (e0 > v - 1 ? e0 : v - 1); };
      u64 TX = tv(oc), TEm[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const u64 t = tv(E[m]);
        TX = t < TX ? t : TX;
        TEm[m] = E[m] ? E[m] - 1 : ~0ull;
      }
      for (int i = 0; i < nd; ++i) {
        const u64 t = tv(vrow[(unsigned long long)i * kWave + lane]);
        TX = t < TX ? t : TX;
      }
      const u64 TN = TE < TX ? TE : TX;
      u64 fail = 0;
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const u64 e2 = qe[b][i], c2 = qc[b][i], o2 = qo[b][i];
        bool cb = (e2 == e0 || (c2 <= TE && e2 <= TB)) && e2 <= TX && o2 <= oc;
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const u64 E2 = (unsigned long long)m < M ? qm[b][m][i] : E[m];  // (E[m] = 0 past M)
          cb = cb && (E2 == E[m] || (E2 <= oc && o2 <= TEm[m]));
        }
        const u64 mN = __ballot(e2 != 0), mB = __ballot(cb), mO = __ballot(c2 <= TN);
#pragma unroll
        for (int s2 = 0; s2 < SPL; ++s2) {
          const u64 Mk = (AA == 64 ? ~0ull : ((1ull << AA) - 1)) << (s2 * AA);
          const u64 sel = (mN & Mk) ? mB : mO;
          fail |= ~sel & Mk;
        }
      }
      if (fail) MO_ST(5);
      return fail == 0;
    };
    // The chunk loop only tests and skips: a chunk that fails the test ends it, and its steps run
    // through the register ring (one copy of the exact step in the kernel, rows in lane = actor
    // layout), then chunks are tested again.  The skip only pays where most chunks pass: after a
    // window of 8 tested chunks with fewer than 3 skipped the ring runs kMoRingSpan steps.
    unsigned hist = ~0u;  // skip bits of the latest tested chunks (uniform)
    auto body = [&](auto B, unsigned long long c) -> bool {  // false: chunk c must run exactly
      constexpr int b = decltype(B)::value;
      if (c >= nch) return true;
      if (c + NB - 1 < nch) load_chunk(std::integral_constant<int, (b + NB - 1) % NB>{}, c + NB - 1);
      const unsigned long long r0 = c * S;
      const unsigned long long n = R - r0 < (unsigned long long)S ? R - r0 : S;
      if (!(n == S && (unsigned long long)nxt >= r0 + S && test_chunk(B))) return false;
      MO_ST(0);
      u64 cm = 0;
#pragma unroll
      for (int i = 0; i < NE; ++i) cm = qc[b][i] > cm ? qc[b][i] : cm;
#pragma unroll
      for (int off = (int)AA; off < kWave; off <<= 1) {
        const u64 o = __shfl_xor(cm, off);
        cm = o > cm ? o : cm;
      }
      C = C > cm ? C : cm;
      liveness(false);
      hist = hist << 1 | 1u;
      return true;
    };
    // chunks c0.. (chunk c0 + j in buffer j % NB) while they skip; the first one that does not (nch: none)
    auto chunk_phase = [&](unsigned long long c0) -> unsigned long long {
      load_chunk(std::integral_constant<int, 0>{}, c0);
      if (c0 + 1 < nch) load_chunk(std::integral_constant<int, 1>{}, c0 + 1);
      for (unsigned long long c = c0; c < nch; c += NB) {
        if (!body(std::integral_constant<int, 0>{}, c)) return c;
        if (!body(std::integral_constant<int, 1>{}, c + 1)) return c + 1;
        if (!body(std::integral_constant<int, 2>{}, c + 2)) return c + 2;
      }
      return nch;
    };
    unsigned long long nring = 0;
    for (unsigned long long c = 0; c < nch;) {
      c = chunk_phase(c);
      if (c >= nch) break;
      hist <<= 1;
      const bool poor = __builtin_popcount(hist & 0xFFu) < 3;
      const unsigned long long span = poor ? kMoRingSpan : (unsigned long long)S;
      const unsigned long long rs = c * S, re = R - rs < span ? R : rs + span;
      ring_phase(rs, re);
      if (poor) hist = ~0u;
      nring += re - rs;
      c = re == R ? nch : re / S;
    }
#ifdef MO_STATS
    if (lane == 0 && gk < 6)
      printf("mo key %llu: chunks %llu skipped %u | nested-rm %u !vnorm %u held-dead %u no-p1 %u test %u | ring steps %llu nd %d\n",
             gk, nch, st[0], st[1], st[2], st[3], st[4], st[5], nring, nd);
#endif
    (void)nring;
  } else {
    ring_phase(0, R);
  }

  // ---- the key's folded entry (an empty entry clock: absent, value rows 0), the group's clock
  const bool pf = mo_nz(e);
  if ((unsigned long long)lane < A) {
    p.o_ec[gk * A + lane] = e;
    p.o_oc[gk * A + lane] = pf ? oc : 0ull;
    for (unsigned long long m = 0; m < M; ++m) {
      u64 x = 0;
#pragma unroll
      for (int q = 0; q < MT; ++q)
        if ((unsigned long long)q == m) x = E[q];
      p.o_ent[(gk * M + m) * A + lane] = pf ? x : 0ull;
    }
    if (k == 0) p.o_clock[g * A + lane] = C;
  }
  const int no = pf ? nd : 0;
  for (int i = 0; i < no; ++i) {
    const u64 x = vrow[(unsigned long long)i * kWave + lane];
    if ((unsigned long long)lane < A) p.o_vd_clock[(gk * p.Vd + i) * A + lane] = x;
    if (lane == 0) p.o_vd_mem[gk * p.Vd + i] = vmsk[i];
  }
  if (lane == 0) p.o_vd_n[gk] = (unsigned)no;
  // past the LDS slots / the live list, where the deep pass has room for both: it re-folds this key
  if ((vfull || full) && p.ovf && (!vfull || p.Vd > (unsigned long long)kMoVd) && (!full || p.Lc > (unsigned long long)kMoLive)) {
    if (lane == 0) p.ovf[gk] = 1;
    vfull = full = false;
  }
  if ((bad || full || vfull) && lane == 0)
    atomicOr(p.o_flags + g, (bad ? 2u : 0u) | (full ? 8u : 0u) | (vfull ? 16u : 0u));
}

// ---- wide shapes (round 5): A <= 1,024 actors, M <= 1,024 members ---------------------------------
// The same fold, step for step (the comments of map_orswot_fold_kernel's step() apply line by line),
// one wave per (group, key) with lane l holding actors l + 64 j (j < APL).  The key's member rows and
// its nested deferred rm rows live in the key's own output rows (o_ent, o_vd_clock: each lane reads
// back only the words it wrote), the nested removes' member masks (Mw words each) and the Map's
// removes naming the key in LDS.  Every replica row is read straight from global memory: a
// correctness path for shapes past the register kernel's, not a fast one.
constexpr int kMoWideMw = 16;  // member-mask words (M <= 1,024)
// DEEP (round 6, the exact overflow pass): one wave per workgroup re-folds only the keys the first
// pass marked in p.ovf, with p.Vd nested slots (their masks in LDS: Vd * Mw words)
template <int APL, bool DEEP = false>
__global__ __launch_bounds__(kMoWaves * kWave) void map_orswot_wide_kernel(MapOrswotPlan p) {
  extern __shared__ u64 lds[];
  const int lane = (int)(threadIdx.x % kWave), wv = (int)(threadIdx.x / kWave);
  const unsigned long long gk = DEEP ? (unsigned long long)blockIdx.x : (unsigned long long)blockIdx.x * kMoWaves + wv;
  if (gk >= p.G * p.K) return;  // (whole waves; nothing below synchronises the workgroup)
  if constexpr (DEEP) {
    if (!p.ovf[gk]) return;
  }
  const unsigned long long g = gk / p.K, k = gk % p.K, A = p.A, R = p.R, K = p.K, M = p.M, Mw = p.Mw;
  const unsigned long long LC = DEEP ? p.Lc : (unsigned long long)kMoLive;  // live Map removes held
  const unsigned long long WQ = kMoList + (LC + 1) / 2 + (DEEP ? p.Vd * Mw : (unsigned long long)kMoVd * kMoWideMw);
  const int cap = DEEP ? (int)p.Vd : kMoVd;
  u64 *lst = lds + (unsigned long long)wv * WQ;
  uint32_t *live = reinterpret_cast<uint32_t *>(lst + kMoList);
  u64 *vmsk = lst + kMoList + (LC + 1) / 2;  // [cap][Mw] nested removes' member masks
  u64 *wE = p.o_ent + gk * M * A;           // [M][A] the key's member rows (working state)
  u64 *wV = p.o_vd_clock + gk * p.Vd * A;   // [cap][A] its nested deferred rm rows
  // row I/O: word j of the lane is actor lane + 64 j; words past A read 0 and are never written
  auto ldr = [&](const u64 *row, u64 (&x)[APL]) {
#pragma unroll
    for (int j = 0; j < APL; ++j) {
      const unsigned long long a = (unsigned long long)lane + 64ull * j;
      x[j] = a < A ? row[a] : 0ull;
    }
  };
  auto str = [&](u64 *row, const u64 (&x)[APL]) {
#pragma unroll
    for (int j = 0; j < APL; ++j) {
      const unsigned long long a = (unsigned long long)lane + 64ull * j;
      if (a < A) row[a] = x[j];
    }
  };
  auto any_nz = [&](const u64 (&x)[APL]) {
    u64 o = 0;
#pragma unroll
    for (int j = 0; j < APL; ++j) o |= x[j];
    return __ballot(o != 0) != 0;
  };
  auto any_gt = [&](const u64 (&x)[APL], const u64 (&c)[APL]) {
    bool b = false;
#pragma unroll
    for (int j = 0; j < APL; ++j) b = b || x[j] > c[j];
    return __ballot(b) != 0;
  };
  auto any_ne = [&](const u64 (&x)[APL], const u64 (&c)[APL]) {
    bool b = false;
#pragma unroll
    for (int j = 0; j < APL; ++j) b = b || x[j] != c[j];
    return __ballot(b) != 0;
  };
  auto fg_row = [&](u64 (&x)[APL], const u64 (&c)[APL]) {
#pragma unroll
    for (int j = 0; j < APL; ++j) x[j] = mo_fg(x[j], c[j]);
  };

  // ---- the Map's removes naming key k, in replica order (map_orswot_fold_kernel's walk)
  const unsigned long long d0 = p.def_off ? p.def_off[g] : 0, d1 = p.def_off ? p.def_off[g + 1] : 0;
  unsigned long long dc = d0;
  int nl = 0, li = 0;
  bool bad = false;
  u64 last_row = 0;
  auto refill = [&]() {
    nl = 0;
    li = 0;
    while (dc < d1 && nl + kWave <= kMoList) {
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
  unsigned nxt = ~0u;
  auto advance = [&]() {
    for (;;) {
      if (li < nl) {
        nxt = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(lst[li] >> 32));
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
  bool full = false, vfull = false;
  int na = 0;
  auto live_row = [&](int i, u64 (&x)[APL]) { ldr(p.def_clock + (d0 + live[i]) * A, x); };
  u64 rk[APL], T[APL];

  // ---- the key's state (members and nested removes in wE / wV / vmsk)
  u64 C[APL], e[APL], oc[APL];
#pragma unroll
  for (int j = 0; j < APL; ++j) C[j] = e[j] = oc[j] = rk[j] = 0, T[j] = ~0ull;
  int nd = 0;

  auto forget_members = [&](const u64 (&rm)[APL], const u64 *msk) {  // apply_rm's member forget
    for (unsigned long long w = 0; w < Mw; ++w) {
      u64 bits = msk[w];
      while (bits) {
        const unsigned long long m = w * 64 + (unsigned long long)__builtin_ctzll(bits);
        bits &= bits - 1;
        if (m >= M) break;
        u64 x[APL];
        ldr(wE + m * A, x);
        fg_row(x, rm);
        str(wE + m * A, x);
      }
    }
  };
  auto vd_add = [&](const u64 (&rm)[APL], const u64 *msk) {  // deferred.entry(clock) extend / insert
    for (int i = 0; i < nd; ++i) {
      u64 x[APL];
      ldr(wV + (unsigned long long)i * A, x);
      if (!any_ne(x, rm)) {
        for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) vmsk[i * Mw + w] |= msk[w];
        return;
      }
    }
    if (nd < cap) {
      str(wV + (unsigned long long)nd * A, rm);
      for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) vmsk[nd * Mw + w] = msk[w];
      ++nd;
    } else {
      vfull = true;
    }
  };
  auto vd_keep_live = [&]() {  // apply_deferred's re-test: keep !(rm <= oc), in order
    int o = 0;
    for (int i = 0; i < nd; ++i) {
      u64 x[APL];
      ldr(wV + (unsigned long long)i * A, x);
      if (any_gt(x, oc)) {
        if (o != i) {
          str(wV + (unsigned long long)o * A, x);
          for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) vmsk[o * Mw + w] = vmsk[i * Mw + w];
        }
        ++o;
      }
    }
    nd = o;
  };
  auto value_forget = [&](const u64 (&X)[APL]) {  // Orswot's Causal::forget
    fg_row(oc, X);
    for (unsigned long long m = 0; m < M; ++m) {
      u64 x[APL];
      ldr(wE + m * A, x);
      fg_row(x, X);
      str(wE + m * A, x);
    }
    int o = 0;
    for (int i = 0; i < nd; ++i) {
      u64 x[APL];
      ldr(wV + (unsigned long long)i * A, x);
      fg_row(x, X);
      if (!any_nz(x)) continue;  // forgotten
      int jj = 0;
      for (; jj < o; ++jj) {  // equal to a kept one: the later members at the earlier place
        u64 y[APL];
        ldr(wV + (unsigned long long)jj * A, y);
        if (!any_ne(y, x)) break;
      }
      if (jj < o) {
        for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) vmsk[jj * Mw + w] = vmsk[i * Mw + w];
        continue;
      }
      str(wV + (unsigned long long)o * A, x);
      if (o != i)
        for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) vmsk[o * Mw + w] = vmsk[i * Mw + w];
      ++o;
    }
    nd = o;
  };
  auto liveness = [&](bool chg) {
    bool hitT = false;
#pragma unroll
    for (int j = 0; j < APL; ++j) hitT = hitT || C[j] >= T[j];
    if (na > 0 && (chg || __ballot(hitT))) {
      bool changed = chg;
#pragma unroll
      for (int j = 0; j < APL; ++j) T[j] = ~0ull;
      for (int i = 0; i < na;) {
        u64 rm[APL];
        live_row(i, rm);
        bool w = false;
#pragma unroll
        for (int j = 0; j < APL; ++j) w = w || rm[j] > C[j];
        const u64 mb = __ballot(w);
        if (mb) {
          if (lane == __builtin_ctzll(mb)) {
            bool done = false;
#pragma unroll
            for (int j = 0; j < APL; ++j) {
              if (!done && rm[j] > C[j]) {
                T[j] = rm[j] < T[j] ? rm[j] : T[j];
                done = true;
              }
            }
          }
          ++i;
          continue;
        }
        changed = true;
        const int lastp = na - 1;
        if (i != lastp) {
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
          for (int j = 0; j < APL; ++j) rk[j] = mo_max(rk[j], rm[j]);
        }
      }
    }
  };

  for (unsigned long long r = 0; r < R; ++r) {
    const unsigned long long rk_ = (g * R + r) * K + k;
    u64 c2[APL], e2[APL], o2[APL];
    ldr(p.clock + (g * R + r) * A, c2);
    ldr(p.ec + rk_ * A, e2);
    ldr(p.oc + rk_ * A, o2);
    u64 vlo = p.vd_off[rk_], vhi = p.vd_off[rk_ + 1];
    vhi = vhi < p.Dv ? vhi : p.Dv;  // (a malformed vd_off never reads past the rows: flags bit 5)
    vlo = vlo < vhi ? vlo : vhi;
    const bool p1 = any_nz(e), p2 = any_nz(e2);
    u64 en[APL], X[APL];
#pragma unroll
    for (int j = 0; j < APL; ++j) {
      en[j] = e[j] == e2[j] ? e[j] : mo_max(mo_fg(e2[j], C[j]), mo_fg(e[j], c2[j]));
      const u64 y = p1 ? (p2 ? mo_max(e[j], e2[j]) : c2[j]) : C[j];
      X[j] = mo_fg(y, en[j]);
    }
    const bool stays = any_nz(en);
    if (p1 && p2 && stays) {  // Orswot::merge
      const u64 *E2 = p.ent + rk_ * M * A;
      for (unsigned long long m = 0; m < M; ++m) {
        u64 x[APL], x2[APL];
        ldr(wE + m * A, x);
        ldr(E2 + m * A, x2);
#pragma unroll
        for (int j = 0; j < APL; ++j) x[j] = x[j] == x2[j] ? x[j] : mo_max(mo_fg(x2[j], oc[j]), mo_fg(x[j], o2[j]));
        str(wE + m * A, x);
      }
      for (u64 d = vlo; d < vhi; ++d) {
        u64 rm[APL];
        ldr(p.vd_clock + d * A, rm);
        const u64 *msk = p.vd_mem + d * Mw;
        forget_members(rm, msk);
        if (any_gt(rm, oc)) vd_add(rm, msk);
      }
#pragma unroll
      for (int j = 0; j < APL; ++j) oc[j] = mo_max(oc[j], o2[j]);
      for (int i = 0; i < nd; ++i) {
        u64 rm[APL];
        ldr(wV + (unsigned long long)i * A, rm);
        forget_members(rm, vmsk + i * Mw);
      }
      vd_keep_live();
    } else if (p2 && !p1 && stays) {  // the replica's entry
      const u64 *E2 = p.ent + rk_ * M * A;
      for (unsigned long long m = 0; m < M; ++m) {
        u64 x[APL];
        ldr(E2 + m * A, x);
        str(wE + m * A, x);
      }
#pragma unroll
      for (int j = 0; j < APL; ++j) oc[j] = o2[j];
      nd = 0;
      for (u64 d = vlo; d < vhi; ++d) {
        u64 rm[APL];
        ldr(p.vd_clock + d * A, rm);
        vd_add(rm, p.vd_mem + d * Mw);
      }
    }
    if (stays && (p1 || p2)) value_forget(X);
#pragma unroll
    for (int j = 0; j < APL; ++j) e[j] = en[j];
    // the Map's removes: replica r's own and the live ones
    bool chg = false;
    u64 f[APL];
#pragma unroll
    for (int j = 0; j < APL; ++j) f[j] = rk[j];
    const unsigned r32 = (unsigned)r;
    while (nxt <= r32) {
      const unsigned idx = (unsigned)lst[li];
      u64 rm[APL];
      ldr(p.def_clock + (d0 + idx) * A, rm);
#pragma unroll
      for (int j = 0; j < APL; ++j) f[j] = mo_max(f[j], rm[j]);
      if ((unsigned long long)na < LC) {
        if (lane == 0) live[na] = idx;
        ++na;
        chg = true;
      } else {
        full = true;
      }
      ++li;
      advance();
    }
    if (na > 0) {
      fg_row(e, f);
      if (any_nz(e)) value_forget(f);
    }
#pragma unroll
    for (int j = 0; j < APL; ++j) C[j] = mo_max(C[j], c2[j]);
    liveness(chg);
  }

  // ---- the key's folded entry (absent: every row 0), the group's clock
  const bool pf = any_nz(e);
  if (!pf) {
    u64 z[APL];
#pragma unroll
    for (int j = 0; j < APL; ++j) z[j] = 0;
    for (unsigned long long m = 0; m < M; ++m) str(wE + m * A, z);
  }
  str(p.o_ec + gk * A, e);
  if (!pf) {
#pragma unroll
    for (int j = 0; j < APL; ++j) oc[j] = 0;
  }
  str(p.o_oc + gk * A, oc);
  if (k == 0) str(p.o_clock + g * A, C);
  const int no = pf ? nd : 0;
  for (int i = 0; i < no; ++i)
    for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave)
      p.o_vd_mem[(gk * p.Vd + i) * Mw + w] = vmsk[i * Mw + w];
  if (lane == 0) p.o_vd_n[gk] = (unsigned)no;
  if constexpr (!DEEP) {  // (as the register kernel: the deep pass re-folds this key)
    if ((vfull || full) && p.ovf && (!vfull || p.Vd > (unsigned long long)kMoVd) &&
        (!full || p.Lc > (unsigned long long)kMoLive)) {
      if (lane == 0) p.ovf[gk] = 1;
      vfull = full = false;
    }
  }
  if ((bad || full || vfull) && lane == 0)
    atomicOr(p.o_flags + g, (bad ? 2u : 0u) | (full ? 8u : 0u) | (vfull ? 16u : 0u));
}

// vd_off's CSR invariants: entry 0 is 0, entries never decrease, the last is Dv.  A
// violation marks the group of the offending entry (flags bit 5); the fold clamps its reads anyway.
__global__ void map_orswot_vd_check_kernel(const u64 *vd_off, unsigned long long n, unsigned long long per_group,
                                           unsigned long long G, unsigned long long Dv, unsigned *flags) {
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i <= n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const u64 x = vd_off[i];
    const bool bad = (i == 0 && x != 0) || (i == n && x != Dv) || (i < n && vd_off[i + 1] < x);
    if (bad) {
      const unsigned long long g = i / per_group;
      atomicOr(flags + (g < G ? g : G - 1), 32u);
    }
  }
}

static size_t mo_lds() {
  return (size_t)kMoWaves * (kMoList * 8 + kMoLive * 4 + kMoRows * kWave * 8 + kMoVd * kWave * 8 + kMoVd * 8);
}

static size_t mo_wide_lds() { return (size_t)kMoWaves * (kMoList * 8 + kMoLive * 4 + kMoVd * kMoWideMw * 8); }

template <int APL>
static hipError_t launch_mo_wide(const MapOrswotPlan &p, hipStream_t s) {
  const unsigned long long blocks = (p.G * p.K + kMoWaves - 1) / kMoWaves;
  hipLaunchKernelGGL((map_orswot_wide_kernel<APL>), dim3((unsigned)blocks), dim3(kMoWaves * kWave), mo_wide_lds(), s, p);
  return hipGetLastError();
}

// the deep pass's LDS: one wave, its Map-remove lists and Vd nested member masks
static size_t mo_deep_lds(size_t Vd, size_t Mw, size_t Lc = kMoLive) { return kMoList * 8 + (Lc + 1) / 2 * 8 + Vd * Mw * 8; }
constexpr size_t kMoDeepLds = 160 * 1024;  // (one workgroup per CU at the most)

template <int APL>
static hipError_t launch_mo_deep(const MapOrswotPlan &p, hipStream_t s) {
  const size_t lds = mo_deep_lds(p.Vd, p.Mw, p.Lc);
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&map_orswot_wide_kernel<APL, true>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((map_orswot_wide_kernel<APL, true>), dim3((unsigned)(p.G * p.K)), dim3(kWave), lds, s, p);
  return hipGetLastError();
}

template <int MT, int SPL = 0, bool SHALLOW = false>
static hipError_t launch_mo(const MapOrswotPlan &p, hipStream_t s) {
  const unsigned long long blocks = (p.G * p.K + kMoWaves - 1) / kMoWaves;
  hipLaunchKernelGGL((map_orswot_fold_kernel<MT, SPL, SHALLOW>), dim3((unsigned)blocks), dim3(kMoWaves * kWave), mo_lds(),
                     s, p);
  return hipGetLastError();
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_map_orswot_lub_many(crdt_ctx *ctx, const crdt_map_orswot_batch *in, crdt_map_orswot_out *out) {
  if (ctx && ctx->mem_kind == CRDT_MEM_HOST) return crdt::map_orswot_lub_many_host(ctx, in, out);
  CRDT_CHECK_CTX(ctx);
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: NULL batch/out");
  const size_t G = in->G, R = in->R, K = in->K, M = in->M, A = in->A;
  if (G == 0 || K == 0 || A == 0) return CRDT_OK;
  if (A > 16 * (size_t)kWave) return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_lub_many: A = %zu > %d", A, 16 * kWave);
  if (M > 64 * (size_t)kMoWideMw)
    return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_lub_many: M = %zu > %d", M, 64 * kMoWideMw);
  if (!out->clock || !out->ec || !out->oc || (M && !out->ent) || !out->vd_n || !out->vd_clock || !out->vd_mem ||
      !out->flags)
    return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: NULL output");
  if (R > 0 && (!in->clock || !in->ec || !in->oc || (M && !in->ent) || !in->vd_off))
    return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: NULL input");
  if (R > 0 && in->Dv > 0 && (!in->vd_clock || !in->vd_mem))
    return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: Dv = %zu nested removes but NULL vd_clock / vd_mem", in->Dv);
  if (G * K > 0x7fffffffULL * (size_t)kMoWaves || R > 0xfffffffeULL)
    return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_lub_many: G*K or R too large");
  if (in->def_off && in->def_off[0] != 0) return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: def_off[0] must be 0");
  const size_t D = (in->def_off && G > 0) ? in->def_off[G] : 0;
  for (size_t i = 0; in->def_off && i < G; ++i)
    if (in->def_off[i + 1] < in->def_off[i])
      return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: def_off not non-decreasing");
  if (D > 0 && (!in->def_row || !in->def_clock || !in->def_keys || !out->def_keep || !out->def_keys))
    return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: deferred buffers missing");
  if (D > 0xffffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_lub_many: too many deferred");
  const size_t Vd = out->Vd ? out->Vd : (size_t)kMoVd, Mw0 = (M + 63) / 64 > 0 ? (M + 63) / 64 : 1;
  if (Vd < (size_t)kMoVd) return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: out->Vd = %zu < %d", Vd, kMoVd);
  if (Vd > (size_t)kMoVd && mo_deep_lds(Vd, Mw0) > kMoDeepLds)
    return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_lub_many: out->Vd = %zu nested slots of %zu mask words exceed the LDS",
                Vd, Mw0);
  // the deep pass's live list: every Map remove of the largest group (beyond kMoLive only when some
  // group has more), as far as the LDS holds it (past that, flags bit 3 as before)
  size_t Lc = kMoLive;
  for (size_t i = 0; in->def_off && i < G; ++i) Lc = std::max<size_t>(Lc, in->def_off[i + 1] - in->def_off[i]);
  while (Lc > (size_t)kMoLive && mo_deep_lds(Vd, Mw0, Lc) > kMoDeepLds) Lc = std::max<size_t>(kMoLive, Lc / 2);
  const bool deep = Vd > (size_t)kMoVd || Lc > (size_t)kMoLive;
  if (deep && G * K > 0x7fffffffULL)
    return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_lub_many: G*K too large for the deep pass");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const size_t Kw = (K + 63) / 64;
  MapOrswotPlan p{(const u64 *)in->clock, (const u64 *)in->ec, (const u64 *)in->oc, (const u64 *)in->ent,
                  (const u64 *)in->vd_off, (const u64 *)in->vd_clock, (const u64 *)in->vd_mem, in->Dv, G, R, K, M, A, Kw,
                  (M + 63) / 64 > 0 ? (M + 63) / 64 : 1, nullptr, in->def_row, (const u64 *)in->def_clock, (const u64 *)in->def_keys,
                  (u64 *)out->clock, (u64 *)out->ec, (u64 *)out->oc, (u64 *)out->ent, (u64 *)out->vd_clock,
                  (u64 *)out->vd_mem, out->vd_n, out->flags, Vd, nullptr, Lc};
  if (int rc = device_fill(ctx, out->flags, G * sizeof(unsigned), 0)) return rc;
  if (R == 0) {  // fold of nothing: Map::new()
    if (int rc = device_fill(ctx, out->clock, G * A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, out->ec, G * K * A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, out->oc, G * K * A * 8, 0)) return rc;
    if (M)
      if (int rc = device_fill(ctx, out->ent, G * K * M * A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, out->vd_n, G * K * sizeof(unsigned), 0)) return rc;
  } else {
    // scratch: [def_off (G+1) when D > 0][the deep pass's per-(g, k) markers when Vd > 16]
    const size_t so = D > 0 ? (G + 1) * sizeof(size_t) : 0, sv = deep ? G * K : 0;
    if (so + sv) {
      if (int rc = ensure_scratch(ctx, so + sv)) return rc;
    }
    if (D > 0) {
      if (int rc = stage_h2d(ctx, ctx->scratch, in->def_off, (G + 1) * sizeof(size_t))) return rc;
      p.def_off = reinterpret_cast<const size_t *>(ctx->scratch);
    }
    if (sv) {
      p.ovf = static_cast<uint8_t *>(ctx->scratch) + so;
      if (int rc = device_fill(ctx, p.ovf, sv, 0)) return rc;
    }
    {
      const unsigned long long n = (unsigned long long)G * R * K;
      const unsigned blocks = (unsigned)std::min<unsigned long long>((n + 256) / 256, 4096);
      hipLaunchKernelGGL(map_orswot_vd_check_kernel, dim3(blocks), dim3(256), 0, ctx->stream, p.vd_off, n,
                         (unsigned long long)R * K, (unsigned long long)G, (unsigned long long)in->Dv, out->flags);
      CRDT_HIP(ctx, hipGetLastError());
    }
    timing_begin(ctx, "map_orswot_fold");
    // (member rows past M are zero and still joined: the register capacity follows M)
    // the whole-chunk skip (round 5, opt-in: CRDT_TUNE mocs=1) for A = 32 / 16 / 8 and up to 4 members
    // past A = 64 or M = 32 (or with CRDT_TUNE mowide=1): the wide kernel, APL actors per lane
    const bool wide = ctx->tune.map_orswot_wide || A > (size_t)kWave || M > 32;
    const int spl = ctx->tune.map_orswot_cs && M <= 4 ? (A == 32 ? 2 : (A == 16 ? 4 : (A == 8 ? 8 : 0))) : 0;
    const hipError_t he = wide ? (A <= 64    ? launch_mo_wide<1>(p, ctx->stream)
                                  : A <= 128 ? launch_mo_wide<2>(p, ctx->stream)
                                  : A <= 256 ? launch_mo_wide<4>(p, ctx->stream)
                                  : A <= 512 ? launch_mo_wide<8>(p, ctx->stream)
                                             : launch_mo_wide<16>(p, ctx->stream))
                          : spl == 2 ? launch_mo<4, 2>(p, ctx->stream)
                          : spl == 4 ? launch_mo<4, 4>(p, ctx->stream)
                          : spl == 8 ? launch_mo<4, 8>(p, ctx->stream)
                          : M <= 4 && G * K >= kMoShallowWaves ? launch_mo<4, 0, true>(p, ctx->stream)
                          : M <= 4   ? launch_mo<4>(p, ctx->stream)
                          : M <= 8   ? launch_mo<8>(p, ctx->stream)
                                     : launch_mo<32>(p, ctx->stream);
    if (he != hipSuccess) return hip_fail(ctx, he, "map_orswot_fold_kernel launch");
    if (sv) {  // the deep pass: the marked keys again, exactly, with all Vd nested slots
      const hipError_t hd = A <= 64    ? launch_mo_deep<1>(p, ctx->stream)
                            : A <= 128 ? launch_mo_deep<2>(p, ctx->stream)
                            : A <= 256 ? launch_mo_deep<4>(p, ctx->stream)
                            : A <= 512 ? launch_mo_deep<8>(p, ctx->stream)
                                       : launch_mo_deep<16>(p, ctx->stream);
      if (hd != hipSuccess) return hip_fail(ctx, hd, "map_orswot deep pass launch");
    }
    timing_end(ctx);
  }
  if (D == 0) return CRDT_OK;
  DefPlan q{};  // the Map's surviving removes (!(rm <= C_final)), identical clocks merged
  q.G = G;
  q.D = D;
  q.M = K;
  q.A = A;
  q.Mw = Kw;
  q.def_clock = (const u64 *)in->def_clock;
  q.def_members = (const u64 *)in->def_keys;
  q.out_clock = (const u64 *)out->clock;
  q.out_entries = nullptr;
  q.apply_ceiling = 0;
  q.out_keep = out->def_keep;
  q.out_members = (u64 *)out->def_keys;
  return launch_deferred(ctx, in->def_off, q);
}
