// Map<K, Map<K2, MVReg<u64>>> lub_many (round 5): the nested type of the reference's own Map tests
// (TMap, test/map.rs:10; TestMap, src/map.rs:359).  The outer Map::merge (map.rs:140-220) carries an
// inner Map as its value, whose merge is Map::merge again (with MVReg::merge, mvreg.rs:112-128, as the
// innermost value merge) and whose forget is Map's Causal::forget (map.rs:85-114: entry clocks,
// values, deferred clocks and the inner Map's own clock).  As for every Map value type the fold
// acc = Map::new(); for r: acc.merge(r) is not associative, so each outer key is folded in replica
// order (exact for any input): one wave per (group, outer key), lane l = actors l + 64 j (A <= 256, round 6).
//
// Step r on the key's state (outer clock C, entry clock e, inner Map: clock ic, entry clocks iec[j],
// MVReg slots in Vec order, inner deferred removes) with replica r's (c2, e2, ic2, iec2, values, D2):
//  - outer entry clock: the branch-free join of map_counter.hip, e' = max(e == e2 ? e : 0,
//    forget(e2, C), forget(e, c2)), and the case's forget clock X (removed_information :151 /
//    we_deleted :200 / deleted :185); an empty e' drops the entry without touching its value;
//  - both present: the inner Map::merge — per inner key the same join over the inner clocks (ic, ic2),
//    MVReg::merge of the slots then their forget by the inner case's clock; then apply_keyset_rm of
//    each of the replica's inner removes against ic (forget, defer iff !(rm <= ic)), ic |= ic2, and
//    apply_deferred (every held remove forgets its keys again, stays iff !(rm <= ic));  only the
//    replica holds the key: its inner Map;  then the inner Map forgets X (Causal::forget);
//  - the outer removes naming the key (apply_keyset_rm / apply_deferred, :213-219, :318-348): one
//    forget by their max — the entry clock, and the inner Map while the entry stays;
//  - C |= c2 and the outer deferral test (witness thresholds, as map_counter.hip / map_orswot.hip).
// The inner Map's rows live in the key's own output rows (global memory, touched by this wave only);
// its deferred removes (<= 16) and slot counts in LDS.  Map::forget collects the deferred removes into
// a new HashMap: two whose clocks become equal keep one entry with the later one's keys at the earlier
// one's place (the reference's HashMap order is unspecified; this is the oracle's dict order —
// parity unpinned for that collision).  Lanes past A hold 0 in every row, so they never change a vote.
#include "common.hpp"

namespace crdt {

constexpr int kNmWaves = 4;   // key waves per workgroup
constexpr int kNmList = 256;  // outer removes naming the key, gathered per window (row << 32 | index)
constexpr int kNmLive = 256;  // live outer removes per key (flags bit 3 past it)
constexpr int kNmRows = 8;    // live outer-remove rows cached in LDS
constexpr int kNmId = 16;     // inner deferred removes per key state (flags bit 4 past it)
constexpr int kNmVs = 8;      // MVReg slots per inner key in the fold state (flags bit 6 past it)
constexpr int kNmVin = 8;     // MVReg slots per inner key in the input
constexpr int kNmK2 = 256;    // inner keys (round 6: 256 — key sets of inner removes as K2w <= 4 mask words)
constexpr int kNmKw = kNmK2 / 64;

struct NestedMapPlan {
  const u64 *clock, *ec, *ic, *iec, *ivc, *ivv;  // (G,R,A) (G,R,K,A) (G,R,K,A) (G,R,K,K2,A) (G,R,K,K2,V,A) (G,R,K,K2,V)
  const u64 *id_off, *id_clock, *id_keys;        // inner deferred CSR over (g, r, k); id_keys [Di][K2w]
  unsigned long long Di;
  unsigned long long G, R, K, K2, V, A, Kw;
  const size_t *def_off;  // device copy (G+1), or null
  const uint32_t *def_row;
  const u64 *def_clock, *def_keys;
  u64 *o_clock, *o_ec, *o_ic, *o_iec, *o_ivc, *o_ivv;
  unsigned *o_nval, *o_id_n;
  u64 *o_id_clock, *o_id_keys;
  unsigned *o_flags;
  // u64 words of LDS per wave for the key's inner Map state (iec [K2][A], slots [K2][8][A], values
  // [K2][8]) and for a staged copy of the replica's inner Map (iec, slots, values); 0 = off (the state
  // then lives in the key's output rows, the replica is read from HBM where it is used)
  unsigned long long xs_state, xs_stage;
  unsigned wpb;  // key waves per workgroup (kNmWaves; fewer for the wide instances' LDS rows)
  unsigned K2w;  // inner-key mask words, ceil(K2 / 64) (1 up to 64 inner keys: the round-5 layout)
  // round 6: the output's inner deferred slots per key (>= kNmId; the first kNmId in LDS during the
  // fold) and when Id > kNmId a per-(g, k) marker: the key's list passed kNmId, re-fold it deep
  unsigned long long Id;
  uint8_t *ovf;
  unsigned long long Lc;  // the deep pass's live outer-remove capacity per key (>= kNmLive)
  unsigned long long Vs;  // the output's MVReg slots per inner key (>= kNmVs; the deep pass holds all)
};
constexpr int kNmVsMax = 64;  // (the deep pass's kept-slot masks are one word)

// A clock across the wave: lane l holds actors l + 64 j, j < APL (A <= 64 APL; round 6: APL 2 and 4 take
// the reference's TMap domain of u8 actors).  Words past A are 0 in every row, so they never change a
// vote.
template <int APL>
struct NVc {
  u64 w[APL];
};
template <int APL>
__device__ __forceinline__ NVc<APL> nv_fill(u64 v) {
  NVc<APL> x;
#pragma unroll
  for (int j = 0; j < APL; ++j) x.w[j] = v;
  return x;
}
template <int APL>
__device__ __forceinline__ NVc<APL> nv_zero() { return nv_fill<APL>(0ull); }
template <int APL>
__device__ __forceinline__ NVc<APL> nv_ld(const u64 *row, int lane, unsigned long long A) {
  NVc<APL> x;
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = (unsigned long long)lane + 64ull * j;
    x.w[j] = a < A ? row[a] : 0ull;
  }
  return x;
}
template <int APL>
__device__ __forceinline__ void nv_st(u64 *row, const NVc<APL> &x, int lane, unsigned long long A) {
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = (unsigned long long)lane + 64ull * j;
    if (a < A) row[a] = x.w[j];
  }
}
// an LDS row array [i][64 APL] (word j of lane l at 64 j + l)
template <int APL>
__device__ __forceinline__ NVc<APL> nv_lr(const u64 *base, int i, int lane) {
  NVc<APL> x;
#pragma unroll
  for (int j = 0; j < APL; ++j) x.w[j] = base[(unsigned long long)i * kWave * APL + 64ull * j + lane];
  return x;
}
template <int APL>
__device__ __forceinline__ void nv_lw(u64 *base, int i, const NVc<APL> &x, int lane) {
#pragma unroll
  for (int j = 0; j < APL; ++j) base[(unsigned long long)i * kWave * APL + 64ull * j + lane] = x.w[j];
}
template <int APL>
__device__ __forceinline__ bool nm_nz(const NVc<APL> &x) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) b = b || x.w[j] != 0;
  return __ballot(b) != 0;
}
template <int APL>  // VClock::forget, per actor
__device__ __forceinline__ NVc<APL> nm_fg(const NVc<APL> &x, const NVc<APL> &c) {
  NVc<APL> r;
#pragma unroll
  for (int j = 0; j < APL; ++j) r.w[j] = x.w[j] > c.w[j] ? x.w[j] : 0ull;
  return r;
}
template <int APL>
__device__ __forceinline__ NVc<APL> nm_max(const NVc<APL> &x, const NVc<APL> &y) {
  NVc<APL> r;
#pragma unroll
  for (int j = 0; j < APL; ++j) r.w[j] = x.w[j] > y.w[j] ? x.w[j] : y.w[j];
  return r;
}
// per actor: x where x == y, else z (the branch-free entry join's first case)
template <int APL>
__device__ __forceinline__ NVc<APL> nm_sel_eq(const NVc<APL> &x, const NVc<APL> &y, const NVc<APL> &z) {
  NVc<APL> r;
#pragma unroll
  for (int j = 0; j < APL; ++j) r.w[j] = x.w[j] == y.w[j] ? x.w[j] : z.w[j];
  return r;
}
template <int APL>  // some actor with x > y
__device__ __forceinline__ bool nm_gt_any(const NVc<APL> &x, const NVc<APL> &y) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) b = b || x.w[j] > y.w[j];
  return __ballot(b) != 0;
}
template <int APL>  // some actor with x >= y
__device__ __forceinline__ bool nm_ge_any(const NVc<APL> &x, const NVc<APL> &y) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) b = b || x.w[j] >= y.w[j];
  return __ballot(b) != 0;
}
// VClock partial order, whole clock: x < y (x <= y everywhere and x != y somewhere)
template <int APL>
__device__ __forceinline__ bool nm_lt(const NVc<APL> &x, const NVc<APL> &y) {
  bool gt = false, ne = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    gt = gt || x.w[j] > y.w[j];
    ne = ne || x.w[j] != y.w[j];
  }
  return !__ballot(gt) && __ballot(ne);
}
template <int APL>
__device__ __forceinline__ bool nm_eq(const NVc<APL> &x, const NVc<APL> &y) {
  bool ne = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) ne = ne || x.w[j] != y.w[j];
  return !__ballot(ne);
}

// an inner-key set (the same in every lane): words past K2w stay 0
struct NKm {
  u64 w[kNmKw];
};
__device__ __forceinline__ bool km_any(const NKm &k) {
  u64 x = 0;
#pragma unroll
  for (int i = 0; i < kNmKw; ++i) x |= k.w[i];
  return x != 0;
}

// DEEP (round 6, the exact overflow pass): one wave per workgroup re-folds only the keys the first
// pass marked in p.ovf, with p.Id inner deferred slots — their rm rows in the key's own output rows
// (each lane reads back only the words it wrote), their key sets in LDS (Id * kNmKw words).
template <int APL, bool DEEP = false>
__global__ __launch_bounds__(kNmWaves * kWave) void map_nested_fold_kernel(NestedMapPlan p) {
  using Vc = NVc<APL>;
  extern __shared__ u64 lds[];
  const int lane = (int)(threadIdx.x % kWave), wv = (int)(threadIdx.x / kWave);
  const unsigned long long gk = (unsigned long long)blockIdx.x * p.wpb + wv;
  if (wv >= (int)p.wpb || gk >= p.G * p.K) return;  // (whole waves; nothing below synchronises the workgroup)
  if constexpr (DEEP) {
    if (!p.ovf[gk]) return;
  }
  const unsigned long long g = gk / p.K, k = gk % p.K, A = p.A, R = p.R, K = p.K, K2 = p.K2, V = p.V;
  const int cap = DEEP ? (int)p.Id : kNmId;  // inner deferred slots
  const unsigned long long LC = DEEP ? p.Lc : (unsigned long long)kNmLive;  // live outer removes held
  const unsigned long long WQ = kNmList + (LC + 1) / 2 + kNmRows * kWave * APL +
                                (DEEP ? 0ull : (unsigned long long)kNmId * kWave * APL) +
                                (unsigned long long)cap * kNmKw + kNmK2 / 8;
  u64 *lst = lds + (unsigned long long)wv * (WQ + p.xs_state + p.xs_stage);
  u64 *const xst = lst + WQ, *const xsg = xst + p.xs_state;  // (LDS state, staged replica)
  uint32_t *live = reinterpret_cast<uint32_t *>(lst + kNmList);
  u64 *rows = lst + kNmList + (LC + 1) / 2;  // [kNmRows][64 APL] live outer-remove rows
  u64 *drow = rows + kNmRows * kWave * APL; // [kNmId][64 APL] inner deferred rm rows (not DEEP)
  u64 *dkey = drow + (DEEP ? 0 : kNmId * kWave * APL);  // [cap][kNmKw] their inner key sets
  uint8_t *nv = reinterpret_cast<uint8_t *>(dkey + (unsigned long long)cap * kNmKw);  // [K2] MVReg slots held per inner key
  u64 *const gdr = p.o_id_clock + gk * p.Id * p.A;  // (DEEP) [Id][A] the rm rows in the output
  auto dr_ld = [&](int i) -> NVc<APL> {
    if constexpr (DEEP) return nv_ld<APL>(gdr + (unsigned long long)i * p.A, lane, p.A);
    else return nv_lr<APL>(drow, i, lane);
  };
  auto dr_st = [&](int i, const NVc<APL> &x) {
    if constexpr (DEEP) nv_st<APL>(gdr + (unsigned long long)i * p.A, x, lane, p.A);
    else nv_lw<APL>(drow, i, x, lane);
  };
  const unsigned K2w = p.K2w;
  auto km_lr = [&](int i) -> NKm {  // held remove i's key set
    NKm k;
#pragma unroll
    for (int x = 0; x < kNmKw; ++x) k.w[x] = dkey[i * kNmKw + x];
    return k;
  };
  auto km_lw = [&](int i, const NKm &k) {
    if (lane == 0)
#pragma unroll
      for (int x = 0; x < kNmKw; ++x) dkey[i * kNmKw + x] = k.w[x];
  };
  auto km_in = [&](unsigned long long d) -> NKm {  // input remove d's key set (id_keys [Di][K2w])
    NKm k;
#pragma unroll
    for (int x = 0; x < kNmKw; ++x) k.w[x] = (unsigned)x < K2w ? p.id_keys[d * K2w + x] : 0ull;
    return k;
  };
  const Vc Z = nv_zero<APL>();
  auto ld = [&](const u64 *row) -> Vc { return nv_ld<APL>(row, lane, A); };
  auto st = [&](u64 *row, const Vc &x) { nv_st<APL>(row, x, lane, A); };

  // ---- the outer removes naming key k, in replica order (map_orswot.hip's walk)
  const unsigned long long d0 = p.def_off ? p.def_off[g] : 0, d1 = p.def_off ? p.def_off[g + 1] : 0;
  unsigned long long dc = d0;
  int nl = 0, li = 0;
  bool bad = false;  // def_row not non-decreasing or >= R (flags bit 1)
  u64 last_row = 0;
  auto refill = [&]() {
    nl = 0;
    li = 0;
    while (dc < d1 && nl + kWave <= kNmList) {
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
  bool full = false, dfull = false, vfull = false;
  int na = 0;
  auto live_row = [&](int i) -> Vc {
    return i < kNmRows ? nv_lr<APL>(rows, i, lane) : ld(p.def_clock + (d0 + live[i]) * A);
  };
  auto put_row = [&](int i, const Vc &x) {
    if (i < kNmRows) nv_lw<APL>(rows, i, x, lane);
  };
  Vc rk = Z, T = nv_fill<APL>(~0ull);

  // ---- the key's state: outer C, e; the inner Map's clock ic (registers), rows in the output
  Vc C = Z, e = Z, ic = Z;
  int nd = 0;  // inner deferred removes held (uniform)
  // (generic pointers: the LDS copy when it fits, else the key's own output rows)
  u64 *const iec_o = p.xs_state ? xst : p.o_iec + gk * K2 * A;
  // MVReg slots: VSt the state rows' stride (the output's Vs, or kNmVs in the LDS copy), VC those held
  const unsigned long long VSt = p.xs_state ? (unsigned long long)kNmVs : p.Vs;
  const int VC = DEEP ? (int)p.Vs : kNmVs;
  u64 *const ivc_o = p.xs_state ? xst + K2 * A : p.o_ivc + gk * K2 * VSt * A;
  u64 *const ivv_o = p.xs_state ? xst + K2 * A + K2 * kNmVs * A : p.o_ivv + gk * K2 * VSt;
  for (unsigned long long j = 0; j < K2; ++j) {
    st(iec_o + j * A, Z);
    if (lane == 0) nv[j] = 0;
  }

  // MVReg::forget (mvreg.rs:88-104) of inner key j's slots by x, compacted in order
  auto vals_forget = [&](unsigned long long j, const Vc &x) {
    const int n = __builtin_amdgcn_readfirstlane((int)nv[j]);
    int o = 0;
    for (int s = 0; s < n; ++s) {
      const Vc c = nm_fg(ld(ivc_o + (j * VSt + s) * A), x);
      if (!nm_nz(c)) continue;
      const u64 v = ivv_o[j * VSt + s];
      st(ivc_o + (j * VSt + o) * A, c);
      ivv_o[j * VSt + o] = v;  // (every lane stores the value: each later reads back its own store)
      ++o;
    }
    if (lane == 0) nv[j] = (uint8_t)o;
  };
  // inner apply_keyset_rm's forget (map.rs:320-333): the keys' entry clocks, their values while they stay
  auto forget_keys = [&](const Vc &rm, const NKm &kset) {
#pragma unroll
    for (int x = 0; x < kNmKw; ++x) {
    u64 km = kset.w[x];
    while (km) {
      const unsigned long long j = 64ull * x + (unsigned long long)__builtin_ctzll(km);
      km &= km - 1;
      if (j >= K2) break;
      const Vc ej = ld(iec_o + j * A);
      if (!nm_nz(ej)) continue;
      const Vc ej2 = nm_fg(ej, rm);
      st(iec_o + j * A, ej2);
      if (!nm_nz(ej2)) {
        if (lane == 0) nv[j] = 0;
      } else {
        vals_forget(j, rm);
      }
    }
    }
  };
  auto id_add = [&](const Vc &rm, const NKm &km) {  // deferred.entry(clock).or_default().append(keys) (map.rs:341-342)
    for (int i = 0; i < nd; ++i) {
      if (nm_eq(dr_ld(i), rm)) {
        NKm mm = km_lr(i);
#pragma unroll
        for (int x = 0; x < kNmKw; ++x) mm.w[x] |= km.w[x];
        km_lw(i, mm);
        return;
      }
    }
    if (nd < cap) {
      dr_st(nd, rm);
      km_lw(nd, km);
      ++nd;
    } else {
      dfull = true;
    }
  };
  // the inner Map's Causal::forget (map.rs:85-114)
  auto inner_forget = [&](const Vc &x) {
    if (!nm_nz(x)) return;  // (forget by the empty clock is the identity)
    for (unsigned long long j = 0; j < K2; ++j) {
      const Vc ej = ld(iec_o + j * A);
      if (!nm_nz(ej)) continue;
      const Vc ej2 = nm_fg(ej, x);
      st(iec_o + j * A, ej2);
      if (!nm_nz(ej2)) {
        if (lane == 0) nv[j] = 0;
      } else {
        vals_forget(j, x);
      }
    }
    int o = 0;
    for (int i = 0; i < nd; ++i) {
      const Vc r2 = nm_fg(dr_ld(i), x);
      const NKm ki = km_lr(i);
      if (!nm_nz(r2)) continue;
      int jj = 0;
      for (; jj < o; ++jj)  // equal to a kept one: the later keys at the earlier place (collect())
        if (nm_eq(dr_ld(jj), r2)) break;
      if (jj < o) {
        km_lw(jj, ki);
        continue;
      }
      dr_st(o, r2);
      km_lw(o, ki);
      ++o;
    }
    nd = o;
    ic = nm_fg(ic, x);
  };

  // replica r's inner Map at key k
  auto rin_iec = [&](unsigned long long r) { return p.iec + ((g * R + r) * K + k) * K2 * A; };
  auto rin_ivc = [&](unsigned long long r) { return p.ivc + ((g * R + r) * K + k) * K2 * V * A; };
  auto rin_ivv = [&](unsigned long long r) { return p.ivv + ((g * R + r) * K + k) * K2 * V; };
  // replica r's inner rows (iec, slots, values: three contiguous blocks) copied to LDS with every
  // load in flight at once; returns the three (generic) base pointers
  struct Rin {
    const u64 *iec, *ivc, *ivv;
  };
  auto rin = [&](unsigned long long r) -> Rin {
    if (!p.xs_stage) return Rin{rin_iec(r), rin_ivc(r), rin_ivv(r)};
    const unsigned long long n1 = K2 * A, n2 = K2 * V * A, n3 = K2 * V;
    const u64 *s1 = rin_iec(r), *s2 = rin_ivc(r), *s3 = rin_ivv(r);
#pragma unroll 4
    for (unsigned long long i = (unsigned long long)lane; i < n1 + n2 + n3; i += kWave)
      xsg[i] = i < n1 ? s1[i] : (i < n1 + n2 ? s2[i - n1] : s3[i - n1 - n2]);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // (other lanes read these words)
    return Rin{xsg, xsg + n1, xsg + n1 + n2};
  };
  auto rin_id = [&](unsigned long long r, u64 &lo, u64 &hi) {
    const u64 *po = p.id_off + (g * R + r) * K + k;
    u64 a = __builtin_amdgcn_readfirstlane((unsigned)po[0]) | ((u64)__builtin_amdgcn_readfirstlane((unsigned)(po[0] >> 32)) << 32);
    u64 b = __builtin_amdgcn_readfirstlane((unsigned)po[1]) | ((u64)__builtin_amdgcn_readfirstlane((unsigned)(po[1] >> 32)) << 32);
    b = b < p.Di ? b : p.Di;  // (a malformed id_off never reads past the rows: flags bit 5)
    lo = a < b ? a : b;
    hi = b;
  };

  // the replica's inner Map as the key's value (map.rs:193-208): clock, entries, slots, deferred
  auto inner_load = [&](unsigned long long r, const Vc &ic2) {
    ic = ic2;
    const Rin rn = rin(r);
    const u64 *ri = rn.iec, *rc = rn.ivc, *rv = rn.ivv;
    for (unsigned long long j = 0; j < K2; ++j) {
      const Vc ej = ld(ri + j * A);
      st(iec_o + j * A, ej);
      int o = 0;
      if (nm_nz(ej)) {
        for (unsigned long long s = 0; s < V; ++s) {
          const Vc c = ld(rc + (j * V + s) * A);
          if (!nm_nz(c)) continue;
          if (o < VC) {
            st(ivc_o + (j * VSt + o) * A, c);
            ivv_o[j * VSt + o] = rv[j * V + s];
            ++o;
          } else {
            vfull = true;
          }
        }
      }
      if (lane == 0) nv[j] = (uint8_t)o;
    }
    nd = 0;
    u64 lo, hi;
    rin_id(r, lo, hi);
    for (u64 d = lo; d < hi; ++d) id_add(ld(p.id_clock + d * A), km_in(d));
  };

  // the inner Map::merge (map.rs:140-220) of replica r's inner Map (clock ic2) into the state
  auto inner_merge = [&](unsigned long long r, const Vc &ic2) {
    const Rin rn = rin(r);
    const u64 *ri = rn.iec, *rc = rn.ivc, *rv = rn.ivv;
    for (unsigned long long j = 0; j < K2; ++j) {
      const Vc ej = ld(iec_o + j * A), e2j = ld(ri + j * A);
      const bool q1 = nm_nz(ej), q2 = nm_nz(e2j);
      if (!q1 && !q2) continue;
      const Vc enj = nm_sel_eq(ej, e2j, nm_max(nm_fg(e2j, ic), nm_fg(ej, ic2)));
      if (!nm_nz(enj)) {  // dropped (or not added): no value merge
        if (q1) {
          st(iec_o + j * A, Z);
          if (lane == 0) nv[j] = 0;
        }
        continue;
      }
      const Vc xj = nm_fg(q1 ? (q2 ? nm_max(ej, e2j) : ic2) : ic, enj);
      if constexpr (DEEP) {  // the same merge with our slots read from the rows one at a time (up to Vs)
        // (the replica's V slots are read from its rows too: V may pass kNmVin here)
        const int n1 = q1 ? __builtin_amdgcn_readfirstlane((int)nv[j]) : 0, n2 = q2 ? (int)V : 0;
        u64 m2 = 0;  // the replica's non-empty slots
        for (int t = 0; t < n2; ++t)
          if (nm_nz(ld(rc + (j * V + t) * A))) m2 |= 1ull << t;
        u64 keep1 = 0;  // ours not strictly below one of the replica's
        for (int s2 = 0; s2 < n1; ++s2) {
          const Vc c = ld(ivc_o + (j * VSt + s2) * A);
          bool dominated = false;
          for (int t = 0; t < n2 && !dominated; ++t)
            if (((m2 >> t) & 1ull) && nm_lt(c, ld(rc + (j * V + t) * A))) dominated = true;
          if (!dominated) keep1 |= 1ull << s2;
        }
        u64 keep2 = 0;  // the replica's not strictly below or equal to a kept one of ours
        for (int t = 0; t < n2; ++t) {
          if (!((m2 >> t) & 1ull)) continue;
          const Vc ct = ld(rc + (j * V + t) * A);
          bool drop = false;
          for (int s2 = 0; s2 < n1 && !drop; ++s2) {
            if (!((keep1 >> s2) & 1ull)) continue;
            const Vc c = ld(ivc_o + (j * VSt + s2) * A);
            if (nm_lt(ct, c) || nm_eq(ct, c)) drop = true;
          }
          if (!drop) keep2 |= 1ull << t;
        }
        int o = 0;  // kept slots forgotten by xj, in order (o <= s2: compacted in place)
        for (int s2 = 0; s2 < n1; ++s2) {
          if (!((keep1 >> s2) & 1ull)) continue;
          const Vc c = nm_fg(ld(ivc_o + (j * VSt + s2) * A), xj);
          if (!nm_nz(c)) continue;
          const u64 v = ivv_o[j * VSt + s2];
          st(ivc_o + (j * VSt + o) * A, c);
          ivv_o[j * VSt + o] = v;
          ++o;
        }
        for (int t = 0; t < n2; ++t) {
          if (!((keep2 >> t) & 1ull)) continue;
          const Vc c = nm_fg(ld(rc + (j * V + t) * A), xj);
          if (!nm_nz(c)) continue;
          if (o < VC) {
            st(ivc_o + (j * VSt + o) * A, c);
            ivv_o[j * VSt + o] = rv[j * V + t];
            ++o;
          } else {
            vfull = true;
          }
        }
        if (lane == 0) nv[j] = (uint8_t)o;
        st(iec_o + j * A, enj);
        continue;
      }
      // the slots: ours (Vec order), then the replica's (MVReg::merge, mvreg.rs:112-128), forgotten by xj
      // (every register array is indexed by unrolled constants only: the replica's slots keep their
      // own positions with a validity mask m2 instead of being compacted by a running count, which
      // made the compiler spill the arrays to scratch)
      Vc cs[kNmVs], co[kNmVin];
      u64 vs[kNmVs], vo[kNmVin];
      const int n1 = q1 ? __builtin_amdgcn_readfirstlane((int)nv[j]) : 0;
      unsigned m2 = 0;
#pragma unroll
      for (int s = 0; s < kNmVs; ++s) {
        cs[s] = s < n1 ? ld(ivc_o + (j * VSt + s) * A) : Z;
        vs[s] = s < n1 ? ivv_o[j * VSt + s] : 0;
      }
#pragma unroll
      for (int s = 0; s < kNmVin; ++s) {
        co[s] = Z;
        vo[s] = 0;
      }
      if (q2) {
#pragma unroll
        for (int s = 0; s < kNmVin; ++s) {
          if ((unsigned long long)s < V) {
            const Vc c = ld(rc + (j * V + s) * A);
            if (nm_nz(c)) {  // (an empty slot is no value)
              co[s] = c;
              vo[s] = rv[j * V + s];
              m2 |= 1u << s;
            }
          }
        }
      }
      // self's values not strictly below one of other's; then other's not strictly below or equal
      // to a kept one of ours
      unsigned keep1 = 0, keep2 = 0;
#pragma unroll
      for (int s = 0; s < kNmVs; ++s) {
        if (s >= n1) break;
        bool dominated = false;
#pragma unroll
        for (int t = 0; t < kNmVin; ++t) {
          if (!(m2 >> t) || dominated) break;  // (uniform exits: the unrolled pairs past the values cost nothing)
          if (((m2 >> t) & 1u) && nm_lt(cs[s], co[t])) dominated = true;
        }
        if (!dominated) keep1 |= 1u << s;
      }
#pragma unroll
      for (int t = 0; t < kNmVin; ++t) {
        if (!(m2 >> t)) break;
        if (!((m2 >> t) & 1u)) continue;
        bool drop = false;
#pragma unroll
        for (int s = 0; s < kNmVs; ++s) {
          if (s >= n1 || drop) break;
          if (((keep1 >> s) & 1u) && (nm_lt(co[t], cs[s]) || nm_eq(co[t], cs[s]))) drop = true;
        }
        if (!drop) keep2 |= 1u << t;
      }
      // write the merged slots forgotten by xj, in order
      int o = 0;
#pragma unroll
      for (int s = 0; s < kNmVs; ++s) {
        if (!((keep1 >> s) & 1u)) continue;
        const Vc c = nm_fg(cs[s], xj);
        if (!nm_nz(c)) continue;
        st(ivc_o + (j * VSt + o) * A, c);  // (the slots were read into registers above)
        ivv_o[j * VSt + o] = vs[s];
        ++o;
      }
#pragma unroll
      for (int t = 0; t < kNmVin; ++t) {
        if (!((keep2 >> t) & 1u)) continue;
        const Vc c = nm_fg(co[t], xj);
        if (!nm_nz(c)) continue;
        if (o < kNmVs) {
          st(ivc_o + (j * VSt + o) * A, c);
          ivv_o[j * VSt + o] = vo[t];
          ++o;
        } else {
          vfull = true;
        }
      }
      if (lane == 0) nv[j] = (uint8_t)o;
      st(iec_o + j * A, enj);
    }
    // apply_keyset_rm of the replica's inner removes, against the pre-merge inner clock (:213-215)
    u64 lo, hi;
    rin_id(r, lo, hi);
    for (u64 d = lo; d < hi; ++d) {
      const Vc rm = ld(p.id_clock + d * A);
      const NKm km = km_in(d);
      forget_keys(rm, km);
      if (nm_gt_any(rm, ic)) id_add(rm, km);
    }
    ic = nm_max(ic, ic2);  // (:217)
    // apply_deferred (:219, :311-316): every held remove forgets its keys again, stays iff !(rm <= ic)
    int o = 0;
    for (int i = 0; i < nd; ++i) {
      const Vc rm = dr_ld(i);
      const NKm km = km_lr(i);
      forget_keys(rm, km);
      if (nm_gt_any(rm, ic)) {
        if (o != i) {
          dr_st(o, rm);
          km_lw(o, km);
        }
        ++o;
      }
    }
    nd = o;
  };

  // ---- one outer replica step
  auto step = [&](unsigned long long r, const Vc &c2, const Vc &e2, const Vc &ic2) __attribute__((always_inline)) {
    const bool p1 = nm_nz(e), p2 = nm_nz(e2);
    const Vc en = nm_sel_eq(e, e2, nm_max(nm_fg(e2, C), nm_fg(e, c2)));
    const bool stays = nm_nz(en);
    if (stays && (p1 || p2)) {
      const Vc X = nm_fg(p1 ? (p2 ? nm_max(e, e2) : c2) : C, en);
      if (p1 && p2) inner_merge(r, ic2);  // our_entry.val.merge(entry.val) (map.rs:183)
      else if (p2) inner_load(r, ic2);    // the replica's entry (:193-208)
      inner_forget(X);
    }
    e = en;
    // the outer removes: replica r's own naming k (apply_keyset_rm) and the live ones (apply_deferred)
    bool chg = false;
    Vc f = rk;
    const unsigned r32 = (unsigned)r;
    if (nxt <= r32) {
      do {
        const unsigned idx = (unsigned)lst[li];
        const Vc rm = ld(p.def_clock + (d0 + idx) * A);
        f = nm_max(f, rm);
        if ((unsigned long long)na < LC) {
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
    if (na > 0 && nm_nz(e)) {
      e = nm_fg(e, f);
      if (nm_nz(e)) inner_forget(f);  // entry.val.forget only while the entry stays (map.rs:321-330)
    }
    C = nm_max(C, c2);
    if (na > 0 && (chg || nm_ge_any(C, T))) {  // outer live set re-test (witness thresholds)
      bool changed = chg;
      T = nv_fill<APL>(~0ull);
      for (int i = 0; i < na;) {
        const Vc rm = live_row(i);
        bool held = false;  // the first actor with rm > C (the witness) holds the remove's threshold
#pragma unroll
        for (int j = 0; j < APL; ++j) {
          const u64 m = __ballot(rm.w[j] > C.w[j]);
          if (!held && m) {
            const int wl = __builtin_ctzll(m);
            T.w[j] = lane == wl && rm.w[j] < T.w[j] ? rm.w[j] : T.w[j];
            held = true;
          }
        }
        if (held) {
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
        rk = Z;
        for (int i = 0; i < na; ++i) rk = nm_max(rk, live_row(i));
      }
    }
  };

  // ---- replica rows (c2, e2, ic2) through a register ring, DEPTH steps ahead
  constexpr int DEPTH = 4;
  const u64 *pc = p.clock + g * R * A, *pe = p.ec + (g * R * K + k) * A, *pi = p.ic + (g * R * K + k) * A;
  Vc c2r[DEPTH], e2r[DEPTH], i2r[DEPTH];
  auto load_step = [&](int s, unsigned long long r) {
    const unsigned long long rr = r < R ? r : R - 1;
    c2r[s] = ld(pc + rr * A);
    e2r[s] = ld(pe + rr * K * A);
    i2r[s] = ld(pi + rr * K * A);
  };
#pragma unroll
  for (int s = 0; s < DEPTH; ++s) load_step(s, (unsigned long long)s);
  // (the DEPTH ring slots written out with constant indices: an unroll pragma over the inlined step
  // is refused as too large at APL > 1, which left the ring in scratch)
  auto ring = [&](auto sc, unsigned long long r0) __attribute__((always_inline)) -> bool {
    constexpr int s = decltype(sc)::value;
    const unsigned long long r = r0 + s;
    if (r >= R) return false;
    const Vc c2 = c2r[s], e2 = e2r[s], i2 = i2r[s];
    load_step(s, r + DEPTH);
    step(r, c2, e2, i2);
    return true;
  };
  static_assert(DEPTH == 4, "the ring below is written for 4 slots");
  for (unsigned long long r0 = 0; r0 < R; r0 += DEPTH) {
    if (!ring(std::integral_constant<int, 0>{}, r0)) break;
    if (!ring(std::integral_constant<int, 1>{}, r0)) break;
    if (!ring(std::integral_constant<int, 2>{}, r0)) break;
    if (!ring(std::integral_constant<int, 3>{}, r0)) break;
  }

  // ---- egress: the key's entry (an empty entry clock: absent, inner rows 0), the group's clock
  const bool pf = nm_nz(e);
  st(p.o_ec + gk * A, e);
  st(p.o_ic + gk * A, pf ? ic : Z);
  u64 *const oiec = p.o_iec + gk * K2 * A, *const oivc = p.o_ivc + gk * K2 * p.Vs * A;
  u64 *const oivv = p.o_ivv + gk * K2 * p.Vs;
  for (unsigned long long j = 0; j < K2; ++j) {
    const int n = pf ? __builtin_amdgcn_readfirstlane((int)nv[j]) : 0;
    st(oiec + j * A, pf ? ld(iec_o + j * A) : Z);  // (the same word when the state is the output)
    for (int s = 0; s < (int)p.Vs; ++s) {  // the held slots, then zeros
      const Vc c = s < n ? ld(ivc_o + (j * VSt + s) * A) : Z;
      const u64 v = s < n ? ivv_o[j * VSt + s] : 0ull;
      st(oivc + (j * p.Vs + s) * A, c);
      oivv[j * p.Vs + s] = v;
    }
    if (lane == 0) p.o_nval[gk * K2 + j] = (unsigned)n;
  }
  if (k == 0) st(p.o_clock + g * A, C);
  const int no = pf ? nd : 0;
  for (int i = 0; i < no; ++i) {
    if constexpr (!DEEP) st(p.o_id_clock + (gk * p.Id + i) * A, dr_ld(i));  // (DEEP: the rows are there)
    if (lane == 0)
      for (unsigned x = 0; x < K2w; ++x) p.o_id_keys[(gk * p.Id + i) * K2w + x] = dkey[i * kNmKw + x];
  }
  if (lane == 0) p.o_id_n[gk] = (unsigned)no;
  if constexpr (!DEEP) {
    // past the LDS slots / the live list, where the deep pass has room for both: it re-folds this key
    if ((dfull || full || vfull) && p.ovf && (!dfull || p.Id > (unsigned long long)kNmId) &&
        (!full || p.Lc > (unsigned long long)kNmLive) && (!vfull || p.Vs > (unsigned long long)kNmVs)) {
      if (lane == 0) p.ovf[gk] = 1;
      dfull = full = vfull = false;
    }
  }
  if ((bad || full || dfull || vfull) && lane == 0)
    atomicOr(p.o_flags + g, (bad ? 2u : 0u) | (full ? 8u : 0u) | (dfull ? 16u : 0u) | (vfull ? 64u : 0u));
}

// id_off's CSR invariants: entry 0 is 0, entries never decrease, the last is Di (flags bit 5)
__global__ void map_nested_id_check_kernel(const u64 *off, unsigned long long n, unsigned long long per_group,
                                           unsigned long long G, unsigned long long Di, unsigned *flags) {
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i <= n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const u64 x = off[i];
    const bool bad = (i == 0 && x != 0) || (i == n && x != Di) || (i < n && off[i + 1] < x);
    if (bad) {
      const unsigned long long g = i / per_group;
      atomicOr(flags + (g < G ? g : G - 1), 32u);
    }
  }
}

// LDS bytes per key wave beyond the optional state / staging rows
static size_t nm_lds(int apl) {
  return kNmList * 8 + kNmLive * 4 + kNmRows * kWave * 8 * apl + kNmId * kWave * 8 * apl + kNmId * kNmKw * 8 + kNmK2;
}
// the deep pass's LDS (one wave): no rm rows (they live in the output), Id key sets
static size_t nm_deep_lds(int apl, size_t Id, size_t Lc = kNmLive) {
  return kNmList * 8 + (Lc + 1) / 2 * 8 + kNmRows * kWave * 8 * apl + Id * kNmKw * 8 + kNmK2;
}
constexpr size_t kNmDeepLds = 160 * 1024;

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_map_nested_lub_many(crdt_ctx *ctx, const crdt_map_nested_batch *in, crdt_map_nested_out *out) {
  if (ctx && ctx->mem_kind == CRDT_MEM_HOST) return crdt::map_nested_lub_many_host(ctx, in, out);
  CRDT_CHECK_CTX(ctx);
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: NULL batch/out");
  const size_t G = in->G, R = in->R, K = in->K, K2 = in->K2, V = in->V, A = in->A;
  if (G == 0 || K == 0 || A == 0) return CRDT_OK;
  if (A > 4 * (size_t)kWave) return fail(ctx, CRDT_EUNSUPPORTED, "map_nested_lub_many: A = %zu > %d", A, 4 * kWave);
  if (K2 > (size_t)kNmK2) return fail(ctx, CRDT_EUNSUPPORTED, "map_nested_lub_many: K2 = %zu > %d", K2, kNmK2);
  if (V > (size_t)kNmVsMax) return fail(ctx, CRDT_EUNSUPPORTED, "map_nested_lub_many: V = %zu > %d", V, kNmVsMax);
  if (!out->clock || !out->ec || !out->ic || (K2 && (!out->iec || !out->ivc || !out->ivv || !out->nval)) ||
      !out->id_n || !out->id_clock || !out->id_keys || !out->flags)
    return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: NULL output");
  if (R > 0 && (!in->clock || !in->ec || !in->ic || !in->id_off || (K2 && !in->iec) || (K2 && V && (!in->ivc || !in->ivv))))
    return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: NULL input");
  if (R > 0 && in->Di > 0 && (!in->id_clock || !in->id_keys))
    return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: Di = %zu inner removes but NULL id_clock / id_keys", in->Di);
  if (G * K > 0x7fffffffULL * (size_t)kNmWaves || R > 0xfffffffeULL)
    return fail(ctx, CRDT_EUNSUPPORTED, "map_nested_lub_many: G*K or R too large");
  if (in->def_off && in->def_off[0] != 0) return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: def_off[0] must be 0");
  const size_t D = (in->def_off && G > 0) ? in->def_off[G] : 0;
  for (size_t i = 0; in->def_off && i < G; ++i)
    if (in->def_off[i + 1] < in->def_off[i])
      return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: def_off not non-decreasing");
  if (D > 0 && (!in->def_row || !in->def_clock || !in->def_keys || !out->def_keep || !out->def_keys))
    return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: deferred buffers missing");
  if (D > 0xffffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_nested_lub_many: too many deferred");
  const size_t Id = out->Id ? out->Id : (size_t)kNmId;  // inner deferred slots per key in the output
  const int apl0 = A <= (size_t)kWave ? 1 : (A <= 2 * (size_t)kWave ? 2 : 4);
  if (Id < (size_t)kNmId) return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: out->Id = %zu < %d", Id, kNmId);
  if (Id > (size_t)kNmId && (nm_deep_lds(apl0, Id) > kNmDeepLds || G * K > 0x7fffffffULL))
    return fail(ctx, CRDT_EUNSUPPORTED, "map_nested_lub_many: out->Id = %zu inner slots past the deep pass's limits", Id);
  // the deep pass's live list: every outer remove of the largest group (beyond kNmLive only when some
  // group has more), as far as the LDS holds it (past that, flags bit 3 as before)
  size_t Lc = kNmLive;
  for (size_t i = 0; in->def_off && i < G; ++i) Lc = std::max<size_t>(Lc, in->def_off[i + 1] - in->def_off[i]);
  while (Lc > (size_t)kNmLive && nm_deep_lds(apl0, Id, Lc) > kNmDeepLds) Lc = std::max<size_t>(kNmLive, Lc / 2);
  const size_t Vs = out->Vs ? out->Vs : (size_t)kNmVs;  // MVReg slots per inner key in the output
  if (Vs < (size_t)kNmVs || Vs > (size_t)kNmVsMax)
    return fail(ctx, CRDT_EUNSUPPORTED, "map_nested_lub_many: out->Vs = %zu outside %d..%d", Vs, kNmVs, kNmVsMax);
  // inputs with more than kNmVin slots per inner key go to the deep pass alone (every key marked)
  const bool deep_only = V > (size_t)kNmVin;
  if (deep_only && Vs < V) return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: out->Vs = %zu < V = %zu", Vs, V);
  const bool deep = deep_only || Id > (size_t)kNmId || Lc > (size_t)kNmLive || Vs > (size_t)kNmVs;
  if (deep && G * K > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_nested_lub_many: G*K too large");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const size_t Kw = (K + 63) / 64;
  NestedMapPlan p{(const u64 *)in->clock, (const u64 *)in->ec, (const u64 *)in->ic, (const u64 *)in->iec,
                  (const u64 *)in->ivc, (const u64 *)in->ivv, (const u64 *)in->id_off, (const u64 *)in->id_clock,
                  (const u64 *)in->id_keys, in->Di, G, R, K, K2, V, A, Kw, nullptr, in->def_row,
                  (const u64 *)in->def_clock, (const u64 *)in->def_keys, (u64 *)out->clock, (u64 *)out->ec,
                  (u64 *)out->ic, (u64 *)out->iec, (u64 *)out->ivc, (u64 *)out->ivv, out->nval, out->id_n,
                  (u64 *)out->id_clock, (u64 *)out->id_keys, out->flags};
  p.K2w = K2 > 64 ? (unsigned)((K2 + 63) / 64) : 1u;
  p.Id = Id;
  p.ovf = nullptr;
  p.Lc = Lc;
  p.Vs = Vs;
  if (int rc = device_fill(ctx, out->flags, G * sizeof(unsigned), 0)) return rc;
  if (R == 0) {  // fold of nothing: Map::new()
    if (int rc = device_fill(ctx, out->clock, G * A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, out->ec, G * K * A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, out->ic, G * K * A * 8, 0)) return rc;
    if (K2) {
      if (int rc = device_fill(ctx, out->iec, G * K * K2 * A * 8, 0)) return rc;
      if (int rc = device_fill(ctx, out->ivc, G * K * K2 * Vs * A * 8, 0)) return rc;
      if (int rc = device_fill(ctx, out->ivv, G * K * K2 * Vs * 8, 0)) return rc;
      if (int rc = device_fill(ctx, out->nval, G * K * K2 * sizeof(unsigned), 0)) return rc;
    }
    if (int rc = device_fill(ctx, out->id_n, G * K * sizeof(unsigned), 0)) return rc;
  } else {
    // scratch: [def_off (G+1) when D > 0][the deep pass's per-(g, k) markers when Id > 16]
    const size_t so = D > 0 ? (G + 1) * sizeof(size_t) : 0, sv = deep ? G * K : 0;
    if (so + sv) {
      if (int rc = ensure_scratch(ctx, so + sv)) return rc;
    }
    if (D > 0) {
      if (int rc = stage_h2d(ctx, ctx->scratch, in->def_off, (G + 1) * sizeof(size_t))) return rc;
      p.def_off = reinterpret_cast<const size_t *>(ctx->scratch);
    }
    if (sv) {  // (deep_only: every key marked, the first pass skipped)
      p.ovf = static_cast<uint8_t *>(ctx->scratch) + so;
      if (int rc = device_fill(ctx, p.ovf, sv, deep_only ? 1 : 0)) return rc;
    }
    {
      const unsigned long long n = (unsigned long long)G * R * K;
      const unsigned blocks = (unsigned)std::min<unsigned long long>((n + 256) / 256, 4096);
      hipLaunchKernelGGL(map_nested_id_check_kernel, dim3(blocks), dim3(256), 0, ctx->stream, p.id_off, n,
                         (unsigned long long)R * K, (unsigned long long)G, (unsigned long long)in->Di, out->flags);
      CRDT_HIP(ctx, hipGetLastError());
    }
    // LDS per wave beyond the fixed lists: the inner state, then the staged replica rows, while the
    // block fits (up to 160 KiB when one block per CU already gives every key a SIMD of its own,
    // else 80 KiB so that two blocks share a CU as without them)
    p.xs_state = p.xs_stage = 0;
    const int apl = A <= (size_t)kWave ? 1 : (A <= 2 * (size_t)kWave ? 2 : 4);  // actor words per lane
    const void *kfn = apl == 1 ? reinterpret_cast<const void *>(&map_nested_fold_kernel<1>)
                      : apl == 2 ? reinterpret_cast<const void *>(&map_nested_fold_kernel<2>)
                                 : reinterpret_cast<const void *>(&map_nested_fold_kernel<4>);
    // waves per workgroup: 4, fewer where the wide rows would pass 64 KiB (APL 2: 2 x 27 KiB, 4: 51 KiB)
    const unsigned wpb = apl == 1 ? kNmWaves : (apl == 2 ? 2 : 1);
    p.wpb = wpb;
    size_t lds = nm_lds(apl) * wpb;
    if (ctx->tune.map_nested_lds && K2 > 0) {
      const size_t base = nm_lds(apl), cap = G * K <= 4 * (size_t)ctx->cu_count ? 160 * 1024 : 80 * 1024;
      const size_t st_w = K2 * (1 + kNmVs) * A + K2 * kNmVs, sg_w = K2 * (1 + V) * A + K2 * V;
      if ((base + st_w * 8) * wpb <= cap) p.xs_state = st_w;
      if ((base + (p.xs_state + sg_w) * 8) * wpb <= cap) p.xs_stage = sg_w;
      lds = (base + (p.xs_state + p.xs_stage) * 8) * wpb;
      if (lds > 64 * 1024) {
        const hipError_t ae = hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (ae != hipSuccess) {
          (void)hipGetLastError();
          p.xs_state = p.xs_stage = 0;
          lds = nm_lds(apl) * wpb;
        }
      }
    }
    timing_begin(ctx, "map_nested_fold");
    const unsigned long long blocks = (G * K + wpb - 1) / wpb;
    if (deep_only) {
    } else if (apl == 1)
      hipLaunchKernelGGL(map_nested_fold_kernel<1>, dim3((unsigned)blocks), dim3(wpb * kWave), lds, ctx->stream, p);
    else if (apl == 2)
      hipLaunchKernelGGL(map_nested_fold_kernel<2>, dim3((unsigned)blocks), dim3(wpb * kWave), lds, ctx->stream, p);
    else
      hipLaunchKernelGGL(map_nested_fold_kernel<4>, dim3((unsigned)blocks), dim3(wpb * kWave), lds, ctx->stream, p);
    hipError_t he = hipGetLastError();
    if (he == hipSuccess && sv) {  // the deep pass: the marked keys again, exactly, with all Id slots
      NestedMapPlan q = p;
      q.xs_state = q.xs_stage = 0;
      q.wpb = 1;
      const size_t dl = nm_deep_lds(apl, Id, Lc);
      const void *dfn = apl == 1 ? reinterpret_cast<const void *>(&map_nested_fold_kernel<1, true>)
                        : apl == 2 ? reinterpret_cast<const void *>(&map_nested_fold_kernel<2, true>)
                                   : reinterpret_cast<const void *>(&map_nested_fold_kernel<4, true>);
      if (dl > 64 * 1024) he = hipFuncSetAttribute(dfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dl);
      if (he == hipSuccess) {
        const dim3 dg((unsigned)(G * K)), db(kWave);
        if (apl == 1) hipLaunchKernelGGL((map_nested_fold_kernel<1, true>), dg, db, dl, ctx->stream, q);
        else if (apl == 2) hipLaunchKernelGGL((map_nested_fold_kernel<2, true>), dg, db, dl, ctx->stream, q);
        else hipLaunchKernelGGL((map_nested_fold_kernel<4, true>), dg, db, dl, ctx->stream, q);
        he = hipGetLastError();
      }
    }
    timing_end(ctx);
    if (he != hipSuccess) return hip_fail(ctx, he, "map_nested_fold_kernel launch");
  }
  if (D == 0) return CRDT_OK;
  DefPlan q{};  // the outer Map's surviving removes (!(rm <= C_final)), identical clocks merged
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
