// Batched CmRDT::apply of Map<K, Orswot<M>> (round 5): Map::apply (map.rs:119-137) with the nested
// Orswot's apply inside (orswot.rs:55-79: Add { dot, members } skipped when the Orswot's clock has
// seen the dot, else every member's clock and the Orswot clock apply it, then apply_deferred
// :281-286; Rm { clock, members } -> apply_rm :230-250), the Map's apply_keyset_rm (:318-348, the
// value forgotten by Orswot::forget :150-183) and apply_deferred (:311-316).  State s applies its
// ops [op_off[s], op_off[s+1]) in order, in place, on the crdt_map_orswot_lub_many output layout.
//
// One wave per state, lane l holding actors l + 64 j (j < APL) of every row: the Map clock in
// registers, the Map's deferred removes (rm clock + key bitmap) in LDS for the whole stream.  The
// nested Orswot of a key lives in its rows (oc, ent, vd_clock, vd_mem, vd_n); an op that touches
// its nested deferred list stages the list's member masks in LDS (the words read by every lane),
// and every global word is read back only by the lane that wrote it (row words by the lane of
// their actor, mask word w by lane w % 64, vd_n by every lane).
#include "common.hpp"

namespace crdt {

// waves per SIMD asked of the register allocator for A <= 128 (build option; A/B in
// profiles/r05_vapply_wpe_ab.log); the wider instances keep the compiler's choice (they would spill)
// op headers batched 64 at a time into lanes and read by v_readlane (build option; 0 = one global
// read of each field per op)
#ifndef CRDT_MOA_HDR
#define CRDT_MOA_HDR 1
#endif
// waves per SIMD asked of the register allocator (build option): 5 with the header batch (6.10 vs
// 6.31 ms at 6, profiles/r05_moa_w5_ab.log; 6 was the best before it, r05_vapply_wpe_ab.log)
#ifndef CRDT_MOA_WPE
#define CRDT_MOA_WPE 5
#endif
#ifndef CRDT_MOA_WPE1  // (the pass-1 instance, Dcap past the LDS slots)
#define CRDT_MOA_WPE1 CRDT_MOA_WPE
#endif

constexpr int kMoaVd = 16;    // nested deferred slots per key by default (crdt_map_orswot_states.Vd)
constexpr int kMoaMw = 16;    // member-mask words (M <= 1,024)
constexpr size_t kMoaDl = 16;  // the Map's deferred slots held in LDS per state (the rest of Dcap in place)

struct MapOrswotApplyPlan {
  u64 *clock, *ec, *oc, *ent, *vd_clock, *vd_mem;
  unsigned *vd_n;
  unsigned long long N, K, M, A, Mw, Kw, Dcap;
  unsigned long long Dl;  // the Map's deferred slots held in LDS (<= Dcap); slots Dl .. Dcap-1 stay in place
  u64 *def_clock, *def_keys;
  unsigned *def_count;
  const u64 *op_off;
  const uint8_t *kind, *vkind;
  const uint32_t *actor, *key, *vactor;
  const u64 *counter, *vcounter;
  const uint32_t *clk_row;
  const u64 *clk_pool;
  unsigned long long n_clk_rows;
  const u64 *key_off;
  const uint32_t *keys;
  unsigned long long n_keys;
  const u64 *mem_off;
  const uint32_t *mems;
  unsigned long long n_mems, n_ops;
  unsigned *status;
  unsigned wpb;
  u64 *resume = nullptr;  // [N] (Dcap > Dl): op offset where a state continues in pass 2, or kMoaDone
  unsigned long long Vd = kMoaVd;  // nested deferred slots per key (round 6: any, their masks in LDS)
  unsigned long long VW = (unsigned long long)kMoaVd * kMoaMw;  // LDS words for them: max(256, Vd * Mw)
};
constexpr u64 kMoaDone = ~0ull;

__device__ __forceinline__ unsigned rl32(unsigned x, int i) { return (unsigned)__builtin_amdgcn_readlane((int)x, i); }
__device__ __forceinline__ u64 rl64(u64 x, int i) {
  return ((u64)rl32((unsigned)(x >> 32), i) << 32) | rl32((unsigned)x, i);
}

// TIER false: every state, the Map's deferred list in the Dl LDS slots only; a state whose list
// needs slot Dl (Dcap > Dl) stores itself and records the op to continue from (resume[s]).  TIER
// true: those states alone, slots past Dl used in place in the caller's slot arrays.  (One body with
// the branch compiles the slot accesses to flat instructions and slows every state; see
// csrc/map_counter_apply.hip.)
template <int APL, int PASS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(APL <= 2 ? (PASS == 1 ? CRDT_MOA_WPE1 : CRDT_MOA_WPE) : 1))) void map_orswot_apply_kernel(MapOrswotApplyPlan p) {
  extern __shared__ u64 lds[];
  const int lane = (int)(threadIdx.x % kWave), wv = (int)(threadIdx.x / kWave);
  const unsigned long long s = (unsigned long long)blockIdx.x * p.wpb + wv;
  if (wv >= (int)p.wpb || s >= p.N) return;  // (whole waves)
  constexpr bool TIER = PASS == 2;
  if constexpr (TIER) {
    if (p.resume[s] == kMoaDone) return;
  }
  const unsigned long long A = p.A, K = p.K, M = p.M, Mw = p.Mw, Kw = p.Kw, Dcap = p.Dcap, Dl = p.Dl;
  const unsigned long long WQ = Dl * (A + Kw) + p.VW;
  // The Map's deferred removes: slots d < Dl in LDS, slots Dl <= d < Dcap in the caller's own slot
  // arrays (global memory: a long list runs slower, never incomplete below Dcap)
  u64 *sclk = lds + (unsigned long long)wv * WQ;  // [Dl][A] the Map's rm clocks
  u64 *skey = sclk + Dl * A;                       // [Dl][Kw] their key bitmaps
  u64 *smsk = skey + Dl * Kw;                      // [Vd][Mw] the current key's nested member masks
  const unsigned long long ob = p.op_off[s], oe = p.op_off[s + 1];
  unsigned dcnt = p.def_count[s];
  if (dcnt > Dcap || oe < ob || oe > p.n_ops) {
    if (lane == 0) {
      p.status[s] = (dcnt > Dcap ? 4u : 0u) | (oe < ob || oe > p.n_ops ? 8u : 0u);
      if (PASS == 1) p.resume[s] = kMoaDone;
    }
    return;  // state left untouched
  }
  if constexpr (PASS == 1) {
    if (dcnt > Dl) {  // arrives with more removes than the LDS slots: the whole stream in pass 2
      if (lane == 0) {
        p.status[s] = 0;
        p.resume[s] = 0;
      }
      return;
    }
  }
  // pass 2 continues with pass 1's status bits; its first deferred pass is full (exact either way)
  unsigned st = TIER ? p.status[s] : 0u, peak = dcnt;  // peak: the most slots held (vacated ones are zeroed)
  const unsigned long long start = TIER ? ob + p.resume[s] : ob;
  // pass 1: the op where pass 2 continues (offset within the state's stream; < 2^32, checked on the host)
  unsigned resume_at = 0xffffffffu;
  auto word = [&](int j) { return (unsigned long long)lane + 64ull * j; };
  u64 *gclk = p.def_clock + s * Dcap * A, *gkey = p.def_keys + s * Dcap * Kw;
  // (d is wave-uniform; the pass-1 body never reaches d >= Dl)
  auto clk = [&](unsigned d, unsigned long long a) -> u64 {
    if (TIER && d >= Dl) return gclk[d * A + a];
    return sclk[d * A + a];
  };
  auto set_clk = [&](unsigned d, unsigned long long a, u64 v) {
    if (TIER && d >= Dl) gclk[d * A + a] = v;
    else sclk[d * A + a] = v;
  };
  auto key = [&](unsigned d, unsigned long long w) -> u64 {
    if (TIER && d >= Dl) return gkey[d * Kw + w];
    return skey[d * Kw + w];
  };
  auto set_key = [&](unsigned d, unsigned long long w, u64 v) {
    if (TIER && d >= Dl) gkey[d * Kw + w] = v;
    else skey[d * Kw + w] = v;
  };
  u64 *C = p.clock + s * A;
  u64 c[APL];
#pragma unroll
  for (int j = 0; j < APL; ++j) c[j] = word(j) < A ? C[word(j)] : 0ull;
  for (unsigned d = 0; d < dcnt && d < Dl; ++d) {
    for (unsigned long long a = (unsigned long long)lane; a < A; a += kWave) sclk[d * A + a] = gclk[d * A + a];
    for (unsigned long long w = (unsigned long long)lane; w < Kw; w += kWave) skey[d * Kw + w] = gkey[d * Kw + w];
  }
  auto ldrow = [&](const u64 *row, u64 (&x)[APL]) {
#pragma unroll
    for (int j = 0; j < APL; ++j) x[j] = word(j) < A ? row[word(j)] : 0ull;
  };
  auto strow = [&](u64 *row, const u64 (&x)[APL]) {
#pragma unroll
    for (int j = 0; j < APL; ++j)
      if (word(j) < A) row[word(j)] = x[j];
  };
  auto any_nz = [&](const u64 (&x)[APL]) {
    bool b = false;
#pragma unroll
    for (int j = 0; j < APL; ++j) b = b || x[j] != 0;
    return __ballot(b) != 0;
  };
  auto leq = [&](const u64 (&x)[APL], const u64 (&y)[APL]) {  // x <= y (every word)
    bool b = false;
#pragma unroll
    for (int j = 0; j < APL; ++j) b = b || x[j] > y[j];
    return __ballot(b) == 0;
  };
  auto word_of = [&](const u64 (&x)[APL], unsigned a) -> u64 {  // x[a] (uniform)
    u64 v = 0;
#pragma unroll
    for (int j = 0; j < APL; ++j)
      if ((unsigned)j == a / 64) v = x[j];
    return __shfl(v, (int)(a % 64));
  };
  auto bump = [&](u64 *row, unsigned a, u64 cnt) {  // VClock::apply(dot) on a global row
    if ((unsigned long long)lane == a % 64) {
      u64 *q = row + a;
      if (*q < cnt) *q = cnt;
    }
  };

  // ---- the nested Orswot of key k (its rows) ----------------------------------------------------
  struct Keyp {
    u64 *ec, *oc, *ent, *vc, *vm;
    unsigned *vn;
  };
  auto keyp = [&](unsigned long long k) {
    const unsigned long long sk = s * K + k;
    return Keyp{p.ec + sk * A, p.oc + sk * A, p.ent + sk * M * A, p.vd_clock + sk * p.Vd * A,
                p.vd_mem + sk * p.Vd * Mw, p.vd_n + sk};
  };
  auto stage_masks = [&](const Keyp &q, unsigned n) {  // global -> LDS (lane w % 64 moves word w)
    for (unsigned i = 0; i < n; ++i)
      for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) smsk[i * Mw + w] = q.vm[i * Mw + w];
  };
  auto unstage_masks = [&](const Keyp &q, unsigned n) {  // LDS -> global, and the count (every lane)
    for (unsigned i = 0; i < n; ++i)
      for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) q.vm[i * Mw + w] = smsk[i * Mw + w];
    *q.vn = n;
  };
  // Orswot::apply_rm's member forget (orswot.rs:231-238): the members of mask row `mrow` (LDS or
  // a member list) forget r; an emptied member row is absent (all zero)
  auto forget_members_mask = [&](const Keyp &q, const u64 *mrow, const u64 (&r)[APL]) {
    for (unsigned long long w = 0; w < Mw; ++w) {
      u64 bits = mrow[w];
      while (bits) {
        const unsigned long long m = w * 64 + (unsigned long long)__builtin_ctzll(bits);
        bits &= bits - 1;
        if (m >= M) break;
        u64 x[APL];
        ldrow(q.ent + m * A, x);
#pragma unroll
        for (int j = 0; j < APL; ++j) x[j] = x[j] > r[j] ? x[j] : 0ull;
        strow(q.ent + m * A, x);
      }
    }
  };
  // the nested apply_deferred (orswot.rs:281-286) over the staged list: every remove forgets its
  // members again and stays while !(rm <= oc); returns the new count
  auto nested_apply_deferred = [&](const Keyp &q, unsigned n, const u64 (&oc)[APL]) -> unsigned {
    unsigned o = 0;
    for (unsigned i = 0; i < n; ++i) {
      u64 r[APL];
      ldrow(q.vc + (unsigned long long)i * A, r);
      forget_members_mask(q, smsk + i * Mw, r);
      if (leq(r, oc)) continue;
      if (o != i) {
        strow(q.vc + (unsigned long long)o * A, r);
        for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) smsk[o * Mw + w] = smsk[i * Mw + w];
      }
      ++o;
    }
    return o;
  };
  // Orswot::forget (orswot.rs:150-183) of key k's value by r (the entry stays)
  auto value_forget = [&](const Keyp &q, const u64 (&r)[APL]) {
    u64 x[APL];
    ldrow(q.oc, x);
#pragma unroll
    for (int j = 0; j < APL; ++j) x[j] = x[j] > r[j] ? x[j] : 0ull;
    strow(q.oc, x);
    for (unsigned long long m = 0; m < M; ++m) {
      ldrow(q.ent + m * A, x);
#pragma unroll
      for (int j = 0; j < APL; ++j) x[j] = x[j] > r[j] ? x[j] : 0ull;
      strow(q.ent + m * A, x);
    }
    const unsigned n = min((unsigned)p.Vd, *q.vn);  // (a count past the slots: clamped)
    if (n == 0) return;
    stage_masks(q, n);
    unsigned o = 0;
    for (unsigned i = 0; i < n; ++i) {
      ldrow(q.vc + (unsigned long long)i * A, x);
#pragma unroll
      for (int j = 0; j < APL; ++j) x[j] = x[j] > r[j] ? x[j] : 0ull;
      if (!any_nz(x)) continue;  // forgotten
      unsigned jj = 0;
      for (; jj < o; ++jj) {  // equal to a kept one: the later members at the earlier place
        u64 y[APL];
        ldrow(q.vc + (unsigned long long)jj * A, y);
        bool ne = false;
#pragma unroll
        for (int j = 0; j < APL; ++j) ne = ne || y[j] != x[j];
        if (!__ballot(ne)) break;
      }
      if (jj < o) {
        for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) smsk[jj * Mw + w] = smsk[i * Mw + w];
        continue;
      }
      strow(q.vc + (unsigned long long)o * A, x);
      if (o != i)
        for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) smsk[o * Mw + w] = smsk[i * Mw + w];
      ++o;
    }
    unstage_masks(q, o);
  };
  // the Map's apply_keyset_rm on key k (map.rs:319-333): forget its entry by r, drop an emptied one
  // (all rows zero, no nested removes), else forget its value
  auto key_rm = [&](unsigned long long k, const u64 (&r)[APL]) {
    const Keyp q = keyp(k);
    u64 e[APL];
    ldrow(q.ec, e);
    if (!any_nz(e)) return;  // no entry
#pragma unroll
    for (int j = 0; j < APL; ++j) e[j] = e[j] > r[j] ? e[j] : 0ull;
    strow(q.ec, e);
    if (any_nz(e)) {
      value_forget(q, r);
      return;
    }
    u64 z[APL];
#pragma unroll
    for (int j = 0; j < APL; ++j) z[j] = 0;
    strow(q.oc, z);
    for (unsigned long long m = 0; m < M; ++m) strow(q.ent + m * A, z);
    *q.vn = 0u;
  };
  // apply_deferred (map.rs:311-316): full on its first run, then restricted to the Up's own key (the
  // only rows an Up changes; forgets are idempotent and commute — see csrc/map_counter_apply.hip)
  bool full = true;
  auto map_apply_deferred = [&](unsigned long long kk) {
    unsigned o = 0;
    for (unsigned d = 0; d < dcnt; ++d) {
      u64 r[APL];
#pragma unroll
      for (int j = 0; j < APL; ++j) r[j] = word(j) < A ? clk(d, word(j)) : 0ull;
      for (unsigned long long w = full ? 0 : kk / 64; w < (full ? Kw : kk / 64 + 1); ++w) {
        u64 bits = key(d, w) & (full ? ~0ull : 1ull << (kk % 64));
        while (bits) {
          const unsigned long long k = w * 64 + (unsigned long long)__builtin_ctzll(bits);
          bits &= bits - 1;
          if (k < K) key_rm(k, r);
        }
      }
      if (leq(r, c)) continue;  // no longer deferred
      if (o != d) {
        for (unsigned long long a = (unsigned long long)lane; a < A; a += kWave) set_clk(o, a, clk(d, a));
        for (unsigned long long w = (unsigned long long)lane; w < Kw; w += kWave) set_key(o, w, key(d, w));
      }
      ++o;
    }
    dcnt = o;
    full = false;
  };

  // Op headers in batches of 64: lane i loads op o0 + i's fields (coalesced, all in flight
  // together) and op o's fields reach the wave by v_readlane, not by a global round trip per op.
  for (unsigned long long o0 = start; o0 < oe; o0 += kWave) {
    const unsigned long long mo = o0 + (unsigned long long)lane;
    const bool hin = CRDT_MOA_HDR && mo < oe;
    const unsigned h_kind = hin ? p.kind[mo] : 0u, h_a = hin ? p.actor[mo] : 0u, h_k = hin ? p.key[mo] : 0u;
    const unsigned h_vk = hin ? p.vkind[mo] : 0u, h_va = hin ? p.vactor[mo] : 0u;
    const u64 h_c = hin ? p.counter[mo] : 0ull, h_vc = hin ? p.vcounter[mo] : 0ull;
    const u64 h_mb = hin ? p.mem_off[mo] : 0ull, h_me = hin ? p.mem_off[mo + 1] : 0ull;
    const unsigned h_rr = hin ? p.clk_row[mo] : 0u;
    const u64 h_kb = hin ? p.key_off[mo] : 0ull, h_ke = hin ? p.key_off[mo + 1] : 0ull;
    const int nb = (int)(oe - o0 < (unsigned long long)kWave ? oe - o0 : (unsigned long long)kWave);
  for (int hi = 0; hi < nb; ++hi) {
    const unsigned long long o = o0 + (unsigned long long)hi;
    const unsigned kind = CRDT_MOA_HDR ? rl32(h_kind, hi) : p.kind[o];
    if (kind == 0) {  // ---- Map Op::Up { dot, key, op: an Orswot op }
      const unsigned a = CRDT_MOA_HDR ? rl32(h_a, hi) : p.actor[o];
      const unsigned long long k = CRDT_MOA_HDR ? rl32(h_k, hi) : p.key[o];
      const u64 cnt = CRDT_MOA_HDR ? rl64(h_c, hi) : p.counter[o];
      const unsigned vk = CRDT_MOA_HDR ? rl32(h_vk, hi) : p.vkind[o];
      const u64 mb = CRDT_MOA_HDR ? rl64(h_mb, hi) : p.mem_off[o], me = CRDT_MOA_HDR ? rl64(h_me, hi) : p.mem_off[o + 1];
      if (a >= A || k >= K || vk > 1 || me < mb || me > p.n_mems) {
        st |= 2u;
        continue;
      }
      if (word_of(c, a) >= cnt) continue;  // seen (map.rs:123-126)
      const Keyp q = keyp(k);
      bump(q.ec, a, cnt);  // entry.clock.apply(dot) (an absent entry: its rows are the default Orswot)
      u64 oc[APL];
      ldrow(q.oc, oc);
      if (vk == 0) {  // Orswot Op::Add { dot, members }
        const unsigned va = CRDT_MOA_HDR ? rl32(h_va, hi) : p.vactor[o];
        const u64 vc = CRDT_MOA_HDR ? rl64(h_vc, hi) : p.vcounter[o];
        if (va >= A) {
          st |= 2u;
        } else if (word_of(oc, va) < vc) {  // (seen by the Orswot's clock: nothing)
          for (u64 i = mb; i < me; ++i) {
            const unsigned long long m = p.mems[i];
            if (m < M) bump(q.ent + m * A, va, vc);
            else st |= 2u;
          }
          bump(q.oc, va, vc);
#pragma unroll
          for (int j = 0; j < APL; ++j)
            if ((unsigned)j == va / 64 && (unsigned long long)lane == va % 64 && oc[j] < vc) oc[j] = vc;
          const unsigned n = min((unsigned)p.Vd, *q.vn);  // (a count past the slots: clamped)
          if (n > 0) {
            stage_masks(q, n);
            unstage_masks(q, nested_apply_deferred(q, n, oc));
          }
        }
      } else {  // Orswot Op::Rm { clock, members } -> apply_rm
        const unsigned rr = CRDT_MOA_HDR ? rl32(h_rr, hi) : p.clk_row[o];
        if (rr >= p.n_clk_rows) {
          st |= 2u;
        } else {
          u64 r[APL];
          ldrow(p.clk_pool + (unsigned long long)rr * A, r);
          for (u64 i = mb; i < me; ++i) {
            const unsigned long long m = p.mems[i];
            if (m >= M) {
              st |= 2u;
              continue;
            }
            u64 x[APL];
            ldrow(q.ent + m * A, x);
#pragma unroll
            for (int j = 0; j < APL; ++j) x[j] = x[j] > r[j] ? x[j] : 0ull;
            strow(q.ent + m * A, x);
          }
          if (!leq(r, oc)) {  // !(clock <= self.clock): deferred, an equal clock's members unioned
            unsigned n = min((unsigned)p.Vd, *q.vn);
            stage_masks(q, n);
            int slot = -1;
            for (unsigned i = 0; i < n && slot < 0; ++i) {
              u64 y[APL];
              ldrow(q.vc + (unsigned long long)i * A, y);
              bool ne = false;
#pragma unroll
              for (int j = 0; j < APL; ++j) ne = ne || y[j] != r[j];
              if (!__ballot(ne)) slot = (int)i;
            }
            if (slot < 0 && n >= p.Vd) {
              st |= 1u;  // nested deferred capacity exceeded
            } else {
              if (slot < 0) {
                slot = (int)n++;
                strow(q.vc + (unsigned long long)slot * A, r);
                for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) smsk[slot * Mw + w] = 0;
              }
              for (u64 i = mb; i < me; ++i) {
                const unsigned long long m = p.mems[i];
                if (m < M && (unsigned long long)lane == (m / 64) % kWave) smsk[slot * Mw + m / 64] |= 1ull << (m % 64);
              }
            }
            unstage_masks(q, n);
          }
        }
      }
      // self.clock.apply(dot), then the Map's apply_deferred
#pragma unroll
      for (int j = 0; j < APL; ++j)
        if ((unsigned)j == a / 64 && (unsigned long long)lane == a % 64 && c[j] < cnt) c[j] = cnt;
      map_apply_deferred(k);
    } else if (kind == 1) {  // ---- Map Op::Rm -> apply_keyset_rm
      const unsigned rr = CRDT_MOA_HDR ? rl32(h_rr, hi) : p.clk_row[o];
      const u64 kb = CRDT_MOA_HDR ? rl64(h_kb, hi) : p.key_off[o], ke = CRDT_MOA_HDR ? rl64(h_ke, hi) : p.key_off[o + 1];
      if (rr >= p.n_clk_rows || ke < kb || ke > p.n_keys) {
        st |= 2u;
        continue;
      }
      u64 r[APL];
      ldrow(p.clk_pool + (unsigned long long)rr * A, r);
      for (u64 i = kb; i < ke; ++i) {
        const unsigned long long k = p.keys[i];
        if (k < K) key_rm(k, r);
        else st |= 2u;
      }
      if (leq(r, c)) continue;
      int slot = -1;
      for (unsigned d = 0; d < dcnt && slot < 0; ++d) {
        bool ne = false;
#pragma unroll
        for (int j = 0; j < APL; ++j) ne = ne || (word(j) < A && clk(d, word(j)) != r[j]);
        if (!__ballot(ne)) slot = (int)d;
      }
      if (slot < 0) {
        if constexpr (PASS == 1) {
          if (dcnt >= Dl) {  // the list outgrows the LDS slots: pass 2 from this op
            resume_at = (unsigned)(o - ob);
            goto done;
          }
        }
        if (dcnt >= Dcap) {
          st |= 1u;
          continue;
        }
        slot = (int)dcnt++;
        if (TIER) peak = dcnt > peak ? dcnt : peak;  // (pass 1: never past the input count's slots in memory)
#pragma unroll
        for (int j = 0; j < APL; ++j)
          if (word(j) < A) set_clk(slot, word(j), r[j]);
        for (unsigned long long w = (unsigned long long)lane; w < Kw; w += kWave) set_key(slot, w, 0);
      }
      for (u64 i = kb; i < ke; ++i) {
        const unsigned long long k = p.keys[i];
        if (k < K && (unsigned long long)lane == (k / 64) % kWave) set_key(slot, k / 64, key(slot, k / 64) | 1ull << (k % 64));
      }
    } else {
      st |= 2u;
    }
  }
  }
done:
#pragma unroll
  for (int j = 0; j < APL; ++j)
    if (word(j) < A) C[word(j)] = c[j];
  for (unsigned d = 0; d < dcnt && d < Dl; ++d) {  // (slots past Dl are already in place)
    for (unsigned long long a = (unsigned long long)lane; a < A; a += kWave) gclk[d * A + a] = sclk[d * A + a];
    for (unsigned long long w = (unsigned long long)lane; w < Kw; w += kWave) gkey[d * Kw + w] = skey[d * Kw + w];
  }
  // slots the deferred list vacated, zeroed as a fresh state's: pass 1 wrote none past its final count
  // to memory, so only the input's [dcnt, def_count[s]) can be stale there; pass 2 tracks its peak
  const unsigned hi = TIER ? peak : p.def_count[s];
  for (unsigned d = dcnt; d < hi; ++d) {
    for (unsigned long long a = (unsigned long long)lane; a < A; a += kWave) gclk[d * A + a] = 0ull;
    for (unsigned long long w = (unsigned long long)lane; w < Kw; w += kWave) gkey[d * Kw + w] = 0ull;
  }
  if (lane == 0) {
    p.def_count[s] = dcnt;
    p.status[s] = st;
    if (PASS == 1) p.resume[s] = resume_at == 0xffffffffu ? kMoaDone : resume_at;
  }
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_map_orswot_apply_batch(crdt_ctx *ctx, const crdt_map_orswot_states *m, uint64_t *def_clock,
                                           uint64_t *def_keys, uint32_t *def_count, size_t Dcap,
                                           const crdt_map_orswot_ops *ops, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!m || !ops || !status) return fail(ctx, CRDT_EINVAL, "map_orswot_apply_batch: NULL argument");
  const size_t N = m->N, K = m->K, M = m->M, A = m->A;
  if (N == 0) return CRDT_OK;
  if (A == 0 || A > 512) return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_apply_batch: A = %zu outside 1..512", A);
  if (M > 64 * (size_t)kMoaMw) return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_apply_batch: M = %zu > %d", M, 64 * kMoaMw);
  if (!m->clock || (K && (!m->ec || !m->oc || (M && !m->ent) || !m->vd_n || !m->vd_clock || !m->vd_mem)) ||
      !def_count || (Dcap && (!def_clock || !def_keys)) || !ops->op_off || !ops->mem_off)
    return fail(ctx, CRDT_EINVAL, "map_orswot_apply_batch: NULL buffer");
  if (ops->n_ops && (!ops->kind || !ops->vkind || !ops->actor || !ops->counter || !ops->key || !ops->vactor ||
                     !ops->vcounter || !ops->clk_row))
    return fail(ctx, CRDT_EINVAL, "map_orswot_apply_batch: NULL op buffer");
  const size_t Kw = K ? (K + 63) / 64 : 1, Mw = M > 64 ? (M + 63) / 64 : 1;
  const size_t Vd = m->Vd ? m->Vd : (size_t)kMoaVd, VW = std::max<size_t>((size_t)kMoaVd * kMoaMw, Vd * Mw);
  if (VW > 8192 - 64) return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_apply_batch: Vd * Mw = %zu words past the LDS", Vd * Mw);
  // the Map's deferred slots in LDS: up to kMoaDl (the rest of Dcap in the caller's slot arrays), fewer
  // where a slot is wide (the wave's LDS at most 8,192 words, the nested masks' VW words included)
  const size_t Dl = std::min<size_t>(Dcap, std::min<size_t>(kMoaDl, (8192 - VW) / (A + Kw)));
  const size_t per_wave = (Dl * (A + Kw) + VW) * 8;
  unsigned wpb = 4;
  while (wpb > 1 && per_wave * wpb > 64 * 1024) --wpb;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  MapOrswotApplyPlan p{(u64 *)m->clock, (u64 *)m->ec, (u64 *)m->oc, (u64 *)m->ent, (u64 *)m->vd_clock,
                       (u64 *)m->vd_mem, m->vd_n, N, K, M, A, Mw, Kw, Dcap, Dl, (u64 *)def_clock, (u64 *)def_keys,
                       def_count, (const u64 *)ops->op_off, ops->kind, ops->vkind, ops->actor, ops->key, ops->vactor,
                       (const u64 *)ops->counter, (const u64 *)ops->vcounter, ops->clk_row,
                       (const u64 *)ops->clk_pool, ops->clk_pool ? ops->n_clk_rows : 0, (const u64 *)ops->key_off,
                       ops->keys, ops->keys ? ops->n_keys : 0, (const u64 *)ops->mem_off, ops->mems,
                       ops->mems ? ops->n_mems : 0, ops->n_ops, status, wpb, nullptr, Vd, VW};
  // scratch: [resume: N words when Dcap > Dl][zero key_off: n_ops + 1 words when there is none]
  const size_t kz = ops->key_off ? 0 : (ops->n_ops + 1) * 8, rz = Dcap > Dl ? N * 8 : 0;
  if (kz + rz) {
    if (int rc = ensure_scratch(ctx, kz + rz)) return rc;
    char *sc = static_cast<char *>(ctx->scratch);
    if (rz) p.resume = reinterpret_cast<u64 *>(sc);
    if (kz) {  // (no Map-level Rm: every key range empty)
      if (int rc = device_fill(ctx, sc + rz, kz, 0)) return rc;
      p.key_off = reinterpret_cast<const u64 *>(sc + rz);
    }
  }
  if (Dcap > Dl && ops->n_ops >= 0xffffffffull)  // (pass 2 resumes at a 32-bit op offset)
    return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_apply_batch: 2^32 or more ops with Dcap past the LDS slots");
  const dim3 grid((unsigned)((N + wpb - 1) / wpb)), block(wpb * kWave);
  const size_t lds = per_wave * wpb;
  timing_begin(ctx, "map_orswot_apply");
  auto go = [&](auto t, dim3 g, dim3 b, size_t l) {
    constexpr int T = decltype(t)::value;
    if (A <= 64) hipLaunchKernelGGL((map_orswot_apply_kernel<1, T>), g, b, l, ctx->stream, p);
    else if (A <= 128) hipLaunchKernelGGL((map_orswot_apply_kernel<2, T>), g, b, l, ctx->stream, p);
    else if (A <= 256) hipLaunchKernelGGL((map_orswot_apply_kernel<4, T>), g, b, l, ctx->stream, p);
    else hipLaunchKernelGGL((map_orswot_apply_kernel<8, T>), g, b, l, ctx->stream, p);
  };
  if (Dcap <= Dl) {
    go(std::integral_constant<int, 0>{}, grid, block, lds);  // one pass: the whole list fits the LDS slots
  } else {
    go(std::integral_constant<int, 1>{}, grid, block, lds);
    // pass 2: the few states pass 1 handed on (the rest exit at once), one wave per workgroup with the
    // whole wave-LDS budget as slots (up to 64 KiB), so a long list mostly stays out of global memory
    const size_t Dl2 = std::min<size_t>(Dcap, (8192 - VW) / (A + Kw));
    p.Dl = Dl2;
    p.wpb = 1;
    go(std::integral_constant<int, 2>{}, dim3((unsigned)N), dim3(kWave), (Dl2 * (A + Kw) + VW) * 8);
  }
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}
