// CmRDT::apply and Causal::forget of whole Map<K, Map<K2, MVReg<u64>>> states (round 5) — the nested
// type of the reference's own Map tests (TMap, test/map.rs:10; TestMap, src/map.rs:359), on the
// crdt_map_nested_lub_many output layout (8 MVReg slots per inner key in Vec order with nval used,
// 16 inner deferred removes per key).
//
// apply (map.rs:119-137), per state its ops in order:
//   Op::Up { dot, key, op }: skipped when clock[dot.actor] >= dot.counter; else the entry (an absent
//     one: all-zero rows = Map::default()) applies the dot to its clock, its inner Map applies `op`,
//     the clock applies the dot, and apply_deferred (:311-316) re-runs every deferred remove;
//   Op::Rm { clock, keyset }: apply_keyset_rm (:318-348): each named key's entry clock forgets the
//     rm clock — an emptied entry is dropped, a kept one's inner Map forgets it (Causal::forget,
//     :85-114) — and the remove is deferred unless clock >= rm (an equal rm clock unions its keys).
// The inner Map's op is the same pair one level down, with MVReg::apply (mvreg.rs:130-166) for
// Op::Up's op Put { clock, val }: an empty clock is a no-op; values whose clock is <= the Put clock are
// dropped (order kept), and the value is appended unless a remaining one strictly dominates it.
// MVReg::forget (mvreg.rs:88-104) forgets every value clock and drops the emptied ones, order kept.
// Map::forget collects the deferred removes into a new map: two whose clocks become equal keep one
// entry with the later one's keys (the fold's rule, csrc/map_nested.hip; the reference's HashMap
// order is unspecified).
//
// One wave per state (apply) or per (state, key) (forget), lane l holding actors l + 64 j (j < APL)
// of every row; the outer deferred removes in LDS for the whole stream.  Every global word is read
// back only by the lane that wrote it (row words by the lane of their actor), or is a scalar every
// lane writes with the same value (nval, ivv, id_n, id_keys).
#include "common.hpp"

namespace crdt {

constexpr int kNaVs = 8;   // MVReg slots per inner key (crdt_map_nested_out)
constexpr int kNaId = 16;  // inner deferred removes per key

struct NestedApplyPlan {
  u64 *clock, *ec, *ic, *iec, *ivc, *ivv, *id_clock, *id_keys;
  unsigned *nval, *id_n;
  unsigned long long N, K, K2, A, Kw, Dcap;
  unsigned long long K2w;  // inner-key mask words per key set (1 up to K2 = 64: the round-5 layout)
  unsigned long long Id;   // inner deferred slots per key (crdt_map_nested_states.Id; 16 if 0)
  unsigned long long Vs;   // MVReg slots per inner key (crdt_map_nested_states.Vs; 8 if 0)
  unsigned long long Dl;  // outer deferred slots held in LDS (<= Dcap); slots Dl .. Dcap-1 stay in place
  u64 *def_clock, *def_keys;
  unsigned *def_count;
  const u64 *op_off;
  const uint8_t *kind, *ikind;
  const uint32_t *actor, *key, *iactor, *ikey;
  const u64 *counter, *icounter, *val, *ikeys;
  const uint32_t *clk_row;
  const u64 *clk_pool;
  unsigned long long n_clk_rows;
  const u64 *key_off;
  const uint32_t *keys;
  unsigned long long n_keys, n_ops;
  unsigned *status;
  unsigned wpb;
  u64 *resume = nullptr;  // [N] (Dcap > Dl): op offset where a state continues in pass 2, or kMnaDone
  const u64 *y;  // forget
  unsigned long long y_stride;
};
constexpr u64 kMnaDone = ~0ull;

// The rows of outer key k of state s, and the inner-Map operations on them.
// op headers batched 64 at a time into lanes and read by v_readlane (build option; 0 = one global
// read of each field per op)
// waves per SIMD asked of the register allocator for A <= 128 (build option).  4 = the round-5 kernel's
// natural 127 VGPRs; the round-6 pass structure needs 131 unforced, which is 3 waves per SIMD and ran
// 25% slower (2.09 vs 1.67 ms, profiles/r06_apply_ab.log).  0 = the compiler's choice.
#ifndef CRDT_MNA_WPE
#define CRDT_MNA_WPE 4
#endif
#if CRDT_MNA_WPE > 0
#define MNA_WPE_ATTR __attribute__((amdgpu_waves_per_eu(APL <= 2 ? CRDT_MNA_WPE : 1)))
#else
#define MNA_WPE_ATTR
#endif
#ifndef CRDT_MNA_HDR
#define CRDT_MNA_HDR 1
#endif
__device__ __forceinline__ unsigned rl32(unsigned x, int i) { return (unsigned)__builtin_amdgcn_readlane((int)x, i); }
__device__ __forceinline__ u64 rl64(u64 x, int i) {
  return ((u64)rl32((unsigned)(x >> 32), i) << 32) | rl32((unsigned)x, i);
}

constexpr int kNaKw = 4;  // inner-key mask words at most (K2 <= 256)

// KW: mask words per key set at compile time, 1 (K2 <= 64: the round-5 code) or kNaKw (kw of them live)
template <int APL, int KW = 1>
struct NaKey {
  u64 *ec, *ic, *iec, *ivc, *ivv, *idc, *idk;  // idk [kNaId][kwn()] inner key sets
  unsigned *nval, *idn;
  unsigned long long A, K2;
  int lane;
  mutable unsigned stb;  // status bits raised by these operations (the caller ORs them in)
  unsigned kw_;          // mask words per key set (KW > 1)
  unsigned cap;          // inner deferred slots (round 6: states->Id)
  unsigned vs;           // MVReg slots per inner key (round 6: states->Vs)
  __device__ __forceinline__ unsigned kwn() const { return KW == 1 ? 1u : kw_; }

  // held remove i's key set in registers (words past kwn(): 0) and back
  __device__ __forceinline__ void ks_ld(unsigned i, u64 (&k)[KW]) const {
#pragma unroll
    for (int x = 0; x < KW; ++x) k[x] = (unsigned)x < kwn() ? idk[(unsigned long long)i * kwn() + x] : 0ull;
  }
  __device__ __forceinline__ void ks_st(unsigned i, const u64 (&k)[KW]) const {
#pragma unroll
    for (int x = 0; x < KW; ++x)
      if ((unsigned)x < kwn()) idk[(unsigned long long)i * kwn() + x] = k[x];
  }
  __device__ __forceinline__ void ks_zero(unsigned i) const {
#pragma unroll
    for (int x = 0; x < KW; ++x)
      if ((unsigned)x < kwn()) idk[(unsigned long long)i * kwn() + x] = 0ull;
  }

  __device__ __forceinline__ unsigned long long word(int j) const { return (unsigned long long)lane + 64ull * j; }
  __device__ __forceinline__ void ld(const u64 *row, u64 (&x)[APL]) const {
#pragma unroll
    for (int j = 0; j < APL; ++j) x[j] = word(j) < A ? row[word(j)] : 0ull;
  }
  __device__ __forceinline__ void st_(u64 *row, const u64 (&x)[APL]) const {
#pragma unroll
    for (int j = 0; j < APL; ++j)
      if (word(j) < A) row[word(j)] = x[j];
  }
  __device__ __forceinline__ void zero(u64 *row) const {
#pragma unroll
    for (int j = 0; j < APL; ++j)
      if (word(j) < A) row[word(j)] = 0ull;
  }
  static __device__ __forceinline__ bool nz(const u64 (&x)[APL]) {
    bool b = false;
#pragma unroll
    for (int j = 0; j < APL; ++j) b = b || x[j] != 0;
    return __ballot(b) != 0;
  }
  static __device__ __forceinline__ bool leq(const u64 (&x)[APL], const u64 (&y)[APL]) {  // x <= y
    bool b = false;
#pragma unroll
    for (int j = 0; j < APL; ++j) b = b || x[j] > y[j];
    return __ballot(b) == 0;
  }
  static __device__ __forceinline__ bool eq(const u64 (&x)[APL], const u64 (&y)[APL]) {
    bool b = false;
#pragma unroll
    for (int j = 0; j < APL; ++j) b = b || x[j] != y[j];
    return __ballot(b) == 0;
  }
  static __device__ __forceinline__ void fg(u64 (&x)[APL], const u64 (&r)[APL]) {  // VClock::forget
#pragma unroll
    for (int j = 0; j < APL; ++j) x[j] = x[j] > r[j] ? x[j] : 0ull;
  }
  __device__ __forceinline__ u64 *slot(unsigned long long jk, unsigned i) const {
    return ivc + (jk * vs + i) * A;
  }

  // MVReg::forget of inner key jk's register (order kept, emptied values dropped)
  __device__ void reg_forget(unsigned long long jk, const u64 (&r)[APL]) const {
    const unsigned n = min(vs, nval[jk]);
    unsigned o = 0;
    for (unsigned i = 0; i < n; ++i) {
      u64 x[APL];
      ld(slot(jk, i), x);
      fg(x, r);
      if (!nz(x)) continue;
      const u64 v = ivv[jk * vs + i];
      st_(slot(jk, o), x);
      ivv[jk * vs + o] = v;
      ++o;
    }
    for (unsigned i = o; i < n; ++i) {
      zero(slot(jk, i));
      ivv[jk * vs + i] = 0;
    }
    nval[jk] = o;
  }
  // drop inner entry jk (its rows all zero)
  __device__ void inner_drop(unsigned long long jk) const {
    zero(iec + jk * A);
    const unsigned n = min(vs, nval[jk]);
    for (unsigned i = 0; i < n; ++i) {
      zero(slot(jk, i));
      ivv[jk * vs + i] = 0;
    }
    nval[jk] = 0;
  }
  // the inner Map's apply_keyset_rm on inner key jk = its entry's forget (map.rs:319-333)
  __device__ void inner_key_rm(unsigned long long jk, const u64 (&r)[APL]) const {
    u64 e[APL];
    ld(iec + jk * A, e);
    if (!nz(e)) return;
    fg(e, r);
    if (!nz(e)) {
      inner_drop(jk);
      return;
    }
    st_(iec + jk * A, e);
    reg_forget(jk, r);
  }
  // Causal::forget of the inner Map (map.rs:85-114)
  __device__ void inner_forget(const u64 (&r)[APL]) const {
    for (unsigned long long jk = 0; jk < K2; ++jk) inner_key_rm(jk, r);
    const unsigned n = min(cap, *idn);  // (a count past the slots: clamped)
    unsigned o = 0;
    for (unsigned i = 0; i < n; ++i) {
      u64 x[APL];
      ld(idc + (unsigned long long)i * A, x);
      fg(x, r);
      if (!nz(x)) continue;
      u64 ks[KW];
      ks_ld(i, ks);
      unsigned jj = 0;
      for (; jj < o; ++jj) {  // equal to a kept one: the later keys at the earlier place
        u64 y[APL];
        ld(idc + (unsigned long long)jj * A, y);
        if (eq(x, y)) break;
      }
      if (jj < o) {
        ks_st(jj, ks);
        continue;
      }
      st_(idc + (unsigned long long)o * A, x);
      ks_st(o, ks);
      ++o;
    }
    for (unsigned i = o; i < n; ++i) {
      zero(idc + (unsigned long long)i * A);
      ks_zero(i);
    }
    *idn = o;
    u64 c[APL];
    ld(ic, c);
    fg(c, r);
    st_(ic, c);
  }
  // the inner Map's apply_deferred (map.rs:311-316) against its clock c
  __device__ void inner_apply_deferred(const u64 (&c)[APL]) const {
    const unsigned n = min(cap, *idn);  // (a count past the slots: clamped)
    unsigned o = 0;
    for (unsigned i = 0; i < n; ++i) {
      u64 r[APL];
      ld(idc + (unsigned long long)i * A, r);
      u64 ks[KW];
      ks_ld(i, ks);
      keys_rm(ks, r);
      if (leq(r, c)) continue;  // seen: no longer deferred
      if (o != i) {
        st_(idc + (unsigned long long)o * A, r);
        ks_st(o, ks);
      }
      ++o;
    }
    for (unsigned i = o; i < n; ++i) {
      zero(idc + (unsigned long long)i * A);
      ks_zero(i);
    }
    *idn = o;
  }
  // MVReg::apply(Put { clock: r, val }) on inner key jk (mvreg.rs:130-166)
  __device__ void reg_put(unsigned long long jk, const u64 (&r)[APL], u64 v) const {
    if (!nz(r)) return;
    const unsigned n = min(vs, nval[jk]);
    unsigned o = 0;
    bool dominated = false;
    for (unsigned i = 0; i < n; ++i) {
      u64 x[APL];
      ld(slot(jk, i), x);
      if (leq(x, r)) continue;             // Less or Equal: dropped
      if (leq(r, x)) dominated = true;     // (x != r here) strictly greater: the Put is not added
      const u64 xv = ivv[jk * vs + i];
      if (o != i) {
        st_(slot(jk, o), x);
        ivv[jk * vs + o] = xv;
      }
      ++o;
    }
    for (unsigned i = o; i < n; ++i) {
      zero(slot(jk, i));
      ivv[jk * vs + i] = 0;
    }
    if (!dominated) {
      if (o < vs) {
        st_(slot(jk, o), r);
        ivv[jk * vs + o] = v;
        ++o;
      } else {
        stb |= 16u;  // the register needed more than vs values
      }
    }
    nval[jk] = o;
  }
  __device__ __forceinline__ u64 word_of(const u64 (&x)[APL], unsigned a) const {
    u64 v = 0;
#pragma unroll
    for (int j = 0; j < APL; ++j)
      if ((unsigned)j == a / 64) v = x[j];
    return __shfl(v, (int)(a % 64));
  }
  __device__ __forceinline__ void bump(u64 *row, unsigned a, u64 cnt) const {  // VClock::apply(dot)
    if ((unsigned long long)lane == a % 64) {
      u64 *q = row + a;
      if (*q < cnt) *q = cnt;
    }
  }
  // the inner Map's Op::Up { dot: (ia, icnt), key: jk, op: Put { clock: r, val: v } }
  __device__ void inner_up(unsigned ia, u64 icnt, unsigned long long jk, const u64 (&r)[APL], u64 v) const {
    u64 c[APL];
    ld(ic, c);
    if (word_of(c, ia) >= icnt) return;  // seen
    bump(iec + jk * A, ia, icnt);
    reg_put(jk, r, v);
    bump(ic, ia, icnt);
#pragma unroll
    for (int j = 0; j < APL; ++j)
      if ((unsigned)j == ia / 64 && (unsigned long long)lane == ia % 64 && c[j] < icnt) c[j] = icnt;
    inner_apply_deferred(c);
  }
  // the inner keys of a key set forgotten by r (apply_keyset_rm's forget, map.rs:320-333)
  __device__ void keys_rm(const u64 (&bits)[KW], const u64 (&r)[APL]) const {
#pragma unroll
    for (int x = 0; x < KW; ++x)
      for (u64 b = bits[x]; b;) {
        const unsigned long long jk = 64ull * x + (unsigned long long)__builtin_ctzll(b);
        b &= b - 1;
        if (jk < K2) inner_key_rm(jk, r);
      }
  }
  // the inner Map's Op::Rm { clock: r, keyset: bits }
  __device__ void inner_rm(const u64 (&r)[APL], const u64 (&bits)[KW]) const {
    keys_rm(bits, r);
    u64 c[APL];
    ld(ic, c);
    if (leq(r, c)) return;
    const unsigned n = min(cap, *idn);  // (a count past the slots: clamped)
    for (unsigned i = 0; i < n; ++i) {
      u64 y[APL];
      ld(idc + (unsigned long long)i * A, y);
      if (eq(y, r)) {
        u64 ks[KW];
        ks_ld(i, ks);
#pragma unroll
        for (int x = 0; x < KW; ++x) ks[x] |= bits[x];
        ks_st(i, ks);
        return;
      }
    }
    if (n >= cap) {
      stb |= 1u;
      return;
    }
    st_(idc + (unsigned long long)n * A, r);
    ks_st(n, bits);
    *idn = n + 1;
  }
  // drop the outer entry: every row of the key zero
  __device__ void drop_all() const {
    zero(ec);
    zero(ic);
    for (unsigned long long jk = 0; jk < K2; ++jk)
      if (nz_row(iec + jk * A) || nval[jk]) inner_drop(jk);
    const unsigned n = min(cap, *idn);  // (a count past the slots: clamped)
    for (unsigned i = 0; i < n; ++i) {
      zero(idc + (unsigned long long)i * A);
      ks_zero(i);
    }
    *idn = 0;
  }
  __device__ __forceinline__ bool nz_row(const u64 *row) const {
    u64 x[APL];
    ld(row, x);
    return nz(x);
  }
  // the outer apply_keyset_rm / forget on this key (map.rs:319-333, :85-98)
  __device__ void key_rm(const u64 (&r)[APL]) const {
    u64 e[APL];
    ld(ec, e);
    if (!nz(e)) return;
    fg(e, r);
    if (!nz(e)) {
      drop_all();
      return;
    }
    st_(ec, e);
    inner_forget(r);
  }
};

template <int APL, int KW = 1>
__device__ __forceinline__ NaKey<APL, KW> na_key(const NestedApplyPlan &p, unsigned long long s, unsigned long long k,
                                             int lane) {
  const unsigned long long sk = s * p.K + k, A = p.A, K2 = p.K2;
  return NaKey<APL, KW>{p.ec + sk * A, p.ic + sk * A, p.iec + sk * K2 * A, p.ivc + sk * K2 * p.Vs * A,
                    p.ivv + sk * K2 * p.Vs, p.id_clock + sk * p.Id * A, p.id_keys + sk * p.Id * p.K2w,
                    p.nval + sk * K2, p.id_n + sk, A, K2, lane, 0u, (unsigned)p.K2w,
                    (unsigned)p.Id, (unsigned)p.Vs};
}

// TIER false: every state, the Map's deferred list in the Dl LDS slots only; a state whose list
// needs slot Dl (Dcap > Dl) stores itself and records the op to continue from (resume[s]).  TIER
// true: those states alone, slots past Dl used in place in the caller's slot arrays.  (One body with
// the branch compiles the slot accesses to flat instructions and slows every state; see
// csrc/map_counter_apply.hip.)
template <int APL, int PASS, int KW>
__global__ __launch_bounds__(256) MNA_WPE_ATTR void map_nested_apply_kernel(NestedApplyPlan p) {
  extern __shared__ u64 lds[];
  const int lane = (int)(threadIdx.x % kWave), wv = (int)(threadIdx.x / kWave);
  const unsigned long long s = (unsigned long long)blockIdx.x * p.wpb + wv;
  if (wv >= (int)p.wpb || s >= p.N) return;  // (whole waves)
  constexpr bool TIER = PASS == 2;
  if constexpr (TIER) {
    if (p.resume[s] == kMnaDone) return;
  }
  const unsigned long long A = p.A, K = p.K, K2 = p.K2, Kw = p.Kw, Dcap = p.Dcap, Dl = p.Dl;
  // The outer deferred removes: slots d < Dl in LDS, slots Dl <= d < Dcap in the caller's own slot
  // arrays (global memory: a long list runs slower, never incomplete below Dcap)
  u64 *sclk = lds + (unsigned long long)wv * Dl * (A + Kw);  // [Dl][A] the outer rm clocks
  u64 *skey = sclk + Dl * A;                                 // [Dl][Kw] their key bitmaps
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
  const unsigned long long ob = p.op_off[s], oe = p.op_off[s + 1];
  unsigned dcnt = p.def_count[s];
  if (dcnt > Dcap || oe < ob || oe > p.n_ops) {
    if (lane == 0) {
      p.status[s] = (dcnt > Dcap ? 4u : 0u) | (oe < ob || oe > p.n_ops ? 8u : 0u);
      if (PASS == 1) p.resume[s] = kMnaDone;
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
  u64 *C = p.clock + s * A;
  u64 c[APL];
#pragma unroll
  for (int j = 0; j < APL; ++j) c[j] = word(j) < A ? C[word(j)] : 0ull;
  for (unsigned d = 0; d < dcnt && d < Dl; ++d) {
    for (unsigned long long a = (unsigned long long)lane; a < A; a += kWave) sclk[d * A + a] = gclk[d * A + a];
    for (unsigned long long w = (unsigned long long)lane; w < Kw; w += kWave) skey[d * Kw + w] = gkey[d * Kw + w];
  }
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
          if (k < K) {
            const NaKey<APL, KW> q = na_key<APL, KW>(p, s, k, lane);
            q.key_rm(r);
            st |= q.stb;
          }
        }
      }
      if (NaKey<APL, KW>::leq(r, c)) continue;  // no longer deferred
      if (o != d) {
        for (unsigned long long a = (unsigned long long)lane; a < A; a += kWave) set_clk(o, a, clk(d, a));
        for (unsigned long long w = (unsigned long long)lane; w < Kw; w += kWave) set_key(o, w, key(d, w));
      }
      ++o;
    }
    dcnt = o;
    full = false;
  };

  // Op headers in batches of 64 (CRDT_MNA_HDR): lane i loads op o0 + i's fields (coalesced, all in
  // flight together) and op o's fields reach the wave by v_readlane, not by a global round trip per op.
  for (unsigned long long o0 = start; o0 < oe; o0 += kWave) {
    const unsigned long long mo = o0 + (unsigned long long)lane;
    const bool hin = CRDT_MNA_HDR && mo < oe;
    const unsigned h_kind = hin ? p.kind[mo] : 0u, h_ik = hin ? p.ikind[mo] : 0u, h_a = hin ? p.actor[mo] : 0u;
    const unsigned h_k = hin ? p.key[mo] : 0u, h_ia = hin ? p.iactor[mo] : 0u, h_jk = hin ? p.ikey[mo] : 0u;
    const unsigned h_rr = hin ? p.clk_row[mo] : 0u;
    const u64 h_c = hin ? p.counter[mo] : 0ull, h_ic = hin ? p.icounter[mo] : 0ull, h_v = hin ? p.val[mo] : 0ull;
    const u64 h_ib = hin && p.K2w == 1 ? p.ikeys[mo] : 0ull, h_kb = hin ? p.key_off[mo] : 0ull, h_ke = hin ? p.key_off[mo + 1] : 0ull;
    const int nb = (int)(oe - o0 < (unsigned long long)kWave ? oe - o0 : (unsigned long long)kWave);
  for (int hi = 0; hi < nb; ++hi) {
    const unsigned long long o = o0 + (unsigned long long)hi;
    const unsigned kind = CRDT_MNA_HDR ? rl32(h_kind, hi) : p.kind[o];
    if (kind == 0) {  // ---- Op::Up { dot, key, op: an inner Map op }
      const unsigned a = CRDT_MNA_HDR ? rl32(h_a, hi) : p.actor[o], ik = CRDT_MNA_HDR ? rl32(h_ik, hi) : p.ikind[o];
      const unsigned long long k = CRDT_MNA_HDR ? rl32(h_k, hi) : p.key[o];
      const u64 cnt = CRDT_MNA_HDR ? rl64(h_c, hi) : p.counter[o];
      const unsigned rr = CRDT_MNA_HDR ? rl32(h_rr, hi) : p.clk_row[o];
      const unsigned ia = ik == 0 ? (CRDT_MNA_HDR ? rl32(h_ia, hi) : p.iactor[o]) : 0u;
      const unsigned long long jk = ik == 0 ? (CRDT_MNA_HDR ? rl32(h_jk, hi) : p.ikey[o]) : 0ull;
      // an inner Rm's key set: K2w words of ikeys [n_ops][K2w] (one word batched with the headers);
      // read here for the range check and again at the Rm, so no word is held across the key's setup
      const auto ibw = [&](int x) -> u64 {
        return ik != 1 || (unsigned long long)x >= p.K2w ? 0ull
               : p.K2w == 1 ? (CRDT_MNA_HDR ? rl64(h_ib, hi) : p.ikeys[o])
                            : p.ikeys[o * p.K2w + x];
      };
      bool kbad = false;  // a key bit past K2
#pragma unroll
      for (int x = 0; x < KW; ++x) {
        const unsigned long long lo = 64ull * x;
        const u64 w = ibw(x);
        kbad = kbad || (K2 < lo + 64 && (K2 <= lo ? w != 0 : (w >> (K2 - lo)) != 0));
      }
      if (a >= A || k >= K || ik > 1 || rr >= p.n_clk_rows || ia >= A || jk >= K2 || kbad) {
        st |= 2u;  // malformed: skipped whole
        continue;
      }
      const NaKey<APL, KW> q = na_key<APL, KW>(p, s, k, lane);
      if (q.word_of(c, a) >= cnt) continue;  // seen (map.rs:123-126)
      q.bump(q.ec, a, cnt);  // entry.clock.apply(dot) (an absent entry: its rows are Map::default())
      u64 r[APL];
      q.ld(p.clk_pool + (unsigned long long)rr * A, r);
      if (ik == 0) q.inner_up(ia, CRDT_MNA_HDR ? rl64(h_ic, hi) : p.icounter[o], jk, r, CRDT_MNA_HDR ? rl64(h_v, hi) : p.val[o]);
      else {
        u64 ib[KW];
#pragma unroll
        for (int x = 0; x < KW; ++x) ib[x] = ibw(x);
        q.inner_rm(r, ib);
      }
      st |= q.stb;
#pragma unroll
      for (int j = 0; j < APL; ++j)
        if ((unsigned)j == a / 64 && (unsigned long long)lane == a % 64 && c[j] < cnt) c[j] = cnt;
      map_apply_deferred(k);
    } else if (kind == 1) {  // ---- Op::Rm -> apply_keyset_rm
      const unsigned rr = CRDT_MNA_HDR ? rl32(h_rr, hi) : p.clk_row[o];
      const u64 kb = CRDT_MNA_HDR ? rl64(h_kb, hi) : p.key_off[o], ke = CRDT_MNA_HDR ? rl64(h_ke, hi) : p.key_off[o + 1];
      if (rr >= p.n_clk_rows || ke < kb || ke > p.n_keys) {
        st |= 2u;
        continue;
      }
      u64 r[APL];
#pragma unroll
      for (int j = 0; j < APL; ++j) r[j] = word(j) < A ? p.clk_pool[(unsigned long long)rr * A + word(j)] : 0ull;
      for (u64 i = kb; i < ke; ++i) {
        const unsigned long long k = p.keys[i];
        if (k < K) {
          const NaKey<APL, KW> q = na_key<APL, KW>(p, s, k, lane);
          q.key_rm(r);
          st |= q.stb;
        } else {
          st |= 2u;
        }
      }
      if (NaKey<APL, KW>::leq(r, c)) continue;
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
    if (PASS == 1) p.resume[s] = resume_at == 0xffffffffu ? kMnaDone : resume_at;
  }
}

// Causal::forget of the entries: one wave per (state, key), y row y[s] (the map clock and the outer
// deferred pool go through crdt_map_forget_batch afterwards)
template <int APL, int KW>
__global__ __launch_bounds__(256) void map_nested_forget_kernel(NestedApplyPlan p) {
  const int lane = (int)(threadIdx.x % kWave);
  const unsigned long long sk = (unsigned long long)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  if (sk >= p.N * p.K) return;  // (whole waves)
  const unsigned long long s = sk / p.K, k = sk % p.K;
  const NaKey<APL, KW> q = na_key<APL, KW>(p, s, k, lane);
  u64 r[APL];
  q.ld(p.y + s * p.y_stride, r);
  q.key_rm(r);  // (Map::forget on an entry = apply_keyset_rm's per-key step)
}

}  // namespace crdt

using namespace crdt;

static int nested_states_check(crdt_ctx *ctx, const crdt_map_nested_states *m, const char *what) {
  if (!m) return fail(ctx, CRDT_EINVAL, "%s: NULL states", what);
  if (m->A > 512) return fail(ctx, CRDT_EUNSUPPORTED, "%s: A = %zu > 512", what, m->A);
  if (m->K2 > 256) return fail(ctx, CRDT_EUNSUPPORTED, "%s: K2 = %zu > 256 (inner key sets of 4 mask words)", what, m->K2);
  if (m->N && (!m->clock || (m->K && (!m->ec || !m->ic || !m->id_n || !m->id_clock || !m->id_keys ||
                                      (m->K2 && (!m->iec || !m->ivc || !m->ivv || !m->nval))))))
    return fail(ctx, CRDT_EINVAL, "%s: NULL state buffer", what);
  return CRDT_OK;
}

static NestedApplyPlan nested_plan(const crdt_map_nested_states *m) {
  NestedApplyPlan p{};
  p.clock = (u64 *)m->clock;
  p.ec = (u64 *)m->ec;
  p.ic = (u64 *)m->ic;
  p.iec = (u64 *)m->iec;
  p.ivc = (u64 *)m->ivc;
  p.ivv = (u64 *)m->ivv;
  p.id_clock = (u64 *)m->id_clock;
  p.id_keys = (u64 *)m->id_keys;
  p.nval = m->nval;
  p.id_n = m->id_n;
  p.N = m->N;
  p.K = m->K;
  p.K2 = m->K2;
  p.K2w = m->K2 > 64 ? (m->K2 + 63) / 64 : 1;
  p.Id = m->Id ? m->Id : (size_t)kNaId;
  p.Vs = m->Vs ? m->Vs : (size_t)kNaVs;
  p.A = m->A;
  p.Kw = m->K ? (m->K + 63) / 64 : 1;
  return p;
}

extern "C" int crdt_map_nested_apply_batch(crdt_ctx *ctx, const crdt_map_nested_states *m, uint64_t *def_clock,
                                           uint64_t *def_keys, uint32_t *def_count, size_t Dcap,
                                           const crdt_map_nested_ops *ops, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (int rc = nested_states_check(ctx, m, "map_nested_apply_batch")) return rc;
  if (!ops || !status) return fail(ctx, CRDT_EINVAL, "map_nested_apply_batch: NULL argument");
  const size_t N = m->N, A = m->A;
  if (N == 0) return CRDT_OK;
  if (A == 0) return fail(ctx, CRDT_EINVAL, "map_nested_apply_batch: A = 0");
  if (!def_count || (Dcap && (!def_clock || !def_keys)) || !ops->op_off)
    return fail(ctx, CRDT_EINVAL, "map_nested_apply_batch: NULL buffer");
  if (ops->n_ops && (!ops->kind || !ops->actor || !ops->counter || !ops->key || !ops->ikind || !ops->iactor ||
                     !ops->icounter || !ops->ikey || !ops->val || !ops->ikeys || !ops->clk_row))
    return fail(ctx, CRDT_EINVAL, "map_nested_apply_batch: NULL op buffer");
  NestedApplyPlan p = nested_plan(m);
  // outer deferred slots in LDS: up to 16 (the rest of Dcap in the caller's slot arrays), fewer where a
  // slot is wide (at most 8,192 words per wave)
  const size_t Dl = std::min<size_t>(Dcap, std::min<size_t>(16, 8192 / (A + p.Kw)));
  const size_t per_wave = Dl * (A + p.Kw) * 8;
  unsigned wpb = 4;
  while (wpb > 1 && per_wave * wpb > 64 * 1024) --wpb;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  p.Dcap = Dcap;
  p.Dl = Dl;
  p.def_clock = (u64 *)def_clock;
  p.def_keys = (u64 *)def_keys;
  p.def_count = def_count;
  p.op_off = (const u64 *)ops->op_off;
  p.kind = ops->kind;
  p.ikind = ops->ikind;
  p.actor = ops->actor;
  p.key = ops->key;
  p.iactor = ops->iactor;
  p.ikey = ops->ikey;
  p.counter = (const u64 *)ops->counter;
  p.icounter = (const u64 *)ops->icounter;
  p.val = (const u64 *)ops->val;
  p.ikeys = (const u64 *)ops->ikeys;
  p.clk_row = ops->clk_row;
  p.clk_pool = (const u64 *)ops->clk_pool;
  p.n_clk_rows = ops->clk_pool ? ops->n_clk_rows : 0;
  p.key_off = (const u64 *)ops->key_off;
  p.keys = ops->keys;
  p.n_keys = ops->keys ? ops->n_keys : 0;
  p.n_ops = ops->n_ops;
  p.status = status;
  p.wpb = wpb;
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
    return fail(ctx, CRDT_EUNSUPPORTED, "map_nested_apply_batch: 2^32 or more ops with Dcap past the LDS slots");
  const dim3 grid((unsigned)((N + wpb - 1) / wpb)), block(wpb * kWave);
  const size_t lds = per_wave * wpb;
  timing_begin(ctx, "map_nested_apply");
  auto go_kw = [&](auto t, auto w, dim3 g, dim3 b, size_t l) {
    constexpr int T = decltype(t)::value, W = decltype(w)::value;
    if (A <= 64) hipLaunchKernelGGL((map_nested_apply_kernel<1, T, W>), g, b, l, ctx->stream, p);
    else if (A <= 128) hipLaunchKernelGGL((map_nested_apply_kernel<2, T, W>), g, b, l, ctx->stream, p);
    else if (A <= 256) hipLaunchKernelGGL((map_nested_apply_kernel<4, T, W>), g, b, l, ctx->stream, p);
    else hipLaunchKernelGGL((map_nested_apply_kernel<8, T, W>), g, b, l, ctx->stream, p);
  };
  auto go = [&](auto t, dim3 g, dim3 b, size_t l) {  // (one mask word per key set up to K2 = 64)
    if (p.K2w == 1) go_kw(t, std::integral_constant<int, 1>{}, g, b, l);
    else go_kw(t, std::integral_constant<int, kNaKw>{}, g, b, l);
  };
  if (Dcap <= Dl) {
    go(std::integral_constant<int, 0>{}, grid, block, lds);  // one pass: the whole list fits the LDS slots
  } else {
    go(std::integral_constant<int, 1>{}, grid, block, lds);
    // pass 2: the few states pass 1 handed on (the rest exit at once), one wave per workgroup with the
    // whole wave-LDS budget as slots (up to 64 KiB), so a long list mostly stays out of global memory
    const size_t Dl2 = std::min<size_t>(Dcap, 8192 / (A + p.Kw));
    p.Dl = Dl2;
    p.wpb = 1;
    go(std::integral_constant<int, 2>{}, dim3((unsigned)N), dim3(kWave), Dl2 * (A + p.Kw) * 8);
  }
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

extern "C" int crdt_map_nested_forget_batch(crdt_ctx *ctx, const crdt_map_nested_states *m, const uint64_t *y,
                                            size_t y_stride, uint64_t *def_clock, const uint32_t *def_state,
                                            size_t D, uint8_t *def_keep) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (int rc = nested_states_check(ctx, m, "map_nested_forget_batch")) return rc;
  const size_t N = m->N, K = m->K, A = m->A;
  if (N == 0 || A == 0) return CRDT_OK;
  if (!y) return fail(ctx, CRDT_EINVAL, "map_nested_forget_batch: NULL y");
  if (y_stride && y_stride < A) return fail(ctx, CRDT_EINVAL, "map_nested_forget_batch: y_stride < A");
  if (K) {
    NestedApplyPlan p = nested_plan(m);
    p.y = (const u64 *)y;
    p.y_stride = y_stride;
    const unsigned long long waves = (unsigned long long)N * K, blocks = (waves + 3) / 4;
    if (blocks > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_nested_forget_batch: N*K too large");
    CRDT_HIP(ctx, hipSetDevice(ctx->device));
    timing_begin(ctx, "map_nested_forget");
    auto fgo = [&](auto w) {
      constexpr int W = decltype(w)::value;
      const dim3 g((unsigned)blocks), b(256);
      if (A <= 64) hipLaunchKernelGGL((map_nested_forget_kernel<1, W>), g, b, 0, ctx->stream, p);
      else if (A <= 128) hipLaunchKernelGGL((map_nested_forget_kernel<2, W>), g, b, 0, ctx->stream, p);
      else if (A <= 256) hipLaunchKernelGGL((map_nested_forget_kernel<4, W>), g, b, 0, ctx->stream, p);
      else hipLaunchKernelGGL((map_nested_forget_kernel<8, W>), g, b, 0, ctx->stream, p);
    };
    if (p.K2w == 1) fgo(std::integral_constant<int, 1>{});
    else fgo(std::integral_constant<int, kNaKw>{});
    timing_end(ctx);
    CRDT_HIP(ctx, hipGetLastError());
  }
  // the map clock and the outer deferred pool (no entries: K = 0)
  crdt_map_states s{N, 0, A, 1, m->clock, A, nullptr, 0, nullptr, 0, nullptr, 0};
  return crdt_map_forget_batch(ctx, &s, y, y_stride, def_clock, def_state, D, def_keep);
}
