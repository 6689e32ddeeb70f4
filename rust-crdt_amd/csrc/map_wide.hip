// Map<K, MVReg<u64>> lub_many for shapes past the fast kernels' register limits (A > 256 actors or
// V > 8 value slots per key): the same exact per-key left fold as map_fold_kernel (csrc/map.hip,
// whose header derives it from map.rs:140-220 with MVReg::merge / forget, mvreg.rs:88-128), with a
// workgroup instead of a wave per key.
//
// Mapping: one workgroup of NT = 64..256 threads per (group, key); thread t holds actors
// t + NT*j, j < kWideApt (A <= 4 * NT <= 1,024).  The fold state (entry clock, acc clock, up to VOS
// value clocks) stays in registers, values and order keys are uniform.  Each replica step is read
// straight from global memory (no staging, no speculative scan: this path is for correctness at
// unusual shapes, not speed).  Every "for all actors" / "any actor" test of a step is a bit of a
// per-thread AND / OR word, and ONE block reduction (wave shuffles, then the waves' words through
// LDS) settles all of a round's bits at once: the entry join's tests in one round, all pairwise
// value-clock orders of the MVReg merge (state x incoming, both directions) in another, so a step
// costs a handful of barriers whatever V is.
//
// Deferred removes: the removes naming the key are gathered once in replica order (LDS, or the
// group's list read directly past kWideList).  At step i the live removes are those held by a replica
// <= i that the acc clock before step i does not dominate (the clock only grows, so a dominated
// remove stays dead) plus every remove held by replica i; the step forgets the key by their max
// (successive forgets compose), exactly as the fast kernel's queue (map.hip, map.rs:213-219,
// :336-345).
#include <algorithm>

#include "common.hpp"

namespace crdt {

constexpr int kWideApt = 4;      // actors per thread
constexpr int kWideVin = 16;     // input value slots per key (V)
constexpr int kWideList = 1024;  // removes naming one key listed in LDS (beyond: the group list)
constexpr int kWideLive = 1024;  // live removes tracked in LDS (beyond: a rescan of the started ones)

struct MapWidePlan {
  const u64 *clock;
  long long c_rs, c_gs;
  const u64 *ec;
  long long e_rs, e_gs;
  const u64 *vclk;
  long long vc_rs, vc_gs;
  const u64 *vval;
  long long vv_rs, vv_gs;
  const size_t *def_off;  // device copy [G+1] (nullptr: no deferred)
  const unsigned *def_row;
  const u64 *def_clock;
  const u64 *def_keys;
  unsigned long long G, R, K, A, V, Kw, Vout;
  u64 *o_clock, *o_ec, *o_vclk, *o_vval;
  unsigned *o_flags, *o_nval;
};

// Block-wide AND / OR of NA + NO 64-bit words: wave shuffles, then one word set per wave in LDS.
// Every thread gets the result.  `red` holds 4 waves * (NA + NO) words.
template <int NA, int NO>
__device__ __forceinline__ void wide_vote(u64 (&a)[NA > 0 ? NA : 1], u64 (&o)[NO > 0 ? NO : 1], u64 *red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int w = 0; w < NA; ++w) a[w] &= __shfl_xor(a[w], off, 64);
#pragma unroll
    for (int w = 0; w < NO; ++w) o[w] |= __shfl_xor(o[w], off, 64);
  }
  const int nw = blockDim.x / 64, wv = threadIdx.x / 64;
  if (nw == 1) return;
  constexpr int NWD = NA + NO;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int w = 0; w < NA; ++w) red[wv * NWD + w] = a[w];
#pragma unroll
    for (int w = 0; w < NO; ++w) red[wv * NWD + NA + w] = o[w];
  }
  __syncthreads();
  for (int x = 0; x < nw; ++x) {
#pragma unroll
    for (int w = 0; w < NA; ++w) a[w] &= red[x * NWD + w];
#pragma unroll
    for (int w = 0; w < NO; ++w) o[w] |= red[x * NWD + NA + w];
  }
  __syncthreads();  // red may be reused by the next round
}

// single-flag forms
__device__ __forceinline__ bool wide_all(bool t, u64 *red) {
  u64 a[1] = {t ? 1ull : 0ull}, o[1] = {0};
  wide_vote<1, 0>(a, o, red);
  return a[0] != 0;
}
__device__ __forceinline__ bool wide_any(bool t, u64 *red) {
  u64 a[1] = {~0ull}, o[1] = {t ? 1ull : 0ull};
  wide_vote<0, 1>(a, o, red);
  return o[0] != 0;
}

template <int VOS>
struct WideMV {
  u64 c[VOS][kWideApt];
  u64 v[VOS], seq[VOS];
  unsigned vm;
  u64 next;
};

// vals.forget(X) for every valid value, dropping the ones emptied (one vote round)
template <int VOS>
__device__ __forceinline__ void wide_mv_forget(WideMV<VOS> &s, const u64 (&X)[kWideApt], u64 *red) {
  u64 a[1] = {~0ull}, o[1] = {0};
#pragma unroll
  for (int q = 0; q < VOS; ++q)
    if (s.vm & (1u << q)) {
      bool nz = false;
#pragma unroll
      for (int j = 0; j < kWideApt; ++j) {
        s.c[q][j] = s.c[q][j] > X[j] ? s.c[q][j] : 0;
        nz |= s.c[q][j] != 0;
      }
      if (nz) o[0] |= 1ull << q;
    }
  wide_vote<0, 1>(a, o, red);
  s.vm &= (unsigned)o[0];
}

template <int VOS>
__device__ __forceinline__ void wide_mv_append(WideMV<VOS> &s, const u64 (&x)[kWideApt], u64 val, int &ovf) {
  const unsigned freem = ~s.vm & ((1u << VOS) - 1u);
  if (freem == 0) {
    ovf |= 4;
    return;
  }
  const int q0 = __builtin_ctz(freem);
#pragma unroll
  for (int q = 0; q < VOS; ++q)
    if (q == q0) {
#pragma unroll
      for (int j = 0; j < kWideApt; ++j) s.c[q][j] = x[j];
      s.v[q] = val;
      s.seq[q] = s.next;
    }
  s.next++;
  s.vm |= 1u << q0;
}

template <int VOS>
__global__ __launch_bounds__(256) void map_fold_wide_kernel(MapWidePlan p) {
  __shared__ u64 red[4 * 16];
  __shared__ unsigned lrow[kWideList], lidx[kWideList], live[kWideLive];
  __shared__ unsigned s_cnt[2];
  const unsigned long long g = blockIdx.x / p.K, k = blockIdx.x % p.K;
  const unsigned nt = blockDim.x, tid = threadIdx.x;
  const unsigned long long A = p.A, R = p.R, V = p.V;
  bool on[kWideApt];
  unsigned long long act[kWideApt];
#pragma unroll
  for (int j = 0; j < kWideApt; ++j) {
    act[j] = tid + (unsigned long long)nt * j;
    on[j] = act[j] < A;
  }
  bool present = false;
  u64 e[kWideApt], cs[kWideApt];
#pragma unroll
  for (int j = 0; j < kWideApt; ++j) e[j] = cs[j] = 0;
  WideMV<VOS> mv;
  mv.vm = 0;
  mv.next = 0;
#pragma unroll
  for (int q = 0; q < VOS; ++q) {
    mv.v[q] = mv.seq[q] = 0;
#pragma unroll
    for (int j = 0; j < kWideApt; ++j) mv.c[q][j] = 0;
  }
  int ovf = 0;
  bool bad = false;

  // the removes naming this key, in replica order (wave 0 gathers them; ballot prefix positions)
  unsigned long long dbeg = 0, dend = 0;
  if (p.def_off) {
    dbeg = p.def_off[g];
    dend = p.def_off[g + 1];
  }
  const unsigned long long kw = k / 64;
  const u64 kbit = 1ull << (k % 64);
  if (tid < 64) {
    unsigned long long nl = 0;
    int badl = 0;
    for (unsigned long long base = dbeg; base < dend; base += 64) {
      const unsigned long long d = base + tid;
      bool hit = false;
      unsigned row = 0;
      if (d < dend) {
        row = p.def_row[d];
        hit = (p.def_keys[d * p.Kw + kw] & kbit) != 0;
        if (k == 0 && (row >= R || (d > dbeg && p.def_row[d - 1] > row))) badl = 1;
      }
      const u64 m = __ballot(hit);
      if (hit) {
        const unsigned long long pos = nl + __popcll(m & ((1ull << tid) - 1));
        if (pos < kWideList) {
          lrow[pos] = row;
          lidx[pos] = (unsigned)d;
        }
      }
      nl += __popcll(m);
    }
    const bool anybad = __ballot(badl) != 0;
    if (tid == 0) {
      s_cnt[0] = (unsigned)(nl > 0xffffffffull ? 0xffffffffu : nl);
      s_cnt[1] = anybad;
    }
  }
  __syncthreads();
  const unsigned long long nl = s_cnt[0];
  bad = s_cnt[1] != 0;
  const bool direct = nl > (unsigned long long)kWideList;  // walk the group's list each step
  unsigned long long lp = 0, dp = dbeg, nlive = 0;
  bool rescan = false;  // more live removes than kWideLive: rescan the started ones every step

  for (unsigned long long i = 0; i < R; ++i) {
    const u64 *ecp = p.ec + g * p.e_gs + i * p.e_rs + k * A;
    const u64 *cop = p.clock + g * p.c_gs + i * p.c_rs;
    const u64 *vcp = p.vclk + g * p.vc_gs + i * p.vc_rs + k * V * A;
    const u64 *vvp = p.vval + g * p.vv_gs + i * p.vv_rs + k * V;
    u64 ie[kWideApt], ico[kWideApt];
#pragma unroll
    for (int j = 0; j < kWideApt; ++j) {
      ie[j] = on[j] ? ecp[act[j]] : 0;
      ico[j] = on[j] ? cop[act[j]] : 0;
    }
    // ---- 1. entry join (map.rs:142-210): every test of the three cases in one round ----
    u64 eA[kWideApt], riA[kWideApt], eB[kWideApt], riB[kWideApt], common[kWideApt], dl[kWideApt];
    bool t_co_ge_e = true, t_cs_ge_ie = true, t_eq = true, n_ie = false, n_common = false, n_dl = false, n_riA = false;
#pragma unroll
    for (int j = 0; j < kWideApt; ++j) {
      t_co_ge_e &= ico[j] >= e[j];
      t_cs_ge_ie &= cs[j] >= ie[j];
      t_eq &= e[j] == ie[j];
      n_ie |= ie[j] != 0;
      eA[j] = e[j] > ico[j] ? e[j] : 0;
      riA[j] = ico[j] > eA[j] ? ico[j] : 0;
      n_riA |= riA[j] != 0;
      eB[j] = ie[j] > cs[j] ? ie[j] : 0;
      riB[j] = cs[j] > eB[j] ? cs[j] : 0;
      const u64 t0 = e[j] == ie[j] ? e[j] : 0;
      const u64 t1 = ie[j] > cs[j] ? ie[j] : 0;
      const u64 t2 = e[j] > ico[j] ? e[j] : 0;
      const u64 c = t0 > t1 ? t0 : t1;
      common[j] = c > t2 ? c : t2;
      const u64 m = e[j] > ie[j] ? e[j] : ie[j];
      dl[j] = m > common[j] ? m : 0;
      n_common |= common[j] != 0;
      n_dl |= dl[j] != 0;
    }
    {
      u64 a[1] = {(t_co_ge_e ? 1ull : 0) | (t_cs_ge_ie ? 2ull : 0) | (t_eq ? 4ull : 0)};
      u64 o[1] = {(n_ie ? 1ull : 0) | (n_common ? 2ull : 0) | (n_dl ? 4ull : 0) | (n_riA ? 8ull : 0)};
      wide_vote<1, 1>(a, o, red);
      t_co_ge_e = a[0] & 1;
      t_cs_ge_ie = a[0] & 2;
      t_eq = a[0] & 4;
      n_ie = o[0] & 1;
      n_common = o[0] & 2;
      n_dl = o[0] & 4;
      n_riA = o[0] & 8;
    }
    const bool p2 = n_ie;
    if (present && !p2) {
      if (t_co_ge_e) {
        present = false;
        mv.vm = 0;
#pragma unroll
        for (int j = 0; j < kWideApt; ++j) e[j] = 0;
      } else {
#pragma unroll
        for (int j = 0; j < kWideApt; ++j) e[j] = eA[j];
        if (n_riA) wide_mv_forget(mv, riA, red);
      }
    } else if (!present && p2) {
      if (!t_cs_ge_ie) {
#pragma unroll
        for (int j = 0; j < kWideApt; ++j) e[j] = eB[j];
        mv.vm = 0;
        mv.next = 0;
        // incoming values that survive forget(riB): one round over every slot
        u64 a[1] = {~0ull}, o[1] = {0};
        for (unsigned long long t = 0; t < V; ++t) {
          bool nz = false;
#pragma unroll
          for (int j = 0; j < kWideApt; ++j) {
            const u64 x = on[j] ? vcp[t * A + act[j]] : 0;
            nz |= (x > riB[j] ? x : 0) != 0;
          }
          if (nz) o[0] |= 1ull << t;
        }
        wide_vote<0, 1>(a, o, red);
        for (unsigned long long t = 0; t < V; ++t)
          if (o[0] & (1ull << t)) {
            u64 x[kWideApt];
#pragma unroll
            for (int j = 0; j < kWideApt; ++j) {
              const u64 y = on[j] ? vcp[t * A + act[j]] : 0;
              x[j] = y > riB[j] ? y : 0;
            }
            wide_mv_append(mv, x, vvp[t], ovf);
          }
        present = true;
      }
    } else if (present && p2) {
      bool dl_any = false;
      if (!t_eq) {
        if (!n_common) {
          present = false;
          mv.vm = 0;
        } else {
          dl_any = n_dl;
        }
#pragma unroll
        for (int j = 0; j < kWideApt; ++j) e[j] = common[j];
      }
      if (present) {
        // MVReg::merge (mvreg.rs:112-128): every pairwise order between the own values (q) and the
        // incoming ones (t) in one round: le_qt = own <= incoming, ne_qt = own != incoming,
        // le_tq = incoming <= own, nz_t = incoming slot non-empty
        // bit (q % 4) * 16 + t of word q / 4 (a compile-time word: q is unrolled, t < kWideVin)
        constexpr int QW = VOS / 4, NA = 2 * QW, NO = QW + 1;  // a: le_qt | le_tq, o: ne_qt | nz_t
        u64 a[NA], o[NO];
#pragma unroll
        for (int w = 0; w < NA; ++w) a[w] = ~0ull;
#pragma unroll
        for (int w = 0; w < NO; ++w) o[w] = 0;
        for (unsigned long long t = 0; t < V; ++t) {
          u64 x[kWideApt];
          bool nz = false;
#pragma unroll
          for (int j = 0; j < kWideApt; ++j) {
            x[j] = on[j] ? vcp[t * A + act[j]] : 0;
            nz |= x[j] != 0;
          }
          if (nz) o[NO - 1] |= 1ull << t;
#pragma unroll
          for (int q = 0; q < VOS; ++q) {
            if (!(mv.vm & (1u << q))) continue;
            bool le_qt = true, le_tq = true, ne = false;
#pragma unroll
            for (int j = 0; j < kWideApt; ++j) {
              le_qt &= mv.c[q][j] <= x[j];
              le_tq &= x[j] <= mv.c[q][j];
              ne |= mv.c[q][j] != x[j];
            }
            const u64 m = 1ull << ((q % 4) * kWideVin + (unsigned)t);
            if (!le_qt) a[q / 4] &= ~m;
            if (!le_tq) a[QW + q / 4] &= ~m;
            if (ne) o[q / 4] |= m;
          }
        }
        wide_vote<NA, NO>(a, o, red);
        const u64 v2m = o[NO - 1];
        unsigned keep = mv.vm;
#pragma unroll
        for (int q = 0; q < VOS; ++q) {  // own < some non-empty incoming value: dropped
          const u64 lt = (a[q / 4] & o[q / 4]) >> ((q % 4) * kWideVin);
          if ((keep & (1u << q)) && (lt & v2m & 0xffffull)) keep &= ~(1u << q);
        }
        mv.vm = keep;
        for (unsigned long long t = 0; t < V; ++t) {
          if (!((v2m >> t) & 1)) continue;
          bool add = true;
#pragma unroll
          for (int q = 0; q < VOS; ++q)  // incoming <= a kept own value: not added
            if ((keep & (1u << q)) && ((a[QW + q / 4] >> ((q % 4) * kWideVin + t)) & 1)) add = false;
          if (add) {
            u64 x[kWideApt];
#pragma unroll
            for (int j = 0; j < kWideApt; ++j) x[j] = on[j] ? vcp[t * A + act[j]] : 0;
            wide_mv_append(mv, x, vvp[t], ovf);
          }
        }
        if (dl_any) wide_mv_forget(mv, dl, red);
      }
    }

    // ---- 2. deferred removes active at step i (map.rs:213-219, :311-348) ----
    bool activating;
    if (direct) {
      activating = dp < dend && p.def_row[dp] <= i;
    } else {
      activating = lp < nl && lrow[lp] <= i;
    }
    if (activating || nlive > 0 || rescan) {
      u64 ceil[kWideApt];
#pragma unroll
      for (int j = 0; j < kWideApt; ++j) ceil[j] = 0;
      bool have = false;
      auto fold_in = [&](unsigned long long d) {
#pragma unroll
        for (int j = 0; j < kWideApt; ++j) {
          const u64 x = on[j] ? p.def_clock[d * A + act[j]] : 0;
          ceil[j] = ceil[j] > x ? ceil[j] : x;
        }
        have = true;
      };
      if (!rescan) {
        // expire: a live remove the acc clock (before step i) dominates is dead for good
        unsigned long long w = 0;
        for (unsigned long long base = 0; base < nlive; base += 64) {
          const unsigned long long nb = nlive - base < 64 ? nlive - base : 64;
          u64 a[1] = {~0ull}, o[1] = {0};
          for (unsigned long long x = 0; x < nb; ++x) {
            const unsigned long long d = live[base + x];
            bool ge = true;
#pragma unroll
            for (int j = 0; j < kWideApt; ++j) ge &= !on[j] || cs[j] >= p.def_clock[d * A + act[j]];
            if (!ge) a[0] &= ~(1ull << x);
          }
          wide_vote<1, 0>(a, o, red);  // bit x: dominated everywhere
          __syncthreads();             // every thread has read live[] of this batch
          if (tid == 0) {              // compaction: entry w <= base + x, never an unread one
            unsigned long long ww = w;
            for (unsigned long long x = 0; x < nb; ++x)
              if (!((a[0] >> x) & 1)) live[ww++] = live[base + x];
          }
          w += nb - __popcll(a[0] & (nb == 64 ? ~0ull : ((1ull << nb) - 1)));
          __syncthreads();
        }
        nlive = w;
      }
      // activate the removes held by replica i that name this key
      while (true) {
        unsigned long long d;
        if (!direct) {
          if (lp >= nl || lrow[lp] > i) break;
          d = lidx[lp++];
        } else {
          if (dp >= dend || p.def_row[dp] > i) break;
          d = dp++;
          if (!(p.def_keys[d * p.Kw + kw] & kbit)) continue;
        }
        if (!rescan && nlive < (unsigned long long)kWideLive) {
          if (tid == 0) live[nlive] = (unsigned)d;
          ++nlive;
        } else {
          rescan = true;
        }
      }
      __syncthreads();  // the activated entries are visible to every thread
      if (!rescan) {
        for (unsigned long long x = 0; x < nlive; ++x) fold_in(live[x]);
      } else {  // every started remove: live iff held by replica i or not dominated by the acc clock
        const unsigned long long nscan = direct ? dp - dbeg : lp;
        for (unsigned long long x = 0; x < nscan; ++x) {
          const unsigned long long d = direct ? dbeg + x : lidx[x];
          if (direct && !(p.def_keys[d * p.Kw + kw] & kbit)) continue;
          bool ge = true;
#pragma unroll
          for (int j = 0; j < kWideApt; ++j) ge &= !on[j] || cs[j] >= p.def_clock[d * A + act[j]];
          if (p.def_row[d] == i || !wide_all(ge, red)) fold_in(d);
        }
      }
      if (have && present) {
        bool nz = false;
#pragma unroll
        for (int j = 0; j < kWideApt; ++j) {
          e[j] = e[j] > ceil[j] ? e[j] : 0;
          nz |= e[j] != 0;
        }
        if (!wide_any(nz, red)) {
          present = false;
          mv.vm = 0;
        } else {
          wide_mv_forget(mv, ceil, red);
        }
      }
    }
    // ---- 3. acc.clock.merge(other.clock) (map.rs:217) ----
#pragma unroll
    for (int j = 0; j < kWideApt; ++j) cs[j] = cs[j] > ico[j] ? cs[j] : ico[j];
  }
  if (direct && dp < dend) bad = true;  // a row >= R was never reached

  // ---- egress: value slots in Vec order (ascending order key) ----
  const int nv = __builtin_popcount(mv.vm);
  if (nv > (int)p.Vout) ovf |= 1;
  int rank[VOS];
#pragma unroll
  for (int q = 0; q < VOS; ++q) {
    rank[q] = -1;
    if (mv.vm & (1u << q)) {
      int r = 0;
#pragma unroll
      for (int q2 = 0; q2 < VOS; ++q2)
        if ((mv.vm & (1u << q2)) && mv.seq[q2] < mv.seq[q]) ++r;
      rank[q] = r;
    }
  }
  const unsigned long long gk = g * p.K + k;
#pragma unroll
  for (int j = 0; j < kWideApt; ++j) {
    if (!on[j]) continue;
    const unsigned long long a = act[j];
    p.o_ec[gk * A + a] = present ? e[j] : 0;
    if (k == 0) p.o_clock[g * A + a] = cs[j];
    for (unsigned long long o = 0; o < p.Vout; ++o) {
      u64 x = 0;
#pragma unroll
      for (int q = 0; q < VOS; ++q)
        if (rank[q] == (int)o) x = mv.c[q][j];
      p.o_vclk[(gk * p.Vout + o) * A + a] = x;
    }
  }
  if (tid == 0) {
    for (unsigned long long o = 0; o < p.Vout; ++o) {
      u64 v = 0;
#pragma unroll
      for (int q = 0; q < VOS; ++q)
        if (rank[q] == (int)o) v = mv.v[q];
      p.o_vval[gk * p.Vout + o] = v;
    }
    if (p.o_nval) p.o_nval[gk] = present ? (unsigned)nv : 0u;
    const unsigned f = (unsigned)ovf | (bad ? 2u : 0u);
    if (f) atomicOr(p.o_flags + g, f);
  }
}

// The wide fold of crdt_map_lub_many (map.hip dispatches here when A > 256 or V > 8): the state
// holds VOS = 4, 8 or 16 values (the caller's Vstate / Vout, retried larger on flags bit 2).
int map_lub_wide(crdt_ctx *ctx, const crdt_map_batch *in, const size_t *def_off_dev, crdt_map_out *out) {
  const size_t A = in->A, V = in->V;
  if (A > 1024) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: A = %zu > 1024 actors", A);
  if (V > (size_t)kWideVin) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: V = %zu > %d value slots", V, kWideVin);
  MapWidePlan p{};
  p.clock = (const u64 *)in->clock;
  p.c_rs = in->clock_rstride;
  p.c_gs = in->clock_gstride;
  p.ec = (const u64 *)in->ec;
  p.e_rs = in->ec_rstride;
  p.e_gs = in->ec_gstride;
  p.vclk = (const u64 *)in->vclk;
  p.vc_rs = in->vclk_rstride;
  p.vc_gs = in->vclk_gstride;
  p.vval = (const u64 *)in->vval;
  p.vv_rs = in->vval_rstride;
  p.vv_gs = in->vval_gstride;
  p.def_off = def_off_dev;
  p.def_row = in->def_row;
  p.def_clock = (const u64 *)in->def_clock;
  p.def_keys = (const u64 *)in->def_keys;
  p.G = in->G;
  p.R = in->R;
  p.K = in->K;
  p.A = A;
  p.V = V;
  p.Kw = (in->K + 63) / 64;
  p.Vout = out->Vout;
  p.o_clock = (u64 *)out->clock;
  p.o_ec = (u64 *)out->ec;
  p.o_vclk = (u64 *)out->vclk;
  p.o_vval = (u64 *)out->vval;
  p.o_nval = out->nval;
  p.o_flags = out->flags;
  const size_t want = std::max<size_t>(std::max(out->Vstate, out->Vout), V);
  const unsigned nt = (unsigned)std::min<size_t>(256, std::max<size_t>(64, (A + 4 * 64 - 1) / (4 * 64) * 64));
  const unsigned long long blocks = in->G * in->K;
  timing_begin(ctx, "map_fold");
  if (want <= 4) hipLaunchKernelGGL(map_fold_wide_kernel<4>, dim3((unsigned)blocks), dim3(nt), 0, ctx->stream, p);
  else if (want <= 8) hipLaunchKernelGGL(map_fold_wide_kernel<8>, dim3((unsigned)blocks), dim3(nt), 0, ctx->stream, p);
  else hipLaunchKernelGGL(map_fold_wide_kernel<16>, dim3((unsigned)blocks), dim3(nt), 0, ctx->stream, p);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

}  // namespace crdt
