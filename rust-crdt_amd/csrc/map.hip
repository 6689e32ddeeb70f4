// Map<K, MVReg<u64>> batched merge: G independent left folds of R replicas (BASELINE config 4).
//
// Reference: Map::merge (map.rs:140-220), apply_keyset_rm (:318-348), apply_deferred (:311-316),
// MVReg::merge (mvreg.rs:112-128), MVReg::forget (:88-104), VClock::forget / intersection /
// clone_without / partial_cmp (vclock.rs:68-80, :95-105, :148-152, :218-227).
//
// Why a per-key sequential fold.  Unlike the lattices and the Orswot dot store, the Map's value
// part is not a per-cell join: MVReg dominance (`clock < c`) compares whole clocks, and the
// reset-remove forgets rewrite value clocks with the other side's map clock, so the merge is not
// known to be associative for arbitrary states (the reference tests associativity only for
// distinct-actor histories, test/map.rs:660-692).  The kernel therefore computes the exact left
// fold `acc = Map::new(); for r: acc.merge(r)` for ANY input.  What makes that parallel: keys are
// independent given (a) the replica clocks, whose prefix max Cs(i) is acc.clock before step i,
// and (b) the deferred removes.  A remove d of replica j forgets its keys at step j and at every
// later step while it sits in acc.deferred, i.e. at step i > j iff !(Cs(i) >= rm)
// (map.rs:213-219 + :336-345); successive forgets compose to one forget by their max, so step
// i applies the max of the active removes naming the key.
//
// Mapping: one wave per (group, key); lane l holds actors l, l+64, ... (APL per lane), so every
// "for all actors" / "any actor" test is one vector compare + a wave vote (__all / __any), and
// all control flow is wave-uniform.  The replica stream (entry clock, VI value clocks, VI values
// and the replica clock) is software-pipelined PF replicas ahead in registers.
//
// Per step i with e = acc entry clock, e2 = replica entry clock, Co = replica clock:
//   acc only      (:146-161): Co >= e ? drop : e = e>Co?e:0, vals.forget(Co>e?Co:0)
//   replica only  (:193-208): Cs >= e2 ? skip : e = e2>Cs?e2:0, vals = vals2.forget(Cs>e?Cs:0)
//   both          (:170-192): common = max(e==e2?e:0, e2>Cs?e2:0, e>Co?e:0); empty ? drop :
//                             vals = mvreg_merge(vals, vals2).forget(max(e,e2) > common ? max : 0),
//                             e = common
//   then the deferred ceiling forgets the entry (and drops it when its clock empties).
#include "common.hpp"

namespace crdt {

struct MapPlan {
  const u64 *clock;
  long long c_rs, c_gs;
  const u64 *ec;  // replica block K*A
  long long e_rs, e_gs;
  const u64 *vclk;  // replica block K*V*A
  long long vc_rs, vc_gs;
  const u64 *vval;  // replica block K*V
  long long vv_rs, vv_gs;
  const size_t *def_off;  // device copy [G+1] (nullptr: no deferred)
  const unsigned *def_row;
  const u64 *def_clock;
  const u64 *def_keys;
  unsigned long long G, R, K, A, V, Kw, Vout;
  u64 *o_clock, *o_ec, *o_vclk, *o_vval;
  unsigned *o_nval;
  unsigned *o_flags;  // per group: bit0 > Vout values, bit1 bad def_row, bit2 state capacity
};

constexpr int kMapQ = 4;  // deferred removes tracked per key in registers before the slow path

template <int APL, int VI>
struct MapStep {
  u64 e[APL];
  u64 c[VI][APL];
  u64 co[APL];
  u64 v[VI];
};

__device__ __forceinline__ bool wall(bool x) { return __all(x); }
__device__ __forceinline__ bool wany(bool x) { return __any(x); }

template <int APL>
__device__ __forceinline__ bool all_ge(const u64 (&x)[APL], const u64 (&y)[APL]) {
  bool t = true;
#pragma unroll
  for (int j = 0; j < APL; ++j) t &= x[j] >= y[j];
  return wall(t);
}
template <int APL>
__device__ __forceinline__ bool any_nz(const u64 (&x)[APL]) {
  bool t = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) t |= x[j] != 0;
  return wany(t);
}
// VClock partial_cmp(x, y) == Less on dense rows: x <= y everywhere and x != y somewhere.
template <int APL>
__device__ __forceinline__ bool vlt(const u64 (&x)[APL], const u64 (&y)[APL]) {
  bool le = true, ne = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    le &= x[j] <= y[j];
    ne |= x[j] != y[j];
  }
  return wall(le) && wany(ne);
}
// x < y || x == y
template <int APL>
__device__ __forceinline__ bool vle(const u64 (&x)[APL], const u64 (&y)[APL]) {
  bool le = true;
#pragma unroll
  for (int j = 0; j < APL; ++j) le &= x[j] <= y[j];
  return wall(le);
}
// VClock::forget: keep x[a] iff x[a] > y[a]
template <int APL>
__device__ __forceinline__ void vforget(u64 (&x)[APL], const u64 (&y)[APL]) {
#pragma unroll
  for (int j = 0; j < APL; ++j) x[j] = x[j] > y[j] ? x[j] : 0;
}

// The MVReg state of one key: n values, value clocks per lane, values wave-uniform.
template <int APL, int VO>
struct MVState {
  u64 c[VO][APL];
  u64 v[VO];
  int n;
};

// Append (x, val) at position n (uniform); past VO the state overflows (flag, value dropped).
template <int APL, int VO>
__device__ __forceinline__ void mv_push(MVState<APL, VO> &s, const u64 (&x)[APL], u64 val, int &ovf) {
  if (s.n >= VO) {
    ovf |= 4;  // the fold state itself ran out of value slots (results incomplete)
    return;
  }
#pragma unroll
  for (int q = 0; q < VO; ++q)
    if (q == s.n) {
#pragma unroll
      for (int j = 0; j < APL; ++j) s.c[q][j] = x[j];
      s.v[q] = val;
    }
  s.n++;
}

// vals.forget(X) (mvreg.rs:88-104): forget every value clock, drop the emptied ones, keep order.
template <int APL, int VO>
__device__ __forceinline__ void mv_forget(MVState<APL, VO> &s, const u64 (&X)[APL], int &ovf) {
  MVState<APL, VO> o;
  o.n = 0;
#pragma unroll
  for (int q = 0; q < VO; ++q) {
    if (q < s.n) {
      u64 x[APL];
#pragma unroll
      for (int j = 0; j < APL; ++j) x[j] = s.c[q][j];
      vforget(x, X);
      if (any_nz(x)) mv_push(o, x, s.v[q], ovf);
    }
  }
  s = o;
}

// Replica stream staging.  A chunk of C replicas is loaded into registers (every load in
// flight at once), written to one half of a per-wave LDS double buffer while the fold runs over
// the other half, so each chunk's loads have a whole chunk of fold steps to land.  The fold
// reads its step from LDS (dynamic index, no unrolled register ring).  LDS step image, W words:
//   [0, A) entry clock | [(1+t)A, (2+t)A) value clock t < VI | [(1+VI)A, (2+VI)A) replica clock
//   | [(2+VI)A, (2+VI)A + VI) values
template <int APL, int VI>
struct MapChunk {
  static constexpr int words = (2 + VI) * APL + 1;  // u64 registers per staged replica per lane
  static constexpr int raw = (APL >= 4 ? 48 : 96) / words;
  static constexpr int C = raw > 16 ? 16 : (raw < 2 ? 2 : raw);
  u64 e[C][APL];
  u64 c[C][VI][APL];
  u64 co[C][APL];
  u64 v[C];  // lane t < VI holds value slot t
};

template <int APL, int VI>
__device__ __forceinline__ void map_chunk_load(MapChunk<APL, VI> &r, const MapPlan &p,
                                               unsigned long long g, unsigned long long k,
                                               unsigned long long i0, int lane) {
  constexpr int C = MapChunk<APL, VI>::C;
#pragma unroll
  for (int s = 0; s < C; ++s) {
    const unsigned long long i = i0 + s;
    if (i < p.R) {
      const u64 *ec = p.ec + g * p.e_gs + i * p.e_rs + k * p.A;
      const u64 *vc = p.vclk + g * p.vc_gs + i * p.vc_rs + k * p.V * p.A;
      const u64 *cl = p.clock + g * p.c_gs + i * p.c_rs;
#pragma unroll
      for (int j = 0; j < APL; ++j) {
        const unsigned long long a = lane + 64ull * j;
        const bool on = a < p.A;
        r.e[s][j] = on ? __builtin_nontemporal_load(ec + a) : 0;
        r.co[s][j] = on ? cl[a] : 0;
#pragma unroll
        for (int t = 0; t < VI; ++t)
          r.c[s][t][j] = (on && (unsigned long long)t < p.V) ? __builtin_nontemporal_load(vc + t * p.A + a) : 0;
      }
      const u64 *vv = p.vval + g * p.vv_gs + i * p.vv_rs + k * p.V;
      r.v[s] = (unsigned long long)lane < p.V ? __builtin_nontemporal_load(vv + lane) : 0;
    }
  }
}

template <int APL, int VI>
__device__ __forceinline__ void map_chunk_store(const MapChunk<APL, VI> &r, u64 *buf,
                                                unsigned long long A, unsigned long long W,
                                                unsigned long long nsteps, int lane) {
  constexpr int C = MapChunk<APL, VI>::C;
#pragma unroll
  for (int s = 0; s < C; ++s) {
    if ((unsigned long long)s < nsteps) {
      u64 *st = buf + s * W;
#pragma unroll
      for (int j = 0; j < APL; ++j) {
        const unsigned long long a = lane + 64ull * j;
        if (a < A) {
          st[a] = r.e[s][j];
#pragma unroll
          for (int t = 0; t < VI; ++t) st[(1 + t) * A + a] = r.c[s][t][j];
          st[(1 + VI) * A + a] = r.co[s][j];
        }
      }
      if (lane < VI) st[(2 + VI) * A + lane] = r.v[s];
    }
  }
}

template <int APL, int VI>
__device__ __forceinline__ MapStep<APL, VI> map_step_read(const u64 *st, unsigned long long A, int lane) {
  MapStep<APL, VI> in;
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = lane + 64ull * j;
    const bool on = a < A;
    in.e[j] = on ? st[a] : 0;
#pragma unroll
    for (int t = 0; t < VI; ++t) in.c[t][j] = on ? st[(1 + t) * A + a] : 0;
    in.co[j] = on ? st[(1 + VI) * A + a] : 0;
  }
#pragma unroll
  for (int t = 0; t < VI; ++t) in.v[t] = st[(2 + VI) * A + t];
  return in;
}

template <int APL, int VI, int VO>
__global__ __launch_bounds__(64) void map_fold_kernel(MapPlan p) {
  const unsigned long long g = blockIdx.x / p.K;
  const unsigned long long k = blockIdx.x % p.K;
  const int lane = threadIdx.x;
  const unsigned long long R = p.R;

  bool present = false;
  u64 e[APL], cs[APL];
#pragma unroll
  for (int j = 0; j < APL; ++j) e[j] = cs[j] = 0;
  MVState<APL, VO> mv;
  mv.n = 0;
#pragma unroll
  for (int q = 0; q < VO; ++q) {
    mv.v[q] = 0;
#pragma unroll
    for (int j = 0; j < APL; ++j) mv.c[q][j] = 0;
  }
  int ovf = 0, bad = 0;

  // deferred removes of this group, in replica order
  unsigned long long dbeg = 0, dend = 0;
  if (p.def_off) {
    dbeg = p.def_off[g];
    dend = p.def_off[g + 1];
  }
  unsigned long long dp = dbeg;
  u64 rq[kMapQ][APL];
  int nq = 0;
  bool slow = false;
#pragma unroll
  for (int q = 0; q < kMapQ; ++q)
#pragma unroll
    for (int j = 0; j < APL; ++j) rq[q][j] = 0;
  const unsigned long long kw = k / 64;
  const u64 kbit = 1ull << (k % 64);

  extern __shared__ u64 map_lds[];
  constexpr int C = MapChunk<APL, VI>::C;
  const unsigned long long A = p.A;
  const unsigned long long W = (2 + VI) * A + VI;
  u64 *lbuf[2] = {map_lds, map_lds + C * W};
  const unsigned long long nch = (R + C - 1) / C;
  MapChunk<APL, VI> regs;
  if (nch > 0) {
    map_chunk_load(regs, p, g, k, 0, lane);
    map_chunk_store(regs, lbuf[0], A, W, R < (unsigned long long)C ? R : C, lane);
    if (nch > 1) map_chunk_load(regs, p, g, k, C, lane);
  }

  for (unsigned long long ch = 0; ch < nch; ++ch) {
    const u64 *buf = lbuf[ch & 1];
    const unsigned long long i0 = ch * C;
    const unsigned long long n = R - i0 < (unsigned long long)C ? R - i0 : C;
    MapStep<APL, VI> nxt = map_step_read<APL, VI>(buf, A, lane);
#pragma unroll 1
    for (unsigned long long s = 0; s < n; ++s) {
      const unsigned long long i = i0 + s;
      const MapStep<APL, VI> in = nxt;
      if (s + 1 < n) nxt = map_step_read<APL, VI>(buf + (s + 1) * W, A, lane);
      {
      // ---- 1. entry join (map.rs:142-210) ----
      const bool p2 = any_nz(in.e);
      if (present && !p2) {
        if (all_ge(in.co, e)) {
          present = false;
          mv.n = 0;
#pragma unroll
          for (int j = 0; j < APL; ++j) e[j] = 0;
        } else {
          u64 ri[APL];
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            e[j] = e[j] > in.co[j] ? e[j] : 0;
            ri[j] = in.co[j] > e[j] ? in.co[j] : 0;
          }
          mv_forget(mv, ri, ovf);
        }
      } else if (!present && p2) {
        if (!all_ge(cs, in.e)) {
          u64 ri[APL];
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            e[j] = in.e[j] > cs[j] ? in.e[j] : 0;
            ri[j] = cs[j] > e[j] ? cs[j] : 0;
          }
          mv.n = 0;
#pragma unroll
          for (int t = 0; t < VI; ++t) {
            if (any_nz(in.c[t])) {
              u64 x[APL];
#pragma unroll
              for (int j = 0; j < APL; ++j) x[j] = in.c[t][j];
              vforget(x, ri);
              if (any_nz(x)) mv_push(mv, x, in.v[t], ovf);
            }
          }
          present = true;
        }
      } else if (present && p2) {
        u64 common[APL], dl[APL];
#pragma unroll
        for (int j = 0; j < APL; ++j) {
          const u64 t0 = e[j] == in.e[j] ? e[j] : 0;
          const u64 t1 = in.e[j] > cs[j] ? in.e[j] : 0;
          const u64 t2 = e[j] > in.co[j] ? e[j] : 0;
          u64 c = t0 > t1 ? t0 : t1;
          common[j] = c > t2 ? c : t2;
          const u64 m = e[j] > in.e[j] ? e[j] : in.e[j];
          dl[j] = m > common[j] ? m : 0;
        }
        if (!any_nz(common)) {
          present = false;
          mv.n = 0;
#pragma unroll
          for (int j = 0; j < APL; ++j) e[j] = 0;
        } else {
          // MVReg::merge then forget(deleted) (map.rs:183-188, mvreg.rs:112-128)
          bool ne2[VI];
#pragma unroll
          for (int t = 0; t < VI; ++t) ne2[t] = any_nz(in.c[t]);
          bool keep1[VO];
#pragma unroll
          for (int s = 0; s < VO; ++s) {
            keep1[s] = s < mv.n;
            if (keep1[s]) {
#pragma unroll
              for (int t = 0; t < VI; ++t)
                if (ne2[t] && vlt(mv.c[s], in.c[t])) keep1[s] = false;
            }
          }
          bool keep2[VI];
#pragma unroll
          for (int t = 0; t < VI; ++t) {
            keep2[t] = ne2[t];
            if (keep2[t]) {
#pragma unroll
              for (int s = 0; s < VO; ++s)
                if (keep1[s] && vle(in.c[t], mv.c[s])) keep2[t] = false;
            }
          }
          MVState<APL, VO> o;
          o.n = 0;
#pragma unroll
          for (int s = 0; s < VO; ++s) {
            if (keep1[s]) {
              u64 x[APL];
#pragma unroll
              for (int j = 0; j < APL; ++j) x[j] = mv.c[s][j];
              vforget(x, dl);
              if (any_nz(x)) mv_push(o, x, mv.v[s], ovf);
            }
          }
#pragma unroll
          for (int t = 0; t < VI; ++t) {
            if (keep2[t]) {
              u64 x[APL];
#pragma unroll
              for (int j = 0; j < APL; ++j) x[j] = in.c[t][j];
              vforget(x, dl);
              if (any_nz(x)) mv_push(o, x, in.v[t], ovf);
            }
          }
          mv = o;
#pragma unroll
          for (int j = 0; j < APL; ++j) e[j] = common[j];
        }
      }

      // ---- 2. deferred removes active at step i (map.rs:213-219, :311-348) ----
      if (dp < dend || nq > 0 || slow) {
        if (!slow) {  // expire: dropped from acc.deferred once acc.clock (= Cs) dominates it
          int w = 0;
#pragma unroll
          for (int q = 0; q < kMapQ; ++q) {
            if (q < nq && !all_ge(cs, rq[q])) {
#pragma unroll
              for (int r2 = 0; r2 < kMapQ; ++r2)
                if (r2 == w)
#pragma unroll
                  for (int j = 0; j < APL; ++j) rq[r2][j] = rq[q][j];
              ++w;
            }
          }
          nq = w;
        }
        while (dp < dend) {
          const unsigned row = p.def_row[dp];
          if (row > i) break;
          if (row < i) bad = 1;  // rows must be non-decreasing within the group
          if (p.def_keys[dp * p.Kw + kw] & kbit) {
            if (!slow && nq < kMapQ) {
#pragma unroll
              for (int q = 0; q < kMapQ; ++q)
                if (q == nq)
#pragma unroll
                  for (int j = 0; j < APL; ++j) {
                    const unsigned long long a = lane + 64ull * j;
                    rq[q][j] = a < p.A ? p.def_clock[dp * p.A + a] : 0;
                  }
              ++nq;
            } else {
              slow = true;
            }
          }
          ++dp;
        }
        u64 ceil[APL];
        bool have = false;
#pragma unroll
        for (int j = 0; j < APL; ++j) ceil[j] = 0;
        if (!slow) {
#pragma unroll
          for (int q = 0; q < kMapQ; ++q)
            if (q < nq) {
              have = true;
#pragma unroll
              for (int j = 0; j < APL; ++j) ceil[j] = ceil[j] > rq[q][j] ? ceil[j] : rq[q][j];
            }
        } else {  // more than kMapQ concurrent removes on this key: rescan every started one
          for (unsigned long long d = dbeg; d < dp; ++d) {
            if (!(p.def_keys[d * p.Kw + kw] & kbit)) continue;
            u64 rm[APL];
#pragma unroll
            for (int j = 0; j < APL; ++j) {
              const unsigned long long a = lane + 64ull * j;
              rm[j] = a < p.A ? p.def_clock[d * p.A + a] : 0;
            }
            if (p.def_row[d] == i || !all_ge(cs, rm)) {
              have = true;
#pragma unroll
              for (int j = 0; j < APL; ++j) ceil[j] = ceil[j] > rm[j] ? ceil[j] : rm[j];
            }
          }
        }
        if (have && present) {
          vforget(e, ceil);
          if (!any_nz(e)) {
            present = false;
            mv.n = 0;
          } else {
            mv_forget(mv, ceil, ovf);
          }
        }
      }

      // ---- 3. acc.clock.merge(other.clock) (map.rs:217) ----
#pragma unroll
      for (int j = 0; j < APL; ++j) cs[j] = cs[j] > in.co[j] ? cs[j] : in.co[j];
      }
    }
    if (ch + 1 < nch) {  // stage the next chunk (its loads were issued a whole chunk ago)
      const unsigned long long nn = R - (ch + 1) * C < (unsigned long long)C ? R - (ch + 1) * C : C;
      map_chunk_store(regs, lbuf[(ch + 1) & 1], A, W, nn, lane);
      if (ch + 2 < nch) map_chunk_load(regs, p, g, k, (ch + 2) * C, lane);
    }
  }
  if (dp < dend) bad = 1;  // a row >= R was never reached

  // ---- egress ----
  if (mv.n > (int)p.Vout) ovf |= 1;
  const unsigned long long gk = g * p.K + k;
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = lane + 64ull * j;
    if (a < p.A) {
      p.o_ec[gk * p.A + a] = present ? e[j] : 0;
      if (k == 0) p.o_clock[g * p.A + a] = cs[j];
#pragma unroll
      for (int q = 0; q < VO; ++q)
        if ((unsigned long long)q < p.Vout) p.o_vclk[(gk * p.Vout + q) * p.A + a] = q < mv.n ? mv.c[q][j] : 0;
    }
  }
  // slots beyond the template capacity (Vout > VO) are zero
  for (unsigned long long q = VO; q < p.Vout; ++q)
    for (unsigned long long a = lane; a < p.A; a += 64) p.o_vclk[(gk * p.Vout + q) * p.A + a] = 0;
  if (lane == 0) {
    for (unsigned long long q = 0; q < p.Vout; ++q) {
      u64 v = 0;
#pragma unroll
      for (int s = 0; s < VO; ++s)
        if ((unsigned long long)s == q && s < mv.n) v = mv.v[s];
      p.o_vval[gk * p.Vout + q] = v;
    }
    if (p.o_nval) p.o_nval[gk] = present ? (unsigned)mv.n : 0u;
    const unsigned f = (unsigned)ovf | (bad ? 2u : 0u);
    if (f) atomicOr(p.o_flags + g, f);
  }
}

}  // namespace crdt

using namespace crdt;

template <int APL, int VI, int VO>
static hipError_t launch_map(const MapPlan &p, unsigned long long blocks, hipStream_t s) {
  const size_t W = (2 + VI) * p.A + VI;
  const size_t lds = 2 * (size_t)MapChunk<APL, VI>::C * W * sizeof(u64);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 64 * 1024) {  // beyond the default dynamic-LDS limit (gfx950 has 160 KB per CU)
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&map_fold_kernel<APL, VI, VO>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((map_fold_kernel<APL, VI, VO>), dim3((unsigned)blocks), dim3(64), lds, s, p);
  return hipGetLastError();
}

template <int APL>
static hipError_t launch_map_vi(const MapPlan &p, int VI, unsigned long long blocks, hipStream_t s) {
  switch (VI) {
    case 1: return launch_map<APL, 1, 2>(p, blocks, s);
    case 2: return launch_map<APL, 2, 4>(p, blocks, s);
    default: return launch_map<APL, 4, 8>(p, blocks, s);
  }
}

extern "C" int crdt_map_lub_many(crdt_ctx *ctx, const crdt_map_batch *in, crdt_map_out *out) {
  CRDT_CHECK_CTX(ctx);
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "map_lub_many: NULL batch/out");
  const size_t G = in->G, R = in->R, K = in->K, A = in->A, V = in->V, Vout = out->Vout;
  if (G == 0 || K == 0 || A == 0) return CRDT_OK;
  if (!out->clock || !out->ec || !out->vclk || !out->vval || !out->flags)
    return fail(ctx, CRDT_EINVAL, "map_lub_many: NULL output");
  if (Vout == 0) return fail(ctx, CRDT_EINVAL, "map_lub_many: Vout must be >= 1");
  if (R > 0 && (!in->clock || !in->ec || (V > 0 && (!in->vclk || !in->vval))))
    return fail(ctx, CRDT_EINVAL, "map_lub_many: NULL input");
  if (A > 256) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: A = %zu > 256 actors", A);
  if (V > 4) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: V = %zu > 4 value slots per key", V);
  if (Vout > 64) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: Vout = %zu > 64", Vout);
  if (G * K > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: G*K too large");
  if (R > 0xfffffffeULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: R too large");
  const size_t D = (in->def_off && G > 0) ? in->def_off[G] - in->def_off[0] : 0;
  if (in->def_off && in->def_off[0] != 0) return fail(ctx, CRDT_EINVAL, "map_lub_many: def_off[0] must be 0");
  if (D > 0 && (!in->def_row || !in->def_clock || !in->def_keys || !out->def_keep || !out->def_keys))
    return fail(ctx, CRDT_EINVAL, "map_lub_many: deferred buffers missing");
  if (D > 0xffffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: too many deferred");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const size_t Kw = (K + 63) / 64;

  MapPlan p{};
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
  p.G = G;
  p.R = R;
  p.K = K;
  p.A = A;
  p.V = V;
  p.Kw = Kw;
  p.Vout = Vout;
  p.o_clock = (u64 *)out->clock;
  p.o_ec = (u64 *)out->ec;
  p.o_vclk = (u64 *)out->vclk;
  p.o_vval = (u64 *)out->vval;
  p.o_nval = out->nval;
  p.o_flags = out->flags;
  if (int rc = device_fill(ctx, out->flags, G * sizeof(unsigned), 0)) return rc;
  if (D > 0) {
    // the kernel walks def_off on the device: stage it (the caller's array may be freed)
    const size_t off_b = (G + 1) * sizeof(size_t);
    if (int rc = ensure_scratch(ctx, off_b)) return rc;
    if (int rc = stage_h2d(ctx, ctx->scratch, in->def_off, off_b)) return rc;
    p.def_off = reinterpret_cast<const size_t *>(ctx->scratch);
    p.def_row = in->def_row;
    p.def_clock = (const u64 *)in->def_clock;
    p.def_keys = (const u64 *)in->def_keys;
  }
  // value-slot templates: VI >= V input slots, VO = 2*VI state slots >= min(8, Vout, Vstate)
  const size_t want = out->Vstate > Vout ? out->Vstate : Vout;
  int VI = 1;
  while ((size_t)VI < V || (size_t)(2 * VI) < (want < 8 ? want : 8)) VI *= 2;
  if (VI > 4) VI = 4;
  const int APL = A <= 64 ? 1 : (A <= 128 ? 2 : 4);
  const unsigned long long blocks = G * K;
  timing_begin(ctx, "map_fold");
  hipError_t he;
  if (APL == 1) he = launch_map_vi<1>(p, VI, blocks, ctx->stream);
  else if (APL == 2) he = launch_map_vi<2>(p, VI, blocks, ctx->stream);
  else he = launch_map_vi<4>(p, VI, blocks, ctx->stream);
  timing_end(ctx);
  if (he != hipSuccess) return hip_fail(ctx, he, "map_fold_kernel launch");

  if (D == 0) return CRDT_OK;
  DefPlan q{};
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
