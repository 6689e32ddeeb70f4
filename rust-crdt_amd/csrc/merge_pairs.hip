// Pairwise in-place merge_batch for the causal types: N independent `self[i].merge(other[i])`
// (CvRDT::merge, traits.rs:4-7) on the per-state layouts of the apply entry points
// (crdt_orswot_states / crdt_map_states + deferred slots), exact for ANY pair of states.
//
// Orswot::merge (orswot.rs:81-149).  Per member m, actor a, with e1/e2 the entry cells and c1/c2
// the clocks BEFORE the merge, the entry phase (:84-138) is the per-cell dot-store join
//   e = max(e1 == e2 ? e1 : 0, e1 > c2 ? e1 : 0, e2 > c1 ? e2 : 0)
// (intersection ∪ clone_without ∪ clone_without, and forget / drop-if-dominated for one-sided
// members; an all-zero row is an absent member, so it is exact without any invariant).  Then
// other.deferred is applied (apply_rm :141-143), the clocks merge (:145) and apply_deferred (:147)
// re-applies self.deferred (its old removes plus other's that were deferred).  Successive forgets
// of one entry compose to one forget by their max, and re-applying is idempotent, so the entry
// result is: join, then forget by the ceiling Rc[m] = max of the rm clocks of EVERY deferred
// remove of either side that names m.  A remove survives iff !(rm <= merged clock) (:240-249);
// survivors with an identical clock merge their member sets (the HashMap<VClock, HashSet<M>>).
//
// Map<K, MVReg<u64>>::merge (map.rs:140-220) has the same skeleton per key (entry clock join with
// the reset-remove value forgets of :146-208, MVReg::merge mvreg.rs:112-128 for keys on both
// sides, then every deferred remove naming the key forgets the entry and its values,
// apply_keyset_rm :318-348).  Keys are independent given the two clocks and the two deferred
// lists: one wave per (pair, key), lane = actor.
//
// Kernels: *_pair_join (entries / keys, bandwidth-bound: read self, read other, write self),
// then pair_deferred_kernel (one wave per pair: merged clock, surviving removes compacted into
// self's slots).  The second launch runs after the first on the ctx stream, so the join reads
// the pre-merge clock and deferred lists of self.
#include "common.hpp"

namespace crdt {

__device__ __forceinline__ void pfence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup"); }
__device__ __forceinline__ bool pany(bool x) { return __ballot(x) != 0; }

// ---- shared: surviving deferred removes of a pair ------------------------------------------------
struct PairDefPlan {
  unsigned long long N, A, BW;  // BW: bitmap words per remove (members / keys)
  u64 *c1;                      // self clock rows (written: merged clock)
  unsigned long long c1_s;
  const u64 *c2;
  unsigned long long c2_s;
  u64 *d1c, *d1b;  // self slots [N][D1][A], [N][D1][BW]
  uint32_t *d1n;
  unsigned long long D1;
  const u64 *d2c, *d2b;  // other slots
  const uint32_t *d2n;
  unsigned long long D2;
  uint32_t *status;
  unsigned status_or;  // bits the join kernel may already have set are OR-ed in (map: bit 4)
};

// One wave per pair: candidates are self's removes then other's (in slot order).  A candidate
// survives iff some rm[a] > max(c1[a], c2[a]); a survivor equal to an already kept clock ORs its
// bitmap into that slot, else it is compacted into self's next slot (never past one not yet read:
// the write slot is always <= the candidate index).
__global__ __launch_bounds__(kBlock) void pair_deferred_kernel(PairDefPlan p) {
  const int lane = threadIdx.x % kWave;
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;
  const unsigned long long nw = (unsigned long long)gridDim.x * (kBlock / kWave);
  for (unsigned long long s = w0; s < p.N; s += nw) {
    const unsigned n1 = p.d1n[s], n2 = p.d2n ? p.d2n[s] : 0u;
    if (n1 > p.D1 || n2 > p.D2) {
      if (lane == 0) p.status[s] = 4u;  // invalid counts: the state was left untouched
      continue;
    }
    u64 *c1 = p.c1 + s * p.c1_s;
    const u64 *c2 = p.c2 + s * p.c2_s;
    u64 *sc = p.d1c + s * p.D1 * p.A, *sb = p.d1b + s * p.D1 * p.BW;
    const u64 *oc = p.d2c ? p.d2c + s * p.D2 * p.A : nullptr, *ob = p.d2b ? p.d2b + s * p.D2 * p.BW : nullptr;
    unsigned st = (p.status_or && p.status) ? (p.status[s] & p.status_or) : 0u;
    unsigned nk = 0;
    for (unsigned j = 0; j < n1 + n2; ++j) {
      const u64 *rc = j < n1 ? sc + (unsigned long long)j * p.A : oc + (unsigned long long)(j - n1) * p.A;
      const u64 *rb = j < n1 ? sb + (unsigned long long)j * p.BW : ob + (unsigned long long)(j - n1) * p.BW;
      bool gt = false;
      for (unsigned long long a = lane; a < p.A; a += kWave) {
        const u64 x = c1[a], y = c2[a];
        gt |= rc[a] > (x > y ? x : y);
      }
      if (!pany(gt)) continue;  // rm <= merged clock: seen, dropped
      int slot = -1;
      for (unsigned t = 0; t < nk; ++t) {
        bool ne = false;
        for (unsigned long long a = lane; a < p.A; a += kWave) ne |= sc[(unsigned long long)t * p.A + a] != rc[a];
        if (!pany(ne)) {
          slot = (int)t;
          break;
        }
      }
      if (slot >= 0) {  // identical clock: union of the member / key sets
        for (unsigned long long w = lane; w < p.BW; w += kWave) sb[(unsigned long long)slot * p.BW + w] |= rb[w];
        pfence();
        continue;
      }
      if (nk >= p.D1) {
        st |= 1u;  // more survivors than self's slots: the state is incomplete
        continue;
      }
      if (!(j < n1 && j == nk)) {
        for (unsigned long long a = lane; a < p.A; a += kWave) sc[(unsigned long long)nk * p.A + a] = rc[a];
        for (unsigned long long w = lane; w < p.BW; w += kWave) sb[(unsigned long long)nk * p.BW + w] = rb[w];
      }
      pfence();
      ++nk;
    }
    // merged clock (:145) last: the survival tests above read the pre-merge c1
    for (unsigned long long a = lane; a < p.A; a += kWave) {
      const u64 x = c1[a], y = c2[a];
      c1[a] = x > y ? x : y;
    }
    if (lane == 0) {
      p.d1n[s] = nk;
      p.status[s] = st;
    }
    pfence();
  }
}

// ---- Orswot entry join --------------------------------------------------------------------------
constexpr int kPairGroups = 16;  // deferred removes per pair handled: 32 * kPairGroups
constexpr int kPairUR = 8;       // member rows per thread with loads in flight together

struct OrswotPairPlan {
  u64 *e1;
  unsigned long long e1_m, e1_s;
  const u64 *e2;
  unsigned long long e2_m, e2_s;
  const u64 *c1;
  unsigned long long c1_s;
  const u64 *c2;
  unsigned long long c2_s;
  const u64 *d1c, *d1b;
  const uint32_t *d1n;
  unsigned long long D1;
  const u64 *d2c, *d2b;
  const uint32_t *d2n;
  unsigned long long D2;
  unsigned long long N, M, A, Mw, mblocks;
  int lp_log;     // log2 lanes per member row (pieces of V words)
  unsigned dbase;  // the removes this launch applies: [dbase, dbase + 32 * kPairGroups) of the pair's
  int join;        // 1: join then forget; 0: forget only (a later pass of a pair with more removes)
};

__device__ __forceinline__ u64 cell_join(u64 e1, u64 e2, u64 c1, u64 c2) {  // orswot.rs:84-138
  const u64 t0 = e1 == e2 ? e1 : 0ull;
  const u64 t1 = e1 > c2 ? e1 : 0ull;
  const u64 t2 = e2 > c1 ? e2 : 0ull;
  const u64 t = t0 > t1 ? t0 : t1;
  return t > t2 ? t : t2;
}

// Workgroup = (pair s, block of kPairRows member rows); 2^lp_log lanes cover a row in V-word
// pieces (V = 2: 16-byte non-temporal accesses), 256 >> lp_log rows per pass.  Per block the
// deferred removes of both sides are turned into hit masks in LDS (bit d of hit[g][row] = remove
// dbase + 32g + d names that member); a cell with hits forgets by each hit remove's rm (global, L2).
// A pair with more than 32 * kPairGroups removes gets further forget-only launches (join = 0) for
// the rest: forgets of the joined entries compose and commute, so the passes give the same result.
template <int V, int kPairRows, int kPairUR = kPairUR>
__global__ __launch_bounds__(kBlock) void orswot_pair_join_kernel(OrswotPairPlan p) {
  __shared__ unsigned hit[kPairGroups][kPairRows];
  const unsigned long long s = blockIdx.x / p.mblocks;
  const unsigned long long m0 = (blockIdx.x % p.mblocks) * kPairRows;
  const unsigned n1 = p.d1n[s], n2 = p.d2n ? p.d2n[s] : 0u;
  if (n1 > p.D1 || n2 > p.D2) return;  // reported by pair_deferred_kernel, state untouched
  const unsigned nd = n1 + n2;
  if (!p.join && nd <= p.dbase) return;  // a forget-only pass with none of this pair's removes
  const unsigned ndp = nd > p.dbase ? (nd - p.dbase < 32u * kPairGroups ? nd - p.dbase : 32u * kPairGroups) : 0u;
  const unsigned ng = (ndp + 31) / 32;
  if (ng) {  // workgroup-uniform: most pairs carry no removes and skip the masks and the barrier
    for (unsigned i = threadIdx.x; i < ng * kPairRows; i += kBlock) {
      const unsigned g = i / kPairRows, r = i % kPairRows;
      const unsigned long long m = m0 + r;
      unsigned mask = 0;
      if (m < p.M) {
        for (unsigned d = p.dbase + g * 32; d < nd && d < p.dbase + g * 32 + 32; ++d) {
          const u64 *b = d < n1 ? p.d1b + (s * p.D1 + d) * p.Mw : p.d2b + (s * p.D2 + (d - n1)) * p.Mw;
          if ((b[m / 64] >> (m % 64)) & 1ull) mask |= 1u << (d - p.dbase - g * 32);
        }
      }
      hit[g][r] = mask;
    }
    __syncthreads();
  }
  const int lpr = 1 << p.lp_log;
  const int piece = threadIdx.x & (lpr - 1);
  const int rows_per_pass = kBlock >> p.lp_log;
  const unsigned long long W = (p.A + V - 1) / V;  // pieces per row
  const u64 *c1 = p.c1 + s * p.c1_s, *c2 = p.c2 + s * p.c2_s;
  for (unsigned long long pc = piece; pc < W; pc += lpr) {
    const unsigned long long a0 = pc * V;
    u64 k1[V], k2[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      k1[v] = a0 + v < p.A ? c1[a0 + v] : 0ull;
      k2[v] = a0 + v < p.A ? c2[a0 + v] : 0ull;
    }
    // UR rows per thread in flight: all their loads are issued before the first store (a store to
    // self's row could otherwise alias the next row's loads and serialize the round trips)
    for (int rb = threadIdx.x >> p.lp_log; rb < kPairRows; rb += rows_per_pass * kPairUR) {
      u64 x[kPairUR][V], y[kPairUR][V];
#pragma unroll
      for (int u = 0; u < kPairUR; ++u) {
        const int r = rb + u * rows_per_pass;
        const unsigned long long m = m0 + r;
        if (r >= kPairRows || m >= p.M) break;
        const u64 *pe1 = p.e1 + s * p.e1_s + m * p.e1_m + a0;
        const u64 *pe2 = p.join ? p.e2 + s * p.e2_s + m * p.e2_m + a0 : pe1;
        if constexpr (V == 2) {
          const u64x2 a = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(pe1));
          const u64x2 b = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(pe2));
          x[u][0] = a.x, x[u][1] = a.y, y[u][0] = b.x, y[u][1] = b.y;
        } else {
          x[u][0] = __builtin_nontemporal_load(pe1);
          y[u][0] = __builtin_nontemporal_load(pe2);
        }
      }
#pragma unroll
      for (int u = 0; u < kPairUR; ++u) {
        const int r = rb + u * rows_per_pass;
        const unsigned long long m = m0 + r;
        if (r >= kPairRows || m >= p.M) break;
        if (p.join) {
#pragma unroll
          for (int v = 0; v < V; ++v) x[u][v] = cell_join(x[u][v], y[u][v], k1[v], k2[v]);
        }
        for (unsigned g = 0; g < ng; ++g) {
          unsigned mask = hit[g][r];
          while (mask) {
            const unsigned d = p.dbase + g * 32 + __builtin_ctz(mask);
            mask &= mask - 1;
            const u64 *rm = d < n1 ? p.d1c + (s * p.D1 + d) * p.A : p.d2c + (s * p.D2 + (d - n1)) * p.A;
#pragma unroll
            for (int v = 0; v < V; ++v)
              if (a0 + v < p.A && x[u][v] <= rm[a0 + v]) x[u][v] = 0;  // VClock::forget, vclock.rs:95-105
          }
        }
        u64 *pe1 = p.e1 + s * p.e1_s + m * p.e1_m + a0;
        if constexpr (V == 2) {
          u64x2 o;
          o.x = x[u][0];
          o.y = x[u][1];
          __builtin_nontemporal_store(o, reinterpret_cast<u64x2 *>(pe1));
        } else {
          __builtin_nontemporal_store(x[u][0], pe1);
        }
      }
    }
  }
}

// ---- Map<K, MVReg> key merge --------------------------------------------------------------------
constexpr int kMapPairMaxV = 32;  // value slots per side (u32 slot masks of the generic kernel)

struct MapPairPlan {
  unsigned long long N, K, A, V1, V2, Kw;
  const u64 *c1;
  unsigned long long c1_s;
  const u64 *c2;
  unsigned long long c2_s;
  u64 *ec1, *vc1, *vv1;
  unsigned long long ec1_s, vc1_s, vv1_s;
  const u64 *ec2, *vc2, *vv2;
  unsigned long long ec2_s, vc2_s, vv2_s;
  const u64 *d1c, *d1k;
  const uint32_t *d1n;
  unsigned long long D1;
  const u64 *d2c, *d2k;
  const uint32_t *d2n;
  unsigned long long D2;
  uint32_t *status;  // bit 4 = a register needed more than V1 slots (set with atomicOr)
};

template <int APL>
struct PRow {
  u64 w[APL];
};
template <int APL>
__device__ __forceinline__ PRow<APL> prow(const u64 *p, int lane, unsigned long long A) {
  PRow<APL> r;
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = lane + j * kWave;
    r.w[j] = a < A ? p[a] : 0ull;
  }
  return r;
}
template <int APL>
__device__ __forceinline__ void pstore(u64 *p, const PRow<APL> &r, int lane, unsigned long long A) {
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = lane + j * kWave;
    if (a < A) p[a] = r.w[j];
  }
}
template <int APL>
__device__ __forceinline__ bool pnz(const PRow<APL> &r) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) b |= r.w[j] != 0;
  return pany(b);
}
template <int APL>
__device__ __forceinline__ bool ple(const PRow<APL> &x, const PRow<APL> &y) {  // x <= y everywhere
  bool b = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) b |= x.w[j] > y.w[j];
  return !pany(b);
}
template <int APL>
__device__ __forceinline__ bool peq(const PRow<APL> &x, const PRow<APL> &y) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) b |= x.w[j] != y.w[j];
  return !pany(b);
}
// partial_cmp == Less (vclock.rs:68-80): x <= y and x != y
template <int APL>
__device__ __forceinline__ bool plt(const PRow<APL> &x, const PRow<APL> &y) {
  return ple(x, y) && !peq(x, y);
}
template <int APL>
__device__ __forceinline__ PRow<APL> pforget(const PRow<APL> &x, const PRow<APL> &y) {  // keep x iff x > y
  PRow<APL> r;
#pragma unroll
  for (int j = 0; j < APL; ++j) r.w[j] = x.w[j] > y.w[j] ? x.w[j] : 0ull;
  return r;
}
template <int APL>
__device__ __forceinline__ PRow<APL> pmax(const PRow<APL> &x, const PRow<APL> &y) {
  PRow<APL> r;
#pragma unroll
  for (int j = 0; j < APL; ++j) r.w[j] = x.w[j] > y.w[j] ? x.w[j] : y.w[j];
  return r;
}
__device__ __forceinline__ u64 prl64(u64 x, int l) {
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)x, l);
  const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(x >> 32), l);
  return ((u64)hi << 32) | lo;
}

// One wave per (pair, key); APL clock words per lane (A <= 64 * APL).
template <int APL>
__global__ __launch_bounds__(kBlock) void map_pair_join_kernel(MapPairPlan p) {
  const int lane = threadIdx.x % kWave;
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;
  const unsigned long long nw = (unsigned long long)gridDim.x * (kBlock / kWave);
  const unsigned long long A = p.A;
  for (unsigned long long it = w0; it < p.N * p.K; it += nw) {
    const unsigned long long s = it / p.K, k = it % p.K;
    const unsigned n1 = p.d1n[s], n2 = p.d2n ? p.d2n[s] : 0u;
    if (n1 > p.D1 || n2 > p.D2) continue;  // reported by pair_deferred_kernel
    u64 *ec1 = p.ec1 + s * p.ec1_s + k * A;
    u64 *vc1 = p.vc1 + s * p.vc1_s + k * p.V1 * A;
    u64 *vv1 = p.vv1 + s * p.vv1_s + k * p.V1;
    const u64 *ec2 = p.ec2 + s * p.ec2_s + k * A;
    const u64 *vc2 = p.vc2 + s * p.vc2_s + k * p.V2 * A;
    const u64 *vv2 = p.vv2 + s * p.vv2_s + k * p.V2;
    const PRow<APL> e1 = prow<APL>(ec1, lane, A), e2 = prow<APL>(ec2, lane, A);
    const bool p1 = pnz(e1), p2 = pnz(e2);
    if (!p1 && !p2) continue;  // no entry on either side: nothing to merge
    const PRow<APL> c1 = prow<APL>(p.c1 + s * p.c1_s, lane, A), c2 = prow<APL>(p.c2 + s * p.c2_s, lane, A);
    // occupied value slots (Vec order = slot order, empty slot <=> zero clock)
    unsigned m1 = 0, m2 = 0;
    for (unsigned q = 0; q < p.V1; ++q)
      if (pnz(prow<APL>(vc1 + q * A, lane, A))) m1 |= 1u << q;
    for (unsigned q = 0; q < p.V2; ++q)
      if (pnz(prow<APL>(vc2 + q * A, lane, A))) m2 |= 1u << q;
    bool present = true;
    PRow<APL> e, X;  // resulting entry clock, forget clock of the values
    unsigned keep1 = 0, add2 = 0;
    if (p1 && !p2) {  // :146-161
      if (ple(e1, c2)) {
        present = false;
      } else {
        e = pforget(e1, c2);
        X = pforget(c2, e);  // removed_information = other.clock.forget(entry.clock)
        keep1 = m1;
      }
    } else if (!p1 && p2) {  // :193-208
      if (ple(e2, c1)) {
        present = false;
      } else {
        e = pforget(e2, c1);
        X = pforget(c1, e);  // information_we_deleted
        add2 = m2;
      }
    } else {  // :170-192
      PRow<APL> common;
#pragma unroll
      for (int j = 0; j < APL; ++j) {
        const u64 a = e1.w[j], b = e2.w[j];
        const u64 t0 = a == b ? a : 0ull, t1 = b > c1.w[j] ? b : 0ull, t2 = a > c2.w[j] ? a : 0ull;
        const u64 t = t0 > t1 ? t0 : t1;
        common.w[j] = t > t2 ? t : t2;
      }
      if (!pnz(common)) {
        present = false;
      } else {
        // MVReg::merge (mvreg.rs:112-128): own values not strictly below one of other's, then
        // other's not strictly below a kept own value and not equal to one
        for (unsigned q = 0; q < p.V1; ++q) {
          if (!((m1 >> q) & 1u)) continue;
          const PRow<APL> x = prow<APL>(vc1 + q * A, lane, A);
          bool dom = false;
          for (unsigned r = 0; r < p.V2 && !dom; ++r)
            if ((m2 >> r) & 1u) dom = plt(x, prow<APL>(vc2 + r * A, lane, A));
          if (!dom) keep1 |= 1u << q;
        }
        for (unsigned r = 0; r < p.V2; ++r) {
          if (!((m2 >> r) & 1u)) continue;
          const PRow<APL> y = prow<APL>(vc2 + r * A, lane, A);
          bool drop = false;
          for (unsigned q = 0; q < p.V1 && !drop; ++q)
            if ((keep1 >> q) & 1u) {
              const PRow<APL> x = prow<APL>(vc1 + q * A, lane, A);
              drop = plt(y, x) || peq(y, x);
            }
          if (!drop) add2 |= 1u << r;
        }
        X = pforget(pmax(e1, e2), common);  // information_that_was_deleted
        e = common;
      }
    }
    // every deferred remove of either side naming k (apply_keyset_rm :318-333, composed by max)
    PRow<APL> Rk;
#pragma unroll
    for (int j = 0; j < APL; ++j) Rk.w[j] = 0;
    bool hasR = false;
    if (present) {
      for (unsigned d = 0; d < n1 + n2; ++d) {
        const u64 *kb = d < n1 ? p.d1k + (s * p.D1 + d) * p.Kw : p.d2k + (s * p.D2 + (d - n1)) * p.Kw;
        if (!((kb[k / 64] >> (k % 64)) & 1ull)) continue;
        const u64 *rc = d < n1 ? p.d1c + (s * p.D1 + d) * A : p.d2c + (s * p.D2 + (d - n1)) * A;
        Rk = pmax(Rk, prow<APL>(rc, lane, A));
        hasR = true;
      }
      if (hasR) {
        e = pforget(e, Rk);
        if (!pnz(e)) present = false;
      }
    }
    // the values' u64 payloads, read before any slot is written (lane q holds slot q)
    const u64 v1l = (unsigned long long)lane < p.V1 ? vv1[lane] : 0ull;
    const u64 v2l = (unsigned long long)lane < p.V2 ? vv2[lane] : 0ull;
    unsigned w = 0;
    if (present) {
      pstore(ec1, e, lane, A);
      // own kept values first (slot order), then other's added ones: the Vec order of :113-127.
      // Writing slot w never clobbers an unread own slot (w <= the slot being read).
      for (unsigned q = 0; q < p.V1; ++q) {
        if (!((keep1 >> q) & 1u)) continue;
        PRow<APL> x = pforget(prow<APL>(vc1 + q * A, lane, A), X);  // MVReg::forget mvreg.rs:88-104
        if (hasR) x = pforget(x, Rk);
        if (!pnz(x)) continue;
        const u64 val = prl64(v1l, (int)q);
        if (w < p.V1) {
          pstore(vc1 + (unsigned long long)w * A, x, lane, A);
          if (lane == 0) vv1[w] = val;
        }
        ++w;
      }
      for (unsigned r = 0; r < p.V2; ++r) {
        if (!((add2 >> r) & 1u)) continue;
        PRow<APL> y = pforget(prow<APL>(vc2 + r * A, lane, A), X);
        if (hasR) y = pforget(y, Rk);
        if (!pnz(y)) continue;
        const u64 val = prl64(v2l, (int)r);
        if (w < p.V1) {
          pstore(vc1 + (unsigned long long)w * A, y, lane, A);
          if (lane == 0) vv1[w] = val;
        }
        ++w;
      }
      if (w > p.V1 && lane == 0) atomicOr(p.status + s, 16u);
    } else {
      PRow<APL> z;
#pragma unroll
      for (int j = 0; j < APL; ++j) z.w[j] = 0;
      pstore(ec1, z, lane, A);
    }
    for (unsigned q = w; q < p.V1; ++q) {  // clear the slots past the last written value
      PRow<APL> z;
#pragma unroll
      for (int j = 0; j < APL; ++j) z.w[j] = 0;
      pstore(vc1 + (unsigned long long)q * A, z, lane, A);
      if (lane == 0) vv1[q] = 0;
    }
  }
}

// Register-resident form of map_pair_join_kernel for V1, V2 <= VM: every row of the key (both
// entry clocks, both map clocks, all value clocks, the value payloads and the key's bit of every
// deferred remove) is loaded in ONE batch of independent loads before any vote, so a key costs
// one memory round trip (two when a remove names it) instead of a chain of dependent ones; the
// MVReg compares then run on registers.  Same statement-by-statement semantics as the generic
// kernel above (map.rs:142-210, mvreg.rs:112-128, apply_keyset_rm :318-333).
template <int APL, int VM>
__global__ __launch_bounds__(kBlock) void map_pair_join_reg_kernel(MapPairPlan p) {
  const int lane = threadIdx.x % kWave;
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;
  const unsigned long long nw = (unsigned long long)gridDim.x * (kBlock / kWave);
  const unsigned long long A = p.A;
  const unsigned V1 = (unsigned)p.V1, V2 = (unsigned)p.V2;
  for (unsigned long long it = w0; it < p.N * p.K; it += nw) {
    const unsigned long long s = it / p.K, k = it % p.K;
    const unsigned n1 = p.d1n[s], n2 = p.d2n ? p.d2n[s] : 0u;
    if (n1 > p.D1 || n2 > p.D2) continue;  // reported by pair_deferred_kernel
    u64 *ec1 = p.ec1 + s * p.ec1_s + k * A;
    u64 *vc1 = p.vc1 + s * p.vc1_s + k * p.V1 * A;
    u64 *vv1 = p.vv1 + s * p.vv1_s + k * p.V1;
    const u64 *ec2 = p.ec2 + s * p.ec2_s + k * A;
    const u64 *vc2 = p.vc2 + s * p.vc2_s + k * p.V2 * A;
    const u64 *vv2 = p.vv2 + s * p.vv2_s + k * p.V2;
    // ---- one batch of loads
    const PRow<APL> e1 = prow<APL>(ec1, lane, A), e2 = prow<APL>(ec2, lane, A);
    const PRow<APL> c1 = prow<APL>(p.c1 + s * p.c1_s, lane, A), c2 = prow<APL>(p.c2 + s * p.c2_s, lane, A);
    PRow<APL> x[VM], y[VM];
#pragma unroll
    for (int q = 0; q < VM; ++q) {
#pragma unroll
      for (int j = 0; j < APL; ++j) x[q].w[j] = y[q].w[j] = 0;
      if ((unsigned)q < V1) x[q] = prow<APL>(vc1 + (unsigned long long)q * A, lane, A);
      if ((unsigned)q < V2) y[q] = prow<APL>(vc2 + (unsigned long long)q * A, lane, A);
    }
    const u64 v1l = (unsigned)lane < V1 ? vv1[lane] : 0ull;
    const u64 v2l = (unsigned)lane < V2 ? vv2[lane] : 0ull;
    const unsigned nd = n1 + n2;
    bool hitl = false;  // lane d: remove d (self's, then other's) names k
    if ((unsigned)lane < nd) {
      const u64 *kb = (unsigned)lane < n1 ? p.d1k + (s * p.D1 + lane) * p.Kw : p.d2k + (s * p.D2 + (lane - n1)) * p.Kw;
      hitl = (kb[k / 64] >> (k % 64)) & 1ull;
    }
    // ---- compute on registers
    const bool p1 = pnz(e1), p2 = pnz(e2);
    if (!p1 && !p2) continue;  // no entry on either side: nothing to merge
    unsigned m1 = 0, m2 = 0;
#pragma unroll
    for (int q = 0; q < VM; ++q) {
      if (pnz(x[q])) m1 |= 1u << q;  // rows past V1 / V2 are zero
      if (pnz(y[q])) m2 |= 1u << q;
    }
    bool present = true;
    PRow<APL> e, X;
    unsigned keep1 = 0, add2 = 0;
    if (p1 && !p2) {  // :146-161
      if (ple(e1, c2)) {
        present = false;
      } else {
        e = pforget(e1, c2);
        X = pforget(c2, e);
        keep1 = m1;
      }
    } else if (!p1 && p2) {  // :193-208
      if (ple(e2, c1)) {
        present = false;
      } else {
        e = pforget(e2, c1);
        X = pforget(c1, e);
        add2 = m2;
      }
    } else {  // :170-192
      PRow<APL> common;
#pragma unroll
      for (int j = 0; j < APL; ++j) {
        const u64 a = e1.w[j], b = e2.w[j];
        const u64 t0 = a == b ? a : 0ull, t1 = b > c1.w[j] ? b : 0ull, t2 = a > c2.w[j] ? a : 0ull;
        const u64 t = t0 > t1 ? t0 : t1;
        common.w[j] = t > t2 ? t : t2;
      }
      if (!pnz(common)) {
        present = false;
      } else {
#pragma unroll
        for (int q = 0; q < VM; ++q) {
          if (!((m1 >> q) & 1u)) continue;
          bool dom = false;
#pragma unroll
          for (int r = 0; r < VM; ++r)
            if (((m2 >> r) & 1u) && !dom) dom = plt(x[q], y[r]);
          if (!dom) keep1 |= 1u << q;
        }
#pragma unroll
        for (int r = 0; r < VM; ++r) {
          if (!((m2 >> r) & 1u)) continue;
          bool drop = false;
#pragma unroll
          for (int q = 0; q < VM; ++q)
            if (((keep1 >> q) & 1u) && !drop) drop = plt(y[r], x[q]) || peq(y[r], x[q]);
          if (!drop) add2 |= 1u << r;
        }
        X = pforget(pmax(e1, e2), common);
        e = common;
      }
    }
    PRow<APL> Rk;
#pragma unroll
    for (int j = 0; j < APL; ++j) Rk.w[j] = 0;
    bool hasR = false;
    if (present) {
      u64 hits = __ballot(hitl);
      for (unsigned base = 64; base < nd; base += 64) {  // more than 64 removes on the pair
        bool h = false;
        const unsigned d = base + lane;
        if (d < nd) {
          const u64 *kb = d < n1 ? p.d1k + (s * p.D1 + d) * p.Kw : p.d2k + (s * p.D2 + (d - n1)) * p.Kw;
          h = (kb[k / 64] >> (k % 64)) & 1ull;
        }
        const u64 hb = __ballot(h);
        for (u64 m = hb; m; m &= m - 1) {
          const unsigned dd = base + (unsigned)__builtin_ctzll(m);
          const u64 *rc = dd < n1 ? p.d1c + (s * p.D1 + dd) * A : p.d2c + (s * p.D2 + (dd - n1)) * A;
          Rk = pmax(Rk, prow<APL>(rc, lane, A));
          hasR = true;
        }
      }
      for (; hits; hits &= hits - 1) {
        const unsigned d = (unsigned)__builtin_ctzll(hits);
        const u64 *rc = d < n1 ? p.d1c + (s * p.D1 + d) * A : p.d2c + (s * p.D2 + (d - n1)) * A;
        Rk = pmax(Rk, prow<APL>(rc, lane, A));
        hasR = true;
      }
      if (hasR) {
        e = pforget(e, Rk);
        if (!pnz(e)) present = false;
      }
    }
    unsigned w = 0;
    if (present) {
      pstore(ec1, e, lane, A);
#pragma unroll
      for (int q = 0; q < VM; ++q) {
        if (!((keep1 >> q) & 1u)) continue;
        PRow<APL> z = pforget(x[q], X);  // MVReg::forget mvreg.rs:88-104
        if (hasR) z = pforget(z, Rk);
        if (!pnz(z)) continue;
        const u64 val = prl64(v1l, q);
        if (w < V1) {
          pstore(vc1 + (unsigned long long)w * A, z, lane, A);
          if (lane == 0) vv1[w] = val;
        }
        ++w;
      }
#pragma unroll
      for (int r = 0; r < VM; ++r) {
        if (!((add2 >> r) & 1u)) continue;
        PRow<APL> z = pforget(y[r], X);
        if (hasR) z = pforget(z, Rk);
        if (!pnz(z)) continue;
        const u64 val = prl64(v2l, r);
        if (w < V1) {
          pstore(vc1 + (unsigned long long)w * A, z, lane, A);
          if (lane == 0) vv1[w] = val;
        }
        ++w;
      }
      if (w > V1 && lane == 0) atomicOr(p.status + s, 16u);
    } else {
      PRow<APL> z;
#pragma unroll
      for (int j = 0; j < APL; ++j) z.w[j] = 0;
      pstore(ec1, z, lane, A);
    }
    for (unsigned q = w; q < V1; ++q) {
      PRow<APL> z;
#pragma unroll
      for (int j = 0; j < APL; ++j) z.w[j] = 0;
      pstore(vc1 + (unsigned long long)q * A, z, lane, A);
      if (lane == 0) vv1[q] = 0;
    }
  }
}

// Sub-wave form for A <= SEG < 64 (one actor per lane): a wave merges 64 / SEG keys at once, one
// SEG-lane segment per key, so a narrow key (A = 32 at config 4) does not leave half the wave
// idle and twice the rows are in flight per wave.  Votes are per segment (the segment's bits of
// the ballot); the segments of a wave may branch differently (divergent, not wrong: every
// segment's lanes only read and write their own key).  Otherwise map_pair_join_reg_kernel.
template <int SEG>
struct Seg {
  int lane, sl, base;
  u64 mask;
  __device__ Seg(int l) : lane(l), sl(l & (SEG - 1)), base(l & ~(SEG - 1)),
                          mask(SEG == 64 ? ~0ull : (((1ull << SEG) - 1) << (l & ~(SEG - 1)))) {}
  __device__ bool any(bool x) const { return (__ballot(x) & mask) != 0; }
  __device__ u64 bits(bool x) const { return (__ballot(x) & mask) >> base; }
};

// PF (round 4): the loads of the wave's NEXT keys (grid-stride successor) are issued before the
// current keys are merged, so each wave keeps two keys' rows in flight instead of one (a wave's
// iteration is one load round trip, then compute and stores: latency-bound at one batch).
template <int SEG, int VM>
struct SegRows {
  unsigned long long s, k;
  bool ok;  // a key of this segment, with valid deferred counts
  unsigned n1, n2;
  u64 e1, e2, c1, c2, x[VM], y[VM], v1l, v2l;
  bool hitl;  // segment lane d: remove d (self's, then other's) names k
};

template <int SEG, int VM, bool PF, bool NT>
__global__ __launch_bounds__(kBlock) void map_pair_join_seg_kernel(MapPairPlan p) {
  constexpr int KPW = kWave / SEG;  // keys per wave
  const Seg<SEG> sg(threadIdx.x % kWave);
  const int sl = sg.sl;
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;
  const unsigned long long nw = (unsigned long long)gridDim.x * (kBlock / kWave);
  const unsigned long long A = p.A, NK = p.N * p.K;
  const unsigned V1 = (unsigned)p.V1, V2 = (unsigned)p.V2;
  const bool act = (unsigned long long)sl < A;
  // ---- one batch of loads for the keys at it0 (this segment's: it0 + segment index)
  auto load = [&](unsigned long long it0, SegRows<SEG, VM> &L) {
    const unsigned long long it = it0 + (unsigned long long)(sg.base / SEG);
    L.ok = false;
    L.hitl = false;
    L.e1 = L.e2 = L.c1 = L.c2 = L.v1l = L.v2l = 0;
#pragma unroll
    for (int q = 0; q < VM; ++q) L.x[q] = L.y[q] = 0;
    if (it >= NK) return;  // a segment past the end (last wave only)
    const unsigned long long s = it / p.K, k = it % p.K;
    L.s = s;
    L.k = k;
    L.n1 = p.d1n[s];
    L.n2 = p.d2n ? p.d2n[s] : 0u;
    const u64 *ec2 = p.ec2 + s * p.ec2_s + k * A;
    const u64 *vc2 = p.vc2 + s * p.vc2_s + k * p.V2 * A;
    const u64 *vv2 = p.vv2 + s * p.vv2_s + k * p.V2;
    const u64 *ec1 = p.ec1 + s * p.ec1_s + k * A;
    const u64 *vc1 = p.vc1 + s * p.vc1_s + k * p.V1 * A;
    const u64 *vv1 = p.vv1 + s * p.vv1_s + k * p.V1;
    // NT: the key rows are streamed once (non-temporal); the map clocks stay cached (every key of
    // the pair reads them)
    auto ld = [](const u64 *x) -> u64 { return NT ? __builtin_nontemporal_load(x) : *x; };
    if (act) {
      L.e1 = ld(ec1 + sl);
      L.e2 = ld(ec2 + sl);
      L.c1 = p.c1[s * p.c1_s + sl];
      L.c2 = p.c2[s * p.c2_s + sl];
#pragma unroll
      for (int q = 0; q < VM; ++q) {
        if ((unsigned)q < V1) L.x[q] = ld(vc1 + (unsigned long long)q * A + sl);
        if ((unsigned)q < V2) L.y[q] = ld(vc2 + (unsigned long long)q * A + sl);
      }
    }
    L.v1l = (unsigned)sl < V1 ? vv1[sl] : 0ull;
    L.v2l = (unsigned)sl < V2 ? vv2[sl] : 0ull;
    L.ok = !(L.n1 > p.D1 || L.n2 > p.D2);  // (else reported by pair_deferred_kernel)
    const unsigned nd = L.ok ? L.n1 + L.n2 : 0u;
    if ((unsigned)sl < nd) {
      const u64 *kb =
          (unsigned)sl < L.n1 ? p.d1k + (s * p.D1 + sl) * p.Kw : p.d2k + (s * p.D2 + (sl - L.n1)) * p.Kw;
      L.hitl = (kb[k / 64] >> (k % 64)) & 1ull;
    }
  };
  // ---- merge the keys whose rows are in L
  auto merge = [&](const SegRows<SEG, VM> &L) {
    // each segment's value payloads to all its lanes (a segment's lanes are all here or all not)
    u64 val1[VM], val2[VM];
#pragma unroll
    for (int q = 0; q < VM; ++q) {
      val1[q] = __shfl(L.v1l, sg.base + q);
      val2[q] = __shfl(L.v2l, sg.base + q);
    }
    if (!L.ok) return;
    const unsigned long long s = L.s, k = L.k;
    const unsigned n1 = L.n1, n2 = L.n2;
    const u64 e1 = L.e1, e2 = L.e2, c1 = L.c1, c2 = L.c2;
    u64 *ec1 = p.ec1 + s * p.ec1_s + k * A;
    u64 *vc1 = p.vc1 + s * p.vc1_s + k * p.V1 * A;
    u64 *vv1 = p.vv1 + s * p.vv1_s + k * p.V1;
    const unsigned nd = n1 + n2;
    auto st = [](u64 *x, u64 v) {
      if (NT) __builtin_nontemporal_store(v, x);
      else *x = v;
    };
    const bool p1 = sg.any(e1 != 0), p2 = sg.any(e2 != 0);
    if (!p1 && !p2) return;
    unsigned m1 = 0, m2 = 0;
#pragma unroll
    for (int q = 0; q < VM; ++q) {
      if (sg.any(L.x[q] != 0)) m1 |= 1u << q;
      if (sg.any(L.y[q] != 0)) m2 |= 1u << q;
    }
    auto le = [&](u64 a, u64 b) { return !sg.any(a > b); };           // a <= b everywhere
    auto lt = [&](u64 a, u64 b) { return le(a, b) && sg.any(a != b); };  // partial_cmp == Less
    bool present = true;
    u64 e = 0, X = 0;
    unsigned keep1 = 0, add2 = 0;
    if (p1 && !p2) {  // :146-161
      if (le(e1, c2)) {
        present = false;
      } else {
        e = e1 > c2 ? e1 : 0;
        X = c2 > e ? c2 : 0;
        keep1 = m1;
      }
    } else if (!p1 && p2) {  // :193-208
      if (le(e2, c1)) {
        present = false;
      } else {
        e = e2 > c1 ? e2 : 0;
        X = c1 > e ? c1 : 0;
        add2 = m2;
      }
    } else {  // :170-192
      const u64 t0 = e1 == e2 ? e1 : 0ull, t1 = e2 > c1 ? e2 : 0ull, t2 = e1 > c2 ? e1 : 0ull;
      const u64 t = t0 > t1 ? t0 : t1;
      const u64 common = t > t2 ? t : t2;
      if (!sg.any(common != 0)) {
        present = false;
      } else {
#pragma unroll
        for (int q = 0; q < VM; ++q) {
          if (!((m1 >> q) & 1u)) continue;
          bool dom = false;
#pragma unroll
          for (int r = 0; r < VM; ++r)
            if (((m2 >> r) & 1u) && !dom) dom = lt(L.x[q], L.y[r]);
          if (!dom) keep1 |= 1u << q;
        }
#pragma unroll
        for (int r = 0; r < VM; ++r) {
          if (!((m2 >> r) & 1u)) continue;
          bool drop = false;
#pragma unroll
          for (int q = 0; q < VM; ++q)
            if (((keep1 >> q) & 1u) && !drop) drop = le(L.y[r], L.x[q]);  // y < x or y == x
          if (!drop) add2 |= 1u << r;
        }
        const u64 mx = e1 > e2 ? e1 : e2;
        X = mx > common ? mx : 0;
        e = common;
      }
    }
    u64 Rk = 0;
    bool hasR = false;
    if (present) {
      for (unsigned b0 = 0; b0 < nd; b0 += SEG) {
        bool h = L.hitl;
        if (b0) {  // more than SEG removes on the pair
          h = false;
          const unsigned d = b0 + sl;
          if (d < nd) {
            const u64 *kb = d < n1 ? p.d1k + (s * p.D1 + d) * p.Kw : p.d2k + (s * p.D2 + (d - n1)) * p.Kw;
            h = (kb[k / 64] >> (k % 64)) & 1ull;
          }
        }
        for (u64 m = sg.bits(h); m; m &= m - 1) {
          const unsigned d = b0 + (unsigned)__builtin_ctzll(m);
          const u64 *rc = d < n1 ? p.d1c + (s * p.D1 + d) * A : p.d2c + (s * p.D2 + (d - n1)) * A;
          const u64 r = act ? rc[sl] : 0ull;
          Rk = Rk > r ? Rk : r;
          hasR = true;
        }
      }
      if (hasR) {
        e = e > Rk ? e : 0;
        if (!sg.any(e != 0)) present = false;
      }
    }
    unsigned w = 0;
    if (present) {
      if (act) st(ec1 + sl, e);
#pragma unroll
      for (int q = 0; q < VM; ++q) {
        if (!((keep1 >> q) & 1u)) continue;
        u64 z = L.x[q] > X ? L.x[q] : 0;  // MVReg::forget mvreg.rs:88-104
        if (hasR) z = z > Rk ? z : 0;
        const u64 val = val1[q];
        if (!sg.any(z != 0)) continue;
        if (w < V1) {
          if (act) st(vc1 + (unsigned long long)w * A + sl, z);
          if (sl == 0) vv1[w] = val;
        }
        ++w;
      }
#pragma unroll
      for (int r = 0; r < VM; ++r) {
        if (!((add2 >> r) & 1u)) continue;
        u64 z = L.y[r] > X ? L.y[r] : 0;
        if (hasR) z = z > Rk ? z : 0;
        const u64 val = val2[r];
        if (!sg.any(z != 0)) continue;
        if (w < V1) {
          if (act) st(vc1 + (unsigned long long)w * A + sl, z);
          if (sl == 0) vv1[w] = val;
        }
        ++w;
      }
      if (w > V1 && sl == 0) atomicOr(p.status + s, 16u);
    } else if (act) {
      st(ec1 + sl, 0);
    }
    for (unsigned q = w; q < V1; ++q) {
      if (act) st(vc1 + (unsigned long long)q * A + sl, 0);
      if (sl == 0) vv1[q] = 0;
    }
  };
  const unsigned long long step = nw * KPW;
  unsigned long long it0 = w0 * KPW;
  if (it0 >= NK) return;
  SegRows<SEG, VM> cur;
  load(it0, cur);
  for (; it0 < NK; it0 += step) {
    if constexpr (PF) {
      SegRows<SEG, VM> nxt;
      load(it0 + step, nxt);  // (nothing when past the end)
      merge(cur);
      cur = nxt;
    } else {
      merge(cur);
      load(it0 + step, cur);
    }
  }
}

static unsigned pair_grid(crdt_ctx *ctx, unsigned long long waves, int per_cu) {
  const unsigned long long want = (waves + (kBlock / kWave) - 1) / (kBlock / kWave);
  const unsigned long long cap = (unsigned long long)ctx->cu_count * per_cu;
  return (unsigned)(want < cap ? (want ? want : 1) : cap);
}

static bool al16p(const void *p) { return ((uintptr_t)p & 15) == 0; }

static int launch_pair_deferred(crdt_ctx *ctx, PairDefPlan q) {
  hipLaunchKernelGGL(pair_deferred_kernel, dim3(pair_grid(ctx, q.N, 8)), dim3(kBlock), 0, ctx->stream, q);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_orswot_merge_batch(crdt_ctx *ctx, const crdt_orswot_states *self, const crdt_orswot_states *other,
                                       uint32_t *status) {
  if (ctx && ctx->mem_kind == CRDT_MEM_HOST) return crdt::orswot_merge_batch_host(ctx, self, other, status);
  CRDT_CHECK_CTX(ctx);
  if (!self || !other || !status) return fail(ctx, CRDT_EINVAL, "orswot_merge_batch: NULL argument");
  const crdt_orswot_states &a = *self, &b = *other;
  if (a.N != b.N || a.M != b.M || a.A != b.A)
    return fail(ctx, CRDT_EINVAL, "orswot_merge_batch: self and other differ in N, M or A");
  const size_t N = a.N, M = a.M, A = a.A;
  if (N == 0) return CRDT_OK;
  if (A == 0) return fail(ctx, CRDT_EINVAL, "orswot_merge_batch: A = 0");
  if (!a.clock || !b.clock || !a.def_count || (M && (!a.entries || !b.entries)))
    return fail(ctx, CRDT_EINVAL, "orswot_merge_batch: NULL buffer");
  if ((a.Dcap && (!a.def_clock || !a.def_members)) || (b.Dcap && (!b.def_clock || !b.def_members || !b.def_count)))
    return fail(ctx, CRDT_EINVAL, "orswot_merge_batch: deferred capacity without deferred buffers");
  if (a.clock_stride < A || b.clock_stride < A ||
      (M && (a.entry_mstride < A || b.entry_mstride < A || a.entry_sstride < M * a.entry_mstride ||
             b.entry_sstride < M * b.entry_mstride)))
    return fail(ctx, CRDT_EINVAL, "orswot_merge_batch: strides smaller than the rows they hold");
  if (a.Dcap + b.Dcap > 0xffffffffull) return fail(ctx, CRDT_EUNSUPPORTED, "orswot_merge_batch: Dcap too large");
  const size_t Mw = (M + 63) / 64;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  if (M) {
    const bool v2 = A % 2 == 0 && a.entry_mstride % 2 == 0 && b.entry_mstride % 2 == 0 && a.entry_sstride % 2 == 0 &&
                    b.entry_sstride % 2 == 0 && al16p(a.entries) && al16p(b.entries);
    const unsigned long long W = v2 ? A / 2 : A;
    int lp = 0;
    while (lp < 6 && (1ull << lp) < W) ++lp;
    const int rows = ctx->tune.pair_rows;  // member rows per workgroup (64, 128, 256)
    const unsigned long long mblocks = (M + rows - 1) / rows;
    if (N * mblocks > 0x7FFFFFFFull) return fail(ctx, CRDT_EUNSUPPORTED, "orswot_merge_batch: grid too large");
    OrswotPairPlan p{(u64 *)a.entries, a.entry_mstride, a.entry_sstride, (const u64 *)b.entries, b.entry_mstride,
                     b.entry_sstride, (const u64 *)a.clock, a.clock_stride, (const u64 *)b.clock, b.clock_stride,
                     (const u64 *)a.def_clock, (const u64 *)a.def_members, a.def_count, a.Dcap,
                     (const u64 *)b.def_clock, (const u64 *)b.def_members, b.Dcap ? b.def_count : nullptr, b.Dcap,
                     N, M, A, Mw, mblocks, lp, 0u, 1};
    timing_begin(ctx, "orswot_pair_join");
    const dim3 grid((unsigned)(N * mblocks));
    // pass 0 joins and applies removes [0, 512); pass k > 0 only forgets by removes [512 k, 512 k + 512)
    for (size_t db = 0; db == 0 || db < a.Dcap + b.Dcap; db += 32 * kPairGroups) {
    p.dbase = (unsigned)db;
    p.join = db == 0 ? 1 : 0;
    // pocc > 0: at most pocc workgroups per CU (dynamic LDS padding), fewer HBM requests in flight
    const size_t pad = ctx->tune.pair_occ > 0 ? (size_t)(160 * 1024 / ctx->tune.pair_occ) - kPairGroups * rows * 4 - 256 : 0;
#define CRDT_PAIR_JOIN(VV, RR) hipLaunchKernelGGL((orswot_pair_join_kernel<VV, RR>), grid, dim3(kBlock), pad, ctx->stream, p)
    if (v2 && rows == 128 && ctx->tune.pair_ur == 2)
      hipLaunchKernelGGL((orswot_pair_join_kernel<2, 128, 2>), grid, dim3(kBlock), pad, ctx->stream, p);
    else if (v2 && rows == 128 && ctx->tune.pair_ur == 4)
      hipLaunchKernelGGL((orswot_pair_join_kernel<2, 128, 4>), grid, dim3(kBlock), pad, ctx->stream, p);
    else if (v2) {
      if (rows == 64) CRDT_PAIR_JOIN(2, 64);
      else if (rows == 256) CRDT_PAIR_JOIN(2, 256);
      else CRDT_PAIR_JOIN(2, 128);
    } else {
      if (rows == 64) CRDT_PAIR_JOIN(1, 64);
      else if (rows == 256) CRDT_PAIR_JOIN(1, 256);
      else CRDT_PAIR_JOIN(1, 128);
    }
    }
#undef CRDT_PAIR_JOIN
    timing_end(ctx);
    CRDT_HIP(ctx, hipGetLastError());
  }
  return launch_pair_deferred(ctx, PairDefPlan{N, A, Mw, (u64 *)a.clock, a.clock_stride, (const u64 *)b.clock,
                                               b.clock_stride, (u64 *)a.def_clock, (u64 *)a.def_members, a.def_count,
                                               a.Dcap, (const u64 *)b.def_clock, (const u64 *)b.def_members,
                                               b.Dcap ? b.def_count : nullptr, b.Dcap, status, 0u});
}

extern "C" int crdt_map_merge_batch(crdt_ctx *ctx, const crdt_map_states *self, const crdt_map_deferred *self_def,
                                    const crdt_map_states *other, const crdt_map_deferred *other_def,
                                    uint32_t *status) {
  if (ctx && ctx->mem_kind == CRDT_MEM_HOST)
    return crdt::map_merge_batch_host(ctx, self, self_def, other, other_def, status);
  CRDT_CHECK_CTX(ctx);
  if (!self || !other || !self_def || !other_def || !status)
    return fail(ctx, CRDT_EINVAL, "map_merge_batch: NULL argument");
  const crdt_map_states &a = *self, &b = *other;
  if (a.N != b.N || a.K != b.K || a.A != b.A)
    return fail(ctx, CRDT_EINVAL, "map_merge_batch: self and other differ in N, K or A");
  const size_t N = a.N, K = a.K, A = a.A;
  if (N == 0) return CRDT_OK;
  if (A == 0 || a.V == 0 || b.V == 0) return fail(ctx, CRDT_EINVAL, "map_merge_batch: need A, V >= 1 on both sides");
  if (A > 16 * (size_t)kWave || a.V > (size_t)kMapPairMaxV || b.V > (size_t)kMapPairMaxV)
    return fail(ctx, CRDT_EUNSUPPORTED, "map_merge_batch: need A <= %d and V <= %d on both sides", 16 * kWave,
                kMapPairMaxV);
  if (!a.clock || !b.clock || !self_def->count || (K && (!a.ec || !a.vclk || !a.vval || !b.ec || !b.vclk || !b.vval)))
    return fail(ctx, CRDT_EINVAL, "map_merge_batch: NULL buffer");
  if ((self_def->Dcap && (!self_def->clock || !self_def->keys)) ||
      (other_def->Dcap && (!other_def->clock || !other_def->keys || !other_def->count)))
    return fail(ctx, CRDT_EINVAL, "map_merge_batch: deferred capacity without deferred buffers");
  if (a.clock_stride < A || b.clock_stride < A || a.ec_stride < K * A || b.ec_stride < K * A ||
      a.vclk_stride < K * a.V * A || b.vclk_stride < K * b.V * A || a.vval_stride < K * a.V || b.vval_stride < K * b.V)
    return fail(ctx, CRDT_EINVAL, "map_merge_batch: strides smaller than the rows they hold");
  const size_t Kw = (K + 63) / 64;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  // status is written whole by the deferred pass; the key pass only ORs bit 4 into it first
  if (int rc = device_fill(ctx, status, N * sizeof(uint32_t), 0)) return rc;
  if (K) {
    MapPairPlan p{N, K, A, a.V, b.V, Kw, (const u64 *)a.clock, a.clock_stride, (const u64 *)b.clock, b.clock_stride,
                  (u64 *)a.ec, (u64 *)a.vclk, (u64 *)a.vval, a.ec_stride, a.vclk_stride, a.vval_stride,
                  (const u64 *)b.ec, (const u64 *)b.vclk, (const u64 *)b.vval, b.ec_stride, b.vclk_stride,
                  b.vval_stride, (const u64 *)self_def->clock, (const u64 *)self_def->keys, self_def->count,
                  self_def->Dcap, (const u64 *)other_def->clock, (const u64 *)other_def->keys,
                  other_def->Dcap ? other_def->count : nullptr, other_def->Dcap, status};
    const unsigned grid = pair_grid(ctx, (unsigned long long)N * K, ctx->tune.map_pair_bpc);
    timing_begin(ctx, "map_pair_join");
    const bool pf = ctx->tune.map_pair_pf, nt = ctx->tune.map_pair_nt;
    if (ctx->tune.map_pair_reg && a.V <= 4 && b.V <= 4 && A <= 4 * (size_t)kWave) {  // register-resident rows
      if (A <= 16 && ctx->tune.map_pair_reg == 1)
        hipLaunchKernelGGL((pf ? (nt ? map_pair_join_seg_kernel<16, 4, true, true> : map_pair_join_seg_kernel<16, 4, true, false>)
                              : (nt ? map_pair_join_seg_kernel<16, 4, false, true> : map_pair_join_seg_kernel<16, 4, false, false>)),
                           dim3(grid), dim3(kBlock), 0, ctx->stream, p);
      else if (A <= 32 && ctx->tune.map_pair_reg == 1)
        hipLaunchKernelGGL((pf ? (nt ? map_pair_join_seg_kernel<32, 4, true, true> : map_pair_join_seg_kernel<32, 4, true, false>)
                              : (nt ? map_pair_join_seg_kernel<32, 4, false, true> : map_pair_join_seg_kernel<32, 4, false, false>)),
                           dim3(grid), dim3(kBlock), 0, ctx->stream, p);
      else if (A <= (size_t)kWave && ctx->tune.map_pair_reg == 1)
        hipLaunchKernelGGL((pf ? (nt ? map_pair_join_seg_kernel<64, 4, true, true> : map_pair_join_seg_kernel<64, 4, true, false>)
                              : (nt ? map_pair_join_seg_kernel<64, 4, false, true> : map_pair_join_seg_kernel<64, 4, false, false>)),
                           dim3(grid), dim3(kBlock), 0, ctx->stream, p);
      else if (A <= (size_t)kWave)
        hipLaunchKernelGGL((map_pair_join_reg_kernel<1, 4>), dim3(grid), dim3(kBlock), 0, ctx->stream, p);
      else if (A <= 2 * (size_t)kWave)
        hipLaunchKernelGGL((map_pair_join_reg_kernel<2, 4>), dim3(grid), dim3(kBlock), 0, ctx->stream, p);
      else
        hipLaunchKernelGGL((map_pair_join_reg_kernel<4, 4>), dim3(grid), dim3(kBlock), 0, ctx->stream, p);
    } else if (A <= (size_t)kWave)
      hipLaunchKernelGGL(map_pair_join_kernel<1>, dim3(grid), dim3(kBlock), 0, ctx->stream, p);
    else if (A <= 2 * (size_t)kWave)
      hipLaunchKernelGGL(map_pair_join_kernel<2>, dim3(grid), dim3(kBlock), 0, ctx->stream, p);
    else if (A <= 4 * (size_t)kWave)
      hipLaunchKernelGGL(map_pair_join_kernel<4>, dim3(grid), dim3(kBlock), 0, ctx->stream, p);
    else if (A <= 8 * (size_t)kWave)  // wide states (round 4): more clock words per lane
      hipLaunchKernelGGL(map_pair_join_kernel<8>, dim3(grid), dim3(kBlock), 0, ctx->stream, p);
    else
      hipLaunchKernelGGL(map_pair_join_kernel<16>, dim3(grid), dim3(kBlock), 0, ctx->stream, p);
    timing_end(ctx);
    CRDT_HIP(ctx, hipGetLastError());
  }
  return launch_pair_deferred(ctx, PairDefPlan{N, A, Kw, (u64 *)a.clock, a.clock_stride, (const u64 *)b.clock,
                                               b.clock_stride, (u64 *)self_def->clock, (u64 *)self_def->keys,
                                               self_def->count, self_def->Dcap, (const u64 *)other_def->clock,
                                               (const u64 *)other_def->keys,
                                               other_def->Dcap ? other_def->count : nullptr, other_def->Dcap, status,
                                               16u});
}
