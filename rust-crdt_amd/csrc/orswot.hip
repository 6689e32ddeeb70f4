// Orswot<member, actor> batched merge (lub of many replicas).
//
// Reference: Orswot::merge (orswot.rs:81-149), apply_rm (:230-250), apply_deferred (:281-286),
// VClock::forget (vclock.rs:95-105), intersection (:218-227), clone_without (:148-152).
//
// Dense restatement per (member m, actor a), with e = entry dot counter (0 = no dot),
// c = the replica clock's counter for a:
//   join((e1,c1),(e2,c2)) = ( max( e1==e2 ? e1 : 0,       // intersection (:113)
//                                  e1>c2  ? e1 : 0,       // our_clock.clone_without(other.clock) (:115)
//                                  e2>c1  ? e2 : 0 ),     // clock.clone_without(self.clock) (:114)
//                             max(c1, c2) )               // self.clock.merge (:145)
// One-sided members reduce to the same formula (:86-101 drop-if-dominated + forget, :124-136),
// and a member is present iff some e != 0 (empty common clock => removed, :116-118).
// On cells with e <= c (the reference's invariant: entry dots covered by their replica's clock)
// the join is associative (exhaustively checked on small counters), so replicas are folded per
// thread, then slice partials are joined by the last-arriving block.  A cell with e > c (a
// deserialized or hand-built state) breaks associativity: every block ORs "some input cell had
// e > c" into its arrival counter and, if any slice of the unit saw one, the last arriver re-folds
// the unit's cells over ALL replicas in replica order — the exact left fold for any input.
// Deferred removes (rm, S) of every replica are then applied after the join: for m in S,
// e = e > rm[a] ? e : 0 (forget); a deferred survives iff !(rm <= final clock) (:240-249);
// survivors with identical rm clocks merge their member sets (:242-246).  Applying them after the
// in-order join instead of at their own step is exact for any input: a forget commutes with every
// later join (forget(join(forget(x), y)) == forget(join(x, y)) per cell), a remove once dominated by
// the clock stays dominated, and a dominated remove's dots (<= rm <= c) never re-enter by the join
// (tests/test_oracle_twins.py checks this against the reference fold on arbitrary states).
#include "common.hpp"

namespace crdt {


template <int V>
struct OVec;
template <>
struct OVec<1> {
  using T = u64;
};
template <>
struct OVec<2> {
  using T = u64x2;
};

__device__ __forceinline__ u64 umax(u64 a, u64 b) { return a > b ? a : b; }

__device__ __forceinline__ u64 dot_join(u64 e1, u64 c1, u64 e2, u64 c2) {
  const u64 t0 = e1 == e2 ? e1 : 0;
  const u64 t1 = e1 > c2 ? e1 : 0;
  const u64 t2 = e2 > c1 ? e2 : 0;
  return umax(t0, umax(t1, t2));
}
__device__ __forceinline__ u64x2 dot_join(u64x2 e1, u64x2 c1, u64x2 e2, u64x2 c2) {
  u64x2 r;
  r.x = dot_join(e1.x, c1.x, e2.x, c2.x);
  r.y = dot_join(e1.y, c1.y, e2.y, c2.y);
  return r;
}
__device__ __forceinline__ u64x2 umax(u64x2 a, u64x2 b) {
  u64x2 r;
  r.x = umax(a.x, b.x);
  r.y = umax(a.y, b.y);
  return r;
}

struct OrPlan {
  const u64 *clock;
  const u64 *entries;
  long long c_rstride, c_gstride, e_mstride, e_rstride, e_gstride;  // words
  unsigned long long G, R, M, A, Rs;
  int Wv, PW, MB, ncolblk, nmblk, S;
  u64 *part;       // per unit: S slabs of (MB*MPT*PW E vectors + PW C vectors)
  unsigned *cnt;   // [units]
  u64 *out_clock;  // [G][A]
  u64 *out_entries;  // [G][M][A]
  const u64 *init_clock;    // optional fold start [G][A] (NULL: the empty Orswot)
  const u64 *init_entries;  // ... [G][M][A] packed
  unsigned *viol;           // optional [G]: bit 0 set where an input cell had e > c
};

// MPT member rows per thread (CRDT_TUNE ompt=4/8/16): a workgroup covers MB*MPT member rows of
// PW actor vectors, so MPT sets the bytes in flight per thread and how many workgroups re-read
// each replica clock row.
// OR_VIOL_BALLOT (build option): the main loop's e > c votes as ballots or-ed on the scalar unit
#ifndef OR_VIOL_BALLOT
#define OR_VIOL_BALLOT 0
#endif
template <int V, int UR, int MPT>
__global__ __launch_bounds__(kBlock) void orswot_join_kernel(OrPlan p) {
  constexpr int kOrMPT = MPT;
  using VT = typename OVec<V>::T;
  __shared__ int s_flag;
  const int l = threadIdx.x;
  const unsigned b = blockIdx.x;
  const int s = b % p.S;
  unsigned u = b / p.S;
  const int cb = u % p.ncolblk;
  const unsigned rest = u / p.ncolblk;
  const int mb = rest % p.nmblk;
  const size_t g = rest / p.nmblk;
  const int cl = l % p.PW;
  const int ml = l / p.PW;
  const int col = cb * kBlock + cl;
  const bool active = ml < p.MB && col < p.Wv;
  const size_t mbase = (size_t)mb * p.MB * kOrMPT + ml;

  VT e[kOrMPT], c;
  bool mok[kOrMPT];
#pragma unroll
  for (int j = 0; j < kOrMPT; ++j) mok[j] = active && (mbase + (size_t)j * p.MB) < p.M;
  bool viol = false;
#if OR_VIOL_BALLOT
  u64 vmask = 0;  // (the violation votes collected on the scalar unit: one compare + one SALU or)
#endif
  auto gt = [](VT x, VT y) -> bool {
    if constexpr (V == 2) return (x.x > y.x) | (x.y > y.y);
    else return x > y;
  };
  // the fold start: the caller's state (slice 0 / the exact re-fold) or the empty Orswot; a start
  // state with e > c is itself a reason to re-fold in order
  auto start = [&](bool from_init) {
    c = VT(0);
#pragma unroll
    for (int j = 0; j < kOrMPT; ++j) e[j] = VT(0);
    if (!from_init || !p.init_clock || !active) return;
    c = reinterpret_cast<const VT *>(p.init_clock + g * p.A)[col];
    const VT *ie = reinterpret_cast<const VT *>(p.init_entries + g * p.M * p.A);
#pragma unroll
    for (int j = 0; j < kOrMPT; ++j)
      if (mok[j]) {
        e[j] = ie[(mbase + (size_t)j * p.MB) * (p.A / V) + col];
        viol |= gt(e[j], c);
      }
  };
  // in-order fold of replicas [rbeg, rend) into (e, c); viol |= some loaded cell had e > c
  auto fold = [&](unsigned long long rbeg, unsigned long long rend) {
    const VT *cp = reinterpret_cast<const VT *>(p.clock + g * p.c_gstride + rbeg * p.c_rstride) + col;
    const VT *ep = reinterpret_cast<const VT *>(p.entries + g * p.e_gstride + rbeg * p.e_rstride +
                                                mbase * p.e_mstride) + col;
    const long long cstep = p.c_rstride / V;
    const long long estep = p.e_rstride / V;
    const long long mstep = (long long)p.MB * p.e_mstride / V;
    unsigned long long r = rbeg;
    // UR replicas' loads in flight, then their joins in fold order.
    for (; r + UR <= rend; r += UR) {
      VT c2[UR], e2[UR][kOrMPT];
#pragma unroll
      for (int q = 0; q < UR; ++q) {
        c2[q] = cp[q * cstep];
#pragma unroll
        for (int j = 0; j < kOrMPT; ++j)
          e2[q][j] = mok[j] ? __builtin_nontemporal_load(ep + q * estep + j * mstep) : VT(0);
      }
#pragma unroll
      for (int q = 0; q < UR; ++q) {
#pragma unroll
        for (int j = 0; j < kOrMPT; ++j) {
#if OR_VIOL_BALLOT
          if constexpr (V == 2) vmask |= __ballot(e2[q][j].x > c2[q].x) | __ballot(e2[q][j].y > c2[q].y);
          else vmask |= __ballot(e2[q][j] > c2[q]);
#else
          viol |= gt(e2[q][j], c2[q]);
#endif
          e[j] = dot_join(e[j], c, e2[q][j], c2[q]);
        }
        c = umax(c, c2[q]);
      }
      cp += UR * cstep;
      ep += UR * estep;
    }
    for (; r < rend; ++r) {
      const VT c2 = *cp;
      VT e2[kOrMPT];
#pragma unroll
      for (int j = 0; j < kOrMPT; ++j)
        e2[j] = mok[j] ? __builtin_nontemporal_load(ep + j * mstep) : VT(0);
#pragma unroll
      for (int j = 0; j < kOrMPT; ++j) {
        viol |= gt(e2[j], c2);
        e[j] = dot_join(e[j], c, e2[j], c2);
      }
      c = umax(c, c2);
      cp += cstep;
      ep += estep;
    }
  };

  start(s == 0);
  if (active) {
    const unsigned long long rbeg = (unsigned long long)s * p.Rs;
    fold(rbeg, min(p.R, rbeg + p.Rs));
  }
#if OR_VIOL_BALLOT
  viol |= vmask != 0;
#endif

  const size_t slab = (size_t)p.MB * kOrMPT * p.PW + p.PW;  // vectors
  auto store_final = [&](void) {
    if (!active) return;
    VT *oe = reinterpret_cast<VT *>(p.out_entries + g * p.M * p.A);
#pragma unroll
    for (int j = 0; j < kOrMPT; ++j)
      if (mok[j]) oe[(mbase + (size_t)j * p.MB) * (p.A / V) + col] = e[j];
    if (mb == 0 && ml == 0) reinterpret_cast<VT *>(p.out_clock + g * p.A)[col] = c;
  };
  if (p.S == 1) {  // one slice: the in-order fold of every replica, exact for any input
    if (p.viol && __syncthreads_or(viol) && l == 0) atomicOr(p.viol + g, 1u);
    store_final();
    return;
  }
  VT *part = reinterpret_cast<VT *>(p.part) + ((size_t)u * p.S + s) * slab;
  if (active) {
#pragma unroll
    for (int j = 0; j < kOrMPT; ++j) part[(ml + j * p.MB) * p.PW + cl] = e[j];
    if (ml == 0) part[(size_t)p.MB * kOrMPT * p.PW + cl] = c;
  }
  // Release this slab; the last slice of the unit joins all slabs (in slice order).  Bit 16 of the
  // unit's arrival counter collects "a slice saw a cell with e > c" (S <= 64 fits below it).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int bviol = __syncthreads_or(viol);
  if (l == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(p.cnt + u, bviol ? 0x10001u : 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t & 0xffffu) == (unsigned)p.S - 1;
    if (last) {
      __hip_atomic_store(p.cnt + u, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if ((bviol || (t >> 16)) && p.viol) atomicOr(p.viol + g, 1u);
    }
    s_flag = last | ((bviol || (t >> 16)) ? 2 : 0);
  }
  __syncthreads();
  if (!(s_flag & 1)) return;
  if (s_flag & 2) {  // some input cell of the unit had e > c: the exact in-order re-fold
    start(true);
    if (active) fold(0, p.R);
#if OR_VIOL_BALLOT
    viol |= vmask != 0;
#endif
  } else if (active) {
    c = VT(0);
#pragma unroll
    for (int j = 0; j < kOrMPT; ++j) e[j] = VT(0);
    const VT *pp = reinterpret_cast<const VT *>(p.part) + (size_t)u * p.S * slab;
    for (int k = 0; k < p.S; ++k, pp += slab) {
      const VT c2 = pp[(size_t)p.MB * kOrMPT * p.PW + cl];
#pragma unroll
      for (int j = 0; j < kOrMPT; ++j) e[j] = dot_join(e[j], c, pp[(ml + j * p.MB) * p.PW + cl], c2);
      c = umax(c, c2);
    }
  }
  store_final();
}


__device__ __forceinline__ unsigned long long group_of(const size_t *off, unsigned long long G,
                                                       unsigned long long d) {
  unsigned long long lo = 0, hi = G;  // find g with off[g] <= d < off[g+1]
  while (hi - lo > 1) {
    const unsigned long long mid = (lo + hi) / 2;
    if (off[mid] <= d) lo = mid;
    else hi = mid;
  }
  return lo;
}

// One workgroup per deferred remove: survival test, row hash, ceiling on the joined entries.
__global__ __launch_bounds__(kBlock) void orswot_deferred_kernel(DefPlan p) {
  __shared__ u64 s_hash[kBlock / kWave];
  const unsigned long long d = blockIdx.x;
  const unsigned long long g = group_of(p.def_off, p.G, d);
  const u64 *rm = p.def_clock + d * p.A;
  const u64 *cf = p.out_clock + g * p.A;
  int greater = 0;
  u64 h = 0;
  for (unsigned long long a = threadIdx.x; a < p.A; a += kBlock) {
    const u64 x = rm[a];
    greater |= x > cf[a];
    // Order-independent row hash (sum of per-cell mixes) to pre-filter identical clocks.
    u64 z = x * 0x9E3779B97F4A7C15ULL + a;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    h += z ^ (z >> 31);
  }
  const int keep = __syncthreads_or(greater);
  for (int off = kWave / 2; off > 0; off >>= 1) h += __shfl_down(h, off, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) s_hash[threadIdx.x / kWave] = h;
  // Ceiling: forget(rm) on every member of S (race-benign: only zeros are written and the
  // test reads the joined value, which no other write can change except to zero).
  const u64 *bits = p.def_members + d * p.Mw;
  u64 *E = p.out_entries + g * p.M * p.A;
  for (unsigned long long w = 0; w < p.Mw && p.apply_ceiling; ++w) {
    u64 word = bits[w];
    while (word) {
      const int bit = __builtin_ctzll(word);
      word &= word - 1;
      const unsigned long long m = w * 64 + bit;
      if (m >= p.M) break;
      u64 *row = E + m * p.A;
      for (unsigned long long a = threadIdx.x; a < p.A; a += kBlock) {
        const u64 e = row[a];
        if (e != 0 && e <= rm[a]) row[a] = 0;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 t = 0;
    for (int w = 0; w < kBlock / kWave; ++w) t += s_hash[w];
    p.hash[d] = t;
    if (keep) p.surv[atomicAdd(p.nsurv, 1u)] = (unsigned)d;
  }
}

// Survivors with identical rm clocks (and group) must find their representative, the smallest
// such index.  Open-addressing table keyed by the row hash mixed with the group: pass 1 inserts
// every survivor and keeps the minimum index per key (atomicMin), pass 2 looks its key up and
// verifies the candidate's clock exactly; only a true 64-bit collision (two different clocks, same
// key) falls back to a scan of the survivor list.  O(survivors), not O(survivors^2).
__device__ __forceinline__ u64 dedup_key(u64 h, unsigned long long g) {
  u64 z = h ^ ((g + 1) * 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 31)) * 0xD6E8FEB86659FD93ULL;
  z ^= z >> 32;
  return z ? z : 1;  // 0 marks an empty slot
}

__device__ __forceinline__ unsigned long long dedup_slot(const DefPlan &p, u64 key, bool insert, unsigned d) {
  unsigned long long t = key & p.tmask;
  while (true) {
    const u64 cur = insert ? atomicCAS(p.tkey + t, 0ull, key) : p.tkey[t];
    if (cur == key || (insert && cur == 0)) return t;
    if (!insert && cur == 0) return ~0ull;  // not found: cannot happen for an inserted key
    t = (t + 1) & p.tmask;
  }
}

__global__ __launch_bounds__(kBlock) void orswot_dedup_insert_kernel(DefPlan p) {
  const unsigned k = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned n = *p.nsurv;
  if (k >= n) return;
  const unsigned d = p.surv[k];
  const u64 key = dedup_key(p.hash[d], group_of(p.def_off, p.G, d));
  atomicMin(p.trep + dedup_slot(p, key, true, d), d);
}

__global__ __launch_bounds__(kBlock) void orswot_dedup_kernel(DefPlan p) {
  const unsigned k = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned n = *p.nsurv;
  if (k >= n) return;
  const unsigned d = p.surv[k];
  const unsigned long long g = group_of(p.def_off, p.G, d);
  const u64 key = dedup_key(p.hash[d], g);
  const unsigned long long t = dedup_slot(p, key, false, d);
  const u64 *rm = p.def_clock + (size_t)d * p.A;
  auto same = [&](unsigned d2) {
    if (d2 < p.def_off[g] || d2 >= p.def_off[g + 1]) return false;
    const u64 *rm2 = p.def_clock + (size_t)d2 * p.A;
    for (unsigned long long a = 0; a < p.A; ++a)
      if (rm[a] != rm2[a]) return false;
    return true;
  };
  unsigned rep = t == ~0ull ? d : p.trep[t];
  if (rep != d && !same(rep)) {  // a true key collision: exact scan of the survivors
    rep = d;
    for (unsigned j = 0; j < n; ++j) {
      const unsigned d2 = p.surv[j];
      if (d2 < rep && p.hash[d2] == p.hash[d] && same(d2)) rep = d2;
    }
  }
  if (rep == d) p.out_keep[d] = 1;
  const u64 *src = p.def_members + (size_t)d * p.Mw;
  u64 *dst = p.out_members + (size_t)rep * p.Mw;
  for (unsigned long long w = 0; w < p.Mw; ++w)
    if (src[w]) atomicOr(dst + w, src[w]);
}

static bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

__global__ __launch_bounds__(kBlock) void def_off_check_kernel(const u64 *src, size_t *dst, unsigned long long G,
                                                               unsigned long long D, unsigned *status,
                                                               unsigned *flags) {
  const unsigned long long i = (unsigned long long)blockIdx.x * kBlock + threadIdx.x;
  if (i > G) return;
  const u64 v = src[i];
  bool bad = i == 0 ? v != 0 : (i == G ? v != D : v > D);
  if (i > 0 && src[i - 1] > v) bad = true;
  dst[i] = i == 0 ? 0 : (i == G ? D : (v > D ? D : v));
  if (bad) {
    if (status) atomicOr(status, 1u);
    if (flags) {
      if (i > 0) atomicOr(flags + i - 1, 2u);
      if (i < G) atomicOr(flags + i, 2u);
    }
  }
}

int stage_def_off_dev(crdt_ctx *ctx, const u64 *src, size_t *dst, size_t G, size_t D, unsigned *status,
                      unsigned *flags) {
  const size_t n = G + 1;
  hipLaunchKernelGGL(def_off_check_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     ctx->stream, src, dst, (unsigned long long)G, (unsigned long long)D, status, flags);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

// Survival, ceiling (optional) and dedup of a pooled deferred-remove list (shared by Orswot and
// Map): stages def_off (from the host, or checked from device memory), fills the outputs,
// launches the two kernels.
int launch_deferred(crdt_ctx *ctx, const size_t *host_def_off, DefPlan q, const u64 *dev_def_off, unsigned *status) {
  const size_t G = q.G, D = q.D;
  // Deferred bookkeeping lives in its own ctx-owned region (plain hipMalloc, like scratch), so
  // the join's scratch, possibly still in flight, is untouched.
  const size_t off_b = (G + 1) * sizeof(size_t);
  size_t T = 64;
  while (T < 2 * D) T <<= 1;  // dedup table: load factor <= 1/2
  const size_t off_pad = (off_b + 255) / 256 * 256;
  const size_t need = 256 + off_pad + D * 8 + D * 4 + 64 + T * 12;
  if (int rc = ensure_dscratch(ctx, need)) return rc;
  char *base = static_cast<char *>(ctx->dscratch);
  q.nsurv = reinterpret_cast<unsigned *>(base);
  q.def_off = reinterpret_cast<const size_t *>(base + 256);
  q.hash = reinterpret_cast<u64 *>(base + 256 + off_pad);
  q.surv = reinterpret_cast<unsigned *>(q.hash + D);
  q.tkey = reinterpret_cast<u64 *>(base + ((256 + off_pad + D * 12 + 63) / 64 * 64));
  q.trep = reinterpret_cast<unsigned *>(q.tkey + T);
  q.tmask = T - 1;
  if (int rc = device_fill(ctx, q.tkey, T * 8, 0)) return rc;
  if (int rc = device_fill(ctx, q.trep, T * 4, 0xFF)) return rc;
  if (int rc = device_fill(ctx, q.nsurv, 4, 0)) return rc;
  if (dev_def_off) {  // device offsets: checked (status) and clamped on the device
    if (int rc = stage_def_off_dev(ctx, dev_def_off, (size_t *)q.def_off, G, D, status, nullptr)) return rc;
  } else {  // the caller's def_off may be freed on return: stage it through pinned ctx memory
    int rc = stage_h2d(ctx, (void *)q.def_off, host_def_off, off_b);
    if (rc) return rc;
  }
  if (int rc = device_fill(ctx, q.out_keep, D, 0)) return rc;
  if (int rc = device_fill(ctx, q.out_members, D * q.Mw * 8, 0)) return rc;
  hipLaunchKernelGGL(orswot_deferred_kernel, dim3((unsigned)D), dim3(kBlock), 0, ctx->stream, q);
  hipLaunchKernelGGL(orswot_dedup_insert_kernel, dim3((unsigned)((D + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     ctx->stream, q);
  hipLaunchKernelGGL(orswot_dedup_kernel, dim3((unsigned)((D + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     ctx->stream, q);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

}  // namespace crdt

using namespace crdt;

// doff: the device-offset variant's def_off (in->def_off is then NULL and D the pool length)
static int orswot_lub_impl(crdt_ctx *ctx, const crdt_orswot_batch *in, const u64 *doff, size_t Ddev,
                           crdt_orswot_out *out, unsigned *status, const OrswotJoinExtra *ex = nullptr) {
  const size_t G = in->G, R = in->R, M = in->M, A = in->A;
  if (G == 0 || A == 0) return CRDT_OK;
  if (!out->clock || (M && !out->entries)) return fail(ctx, CRDT_EINVAL, "orswot_lub_many: NULL output");
  if (R > 0 && (!in->clock || (M && !in->entries)))
    return fail(ctx, CRDT_EINVAL, "orswot_lub_many: NULL input");
  if (in->entry_mstride < A && M > 1)
    return fail(ctx, CRDT_EINVAL, "orswot_lub_many: entry_mstride < A");
  if (A > (1u << 20) || M > (1ull << 32))
    return fail(ctx, CRDT_EUNSUPPORTED, "orswot_lub_many: A or M too large");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const size_t D = doff ? Ddev : (in->def_off && G > 0) ? in->def_off[G] - in->def_off[0] : 0;
  if (in->def_off && in->def_off[0] != 0)
    return fail(ctx, CRDT_EINVAL, "orswot_lub_many: def_off[0] must be 0");
  const size_t Mw = (M + 63) / 64;
  if (D > 0 && (!in->def_clock || !out->def_keep || (Mw && (!in->def_members || !out->def_members))))
    return fail(ctx, CRDT_EINVAL, "orswot_lub_many: deferred buffers missing");
  if (D > 0xffffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "orswot_lub_many: too many deferred");

  if (ex && ex->viol)
    if (int rc = device_fill(ctx, ex->viol, G * 4, 0)) return rc;
  if (R == 0 && ex && ex->init_clock) {  // nothing to fold: the start state
    CRDT_HIP(ctx, hipMemcpyAsync(out->clock, ex->init_clock, G * A * 8, hipMemcpyDeviceToDevice, ctx->stream));
    if (M)
      CRDT_HIP(ctx, hipMemcpyAsync(out->entries, ex->init_entries, G * M * A * 8, hipMemcpyDeviceToDevice,
                                   ctx->stream));
  } else if (R == 0) {
    int rc = device_fill(ctx, out->clock, G * A * 8, 0);
    if (!rc && M) rc = device_fill(ctx, out->entries, G * M * A * 8, 0);
    if (rc) return rc;
  } else if (M == 0) {  // no members: the state is its clock (plus the removes' survival below)
    if (int rc = lattice_lub_many(ctx, Op::Max, (const u64 *)in->clock, G, R, A, in->clock_rstride,
                                  in->clock_gstride, (u64 *)out->clock, A, 0))
      return rc;
  } else {
    const bool vec2 = A % 2 == 0 && in->clock_rstride % 2 == 0 && in->clock_gstride % 2 == 0 &&
                      in->entry_mstride % 2 == 0 && in->entry_rstride % 2 == 0 &&
                      in->entry_gstride % 2 == 0 && al16(in->clock) && al16(in->entries) &&
                      al16(out->clock) && al16(out->entries) &&
                      (!ex || !ex->init_clock || (al16(ex->init_clock) && al16(ex->init_entries)));
    const int V = vec2 ? 2 : 1;
    OrPlan p{};
    p.clock = (const u64 *)in->clock;
    p.entries = (const u64 *)in->entries;
    p.c_rstride = in->clock_rstride;
    p.c_gstride = in->clock_gstride;
    p.e_mstride = in->entry_mstride;
    p.e_rstride = in->entry_rstride;
    p.e_gstride = in->entry_gstride;
    p.G = G;
    p.R = R;
    p.M = M;
    p.A = A;
    p.Wv = (int)(A / V);
    p.PW = p.Wv <= kBlock ? p.Wv : kBlock;
    p.MB = kBlock / p.PW;
    p.ncolblk = (p.Wv + kBlock - 1) / kBlock;
    const int MPT = ctx->tune.orswot_mpt == 8 ? 8 : (ctx->tune.orswot_mpt == 16 ? 16 : 4);
    const size_t mpb = (size_t)p.MB * MPT;
    p.nmblk = (int)((M + mpb - 1) / mpb);
    p.out_clock = (u64 *)out->clock;
    p.out_entries = (u64 *)out->entries;
    if (ex) {
      p.init_clock = ex->init_clock;
      p.init_entries = ex->init_entries;
      p.viol = ex->viol;
    }
    const size_t units = G * (size_t)p.nmblk * p.ncolblk;
    const size_t target = (size_t)ctx->cu_count * ctx->tune.orswot_blocks_per_cu;
    size_t S = 1;
    if (units < target) {
      S = (target + units - 1) / units;
      size_t max_s = R / 8;
      if (max_s < 1) max_s = 1;
      if (S > max_s) S = max_s;
      if (S > 64) S = 64;
    }
    size_t Rs = (R + S - 1) / S;
    S = (R + Rs - 1) / Rs;
    p.S = (int)S;
    p.Rs = Rs;
    if (units * S > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "orswot_lub_many: grid too large");
    if (S > 1) {
      const size_t slab_b = (mpb * p.PW + p.PW) * V * 8;
      int rc = ensure_scratch(ctx, units * S * slab_b);
      if (rc) return rc;
      rc = ensure_counters(ctx, units);
      if (rc) return rc;
      p.cnt = ctx->counters;
      p.part = reinterpret_cast<u64 *>(ctx->scratch);
    }
    timing_begin(ctx, "orswot_join");
    const dim3 grid((unsigned)(units * S));
    const int UR = ctx->tune.orswot_unroll;
#define CRDT_ORJ(VV, UU, MM) hipLaunchKernelGGL((orswot_join_kernel<VV, UU, MM>), grid, dim3(kBlock), 0, ctx->stream, p)
    if (V == 2) {
      if (MPT == 4) {
        if (UR == 1) CRDT_ORJ(2, 1, 4);
        else if (UR == 4) CRDT_ORJ(2, 4, 4);
        else CRDT_ORJ(2, 2, 4);
      } else if (MPT == 8) {
        if (UR == 1) CRDT_ORJ(2, 1, 8);
        else CRDT_ORJ(2, 2, 8);
      } else {
        CRDT_ORJ(2, 1, 16);
      }
    } else {
      CRDT_ORJ(1, 2, 4);
    }
#undef CRDT_ORJ
    timing_end(ctx);
    CRDT_HIP(ctx, hipGetLastError());
  }

  if (D == 0) return CRDT_OK;
  DefPlan q{};
  q.G = G;
  q.D = D;
  q.M = M;
  q.A = A;
  q.Mw = Mw;
  q.def_clock = (const u64 *)in->def_clock;
  q.def_members = (const u64 *)in->def_members;
  q.out_clock = (const u64 *)out->clock;
  q.out_entries = (u64 *)out->entries;
  q.apply_ceiling = 1;
  q.out_keep = out->def_keep;
  q.out_members = (u64 *)out->def_members;
  return launch_deferred(ctx, in->def_off, q, doff, status);
}

namespace crdt {
int orswot_lub_many_ex(crdt_ctx *ctx, const crdt_orswot_batch *in, crdt_orswot_out *out, const OrswotJoinExtra &ex) {
  return orswot_lub_impl(ctx, in, nullptr, 0, out, nullptr, &ex);
}
}  // namespace crdt

extern "C" int crdt_orswot_lub_many(crdt_ctx *ctx, const crdt_orswot_batch *in,
                                    crdt_orswot_out *out) {
  if (ctx && ctx->mem_kind == CRDT_MEM_HOST) return crdt::orswot_lub_many_host(ctx, in, out);
  CRDT_CHECK_CTX(ctx);
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "orswot_lub_many: NULL batch/out");
  return orswot_lub_impl(ctx, in, nullptr, 0, out, nullptr);
}

extern "C" int crdt_orswot_lub_many_doff(crdt_ctx *ctx, const crdt_orswot_batch *in, const uint64_t *def_off,
                                         size_t D, crdt_orswot_out *out, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "orswot_lub_many_doff: NULL batch/out");
  if (in->def_off) return fail(ctx, CRDT_EINVAL, "orswot_lub_many_doff: in->def_off must be NULL");
  if (!def_off && D) return fail(ctx, CRDT_EINVAL, "orswot_lub_many_doff: D > 0 without def_off");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  if (status)  // written for every call, an empty batch included
    if (int rc = device_fill(ctx, status, sizeof(uint32_t), 0)) return rc;
  if (in->G == 0 || in->A == 0) return CRDT_OK;
  if (def_off && D == 0) {  // no pool: only the offsets' check (every entry must be 0)
    if (int rc = ensure_dscratch(ctx, (in->G + 1) * sizeof(size_t))) return rc;
    if (int rc = stage_def_off_dev(ctx, (const u64 *)def_off, (size_t *)ctx->dscratch, in->G, 0, status, nullptr))
      return rc;
    def_off = nullptr;
  }
  return orswot_lub_impl(ctx, in, (const u64 *)def_off, def_off ? D : 0, out, status);
}
