// Batched Orswot CmRDT::apply: N independent states, each with its own ordered op stream
// (the order-dependent half of the kept trait surface).
//
// Reference (orswot.rs:55-79, 230-250, 281-286), restated on the dense layout
// (clock C[a], entries E[m][a] with a 0 cell = actor absent, deferred list of (rm clock, member
// set) with pairwise-distinct clocks):
//   Op::Add { dot (a, k), members }:
//       if C[a] >= k: seen, no-op                                          (:60-63)
//       for m in members: E[m][a] = max(E[m][a], k)     (entry().or_default().apply(dot), :65-68)
//       C[a] = k                                                           (:70)
//       apply_deferred(): every deferred (rm, S) is re-applied: forget E[m] by rm for m in S,
//           kept iff !(rm <= C); no two kept clocks are equal, so no sets merge   (:71, :281-286)
//   Op::Rm { clock rm, members }:  apply_rm                                (:74-76, :230-250)
//       for m in members: E[m][a] = E[m][a] > rm[a] ? E[m][a] : 0   (VClock::forget, vclock.rs:95-105;
//                                                   an all-zero row is the removed entry)
//       if !(rm <= C) (partial_cmp in {None, Greater}): defer (rm, members), OR-ing the set into
//       an existing deferred with the identical clock (HashMap keyed by the whole VClock)
// Ops of one state are sequential (apply is not commutative: the seen test and the deferred
// removes depend on order), so the unit of parallelism is the state: one wave per state, lanes
// over actors (clock rows in registers, A <= 1,024) or over the op's member list.  The op headers
// of 64 ops are loaded at once (lane = op) and read out with readlane; the deferred list lives in
// LDS for the whole stream.  Exact for ANY input state (apply_deferred re-forgets every deferred
// member row, as the reference does, instead of assuming the invariant the reference's own
// states keep).
#include "common.hpp"
#include "group.hpp"

namespace crdt {

constexpr int kApplyMaxA = 1024;  // the A <= 1,024 instance: 16 clock words per lane
constexpr int kCAMax = 4;         // clock words per lane of the A <= 256 instance
constexpr unsigned kBadOp = 0xFFFFFFFFu, kRmOp = 0xFFFFFFFEu;  // packed op header tags

struct OrswotApplyPlan {
  u64 *clock;
  unsigned long long clock_stride;
  u64 *entries;
  unsigned long long entry_mstride, entry_sstride;
  u64 *def_clock, *def_members;
  uint32_t *def_count;
  unsigned long long N, M, A, Mw, Dcap, Dh;  // Dh: hot deferred slots kept in LDS (the rest in HBM)
  const u64 *op_off;
  const uint8_t *kind;
  const uint32_t *actor;
  const u64 *counter;
  const uint32_t *rm_row;
  const u64 *rm_clock;
  unsigned long long n_rm_rows;
  const u64 *mem_off;
  const uint32_t *mem;
  unsigned long long n_mem;
  unsigned long long n_ops;
  uint32_t *status;
  int wpb;
  int fence;  // 1: a workgroup fence after every op's stores (CRDT_TUNE afence=1, the round-2 form)
  int l2pf;   // 1: touch a one-member Rm's entry row with the batch header (CRDT_TUNE oal2=1)
};

__device__ __forceinline__ u64 rl64(u64 x, int l) {
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)x, l);
  const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(x >> 32), l);
  return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ unsigned rl32(unsigned x, int l) {
  return (unsigned)__builtin_amdgcn_readlane((int)x, l);
}

__device__ __forceinline__ void wave_fence() {
  // Stores of this wave (global and LDS) are complete and visible to its later loads (all lanes of
  // a workgroup share the CU's L1, so workgroup scope is enough).
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
}

// forget one entry row by the clock held in registers: keep e[a] iff e[a] > rm[a]
template <int kCA>
__device__ __forceinline__ void forget_row(u64 *row, const u64 (&r)[kCA], int lane, unsigned long long A) {
#pragma unroll
  for (int j = 0; j < kCA; ++j) {
    const unsigned long long a = lane + j * kWave;
    if (a < A) {
      const u64 v = row[a];
      if (v != 0 && v <= r[j]) row[a] = 0;
    }
  }
}

// forget every member row named in an LDS bitmap of Mw words
template <int kCA>
__device__ __forceinline__ void forget_members(const OrswotApplyPlan &p, u64 *E, const u64 *bits,
                                               const u64 (&r)[kCA], int lane) {
  for (unsigned long long w0 = 0; w0 < p.Mw; w0 += kWave) {
    const u64 word = (w0 + lane < p.Mw) ? bits[w0 + lane] : 0;
    u64 nz = __ballot(word != 0);
    while (nz) {
      const int l = __builtin_ctzll(nz);
      nz &= nz - 1;
      u64 wv = rl64(word, l);
      while (wv) {
        const unsigned long long m = (w0 + l) * 64 + __builtin_ctzll(wv);
        wv &= wv - 1;
        if (m < p.M) forget_row(E + m * p.entry_mstride, r, lane, p.A);
      }
    }
  }
}

template <int kCA>
__device__ __forceinline__ bool any_greater(const u64 (&r)[kCA], const u64 (&c)[kCA], int lane,
                                            unsigned long long A) {
  bool g = false;
#pragma unroll
  for (int j = 0; j < kCA; ++j)
    if (lane + j * kWave < (int)A && r[j] > c[j]) g = true;
  return __ballot(g) != 0;
}

// kCA clock words per lane: 1 for A <= 64 (fewer VGPRs, more waves per SIMD), 4 up to A = 256
template <int kCA>
__device__ __forceinline__ void orswot_apply_body(const OrswotApplyPlan &p) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x % kWave;
  const int wib = threadIdx.x / kWave;
  const unsigned long long per_wave = p.Dh * (p.A + p.Mw);
  u64 *lcl = lds + wib * per_wave;  // [Dh][A] rm clocks of the hot slots
  u64 *lmb = lcl + p.Dh * p.A;      // [Dh][Mw] their member bitmaps
  const unsigned long long A = p.A;

  for (unsigned long long s = (unsigned long long)blockIdx.x * p.wpb + wib; s < p.N;
       s += (unsigned long long)gridDim.x * p.wpb) {
    unsigned st = 0;
    const unsigned long long ob = p.op_off[s], oe = p.op_off[s + 1];
    unsigned dcnt = p.def_count[s];
    if (dcnt > p.Dcap || oe < ob || oe > p.n_ops) {
      if (lane == 0) p.status[s] = (dcnt > p.Dcap ? 4u : 0u) | (oe < ob || oe > p.n_ops ? 8u : 0u);
      continue;  // state left untouched
    }
    u64 c[kCA];
    u64 *C = p.clock + s * p.clock_stride;
#pragma unroll
    for (int j = 0; j < kCA; ++j) {
      const unsigned long long a = lane + j * kWave;
      c[j] = a < A ? C[a] : 0;
    }
    u64 *E = p.entries + s * p.entry_sstride;
    // slot d lives in LDS for d < Dh, else in the state's own HBM slot (generic pointers: the
    // same code reads either; most states never hold more than Dh deferred removes)
    u64 *gdc = p.def_clock + s * p.Dcap * A;
    u64 *gdm = p.def_members + s * p.Dcap * p.Mw;
    auto SC = [&](unsigned long long d) -> u64 * { return d < p.Dh ? lcl + d * A : gdc + d * A; };
    auto SM = [&](unsigned long long d) -> u64 * { return d < p.Dh ? lmb + d * p.Mw : gdm + d * p.Mw; };
    const unsigned long long dhot = dcnt < p.Dh ? dcnt : p.Dh;
    for (unsigned long long i = lane; i < dhot * A; i += kWave) lcl[i] = gdc[i];
    for (unsigned long long i = lane; i < dhot * p.Mw; i += kWave) lmb[i] = gdm[i];
    wave_fence();
    // apply_deferred re-forgets every member of every deferred slot (orswot.rs:281-286).  After
    // one full pass each slot's members are forgotten by its clock; a Rm only forgets more (forgets
    // commute) and a new slot's members were just forgotten by it, so a later one-member Add only
    // needs its own member's row re-forgotten (idempotent elsewhere).  The first pass stays full:
    // the input state need not hold the invariant.
    bool full = true;

    for (unsigned long long base = ob; base < oe; base += kWave) {
      // op headers, lane = op
      const unsigned long long o = base + lane;
      const bool ov = o < oe;
      // packed to keep VGPRs down: h_ka = actor of a valid Add, kRmOp for a Rm, kBadOp for a
      // malformed op (kind > 1, actor >= A or member range reversed); h_cr = counter of an Add,
      // rm row of a Rm; member offsets as 32 bits (an op whose member range ends at or beyond
      // 2^32 is reported malformed, status bit 1, never silently truncated; so is a range that
      // runs past the n_mem entries of mem)
      unsigned h_ka = kBadOp, h_mb = 0, h_me = 0, h_m0 = 0;  // h_m0: an Add's first member
      u64 h_cr = 0;
      if (ov) {
        const unsigned kind = p.kind[o];
        const u64 mb = p.mem_off[o], me = p.mem_off[o + 1];
        h_mb = (unsigned)mb;
        h_me = (unsigned)me;
        const bool range_ok = me >= mb && me <= 0xFFFFFFFFull && me <= p.n_mem;
        if (range_ok && kind == 0) {
          const unsigned a = p.actor ? p.actor[o] : 0u;
          h_ka = a < A ? a : kBadOp;
          h_cr = p.counter ? p.counter[o] : 0ull;
          if (me > mb) h_m0 = p.mem[mb];  // loaded with the headers: a one-member Add skips that round trip
        } else if (range_ok && kind == 1) {
          h_ka = kRmOp;
          h_cr = p.rm_row ? p.rm_row[o] : 0u;
          if (me > mb) h_m0 = p.mem[mb];  // a one-member Rm skips that round trip too
        }
      }
      const int nb = (int)((oe - base) < (unsigned long long)kWave ? (oe - base) : kWave);
      // The cell of the NEXT op when it is a one-member Add is loaded (lane 0) while this op runs,
      // so its read is not one more dependent round trip.  It is dropped (the op then loads its
      // cell itself) when this op may write that member's row: a write to the same member (an Add's
      // cell or its restricted re-forget, a one-member Rm), or to rows not tracked here (several
      // members, a full apply_deferred pass).  A wave's later loads see its earlier stores (all
      // lanes of a wave go through one L1 in program order), so the prefetch after them is exact.
      bool pf_have = false;
      unsigned long long pf_m = 0;
      u64 pf_val = 0;
      for (int i = 0; i < nb; ++i) {
        const unsigned ka = rl32(h_ka, i);
        const u64 mb = rl32(h_mb, i), me = rl32(h_me, i);
        const bool pf_use = pf_have;  // the prefetch made for this op is still valid
        const u64 pf_cur = pf_val;
        pf_have = false;
        if (i + 1 < nb) {
          const unsigned ka1 = rl32(h_ka, i + 1);
          if (ka1 != kBadOp && ka1 != kRmOp && rl32(h_me, i + 1) - rl32(h_mb, i + 1) == 1) {
            const unsigned long long m1 = rl32(h_m0, i + 1);
            if (m1 < p.M) {
              if (lane == 0) pf_val = E[m1 * p.entry_mstride + ka1];
              pf_have = true;
              pf_m = m1;
            }
          }
        }
        if (ka == kBadOp) {
          st |= 2u;
          continue;
        }
        if (ka != kRmOp) {  // ---- Op::Add
          const unsigned long long a = ka;
          const u64 k = rl64(h_cr, i);
          const int ja = (int)(a / kWave), la = (int)(a % kWave);
          u64 cj = c[0];
#pragma unroll
          for (int j = 1; j < kCA; ++j)
            if (j == ja) cj = c[j];
          if (rl64(cj, la) >= k) continue;  // already seen (:60-63)
          bool bad = false;
          if (me - mb == 1) {
            const unsigned long long m = rl32(h_m0, i);
            if (m >= p.M) {
              bad = true;
            } else {
              if (m == pf_m) pf_have = false;  // this op writes the next op's row
              if (lane == 0) {
                u64 *cell = E + m * p.entry_mstride + a;
                const u64 old = pf_use ? pf_cur : *cell;
                if (old < k) *cell = k;
              }
            }
          } else {
            pf_have = false;
            for (u64 jm = mb + lane; jm < me; jm += kWave) {
              const unsigned long long m = p.mem[jm];
              if (m >= p.M) {
                bad = true;
                continue;
              }
              u64 *cell = E + m * p.entry_mstride + a;
              if (*cell < k) *cell = k;
            }
          }
          if (__ballot(bad)) st |= 2u;
#pragma unroll
          for (int j = 0; j < kCA; ++j)
            if (j == ja && lane == la) c[j] = k;
          if (p.fence) wave_fence();
          // apply_deferred (:281-286)
          if (full || me - mb != 1) pf_have = false;  // rows of every slot's members may change
          unsigned nk = 0;
          for (unsigned d = 0; d < dcnt; ++d) {
            u64 r[kCA];
#pragma unroll
            for (int j = 0; j < kCA; ++j) {
              const unsigned long long aa = lane + j * kWave;
              r[j] = aa < A ? SC(d)[aa] : 0;
            }
            if (full || me - mb != 1) {
              forget_members(p, E, SM(d), r, lane);
            } else {  // a one-member Add after a full pass: only member m0's row can need it
              const unsigned long long m0 = rl32(h_m0, i);
              if (m0 < p.M && ((rl64(SM(d)[m0 / 64], 0) >> (m0 % 64)) & 1ull))
                forget_row(E + m0 * p.entry_mstride, r, lane, A);
            }
            if (any_greater(r, c, lane, A)) {
              if (nk != d) {
                u64 *dc = SC(nk), *sc = SC(d), *dm = SM(nk), *sm = SM(d);
                for (unsigned long long t = lane; t < A; t += kWave) dc[t] = sc[t];
                for (unsigned long long t = lane; t < p.Mw; t += kWave) dm[t] = sm[t];
              }
              ++nk;
            }
          }
          dcnt = nk;
          full = false;
          if (p.fence) wave_fence();
        } else {  // ---- Op::Rm -> apply_rm (:230-250)
          const unsigned rr = (unsigned)rl64(h_cr, i);
          if (rr >= p.n_rm_rows) {
            st |= 2u;
            continue;
          }
          u64 r[kCA];
          const u64 *R = p.rm_clock + (unsigned long long)rr * A;
#pragma unroll
          for (int j = 0; j < kCA; ++j) {
            const unsigned long long aa = lane + j * kWave;
            r[j] = aa < A ? R[aa] : 0;
          }
          if (me - mb == 1) {
            const unsigned long long m = rl32(h_m0, i);
            if (m >= p.M) st |= 2u;
            else forget_row(E + m * p.entry_mstride, r, lane, A);
            if (m == pf_m) pf_have = false;
          } else {
            pf_have = false;
            for (u64 jb = mb; jb < me; jb += kWave) {
              const unsigned mm = jb + lane < me ? p.mem[jb + lane] : 0u;
              const int n = (int)((me - jb) < (u64)kWave ? (me - jb) : kWave);
              for (int t = 0; t < n; ++t) {
                const unsigned long long m = rl32(mm, t);
                if (m >= p.M) {
                  st |= 2u;
                  continue;
                }
                forget_row(E + m * p.entry_mstride, r, lane, A);
              }
            }
          }
          if (p.fence) wave_fence();
          if (!any_greater(r, c, lane, A)) continue;  // rm <= C: already seen (:239-249)
          int slot = -1;
          for (unsigned d = 0; d < dcnt; ++d) {
            bool ne = false;
#pragma unroll
            for (int j = 0; j < kCA; ++j) {
              const unsigned long long aa = lane + j * kWave;
              if (aa < A && SC(d)[aa] != r[j]) ne = true;
            }
            if (__ballot(ne) == 0) {
              slot = (int)d;
              break;
            }
          }
          if (slot < 0) {
            if (dcnt >= p.Dcap) {
              st |= 1u;  // deferred capacity exceeded: this state's result is incomplete
              continue;
            }
            slot = (int)dcnt++;
#pragma unroll
            for (int j = 0; j < kCA; ++j) {
              const unsigned long long aa = lane + j * kWave;
              if (aa < A) SC(slot)[aa] = r[j];
            }
            for (unsigned long long t = lane; t < p.Mw; t += kWave) SM(slot)[t] = 0;
            wave_fence();
          }
          u64 *bits = SM(slot);
          if ((unsigned long long)slot < p.Dh) {  // LDS: lanes OR their members in at once
            for (u64 jm = mb + lane; jm < me; jm += kWave) {
              const unsigned long long m = p.mem[jm];
              if (m < p.M) atomicOr(bits + m / 64, 1ull << (m % 64));
            }
          } else {  // an HBM slot: plain read-modify-writes one member at a time (L2 atomics would
                    // leave this wave's L1 free to serve a stale line to its later plain loads)
            for (u64 jb = mb; jb < me; jb += kWave) {
              const unsigned mm = jb + lane < me ? (unsigned)p.mem[jb + lane] : 0u;
              const int n = (int)((me - jb) < (u64)kWave ? (me - jb) : kWave);
              for (int t = 0; t < n; ++t) {
                const unsigned long long m = (unsigned)__builtin_amdgcn_readlane((int)mm, t);
                if (m < p.M && lane == 0) bits[m / 64] |= 1ull << (m % 64);
                wave_fence();
              }
            }
          }
          wave_fence();
        }
      }
    }
    // write the state back
#pragma unroll
    for (int j = 0; j < kCA; ++j) {
      const unsigned long long a = lane + j * kWave;
      if (a < A) C[a] = c[j];
    }
    const unsigned long long dout = dcnt < p.Dh ? dcnt : p.Dh;  // slots >= Dh are already in HBM
    for (unsigned long long i = lane; i < dout * A; i += kWave) gdc[i] = lcl[i];
    for (unsigned long long i = lane; i < dout * p.Mw; i += kWave) gdm[i] = lmb[i];
    if (lane == 0) {
      p.def_count[s] = dcnt;
      p.status[s] = st;
    }
    wave_fence();
  }
}

// A <= 64: 72 VGPRs, no scratch, and asking for 7 waves per SIMD (the scheduler's target, the
// same register count) is 9% faster (1.99 -> 1.80 ms, profiles/r01_apply_wpe.log).  The A <= 256
// instance would spill at 7 waves, so it keeps the compiler's choice.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(7))) void orswot_apply_kernel_a64(
    OrswotApplyPlan p) {
  orswot_apply_body<1>(p);
}
__global__ __launch_bounds__(kBlock) void orswot_apply_kernel_a256(OrswotApplyPlan p) {
  orswot_apply_body<kCAMax>(p);
}
// Wide states (A <= 1,024, round 4: the reference's VClock is unbounded): 16 clock words per lane,
// the same body — a correctness path, not a tuned one.
__global__ __launch_bounds__(kBlock) void orswot_apply_kernel_a1024(OrswotApplyPlan p) {
  orswot_apply_body<16>(p);
}

// ---- Sixteen lanes per state (A <= 64) --------------------------------------------------------
// The wave-per-state kernel above spends a whole wave on ops that touch one cell: a one-member Add
// is a seen test, one cell read-modify-write and a clock word, so its wave issues ~70 instructions
// for one state's op (VALU ~20% busy, profiles/r02k_apply_sq_counters.json) and the kernel is
// bound by instruction issue.  Here a GROUP of 16 lanes runs one state's op stream (4 states per
// wave): lane g holds actors a = g + 16j (the clock in registers, rows read 128 contiguous bytes
// per group), a row operation costs each lane 4 words, a cell operation one lane.  (One lane per
// state was tried first: a Rm's row work then costs every lane 64 scattered words, 3.5x slower;
// 8 lanes per state held 157 VGPRs, 3 waves per SIMD.)
// apply_deferred without rescanning every slot on every Add (orswot.rs:281-286):
//  * keep test !(rm <= C): each slot keeps a WITNESS, the first actor with rm[a] > C[a] (an LDS
//    byte).  C only grows, so actors before the witness stay dominated and the witness only moves
//    forward: an Add to actor a re-examines only slots whose witness is a (W: bit a set iff some
//    slot's witness is a; exact for A <= 64), from a + 1 on; a slot left without one is dropped.
//  * re-forget: a slot's members were forgotten by its clock when it was created (apply_rm,
//    :230-250) or, for the input's slots, by the full pass at the first Add; forgets commute and
//    are idempotent, so an Add re-forgets only the cells it wrote, and only when one of its members
//    may be in a slot (bloom: bit m % 64 of the OR of every slot's member-bitmap words).
//  * identical clocks (HashMap keyed by VClock): the witness is a function of the clock (at the
//    current C), so a Rm's clock is compared in full only with slots of the same witness.
// Exact for ANY input state (the first Add re-forgets every input slot's members in full).
__device__ __forceinline__ void glds16_oa(const void *g, u64 *lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
}
constexpr int kG = grp::kG;            // lanes per state (group.hpp)
constexpr unsigned kGMask = grp::kMask;
constexpr int kJ = kWave / kG;         // actors per lane (A <= 64)
constexpr unsigned kNoWitness = grp::kNone;

__device__ __forceinline__ unsigned grp_bits(u64 ballot, int lane) { return grp::bits(ballot, lane); }
__device__ __forceinline__ bool grp_any(bool x, int lane) { return grp::any(x, lane); }
__device__ __forceinline__ bool grp_all(bool x, int lane) { return grp::all(x, lane); }
__device__ __forceinline__ u64 grp_or(u64 x) { return grp::orx(x); }
__device__ __forceinline__ unsigned grp_witness(const u64 (&x)[kJ], const u64 (&c)[kJ], int g, unsigned from,
                                                unsigned long long A) {
  return grp::witness<kJ>(x, c, g, from, A);
}
__device__ __forceinline__ void grp_load_row(u64 (&x)[kJ], const u64 *row, int g, unsigned long long A) {
  grp::load_row<kJ>(x, row, g, A);
}

// forget a member row by the rm clock in registers: keep e[a] iff e[a] > rm[a]
__device__ __forceinline__ void grp_forget_row(u64 *row, const u64 (&r)[kJ], int g, unsigned long long A) {
  u64 e[kJ];
  grp_load_row(e, row, g, A);
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const unsigned a = g + kG * j;
    if (a < A && e[j] != 0 && e[j] <= r[j]) row[a] = 0;
  }
}

// L2PF (round 5): a one-member Rm forgets its member's whole entry row, a dependent HBM round trip
// in the op loop (the Add's cell comes with the header; the Rm's 64-word row cannot be held per
// lane).  With p.l2pf the header lane of such an Rm loads one word of each 128-byte line of the row
// alongside the batch's other header loads; the XOR of those words goes into the Rm's unused cell
// field of the header (so the loads are kept, and waited for where the header is written), and the
// op's own row load later finds its lines in the cache.  Nothing reads the value.
__device__ __forceinline__ u64 touch_row(const u64 *row, unsigned long long A) {
  u64 x = 0;
#pragma unroll
  for (int j = 0; j < kWave / 16; ++j)
    if (16ull * j < A) x ^= row[16 * j];
  return x;
}

#ifndef CRDT_GRP_WPE
#define CRDT_GRP_WPE 4
#endif
// RPF (round 4): an Rm's clock row (the read-only rm pool) is loaded while the op before it runs,
// as the Map kernel does for its Put / rm clocks, so an Rm starts with its clock in registers.
// HPF (round 4): a batch header is three dependent round trips (kind / member range, then the
// first member / actor / counter, then a one-member Add's cell).  With HPF the next batch's kinds
// and member ranges are loaded at this batch's start and its first members at the middle op, so a
// batch boundary costs two round trips (actor / counter, then the cell).
// STG (round 5, opt-in: measured 2% slower, profiles/r05_oapply_stg_ab.log — the batch start's added
// wait costs more than the Rm round trips it removes): the clock rows of a batch's first STG Rm ops
// are moved into LDS by LDS-DMA with the
// batch's headers (issued before the one-member Adds' cell loads, whose wait then covers them), and
// an Rm reads its clock there: no dependent HBM round trip, no registers held across ops.  A DMA
// piece puts lane l's 16 bytes at byte 16 l of a 1-KiB block, so a group's 16 lanes fill its own
// quarter of each block: half a row (32 words) per block, 2 STG blocks per batch (A even, rm_clock
// 16-byte aligned; otherwise STG = 0).
// MT (round 5, default while Dcap <= kMetaSlots): per slot, next to its witness byte, the OR of the
// slot's member words in LDS — the bloom is rebuilt from LDS alone after a slot is dropped (no HBM
// read of every slot's member words) and an Add's re-forget tests a slot's LDS word before reading
// its member word.  At the apply bench's default mix, where the deferred slots cost ~40% of the
// kernel (profiles/r05_oapply_mix.log): 855 -> 808 us, no change without deferred removes.  Also the
// slot's rm counter at its witness (an Add to the witness actor tests it in LDS, not HBM; written by
// the lane that holds that actor, or read back by the group's first lane on the rare paths): 817 ->
// 813 us (profiles/r05_apply_witv_ab.log).  Measured and not kept (profiles/r05_oapply_meta_ab.log):
// that counter moved between lanes by shuffles plus a candidate-actor mask by ballots (an Add
// dropping a dominated slot without loading its row), and an Rm's same-clock filter on the counter:
// 969-1,055 us, and 705 vs 522 us without deferred removes at all — the cross-lane moves cost more in
// every op step than the HBM reads they remove.
constexpr unsigned long long kMetaSlots = 64;
#ifndef CRDT_OA_WITV
#define CRDT_OA_WITV 1  // (MT) the witness counter in LDS too (build option, for the A/B)
#endif
template <bool RPF, bool HPF, int STG = 0, bool MT = true>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(CRDT_GRP_WPE))) void orswot_apply_grp_kernel(
    OrswotApplyPlan p) {
  extern __shared__ u64 lds[];
  const int lane = (int)(threadIdx.x % kWave), g = lane & (kG - 1);
  const unsigned long long s = ((unsigned long long)blockIdx.x * kBlock + threadIdx.x) / kG;
  if (s >= p.N) return;  // (whole groups)
  const unsigned long long A = p.A, M = p.M, Mw = p.Mw, Dcap = p.Dcap;
  // LDS: per group the kG op headers of the current batch (32 bytes each), then the slot witnesses,
  // then (STG) per wave 2 STG blocks of 128 words, group q's words at 32 q .. 32 q + 31 of each
  u64 *hdr = lds + (threadIdx.x / kG) * (4 * kG);
  uint8_t *wit = reinterpret_cast<uint8_t *>(lds + (kBlock / kG) * 4 * kG) + (threadIdx.x / kG) * Dcap;
  const unsigned long long witw = ((kBlock / kG) * Dcap + 15) / 16 * 2;  // the witness bytes, in words
  u64 *sbl = lds + (kBlock / kG) * 4 * kG + witw + (threadIdx.x / kG) * 2 * Dcap;  // (MT) slot member blooms
  u64 *witv = sbl + Dcap;  // (MT) each slot's rm counter at its witness
  constexpr bool MB = MT, MW = MT && CRDT_OA_WITV;
  u64 *stg = lds + (kBlock / kG) * 4 * kG + witw + (MT ? (kBlock / kG) * 2 * Dcap : 0) + (threadIdx.x / kWave) * (2 * STG * 128);
  const unsigned gw32 = (unsigned)(lane / kG) * 32;  // the group's quarter of a block
  const bool lead = g == 0;

  const unsigned long long ob = p.op_off[s], oe = p.op_off[s + 1];
  unsigned dcnt = p.def_count[s];
  if (dcnt > Dcap || oe < ob || oe > p.n_ops) {
    if (lead) p.status[s] = (dcnt > Dcap ? 4u : 0u) | (oe < ob || oe > p.n_ops ? 8u : 0u);
    return;  // state left untouched
  }
  unsigned st = 0;
  u64 *C = p.clock + s * p.clock_stride;
  u64 *E = p.entries + s * p.entry_sstride;
  u64 *DC = p.def_clock + s * Dcap * A;
  u64 *DM = p.def_members + s * Dcap * Mw;
  u64 c[kJ];
  grp_load_row(c, C, g, A);

  // W (witness actors) and bloom (member bits mod 64) of the slots, identical in the group's lanes
  u64 W = 0, bloom = 0;
  auto rebuild = [&]() {
    W = 0;
    u64 b = 0;
    for (unsigned d = 0; d < dcnt; ++d) {
      const unsigned w = wit[d];
      if (w != kNoWitness) W |= 1ull << w;
      if (MB) b |= sbl[d];
      else
        for (unsigned long long x = g; x < Mw; x += kG) b |= DM[d * Mw + x];
    }
    bloom = MB ? b : grp_or(b);
  };
  for (unsigned d = 0; d < dcnt; ++d) {  // the input slots' witnesses at the input clock
    u64 x[kJ];
    grp_load_row(x, DC + d * A, g, A);
    const unsigned w = grp_witness(x, c, g, 0, A);
    if (lead) wit[d] = (uint8_t)w;
    if (MW && lead && w != kNoWitness) witv[d] = DC[d * A + w];
    if (MB) {
      u64 b = 0;
      for (unsigned long long y = g; y < Mw; y += kG) b |= DM[d * Mw + y];
      b = grp_or(b);
      if (lead) sbl[d] = b;
    }
  }
  rebuild();
  bool full = true;  // no Add yet: the input slots' members are re-forgotten in full at the first

  // drop slot d: the last slot moves over it
  auto drop = [&](unsigned d) {
    const unsigned last = dcnt - 1;
    if (d != last) {
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        const unsigned a = g + kG * j;
        if (a < A) DC[d * A + a] = DC[last * A + a];
      }
      for (unsigned long long x = g; x < Mw; x += kG) DM[d * Mw + x] = DM[last * Mw + x];
      if (lead) wit[d] = wit[last];
      if (MB && lead) {
        sbl[d] = sbl[last];
        if (MW) witv[d] = witv[last];
      }
    }
    dcnt = last;
    if (p.fence) wave_fence();  // (a wave's later loads see its earlier stores; afence=1 adds fences)
  };

  // Ops go in batches of kG: lane g loads op (base + g)'s header, first member and — for a
  // one-member Add — its cell, all at once; op i then reads them from lane i of the group.  A
  // prefetched cell is stale once an earlier op of the batch wrote that member's row (same first
  // member, any multi-member op, the full pass): `stale` marks those ops, which load it again.
  const int gb = lane & ~(kG - 1);
  // HPF: op (base + g)'s kind, member range and first member, loaded a batch ahead
  unsigned nx_kind = 0xFFu, nx_m0 = 0xFFFFFFFFu;
  u64 nx_mb = 0, nx_me = 0;
  auto pre_fields = [&](unsigned long long oo) {
    nx_kind = 0xFFu;
    if (oo < oe) {
      nx_kind = p.kind[oo];
      nx_mb = p.mem_off[oo];
      nx_me = p.mem_off[oo + 1];
    }
  };
  auto pre_member = [&]() {  // the first member of the op whose range is in nx_*
    nx_m0 = 0xFFFFFFFFu;
    if (nx_kind <= 1 && nx_me > nx_mb && nx_me <= p.n_mem) nx_m0 = p.mem[nx_mb];
  };
  if (HPF) {
    pre_fields(ob + g);
    pre_member();
  }
  for (unsigned long long base = ob; base < oe; base += kG) {
    const unsigned long long oo = base + g;
    unsigned h_ka = kBadOp, h_mb = 0, h_me = 0, h_m0 = 0xFFFFFFFFu;
    u64 h_cr = 0, h_cell = 0;
    if (HPF) {
      if (oo < oe) {  // the actor / counter / rm row now, with the range and member already here
        const u64 mb = nx_mb, me = nx_me;
        h_mb = (unsigned)mb;
        h_me = (unsigned)me;
        const bool range_ok = me >= mb && me <= 0xFFFFFFFFull && me <= p.n_mem;
        if (range_ok && nx_kind == 0) {
          const unsigned a = p.actor ? p.actor[oo] : 0u;
          h_ka = a < A ? a : kBadOp;
          h_cr = p.counter ? p.counter[oo] : 0ull;
          if (me > mb) h_m0 = nx_m0;
          if (h_ka != kBadOp && me - mb == 1 && h_m0 < M) h_cell = E[(unsigned long long)h_m0 * p.entry_mstride + a];
        } else if (range_ok && nx_kind == 1) {
          h_ka = kRmOp;
          h_cr = p.rm_row ? p.rm_row[oo] : 0u;
          if (me > mb) h_m0 = nx_m0;
          if (p.l2pf && me - mb == 1 && h_m0 < M) h_cell = touch_row(E + (unsigned long long)h_m0 * p.entry_mstride, A);
        }
      }
      pre_fields(oo + kG);  // the next batch's kind and range while this one runs
    } else if (oo < oe) {
      const unsigned kind = p.kind[oo];
      const u64 mb = p.mem_off[oo], me = p.mem_off[oo + 1];
      h_mb = (unsigned)mb;
      h_me = (unsigned)me;
      const bool range_ok = me >= mb && me <= 0xFFFFFFFFull && me <= p.n_mem;
      if (range_ok && kind == 0) {
        const unsigned a = p.actor ? p.actor[oo] : 0u;
        h_ka = a < A ? a : kBadOp;
        h_cr = p.counter ? p.counter[oo] : 0ull;
        if (me > mb) h_m0 = p.mem[mb];
        if (h_ka != kBadOp && me - mb == 1 && h_m0 < M) h_cell = E[(unsigned long long)h_m0 * p.entry_mstride + a];
      } else if (range_ok && kind == 1) {
        h_ka = kRmOp;
        h_cr = p.rm_row ? p.rm_row[oo] : 0u;
        if (me > mb) h_m0 = p.mem[mb];
        if (p.l2pf && me - mb == 1 && h_m0 < M) h_cell = touch_row(E + (unsigned long long)h_m0 * p.entry_mstride, A);
      }
    }
    const int nb = (int)((oe - base) < (unsigned long long)kG ? (oe - base) : kG);
    unsigned rmask = 0;  // (STG) the batch's valid Rm ops, bit i = op base + i (group-uniform)
    if constexpr (STG > 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last batch's staged rows are read
      rmask = grp_bits(__ballot(h_ka == kRmOp && h_cr < p.n_rm_rows), lane);
      unsigned m = rmask;
#pragma unroll
      for (int t = 0; t < STG; ++t) {
        const int pos = m ? __builtin_ctz(m) : 0;
        const u64 rr = __shfl(h_cr, gb | pos);  // the t-th Rm's rm row
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const unsigned long long w = 32ull * h + 2ull * g;
          if (m && w < A) glds16_oa(p.rm_clock + rr * A + w, stg + (2 * t + h) * 128);
        }
        m &= m ? m - 1 : 0u;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the rows (and the cells before them) landed
    }
    *reinterpret_cast<u64x2 *>(hdr + 4 * g) = u64x2{((u64)h_m0 << 32) | h_ka, ((u64)h_me << 32) | h_mb};
    *reinterpret_cast<u64x2 *>(hdr + 4 * g + 2) = u64x2{h_cr, h_cell};
    unsigned stale = 0;
    auto rm_row = [&](int i, u64 (&x)[kJ]) {  // op i's rm clock (0 unless a valid Rm)
      const unsigned ka = (unsigned)hdr[4 * i];
      const u64 rr = hdr[4 * i + 2];
      if (ka == kRmOp && rr < p.n_rm_rows) {
        grp_load_row(x, p.rm_clock + rr * A, g, A);
      } else {
#pragma unroll
        for (int j = 0; j < kJ; ++j) x[j] = 0;
      }
    };
    u64 rn[kJ];
    if (RPF) rm_row(0, rn);
    for (int i = 0; i < nb; ++i) {
      u64 rcur[kJ];
#pragma unroll
      for (int j = 0; j < kJ; ++j) rcur[j] = RPF ? rn[j] : 0ull;
      if (RPF && i + 1 < nb) rm_row(i + 1, rn);
      if (HPF && i == kG / 2) pre_member();
      // op i's header: two 16-byte LDS reads, the same address for the group's lanes
      const u64x2 h0 = *reinterpret_cast<const u64x2 *>(hdr + 4 * i);
      const u64x2 h1 = *reinterpret_cast<const u64x2 *>(hdr + 4 * i + 2);
      const unsigned ka = (unsigned)h0[0], m0 = (unsigned)(h0[0] >> 32);
      const u64 mb = (unsigned)h0[1], me = (unsigned)(h0[1] >> 32);
      const u64 cr = h1[0], cellv = h1[1];
      const bool one = me - mb == 1;
      // later ops of the batch whose first member this op may write
      const unsigned same = grp_bits(__ballot(h_m0 == m0), lane) & ~((2u << i) - 1);
      if (ka == kBadOp) {
        st |= 2u;
        continue;
      }
      if (ka != kRmOp) {  // ---- Op::Add (:57-72)
        const unsigned a = ka;
        const u64 k = cr;
        const unsigned ja = a / kG, ga = a % kG;
        u64 mine = c[0];
#pragma unroll
        for (int j = 1; j < kJ; ++j)
          if ((unsigned)j == ja) mine = c[j];
        const u64 ca = __shfl(mine, gb | (int)ga);
        if (ca >= k) continue;  // already seen (:60-63)
        if (one) {
          if (m0 >= M) {
            st |= 2u;
          } else if (lead) {
            u64 *cell = E + (unsigned long long)m0 * p.entry_mstride + a;
            const u64 old = ((stale >> i) & 1u) ? *cell : cellv;
            if (old < k) *cell = k;
          }
          stale |= same;
        } else {
          bool bad = false;
          for (u64 j = mb + g; j < me; j += kG) {
            const unsigned long long m = p.mem[j];
            if (m >= M) {
              bad = true;
              continue;
            }
            u64 *cell = E + m * p.entry_mstride + a;
            if (*cell < k) *cell = k;
          }
          if (grp_any(bad, lane)) st |= 2u;
          stale = kGMask;
          if (p.fence) wave_fence();  // cells written by other lanes of the group, read below
        }
        if ((unsigned)g == ga) {
#pragma unroll
          for (int j = 0; j < kJ; ++j)
            if ((unsigned)j == ja) c[j] = k;
        }
        // apply_deferred (:281-286)
        if (full) {  // every slot's members forgotten in full, every witness recomputed
          full = false;
          if (dcnt > 0) stale = kGMask;
          for (unsigned d = 0; d < dcnt;) {
            u64 rm[kJ];
            grp_load_row(rm, DC + d * A, g, A);
            for (unsigned long long x = 0; x < Mw; ++x) {
              u64 bits = DM[d * Mw + x];
              while (bits) {
                const unsigned long long m = x * 64 + __builtin_ctzll(bits);
                bits &= bits - 1;
                if (m < M) grp_forget_row(E + m * p.entry_mstride, rm, g, A);
              }
            }
            const unsigned w = grp_witness(rm, c, g, 0, A);
            if (w == kNoWitness) {
              drop(d);
            } else {
              if (lead) wit[d] = (uint8_t)w;
              if (MW && lead) witv[d] = DC[d * A + w];
              ++d;
            }
          }
          if (p.fence) wave_fence();
          rebuild();
          continue;
        }
        // the cells this Add wrote, re-forgotten by every slot naming their member
        if (dcnt > 0) {
          for (u64 j = mb; j < me; ++j) {
            const unsigned long long m = one ? m0 : p.mem[j];
            if (m >= M || !((bloom >> (m % 64)) & 1ull)) continue;
            for (unsigned d = 0; d < dcnt; ++d)
              if ((!MB || ((sbl[d] >> (m % 64)) & 1ull)) && ((DM[d * Mw + m / 64] >> (m % 64)) & 1ull)) {
                const u64 rv = DC[d * A + a];
                if (lead) {
                  u64 *cell = E + m * p.entry_mstride + a;
                  const u64 v = *cell;
                  if (v != 0 && v <= rv) *cell = 0;
                }
              }
          }
        }
        // the slots whose witness was actor a: move the witness on, drop a slot left without one
        if ((W >> a) & 1ull) {
          bool dropped = false;
          for (unsigned d = 0; d < dcnt;) {
            if (wit[d] == a && (MW ? witv[d] : DC[d * A + a]) <= k) {
              u64 x[kJ];
              grp_load_row(x, DC + d * A, g, A);
              const unsigned w = grp_witness(x, c, g, a + 1, A);
              if (w == kNoWitness) {
                drop(d);
                dropped = true;
                continue;
              }
              if (lead) wit[d] = (uint8_t)w;
              if (MW && lead) witv[d] = DC[d * A + w];  // (the row just loaded: a cache hit)
            }
            ++d;
          }
          if (dropped) {
            rebuild();
          } else {
            W = 0;
            for (unsigned d = 0; d < dcnt; ++d) {
              const unsigned w = wit[d];
              if (w != kNoWitness) W |= 1ull << w;
            }
          }
        }
      } else {  // ---- Op::Rm -> apply_rm (:230-250)
        const unsigned rr = (unsigned)cr;
        if (rr >= p.n_rm_rows) {
          st |= 2u;
          continue;
        }
        u64 r[kJ];
        const unsigned rank = STG > 0 ? (unsigned)__builtin_popcount(rmask & ((1u << i) - 1)) : 0u;
        if (STG > 0 && rank < (unsigned)STG) {  // staged with the batch (rmask bit i is set: a valid Rm)
#pragma unroll
          for (int j = 0; j < kJ; ++j) {
            const unsigned a = g + kG * j;
            r[j] = a < A ? stg[(2 * rank + (a >> 5)) * 128 + gw32 + (a & 31)] : 0ull;
          }
        } else if (RPF) {
#pragma unroll
          for (int j = 0; j < kJ; ++j) r[j] = rcur[j];
        } else {
          grp_load_row(r, p.rm_clock + (unsigned long long)rr * A, g, A);
        }
        if (one) {
          if (m0 >= M) st |= 2u;
          else grp_forget_row(E + (unsigned long long)m0 * p.entry_mstride, r, g, A);
          stale |= same;
        } else {
          for (u64 j = mb; j < me; ++j) {
            const unsigned long long m = p.mem[j];
            if (m >= M) {
              st |= 2u;
              continue;
            }
            grp_forget_row(E + m * p.entry_mstride, r, g, A);
          }
          stale = kGMask;
        }
        const unsigned wr = grp_witness(r, c, g, 0, A);
        if (wr == kNoWitness) continue;  // rm <= C: already seen (:239-249)
        int slot = -1;
        for (unsigned d = 0; d < dcnt; ++d) {
          if (wit[d] != wr) continue;
          u64 x[kJ];
          grp_load_row(x, DC + d * A, g, A);
          bool eq = true;
#pragma unroll
          for (int j = 0; j < kJ; ++j) eq &= x[j] == r[j];
          if (grp_all(eq, lane)) {
            slot = (int)d;
            break;
          }
        }
        if (slot < 0) {
          if (dcnt >= Dcap) {
            st |= 1u;  // deferred capacity exceeded: this state's result is incomplete
            continue;
          }
          slot = (int)dcnt++;
#pragma unroll
          for (int j = 0; j < kJ; ++j) {
            const unsigned a = g + kG * j;
            if (a < A) DC[slot * A + a] = r[j];
          }
          // a new slot's member words are written whole: a one-member Rm's bit goes in with the
          // zeros (no read-modify-write round trip behind the stores)
          const unsigned long long wm = one && m0 < M ? (unsigned long long)m0 / 64 : ~0ull;
          for (unsigned long long x = g; x < Mw; x += kG) DM[slot * Mw + x] = x == wm ? 1ull << (m0 % 64) : 0ull;
          if (lead) wit[slot] = (uint8_t)wr;
          if (MB && lead) sbl[slot] = one && m0 < M ? 1ull << (m0 % 64) : 0ull;
          if (MW && (unsigned)g == wr % kG) {  // the lane holding actor wr: no cross-lane move
            u64 v = r[0];
#pragma unroll
            for (int j = 1; j < kJ; ++j)
              if ((unsigned)j == wr / kG) v = r[j];
            witv[slot] = v;
          }
          W |= 1ull << wr;
          if (p.fence) wave_fence();  // the zeroed words are or-ed by the group's first lane below
          if (one) {
            if (m0 < M) bloom |= 1ull << (m0 % 64);
            if (p.fence) wave_fence();
            continue;
          }
        }
        for (u64 j = mb; j < me; ++j) {
          const unsigned long long m = one ? m0 : p.mem[j];
          if (m >= M) continue;
          if (lead) DM[slot * Mw + m / 64] |= 1ull << (m % 64);
          if (MB && lead) sbl[slot] |= 1ull << (m % 64);
          bloom |= 1ull << (m % 64);
        }
        if (p.fence) wave_fence();
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const unsigned a = g + kG * j;
    if (a < A) C[a] = c[j];
  }
  if (lead) {
    p.def_count[s] = dcnt;
    p.status[s] = st;
  }
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_orswot_apply_batch(crdt_ctx *ctx, const crdt_orswot_states *sv, const crdt_orswot_ops *ops,
                                       uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!sv || !ops || !status) return fail(ctx, CRDT_EINVAL, "orswot_apply_batch: NULL argument");
  const crdt_orswot_states &s = *sv;
  if (s.N == 0) return CRDT_OK;
  if (s.A == 0 || s.A > (size_t)kApplyMaxA)
    return fail(ctx, CRDT_EINVAL, "orswot_apply_batch: A = %zu outside 1..%d", s.A, kApplyMaxA);
  if (!s.clock || !s.entries || !s.def_count || !ops->op_off || !ops->mem_off || !status)
    return fail(ctx, CRDT_EINVAL, "orswot_apply_batch: NULL buffer");
  if (s.Dcap && (!s.def_clock || !s.def_members))
    return fail(ctx, CRDT_EINVAL, "orswot_apply_batch: deferred capacity without deferred buffers");
  if (ops->n_ops && (!ops->kind || !ops->mem))
    return fail(ctx, CRDT_EINVAL, "orswot_apply_batch: NULL op buffer");
  if (s.clock_stride < s.A || s.entry_mstride < s.A || s.entry_sstride < s.M * s.entry_mstride)
    return fail(ctx, CRDT_EINVAL, "orswot_apply_batch: strides smaller than the rows they hold");
  const size_t Mw = (s.M + 63) / 64;
  // hot deferred slots in LDS: as many as fit (wide member bitmaps leave fewer, down to none: every
  // slot then lives in the state's HBM slots, the same code path), so Dcap itself is not bounded
  const size_t lds_cap = 64 * 1024;
  size_t Dh = s.Dcap < (size_t)ctx->tune.apply_hot_slots ? s.Dcap : (size_t)ctx->tune.apply_hot_slots;
  const size_t slot_b = (s.A + Mw) * 8;
  if (Dh * slot_b > lds_cap) Dh = lds_cap / slot_b;
  const size_t per_wave = Dh * slot_b;
  int wpb = kBlock / kWave;
  while (wpb > 1 && per_wave * wpb > lds_cap) --wpb;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  OrswotApplyPlan p{(u64 *)s.clock, s.clock_stride, (u64 *)s.entries, s.entry_mstride, s.entry_sstride,
                    (u64 *)s.def_clock, (u64 *)s.def_members, s.def_count, s.N, s.M, s.A, Mw, s.Dcap, Dh,
                    (const u64 *)ops->op_off, ops->kind, ops->actor, (const u64 *)ops->counter, ops->rm_row,
                    (const u64 *)ops->rm_clock, ops->rm_clock ? ops->n_rm_rows : 0, (const u64 *)ops->mem_off,
                    ops->mem, ops->mem ? ops->n_mem : 0, ops->n_ops, status, wpb, ctx->tune.apply_fence,
                    ctx->tune.orswot_apply_l2pf};
  if (ctx->tune.apply_lane && s.A <= (size_t)kWave && s.Dcap <= 2048) {
    // kG lanes per state: kBlock / kG states per block, the slots' witness bytes in LDS
    timing_begin(ctx, "orswot_apply");
    const unsigned long long per_block = kBlock / kG;
    const dim3 grid((unsigned)((s.N + per_block - 1) / per_block));
    const bool rpf = ctx->tune.orswot_apply_pf, hpf = ctx->tune.orswot_apply_hpf;
    // STG: the batch's first 2 Rm clock rows by LDS-DMA (opt-in, CRDT_TUNE oastg=1)
    const bool stg = ctx->tune.orswot_apply_stg && !rpf && !hpf && s.A % 2 == 0 && ops->rm_clock &&
                     ((uintptr_t)ops->rm_clock & 15) == 0;
    // MT: the slots' member blooms in LDS (CRDT_TUNE oameta=0: the round-4 form, HBM only)
    // (the opt-in prefetch forms rpf / hpf keep the round-4 form)
    const bool mt = ctx->tune.orswot_apply_meta && s.Dcap <= kMetaSlots && !rpf && !hpf;
    const size_t lds = per_block * 4 * kG * 8 + (per_block * s.Dcap + 15) / 16 * 16 +
                       (mt ? per_block * 2 * s.Dcap * 8 : 0) + (stg ? (kBlock / kWave) * 2 * 2 * 128 * 8 : 0);
    if (stg && mt) hipLaunchKernelGGL((orswot_apply_grp_kernel<false, false, 2, true>), grid, dim3(kBlock), lds, ctx->stream, p);
    else if (stg) hipLaunchKernelGGL((orswot_apply_grp_kernel<false, false, 2, false>), grid, dim3(kBlock), lds, ctx->stream, p);
    else if (rpf && hpf) hipLaunchKernelGGL((orswot_apply_grp_kernel<true, true, 0, false>), grid, dim3(kBlock), lds, ctx->stream, p);
    else if (rpf) hipLaunchKernelGGL((orswot_apply_grp_kernel<true, false, 0, false>), grid, dim3(kBlock), lds, ctx->stream, p);
    else if (hpf) hipLaunchKernelGGL((orswot_apply_grp_kernel<false, true, 0, false>), grid, dim3(kBlock), lds, ctx->stream, p);
    else if (mt) hipLaunchKernelGGL((orswot_apply_grp_kernel<false, false, 0, true>), grid, dim3(kBlock), lds, ctx->stream, p);
    else hipLaunchKernelGGL((orswot_apply_grp_kernel<false, false, 0, false>), grid, dim3(kBlock), lds, ctx->stream, p);
    timing_end(ctx);
    CRDT_HIP(ctx, hipGetLastError());
    return CRDT_OK;
  }
  const unsigned long long want = (s.N + wpb - 1) / wpb;
  const unsigned long long cap = (unsigned long long)ctx->cu_count * 64;
  timing_begin(ctx, "orswot_apply");
  const dim3 grid((unsigned)(want < cap ? want : cap)), block(wpb * kWave);
  if (s.A <= (size_t)kWave)
    hipLaunchKernelGGL(orswot_apply_kernel_a64, grid, block, per_wave * wpb, ctx->stream, p);
  else if (s.A <= (size_t)(kCAMax * kWave))
    hipLaunchKernelGGL(orswot_apply_kernel_a256, grid, block, per_wave * wpb, ctx->stream, p);
  else
    hipLaunchKernelGGL(orswot_apply_kernel_a1024, grid, block, per_wave * wpb, ctx->stream, p);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}
