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
// and the replica clock) is staged chunk by chunk through a per-wave LDS double buffer; the
// MVReg lives in fixed register slots (MVState).
//
// Per step i with e = acc entry clock, e2 = replica entry clock, Co = replica clock:
//   acc only      (:146-161): Co >= e ? drop : e = e>Co?e:0, vals.forget(Co>e?Co:0)
//   replica only  (:193-208): Cs >= e2 ? skip : e = e2>Cs?e2:0, vals = vals2.forget(Cs>e?Cs:0)
//   both          (:170-192): common = max(e==e2?e:0, e2>Cs?e2:0, e>Co?e:0); empty ? drop :
//                             vals = mvreg_merge(vals, vals2).forget(max(e,e2) > common ? max : 0),
//                             e = common
//   then the deferred ceiling forgets the entry (and drops it when its clock empties).
#include <type_traits>

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
  unsigned *o_flags;  // per group: bit0 > Vout values, bit1 bad def_row, bit2 state capacity,
                      // bit3 SH ring arrival wait past its bound (internal fault)
  int spec;           // speculative no-op scan on (tuning / diagnosis knob; results are identical)
  int nt;             // LDS-DMA step images with the non-temporal policy (tuning knob)
  int scan2;          // speculative scan with two actors per 16-byte LDS read (A even)
  int scan3;          // speculative scan from per-actor thresholds, every LDS read issued first
  // LDS-DMA path: per (group, chunk of C replicas) the max of the chunk's replica clocks,
  // [G][nch][A] (map_chunk_max_kernel), staged with each chunk so a wholly skipped chunk merges
  // its clocks with one compare (the acc clock only ever takes maxima of replica clocks, map.rs:217)
  const u64 *cmax;
  unsigned long long nch;
  int batch;  // RS chunk test: compares batched ahead of their scalar ANDs (1) or interleaved (0)
  int lazyv;  // RS path: the values of a chunk fetched only when the exact loop runs it
  int diag;   // timing probes (results wrong): bit0 no clock-max piece, bit1 3 fewer step pieces,
              // bit2 SH path without arrival waits
  int st;  // ST path (A = 32, V = 2 on the RS shapes): two waves per key, each testing 8 steps of a chunk
};

constexpr int kMapQ = 4;    // deferred removes tracked per key in registers before the slow path
// MAP_RS_WS8 (build option): the RS / ST step images at a stride of 8 (mod 32) words instead of 4, which
// makes the register test's 16-byte reloads (lane (s, gq), steps 0/3/5/6 and 1/2/4/7 in one LDS lane
// group) bank-conflict free; the remove list shrinks to 128 entries to keep 4 key waves per CU.
// MAP_RS_NT (build option, default 1 since round 6): the RS / ST LDS-DMA with the non-temporal policy
// (aux = 2) — each step image is read once, and keeping it out of the caches' LRU measured 2.175 ms
// against 2.24 ms at config 4 (profiles/r06_map_ab2.log); 0 restores the default policy.
#ifndef MAP_RS_WS8
#define MAP_RS_WS8 0
#endif
#ifndef MAP_RS_NT
#define MAP_RS_NT 1
#endif
#ifndef MAP_RS_AUX  // the policy bits themselves (2 = nt; 16 = sc1, 18 = sc1 nt: A/B options)
#define MAP_RS_AUX (MAP_RS_NT ? 2 : 0)
#endif
// MAP_RS_LATE (build option, round 6, off): with the next chunk's pieces spread through the register
// test, the slot's reload is no longer waited for in full before the test — the wait moves into the DMA
// hook (before piece 0, which overwrites step 0's image) and every element's two pieces issue after
// that element's compares, so element 0's compares run while the later reads land.  Parity green, but
// 2.188 / 2.209 ms against 2.166 / 2.171 ms for the default, interleaved on one box
// (profiles/r06_map_late_ab.log): the later DMA issue costs more than the overlap gains.
#ifndef MAP_RS_LATE
#define MAP_RS_LATE 0
#endif
constexpr int kMapL = MAP_RS_WS8 ? 128 : 256;  // removes naming one key listed in LDS (beyond: walk the group list)

template <int APL, int VI>
struct MapStep {
  u64 e[APL];
  u64 c[VI][APL];
  u64 co[APL];
  u64 v[VI];
};

// Wave votes as ballots: the results are provably uniform (scalar registers), so the control
// flow built on them stays scalar — no EXEC-masked regions, no divergent loops whose live-outs
// the compiler would have to move to vector registers.
__device__ __forceinline__ bool wall(bool x) { return __ballot(!x) == 0; }
// A wave-uniform condition the compiler cannot prove uniform: make it so.
__device__ __forceinline__ bool uni(bool x) { return __builtin_amdgcn_readfirstlane((int)x) != 0; }
__device__ __forceinline__ bool wany(bool x) { return __ballot(x) != 0; }

template <int APL>
__device__ __forceinline__ bool all_ge(const u64 (&x)[APL], const u64 (&y)[APL]) {
  bool t = true;
#pragma unroll
  for (int j = 0; j < APL; ++j) t &= x[j] >= y[j];
  return wall(t);
}
template <int APL>
__device__ __forceinline__ bool all_eq(const u64 (&x)[APL], const u64 (&y)[APL]) {
  bool t = true;
#pragma unroll
  for (int j = 0; j < APL; ++j) t &= x[j] == y[j];
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

// The MVReg of one key: VO slots (clocks per lane, values / order keys wave-uniform), a valid
// mask, and the next order key.  The Vec order (mvreg.rs:34) only decides the output order, so
// values never move when others are dropped: an appended value takes a free slot and the next
// order key, and egress writes the slots in key order.
template <int APL, int VO>
struct MVState {
  u64 c[VO][APL];
  u64 v[VO];
  u64 seq[VO];
  unsigned vm;
  u64 next;
};

// vals.forget(X) (mvreg.rs:88-104): forget every value clock, drop the emptied ones.
template <int APL, int VO>
__device__ __forceinline__ void mv_forget(MVState<APL, VO> &s, const u64 (&X)[APL]) {
#pragma unroll
  for (int q = 0; q < VO; ++q)
    if (s.vm & (1u << q)) {
      vforget(s.c[q], X);
      if (!any_nz(s.c[q])) s.vm &= ~(1u << q);
    }
}

// Append (x, val) at the end of the Vec order, in the first free slot.
template <int APL, int VO>
__device__ __forceinline__ void mv_append(MVState<APL, VO> &s, const u64 (&x)[APL], u64 val, int &ovf) {
  const unsigned freem = ~s.vm & ((1u << VO) - 1u);
  if (freem == 0) {
    ovf |= 4;  // the fold state itself ran out of value slots (results incomplete)
    return;
  }
  const int q0 = __builtin_ctz(freem);
#pragma unroll
  for (int q = 0; q < VO; ++q)
    if (q == q0) {
#pragma unroll
      for (int j = 0; j < APL; ++j) s.c[q][j] = x[j];
      s.v[q] = val;
      s.seq[q] = s.next;
    }
  s.next++;
  s.vm |= 1u << q0;
}

// Replica stream staging.  The fold reads its steps from a per-wave LDS ring of NB chunk slots
// of C replicas (dynamic index, no unrolled register ring).  LDS step image, W = (2+VI)*A words:
//   [0, A) entry clock | [(1+t)A, (2+t)A) value clock t < VI | [(1+VI)A, (2+VI)A) replica clock
// and, in a separate per-slot array, the VI values of each step.
// Two ways to fill a slot:
//  * LDS-DMA (map_chunk_glds, A <= 64 even, VI = V, 16-byte aligned rows): global_load_lds
//    writes each step image straight into its slot (no VGPRs held by loads in flight), NB-1
//    chunks ahead; the fold waits for a chunk with a counted vmcnt.
//  * register staging (map_chunk_load / map_chunk_store, any shape): a chunk is loaded into
//    registers (every load in flight at once) and written to the other slot of a double buffer
//    while the fold runs over the current one.
template <int APL, int VI, int CM>
struct MapChunk {
  static constexpr int words = (2 + VI) * APL + 1;  // u64 registers per staged replica per lane
  static constexpr int raw = (APL >= 4 ? 48 : 96) / words;
  static constexpr int C0 = raw > 16 ? 16 : (raw < 2 ? 2 : raw);
  static constexpr int C = C0 > CM ? CM : C0;
  u64 e[C][APL];
  u64 c[C][VI][APL];
  u64 co[C][APL];
  u64 v[C];  // lane t < VI holds value slot t
};

template <int APL, int VI, int CM>
__device__ __forceinline__ void map_chunk_load(MapChunk<APL, VI, CM> &r, const MapPlan &p,
                                               unsigned long long g, unsigned long long k,
                                               unsigned long long i0, unsigned long long iend,
                                               int lane) {
  constexpr int C = MapChunk<APL, VI, CM>::C;
#pragma unroll
  for (int s = 0; s < C; ++s) {
    const unsigned long long i = i0 + s;
    if (i < iend) {
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

template <int APL, int VI, int CM>
__device__ __forceinline__ void map_chunk_store(const MapChunk<APL, VI, CM> &r, u64 *buf, u64 *vals,
                                                unsigned long long A, unsigned long long W,
                                                unsigned long long nsteps, int lane) {
  constexpr int C = MapChunk<APL, VI, CM>::C;
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
      if (lane < VI) vals[s * VI + lane] = r.v[s];
    }
  }
}

// LDS stride of a staged step image: W words padded to 4 (mod 32), so the steps the scan reads
// side by side start 8 banks apart instead of on the same bank.
__host__ __device__ __forceinline__ unsigned long long map_ws(unsigned long long W) {
  return W + (36 - W % 32) % 32;
}
// The RS / ST step stride (MAP_RS_WS8: 8 mod 32 words).
__host__ __device__ __forceinline__ unsigned long long map_ws_rs(unsigned long long W) {
  return MAP_RS_WS8 ? W + (40 - W % 32) % 32 : map_ws(W);
}

// AUX = the cache-policy bits of the load (0: default; 2: non-temporal, the streamed step images)
template <int AUX = 0>
__device__ __forceinline__ void glds16(const void *g, u64 *lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)lds, 16, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void glds4(const void *g, u64 *lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)lds, 4, 0, AUX);
}

// Per-lane source of the LDS-DMA pieces: piece j of a step image covers image words
// [j*128, j*128+128); lane l moves words o = j*128 + 2l, 2l+1 of replica i from
// src0[j] + i * stride[j] bytes (entry clock, value clock or replica clock row).  Computed once.
template <int NI>
struct GldsLanes {
  const char *src0[NI];
  unsigned long long stride[NI];
  bool on[NI];
};

template <int VI, int NI>
__device__ __forceinline__ GldsLanes<NI> glds_lanes(const MapPlan &p, unsigned long long g, unsigned long long k,
                                                    int lane) {
  GldsLanes<NI> L;
  const unsigned long long A = p.A, W = (2 + VI) * A;
  // the three row sources as values first: a per-lane choice between struct FIELDS would be
  // lowered as a dynamic-offset load, which forces the whole plan into scratch memory
  const unsigned long long be = (unsigned long long)(p.ec + g * p.e_gs + k * A);
  const unsigned long long bv = (unsigned long long)(p.vclk + g * p.vc_gs + k * VI * A);
  const unsigned long long bc = (unsigned long long)(p.clock + g * p.c_gs);
  const unsigned long long se = (unsigned long long)p.e_rs * 8, sv = (unsigned long long)p.vc_rs * 8,
                           sc = (unsigned long long)p.c_rs * 8;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const unsigned long long o = (unsigned long long)(j * 64 + lane) * 2;
    L.on[j] = o < W;
    const bool ie = o < A, iv = !ie && o < (1 + VI) * A;
    const unsigned long long off = ie ? o : (iv ? o - A : (o < W ? o - (1 + VI) * A : 0));
    const unsigned long long base = ie ? be : (iv ? bv : bc);
    L.src0[j] = reinterpret_cast<const char *>(base + off * 8);
    L.stride[j] = ie ? se : (iv ? sv : sc);
  }
  return L;
}

// DMA one chunk (steps i0 .. i0+C-1, clamped to iend-1: past the end a slot holds copies that
// are never read) into an LDS slot.  Exactly C*NI + 2 global_load_lds per call, each with at
// least one active lane (NI = ceil(W / 128) 1-KiB pieces per step image; the values of all C
// steps in one 4-byte-per-lane piece; the chunk's clock max in one), so a fixed vmcnt count
// retires a chunk.  Sources advance by their row stride (no per-step 64-bit multiply).
template <int VI, int C, int NI, int AUX = 0>
__device__ __forceinline__ void map_chunk_glds(const MapPlan &p, const GldsLanes<NI> &L, unsigned long long g,
                                               unsigned long long k, unsigned long long i0, unsigned long long iend,
                                               u64 *img, unsigned long long WS, u64 *vals, u64 *cm, int lane,
                                               bool vpiece = true, int diag = 0) {
  if (i0 + C <= iend) {  // a whole chunk (uniform)
    const char *src[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) src[j] = L.src0[j] + i0 * L.stride[j];
    if ((2 + VI) * p.A == NI * 128) {  // every lane moves a piece: no EXEC-masked regions
#pragma unroll
      for (int s = 0; s < C; ++s)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          if (!(diag & 2) || s < C - 3) glds16<AUX>(src[j], img + s * WS + j * 128);
          src[j] += L.stride[j];
        }
    } else {
#pragma unroll
      for (int s = 0; s < C; ++s)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          if (L.on[j]) glds16<AUX>(src[j], img + s * WS + j * 128);
          src[j] += L.stride[j];
        }
    }
  } else {
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const unsigned long long i = i0 + s < iend ? i0 + s : iend - 1;
#pragma unroll
      for (int j = 0; j < NI; ++j)
        if (L.on[j]) glds16<AUX>(L.src0[j] + i * L.stride[j], img + s * WS + j * 128);
    }
  }
  const int sv = lane / (2 * VI), dw = lane % (2 * VI);
  if (vpiece) {  // (uniform)
    if (sv < C) {
      const unsigned long long i = i0 + sv < iend ? i0 + sv : iend - 1;
      const unsigned *src = reinterpret_cast<const unsigned *>(p.vval + g * p.vv_gs + i * p.vv_rs + k * VI) + dw;
      glds4<AUX>(src, vals);
    }
  }
  // the chunk's clock max: one more piece (lanes 0 .. A/2-1, A even)
  if (!(diag & 1)) {
    if ((unsigned long long)(2 * lane) < p.A) glds16(p.cmax + (g * p.nch + i0 / C) * p.A + 2 * lane, cm);
  }
}

// Wait until at most N vector-memory ops are outstanding (counts above the 6-bit field clamp
// to 63: waiting for more than needed is safe).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N > 63 ? 63 : N) : "memory");
}

template <int APL, int VI>
__device__ __forceinline__ MapStep<APL, VI> map_step_read(const u64 *st, const u64 *vals,
                                                          unsigned long long A, int lane) {
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
  for (int t = 0; t < VI; ++t) in.v[t] = vals[t];
  return in;
}

// Speculative no-op scan over the steps of a staged chunk (A <= 64).  The wave checks NS steps
// at once: lane (s, g) = (lane / LPS, lane % LPS), LPS = 64 / NS, checks step s on actors g,
// g+LPS, ... against the CURRENT fold state, mirrored in LDS (me = entry clock, mc = value
// clocks, vm = valid slots, mmx = max(entry clock, acc clock Cs)); the LPS lanes of a step are
// combined bitwise on the ballot masks.  Bit LPS*s of the result is set only if step s provably leaves (present, e,
// vals) unchanged.  With e = acc entry clock, e2 / c2[t] / Co = the replica's entry clock /
// value clocks / clock, and Cs' >= Cs the acc clock at step s (so e2 <= Cs implies e2 <= Cs'):
//   present, replica has the key (map.rs:170-192): common = max(e==e2?e:0, e2>Cs'?e2:0,
//     e>Co?e:0) equals e if every actor has (e == 0 | e == e2 | e > Co) and e2 <= max(e, Cs);
//     then deleted = (e2 > e ? e2 : 0).  The MVReg is unchanged if (a) the own values are an
//     antichain (the caller only scans then), (b) forget(deleted) changes no own value clock
//     (no actor with 0 < x <= deleted), and (c) every incoming value is <= an own one (not
//     appended, mvreg.rs:120-126) or forgotten to empty by deleted (appended, then dropped:
//     only the Vec order key counter moves).  No own value is dropped by the merge then
//     (mvreg.rs:114-118): own < incoming t <= own' contradicts (a); own < t with t <= deleted
//     means own <= deleted, which (b) excludes for a non-empty clock;
//   present, replica lacks the key (:146-161): e[a] == 0 | e[a] > Co[a] (e survives the forget)
//     and no value clock changes under forget(Co > e ? Co : 0);
//   absent, replica has the key (:193-197): e2 <= Cs (seen and dropped);
//   absent, replica lacks the key: always.
// The deferred forget of such a step is the identity too: the state was forgotten by the max
// of the active removes at the last exact step, the active set only shrinks until the next
// activation (scans stop there), and forget(x) of a state already forgotten by y >= x is the
// identity (vclock.rs:98-104).
// Most steps of a fold change nothing, so their cost drops from a full exact step to a share
// of this wave-wide scan: per actor and step one vector compare and one scalar mask op per
// test, all LDS reads unpredicated.
template <int LPS>
__device__ __forceinline__ u64 grp_mask() {
  u64 m = 0;
#pragma unroll
  for (int b = 0; b < 64; b += LPS) m |= 1ull << b;
  return m;
}
template <int LPS>
__device__ __forceinline__ u64 andN(u64 m) {  // bit LPS*s: AND of the LPS bits of step s
#pragma unroll
  for (int sh = 1; sh < LPS; sh <<= 1) m &= m >> sh;
  return m & grp_mask<LPS>();
}
template <int LPS>
__device__ __forceinline__ u64 orN(u64 m) {
#pragma unroll
  for (int sh = 1; sh < LPS; sh <<= 1) m |= m >> sh;
  return m & grp_mask<LPS>();
}

template <int VI, int NQ, int LPS, int IT, bool PRESENT>
__device__ __forceinline__ u64 map_noop_steps(const u64 *buf, unsigned W, unsigned A, const u64 *me,
                                              const u64 *mc, const u64 *mmx, unsigned n, int lane) {
  // NQ = the number of own values, compacted into mirror slots 0..NQ-1 (PRESENT only)
  const unsigned st = (unsigned)lane / LPS;
  const unsigned gq = (unsigned)lane % LPS;
  const u64 *stp = buf + (st < n ? st : n - 1) * W;
  // Tests ANDed into the same verdict share one accumulator (andN(x) & andN(y) = andN(x & y)):
  // mB for "replica has the key", mO for "replica lacks it"; the value-cover tests are ORed over
  // own values after andN, so each keeps its own.
  u64 mP2 = 0, mB = ~0ull, mO = ~0ull;
  u64 mLe2[VI][NQ > 0 ? NQ : 1], mVan[VI];
#pragma unroll
  for (int t = 0; t < VI; ++t) {
    mVan[t] = ~0ull;
#pragma unroll
    for (int q = 0; q < NQ; ++q) mLe2[t][q] = ~0ull;
  }
  // IT >= ceil(A / LPS) iterations, fully unrolled: every LDS read of the scan can be in
  // flight at once.  Lanes past the last actor re-read actor A-1 of their own step: every test
  // bit is a function of (step, actor) alone and the masks are only ANDed / ORed, so a duplicate
  // is neutral and no range mask is needed.
#pragma unroll
  for (unsigned m = 0; m < IT; ++m) {
    const unsigned a0 = gq + LPS * m;
    const unsigned a = a0 < A ? a0 : A - 1;
    const u64 e2 = stp[a];
    const u64 mx = mmx[a];  // max(e, Cs); = Cs when absent (e == 0 then)
    // one vector compare per test, combined on the (scalar) ballot masks
    if constexpr (!PRESENT) {
      mP2 |= __ballot(e2 != 0);
      mB &= __ballot(e2 <= mx);
    } else {
      const u64 co = stp[(1 + VI) * A + a];
      const u64 ea = me[a];
      u64 c2[VI], sq[NQ > 0 ? NQ : 1], sq1[NQ > 0 ? NQ : 1];
#pragma unroll
      for (int t = 0; t < VI; ++t) c2[t] = stp[(1 + t) * A + a];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        sq[q] = mc[q * A + a];
        sq1[q] = sq[q] - 1;  // x - 1 >= y <=> x == 0 | x > y (wrapping)
      }
      const u64 eGtCo = __ballot(ea - 1 >= co);  // ea == 0 | ea > co
      const u64 del = e2 > ea ? e2 : 0;          // deleted
      mP2 |= __ballot(e2 != 0);
      mB &= __ballot(e2 <= mx) & (eGtCo | __ballot(ea == e2));
      mO &= eGtCo;
#pragma unroll
      for (int t = 0; t < VI; ++t) mVan[t] &= __ballot(c2[t] <= del);  // appended, forgotten to empty
      if constexpr (NQ > 0) {
        const u64 ri = co > ea ? co : 0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          mO &= __ballot(sq1[q] >= ri);   // sq == 0 | sq > ri
          mB &= __ballot(sq1[q] >= del);  // sq == 0 | sq > deleted
#pragma unroll
          for (int t = 0; t < VI; ++t) mLe2[t][q] &= __ballot(c2[t] <= sq[q]);
        }
      }
    }
  }
  const u64 G1 = grp_mask<LPS>();
  const u64 P2 = orN<LPS>(mP2);
  if constexpr (!PRESENT) return (~P2 | andN<LPS>(mB)) & G1;
  u64 both = P2 & andN<LPS>(mB);
  const u64 only = ~P2 & andN<LPS>(mO);
#pragma unroll
  for (int t = 0; t < VI; ++t) {
    u64 cov = andN<LPS>(mVan[t]);  // appended, then forgotten to empty
#pragma unroll
    for (int q = 0; q < NQ; ++q) cov |= andN<LPS>(mLe2[t][q]);
    both &= cov;
  }
  return (both | only) & G1;
}

// The same scan with two adjacent actors per lane and read (A even): every operand is one 16-byte
// LDS read (ds_read_b128) covering actors a, a+1, and the two actors' tests are combined per lane
// before the ballot (AND for the all-actor tests, OR for "replica has the key"), so the scan
// issues half the LDS reads and half the ballots of map_noop_steps for the same verdict.
__device__ __forceinline__ u64x2 lds2(const u64 *p) { return *reinterpret_cast<const u64x2 *>(p); }

template <int VI, int NQ, int LPS, int IT, bool PRESENT>
__device__ __forceinline__ u64 map_noop_steps2(const u64 *buf, unsigned W, unsigned A, const u64 *me,
                                               const u64 *mc, const u64 *mmx, unsigned n, int lane) {
  const unsigned st = (unsigned)lane / LPS;
  const unsigned gq = (unsigned)lane % LPS;
  const u64 *stp = buf + (st < n ? st : n - 1) * W;
  u64 mP2 = 0, mB = ~0ull, mO = ~0ull;
  u64 mLe2[VI][NQ > 0 ? NQ : 1], mVan[VI];
#pragma unroll
  for (int t = 0; t < VI; ++t) {
    mVan[t] = ~0ull;
#pragma unroll
    for (int q = 0; q < NQ; ++q) mLe2[t][q] = ~0ull;
  }
  constexpr int IT2 = (IT + 1) / 2;
#pragma unroll
  for (unsigned m = 0; m < IT2; ++m) {
    const unsigned a0 = 2 * (gq + LPS * m);
    const unsigned a = a0 < A ? a0 : A - 2;  // a duplicate pair is neutral (masks only AND / OR)
    const u64x2 e2 = lds2(stp + a);
    const u64x2 mx = lds2(mmx + a);
    if constexpr (!PRESENT) {
      mP2 |= __ballot((e2.x != 0) | (e2.y != 0));
      mB &= __ballot((e2.x <= mx.x) & (e2.y <= mx.y));
    } else {
      const u64x2 co = lds2(stp + (1 + VI) * A + a);
      const u64x2 ea = lds2(me + a);
      u64x2 c2[VI], sq[NQ > 0 ? NQ : 1];
#pragma unroll
      for (int t = 0; t < VI; ++t) c2[t] = lds2(stp + (1 + t) * A + a);
#pragma unroll
      for (int q = 0; q < NQ; ++q) sq[q] = lds2(mc + q * A + a);
      const bool gx = ea.x - 1 >= co.x, gy = ea.y - 1 >= co.y;  // e == 0 | e > Co
      const u64 eGtCo = __ballot(gx & gy);
      const u64 dx = e2.x > ea.x ? e2.x : 0, dy = e2.y > ea.y ? e2.y : 0;  // deleted
      mP2 |= __ballot((e2.x != 0) | (e2.y != 0));
      mB &= __ballot((e2.x <= mx.x) & (e2.y <= mx.y) & (gx | (ea.x == e2.x)) & (gy | (ea.y == e2.y)));
      mO &= eGtCo;
#pragma unroll
      for (int t = 0; t < VI; ++t) mVan[t] &= __ballot((c2[t].x <= dx) & (c2[t].y <= dy));
      if constexpr (NQ > 0) {
        const u64 rx = co.x > ea.x ? co.x : 0, ry = co.y > ea.y ? co.y : 0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const u64 sx = sq[q].x - 1, sy = sq[q].y - 1;  // x - 1 >= y <=> x == 0 | x > y
          mO &= __ballot((sx >= rx) & (sy >= ry));
          mB &= __ballot((sx >= dx) & (sy >= dy));
#pragma unroll
          for (int t = 0; t < VI; ++t) mLe2[t][q] &= __ballot((c2[t].x <= sq[q].x) & (c2[t].y <= sq[q].y));
        }
      }
    }
  }
  const u64 G1 = grp_mask<LPS>();
  const u64 P2 = orN<LPS>(mP2);
  if constexpr (!PRESENT) return (~P2 | andN<LPS>(mB)) & G1;
  u64 both = P2 & andN<LPS>(mB);
  const u64 only = ~P2 & andN<LPS>(mO);
#pragma unroll
  for (int t = 0; t < VI; ++t) {
    u64 cov = andN<LPS>(mVan[t]);
#pragma unroll
    for (int q = 0; q < NQ; ++q) cov |= andN<LPS>(mLe2[t][q]);
    both &= cov;
  }
  return (both | only) & G1;
}

// The same verdict from per-actor thresholds the fold keeps beside the mirror (thr = [TB | TO],
// A words each, rewritten after every exact step and every skip), with every LDS read of the scan
// issued before the first compare.  With m1 = (min of the nonzero own value clocks) - 1, or
// UINT64_MAX when none is nonzero, "sq == 0 | sq > x for every own value" is x <= m1, so
//   both:  e2 <= max(e, Cs) and (every sq == 0 | sq > deleted)  <=>  e2 <= TB = max(e, min(Cs, m1))
//          (deleted = e2 > e ? e2 : 0 is <= m1 iff e2 <= e or e2 <= m1)
//   only:  (e == 0 | e > Co) and (every sq == 0 | sq > ri)       <=>  Co <= TO = e > 0 ? e - 1 : m1
//          (e > 0: Co < e, then ri = 0; e == 0: ri = Co)
// (tests/test_map_scan_model.py checks both forms give the same verdict.)  The compares per
// (step, actor) drop from 5 + 2 NQ + VI NQ + VI to 5 + VI NQ + VI, and none of them waits on an LDS
// read issued in the same iteration: one wave per SIMD has no other wave to hide that latency.
template <int VI, int NQ, int LPS, int IT, bool PRESENT>
__device__ __forceinline__ u64 map_noop_steps3(const u64 *buf, unsigned W, unsigned A, const u64 *me,
                                               const u64 *mc, const u64 *thr, unsigned n, int lane) {
  const unsigned st = (unsigned)lane / LPS;
  const unsigned gq = (unsigned)lane % LPS;
  const u64 *stp = buf + (st < n ? st : n - 1) * W;
  constexpr int NQ1 = NQ > 0 ? NQ : 1;
  // batches of IB iterations (all of them up to 8; 4 at a time beyond, so the loads in flight fit)
  constexpr int IB = IT <= 8 ? IT : 4;
  u64 mP2 = 0, mB = ~0ull, mO = ~0ull;
  u64 mLe2[VI][NQ1], mVan[VI];
#pragma unroll
  for (int t = 0; t < VI; ++t) {
    mVan[t] = ~0ull;
#pragma unroll
    for (int q = 0; q < NQ1; ++q) mLe2[t][q] = ~0ull;
  }
#pragma unroll
  for (int b = 0; b < IT; b += IB) {
  u64 e2[IB], tb[IB], co[IB], to[IB], ea[IB], c2[VI][IB], sq[NQ1][IB];
#pragma unroll
  for (int m = 0; m < IB; ++m) {
    const unsigned a0 = gq + LPS * (b + m);
    const unsigned a = a0 < A ? a0 : A - 1;  // a duplicate actor is neutral (masks only AND / OR)
    e2[m] = stp[a];
    tb[m] = thr[a];
    if constexpr (PRESENT) {
      co[m] = stp[(1 + VI) * A + a];
      to[m] = thr[A + a];
      ea[m] = me[a];
#pragma unroll
      for (int t = 0; t < VI; ++t) c2[t][m] = stp[(1 + t) * A + a];
#pragma unroll
      for (int q = 0; q < NQ; ++q) sq[q][m] = mc[q * A + a];
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // every read above is in flight before the first compare
#pragma unroll
  for (int m = 0; m < IB; ++m) {
    mP2 |= __ballot(e2[m] != 0);
    if constexpr (!PRESENT) {
      mB &= __ballot(e2[m] <= tb[m]);
    } else {
      // e == 0 | e > Co | e == e2  (e - 1 wraps to UINT64_MAX at e == 0)
      mB &= __ballot((e2[m] <= tb[m]) & ((ea[m] - 1 >= co[m]) | (ea[m] == e2[m])));
      mO &= __ballot(co[m] <= to[m]);
      const u64 del = e2[m] > ea[m] ? e2[m] : 0;
#pragma unroll
      for (int t = 0; t < VI; ++t) {
        mVan[t] &= __ballot(c2[t][m] <= del);  // appended, then forgotten to empty
#pragma unroll
        for (int q = 0; q < NQ; ++q) mLe2[t][q] &= __ballot(c2[t][m] <= sq[q][m]);
      }
    }
  }
  }
  const u64 G1 = grp_mask<LPS>();
  const u64 P2 = orN<LPS>(mP2);
  if constexpr (!PRESENT) return (~P2 | andN<LPS>(mB)) & G1;
  u64 both = P2 & andN<LPS>(mB);
  const u64 only = ~P2 & andN<LPS>(mO);
#pragma unroll
  for (int t = 0; t < VI; ++t) {
    u64 cov = andN<LPS>(mVan[t]);
#pragma unroll
    for (int q = 0; q < NQ; ++q) cov |= andN<LPS>(mLe2[t][q]);
    both &= cov;
  }
  return (both | only) & G1;
}

// Dispatch on (present, number of own values); more than 3 own values: no scan (returns 0 = no
// step provably a no-op).
template <int VI, int LPS, int IT, bool PAIR = false>
__device__ __forceinline__ u64 map_noop_nv3(const u64 *buf, unsigned W, unsigned A, const u64 *mirror,
                                            const u64 *thr, bool present, int nv, unsigned n, int lane) {
  const u64 *me = mirror, *mc = mirror + A;
  if (!present) return map_noop_steps3<VI, 0, LPS, IT, false>(buf, W, A, me, mc, thr, n, lane);
  switch (nv) {
    case 0: return map_noop_steps3<VI, 0, LPS, IT, true>(buf, W, A, me, mc, thr, n, lane);
    case 1: return map_noop_steps3<VI, 1, LPS, IT, true>(buf, W, A, me, mc, thr, n, lane);
    case 2: return map_noop_steps3<VI, 2, LPS, IT, true>(buf, W, A, me, mc, thr, n, lane);
    case 3: return map_noop_steps3<VI, 3, LPS, IT, true>(buf, W, A, me, mc, thr, n, lane);
    default: return 0;
  }
}

template <int VI, int LPS, int IT, bool PAIR = false>
__device__ __forceinline__ u64 map_noop_nv(const u64 *buf, unsigned W, unsigned A, const u64 *mirror,
                                           unsigned VO, bool present, int nv, unsigned n, int lane) {
  const u64 *me = mirror, *mc = mirror + A, *mmx = mirror + (1 + VO) * A;
  if constexpr (PAIR) {
    if (!present) return map_noop_steps2<VI, 0, LPS, IT, false>(buf, W, A, me, mc, mmx, n, lane);
    switch (nv) {
      case 0: return map_noop_steps2<VI, 0, LPS, IT, true>(buf, W, A, me, mc, mmx, n, lane);
      case 1: return map_noop_steps2<VI, 1, LPS, IT, true>(buf, W, A, me, mc, mmx, n, lane);
      case 2: return map_noop_steps2<VI, 2, LPS, IT, true>(buf, W, A, me, mc, mmx, n, lane);
      case 3: return map_noop_steps2<VI, 3, LPS, IT, true>(buf, W, A, me, mc, mmx, n, lane);
      default: return 0;
    }
  }
  if (!present) return map_noop_steps<VI, 0, LPS, IT, false>(buf, W, A, me, mc, mmx, n, lane);
  switch (nv) {
    case 0: return map_noop_steps<VI, 0, LPS, IT, true>(buf, W, A, me, mc, mmx, n, lane);
    case 1: return map_noop_steps<VI, 1, LPS, IT, true>(buf, W, A, me, mc, mmx, n, lane);
    case 2: return map_noop_steps<VI, 2, LPS, IT, true>(buf, W, A, me, mc, mmx, n, lane);
    case 3: return map_noop_steps<VI, 3, LPS, IT, true>(buf, W, A, me, mc, mmx, n, lane);
    default: return 0;
  }
}

// Own values pairwise not strictly ordered (precondition (a) of the scan).
template <int APL, int VO>
__device__ __forceinline__ bool mv_antichain(const MVState<APL, VO> &s) {
  bool ok = true;
#pragma unroll
  for (int q = 0; q < VO; ++q)
#pragma unroll
    for (int q2 = 0; q2 < VO; ++q2)
      if (q != q2 && (s.vm & (1u << q)) && (s.vm & (1u << q2)) && vlt(s.c[q], s.c[q2])) ok = false;
  return ok;
}

// ---- Register-tested whole-chunk skip (RS path, A <= 32 even, 16-replica chunks) -------------
// Almost every 16-replica chunk of a long fold changes nothing for a key.  The RS path keeps two
// chunks in flight (LDS-DMA into two slots) while it tests a third: chunk ch is copied from its slot
// into registers in the scan's own layout — lane (s, gq) = (lane / 4, lane % 4) holds step s, actor
// pairs (2gq + 8m, 2gq + 8m + 1), m < NP — the slot is refilled with chunk ch+2 at once, and the
// whole chunk is tested in registers against the fold state's scan operands (entry clock, TB, TO,
// own value clocks) read from the LDS mirror.  A skipped chunk costs the copy, one register scan
// and a clock max (lane = actor, from the chunk's clock max); any other chunk (a failed test, a
// remove naming the key, the scan's preconditions off) is written back over its slot and runs
// through the exact per-step loop, after which chunk ch+2 is issued again.
// MAP_VAN_MASK (build option): the chunk test's "incoming value forgotten to empty" (c2 <= deleted,
// deleted = e2 > e ? e2 : 0) as a combination of ballots instead of a select then a compare.
#ifndef MAP_VAN_MASK
#define MAP_VAN_MASK 0
#endif
// MAP_TB_INC (build option): the register operands hold TB = max(e, min(Cs, m1)) itself instead of the
// acc clock Cs, advanced on a skipped chunk by TB' = max(TB, min(chunk clock max, m1)) (min distributes
// over max), so the chunk test no longer recomputes it (-24 VALU per chunk); reloaded from thr after
// the exact loop.  RsReg::cs then holds TB.
#ifndef MAP_TB_INC
#define MAP_TB_INC 0
#endif
// The register operands' clock word after a skipped chunk (Cs, or TB under MAP_TB_INC).
__device__ __forceinline__ u64 rs_adv(u64 cur, u64 cmax, u64 m1) {
  if (MAP_TB_INC) cmax = cmax < m1 ? cmax : m1;
  return cur > cmax ? cur : cmax;
}

template <int VI, int NP>
struct RsChunk {
  u64x2 e[NP];
  u64x2 c[VI][NP];
  u64x2 co[NP];
  u64 cm;     // the chunk's clock max of actor `lane` (map_chunk_max_kernel)
  u64 v[VI];  // the VI values of step s
  u64x2 cmp[NP];  // the same clock max at the lane's actor pairs (scan layout)
};

// The fold state's scan operands kept in registers in the scan layout between exact steps
// (reloaded from the LDS mirror after each chunk handed to the exact loop; the acc clock also
// advances by each skipped chunk's clock max).
template <int NP>
struct RsReg {
  u64x2 ea[NP], to[NP], m1[NP], cs[NP];
  u64x2 sq[3][NP];
};

template <int NQ, int NP>
struct RsOwn {
  u64x2 ea[NP], tb[NP], to[NP];
  u64x2 sq[NQ > 0 ? NQ : 1][NP];
};

// The scan operands of the fold state from the LDS mirror (me / mc) and thresholds (TB / TO).
// The actor pair element m of lane (s, gq) holds in the scan layout: 2gq + 8m, or with PERM (the
// SH path, whose reads are bank-conflict free only when each lane walks its pairs rotated by its
// step) 2gq + 8((m + s) % 4) (NP == 4).
template <bool PERM>
__device__ __forceinline__ unsigned rs_a0(int lane, int m) {
  const unsigned gq = (unsigned)lane & 3;
  if constexpr (PERM) return 2 * gq + 8 * ((m + ((unsigned)lane >> 2)) & 3);
  return 2 * gq + 8 * m;
}

// The ST path's layout (two waves per key, each testing 8 steps of a chunk): lane (s, g8) = (lane / 8,
// lane % 8) holds actor pairs (2 g8 + 16 m, 2 g8 + 16 m + 1), m < 2.
__device__ __forceinline__ unsigned st_a0(int lane, int m) { return 2 * ((unsigned)lane & 7) + 16 * m; }

template <int NQ, bool PRESENT, int NP, bool PERM = false, int LPS = 4>
__device__ __forceinline__ RsOwn<NQ, NP> rs_own(const u64 *mirror, const u64 *thr, unsigned long long A, int lane,
                                                int nv = NQ) {
  RsOwn<NQ, NP> o;
#pragma unroll
  for (int m = 0; m < NP; ++m) {
    const unsigned a0 = LPS == 8 ? st_a0(lane, m) : rs_a0<PERM>(lane, m);
    const unsigned long long a = a0 < A ? a0 : A - 2;
    o.tb[m] = lds2(thr + a);
    if constexpr (PRESENT) {
      o.ea[m] = lds2(mirror + a);
      o.to[m] = lds2(thr + A + a);
#pragma unroll
      for (int q = 0; q < NQ; ++q) o.sq[q][m] = q < nv ? lds2(mirror + (1 + q) * A + a) : u64x2{0, 0};
    }
  }
  return o;
}

// The no-op verdict of map_noop_steps3 on the register chunk (bit 4s: step s provably a no-op).
// An optional hook issuing the next chunk's LDS-DMA pieces between the test's compares: 18
// back-to-back pieces stall the wave on the address unit (~65 cycles each with four waves per CU
// issuing), while spread over the test they issue under its VALU work.
struct RsNoDma {
  static constexpr int count = 0;
  static constexpr bool late = false;
  __device__ __forceinline__ void operator()(int) {}
};

// The test's per-step results (bit LPS*s: step s), its LPS lanes combined: p2 "the replica has the
// key" (an OR over actors), the rest ANDs over actors — b the both-present entry test, o the
// acc-only test, van[t] "incoming value t forgotten to empty", le[t][q] "incoming value t <= own value
// q"; rs_verdict then ORs over q.
template <int VI, int NQ>
struct RsPart {
  u64 p2, b, o, van[VI], le[VI][NQ > 0 ? NQ : 1];
};

template <int VI, int NQ, bool PRESENT, int LPS = 4>
__device__ __forceinline__ u64 rs_verdict(const RsPart<VI, NQ> &x) {
  const u64 G1 = grp_mask<LPS>();
  if constexpr (!PRESENT) return (~x.p2 | x.b) & G1;
  u64 both = x.p2 & x.b;
  const u64 only = ~x.p2 & x.o;
#pragma unroll
  for (int t = 0; t < VI; ++t) {
    u64 cov = x.van[t];
#pragma unroll
    for (int q = 0; q < NQ; ++q) cov |= x.le[t][q];
    both &= cov;
  }
  return (both | only) & G1;
}

template <int VI, int NP, int NQ, bool PRESENT, bool BATCH = false, int LPS = 4, class F = RsNoDma>
__device__ __forceinline__ RsPart<VI, NQ> rs_part(const RsChunk<VI, NP> &r, const RsOwn<NQ, NP> &o, F &&dma = F{}) {
  constexpr int ND = std::remove_reference_t<F>::count;  // pieces to issue: two per element, the rest after
  constexpr int NQ1 = NQ > 0 ? NQ : 1;
  // per-test ballot masks (bit = lane), combined per step at the end
  u64 mP2 = 0, mB = ~0ull, mO = ~0ull, mVan[VI], mLe[VI][NQ1];
#pragma unroll
  for (int t = 0; t < VI; ++t) {
    mVan[t] = ~0ull;
#pragma unroll
    for (int q = 0; q < NQ1; ++q) mLe[t][q] = ~0ull;
  }
  constexpr int JS = (MAP_RS_LATE && std::remove_reference_t<F>::late) ? 2 : 0;  // (pieces one element later)
#pragma unroll
  for (int m = 0; m < NP; ++m) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if constexpr (ND > 0) {  // the masks so far are computed before these pieces issue
        const int j = 2 * (2 * m + h) - JS;
        asm volatile("" : "+s"(mP2), "+s"(mB), "+s"(mO));
#pragma unroll
        for (int t = 0; t < VI; ++t) {
          asm volatile("" : "+s"(mVan[t]));
#pragma unroll
          for (int q = 0; q < NQ1; ++q) asm volatile("" : "+s"(mLe[t][q]));
        }
        if (j >= 0 && j < ND) dma(j);
        if (j + 1 >= 0 && j + 1 < ND) dma(j + 1);
      }
      const u64 e2 = r.e[m][h], tb = o.tb[m][h];
      if constexpr (BATCH) {
        // Every compare of the element first, then the scalar ANDs: a compare's lane mask reaches the
        // scalar unit ~25 cycles after issue, so an AND right behind its compare stalls the wave for
        // that long, while a batch of compares overlaps those latencies (scripts/probe_cmp.hip:
        // 25 -> 11.5 cycles per compare + AND on gfx950).
        const u64 bP2 = __ballot(e2 != 0), bB0 = __ballot(e2 <= tb);
        if constexpr (!PRESENT) {
          __builtin_amdgcn_sched_barrier(0);
          mP2 |= bP2;
          mB &= bB0;
        } else {
          const u64 co = r.co[m][h], ea = o.ea[m][h];
          const u64 bB1 = __ballot(ea - 1 >= co), bB2 = __ballot(ea == e2), bO = __ballot(co <= o.to[m][h]);
          const u64 del = e2 > ea ? e2 : 0;
          const u64 bGt = MAP_VAN_MASK ? __ballot(e2 > ea) : 0;
          u64 bV[VI], bL[VI][NQ1];
#pragma unroll
          for (int t = 0; t < VI; ++t) {
            const u64 c2 = r.c[t][m][h];
            // c2 <= deleted: (e2 > ea && c2 <= e2) || (e2 <= ea && c2 == 0), as masks (no select chain)
            bV[t] = MAP_VAN_MASK ? (bGt & __ballot(c2 <= e2)) | (~bGt & __ballot(c2 == 0)) : __ballot(c2 <= del);
#pragma unroll
            for (int q = 0; q < NQ; ++q) bL[t][q] = __ballot(c2 <= o.sq[q][m][h]);
          }
          __builtin_amdgcn_sched_barrier(0);
          mP2 |= bP2;
          mB &= bB0 & (bB1 | bB2);
          mO &= bO;
#pragma unroll
          for (int t = 0; t < VI; ++t) {
            mVan[t] &= bV[t];
#pragma unroll
            for (int q = 0; q < NQ; ++q) mLe[t][q] &= bL[t][q];
          }
        }
        continue;
      }
      mP2 |= __ballot(e2 != 0);
      if constexpr (!PRESENT) {
        mB &= __ballot(e2 <= tb);
      } else {
        const u64 co = r.co[m][h], ea = o.ea[m][h];
        mB &= __ballot((e2 <= tb) & ((ea - 1 >= co) | (ea == e2)));
        mO &= __ballot(co <= o.to[m][h]);
        const u64 del = e2 > ea ? e2 : 0;
        const u64 bGt = MAP_VAN_MASK ? __ballot(e2 > ea) : 0;
#pragma unroll
        for (int t = 0; t < VI; ++t) {
          const u64 c2 = r.c[t][m][h];
          mVan[t] &= MAP_VAN_MASK ? (bGt & __ballot(c2 <= e2)) | (~bGt & __ballot(c2 == 0)) : __ballot(c2 <= del);
#pragma unroll
          for (int q = 0; q < NQ; ++q) mLe[t][q] &= __ballot(c2 <= o.sq[q][m][h]);
        }
      }
    }
  }
  if constexpr (ND > 0) {
#pragma unroll
    for (int j = 4 * NP - JS; j < ND; ++j) dma(j);
  }
  RsPart<VI, NQ> x;
  x.p2 = orN<LPS>(mP2);
  x.b = andN<LPS>(mB);
  x.o = PRESENT ? andN<LPS>(mO) : 0;
#pragma unroll
  for (int t = 0; t < VI; ++t) {
    x.van[t] = PRESENT ? andN<LPS>(mVan[t]) : 0;
#pragma unroll
    for (int q = 0; q < NQ1; ++q) x.le[t][q] = (PRESENT && q < NQ) ? andN<LPS>(mLe[t][q]) : 0;
  }
  return x;
}

template <int VI, int NP, int NQ, bool PRESENT, bool BATCH = false, class F = RsNoDma>
__device__ __forceinline__ u64 rs_noop(const RsChunk<VI, NP> &r, const RsOwn<NQ, NP> &o, F &&dma = F{}) {
  return rs_verdict<VI, NQ, PRESENT>(rs_part<VI, NP, NQ, PRESENT, BATCH>(r, o, dma));
}

// The verdict from the LDS mirror (the exact loop's scan): one instantiation per presence, own
// values as 3 zero-padded slots (see rs_reg_noop_nv).
template <int VI, int NP, bool PERM = false>
__device__ __forceinline__ u64 rs_lds_own_noop(const RsChunk<VI, NP> &r, const u64 *mirror, const u64 *thr,
                                               unsigned long long A, bool present, int nv, int lane) {
  if (!present) return rs_noop<VI, NP, 0, false>(r, rs_own<0, false, NP, PERM>(mirror, thr, A, lane));
  if (nv > 3) return 0;
  return rs_noop<VI, NP, 3, true>(r, rs_own<3, true, NP, PERM>(mirror, thr, A, lane, nv));
}
template <int VI, int NP>
__device__ __forceinline__ void rs_reload(RsChunk<VI, NP> &r, const u64 *img, unsigned long long WS, const u64 *vals,
                                          const u64 *cm, unsigned long long A, int lane, bool vload = true) {
  const unsigned s = (unsigned)lane >> 2, gq = (unsigned)lane & 3;
  const u64 *st = img + s * WS;
#pragma unroll
  for (int m = 0; m < NP; ++m) {
    const unsigned a0 = 2 * gq + 8 * m;
    const unsigned long long a = a0 < A ? a0 : A - 2;
    r.e[m] = lds2(st + a);
#pragma unroll
    for (int t = 0; t < VI; ++t) r.c[t][m] = lds2(st + (1 + t) * A + a);
    r.co[m] = lds2(st + (1 + VI) * A + a);
  }
  r.cm = cm[(unsigned long long)lane < A ? lane : A - 1];
#pragma unroll
  for (int m = 0; m < NP; ++m) {
    const unsigned a0 = 2 * gq + 8 * m;
    r.cmp[m] = lds2(cm + (a0 < A ? a0 : A - 2));
  }
  if (vload) {
#pragma unroll
    for (int t = 0; t < VI; ++t) r.v[t] = vals[s * VI + t];
  }
}

// The verdict from the register-held operands: TB = max(e, min(Cs, m1)) computed here.
template <int VI, int NP, int NQ, bool PRESENT, bool BATCH = false, class F = RsNoDma>
__device__ __forceinline__ u64 rs_reg_noop(const RsChunk<VI, NP> &r, const RsReg<NP> &g, F &&dma = F{}) {
  RsOwn<NQ, NP> o;
#pragma unroll
  for (int m = 0; m < NP; ++m) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (MAP_TB_INC) {
        o.tb[m][h] = g.cs[m][h];
      } else {
        const u64 lo = g.cs[m][h] < g.m1[m][h] ? g.cs[m][h] : g.m1[m][h];
        o.tb[m][h] = g.ea[m][h] > lo ? g.ea[m][h] : lo;
      }
    }
    o.ea[m] = g.ea[m];
    o.to[m] = g.to[m];
#pragma unroll
    for (int q = 0; q < (NQ > 0 ? NQ : 1); ++q) o.sq[q][m] = g.sq[q < 3 ? q : 0][m];
  }
  return rs_noop<VI, NP, NQ, PRESENT, BATCH>(r, o, dma);
}
template <int VI, int NP, int NQ, bool PRESENT, bool BATCH = false, int LPS = 4, class F = RsNoDma>
__device__ __forceinline__ RsPart<VI, NQ> rs_reg_part(const RsChunk<VI, NP> &r, const RsReg<NP> &g, F &&dma = F{}) {
  RsOwn<NQ, NP> o;
#pragma unroll
  for (int m = 0; m < NP; ++m) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (MAP_TB_INC) {
        o.tb[m][h] = g.cs[m][h];
      } else {
        const u64 lo = g.cs[m][h] < g.m1[m][h] ? g.cs[m][h] : g.m1[m][h];
        o.tb[m][h] = g.ea[m][h] > lo ? g.ea[m][h] : lo;
      }
    }
    o.ea[m] = g.ea[m];
    o.to[m] = g.to[m];
#pragma unroll
    for (int q = 0; q < (NQ > 0 ? NQ : 1); ++q) o.sq[q][m] = g.sq[q < 3 ? q : 0][m];
  }
  return rs_part<VI, NP, NQ, PRESENT, BATCH, LPS>(r, o, dma);
}
// One instantiation per presence: own values are compared as 3 slots, the unused ones zero —
// neutral, since "c2 <= 0 everywhere" only covers an empty incoming slot, which the "appended, then
// forgotten" test covers anyway — so the kernel carries two copies of the test, not five (the
// fast path's code footprint is what sets its speed: the instruction cache is shared by two CUs).
// MAP_REG_NQ (build option, 2 by default; 3 before round 5): own-value slots the register test compares;
// 2 drops two compares per element and sends a 3-value state's chunks to the exact loop (config 4:
// 2.29 -> 2.155 ms by HIP events, profiles/r05_map_nq2_ab.log).
#ifndef MAP_REG_NQ
#define MAP_REG_NQ 2
#endif
// MAP_BATCH_ONLY (build option, 0 by default): compile only the batched-compare form of the register
// test (CRDT_TUNE mbatch=0 then has no effect), halving the test's code in the kernel.
#ifndef MAP_BATCH_ONLY
#define MAP_BATCH_ONLY 0
#endif
template <int VI, int NP, bool BATCH = false, class F = RsNoDma>
__device__ __forceinline__ u64 rs_reg_noop_nv(const RsChunk<VI, NP> &r, const RsReg<NP> &g, bool present, int nv,
                                              F &&dma = F{}) {
  if (!present) return rs_reg_noop<VI, NP, 0, false, BATCH>(r, g, dma);
  if (nv > MAP_REG_NQ) {  // (a state holding more values: the exact loop's own test settles the chunk)
#pragma unroll
    for (int j = 0; j < std::remove_reference_t<F>::count; ++j) dma(j);
    return 0;
  }
  return rs_reg_noop<VI, NP, MAP_REG_NQ, true, BATCH>(r, g, dma);
}

// The next chunk's LDS-DMA pieces as that hook (a whole chunk, every lane moving a piece of every
// step image: (2+VI)*A == 128): pieces 0..15 the step images, 16 the values, 17 the clock max —
// the same instructions, in the same order, as map_chunk_glds.
struct RsDma {
  static constexpr int count = 18;
  static constexpr bool late = true;  // (its piece 0 waits for the slot's reads: MAP_RS_LATE)
  const char *src;
  unsigned long long stride;
  u64 *img;
  unsigned long long WS;
  const unsigned *vsrc;
  u64 *vals;
  bool von;
  const u64 *csrc;
  u64 *cm;
  bool con;
  bool vp;   // the values piece streamed (uniform; off: fetched for exact chunks only)
  int diag;  // MapPlan::diag timing probes
  __device__ __forceinline__ void operator()(int j) {
    if (MAP_RS_LATE && j == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is read
    if (j < 16) {
      if (!(diag & 2) || j < 13) glds16<MAP_RS_AUX>(src, img + j * WS);
      src += stride;
    } else if (j == 16) {
      if (vp)
        if (von) glds4(vsrc, vals);
    } else {
      if (!(diag & 1))
        if (con) glds16(csrc, cm);
    }
  }
};

// The same test on a chunk handed to the exact loop (LDS slot 0, the step images rs_store wrote),
// against the fold state after its exact steps: the RS kernel's only scan, so the exact loop holds
// no scan of its own.
template <int VI, int NP>
__device__ __forceinline__ u64 rs_lds_noop_nv(const u64 *img, unsigned long long WS, const u64 *mirror,
                                              const u64 *thr, unsigned long long A, bool present, int nv,
                                              int lane) {
  RsChunk<VI, NP> r;
  const unsigned s = (unsigned)lane >> 2, gq = (unsigned)lane & 3;
  const u64 *st = img + s * WS;
#pragma unroll
  for (int m = 0; m < NP; ++m) {
    const unsigned a0 = 2 * gq + 8 * m;
    const unsigned long long a = a0 < A ? a0 : A - 2;
    r.e[m] = lds2(st + a);
#pragma unroll
    for (int t = 0; t < VI; ++t) r.c[t][m] = lds2(st + (1 + t) * A + a);
    r.co[m] = lds2(st + (1 + VI) * A + a);
  }
  r.cm = 0;
#pragma unroll
  for (int t = 0; t < VI; ++t) r.v[t] = 0;
  return rs_lds_own_noop<VI, NP>(r, mirror, thr, A, present, nv, lane);
}

// A chunk the register test could not skip: its step images, values and clock max into LDS slot 0
// in the layout the exact loop reads (map_step_read, the LDS scans, cml).
template <int VI, int NP>
__device__ __forceinline__ void rs_store(const RsChunk<VI, NP> &r, u64 *img, unsigned long long WS, u64 *vals,
                                         u64 *cm, unsigned long long A, int lane, bool vstore = true) {
  const unsigned s = (unsigned)lane >> 2, gq = (unsigned)lane & 3;
  u64 *st = img + s * WS;
#pragma unroll
  for (int m = 0; m < NP; ++m) {
    const unsigned a0 = 2 * gq + 8 * m;
    const unsigned long long a = a0 < A ? a0 : A - 2;
    *reinterpret_cast<u64x2 *>(st + a) = r.e[m];
#pragma unroll
    for (int t = 0; t < VI; ++t) *reinterpret_cast<u64x2 *>(st + (1 + t) * A + a) = r.c[t][m];
    *reinterpret_cast<u64x2 *>(st + (1 + VI) * A + a) = r.co[m];
  }
  if ((unsigned long long)lane < A) cm[lane] = r.cm;
  if (vstore && gq == 0)
#pragma unroll
    for (int t = 0; t < VI; ++t) vals[s * VI + t] = r.v[t];
}

// ---- Step-split pair (ST path: the RS path at A = 32, V = 2 with two waves per key) ------------------
// The RS path runs one wave per key: config 4's 1,024 keys are one wave per SIMD, so nothing hides the
// chunk test's latencies (LDS reads, compare -> scalar mask hand-offs, LDS-DMA issue).  In the ST path
// a key is a workgroup of two waves, wave h testing steps 8h .. 8h+7 of every 16-step chunk over all
// 32 actors (lane (s, g8): step 8h + s, actor pairs 2 g8 + 16 m): each moves its 8 step images (8
// LDS-DMA instructions + the chunk's clock max) into the standard slot layout and runs half the test,
// and the 2,048 waves are two per SIMD.  A step's verdict needs only its own lanes, so the waves
// exchange one bit per chunk (their steps all skippable) around one s_barrier.  A chunk either wave
// cannot skip: both write their steps back over the slot, wave 0 runs the RS exact loop over the whole
// chunk while wave 1 waits at a barrier, and both reload their scan operands from the fold-state mirror.
// (Round 6's first two-wave form split the ACTORS and exchanged nine partial masks per chunk: parity
// green, 2.40 vs 2.245 ms for the one-wave RS path, profiles/r06_s4_map_sp_ab.log.)
// scripts/micro/map_stream.hip put this access pattern's ceiling at 2.05-2.06 ms for config 4 (80% of
// 8 TB/s), with two waves per key holding it near 2.1 ms at half the per-wave work of one
// (profiles/r06_map_stream.log).

// DMA the 8 step images of wave h of chunk ch (steps clamped to R - 1 past the end: copies never read)
// into the slot, then the chunk's clock max (each wave keeps its own copy).  Exactly 9 global_load_lds.
// (2 + V) * A == 128: every lane moves 16 bytes of every image.
__device__ __forceinline__ void st_chunk_glds(const MapPlan &p, const GldsLanes<1> &L, unsigned long long g,
                                              unsigned long long ch, unsigned long long R, u64 *img,
                                              unsigned long long WS, u64 *cm, int lane, unsigned h) {
  const unsigned long long i0 = ch * 16 + 8 * h;
  u64 *dst = img + 8 * h * WS;
  if (ch * 16 + 16 <= R) {  // (uniform)
    const char *src = L.src0[0] + i0 * L.stride[0];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      glds16<MAP_RS_AUX>(src, dst + j * WS);
      src += L.stride[0];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned long long i = i0 + j < R ? i0 + j : R - 1;
      glds16<MAP_RS_AUX>(L.src0[0] + i * L.stride[0], dst + j * WS);
    }
  }
  if ((unsigned long long)(2 * lane) < p.A) glds16(p.cmax + (g * p.nch + ch) * p.A + 2 * lane, cm);
}

// st_chunk_glds of a whole chunk as the chunk test's DMA hook.
struct StDma {
  static constexpr int count = 9;
  static constexpr bool late = false;
  const char *src;
  unsigned long long stride;
  u64 *img;  // the wave's first step image of the slot
  unsigned long long WS;
  const u64 *csrc;
  u64 *cm;
  bool con;
  __device__ __forceinline__ void operator()(int j) {
    if (j < 8) {
      glds16<MAP_RS_AUX>(src, img + j * WS);
      src += stride;
    } else if (con) {
      glds16(csrc, cm);
    }
  }
};

// Wave h's 8 steps of a slot into the ST scan layout, and the chunk's clock max (lane = actor, and at
// the lane's pairs).
template <int VI, int NP>
__device__ __forceinline__ void st_reload(RsChunk<VI, NP> &r, const u64 *img, unsigned long long WS, const u64 *cm,
                                          unsigned long long A, int lane, unsigned h, bool wcm = true) {
  const u64 *st = img + (8 * h + ((unsigned)lane >> 3)) * WS;
#pragma unroll
  for (int m = 0; m < NP; ++m) {
    const unsigned a0 = st_a0(lane, m);
    const unsigned long long a = a0 < A ? a0 : A - 2;
    r.e[m] = lds2(st + a);
#pragma unroll
    for (int t = 0; t < VI; ++t) r.c[t][m] = lds2(st + (1 + t) * A + a);
    r.co[m] = lds2(st + (1 + VI) * A + a);
  }
  if (wcm) {
    r.cm = cm[(unsigned long long)lane < A ? lane : A - 1];
#pragma unroll
    for (int m = 0; m < NP; ++m) {
      const unsigned a0 = st_a0(lane, m);
      r.cmp[m] = lds2(cm + (a0 < A ? a0 : A - 2));
    }
  }
}

// A chunk neither wave could skip: the wave's steps back over the slot, and its clock-max copy.
template <int VI, int NP>
__device__ __forceinline__ void st_store(const RsChunk<VI, NP> &r, u64 *img, unsigned long long WS, u64 *cm,
                                         unsigned long long A, int lane, unsigned h) {
  u64 *st = img + (8 * h + ((unsigned)lane >> 3)) * WS;
#pragma unroll
  for (int m = 0; m < NP; ++m) {
    const unsigned a0 = st_a0(lane, m);
    const unsigned long long a = a0 < A ? a0 : A - 2;
    *reinterpret_cast<u64x2 *>(st + a) = r.e[m];
#pragma unroll
    for (int t = 0; t < VI; ++t) *reinterpret_cast<u64x2 *>(st + (1 + t) * A + a) = r.c[t][m];
    *reinterpret_cast<u64x2 *>(st + (1 + VI) * A + a) = r.co[m];
  }
  if ((unsigned long long)lane < A) cm[lane] = r.cm;
}

// This wave's verdict (bit 8s: its step s skippable) from the register-held operands, with the RS
// dispatch on presence / own value count (a state holding more than MAP_REG_NQ values settles nothing
// here, as rs_reg_noop_nv); `test` off: the DMA hook still issues its pieces.
template <bool BATCH, class F = RsNoDma>
__device__ __forceinline__ u64 st_reg_verdict(const RsChunk<2, 2> &r, const RsReg<2> &g, bool present, int nv,
                                              bool test, F &&dma = F{}) {
  if (!test || (present && nv > MAP_REG_NQ)) {
#pragma unroll
    for (int j = 0; j < std::remove_reference_t<F>::count; ++j) dma(j);
    return 0;
  }
  if (!present) return rs_verdict<2, 0, false, 8>(rs_reg_part<2, 2, 0, false, BATCH, 8>(r, g, dma));
  return rs_verdict<2, MAP_REG_NQ, true, 8>(rs_reg_part<2, 2, MAP_REG_NQ, true, BATCH, 8>(r, g, dma));
}

// The steps of wave h a chunk of n0 steps holds, as verdict bits.
__device__ __forceinline__ u64 st_want(unsigned long long n0, unsigned h) {
  const unsigned long long nh = n0 > 8 * h ? (n0 - 8 * h < 8 ? n0 - 8 * h : 8) : 0;
  return nh >= 8 ? grp_mask<8>() : (grp_mask<8>() & ((1ull << (8 * nh)) - 1));
}

// The pair's barrier: this wave's LDS writes done, both waves here, no LDS access moved across it.
// (No vmcnt wait: the LDS-DMA of later chunks stays in flight.)
__device__ __forceinline__ void st_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One chunk's vote: both waves' steps skippable.  vw: this chunk parity's two words.
__device__ __forceinline__ bool st_vote(unsigned *vw, bool mine, unsigned h, int lane) {
  if (lane == 0) reinterpret_cast<volatile unsigned *>(vw)[h] = mine ? 1u : 0u;
  st_barrier();
  const unsigned other = __builtin_amdgcn_readfirstlane(reinterpret_cast<const volatile unsigned *>(vw)[h ^ 1]);
  return mine && other != 0;
}

// The exact loop's test of a chunk from LDS (wave 0 alone, all 16 steps, in two 8-step passes of the
// ST layout), as bits 4s (the exact loop's LPS = 4 convention).
__device__ __forceinline__ u64 st_lds_noop(const u64 *img, unsigned long long WS, const u64 *mirror, const u64 *thr,
                                           unsigned long long A, bool present, int nv, int lane) {
  if (present && nv > 3) return 0;
  u64 out = 0;
#pragma unroll
  for (unsigned hh = 0; hh < 2; ++hh) {
    RsChunk<2, 2> r;
    r.cm = 0;
    r.v[0] = r.v[1] = 0;
    st_reload(r, img, WS, nullptr, A, lane, hh, false);
    const u64 v8 = present ? rs_verdict<2, 3, true, 8>(rs_part<2, 2, 3, true, false, 8>(
                                 r, rs_own<3, true, 2, false, 8>(mirror, thr, A, lane, nv)))
                           : rs_verdict<2, 0, false, 8>(rs_part<2, 2, 0, false, false, 8>(
                                 r, rs_own<0, false, 2, false, 8>(mirror, thr, A, lane, 0)));
#pragma unroll
    for (int sv = 0; sv < 8; ++sv)
      if ((v8 >> (8 * sv)) & 1ull) out |= 1ull << (4 * (8 * hh + sv));
  }
  return out;
}

// ---- Shared replica-clock ring (SH path: the RS path at A = 32, V = 2, four key waves per CU) ------
// A chunk's replica-clock rows are the same for every key of a group and a quarter of each step
// image, and a CU's LDS-DMA engine takes one instruction per ~17 cycles whatever its lane count
// (scripts/micro/glds_rate.hip: 68 cycles per piece per wave at four waves per CU, 1 KiB or 256 B
// alike).  In the SH path the four waves of a workgroup fold four keys of one group: each wave
// streams its key's entry / value clocks into two private slots, packed 4 steps to 3 pieces (12
// per chunk instead of 16), and the clock rows and clock max of a chunk are staged ONCE per
// workgroup into a ring of kShS shared slots — wave w moves steps 4w..4w+3 and a quarter of the
// clock max.  14 instructions per chunk and wave instead of 17, and the clock rows leave L2 once
// per workgroup instead of once per key (the excess PMC traffic of the RS path).
// Layouts, in 16-byte units (a pair of u64 words): every 16 consecutive DMA lanes move one 256-byte
// row (a DMA instruction whose lane quads span rows costs its CU 1.3-4x, scripts/micro/glds_rate.hip)
//   private slot  192*(s/4) + 64*part + 16*(s%4) + pair   (part 0 entry clock, 1.. value clocks;
//                 pair = actor / 2; 1,536 words)
//   shared slot   64*(s/4) + 16*(s%4) + pair  (the clock rows, 512 words), then the chunk clock max [A]
// and lane (s, gq) of the chunk test reads its pairs gq + 4m rotated by its step (rs_a0<true>), so
// that the 16 lanes of one LDS read cycle hit 16 different banks.
// Hand-over: a wave's pieces are in LDS once its own vmcnt retires them; it then adds 1 to the
// slot's arrival counter, and a wave reads chunk c's shared slot only once the counter reached
// 4 * (c / kShS + 1).  Shared pieces go out kShD chunks ahead of their use and are signalled two
// chunks after issue (the private ring's depth), so a wave waits on another only when that one
// runs more than kShD - 2 chunks behind (an exact loop).  A slot is refilled (chunk c + kShD, at
// iteration c, after chunk c arrived: every wave has then signalled chunk c, i.e. finished
// iteration c - 3) only once chunk c + kShD - kShS <= c - 3 is done everywhere: kShS = 2*kShD - 1.
constexpr int kShD = 5;
constexpr int kShS = 2 * kShD - 1;
constexpr unsigned kShSlot = 1536;            // private slot, u64 words (16 steps x 3 rows x 32)
constexpr unsigned kShShared = 512 + 32;      // shared slot: clock rows + clock max
constexpr unsigned kShSpin = 1u << 22;        // arrival-wait bound (a protocol fault is reported, never hangs)

// Per-lane LDS-DMA sources of the SH path: piece v (part v) of a 4-step group moves pair lane%16 of
// part v of step lane/16; the shared piece of wave w the same pair of the clock row of step
// 4w + lane/16.
struct ShLanes {
  const char *b[3];            // part v's row of replica 0 at the lane's pair (bytes)
  unsigned long long st[3];    // part v's replica stride (bytes)
  const char *cb;              // clock row of replica 0 at the lane's pair
  unsigned long long cst;      // clock replica stride (bytes)
  unsigned sub;                // lane / 16: the step of a 4-step group this lane moves
};

__device__ __forceinline__ ShLanes sh_lanes(const MapPlan &p, unsigned long long g, unsigned long long k, int lane) {
  ShLanes L;
  const unsigned long long A = p.A, pr = (unsigned)lane & 15;
  const unsigned long long be = (unsigned long long)(p.ec + g * p.e_gs + k * A);
  const unsigned long long bv = (unsigned long long)(p.vclk + g * p.vc_gs + k * 2 * A);
  L.b[0] = reinterpret_cast<const char *>(be + pr * 16);
  L.b[1] = reinterpret_cast<const char *>(bv + pr * 16);
  L.b[2] = reinterpret_cast<const char *>(bv + A * 8 + pr * 16);
  L.st[0] = (unsigned long long)p.e_rs * 8;
  L.st[1] = L.st[2] = (unsigned long long)p.vc_rs * 8;
  L.cb = reinterpret_cast<const char *>((unsigned long long)(p.clock + g * p.c_gs) + pr * 16);
  L.cst = (unsigned long long)p.c_rs * 8;
  L.sub = (unsigned)lane >> 4;
  return L;
}

// The 12 private pieces of chunk [i0, i0 + 16) (steps past iend - 1 clamped: copies never read).
__device__ __forceinline__ void sh_chunk_images(const ShLanes &L, unsigned long long i0, unsigned long long iend,
                                                u64 *img) {
  if (i0 + 16 <= iend) {
    const char *src[3];
#pragma unroll
    for (int v = 0; v < 3; ++v) src[v] = L.b[v] + (i0 + L.sub) * L.st[v];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int v = 0; v < 3; ++v) {
        glds16(src[v], img + (3 * q + v) * 128);
        src[v] += 4 * L.st[v];
      }
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned long long i = i0 + 4 * q + L.sub < iend ? i0 + 4 * q + L.sub : iend - 1;
#pragma unroll
      for (int v = 0; v < 3; ++v) glds16(L.b[v] + i * L.st[v], img + (3 * q + v) * 128);
    }
  }
}

// Wave w's 2 shared pieces of chunk c: clock rows of steps 4w..4w+3, clock max words 8w..8w+7.
__device__ __forceinline__ void sh_chunk_shared(const MapPlan &p, const ShLanes &L, unsigned long long g,
                                                unsigned long long c, unsigned long long iend, unsigned w, u64 *shs,
                                                int lane) {
  const unsigned long long i0 = c * 16 + 4 * w + L.sub;
  glds16(L.cb + (i0 < iend ? i0 : iend - 1) * L.cst, shs + 128 * w);
  if (lane < 4) glds16(p.cmax + (g * p.nch + c) * p.A + 8 * w + 2 * lane, shs + 512 + 8 * w);
}

// The same 14 pieces as the chunk test's DMA hook (RsNoDma's interface).
struct ShDma {
  static constexpr int count = 14;
  static constexpr bool late = false;
  const char *src[3];
  unsigned long long st4[3];
  u64 *img;
  const char *csrc;
  u64 *cdst;
  const u64 *msrc;
  u64 *mdst;
  bool mon;
  __device__ __forceinline__ void operator()(int j) {
    if (j < 12) {
      const int v = j % 3;
      glds16(src[v], img + j * 128);
      src[v] += st4[v];
    } else if (j == 12) {
      glds16(csrc, cdst);
    } else {
      if (mon) glds16(msrc, mdst);
    }
  }
};

// u64 offsets of element m (actor pair rs_a0<true>) of lane (s, gq) = (lane / 4, lane % 4) of the
// chunk test in the SH layouts (part t of the private slot at +128t words).
__device__ __forceinline__ unsigned sh_poff(int lane, int m) {
  const unsigned s = (unsigned)lane >> 2;
  return 2 * (192 * (s >> 2) + 16 * (s & 3)) + rs_a0<true>(lane, m);
}
__device__ __forceinline__ unsigned sh_coff(int lane, int m) {
  const unsigned s = (unsigned)lane >> 2;
  return 2 * (64 * (s >> 2) + 16 * (s & 3)) + rs_a0<true>(lane, m);
}
// ... and of actor a at step s (lane = actor: the exact loop's reads)
__device__ __forceinline__ unsigned sh_pword(unsigned s, unsigned a) {
  return 2 * (192 * (s >> 2) + 16 * (s & 3)) + a;
}
__device__ __forceinline__ unsigned sh_cword(unsigned s, unsigned a) {
  return 2 * (64 * (s >> 2) + 16 * (s & 3)) + a;
}

template <int VI, int NP>
__device__ __forceinline__ void sh_reload(RsChunk<VI, NP> &r, const u64 *img, const u64 *shs, unsigned long long A,
                                          int lane, bool cmload = true) {
#pragma unroll
  for (int m = 0; m < NP; ++m) {
    const unsigned po = sh_poff(lane, m);
    r.e[m] = lds2(img + po);
#pragma unroll
    for (int t = 0; t < VI; ++t) r.c[t][m] = lds2(img + po + 128 * (1 + t));
    r.co[m] = lds2(shs + sh_coff(lane, m));
  }
  if (cmload) {
    r.cm = shs[512 + ((unsigned long long)lane < A ? lane : A - 1)];
#pragma unroll
    for (int m = 0; m < NP; ++m) r.cmp[m] = lds2(shs + 512 + rs_a0<true>(lane, m));
  } else {
    r.cm = 0;
#pragma unroll
    for (int m = 0; m < NP; ++m) r.cmp[m] = u64x2{0, 0};
  }
}

// A chunk the test could not skip: its entry / value clocks back into the private slot (the slot
// was being refilled); the clock rows and clock max stay in the shared slot.
template <int VI, int NP>
__device__ __forceinline__ void sh_store(const RsChunk<VI, NP> &r, u64 *img, int lane) {
#pragma unroll
  for (int m = 0; m < NP; ++m) {
    const unsigned po = sh_poff(lane, m);
    *reinterpret_cast<u64x2 *>(img + po) = r.e[m];
#pragma unroll
    for (int t = 0; t < VI; ++t) *reinterpret_cast<u64x2 *>(img + po + 128 * (1 + t)) = r.c[t][m];
  }
}

// The SH arrival counter of a shared slot, read through LDS each time (other waves add to it).
__device__ __forceinline__ unsigned sh_arrived(const unsigned *cnt) {
  return __builtin_amdgcn_readfirstlane(*reinterpret_cast<const volatile unsigned *>(cnt));
}

// ITM: unrolled scan iterations ceil(A / LPS) rounded up to a power of two, fixed per launch so
// each kernel's register allocation only covers its own scan shape.  NP > 0: the RS path (above).
template <int APL, int VI, int VO, int CM, int NB, bool GL, int ITM, int NP = 0, bool SH = false, bool ST = false>
__global__ __launch_bounds__(SH ? 256 : (ST ? 128 : 64), ST ? 2 : 1) void map_fold_kernel(MapPlan pk) {
  constexpr bool RS = NP > 0;
  static_assert(!SH || (RS && VI == 2 && NP == 4), "SH path: the RS path at A = 32, V = 2");
  static_assert(!ST || (RS && !SH && NB == 2 && VI == 2 && NP == 2 && CM == 16), "ST path: the RS path at A = 32, V = 2");
  const MapPlan p = pk;  // a local copy the optimizer can split into registers (the by-value
                         // kernel argument itself would be materialized in scratch memory)
  // SH: a workgroup of four waves, wave w folding key 4*blockIdx + w (K % 4 == 0: one group)
  const unsigned wv = SH ? (unsigned)threadIdx.x >> 6 : 0u;
  const unsigned long long gk0 = SH ? 4ull * blockIdx.x + wv : (unsigned long long)blockIdx.x;
  const unsigned long long g = gk0 / p.K;
  const unsigned long long k = gk0 % p.K;
  const int lane = (SH || ST) ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  const unsigned hw = ST ? (unsigned)threadIdx.x >> 6 : 0u;  // ST: the wave's 8 steps of each chunk
  const unsigned long long R = p.R;

  bool present = false;
  u64 e[APL], cs[APL];
#pragma unroll
  for (int j = 0; j < APL; ++j) e[j] = cs[j] = 0;
  MVState<APL, VO> mv;
  mv.vm = 0;
  mv.next = 0;
#pragma unroll
  for (int q = 0; q < VO; ++q) {
    mv.v[q] = 0;
    mv.seq[q] = 0;
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
  constexpr int C = (GL || RS) ? CM : MapChunk<APL, VI, CM>::C;
  static_assert(!SH || C == 16, "SH path: 16-replica chunks");
  static_assert(!GL || (APL == 1 && NB >= 2), "LDS-DMA staging: one actor per lane");
  static_assert(GL || RS || NB == 2, "register staging double-buffers");
  static_assert(!RS || (APL == 1 && !GL && NB == 2 && CM == 16 && VO <= 4 && VI <= 2), "RS path shape");
  // speculative scan geometry: NS >= C steps per scan, LPS lanes per step
  constexpr int NS = C > 8 ? 16 : (C > 4 ? 8 : (C > 2 ? 4 : 2));
  constexpr int LPS = 64 / NS;
  const unsigned long long A = p.A;
  const unsigned long long W = (2 + VI) * A;
  const unsigned long long WS = RS ? map_ws_rs(W) : map_ws(W);  // padded step stride in the ring
  // LDS: NB image slots (C*WS words each; SH: kShSlot), NB value slots (C*VI), the per-key remove
  // list, the fold-state mirror.  (Addresses are always computed from map_lds: a pointer table
  // would hide the LDS address space and turn every access into a flat op.)  SH: four such wave
  // regions (no clock-max slots), then the shared ring and its arrival counters.
  // ST: both waves' clock-max copies (wave h's at cml + h * NB * CMS), and after the thresholds the vote
  // words [chunk parity][wave] (u32) and the fold-state word for the partner (present, own value count)
  const unsigned long long SLOT = SH ? kShSlot : C * WS;
  constexpr unsigned long long NW = ST ? 2 : 1;
  const unsigned long long CMS = A;  // staged clock-max stride
  const unsigned long long PW =
      NB * SLOT + NB * C * VI + kMapL + (2 + VO) * A + ((GL || RS) && !SH ? NW * NB * CMS : 0) + 4 * A + (ST ? 4 : 0);
  u64 *const wl = map_lds + (SH ? wv * PW : 0);
  u64 *const shr = map_lds + 4 * PW;  // SH: kShS shared slots
  unsigned *const arr = reinterpret_cast<unsigned *>(shr + kShS * kShShared);
  u64 *const vbase = wl + NB * SLOT;
  unsigned *lrow = reinterpret_cast<unsigned *>(vbase + NB * C * VI);
  unsigned *lidx = lrow + kMapL;
  // fold-state mirror read by the speculative scan: entry clock, VO value clocks, acc clock
  u64 *mirror = vbase + NB * C * VI + kMapL;  // (kMapL u64 = the two u32 lists)
  constexpr bool kSpec = APL == 1 && VO <= 4;
  u64 *const cml = mirror + (2 + VO) * A;  // GL: NB staged chunk clock maxima (A words each)
  // scan thresholds (map_noop_steps3, RS): TB [A] | TO [A]; m1 = (min nonzero own value clock) - 1
  u64 *const thr = cml + ((GL || RS) && !SH ? NW * NB * CMS : 0);
  u64 *const csm = thr + 2 * A;  // RS: the acc clock and m1 handed back to the register operands
  u64 *const m1m = thr + 3 * A;
  unsigned *const vw = reinterpret_cast<unsigned *>(m1m + A);  // ST: vote words [parity][wave]
  unsigned *const spst = vw + 4;                                 // ST: present | own values << 1
  u64 m1 = ~0ull;
  const unsigned long long nch = (R + C - 1) / C;
  if constexpr (ST) {
    if (hw == 1) {  // the partner wave: steps 8 .. 15 of every chunk (wave 0 holds the fold state)
      const GldsLanes<1> gp = glds_lanes<VI, 1>(p, g, k, lane);
      u64 *const cm1 = cml + NB * CMS;  // this wave's clock-max copies
      RsChunk<VI, NP> r;
      RsReg<NP> q;
#pragma unroll
      for (int m = 0; m < NP; ++m) {
        q.ea[m] = 0;
        q.cs[m] = 0;
        q.to[m] = ~0ull;
        q.m1[m] = ~0ull;
#pragma unroll
        for (int x = 0; x < 3; ++x) q.sq[x][m] = 0;
      }
      bool pres = false;
      int nvp = 0;
      const bool batch = MAP_BATCH_ONLY || p.batch;
      for (unsigned long long c = 0; c < 2 && c < nch; ++c)
        st_chunk_glds(p, gp, g, c, R, wl + c * SLOT, WS, cm1 + c * CMS, lane, 1);
      for (unsigned long long ch = 0; ch < nch; ++ch) {
        const unsigned slot = (unsigned)(ch & 1);
        u64 *const img = wl + slot * SLOT;
        u64 *const cms = cm1 + slot * CMS;
        if (ch + 1 < nch) wait_vmcnt<9>();
        else wait_vmcnt<0>();
        st_reload(r, img, WS, cms, A, lane, 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's steps are read: refill them
        const unsigned long long n0 = R - ch * C < (unsigned long long)C ? R - ch * C : C;
        const u64 want = st_want(n0, 1);
        const unsigned long long i2 = (ch + 2) * C;
        const bool spread = p.spec && ch + 2 < nch && i2 + C <= R;
        if (!spread && ch + 2 < nch) st_chunk_glds(p, gp, g, ch + 2, R, img, WS, cms, lane, 1);
        u64 verdict;
        if (spread) {
          StDma d{gp.src0[0] + (i2 + 8) * gp.stride[0], gp.stride[0], img + 8 * WS, WS,
                  p.cmax + (g * p.nch + ch + 2) * A + 2 * lane, cms, (unsigned long long)(2 * lane) < A};
          verdict = batch ? st_reg_verdict<true>(r, q, pres, nvp, true, d) : st_reg_verdict<false>(r, q, pres, nvp, true, d);
        } else {
          verdict = batch ? st_reg_verdict<true>(r, q, pres, nvp, p.spec != 0)
                          : st_reg_verdict<false>(r, q, pres, nvp, p.spec != 0);
        }
        if (st_vote(vw + 2 * slot, (verdict & want) == want, 1, lane)) {
#pragma unroll
          for (int m = 0; m < NP; ++m)
#pragma unroll
            for (int h = 0; h < 2; ++h) q.cs[m][h] = rs_adv(q.cs[m][h], r.cmp[m][h], q.m1[m][h]);
          continue;
        }
        wait_vmcnt<0>();  // chunk ch+2's copy into these steps has landed: write chunk ch back over it
        st_store(r, img, WS, cms, A, lane, 1);
        st_barrier();  // (A) the whole chunk is in LDS: wave 0 runs the exact loop
        st_barrier();  // (B) the exact loop is done, the mirror and the state word written
        const unsigned sw = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const volatile unsigned *>(spst));
        pres = (sw & 1) != 0;
        nvp = (int)(sw >> 1);
#pragma unroll
        for (int m = 0; m < NP; ++m) {
          const unsigned a0 = st_a0(lane, m);
          q.ea[m] = lds2(mirror + a0);
          q.to[m] = lds2(thr + A + a0);
          q.m1[m] = lds2(m1m + a0);
          q.cs[m] = lds2((MAP_TB_INC ? thr : csm) + a0);
#pragma unroll
          for (int x = 0; x < 3; ++x) q.sq[x][m] = x < nvp ? lds2(mirror + (1 + x) * A + a0) : u64x2{0, 0};
        }
        if (ch + 2 < nch) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          st_chunk_glds(p, gp, g, ch + 2, R, img, WS, cms, lane, 1);
        }
      }
      return;
    }
  }
  if (kSpec) {
    for (unsigned long long x = lane; x < (2 + VO) * A; x += 64) mirror[x] = 0;
    for (unsigned long long x = lane; x < A; x += 64) {
      thr[x] = 0;         // max(e, min(Cs, m1)) with e = Cs = 0
      thr[A + x] = ~0ull;  // e == 0: m1, no own values
    }
  }

  // The removes naming this key, in replica order, gathered once into LDS (row, index), so the
  // fold loop never waits on a global load for them (a vector load would drain the prefetched
  // chunks: vmcnt is in order).  More than kMapL of them: walk the group list.
  unsigned long long nl = 0;
  {
    int badl = 0;
    for (unsigned long long base = dbeg; base < dend; base += 64) {
      const unsigned long long d = base + lane;
      bool hit = false;
      unsigned row = 0;
      if (d < dend) {
        row = p.def_row[d];
        hit = (p.def_keys[d * p.Kw + kw] & kbit) != 0;
        if (k == 0 && (row >= R || (d > dbeg && p.def_row[d - 1] > row))) badl = 1;
      }
      const u64 m = __ballot(hit);
      if (hit) {
        const unsigned long long pos = nl + __popcll(m & ((1ull << lane) - 1));
        if (pos < kMapL) {
          lrow[pos] = row;
          lidx[pos] = (unsigned)d;
        }
      }
      nl += __popcll(m);
    }
    if (wany(badl)) bad = 1;
  }
  const bool direct = nl > kMapL;
  unsigned long long lp = 0;
  // (uniform values read through LDS / global memory go through readfirstlane, so that the fold's
  // control flow stays scalar)
  unsigned next_row = (!direct && nl > 0) ? __builtin_amdgcn_readfirstlane(lrow[0]) : 0xffffffffu;
  int cool = 0;
  bool anti = true;  // own values an antichain (scan precondition), refreshed after exact steps
#ifdef MAP_STATS
  unsigned st_exact = 0, st_scan = 0, st_fail = 0, st_nq = 0, st_pres = 0, st_spin = 0;
  u64 cy_arr = 0, cy_issue = 0, cy_wait = 0, cy_scan = 0, cy_skip = 0, cy_exact = 0, cy_t0 = 0, cy_all = __builtin_amdgcn_s_memtime();
#define MAP_TICK() (cy_t0 = __builtin_amdgcn_s_memtime())
#define MAP_TOCK(acc) (acc += __builtin_amdgcn_s_memtime() - cy_t0)
#else
#define MAP_TICK() ((void)0)
#define MAP_TOCK(acc) ((void)0)
#endif
  // chunk staging
  MapChunk<APL, VI, ((GL || RS) ? 2 : CM)> regs;
  RsChunk<VI, (RS ? NP : 1)> rA;
  RsReg<(RS ? NP : 1)> rg;
  if constexpr (RS) {
#pragma unroll
    for (int m = 0; m < NP; ++m) {
      rg.ea[m] = 0;
      rg.cs[m] = 0;
      rg.to[m] = ~0ull;
      rg.m1[m] = ~0ull;
#pragma unroll
      for (int q = 0; q < 3; ++q) rg.sq[q][m] = 0;
    }
  }
  const int ni = GL ? (int)((W + 127) / 128) : 0;  // 1-KiB pieces per step image (GL: 1 or 2)
  GldsLanes<1> gl1;
  GldsLanes<2> gl2;
  const bool vpiece = !(RS && (SH || ST || p.lazyv));
  ShLanes shl;
  // SH ring bookkeeping (uniform): the shared slot of chunk ch and the arrival count it needs, the
  // slot of chunk ch + kShD - 2 (signalled at iteration ch) and of chunk ch + kShD (issued)
  unsigned sh_use = 0, sh_need = 4, sh_sig = kShD - 2, sh_iss = kShD;
  bool sh_late = false;  // an arrival wait ran past kShSpin (reported as flag bit 3)
  unsigned sh_pre = 0;    // chunk ch's arrival count as read during iteration ch-1 (0: not read)
  if constexpr (SH) {
    shl = sh_lanes(p, g, k, lane);
    if (threadIdx.x < kShS) arr[threadIdx.x] = 0;
    __syncthreads();
    // chunks 0 .. kShD-3: shared pieces issued, retired and signalled at once; then, in the order
    // every iteration issues them, chunk 0's images + chunk kShD-2's shared pieces, chunk 1's
    // images + chunk kShD-1's shared pieces
    for (unsigned long long c = 0; c + 2 < (unsigned long long)kShD && c < nch; ++c)
      sh_chunk_shared(p, shl, g, c, R, wv, shr + c * kShShared, lane);
    wait_vmcnt<0>();
    for (unsigned long long c = 0; c + 2 < (unsigned long long)kShD && c < nch; ++c)
      if (lane == 0) atomicAdd(arr + c, 1u);
    for (unsigned long long c = 0; c < 2 && c < nch; ++c) {
      sh_chunk_images(shl, c * C, R, wl + c * SLOT);
      if (c + kShD - 2 < nch) sh_chunk_shared(p, shl, g, c + kShD - 2, R, wv, shr + (c + kShD - 2) * kShShared, lane);
    }
  } else if constexpr (ST) {  // steps 0 .. 7 of chunks 0 and 1
    gl1 = glds_lanes<VI, 1>(p, g, k, lane);
    for (unsigned long long c = 0; c < 2 && c < nch; ++c)
      st_chunk_glds(p, gl1, g, c, R, wl + c * SLOT, WS, cml + c * CMS, lane, 0);
  } else if constexpr (RS) {  // chunks 0 and 1 into the two slots (W <= 128: one piece per step)
    gl1 = glds_lanes<VI, 1>(p, g, k, lane);
    for (unsigned long long c = 0; c < 2 && c < nch; ++c)
      map_chunk_glds<VI, C, 1, MAP_RS_AUX>(p, gl1, g, k, c * C, R, wl + c * SLOT, WS, vbase + c * C * VI, cml + c * A, lane,
                               vpiece, p.diag);
  }
  if constexpr (GL) {
    if (ni == 1) gl1 = glds_lanes<VI, 1>(p, g, k, lane);
    else gl2 = glds_lanes<VI, 2>(p, g, k, lane);
    for (unsigned long long c = 0; c + 1 < NB && c < nch; ++c) {
      if (ni == 1) {
        if (p.nt) map_chunk_glds<VI, C, 1, 2>(p, gl1, g, k, c * C, R, wl + c * SLOT, WS, vbase + c * C * VI, cml + c * A, lane);
        else map_chunk_glds<VI, C, 1>(p, gl1, g, k, c * C, R, wl + c * SLOT, WS, vbase + c * C * VI, cml + c * A, lane);
      } else {
        map_chunk_glds<VI, C, 2>(p, gl2, g, k, c * C, R, wl + c * SLOT, WS, vbase + c * C * VI, cml + c * A, lane);
      }
    }
  } else if constexpr (!RS) {
    if (nch > 0) {
      map_chunk_load(regs, p, g, k, 0, R, lane);
      map_chunk_store(regs, wl, vbase, A, WS, R < (unsigned long long)C ? R : C, lane);
      if (nch > 1) map_chunk_load(regs, p, g, k, C, R, lane);
    }
  }

  for (unsigned long long ch = 0; ch < nch; ++ch) {
    const unsigned slot = (unsigned)(ch % NB);
    const u64 *buf = wl + slot * SLOT;
    const u64 *vb = vbase + slot * C * VI;
    const u64 *shx = shr;  // SH: chunk ch's shared slot (clock rows, clock max)
    if constexpr (RS) {
      // Chunk ch sits in slot ch&1 (LDS-DMA, issued two chunks ago), chunk ch+1 in the other slot.
      // Copy chunk ch into registers, refill its slot with chunk ch+2 at once — two chunks stay in
      // flight while this one is tested — and test it whole in registers.  A chunk that is not
      // skipped is written back over its slot (chunk ch+2's copy is dropped and re-issued after the
      // exact loop).
      constexpr int P1 = C + 2;  // LDS-DMA instructions per chunk (map_chunk_glds, one piece per step)
      const bool elig0 = uni(p.spec && cool == 0 && anti && !slow && !direct);
      const int nv = __builtin_popcount(__builtin_amdgcn_readfirstlane(mv.vm));
      const unsigned long long n0 = R - ch * C < (unsigned long long)C ? R - ch * C : C;
      const u64 want = n0 >= 16 ? grp_mask<4>() : (grp_mask<4>() & ((1ull << (4 * n0)) - 1));
      const bool el = elig0 && (unsigned long long)next_row >= ch * C + n0;
      u64 *const img = wl + slot * SLOT;
      u64 *const vsl = vbase + slot * C * VI;
      u64 *const cms = SH ? shr + sh_use * kShShared + 512 : cml + slot * CMS;
      u64 *const shs = shr + sh_use * kShShared;  // SH: chunk ch's shared slot
      shx = shs;
      MAP_TICK();
      if constexpr (SH) {
        // the pieces iteration ch-1 issued may still be in flight: 12 images (chunk ch+1) and,
        // while chunk ch+kShD-1 exists, 2 shared pieces
        if (ch + kShD - 1 < nch) wait_vmcnt<14>();
        else if (ch + 1 < nch) wait_vmcnt<12>();
        else wait_vmcnt<0>();
        // this wave's shared pieces of chunk ch+kShD-2 (issued at iteration ch-2) have landed
        if (ch + kShD - 2 < nch && lane == 0) atomicAdd(arr + sh_sig, 1u);
        // chunk ch's shared slot: every wave's pieces landed
        unsigned spins = 0;
        MAP_TOCK(cy_wait);
        MAP_TICK();
        // (read one iteration ahead, so normally known; after one timeout: no more waits)
        while (!(p.diag & 4) && !sh_late && sh_pre < sh_need && (sh_pre = sh_arrived(arr + sh_use)) < sh_need) {
#ifdef MAP_STATS
          ++st_spin;
#endif
          if (++spins > kShSpin) {
            sh_late = true;
            break;
          }
        }
        MAP_TOCK(cy_arr);
        MAP_TICK();
      } else if constexpr (ST) {  // 9 pieces per chunk (st_chunk_glds)
        if (ch + 1 < nch) wait_vmcnt<9>();
        else wait_vmcnt<0>();
      } else {
        if (ch + 1 < nch) {
          if (vpiece) wait_vmcnt<P1>();
          else wait_vmcnt<P1 - 1>();  // (no values piece)
        } else {
          wait_vmcnt<0>();
        }
      }
      MAP_TOCK(cy_wait);
      MAP_TICK();
      unsigned pre_raw = 0;
      if constexpr (SH) {
        sh_reload(rA, img, shs, A, lane);
        // next chunk's arrival count, read with this chunk's slots
        pre_raw = *reinterpret_cast<const volatile unsigned *>(arr + (sh_use + 1 == kShS ? 0 : sh_use + 1));
      } else if constexpr (ST) {
        st_reload(rA, img, WS, cms, A, lane, 0);
      } else {
        rs_reload(rA, img, WS, vsl, cms, A, lane, vpiece);
      }
      // a whole next chunk with every lane moving a piece: its pieces go out during the test
      const unsigned long long i2 = (ch + 2) * C;
      const bool spread = el && ch + 2 < nch && i2 + C <= R && (2 + VI) * A == 128 && (!SH || ch + kShD < nch);
      // the slot is read: refill it (MAP_RS_LATE, RS path spreading the refill: the DMA hook waits)
      if (SH || ST || !MAP_RS_LATE || !spread) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (SH) sh_pre = __builtin_amdgcn_readfirstlane(pre_raw);
      if constexpr (SH) {
        if (!spread) {
          if (ch + 2 < nch) sh_chunk_images(shl, i2, R, img);
          if (ch + kShD < nch) sh_chunk_shared(p, shl, g, ch + kShD, R, wv, shr + sh_iss * kShShared, lane);
        }
      } else if constexpr (ST) {
        if (ch + 2 < nch && !spread) st_chunk_glds(p, gl1, g, ch + 2, R, img, WS, cms, lane, 0);
      } else {
        if (ch + 2 < nch && !spread)
          map_chunk_glds<VI, C, 1, MAP_RS_AUX>(p, gl1, g, k, i2, R, img, WS, vsl, cms, lane, vpiece, p.diag);
      }
      MAP_TOCK(cy_issue);
      // advance the ring bookkeeping (the rest of the iteration uses sh_use only through shs / cms)
      if constexpr (SH) {
        if (++sh_use == kShS) {
          sh_use = 0;
          sh_need += 4;
        }
        if (++sh_sig == kShS) sh_sig = 0;
      }
      const unsigned sh_iss_now = sh_iss;
      if constexpr (SH) {
        if (++sh_iss == kShS) sh_iss = 0;
      }
      MAP_TICK();
      bool skip = false;
      if constexpr (ST) {  // this wave's steps, then the pair's vote
        const bool batch = MAP_BATCH_ONLY || p.batch;
        u64 verdict;
        if (spread) {
          StDma d{gl1.src0[0] + i2 * gl1.stride[0], gl1.stride[0], img, WS, p.cmax + (g * p.nch + ch + 2) * A + 2 * lane,
                  cms, (unsigned long long)(2 * lane) < A};
          verdict = batch ? st_reg_verdict<true>(rA, rg, present, nv, true, d) : st_reg_verdict<false>(rA, rg, present, nv, true, d);
        } else {
          verdict = batch ? st_reg_verdict<true>(rA, rg, present, nv, el) : st_reg_verdict<false>(rA, rg, present, nv, el);
        }
        const u64 want0 = st_want(n0, 0);
        skip = st_vote(vw + 2 * slot, el && (verdict & want0) == want0, 0, lane);
      } else if (SH && spread) {
        const unsigned long long ic = (ch + kShD) * C + 4 * wv + shl.sub;
        ShDma d{{shl.b[0] + (i2 + shl.sub) * shl.st[0], shl.b[1] + (i2 + shl.sub) * shl.st[1],
                 shl.b[2] + (i2 + shl.sub) * shl.st[2]},
                {4 * shl.st[0], 4 * shl.st[1], 4 * shl.st[2]},
                img,
                shl.cb + (ic < R ? ic : R - 1) * shl.cst,
                shr + sh_iss_now * kShShared + 128 * wv,
                p.cmax + (g * p.nch + ch + kShD) * A + 8 * wv + 2 * lane,
                shr + sh_iss_now * kShShared + 512 + 8 * wv,
                lane < 4};
        skip = (((MAP_BATCH_ONLY || p.batch) ? rs_reg_noop_nv<VI, NP, true>(rA, rg, present, nv, d)
                         : rs_reg_noop_nv<VI, NP, false>(rA, rg, present, nv, d)) &
                want) == want;
      } else if (spread) {
        const int sv = lane / (2 * VI), dw = lane % (2 * VI);
        RsDma d{gl1.src0[0] + i2 * gl1.stride[0], gl1.stride[0], img, WS,
                reinterpret_cast<const unsigned *>(p.vval + g * p.vv_gs + (i2 + (sv < C ? sv : 0)) * p.vv_rs + k * VI) + dw,
                vsl, sv < C, p.cmax + (g * p.nch + i2 / C) * A + 2 * lane, cms, (unsigned long long)(2 * lane) < A,
                vpiece, p.diag};
        skip = (((MAP_BATCH_ONLY || p.batch) ? rs_reg_noop_nv<VI, NP, true>(rA, rg, present, nv, d)
                         : rs_reg_noop_nv<VI, NP, false>(rA, rg, present, nv, d)) &
                want) == want;
      } else if (el) {
        skip = (((MAP_BATCH_ONLY || p.batch) ? rs_reg_noop_nv<VI, NP, true>(rA, rg, present, nv)
                         : rs_reg_noop_nv<VI, NP, false>(rA, rg, present, nv)) &
                want) == want;
      }
      MAP_TOCK(cy_scan);
#ifdef MAP_STATS
      ++st_scan;
      if (!skip) ++st_fail;
#endif
      if (skip) {  // acc.clock.merge of the chunk's replicas (both layouts)
        if ((unsigned long long)lane < A) cs[0] = cs[0] > rA.cm ? cs[0] : rA.cm;
#pragma unroll
        for (int m = 0; m < NP; ++m)
#pragma unroll
          for (int h = 0; h < 2; ++h) rg.cs[m][h] = rs_adv(rg.cs[m][h], rA.cmp[m][h], rg.m1[m][h]);
        continue;
      }
      wait_vmcnt<0>();
      if constexpr (SH) sh_store(rA, img, lane);
      else if constexpr (ST) st_store(rA, img, WS, cms, A, lane, 0);
      else rs_store(rA, img, WS, vsl, cms, A, lane, vpiece);
      if (!vpiece && lane < C * VI) {  // the chunk's values, fetched now (a chunk the exact loop runs)
        const unsigned long long iv = ch * C + lane / VI;
        vsl[lane] = p.vval[g * p.vv_gs + (iv < R ? iv : R - 1) * p.vv_rs + k * VI + lane % VI];
      }
      // the exact loop's scans read max(e, Cs) and TB from LDS
      if ((unsigned long long)lane < A) {
        mirror[(1 + VO) * A + lane] = e[0] > cs[0] ? e[0] : cs[0];
        const u64 lo = cs[0] < m1 ? cs[0] : m1;
        thr[lane] = e[0] > lo ? e[0] : lo;
      }
      if constexpr (ST) st_barrier();  // (A) both waves' steps are back in LDS: the exact loop reads the whole chunk
    }
    if constexpr (GL) {
      // issue chunk ch+NB-1 into the slot chunk ch-1 used, then wait for chunk ch
      const unsigned long long nx = ch + NB - 1;
      MAP_TICK();
      if (nx < nch) {
        const unsigned ns = (unsigned)(nx % NB);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's last LDS reads are done
        if (ni == 1) {
          if (p.nt) map_chunk_glds<VI, C, 1, 2>(p, gl1, g, k, nx * C, R, wl + ns * SLOT, WS, vbase + ns * C * VI, cml + ns * A, lane);
          else map_chunk_glds<VI, C, 1>(p, gl1, g, k, nx * C, R, wl + ns * SLOT, WS, vbase + ns * C * VI, cml + ns * A, lane);
        } else {
          map_chunk_glds<VI, C, 2>(p, gl2, g, k, nx * C, R, wl + ns * SLOT, WS, vbase + ns * C * VI, cml + ns * A, lane);
        }
      }
      MAP_TOCK(cy_issue);
      MAP_TICK();
      const unsigned long long after = (nch - 1 - ch) < (unsigned long long)(NB - 1) ? nch - 1 - ch : NB - 1;
      if (ni == 1) {
        constexpr int P1 = C + 2;
        if (after == 0) wait_vmcnt<0>();
        else if (after == 1) wait_vmcnt<P1>();
        else if (NB > 2 && after == 2) wait_vmcnt<(NB > 2 ? 2 * P1 : 0)>();
        else wait_vmcnt<(NB > 3 ? 3 * P1 : 0)>();
      } else {
        constexpr int P2 = 2 * C + 2;
        if (after == 0) wait_vmcnt<0>();
        else if (after == 1) wait_vmcnt<P2>();
        else if (NB > 2 && after == 2) wait_vmcnt<(NB > 2 ? 2 * P2 : 0)>();
        else wait_vmcnt<(NB > 3 ? 3 * P2 : 0)>();
      }
      MAP_TOCK(cy_wait);
    }
    const unsigned long long i0 = ch * C;
    const unsigned long long n = R - i0 < (unsigned long long)C ? R - i0 : C;
    unsigned long long s = 0;
#pragma unroll 1
    while (s < n) {
      if (uni(kSpec && p.spec && cool == 0 && anti && !slow && !direct)) {
        // steps s.. that provably change nothing, up to the next remove naming this key
        const unsigned long long lim0 = next_row < i0 + n ? next_row - i0 : n;
        const unsigned long long lim = lim0 > s ? lim0 : s;
        unsigned long long j = s;
        if (uni(lim > s)) {
          MAP_TICK();
          const int nv = __builtin_popcount(__builtin_amdgcn_readfirstlane(mv.vm));
          // (the RS path and register staging keep the round-1 scan: the threshold scan's loads in
          // flight would not fit beside their chunk registers)
          u64 noop;
          if constexpr (SH) {
            RsChunk<VI, NP> r;
            sh_reload(r, buf, shx, A, lane, false);
#pragma unroll
            for (int t = 0; t < VI; ++t) r.v[t] = 0;
            noop = rs_lds_own_noop<VI, NP, true>(r, mirror, thr, A, present, nv, lane);
          } else if constexpr (ST)
            noop = st_lds_noop(buf, WS, mirror, thr, A, present, nv, lane);
          else if constexpr (RS)
            noop = rs_lds_noop_nv<VI, (RS ? NP : 1)>(buf, WS, mirror, thr, A, present, nv, lane);
          else
            noop = (p.scan3 && GL) ? map_noop_nv3<VI, LPS, ITM>(buf, (unsigned)WS, (unsigned)A, mirror, thr,
                                                                  present, nv, (unsigned)n, lane)
                           : p.scan2 ? map_noop_nv<VI, LPS, ITM, true>(buf, (unsigned)WS, (unsigned)A, mirror, VO,
                                                                        present, nv, (unsigned)n, lane)
                                     : map_noop_nv<VI, LPS, ITM>(buf, (unsigned)WS, (unsigned)A, mirror, VO, present,
                                                                 nv, (unsigned)n, lane);
          const u64 from = (s >= NS) ? 0 : (~0ull << (LPS * s));
          const u64 upto = (lim >= NS) ? ~0ull : ((1ull << (LPS * lim)) - 1);
          const u64 stop = ~noop & grp_mask<LPS>() & from & upto;
          j = stop ? (unsigned long long)(__builtin_ctzll(stop) / LPS) : lim;
          MAP_TOCK(cy_scan);
          MAP_TICK();
          if ((GL || RS) && s == 0 && j == n) {  // the whole chunk: its staged clock max
            const unsigned long long a = (unsigned long long)lane < A ? lane : A - 1;
            const u64 x = SH ? shx[512 + a] : cml[slot * CMS + a];
            if ((unsigned long long)lane < A) cs[0] = cs[0] > x ? cs[0] : x;
          } else {  // acc.clock.merge of the skipped replicas: every read issued at once, range masked
            const unsigned long long a = (unsigned long long)lane < A ? lane : A - 1;
            u64 mx = cs[0];
#pragma unroll
            for (int u = 0; u < C; ++u) {
              const u64 co = SH ? shx[sh_cword(u, (unsigned)a)] : buf[u * WS + (1 + VI) * A + a];
              const u64 take = ((unsigned long long)u >= s && (unsigned long long)u < j) ? ~0ull : 0ull;
              const u64 x = co & take;
              mx = mx > x ? mx : x;
            }
            if ((unsigned long long)lane < A) cs[0] = mx;
          }
          if (j > s && (unsigned long long)lane < A) {
            mirror[(1 + VO) * A + lane] = e[0] > cs[0] ? e[0] : cs[0];
            const u64 lo = cs[0] < m1 ? cs[0] : m1;
            thr[lane] = e[0] > lo ? e[0] : lo;
          }
          MAP_TOCK(cy_skip);
          if (j == s) cool = 4;  // the scan found nothing to skip: run a few exact steps first
#ifdef MAP_STATS
          ++st_scan; if (j == s) ++st_fail;
#endif
        }
        s = j;
        if (s >= n) break;
      }
      if (cool > 0) --cool;
#ifdef MAP_STATS
      ++st_exact; if (nq) ++st_nq; if (present) ++st_pres;
#endif
      MAP_TICK();
      const unsigned long long i = i0 + s;
      MapStep<APL, VI> in;
      if constexpr (SH) {  // lane = actor: entry / value clocks from the private slot, clock row shared
        const bool on = (unsigned long long)lane < A;
        const unsigned pw = sh_pword((unsigned)s, on ? (unsigned)lane : 0u);
        in.e[0] = on ? buf[pw] : 0;
#pragma unroll
        for (int t = 0; t < VI; ++t) in.c[t][0] = on ? buf[pw + 128 * (1 + t)] : 0;
        in.co[0] = on ? shx[sh_cword((unsigned)s, (unsigned)lane)] : 0;
#pragma unroll
        for (int t = 0; t < VI; ++t) in.v[t] = vb[s * VI + t];
      } else {
        in = map_step_read<APL, VI>(buf + s * WS, vb + s * VI, A, lane);
      }
      ++s;
      // ---- 1. entry join (map.rs:142-210) ----
      const bool p2 = any_nz(in.e);
      if (present && !p2) {
        if (all_ge(in.co, e)) {
          present = false;
          mv.vm = 0;
#pragma unroll
          for (int j = 0; j < APL; ++j) e[j] = 0;
        } else {
          u64 ri[APL];
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            e[j] = e[j] > in.co[j] ? e[j] : 0;
            ri[j] = in.co[j] > e[j] ? in.co[j] : 0;
          }
          if (any_nz(ri)) mv_forget(mv, ri);
        }
      } else if (!present && p2) {
        if (!all_ge(cs, in.e)) {
          u64 ri[APL];
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            e[j] = in.e[j] > cs[j] ? in.e[j] : 0;
            ri[j] = cs[j] > e[j] ? cs[j] : 0;
          }
          mv.vm = 0;
          mv.next = 0;
#pragma unroll
          for (int t = 0; t < VI; ++t) {
            if (any_nz(in.c[t])) {
              u64 x[APL];
#pragma unroll
              for (int j = 0; j < APL; ++j) x[j] = in.c[t][j];
              vforget(x, ri);
              if (any_nz(x)) mv_append(mv, x, in.v[t], ovf);
            }
          }
          present = true;
        }
      } else if (present && p2) {
        u64 dl[APL];
        bool dl_any = false;
#pragma unroll
        for (int j = 0; j < APL; ++j) dl[j] = 0;
        if (!all_eq(e, in.e)) {  // (e == e2 everywhere: common = e, nothing forgotten)
          u64 common[APL];
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            const u64 t0 = e[j] == in.e[j] ? e[j] : 0;
            const u64 t1 = in.e[j] > cs[j] ? in.e[j] : 0;
            const u64 t2 = e[j] > in.co[j] ? e[j] : 0;
            const u64 c = t0 > t1 ? t0 : t1;
            common[j] = c > t2 ? c : t2;
            const u64 m = e[j] > in.e[j] ? e[j] : in.e[j];
            dl[j] = m > common[j] ? m : 0;
          }
          if (!any_nz(common)) {
            present = false;
            mv.vm = 0;
          } else {
            dl_any = any_nz(dl);
          }
#pragma unroll
          for (int j = 0; j < APL; ++j) e[j] = common[j];
        }
        if (present) {
          // MVReg::merge then forget(deleted) (map.rs:183-188, mvreg.rs:112-128)
          unsigned v2m = 0;
#pragma unroll
          for (int t = 0; t < VI; ++t)
            if (any_nz(in.c[t])) v2m |= 1u << t;
          unsigned keep = mv.vm;
#pragma unroll
          for (int q = 0; q < VO; ++q) {
            if (keep & (1u << q)) {
#pragma unroll
              for (int t = 0; t < VI; ++t)
                if ((v2m & (1u << t)) && vlt(mv.c[q], in.c[t])) {
                  keep &= ~(1u << q);
                  break;
                }
            }
          }
          unsigned addm = 0;
#pragma unroll
          for (int t = 0; t < VI; ++t) {
            if (v2m & (1u << t)) {
              bool add = true;
#pragma unroll
              for (int q = 0; q < VO; ++q)
                if ((keep & (1u << q)) && vle(in.c[t], mv.c[q])) {
                  add = false;
                  break;
                }
              if (add) addm |= 1u << t;
            }
          }
          mv.vm = keep;
#pragma unroll
          for (int t = 0; t < VI; ++t)
            if (addm & (1u << t)) mv_append(mv, in.c[t], in.v[t], ovf);
          if (dl_any) mv_forget(mv, dl);
        }
      }

      // ---- 2. deferred removes active at step i (map.rs:213-219, :311-348) ----
      if ((direct ? dp < dend : next_row <= i) || nq > 0 || slow) {
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
        // activate the removes held by replica i that name this key
        while (true) {
          unsigned long long d;
          if (!direct) {
            if (next_row > i) break;
            d = __builtin_amdgcn_readfirstlane(lidx[lp]);
            ++lp;
            next_row = lp < nl ? __builtin_amdgcn_readfirstlane(lrow[lp]) : 0xffffffffu;
          } else {
            if (dp >= dend) break;
            const unsigned long long row = __builtin_amdgcn_readfirstlane(p.def_row[dp]);
            if (row > i) break;
            d = dp++;
            if (!(p.def_keys[d * p.Kw + kw] & kbit)) continue;
          }
          if (!slow && nq < kMapQ) {
#pragma unroll
            for (int q = 0; q < kMapQ; ++q)
              if (q == nq)
#pragma unroll
                for (int j = 0; j < APL; ++j) {
                  const unsigned long long a = lane + 64ull * j;
                  u64 x = a < p.A ? p.def_clock[d * p.A + a] : 0;
                  // consume the load here (one wait per activation): a register still pending
                  // at the loop back-edge would make every later step wait on vmcnt(0), i.e.
                  // on the whole prefetched chunk
                  asm volatile("; rm clock landed" : "+v"(x));
                  rq[q][j] = x;
                }
            ++nq;
          } else {
            slow = true;
          }
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
          const unsigned long long nscan = direct ? dp - dbeg : lp;
          for (unsigned long long x = 0; x < nscan; ++x) {
            const unsigned long long d = direct ? dbeg + x : __builtin_amdgcn_readfirstlane(lidx[x]);
            if (direct && !(p.def_keys[d * p.Kw + kw] & kbit)) continue;
            u64 rm[APL];
#pragma unroll
            for (int j = 0; j < APL; ++j) {
              const unsigned long long a = lane + 64ull * j;
              rm[j] = a < p.A ? p.def_clock[d * p.A + a] : 0;
            }
            if (__builtin_amdgcn_readfirstlane(p.def_row[d]) == i || !all_ge(cs, rm)) {
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
            mv.vm = 0;
          } else {
            mv_forget(mv, ceil);
          }
        }
      }

      // ---- 3. acc.clock.merge(other.clock) (map.rs:217) ----
#pragma unroll
      for (int j = 0; j < APL; ++j) cs[j] = cs[j] > in.co[j] ? cs[j] : in.co[j];

      if (kSpec) {  // refresh the state mirror for the next scan
        anti = mv_antichain(mv);
        if ((unsigned long long)lane < A) {
          mirror[lane] = e[0];
          mirror[(1 + VO) * A + lane] = e[0] > cs[0] ? e[0] : cs[0];
          int r = 0;  // own value clocks compacted into slots 0..nv-1 (any order)
          m1 = ~0ull;
#pragma unroll
          for (int q = 0; q < VO; ++q)
            if (mv.vm & (1u << q)) {
              const u64 x = mv.c[q][0];
              mirror[(1 + r++) * A + lane] = x;
              const u64 x1 = x != 0 ? x - 1 : ~0ull;
              m1 = x1 < m1 ? x1 : m1;
            }
          const u64 lo = cs[0] < m1 ? cs[0] : m1;
          thr[lane] = e[0] > lo ? e[0] : lo;
          thr[A + lane] = e[0] > 0 ? e[0] - 1 : m1;
        }
      }
      MAP_TOCK(cy_exact);
    }
    if constexpr (RS) {
      // the register operands from the fold state after the exact loop
      if ((unsigned long long)lane < A) {
        csm[lane] = cs[0];
        m1m[lane] = m1;
      }
      {
        const int nvx = __builtin_popcount(__builtin_amdgcn_readfirstlane(mv.vm));  // own values, compacted
#pragma unroll
        for (int m = 0; m < NP; ++m) {
          const unsigned a0 = ST ? st_a0(lane, m) : rs_a0<SH>(lane, m);
          const unsigned long long a = a0 < A ? a0 : A - 2;
          rg.ea[m] = lds2(mirror + a);
          rg.to[m] = lds2(thr + A + a);
          rg.m1[m] = lds2(m1m + a);
          rg.cs[m] = lds2((MAP_TB_INC ? thr : csm) + a);
#pragma unroll
          for (int q = 0; q < 3; ++q) rg.sq[q][m] = q < nvx ? lds2(mirror + (1 + q) * A + a) : u64x2{0, 0};
        }
        if constexpr (ST) {  // (B) the partner reloads its operands from the same mirror
          if (lane == 0) *reinterpret_cast<volatile unsigned *>(spst) = (present ? 1u : 0u) | ((unsigned)nvx << 1);
          st_barrier();
        }
      }
      // re-issue chunk ch+2 into the slot the exact loop used
      if (SH && ch + 2 < nch) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        sh_chunk_images(shl, (ch + 2) * C, R, wl + slot * SLOT);
      } else if (ST && ch + 2 < nch) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        st_chunk_glds(p, gl1, g, ch + 2, R, wl + slot * SLOT, WS, cml + slot * CMS, lane, 0);
      } else if (ch + 2 < nch) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        map_chunk_glds<VI, C, 1, MAP_RS_AUX>(p, gl1, g, k, (ch + 2) * C, R, wl + slot * SLOT, WS, vbase + slot * C * VI,
                                 cml + slot * CMS, lane, vpiece, p.diag);
      }
    }
    if constexpr (!GL && !RS) {
      if (ch + 1 < nch) {  // stage the next chunk (its loads were issued a whole chunk ago)
        const unsigned long long nn = R - (ch + 1) * C < (unsigned long long)C ? R - (ch + 1) * C : C;
        const unsigned ns = (unsigned)((ch + 1) % NB);
        map_chunk_store(regs, wl + ns * SLOT, vbase + ns * C * VI, A, WS, nn, lane);
        if (ch + 2 < nch) map_chunk_load(regs, p, g, k, (ch + 2) * C, R, lane);
      }
    }
  }
  if (direct && dp < dend) bad = 1;  // a row >= R was never reached

#ifdef MAP_STATS
  cy_all = __builtin_amdgcn_s_memtime() - cy_all;
  if (lane == 0 && (k % 97) == 0)
    printf("k=%llu exact=%u scan=%u fail=%u nq=%u pres=%u nl=%llu spin=%u | cyc all=%llu issue=%llu wait=%llu arr=%llu scan=%llu skip=%llu exact=%llu\n",
           k, st_exact, st_scan, st_fail, st_nq, st_pres, nl, st_spin, cy_all, cy_issue, cy_wait, cy_arr, cy_scan, cy_skip, cy_exact);
#endif
  // ---- egress: slots in Vec order (ascending order key) ----
  const int nv = __builtin_popcount(mv.vm);
  if (nv > (int)p.Vout) ovf |= 1;
  int rank[VO];
#pragma unroll
  for (int q = 0; q < VO; ++q) {
    rank[q] = -1;
    if (mv.vm & (1u << q)) {
      int r = 0;
#pragma unroll
      for (int q2 = 0; q2 < VO; ++q2)
        if ((mv.vm & (1u << q2)) && mv.seq[q2] < mv.seq[q]) ++r;
      rank[q] = r;
    }
  }
  const unsigned long long gk = g * p.K + k;
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = lane + 64ull * j;
    if (a < p.A) {
      p.o_ec[gk * p.A + a] = present ? e[j] : 0;
      if (k == 0) p.o_clock[g * p.A + a] = cs[j];
      for (unsigned long long o = 0; o < p.Vout; ++o) {
        u64 x = 0;
#pragma unroll
        for (int q = 0; q < VO; ++q)
          if (rank[q] == (int)o) x = mv.c[q][j];
        p.o_vclk[(gk * p.Vout + o) * p.A + a] = x;
      }
    }
  }
  if (lane == 0) {
    for (unsigned long long o = 0; o < p.Vout; ++o) {
      u64 v = 0;
#pragma unroll
      for (int q = 0; q < VO; ++q)
        if (rank[q] == (int)o) v = mv.v[q];
      p.o_vval[gk * p.Vout + o] = v;
    }
    if (p.o_nval) p.o_nval[gk] = present ? (unsigned)nv : 0u;
    const unsigned f = (unsigned)ovf | (bad ? 2u : 0u) | (sh_late ? 8u : 0u);
    if (f) atomicOr(p.o_flags + g, f);
  }
}

}  // namespace crdt

using namespace crdt;

// Max of the replica clocks of each chunk of C replicas, [G][nch][A]: the clock merge of a
// chunk the fold skips entirely (one block per (group, chunk), lane = actor).
__global__ __launch_bounds__(64) void map_chunk_max_kernel(const u64 *clock, long long c_rs, long long c_gs,
                                                           unsigned long long R, unsigned long long A,
                                                           unsigned long long nch, unsigned C, u64 *out) {
  const unsigned long long g = blockIdx.x / nch, ch = blockIdx.x % nch;
  const unsigned long long i0 = ch * C, i1 = R < i0 + C ? R : i0 + C;
  for (unsigned long long a = threadIdx.x; a < A; a += 64) {
    u64 m = 0;
    for (unsigned long long i = i0; i < i1; ++i) {
      const u64 x = __builtin_nontemporal_load(clock + g * c_gs + i * c_rs + a);
      m = m > x ? m : x;
    }
    out[(g * nch + ch) * A + a] = m;
  }
}

template <int APL, int VI, int VO, int CM, int NB, bool GL, int ITM, int NP = 0, bool ST = false>
static hipError_t launch_map_it(const MapPlan &p, unsigned long long blocks, hipStream_t s) {
  constexpr bool RS = NP > 0;
  constexpr int C = (GL || RS) ? CM : MapChunk<APL, VI, CM>::C;
  const size_t W = (2 + VI) * p.A;
  // (the kernel's PW: slots, values, remove lists, mirror, clock-max copies, thresholds, ST words)
  const size_t lds = (size_t)NB * C * ((RS ? map_ws_rs(W) : map_ws(W)) + VI) * sizeof(u64) + kMapL * 2 * sizeof(unsigned) +
                     (2 + VO) * p.A * sizeof(u64) + ((GL || RS) ? (ST ? 2 : 1) * NB * p.A * sizeof(u64) : 0) +
                     4 * p.A * sizeof(u64) + (ST ? 4 * sizeof(u64) : 0);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  auto *fn = &map_fold_kernel<APL, VI, VO, CM, NB, GL, ITM, NP, false, ST>;
  if (lds > 64 * 1024) {  // beyond the default dynamic-LDS limit (gfx950 has 160 KB per CU)
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(ST ? 128 : 64), lds, s, p);
  return hipGetLastError();
}

// RS path (A <= 32 even, V <= 2, 16-replica chunks): NP actor pairs per lane, LPS = 4 scan lanes per
// step so the LDS scans of the exact loop unroll ceil(A / 4) iterations.
template <int VI>
static hipError_t launch_map_rs(const MapPlan &p, unsigned long long blocks, hipStream_t s) {
  // two waves per key at config 4's shape (A = 32, V = 2)
  if constexpr (VI == 2) {
    if (p.st && p.A == 32) return launch_map_it<1, 2, 4, 16, 2, false, 4, 2, true>(p, blocks, s);
  }
  if (p.A <= 8) return launch_map_it<1, VI, 4, 16, 2, false, 2, 1>(p, blocks, s);
  if (p.A <= 16) return launch_map_it<1, VI, 4, 16, 2, false, 4, 2>(p, blocks, s);
  return launch_map_it<1, VI, 4, 16, 2, false, 8, 4>(p, blocks, s);
}

// SH path (A = 32, V = 2, K % 4 == 0): blocks of four key waves, the shared clock-row ring after
// the four wave regions.
static hipError_t launch_map_sh(const MapPlan &p, unsigned long long blocks, hipStream_t s) {
  constexpr int VI = 2, VO = 4, C = 16, NB = 2;
  const size_t PW = NB * kShSlot + NB * C * VI + kMapL + (2 + VO) * p.A + 4 * p.A;
  const size_t lds = (4 * PW + kShS * kShShared) * sizeof(u64) + kShS * sizeof(unsigned);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  auto *fn = &map_fold_kernel<1, VI, VO, C, NB, false, 8, 4, true>;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fn, dim3((unsigned)(blocks / 4)), dim3(256), lds, s, p);
  return hipGetLastError();
}

// Scan shape: NS steps per scan (C rounded up to a power of two, <= 16), LPS = 64 / NS lanes per
// step, ceil(A / LPS) iterations rounded up to a power of two (A <= 64 when the scan runs).
template <int APL, int VI, int VO, int CM, int NB, bool GL>
static hipError_t launch_map(const MapPlan &p, unsigned long long blocks, hipStream_t s) {
  if constexpr (APL != 1 || VO > 4) {
    return launch_map_it<APL, VI, VO, CM, NB, GL, 2>(p, blocks, s);  // no scan: A > 64 or a wide state
  } else {
    constexpr int C = GL ? CM : MapChunk<APL, VI, CM>::C;
    constexpr int NS = C > 8 ? 16 : (C > 4 ? 8 : (C > 2 ? 4 : 2));
    constexpr int LPS = 64 / NS;
    const unsigned long long it = (p.A + LPS - 1) / LPS;
    if (it <= 2) return launch_map_it<APL, VI, VO, CM, NB, GL, 2>(p, blocks, s);
    if (it <= 4) return launch_map_it<APL, VI, VO, CM, NB, GL, 4>(p, blocks, s);
    if constexpr (LPS >= 8) {
      return launch_map_it<APL, VI, VO, CM, NB, GL, 8>(p, blocks, s);
    } else {
      if (it <= 8) return launch_map_it<APL, VI, VO, CM, NB, GL, 8>(p, blocks, s);
      return launch_map_it<APL, VI, VO, CM, NB, GL, 16>(p, blocks, s);
    }
  }
}

// Register-staged fold for VI input / 2*VI state value slots (any shape within the limits).
template <int APL>
static hipError_t launch_map_vi(const MapPlan &p, int VI, unsigned long long blocks, hipStream_t s) {
  switch (VI) {
    case 1: return launch_map<APL, 1, 2, 16, 2, false>(p, blocks, s);
    case 2: return launch_map<APL, 2, 4, 16, 2, false>(p, blocks, s);
    case 4: return launch_map<APL, 4, 8, 16, 2, false>(p, blocks, s);
    default: return launch_map<APL, 8, 16, 16, 2, false>(p, blocks, s);  // no scan: exact steps only
  }
}

// LDS-DMA fold (A <= 64, even; VI = V <= 2; 4 state values): 16-replica chunks in 2 slots
// (default) or 8-replica chunks in 4 slots.
template <int VI>
static hipError_t launch_map_glds(const MapPlan &p, int cm, int nb, unsigned long long blocks, hipStream_t s) {
  if (cm == 8 && nb == 4) return launch_map<1, VI, 4, 8, 4, true>(p, blocks, s);
  return launch_map<1, VI, 4, 16, 2, true>(p, blocks, s);
}

// Smallest VI (1, 2, 4, 8) with VI >= V and 2*VI >= min(16, want): the fold state holds 2*VI values.
static int map_vi(size_t V, size_t want) {
  int VI = 1;
  while ((size_t)VI < V || (size_t)(2 * VI) < (want < 16 ? want : 16)) VI *= 2;
  return VI > 8 ? 8 : VI;
}

static bool aligned16(const void *x) { return (reinterpret_cast<uintptr_t>(x) & 15) == 0; }

// doff: the device-offset variant's def_off (in->def_off is then NULL and Ddev the pool length)
static int map_lub_impl(crdt_ctx *ctx, const crdt_map_batch *in, const u64 *doff, size_t Ddev, crdt_map_out *out) {
  const size_t G = in->G, R = in->R, K = in->K, A = in->A, V = in->V, Vout = out->Vout;
  if (G == 0 || K == 0 || A == 0) return CRDT_OK;
  if (!out->clock || !out->ec || !out->vclk || !out->vval || !out->flags)
    return fail(ctx, CRDT_EINVAL, "map_lub_many: NULL output");
  if (Vout == 0) return fail(ctx, CRDT_EINVAL, "map_lub_many: Vout must be >= 1");
  if (R > 0 && (!in->clock || !in->ec || (V > 0 && (!in->vclk || !in->vval))))
    return fail(ctx, CRDT_EINVAL, "map_lub_many: NULL input");
  // past the fast kernels' register shapes: the workgroup-per-key fold (map_wide.hip)
  const bool wide = A > 256 || V > 8;
  if (Vout > 64) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: Vout = %zu > 64", Vout);
  if (G * K > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: G*K too large");
  if (R > 0xfffffffeULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: R too large");
  const size_t D = doff ? Ddev : (in->def_off && G > 0) ? in->def_off[G] - in->def_off[0] : 0;
  if (in->def_off && in->def_off[0] != 0) return fail(ctx, CRDT_EINVAL, "map_lub_many: def_off[0] must be 0");
  if (D > 0 && (!in->def_row || !in->def_clock || !in->def_keys || !out->def_keep || !out->def_keys))
    return fail(ctx, CRDT_EINVAL, "map_lub_many: deferred buffers missing");
  if (D > 0xffffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_lub_many: too many deferred");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const size_t Kw = (K + 63) / 64;
  const size_t want = out->Vstate > Vout ? out->Vstate : Vout;

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
  p.spec = ctx->tune.map_spec;
  p.nt = ctx->tune.map_nt;
  p.scan2 = ctx->tune.map_scan2 && A % 2 == 0;
  p.scan3 = ctx->tune.map_scan3;
  p.lazyv = ctx->tune.map_lazyv;
  p.batch = ctx->tune.map_batch;
  p.diag = ctx->tune.map_diag;
  if (int rc = device_fill(ctx, out->flags, G * sizeof(unsigned), 0)) return rc;
  // LDS-DMA staging when every step image is whole 16-byte pieces (A even, 16-byte aligned
  // rows and strides) and the state fits 4 values; register staging otherwise
  const bool even = ((p.c_rs | p.c_gs | p.e_rs | p.e_gs | p.vc_rs | p.vc_gs) & 1) == 0;
  const bool glds = !wide && ctx->tune.map_glds && R > 0 && A <= 64 && (A & 1) == 0 && (V == 1 || V == 2) &&
                    want <= 4 && even && aligned16(p.clock) && aligned16(p.ec) && aligned16(p.vclk) &&
                    G * ((R + 7) / 8) < 0x7fffffffULL;
  // the RS path: register-staged whole-chunk skip, LDS only for chunks it cannot skip
  const bool rs = glds && ctx->tune.map_rs && A <= 32;
  const unsigned gC = (!rs && ctx->tune.map_chunk == 8 && ctx->tune.map_ring == 4) ? 8 : 16;  // launch_map_glds
  // scratch: [def_off copy | chunk clock maxima]
  const size_t off_b = D > 0 || doff ? ((G + 1) * sizeof(size_t) + 255) / 256 * 256 : 0;
  if (glds) p.nch = (R + gC - 1) / gC;
  p.st = rs && ctx->tune.map_st && A == 32 && V == 2 && !(ctx->tune.map_sh && K % 4 == 0);
  const size_t cm_b = glds ? G * p.nch * A * sizeof(u64) : 0;
  if (off_b + cm_b > 0)
    if (int rc = ensure_scratch(ctx, off_b + cm_b)) return rc;
  if (doff && D == 0)  // no pool: only the offsets' check (every entry must be 0)
    if (int rc = stage_def_off_dev(ctx, doff, (size_t *)ctx->scratch, G, 0, nullptr, out->flags)) return rc;
  if (D > 0) {
    // the kernel walks def_off on the device: stage it (the caller's array may be freed), or check
    // and clamp the caller's device offsets into the same place (flags bit 1 of a bad group)
    if (doff) {
      if (int rc = stage_def_off_dev(ctx, doff, (size_t *)ctx->scratch, G, D, nullptr, out->flags)) return rc;
    } else if (int rc = stage_h2d(ctx, ctx->scratch, in->def_off, (G + 1) * sizeof(size_t))) {
      return rc;
    }
    p.def_off = reinterpret_cast<const size_t *>(ctx->scratch);
    p.def_row = in->def_row;
    p.def_clock = (const u64 *)in->def_clock;
    p.def_keys = (const u64 *)in->def_keys;
  }
  const unsigned long long blocks = G * K;
  hipError_t he;
  if (wide) {
    if (int rc = map_lub_wide(ctx, in, p.def_off, out)) return rc;
    he = hipSuccess;
  } else {
  if (glds) {
    u64 *cm = reinterpret_cast<u64 *>(static_cast<char *>(ctx->scratch) + off_b);
    p.cmax = cm;
    // (its own timer section: "map_fold" times the fold kernel alone, as rocprofv3 does)
    timing_begin(ctx, "map_chunk_max");
    hipLaunchKernelGGL(map_chunk_max_kernel, dim3((unsigned)(G * p.nch)), dim3(64), 0, ctx->stream, p.clock,
                       p.c_rs, p.c_gs, (unsigned long long)R, (unsigned long long)A, p.nch, gC, cm);
    timing_end(ctx);
  }
  timing_begin(ctx, "map_fold");
  if (glds) {
    if (rs && ctx->tune.map_sh && A == 32 && V == 2 && K % 4 == 0)
      he = launch_map_sh(p, blocks, ctx->stream);
    else if (rs)
      he = V == 1 ? launch_map_rs<1>(p, blocks, ctx->stream) : launch_map_rs<2>(p, blocks, ctx->stream);
    else
      he = V == 1 ? launch_map_glds<1>(p, ctx->tune.map_chunk, ctx->tune.map_ring, blocks, ctx->stream)
                  : launch_map_glds<2>(p, ctx->tune.map_chunk, ctx->tune.map_ring, blocks, ctx->stream);
  } else {
    const int VI = map_vi(V, want);
    if (A <= 64) he = launch_map_vi<1>(p, VI, blocks, ctx->stream);
    else if (A <= 128) he = launch_map_vi<2>(p, VI, blocks, ctx->stream);
    else he = launch_map_vi<4>(p, VI, blocks, ctx->stream);
  }
  timing_end(ctx);
  }
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
  return launch_deferred(ctx, in->def_off, q, doff);
}

extern "C" int crdt_map_lub_many(crdt_ctx *ctx, const crdt_map_batch *in, crdt_map_out *out) {
  if (ctx && ctx->mem_kind == CRDT_MEM_HOST) return crdt::map_lub_many_host(ctx, in, out);
  CRDT_CHECK_CTX(ctx);
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "map_lub_many: NULL batch/out");
  return map_lub_impl(ctx, in, nullptr, 0, out);
}

extern "C" int crdt_map_lub_many_doff(crdt_ctx *ctx, const crdt_map_batch *in, const uint64_t *def_off, size_t D,
                                      crdt_map_out *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "map_lub_many_doff: NULL batch/out");
  if (in->def_off) return fail(ctx, CRDT_EINVAL, "map_lub_many_doff: in->def_off must be NULL");
  if (!def_off && D) return fail(ctx, CRDT_EINVAL, "map_lub_many_doff: D > 0 without def_off");
  return map_lub_impl(ctx, in, (const u64 *)def_off, D, out);
}
