// Batched CmRDT::apply of Map<K, GCounter> / Map<K, PNCounter> (round 5): Map::apply (map.rs:119-137)
// with the counter's apply inside (gcounter.rs:36-42: the value op is a Dot, VClock::apply;
// pncounter.rs:59-68: a Dot and a direction, applied to P or N), apply_keyset_rm (:318-348) and
// apply_deferred (:311-316).  State s applies its ops [op_off[s], op_off[s+1]) in order, in place.
//
// One wave per state (ops are ordered: the "seen" test and the deferred removes depend on what came
// before), lane l holding actors l + 64 j of every row (j < APL), the map clock in registers, the
// state's deferred removes (rm clock + key bitmap) staged in LDS for the whole stream and written
// back at the end.  Per op:
//  * Up { dot (a, c), key k, op (va, vc, dir) }: skipped when clock[a] >= c (seen); else the entry
//    clock's word a and the value row dir's word va take the max with c / vc (VClock::apply), the map
//    clock's word a too, then every deferred remove is re-applied (apply_deferred): its keys' entries
//    forget its clock (an emptied entry is dropped: all-zero rows; a surviving one's value rows
//    forget it too) and it stays deferred while !(clock >= rm);
//  * Rm { clock rm, keyset }: the keys' entries forget rm as above, then rm is deferred unless
//    clock >= rm (an equal clock already deferred unions its key set).
// The forgets of apply_deferred commute (each forget is idempotent; an entry emptied by one stays
// empty), so the HashMap's iteration order does not matter.  Each row word is read and written by
// the lane owning its actor (lane-local), the deferred slots live in LDS.
#include "common.hpp"

namespace crdt {

// waves per SIMD asked of the register allocator for A <= 128 (build option; A/B in
// profiles/r05_vapply_wpe_ab.log); the wider instances keep the compiler's choice (they would spill)
// op headers batched 64 at a time into lanes and read by v_readlane (build option; 0 = one global
// read of each field per op).  With it the kernel runs at 7 waves per SIMD (room for the batch's
// registers): 1.89 ms against 2.17 ms for per-op reads at 8 and 2.30 ms for the batch at 8
// (profiles/r05_vapply_hdr_ab.log, r05_mca_h1w_ab.log)
// Deferred slots held in LDS per state (the rest of the caller's Dcap slots are used in place, in global
// memory: exact up to Dcap, slower past kMcaDl).  16 = the round-5 LDS footprint.
constexpr size_t kMcaDl = 16;
#ifndef CRDT_MCA_HDR
#define CRDT_MCA_HDR 1
#endif
#ifndef CRDT_MCA_WPE
#define CRDT_MCA_WPE 7
#endif
#ifndef CRDT_MCA_WPE1  // the pass-1 instance (Dcap past the LDS slots): 6, 2.185 vs 2.334 ms at 7
#define CRDT_MCA_WPE1 6    // (profiles/r06_apply_ab.log)
#endif

struct MapCounterApplyPlan {
  u64 *clock, *ec, *val;
  unsigned long long c_s, e_s, v_s;  // state strides (words)
  unsigned long long N, K, A, W, Kw, Dcap;
  unsigned long long Dl;  // deferred slots held in LDS (<= Dcap); slots Dl .. Dcap-1 stay in def_clock / def_keys
  u64 *def_clock, *def_keys;
  unsigned *def_count;
  const u64 *op_off;
  const uint8_t *kind;
  const uint32_t *actor, *key, *vactor;
  const u64 *counter, *vcounter;
  const uint8_t *vdir;
  const uint32_t *clk_row;
  const u64 *clk_pool;
  unsigned long long n_clk_rows;
  const u64 *key_off;
  const uint32_t *keys;
  unsigned long long n_keys, n_ops;
  unsigned *status;
  unsigned wpb;  // waves per block
  u64 *resume;   // [N] (Dcap > Dl): op offset where the state's stream continues in the tier-2 pass, or kMcaDone
};
constexpr u64 kMcaDone = ~0ull;

__device__ __forceinline__ unsigned rl32(unsigned x, int i) { return (unsigned)__builtin_amdgcn_readlane((int)x, i); }
__device__ __forceinline__ u64 rl64(u64 x, int i) {
  return ((u64)rl32((unsigned)(x >> 32), i) << 32) | rl32((unsigned)x, i);
}

// TIER false: every state, its deferred list in the Dl LDS slots only; a state whose list needs slot
// Dl (Dcap > Dl) stores itself and records the op to continue from (resume[s]).  TIER true: those
// states alone, the list's slots past Dl used in place in the caller's slot arrays (one branch per
// access).  Two passes rather than one body with the branch: that body compiles the slot accesses to
// flat instructions and cost every state ~40% (2.73 vs 1.90 ms at the bench shape).
template <int APL, int PASS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(APL <= 2 ? (PASS == 1 ? CRDT_MCA_WPE1 : CRDT_MCA_WPE) : 1))) void map_counter_apply_kernel(MapCounterApplyPlan p) {
  extern __shared__ u64 lds[];
  const int lane = (int)(threadIdx.x % kWave), wv = (int)(threadIdx.x / kWave);
  const unsigned long long s = (unsigned long long)blockIdx.x * p.wpb + wv;
  if (wv >= (int)p.wpb || s >= p.N) return;  // (whole waves)
  constexpr bool TIER = PASS == 2;
  if constexpr (TIER) {
    if (p.resume[s] == kMcaDone) return;
  }
  const unsigned long long A = p.A, K = p.K, W = p.W, Kw = p.Kw, Dcap = p.Dcap, Dl = p.Dl;
  // The Map's deferred removes: slots d < Dl in LDS, slots Dl <= d < Dcap in the caller's own slot
  // arrays (global memory: a long list runs slower, never incomplete below Dcap)
  u64 *sclk = lds + (unsigned long long)wv * Dl * (A + Kw);  // [Dl][A] rm clocks
  u64 *skey = sclk + Dl * A;                                 // [Dl][Kw] key bitmaps
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
      if (PASS == 1) p.resume[s] = kMcaDone;
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
  // pass 2 continues with pass 1's status bits and from a state whose first deferred pass is not known
  // to have run (full = true below re-forgets every listed key: exact either way)
  unsigned st = TIER ? p.status[s] : 0u, peak = dcnt;  // peak: the most slots held (vacated ones are zeroed)
  const unsigned long long start = TIER ? ob + p.resume[s] : ob;
  u64 *C = p.clock + s * p.c_s, *E = p.ec + s * p.e_s, *V = p.val + s * p.v_s;
  auto word = [&](int j) { return (unsigned long long)lane + 64ull * j; };
  u64 c[APL];
#pragma unroll
  for (int j = 0; j < APL; ++j) c[j] = word(j) < A ? C[word(j)] : 0ull;
  for (unsigned d = 0; d < dcnt && d < Dl; ++d) {
    for (unsigned long long a = (unsigned long long)lane; a < A; a += kWave) sclk[d * A + a] = gclk[d * A + a];
    for (unsigned long long w = (unsigned long long)lane; w < Kw; w += kWave) skey[d * Kw + w] = gkey[d * Kw + w];
  }

  // the clock's word of actor a (uniform)
  auto clock_of = [&](unsigned a) -> u64 {
    u64 x = 0;
#pragma unroll
    for (int j = 0; j < APL; ++j)
      if ((unsigned)j == a / 64) x = c[j];
    return __shfl(x, (int)(a % 64));
  };
  // clock >= r (every word): r is dominated
  auto dominated = [&](const u64 (&r)[APL]) {
    bool b = false;
#pragma unroll
    for (int j = 0; j < APL; ++j) b = b || r[j] > c[j];
    return __ballot(b) == 0;
  };
  // key k's entry forgets r: dropped (all-zero rows) when its clock empties, else its value too
  auto key_rm = [&](unsigned long long k, const u64 (&r)[APL]) {
    u64 e[APL];
    bool live = false, left = false;
#pragma unroll
    for (int j = 0; j < APL; ++j) {
      e[j] = word(j) < A ? E[k * A + word(j)] : 0ull;
      live = live || e[j] != 0;
      e[j] = e[j] > r[j] ? e[j] : 0ull;
      left = left || e[j] != 0;
    }
    if (!__ballot(live)) return;  // no entry
    const bool keep = __ballot(left) != 0;
#pragma unroll
    for (int j = 0; j < APL; ++j)
      if (word(j) < A) E[k * A + word(j)] = e[j];
    for (unsigned long long w = 0; w < W; ++w) {
#pragma unroll
      for (int j = 0; j < APL; ++j) {
        if (word(j) >= A) continue;
        u64 *vp = V + (k * W + w) * A + word(j);
        const u64 v = *vp;
        const u64 nv = keep && v > r[j] ? v : 0ull;
        if (nv != v) *vp = nv;
      }
    }
  };
  // apply_deferred re-forgets every key of every deferred remove (map.rs:311-316).  After one full
  // pass each remove's keys are forgotten by its clock, and later ops keep that (an Rm forgets its own
  // keys by its clock; forgets are idempotent and commute) except an Up, which changes only its own
  // key's rows: every later pass re-forgets that key alone — the same rows the full pass would
  // change.  The first pass stays full (the input state need not hold the invariant).
  bool full = true;
  auto apply_deferred = [&](unsigned long long kk) {
    unsigned o = 0;
    for (unsigned d = 0; d < dcnt; ++d) {
      u64 r[APL];
#pragma unroll
      for (int j = 0; j < APL; ++j) r[j] = word(j) < A ? clk(d, word(j)) : 0ull;
      if (full) {
        for (unsigned long long w = 0; w < Kw; ++w) {
          u64 bits = key(d, w);
          while (bits) {
            const unsigned long long k = w * 64 + (unsigned long long)__builtin_ctzll(bits);
            bits &= bits - 1;
            if (k < K) key_rm(k, r);
          }
        }
      } else if ((key(d, kk / 64) >> (kk % 64)) & 1ull) {
        key_rm(kk, r);
      }
      if (dominated(r)) continue;  // no longer deferred
      if (o != d) {
        for (unsigned long long a = (unsigned long long)lane; a < A; a += kWave) set_clk(o, a, clk(d, a));
        for (unsigned long long w = (unsigned long long)lane; w < Kw; w += kWave) set_key(o, w, key(d, w));
      }
      ++o;
    }
    dcnt = o;
    full = false;
  };

  // pass 1: the op where pass 2 continues (offset within the state's stream; < 2^32, checked on the host)
  unsigned resume_at = 0xffffffffu;
  // Op headers in batches of 64: lane i loads op o0 + i's fields (coalesced, all in flight
  // together) and op o's fields reach the wave by v_readlane, not by a global round trip per op.
  for (unsigned long long o0 = start; o0 < oe; o0 += kWave) {
    const unsigned long long mo = o0 + (unsigned long long)lane;
    const bool hin = CRDT_MCA_HDR && mo < oe;
    const unsigned h_kind = hin ? p.kind[mo] : 0u;
    const unsigned h_a = hin ? p.actor[mo] : 0u, h_va = hin ? p.vactor[mo] : 0u, h_k = hin ? p.key[mo] : 0u;
    const u64 h_c = hin ? p.counter[mo] : 0ull, h_vc = hin ? p.vcounter[mo] : 0ull;
    const unsigned h_dir = hin && p.vdir ? p.vdir[mo] : 0u;
    const unsigned h_rr = hin && p.clk_row ? p.clk_row[mo] : 0xffffffffu;
    const u64 h_kb = hin ? p.key_off[mo] : 0ull, h_ke = hin ? p.key_off[mo + 1] : 0ull;
    const int nb = (int)(oe - o0 < (unsigned long long)kWave ? oe - o0 : (unsigned long long)kWave);
  for (int i = 0; i < nb; ++i) {
    const unsigned long long o = o0 + (unsigned long long)i;
    const unsigned kind = CRDT_MCA_HDR ? rl32(h_kind, i) : p.kind[o];
    if (kind == 0) {  // ---- Op::Up
      const unsigned a = CRDT_MCA_HDR ? rl32(h_a, i) : p.actor[o], va = CRDT_MCA_HDR ? rl32(h_va, i) : p.vactor[o];
      const unsigned long long k = CRDT_MCA_HDR ? rl32(h_k, i) : p.key[o];
      const u64 cnt = CRDT_MCA_HDR ? rl64(h_c, i) : p.counter[o], vc = CRDT_MCA_HDR ? rl64(h_vc, i) : p.vcounter[o];
      const unsigned dir = CRDT_MCA_HDR ? rl32(h_dir, i) : (p.vdir ? p.vdir[o] : 0u);
      if (a >= A || va >= A || k >= K || dir >= W) {
        st |= 2u;
        continue;
      }
      if (clock_of(a) >= cnt) continue;  // seen (map.rs:123-126)
      if ((unsigned long long)lane == a % 64) {
        u64 *ep = E + k * A + a;
        if (*ep < cnt) *ep = cnt;  // entry.clock.apply(dot)
#pragma unroll
        for (int j = 0; j < APL; ++j)
          if ((unsigned)j == a / 64 && c[j] < cnt) c[j] = cnt;  // self.clock.apply(dot)
      }
      if ((unsigned long long)lane == va % 64) {
        u64 *vp = V + (k * W + dir) * A + va;
        if (*vp < vc) *vp = vc;  // entry.val.apply(op)
      }
      apply_deferred(k);
    } else if (kind == 1) {  // ---- Op::Rm -> apply_keyset_rm
      const unsigned rr = CRDT_MCA_HDR ? rl32(h_rr, i) : (p.clk_row ? p.clk_row[o] : 0xffffffffu);
      const u64 kb = CRDT_MCA_HDR ? rl64(h_kb, i) : p.key_off[o], ke = CRDT_MCA_HDR ? rl64(h_ke, i) : p.key_off[o + 1];
      if (rr >= p.n_clk_rows || ke < kb || ke > p.n_keys) {
        st |= 2u;
        continue;
      }
      u64 r[APL];
#pragma unroll
      for (int j = 0; j < APL; ++j) r[j] = word(j) < A ? p.clk_pool[(unsigned long long)rr * A + word(j)] : 0ull;
      for (u64 i = kb; i < ke; ++i) {
        const unsigned long long k = p.keys[i];
        if (k < K) key_rm(k, r);
        else st |= 2u;
      }
      if (dominated(r)) continue;  // every key this clock has seen, we have seen
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
          st |= 1u;  // deferred capacity exceeded: the state is incomplete
          continue;
        }
        slot = (int)dcnt++;
        if (TIER) peak = dcnt > peak ? dcnt : peak;  // (pass 1: never past the input count's slots in memory)
#pragma unroll
        for (int j = 0; j < APL; ++j)
          if (word(j) < A) set_clk(slot, word(j), r[j]);
        for (unsigned long long w = (unsigned long long)lane; w < Kw; w += kWave) set_key(slot, w, 0);
      }
      // deferred_set.append(keyset): one lane per key word
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
  // the state back to memory: clock, the LDS slots, the count and status (and, at a pass-1 exit, the
  // op to continue from)
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
    if (PASS == 1) p.resume[s] = resume_at == 0xffffffffu ? kMcaDone : resume_at;
  }
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_map_counter_apply_batch(crdt_ctx *ctx, const crdt_map_counter_states *m, uint64_t *def_clock,
                                            uint64_t *def_keys, uint32_t *def_count, size_t Dcap,
                                            const crdt_map_counter_ops *ops, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!m || !ops || !status) return fail(ctx, CRDT_EINVAL, "map_counter_apply_batch: NULL argument");
  const size_t N = m->N, K = m->K, A = m->A, W = m->W;
  if (W != 1 && W != 2) return fail(ctx, CRDT_EINVAL, "map_counter_apply_batch: W = %zu (1 GCounter, 2 PNCounter)", W);
  if (N == 0) return CRDT_OK;
  if (A == 0 || A > 512) return fail(ctx, CRDT_EUNSUPPORTED, "map_counter_apply_batch: A = %zu outside 1..512", A);
  if (!m->clock || !m->ec || (K && !m->val) || !def_count || (Dcap && (!def_clock || !def_keys)) || !ops->op_off)
    return fail(ctx, CRDT_EINVAL, "map_counter_apply_batch: NULL buffer");
  if (ops->n_ops && (!ops->kind || !ops->actor || !ops->counter || !ops->key || !ops->vactor || !ops->vcounter))
    return fail(ctx, CRDT_EINVAL, "map_counter_apply_batch: NULL op buffer");
  if (m->clock_stride < A || m->ec_stride < K * A || m->val_stride < K * W * A)
    return fail(ctx, CRDT_EINVAL, "map_counter_apply_batch: strides smaller than the rows they hold");
  const size_t Kw = K ? (K + 63) / 64 : 1;
  // deferred slots in LDS: up to kMcaDl (the rest of Dcap in the caller's slot arrays), fewer where a
  // slot is wide (at most 8,192 words per wave)
  const size_t Dl = std::min<size_t>(Dcap, std::min<size_t>(kMcaDl, 8192 / (A + Kw)));
  const size_t per_wave = Dl * (A + Kw) * 8;
  unsigned wpb = 4;
  while (wpb > 1 && per_wave * wpb > 64 * 1024) --wpb;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  MapCounterApplyPlan p{(u64 *)m->clock, (u64 *)m->ec, (u64 *)m->val, m->clock_stride, m->ec_stride, m->val_stride,
                        N, K, A, W, Kw, Dcap, Dl, (u64 *)def_clock, (u64 *)def_keys, def_count,
                        (const u64 *)ops->op_off, ops->kind, ops->actor, ops->key, ops->vactor,
                        (const u64 *)ops->counter, (const u64 *)ops->vcounter, ops->vdir, ops->clk_row,
                        (const u64 *)ops->clk_pool, ops->clk_pool ? ops->n_clk_rows : 0,
                        (const u64 *)ops->key_off, ops->keys, ops->keys ? ops->n_keys : 0, ops->n_ops, status, wpb,
                        nullptr};
  // an Rm op needs key_off (n_ops + 1 entries); without it every Rm reads an empty key range.  Scratch:
  // [resume: N words when Dcap > Dl][zero key_off: n_ops + 1 words when absent]
  const bool tier = Dcap > Dl;
  const size_t kz = ops->key_off ? 0 : (ops->n_ops + 1) * 8, rz = tier ? N * 8 : 0;
  if (kz + rz) {
    if (int rc = ensure_scratch(ctx, kz + rz)) return rc;
    char *sc = static_cast<char *>(ctx->scratch);
    if (tier) p.resume = reinterpret_cast<u64 *>(sc);
    if (kz) {
      if (int rc = device_fill(ctx, sc + rz, kz, 0)) return rc;
      p.key_off = reinterpret_cast<const u64 *>(sc + rz);
    }
  }
  if (Dcap > Dl && ops->n_ops >= 0xffffffffull)  // (pass 2 resumes at a 32-bit op offset)
    return fail(ctx, CRDT_EUNSUPPORTED, "map_counter_apply_batch: 2^32 or more ops with Dcap past the LDS slots");
  const dim3 grid((unsigned)((N + wpb - 1) / wpb)), block(wpb * kWave);
  const size_t lds = per_wave * wpb;
  timing_begin(ctx, "map_counter_apply");
  auto go = [&](auto t, dim3 g, dim3 b, size_t l) {
    constexpr int T = decltype(t)::value;
    if (A <= 64) hipLaunchKernelGGL((map_counter_apply_kernel<1, T>), g, b, l, ctx->stream, p);
    else if (A <= 128) hipLaunchKernelGGL((map_counter_apply_kernel<2, T>), g, b, l, ctx->stream, p);
    else if (A <= 256) hipLaunchKernelGGL((map_counter_apply_kernel<4, T>), g, b, l, ctx->stream, p);
    else hipLaunchKernelGGL((map_counter_apply_kernel<8, T>), g, b, l, ctx->stream, p);
  };
  if (Dcap <= Dl) {
    go(std::integral_constant<int, 0>{}, grid, block, lds);  // one pass: the whole list fits the LDS slots
  } else {
    go(std::integral_constant<int, 1>{}, grid, block, lds);
    // pass 2: the few states pass 1 handed on (the rest exit at once), one wave per workgroup with the
    // whole wave-LDS budget as slots (up to 64 KiB), so a long list mostly stays out of global memory
    const size_t Dl2 = std::min<size_t>(Dcap, 8192 / (A + Kw));
    p.Dl = Dl2;
    p.wpb = 1;
    go(std::integral_constant<int, 2>{}, dim3((unsigned)N), dim3(kWave), Dl2 * (A + Kw) * 8);
  }
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}
