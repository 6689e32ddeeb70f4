// Batched Causal::forget of whole value-typed Map states (round 5): Map::forget (map.rs:85-114) —
// entry clocks forgotten, an entry whose clock empties dropped with its value, every surviving
// value forgotten (V::forget), the deferred rm clocks forgotten (an emptied one dropped), the map
// clock forgotten — for the value types of crdt_map_counter_lub_many / crdt_map_orswot_lub_many.
//
//  * GCounter / PNCounter (gcounter.rs:51-53, pncounter.rs:78-81): the value is W VClock rows, each
//    forgotten word by word — exactly what the MVReg Map's forget does to a value slot's clock
//    (an emptied slot is all-zero either way).  So the rows go through crdt_map_forget_batch with
//    the counter rows as W "slots" and a zero value array beside them (csrc/forget.hip).
//  * Orswot (orswot.rs:150-183): its clock and member rows forget word by word as well (an emptied
//    member row is the layout's "absent"), so they take the same path (the member rows as M slots,
//    then the Orswot clock as one); the nested deferred removes are forgotten, the emptied ones
//    dropped and the survivors collected anew (two that became equal keep one entry, the later one's
//    members at the earlier one's place — the fold kernel's rule, csrc/map_orswot.hip), and a dropped
//    entry drops its nested removes.
#include "common.hpp"

namespace crdt {

// one wave per (state, key): the key's nested deferred list after the forget by y[s]
template <int APL>
__global__ __launch_bounds__(256) void map_orswot_vd_forget_kernel(const u64 *ec, unsigned *vd_n, u64 *vd_clock,
                                                                   u64 *vd_mem, const u64 *y, unsigned long long y_stride,
                                                                   unsigned long long N, unsigned long long K,
                                                                   unsigned long long A, unsigned long long Mw,
                                                                   unsigned long long Vd) {
  const int lane = (int)(threadIdx.x % kWave);
  const unsigned long long sk = (unsigned long long)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  if (sk >= N * K) return;  // (whole waves)
  const unsigned long long s = sk / K;
  const unsigned nd = vd_n[sk];
  if (nd == 0) return;
  u64 yr[APL];
  bool live = false;  // the entry survived the forget (its clock, already forgotten, non-empty)
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = (unsigned long long)lane + 64ull * j;
    yr[j] = a < A ? y[s * y_stride + a] : 0ull;
    live = live || (a < A && ec[sk * A + a] != 0);
  }
  if (!__ballot(live)) {
    if (lane == 0) vd_n[sk] = 0;
    return;
  }
  u64 *rows = vd_clock + sk * Vd * A;  // [Vd][A] the key's nested slots (Vd: crdt_map_orswot_states)
  u64 *msk = vd_mem + sk * Vd * Mw;
  unsigned o = 0;
  for (unsigned i = 0; i < nd && i < Vd; ++i) {
    u64 x[APL];
    bool nz = false;
#pragma unroll
    for (int j = 0; j < APL; ++j) {
      const unsigned long long a = (unsigned long long)lane + 64ull * j;
      const u64 v = a < A ? rows[(unsigned long long)i * A + a] : 0ull;
      x[j] = v > yr[j] ? v : 0ull;  // VClock::forget
      nz = nz || x[j] != 0;
    }
    if (!__ballot(nz)) continue;  // forgotten: dropped
    unsigned jj = 0;
    for (; jj < o; ++jj) {  // equal to a kept one: the later members at the earlier place
      bool ne = false;
#pragma unroll
      for (int j = 0; j < APL; ++j) {
        const unsigned long long a = (unsigned long long)lane + 64ull * j;
        ne = ne || (a < A && rows[(unsigned long long)jj * A + a] != x[j]);
      }
      if (!__ballot(ne)) break;
    }
    // (each lane reads back only the words it writes: rows of index <= i)
    if (jj < o) {
      for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) msk[jj * Mw + w] = msk[i * Mw + w];
      continue;
    }
#pragma unroll
    for (int j = 0; j < APL; ++j) {
      const unsigned long long a = (unsigned long long)lane + 64ull * j;
      if (a < A) rows[(unsigned long long)o * A + a] = x[j];
    }
    if (o != i)
      for (unsigned long long w = (unsigned long long)lane; w < Mw; w += kWave) msk[o * Mw + w] = msk[i * Mw + w];
    ++o;
  }
  if (lane == 0) vd_n[sk] = o;
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_map_counter_forget_batch(crdt_ctx *ctx, const crdt_map_counter_states *m, const uint64_t *y,
                                             size_t y_stride, uint64_t *def_clock, const uint32_t *def_state,
                                             size_t D, uint8_t *def_keep) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!m) return fail(ctx, CRDT_EINVAL, "map_counter_forget_batch: NULL states");
  const size_t N = m->N, K = m->K, A = m->A, W = m->W;
  if (W != 1 && W != 2) return fail(ctx, CRDT_EINVAL, "map_counter_forget_batch: W = %zu (1 GCounter, 2 PNCounter)", W);
  if (N == 0 || A == 0) return CRDT_OK;
  if (!m->val && K) return fail(ctx, CRDT_EINVAL, "map_counter_forget_batch: NULL buffer");
  // the value rows as W slots of the MVReg Map's forget, beside a zero value array
  const size_t zwords = N * K * W;
  if (int rc = ensure_scratch(ctx, (zwords ? zwords : 1) * 8)) return rc;
  if (zwords)
    if (int rc = device_fill(ctx, ctx->scratch, zwords * 8, 0)) return rc;
  crdt_map_states s{N, K, A, W, m->clock, m->clock_stride, m->ec, m->ec_stride, m->val, m->val_stride,
                    static_cast<uint64_t *>(ctx->scratch), K * W};
  return crdt_map_forget_batch(ctx, &s, y, y_stride, def_clock, def_state, D, def_keep);
}

extern "C" int crdt_map_orswot_forget_batch(crdt_ctx *ctx, const crdt_map_orswot_states *m, const uint64_t *y,
                                            size_t y_stride, uint64_t *def_clock, const uint32_t *def_state,
                                            size_t D, uint8_t *def_keep) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!m) return fail(ctx, CRDT_EINVAL, "map_orswot_forget_batch: NULL states");
  const size_t N = m->N, K = m->K, M = m->M, A = m->A;
  if (N == 0 || A == 0) return CRDT_OK;
  if (A > 16 * (size_t)kWave) return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_forget_batch: A = %zu > %d", A, 16 * kWave);
  if (!m->clock || !y || (K && (!m->ec || !m->oc || (M && !m->ent) || !m->vd_n || !m->vd_clock || !m->vd_mem)))
    return fail(ctx, CRDT_EINVAL, "map_orswot_forget_batch: NULL buffer");
  const size_t Mw = M > 64 ? (M + 63) / 64 : 1;
  const size_t zwords = N * K * (M > 1 ? M : 1);
  if (int rc = ensure_scratch(ctx, (zwords ? zwords : 1) * 8)) return rc;
  if (zwords)
    if (int rc = device_fill(ctx, ctx->scratch, zwords * 8, 0)) return rc;
  uint64_t *z = static_cast<uint64_t *>(ctx->scratch);
  // 1. entry clocks, member rows (M slots), the Map-level removes and the map clock
  crdt_map_states s1{N, K, A, M, m->clock, A, m->ec, K * A, m->ent, K * M * A, z, K * M};
  if (int rc = crdt_map_forget_batch(ctx, &s1, y, y_stride, def_clock, def_state, D, def_keep)) return rc;
  if (K == 0) return CRDT_OK;
  // 2. the Orswot clocks (one slot; the entry clocks are forgotten again: idempotent, same drops)
  crdt_map_states s2{N, K, A, 1, m->clock, A, m->ec, K * A, m->oc, K * A, z, K};
  if (int rc = crdt_map_forget_batch(ctx, &s2, y, y_stride, nullptr, nullptr, 0, nullptr)) return rc;
  // 3. the nested deferred removes
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const unsigned long long waves = (unsigned long long)N * K, blocks = (waves + 3) / 4;
  if (blocks > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "map_orswot_forget_batch: N*K too large");
#define MVF(APL)                                                                                              \
  hipLaunchKernelGGL(map_orswot_vd_forget_kernel<APL>, dim3((unsigned)blocks), dim3(256), 0, ctx->stream,       \
                     (const u64 *)m->ec, m->vd_n, (u64 *)m->vd_clock, (u64 *)m->vd_mem, (const u64 *)y,         \
                     (unsigned long long)y_stride, (unsigned long long)N, (unsigned long long)K,                \
                     (unsigned long long)A, (unsigned long long)Mw, (unsigned long long)(m->Vd ? m->Vd : 16))
  if (A <= 64) MVF(1);
  else if (A <= 128) MVF(2);
  else if (A <= 256) MVF(4);
  else if (A <= 512) MVF(8);
  else MVF(16);
#undef MVF
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}
