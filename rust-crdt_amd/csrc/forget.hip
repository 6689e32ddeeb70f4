// Batched Causal::forget of whole Orswot and Map<K, MVReg> states: state s
// forgets the clock y_s, in place.  Every piece is VClock::forget (vclock.rs:95-105: keep x[a]
// iff x[a] > y[a]) on a dense row; what makes it a state op is the bookkeeping the reference
// does around it:
//   Orswot::forget (orswot.rs:150-183): clock, every entry clock (an emptied entry is dropped =
//       an all-zero row), every deferred rm clock (an emptied one is dropped: keep[d] = 0).
//   Map::forget (map.rs:85-114): every entry clock and its MVReg (MVReg::forget mvreg.rs:88-104
//       drops a value whose clock empties); the entry is dropped iff its own clock empties (then
//       its values go too), deferred rm clocks as for Orswot, then the map clock.
// Rows are processed by LR-lane groups (causal.hip's row-group shape): HBM-bound streaming,
// read + write of every row.
#include "common.hpp"

namespace crdt {

struct ForgetPlan {
  u64 *x;
  const u64 *y;
  unsigned long long nrows, per_state, sstride, rstride, ystride, A;
  const uint32_t *ysel;  // row -> state (deferred pools); null: state = row / per_state
  unsigned long long nstates;  // rows naming a state >= nstates are left untouched (keep = 1)
  uint8_t *keep;         // row nonempty after forget (may be null)
  int lr_log, vec2;
};

__device__ __forceinline__ u64 fgt(u64 x, u64 y) { return x > y ? x : 0ull; }

// Bits g*LR of the LR-lane groups with any bit set in m.
__device__ __forceinline__ u64 group_any(u64 m, int lr_log) {
  for (int sh = 1; sh < (1 << lr_log); sh <<= 1) m |= m >> sh;
  return m;
}

// Row r -> its state and its row pointer.
__device__ __forceinline__ u64 *forget_row_ptr(const ForgetPlan &p, unsigned long long r, unsigned long long &s) {
  s = p.ysel ? p.ysel[r] : r / p.per_state;
  return p.ysel ? p.x + r * p.rstride : p.x + (r / p.per_state) * p.sstride + (r % p.per_state) * p.rstride;
}

// Row width <= 64 pieces: LR = pow2 >= pieces lanes per row (one coalesced access per row), and
// kU row groups per lane in flight at once (ILP across rows, not within a row).
constexpr int kU = 4;

__global__ __launch_bounds__(kBlock) void forget_rows_kernel(ForgetPlan p) {
  const int lane = threadIdx.x % kWave;
  const int LR = 1 << p.lr_log;
  const int gl = lane & (LR - 1);
  const unsigned long long RW = kWave >> p.lr_log;
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;
  const unsigned long long nw = (unsigned long long)gridDim.x * (kBlock / kWave);
  const unsigned long long W = p.vec2 ? (p.A + 1) / 2 : p.A;  // pieces per row
  for (unsigned long long rb = w0 * RW * kU; rb < p.nrows; rb += nw * RW * kU) {
    u64 *xr[kU];
    const u64 *yr[kU];
    bool on[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const unsigned long long r = rb + j * RW + (lane >> p.lr_log);
      unsigned long long s = 0;
      xr[j] = forget_row_ptr(p, r < p.nrows ? r : p.nrows - 1, s);
      on[j] = r < p.nrows && s < p.nstates && (unsigned long long)gl < W;
      yr[j] = p.y + (on[j] ? s : 0) * p.ystride;
    }
    bool nz[kU];
    if (p.vec2) {
      u64x2 a[kU], b[kU];
#pragma unroll
      for (int j = 0; j < kU; ++j)
        if (on[j]) {
          a[j] = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(xr[j] + 2 * gl));
          b[j] = *reinterpret_cast<const u64x2 *>(yr[j] + 2 * gl);
        }
#pragma unroll
      for (int j = 0; j < kU; ++j) {
        nz[j] = false;
        if (on[j]) {
          a[j].x = fgt(a[j].x, b[j].x);
          a[j].y = fgt(a[j].y, b[j].y);
          nz[j] = (a[j].x | a[j].y) != 0;
          __builtin_nontemporal_store(a[j], reinterpret_cast<u64x2 *>(xr[j] + 2 * gl));
        }
      }
    } else {
      u64 a[kU], b[kU];
#pragma unroll
      for (int j = 0; j < kU; ++j)
        if (on[j]) {
          a[j] = xr[j][gl];
          b[j] = yr[j][gl];
        }
#pragma unroll
      for (int j = 0; j < kU; ++j) {
        nz[j] = false;
        if (on[j]) {
          a[j] = fgt(a[j], b[j]);
          nz[j] = a[j] != 0;
          xr[j][gl] = a[j];
        }
      }
    }
    if (p.keep) {
#pragma unroll
      for (int j = 0; j < kU; ++j) {
        const unsigned long long r = rb + j * RW + (lane >> p.lr_log);
        const u64 any = group_any(__ballot(nz[j]), p.lr_log);
        if (r < p.nrows && gl == 0) {
          unsigned long long s = 0;
          (void)forget_row_ptr(p, r, s);
          p.keep[r] = (uint8_t)(s < p.nstates ? (any >> lane) & 1 : 1);
        }
      }
    }
  }
}

// Rows wider than 64 pieces: LR = 64 lanes walk the row.
__global__ __launch_bounds__(kBlock) void forget_wide_rows_kernel(ForgetPlan p) {
  ROW_GROUP_LOOP(p.nrows, p.lr_log) {
    const unsigned long long r = rb + (lane >> p.lr_log);
    const unsigned long long rr = r < p.nrows ? r : p.nrows - 1;
    unsigned long long s = 0;
    u64 *xr = forget_row_ptr(p, rr, s);
    const bool on = r < p.nrows && s < p.nstates;
    const u64 *yr = p.y + (on ? s : 0) * p.ystride;
    bool nz = false;
    if (on) {
#pragma unroll 4
      for (unsigned long long c = gl; c < p.A; c += LR) {
        const u64 v = fgt(xr[c], yr[c]);
        nz |= v != 0;
        xr[c] = v;
      }
    }
    if (p.keep) {
      const u64 any = group_any(__ballot(nz), p.lr_log);
      if (r < p.nrows && gl == 0) p.keep[r] = (uint8_t)(on ? (any >> lane) & 1 : 1);
    }
  }
}

struct MapForgetPlan {
  u64 *ec, *vclk, *vval;
  unsigned long long N, K, A, V, ec_s, vclk_s, vval_s;
  const u64 *y;
  unsigned long long ystride;
  int lr_log;
};

// one (state, key) per LR-lane group: entry clock, then the key's V value slots
__global__ __launch_bounds__(kBlock) void map_forget_kernel(MapForgetPlan p) {
  const unsigned long long rows = p.N * p.K;
  ROW_GROUP_LOOP(rows, p.lr_log) {
    const unsigned long long r = rb + (lane >> p.lr_log);
    const bool on = r < rows;
    const unsigned long long rr = on ? r : rows - 1;
    const unsigned long long s = rr / p.K, k = rr % p.K;
    u64 *er = p.ec + s * p.ec_s + k * p.A;
    const u64 *yr = p.y + s * p.ystride;
    bool nz = false;
    if (on)
      for (unsigned long long c = gl; c < p.A; c += LR) {
        const u64 v = fgt(er[c], yr[c]);
        nz |= v != 0;
        er[c] = v;
      }
    const bool alive = (group_any(__ballot(nz), p.lr_log) >> (lane & ~(LR - 1))) & 1;  // map.rs:93-98
    for (unsigned long long j = 0; j < p.V; ++j) {
      u64 *vr = p.vclk + s * p.vclk_s + (k * p.V + j) * p.A;
      bool vz = false;
      if (on)
        for (unsigned long long c = gl; c < p.A; c += LR) {
          const u64 v = alive ? fgt(vr[c], yr[c]) : 0ull;  // MVReg::forget mvreg.rs:88-104
          vz |= v != 0;
          vr[c] = v;
        }
      const bool keepv = (group_any(__ballot(vz), p.lr_log) >> (lane & ~(LR - 1))) & 1;
      if (on && gl == 0 && !keepv) p.vval[s * p.vval_s + k * p.V + j] = 0;
    }
  }
}

// grid: workgroups per CU (CRDT_TUNE rows_blocks_per_cu, else 4), never more than the rows need
static unsigned forget_grid(crdt_ctx *ctx, unsigned long long rows, int lr_log, int dflt = 4) {
  const unsigned long long per_block = kBlock >> lr_log;
  const unsigned long long want = (rows + per_block - 1) / per_block;
  const int bpc = ctx->tune.rows_blocks_per_cu > 0 ? ctx->tune.rows_blocks_per_cu : dflt;
  const unsigned long long cap = (unsigned long long)ctx->cu_count * bpc;
  return (unsigned)(want < cap ? want : cap);
}

// A <= 64 and V <= 4: one word per lane, kU (state, key) rows per lane group in flight at once
// (entry clock, value clocks and y of all of them loaded before any vote).
__global__ __launch_bounds__(kBlock) void map_forget_narrow_kernel(MapForgetPlan p) {
  const unsigned long long rows = p.N * p.K;
  const int lane = threadIdx.x % kWave;
  const int LR = 1 << p.lr_log;
  const int gl = lane & (LR - 1);
  const unsigned long long RW = kWave >> p.lr_log;
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;
  const unsigned long long nw = (unsigned long long)gridDim.x * (kBlock / kWave);
  for (unsigned long long rb = w0 * RW * kU; rb < rows; rb += nw * RW * kU) {
    u64 *er[kU], *vr[kU];
    u64 ev[kU], yv[kU], vv[kU][4];
    bool act[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const unsigned long long r = rb + u * RW + (lane >> p.lr_log);
      const unsigned long long rr = r < rows ? r : rows - 1;
      const unsigned long long s = rr / p.K, k = rr % p.K;
      act[u] = r < rows && (unsigned long long)gl < p.A;
      er[u] = p.ec + s * p.ec_s + k * p.A + gl;
      vr[u] = p.vclk + s * p.vclk_s + k * p.V * p.A + gl;
      yv[u] = act[u] ? p.y[s * p.ystride + gl] : 0ull;
      ev[u] = act[u] ? *er[u] : 0ull;
#pragma unroll
      for (int j = 0; j < 4; ++j) vv[u][j] = (act[u] && (unsigned long long)j < p.V) ? vr[u][j * p.A] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const unsigned long long r = rb + u * RW + (lane >> p.lr_log);
      const unsigned long long rr = r < rows ? r : rows - 1;
      const u64 e = fgt(ev[u], yv[u]);
      const bool alive = (group_any(__ballot(e != 0), p.lr_log) >> (lane & ~(LR - 1))) & 1;  // map.rs:93-98
      if (act[u]) *er[u] = e;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if ((unsigned long long)j >= p.V) break;
        const u64 v = alive ? fgt(vv[u][j], yv[u]) : 0ull;  // MVReg::forget mvreg.rs:88-104
        if (act[u]) vr[u][j * p.A] = v;
        const bool keepv = (group_any(__ballot(v != 0), p.lr_log) >> (lane & ~(LR - 1))) & 1;
        if (r < rows && gl == 0 && !keepv) p.vval[(rr / p.K) * p.vval_s + (rr % p.K) * p.V + j] = 0;
      }
    }
  }
}

static bool al16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// A <= 128 even, V <= 4, 16-byte aligned rows: the narrow kernel with two pieces per lane (one
// 16-byte non-temporal access per lane, LR = pow2 >= A/2 lanes per row) and 32-bit (state, key)
// index math (N*K < 2^32, checked on the host).
__global__ __launch_bounds__(kBlock) void map_forget_vec2_kernel(MapForgetPlan p) {
  const unsigned rows = (unsigned)(p.N * p.K), K = (unsigned)p.K;
  const int lane = threadIdx.x % kWave;
  const int LR = 1 << p.lr_log;
  const unsigned gl = lane & (LR - 1);
  const unsigned RW = kWave >> p.lr_log;
  const unsigned W = (unsigned)(p.A / 2);
  const unsigned w0 = (blockIdx.x * (unsigned)kBlock + threadIdx.x) / kWave;
  const unsigned nw = gridDim.x * (unsigned)(kBlock / kWave);
  for (unsigned rb = w0 * RW * kU; rb < rows; rb += nw * RW * kU) {
    u64x2 *er[kU], *vr[kU];
    u64x2 ev[kU], yv[kU], vv[kU][4];
    bool act[kU];
    unsigned sk[kU][2];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const unsigned r = rb + u * RW + (lane >> p.lr_log);
      const unsigned rr = r < rows ? r : rows - 1;
      const unsigned s = rr / K, k = rr - s * K;
      sk[u][0] = s;
      sk[u][1] = k;
      act[u] = r < rows && gl < W;
      er[u] = reinterpret_cast<u64x2 *>(p.ec + s * p.ec_s + (unsigned long long)k * p.A) + gl;
      vr[u] = reinterpret_cast<u64x2 *>(p.vclk + s * p.vclk_s + (unsigned long long)k * p.V * p.A) + gl;
      const u64x2 z = {0ull, 0ull};
      yv[u] = act[u] ? reinterpret_cast<const u64x2 *>(p.y + s * p.ystride)[gl] : z;
      ev[u] = act[u] ? __builtin_nontemporal_load(er[u]) : z;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        vv[u][j] = (act[u] && (unsigned long long)j < p.V) ? __builtin_nontemporal_load(vr[u] + j * W) : z;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const unsigned r = rb + u * RW + (lane >> p.lr_log);
      u64x2 e;
      e.x = fgt(ev[u].x, yv[u].x);
      e.y = fgt(ev[u].y, yv[u].y);
      const bool alive = (group_any(__ballot((e.x | e.y) != 0), p.lr_log) >> (lane & ~(LR - 1))) & 1;  // map.rs:93-98
      if (act[u]) __builtin_nontemporal_store(e, er[u]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if ((unsigned long long)j >= p.V) break;
        u64x2 v;  // MVReg::forget mvreg.rs:88-104
        v.x = alive ? fgt(vv[u][j].x, yv[u].x) : 0ull;
        v.y = alive ? fgt(vv[u][j].y, yv[u].y) : 0ull;
        if (act[u]) __builtin_nontemporal_store(v, vr[u] + j * W);
        const bool keepv = (group_any(__ballot((v.x | v.y) != 0), p.lr_log) >> (lane & ~(LR - 1))) & 1;
        if (r < rows && gl == 0 && !keepv) p.vval[sk[u][0] * p.vval_s + (unsigned long long)sk[u][1] * p.V + j] = 0;
      }
    }
  }
}


static int launch_forget(crdt_ctx *ctx, ForgetPlan p) {
  if (p.nrows == 0 || p.A == 0) return CRDT_OK;
  p.vec2 = (p.A % 2 == 0) && (p.rstride % 2 == 0) && (p.sstride % 2 == 0 || p.ysel) && (p.ystride % 2 == 0) &&
           al16(p.x) && al16(p.y);
  const unsigned long long W = p.vec2 ? (p.A + 1) / 2 : p.A;
  if (W <= (unsigned long long)kWave) {
    p.lr_log = 0;
    while ((1ull << p.lr_log) < W) ++p.lr_log;
    hipLaunchKernelGGL(forget_rows_kernel, dim3(forget_grid(ctx, (p.nrows + kU - 1) / kU, p.lr_log)), dim3(kBlock), 0,
                       ctx->stream, p);
  } else {
    p.vec2 = 0;
    p.lr_log = 6;
    hipLaunchKernelGGL(forget_wide_rows_kernel, dim3(forget_grid(ctx, p.nrows, p.lr_log)), dim3(kBlock), 0,
                       ctx->stream, p);
  }
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_orswot_forget_batch(crdt_ctx *ctx, uint64_t *clock, size_t clock_stride, uint64_t *entries,
                                        size_t entry_mstride, size_t entry_sstride, size_t N, size_t M, size_t A,
                                        const uint64_t *y, size_t y_stride, uint64_t *def_clock,
                                        const uint32_t *def_state, size_t D, uint8_t *def_keep) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (N == 0 || A == 0) return CRDT_OK;
  if (!clock || !y || (M && !entries) || (D && (!def_clock || !def_state || !def_keep)))
    return fail(ctx, CRDT_EINVAL, "orswot_forget_batch: NULL buffer");
  if (clock_stride < A || (M && (entry_mstride < A || entry_sstride < M * entry_mstride)))
    return fail(ctx, CRDT_EINVAL, "orswot_forget_batch: stride smaller than the rows it holds");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  timing_begin(ctx, "forget_rows");
  // entries of every state (orswot.rs:154-166), then the deferred rm clocks (:168-180)
  if (M) {
    int rc = launch_forget(ctx, ForgetPlan{(u64 *)entries, (const u64 *)y, N * M, M, entry_sstride, entry_mstride,
                                           y_stride, A, nullptr, N, nullptr, 0, 0});
    if (rc) return rc;
  }
  timing_end(ctx);
  if (D) {
    int rc = launch_forget(ctx, ForgetPlan{(u64 *)def_clock, (const u64 *)y, D, 1, A, A, y_stride, A, def_state,
                                           N, def_keep, 0, 0});
    if (rc) return rc;
  }
  // the clock last: y may alias a state's own clock row (forget by oneself empties the state)
  return launch_forget(ctx, ForgetPlan{(u64 *)clock, (const u64 *)y, N, 1, clock_stride, clock_stride, y_stride, A,
                                       nullptr, N, nullptr, 0, 0});
}

extern "C" int crdt_map_forget_batch(crdt_ctx *ctx, const crdt_map_states *m, const uint64_t *y, size_t y_stride,
                                     uint64_t *def_clock, const uint32_t *def_state, size_t D, uint8_t *def_keep) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!m) return fail(ctx, CRDT_EINVAL, "map_forget_batch: NULL states");
  const size_t N = m->N, K = m->K, A = m->A, V = m->V;
  if (N == 0 || A == 0) return CRDT_OK;
  if (!m->clock || !y || (K && (!m->ec || (V && (!m->vclk || !m->vval)))) ||
      (D && (!def_clock || !def_state || !def_keep)))
    return fail(ctx, CRDT_EINVAL, "map_forget_batch: NULL buffer");
  if (m->clock_stride < A || (K && (m->ec_stride < K * A || (V && (m->vclk_stride < K * V * A || m->vval_stride < K * V)))))
    return fail(ctx, CRDT_EINVAL, "map_forget_batch: stride smaller than the rows it holds");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  if (K) {
    MapForgetPlan p{(u64 *)m->ec, (u64 *)m->vclk, (u64 *)m->vval, N, K, A, V, m->ec_stride, m->vclk_stride, m->vval_stride,
                    (const u64 *)y, y_stride, 0};
    // the vec2 kernel walks rows with 32-bit indices: the last row plus one whole grid step must
    // stay below 2^32 so `rb += step` can never wrap (a wrapped walk would never exit)
    int lr2 = 0;
    while (lr2 < 6 && (1ull << lr2) < A / 2) ++lr2;
    const unsigned long long grid2 = forget_grid(ctx, (N * K + kU - 1) / kU, lr2, ctx->tune.map_forget_bpc);
    const unsigned long long step2 = grid2 * (kBlock / kWave) * (kWave >> lr2) * kU;
    const bool vec2 = A % 2 == 0 && A <= 2 * (size_t)kWave && V <= 4 && N * K + step2 <= (1ull << 32) &&
                      m->ec_stride % 2 == 0 && m->vclk_stride % 2 == 0 && y_stride % 2 == 0 && al16(m->ec) &&
                      al16(m->vclk) && al16(y) && ctx->tune.map_forget_vec2 != 0;
    const size_t W = vec2 ? A / 2 : A;  // pieces per row
    while (p.lr_log < 6 && (1ull << p.lr_log) < W) ++p.lr_log;  // a key's rows: one access per row
    timing_begin(ctx, "map_forget");
    if (vec2)
      hipLaunchKernelGGL(map_forget_vec2_kernel, dim3((unsigned)grid2), dim3(kBlock), 0, ctx->stream, p);
    else if (A <= (size_t)kWave && V <= 4)
      hipLaunchKernelGGL(map_forget_narrow_kernel, dim3(forget_grid(ctx, (N * K + kU - 1) / kU, p.lr_log)),
                         dim3(kBlock), 0, ctx->stream, p);
    else
      hipLaunchKernelGGL(map_forget_kernel, dim3(forget_grid(ctx, N * K, p.lr_log)), dim3(kBlock), 0, ctx->stream, p);
    timing_end(ctx);
    CRDT_HIP(ctx, hipGetLastError());
  }
  if (D) {
    int rc = launch_forget(ctx, ForgetPlan{(u64 *)def_clock, (const u64 *)y, D, 1, A, A, y_stride, A, def_state,
                                           N, def_keep, 0, 0});
    if (rc) return rc;
  }
  return launch_forget(ctx, ForgetPlan{(u64 *)m->clock, (const u64 *)y, N, 1, m->clock_stride, m->clock_stride,
                                       y_stride, A, nullptr, N, nullptr, 0, 0});
}
