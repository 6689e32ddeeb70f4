// Pairwise in-place merge of value-typed Map states (round 6): self[i].merge(other[i]) for
// Map<K, GCounter / PNCounter>, Map<K, Orswot<M>> and Map<K, Map<K2, MVReg<u64>>> on their apply
// layouts (crdt_map_{counter,orswot,nested}_states + crdt_map_deferred slots).
//
// Each pair is one group of the exact left-fold kernels (map_counter.hip / map_orswot.hip /
// map_nested.hip) with R = 2: Map::new() merged with self, then with other (map.rs:140-220).  A Map
// merged from empty reproduces any state whose deferred removes are applied and not dominated by its
// clock — every state apply, merge, forget or ingest leaves — so the fold of [self, other] is
// self.merge(other) on those states.  Steps, all on the ctx stream:
//   1. the two sides stacked per pair into one (N, 2, ...) batch (strided 2-D copies);
//   2. the Map-level deferred slots of both sides as one pool grouped by pair (self's first), the
//      nested deferred lists (16 slots per key) as a device CSR over (pair, side, key);
//   3. the fold, its outputs written straight into self's rows (the packed layouts) or through a
//      scratch copy (the counter states' strides);
//   4. the pool's survivors (def_keep, their merged key sets) compacted into self's slots in pool
//      order; slots past them zeroed up to self's old count.
// Host work: the slot counts are read once (the pool's offsets are host arrays for the fold), so the
// call synchronises the stream once.
#include "common.hpp"

#include <vector>

namespace crdt {

// pool gather: pair i's self slots [0, ca_i) then other's [0, cb_i) at rows off[i]..; row = side
__global__ __launch_bounds__(64) void vmm_pool_kernel(unsigned long long N, unsigned long long A,
                                                      unsigned long long Kw, const u64 *sc, const u64 *sk,
                                                      const unsigned *scnt, unsigned long long sDcap, const u64 *oc,
                                                      const u64 *ok, const unsigned *ocnt, unsigned long long oDcap,
                                                      const size_t *off, uint32_t *prow, u64 *pclk, u64 *pkey) {
  const unsigned long long i = blockIdx.x;
  if (i >= N) return;
  const unsigned lane = threadIdx.x;
  const unsigned ca = scnt[i], cb = ocnt[i];
  unsigned long long d = off[i];
  for (unsigned s = 0; s < 2; ++s) {
    const unsigned n = s ? cb : ca;
    const u64 *c = s ? oc + i * oDcap * A : sc + i * sDcap * A;
    const u64 *k = s ? ok + i * oDcap * Kw : sk + i * sDcap * Kw;
    for (unsigned j = 0; j < n; ++j, ++d) {
      for (unsigned long long a = lane; a < A; a += 64) pclk[d * A + a] = c[j * A + a];
      for (unsigned long long w = lane; w < Kw; w += 64) pkey[d * Kw + w] = k[j * Kw + w];
      if (lane == 0) prow[d] = s;
    }
  }
}

// nested slot lists (cnt [N][K], rows [N][K][S][A], words [N][K][S][W], S = Sa / Sb slots per key) of
// both sides as a CSR over (pair, side, key): voff[(i*2 + s)*K + k] = the first row
__global__ __launch_bounds__(64) void vmm_csr_kernel(unsigned long long N, unsigned long long K, unsigned long long A,
                                                     unsigned long long W, const unsigned *na, const u64 *ca,
                                                     const u64 *wa, const unsigned *nb, const u64 *cb, const u64 *wb,
                                                     const u64 *voff, u64 *oc, u64 *ow, unsigned long long Sa,
                                                     unsigned long long Sb) {
  const unsigned long long b = blockIdx.x;  // (i, s, k)
  if (b >= N * 2 * K) return;
  const unsigned long long i = b / (2 * K), s = (b / K) % 2, k = b % K;
  const unsigned lane = threadIdx.x;
  const unsigned long long sk = i * K + k;
  const unsigned n = s ? nb[sk] : na[sk];
  const unsigned long long S = s ? Sb : Sa;
  const u64 *c = (s ? cb : ca) + sk * S * A;
  const u64 *w = (s ? wb : wa) + sk * S * W;
  const unsigned long long d0 = voff[b];
  for (unsigned j = 0; j < n; ++j) {
    for (unsigned long long a = lane; a < A; a += 64) oc[(d0 + j) * A + a] = c[j * A + a];
    for (unsigned long long x = lane; x < W; x += 64) ow[(d0 + j) * W + x] = w[j * W + x];
  }
}

// the survivors of pair i's pool rows, in order, into self's slots; status bit 0 past Dcap, bit 3
// where the fold flagged a capacity (the pair's result incomplete)
__global__ __launch_bounds__(64) void vmm_survive_kernel(unsigned long long N, unsigned long long A,
                                                         unsigned long long Kw, const size_t *off, const uint8_t *keep,
                                                         const u64 *pclk, const u64 *kout, u64 *sc, u64 *sk,
                                                         unsigned *scnt, unsigned long long Dcap, const unsigned *flags,
                                                         unsigned *status) {
  const unsigned long long i = blockIdx.x;
  if (i >= N) return;
  const unsigned lane = threadIdx.x;
  const unsigned old = scnt[i];
  unsigned long long n = 0;
  if (keep) {
    for (unsigned long long d = off[i]; d < off[i + 1]; ++d) {
      if (!keep[d]) continue;
      if (n < Dcap) {
        for (unsigned long long a = lane; a < A; a += 64) sc[(i * Dcap + n) * A + a] = pclk[d * A + a];
        for (unsigned long long w = lane; w < Kw; w += 64) sk[(i * Dcap + n) * Kw + w] = kout[d * Kw + w];
      }
      ++n;
    }
  }
  const unsigned long long kept = n < Dcap ? n : Dcap;
  for (unsigned long long j = kept; j < old && j < Dcap; ++j) {  // slots the list vacated: zero
    for (unsigned long long a = lane; a < A; a += 64) sc[(i * Dcap + j) * A + a] = 0ull;
    for (unsigned long long w = lane; w < Kw; w += 64) sk[(i * Dcap + j) * Kw + w] = 0ull;
  }
  __syncthreads();  // (every lane read `old` before lane 0 overwrites it)
  if (lane == 0) {
    scnt[i] = (unsigned)kept;
    status[i] = (n > Dcap ? 1u : 0u) | (flags[i] ? 8u : 0u);
  }
}

namespace {

// a bump allocator over ctx->dscratch (256-byte aligned pieces)
struct Carve {
  size_t used = 0;
  size_t take(size_t bytes) {
    const size_t at = used;
    used += (bytes + 255) / 256 * 256;
    return at;
  }
};

int read_counts(crdt_ctx *ctx, const uint32_t *dev, size_t n, std::vector<uint32_t> &host) {
  host.assign(n, 0);
  if (n == 0) return CRDT_OK;
  CRDT_HIP(ctx, hipMemcpyAsync(host.data(), dev, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return CRDT_OK;
}

int check_def(crdt_ctx *ctx, const crdt_map_deferred *d, size_t N, const char *what) {
  if (!d || !d->count) return fail(ctx, CRDT_EINVAL, "%s: NULL deferred slots", what);
  if (N && d->Dcap && (!d->clock || !d->keys)) return fail(ctx, CRDT_EINVAL, "%s: NULL deferred slot buffers", what);
  return CRDT_OK;
}

// the pool's host offsets from both sides' counts (validated against their Dcap)
int pool_offsets(crdt_ctx *ctx, const crdt_map_deferred *ad, const crdt_map_deferred *bd, size_t N,
                 std::vector<size_t> &off, const char *what) {
  std::vector<uint32_t> ca, cb;
  if (int rc = read_counts(ctx, ad->count, N, ca)) return rc;
  if (int rc = read_counts(ctx, bd->count, N, cb)) return rc;
  off.assign(N + 1, 0);
  for (size_t i = 0; i < N; ++i) {
    if (ca[i] > ad->Dcap || cb[i] > bd->Dcap) return fail(ctx, CRDT_EINVAL, "%s: def_count[%zu] above Dcap", what, i);
    off[i + 1] = off[i] + ca[i] + cb[i];
  }
  return CRDT_OK;
}

// the nested lists' CSR offsets over (pair, side, key) from both sides' counts (<= each side's slots)
int nested_offsets(crdt_ctx *ctx, const uint32_t *na, const uint32_t *nb, size_t N, size_t K,
                   std::vector<u64> &voff, const char *what, size_t ca = 16, size_t cb = 16) {
  std::vector<uint32_t> ha, hb;
  if (int rc = read_counts(ctx, na, N * K, ha)) return rc;
  if (int rc = read_counts(ctx, nb, N * K, hb)) return rc;
  voff.assign(N * 2 * K + 1, 0);
  size_t b = 0;
  for (size_t i = 0; i < N; ++i)
    for (size_t s = 0; s < 2; ++s)
      for (size_t k = 0; k < K; ++k, ++b) {
        const uint32_t n = s ? hb[i * K + k] : ha[i * K + k];
        if (n > (s ? cb : ca)) return fail(ctx, CRDT_EINVAL, "%s: a nested deferred count above its slots", what);
        voff[b + 1] = voff[b] + n;
      }
  return CRDT_OK;
}

// dst (N, 2, block) <- side s's (N, block) rows with source pitch
int stack2(crdt_ctx *ctx, void *dst, size_t block_bytes, const void *a, size_t apitch, const void *b, size_t bpitch,
           size_t N) {
  if (N == 0 || block_bytes == 0) return CRDT_OK;
  CRDT_HIP(ctx, hipMemcpy2DAsync(dst, 2 * block_bytes, a, apitch, block_bytes, N, hipMemcpyDeviceToDevice, ctx->stream));
  CRDT_HIP(ctx, hipMemcpy2DAsync(static_cast<char *>(dst) + block_bytes, 2 * block_bytes, b, bpitch, block_bytes, N,
                                 hipMemcpyDeviceToDevice, ctx->stream));
  return CRDT_OK;
}

// the pool (Map-level slots of both sides) into scratch; returns D
struct Pool {
  size_t D = 0;
  size_t *off_dev = nullptr;
  uint32_t *row = nullptr;
  u64 *clk = nullptr, *key = nullptr, *kout = nullptr;
  uint8_t *keep = nullptr;
};

size_t pool_bytes(size_t N, size_t D, size_t A, size_t Kw, Carve &cv, size_t (&at)[6]) {
  at[0] = cv.take((N + 1) * sizeof(size_t));
  at[1] = cv.take(D * 4);
  at[2] = cv.take(D * A * 8);
  at[3] = cv.take(D * Kw * 8);
  at[4] = cv.take(D * Kw * 8);
  at[5] = cv.take(D);
  return cv.used;
}

int build_pool(crdt_ctx *ctx, char *base, const size_t (&at)[6], const std::vector<size_t> &off, size_t N, size_t A,
               size_t Kw, const crdt_map_deferred *ad, const crdt_map_deferred *bd, Pool &pl) {
  pl.D = off[N];
  pl.off_dev = reinterpret_cast<size_t *>(base + at[0]);
  pl.row = reinterpret_cast<uint32_t *>(base + at[1]);
  pl.clk = reinterpret_cast<u64 *>(base + at[2]);
  pl.key = reinterpret_cast<u64 *>(base + at[3]);
  pl.kout = reinterpret_cast<u64 *>(base + at[4]);
  pl.keep = pl.D ? reinterpret_cast<uint8_t *>(base + at[5]) : nullptr;
  if (int rc = stage_h2d(ctx, pl.off_dev, off.data(), (N + 1) * sizeof(size_t))) return rc;
  if (pl.D) {
    hipLaunchKernelGGL(vmm_pool_kernel, dim3((unsigned)N), dim3(64), 0, ctx->stream, (unsigned long long)N,
                       (unsigned long long)A, (unsigned long long)Kw, (const u64 *)ad->clock, (const u64 *)ad->keys,
                       ad->count, (unsigned long long)ad->Dcap, (const u64 *)bd->clock, (const u64 *)bd->keys,
                       bd->count, (unsigned long long)bd->Dcap, pl.off_dev, pl.row, pl.clk, pl.key);
    CRDT_HIP(ctx, hipGetLastError());
  }
  return CRDT_OK;
}

int survive(crdt_ctx *ctx, const Pool &pl, size_t N, size_t A, size_t Kw, const crdt_map_deferred *ad,
            const unsigned *flags, uint32_t *status) {
  hipLaunchKernelGGL(vmm_survive_kernel, dim3((unsigned)N), dim3(64), 0, ctx->stream, (unsigned long long)N,
                     (unsigned long long)A, (unsigned long long)Kw, pl.off_dev, pl.D ? pl.keep : nullptr, pl.clk, pl.kout,
                     (u64 *)ad->clock, (u64 *)ad->keys, ad->count, (unsigned long long)ad->Dcap, flags, status);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

}  // namespace
}  // namespace crdt

using namespace crdt;

extern "C" int crdt_map_counter_merge_batch(crdt_ctx *ctx, const crdt_map_counter_states *a,
                                            const crdt_map_deferred *ad, const crdt_map_counter_states *b,
                                            const crdt_map_deferred *bd, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  static const char *what = "map_counter_merge_batch";
  CRDT_CHECK_CTX(ctx);
  if (!a || !b || !status) return fail(ctx, CRDT_EINVAL, "%s: NULL argument", what);
  const size_t N = a->N, K = a->K, A = a->A, W = a->W;
  if (b->N != N || b->K != K || b->A != A || b->W != W)
    return fail(ctx, CRDT_EINVAL, "%s: self and other differ in N, K, A or W", what);
  if (W != 1 && W != 2) return fail(ctx, CRDT_EINVAL, "%s: W = %zu (1 GCounter, 2 PNCounter)", what, W);
  if (int rc = check_def(ctx, ad, N, what)) return rc;
  if (int rc = check_def(ctx, bd, N, what)) return rc;
  if (N == 0) return CRDT_OK;
  if (A == 0 || K == 0) return fail(ctx, CRDT_EINVAL, "%s: need A, K >= 1", what);
  for (const crdt_map_counter_states *s : {a, b}) {
    if (!s->clock || !s->ec || !s->val) return fail(ctx, CRDT_EINVAL, "%s: NULL state buffer", what);
    if (s->clock_stride < A || s->ec_stride < K * A || s->val_stride < K * W * A)
      return fail(ctx, CRDT_EINVAL, "%s: strides smaller than the rows they hold", what);
  }
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const size_t Kw = (K + 63) / 64;
  std::vector<size_t> off;
  if (int rc = pool_offsets(ctx, ad, bd, N, off, what)) return rc;
  const size_t D = off[N];
  Carve cv;
  const size_t c2 = cv.take(N * 2 * A * 8), e2 = cv.take(N * 2 * K * A * 8), v2 = cv.take(N * 2 * K * W * A * 8);
  const size_t oc = cv.take(N * A * 8), oe = cv.take(N * K * A * 8), ov = cv.take(N * K * W * A * 8);
  const size_t of = cv.take(N * 4);
  size_t at[6];
  pool_bytes(N, D, A, Kw, cv, at);
  if (int rc = ensure_dscratch(ctx, cv.used)) return rc;
  char *base = static_cast<char *>(ctx->dscratch);
  if (int rc = stack2(ctx, base + c2, A * 8, a->clock, a->clock_stride * 8, b->clock, b->clock_stride * 8, N)) return rc;
  if (int rc = stack2(ctx, base + e2, K * A * 8, a->ec, a->ec_stride * 8, b->ec, b->ec_stride * 8, N)) return rc;
  if (int rc = stack2(ctx, base + v2, K * W * A * 8, a->val, a->val_stride * 8, b->val, b->val_stride * 8, N)) return rc;
  Pool pl;
  if (int rc = build_pool(ctx, base, at, off, N, A, Kw, ad, bd, pl)) return rc;
  crdt_map_counter_batch in{};
  in.G = N;
  in.R = 2;
  in.K = K;
  in.A = A;
  in.W = W;
  in.clock = reinterpret_cast<const uint64_t *>(base + c2);
  in.clock_rstride = A;
  in.clock_gstride = 2 * A;
  in.ec = reinterpret_cast<const uint64_t *>(base + e2);
  in.ec_rstride = K * A;
  in.ec_gstride = 2 * K * A;
  in.val = reinterpret_cast<const uint64_t *>(base + v2);
  in.val_rstride = K * W * A;
  in.val_gstride = 2 * K * W * A;
  in.def_off = D ? off.data() : nullptr;
  in.def_row = pl.row;
  in.def_clock = reinterpret_cast<const uint64_t *>(pl.clk);
  in.def_keys = reinterpret_cast<const uint64_t *>(pl.key);
  crdt_map_counter_out out{};
  out.clock = reinterpret_cast<uint64_t *>(base + oc);
  out.ec = reinterpret_cast<uint64_t *>(base + oe);
  out.val = reinterpret_cast<uint64_t *>(base + ov);
  out.flags = reinterpret_cast<uint32_t *>(base + of);
  out.def_keep = pl.keep;
  out.def_keys = reinterpret_cast<uint64_t *>(pl.kout);
  if (int rc = crdt_map_counter_lub_many(ctx, &in, &out)) return rc;
  // the fold's state back into self's rows (its own strides)
  CRDT_HIP(ctx, hipMemcpy2DAsync(a->clock, a->clock_stride * 8, out.clock, A * 8, A * 8, N, hipMemcpyDeviceToDevice,
                                 ctx->stream));
  CRDT_HIP(ctx, hipMemcpy2DAsync(a->ec, a->ec_stride * 8, out.ec, K * A * 8, K * A * 8, N, hipMemcpyDeviceToDevice,
                                 ctx->stream));
  CRDT_HIP(ctx, hipMemcpy2DAsync(a->val, a->val_stride * 8, out.val, K * W * A * 8, K * W * A * 8, N,
                                 hipMemcpyDeviceToDevice, ctx->stream));
  return survive(ctx, pl, N, A, Kw, ad, out.flags, status);
}

extern "C" int crdt_map_orswot_merge_batch(crdt_ctx *ctx, const crdt_map_orswot_states *a,
                                           const crdt_map_deferred *ad, const crdt_map_orswot_states *b,
                                           const crdt_map_deferred *bd, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  static const char *what = "map_orswot_merge_batch";
  CRDT_CHECK_CTX(ctx);
  if (!a || !b || !status) return fail(ctx, CRDT_EINVAL, "%s: NULL argument", what);
  const size_t N = a->N, K = a->K, M = a->M, A = a->A;
  if (b->N != N || b->K != K || b->M != M || b->A != A)
    return fail(ctx, CRDT_EINVAL, "%s: self and other differ in N, K, M or A", what);
  if (int rc = check_def(ctx, ad, N, what)) return rc;
  if (int rc = check_def(ctx, bd, N, what)) return rc;
  if (N == 0) return CRDT_OK;
  if (A == 0 || K == 0) return fail(ctx, CRDT_EINVAL, "%s: need A, K >= 1", what);
  for (const crdt_map_orswot_states *s : {a, b})
    if (!s->clock || !s->ec || !s->oc || (M && !s->ent) || !s->vd_n || !s->vd_clock || !s->vd_mem)
      return fail(ctx, CRDT_EINVAL, "%s: NULL state buffer", what);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const size_t Kw = (K + 63) / 64, Mw = M > 64 ? (M + 63) / 64 : 1;
  std::vector<size_t> off;
  if (int rc = pool_offsets(ctx, ad, bd, N, off, what)) return rc;
  std::vector<u64> voff;
  const size_t Va = a->Vd ? a->Vd : 16, Vb = b->Vd ? b->Vd : 16;  // nested slots per key, each side
  if (int rc = nested_offsets(ctx, a->vd_n, b->vd_n, N, K, voff, what, Va, Vb)) return rc;
  const size_t D = off[N], Dv = voff[N * 2 * K];
  Carve cv;
  const size_t c2 = cv.take(N * 2 * A * 8), e2 = cv.take(N * 2 * K * A * 8), o2 = cv.take(N * 2 * K * A * 8);
  const size_t m2 = cv.take(N * 2 * K * M * A * 8), of = cv.take(N * 4);
  const size_t vo = cv.take((N * 2 * K + 1) * 8), vc = cv.take(Dv * A * 8), vm = cv.take(Dv * Mw * 8);
  size_t at[6];
  pool_bytes(N, D, A, Kw, cv, at);
  if (int rc = ensure_dscratch(ctx, cv.used)) return rc;
  char *base = static_cast<char *>(ctx->dscratch);
  if (int rc = stack2(ctx, base + c2, A * 8, a->clock, A * 8, b->clock, A * 8, N)) return rc;
  if (int rc = stack2(ctx, base + e2, K * A * 8, a->ec, K * A * 8, b->ec, K * A * 8, N)) return rc;
  if (int rc = stack2(ctx, base + o2, K * A * 8, a->oc, K * A * 8, b->oc, K * A * 8, N)) return rc;
  if (int rc = stack2(ctx, base + m2, K * M * A * 8, a->ent, K * M * A * 8, b->ent, K * M * A * 8, N)) return rc;
  if (int rc = stage_h2d(ctx, base + vo, voff.data(), voff.size() * 8)) return rc;
  if (Dv) {
    hipLaunchKernelGGL(vmm_csr_kernel, dim3((unsigned)(N * 2 * K)), dim3(64), 0, ctx->stream, (unsigned long long)N,
                       (unsigned long long)K, (unsigned long long)A, (unsigned long long)Mw, a->vd_n,
                       (const u64 *)a->vd_clock, (const u64 *)a->vd_mem, b->vd_n, (const u64 *)b->vd_clock,
                       (const u64 *)b->vd_mem, reinterpret_cast<const u64 *>(base + vo),
                       reinterpret_cast<u64 *>(base + vc), reinterpret_cast<u64 *>(base + vm), (unsigned long long)Va,
                       (unsigned long long)Vb);
    CRDT_HIP(ctx, hipGetLastError());
  }
  Pool pl;
  if (int rc = build_pool(ctx, base, at, off, N, A, Kw, ad, bd, pl)) return rc;
  crdt_map_orswot_batch in{};
  in.G = N;
  in.R = 2;
  in.K = K;
  in.M = M;
  in.A = A;
  in.clock = reinterpret_cast<const uint64_t *>(base + c2);
  in.ec = reinterpret_cast<const uint64_t *>(base + e2);
  in.oc = reinterpret_cast<const uint64_t *>(base + o2);
  in.ent = reinterpret_cast<const uint64_t *>(base + m2);
  in.vd_off = reinterpret_cast<const uint64_t *>(base + vo);
  in.vd_clock = Dv ? reinterpret_cast<const uint64_t *>(base + vc) : nullptr;
  in.vd_mem = Dv ? reinterpret_cast<const uint64_t *>(base + vm) : nullptr;
  in.Dv = Dv;
  in.def_off = D ? off.data() : nullptr;
  in.def_row = pl.row;
  in.def_clock = reinterpret_cast<const uint64_t *>(pl.clk);
  in.def_keys = reinterpret_cast<const uint64_t *>(pl.key);
  crdt_map_orswot_out out{};  // (the packed state layout is the fold's output layout: straight into self)
  out.clock = a->clock;
  out.ec = a->ec;
  out.oc = a->oc;
  out.ent = a->ent;
  out.vd_n = a->vd_n;
  out.vd_clock = a->vd_clock;
  out.vd_mem = a->vd_mem;
  out.Vd = Va;  // (self's slots: other's lists merge into them, bit 3 past Va)
  out.flags = reinterpret_cast<uint32_t *>(base + of);
  out.def_keep = pl.keep;
  out.def_keys = reinterpret_cast<uint64_t *>(pl.kout);
  if (int rc = crdt_map_orswot_lub_many(ctx, &in, &out)) return rc;
  return survive(ctx, pl, N, A, Kw, ad, out.flags, status);
}

extern "C" int crdt_map_nested_merge_batch(crdt_ctx *ctx, const crdt_map_nested_states *a,
                                           const crdt_map_deferred *ad, const crdt_map_nested_states *b,
                                           const crdt_map_deferred *bd, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  static const char *what = "map_nested_merge_batch";
  CRDT_CHECK_CTX(ctx);
  if (!a || !b || !status) return fail(ctx, CRDT_EINVAL, "%s: NULL argument", what);
  const size_t N = a->N, K = a->K, K2 = a->K2, A = a->A;
  if (b->N != N || b->K != K || b->K2 != K2 || b->A != A)
    return fail(ctx, CRDT_EINVAL, "%s: self and other differ in N, K, K2 or A", what);
  if (int rc = check_def(ctx, ad, N, what)) return rc;
  if (int rc = check_def(ctx, bd, N, what)) return rc;
  if (N == 0) return CRDT_OK;
  if (A == 0 || K == 0) return fail(ctx, CRDT_EINVAL, "%s: need A, K >= 1", what);
  for (const crdt_map_nested_states *s : {a, b})
    if (!s->clock || !s->ec || !s->ic || (K2 && (!s->iec || !s->ivc || !s->ivv || !s->nval)) || !s->id_n ||
        !s->id_clock || !s->id_keys)
      return fail(ctx, CRDT_EINVAL, "%s: NULL state buffer", what);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const size_t Kw = (K + 63) / 64, VS = a->Vs ? a->Vs : 8;  // MVReg slots per inner key (both sides)
  if ((b->Vs ? b->Vs : 8) != VS) return fail(ctx, CRDT_EINVAL, "%s: self and other differ in Vs", what);
  const size_t K2w = K2 > 64 ? (K2 + 63) / 64 : 1;  // inner key-set mask words (the fold's layout)
  std::vector<size_t> off;
  if (int rc = pool_offsets(ctx, ad, bd, N, off, what)) return rc;
  std::vector<u64> ioff;
  const size_t Ia = a->Id ? a->Id : 16, Ib = b->Id ? b->Id : 16;  // inner deferred slots per key, each side
  if (int rc = nested_offsets(ctx, a->id_n, b->id_n, N, K, ioff, what, Ia, Ib)) return rc;
  const size_t D = off[N], Di = ioff[N * 2 * K];
  Carve cv;
  const size_t c2 = cv.take(N * 2 * A * 8), e2 = cv.take(N * 2 * K * A * 8), i2 = cv.take(N * 2 * K * A * 8);
  const size_t ie2 = cv.take(N * 2 * K * K2 * A * 8), vc2 = cv.take(N * 2 * K * K2 * VS * A * 8);
  const size_t vv2 = cv.take(N * 2 * K * K2 * VS * 8), of = cv.take(N * 4);
  const size_t io = cv.take((N * 2 * K + 1) * 8), ic = cv.take(Di * A * 8), ik = cv.take(Di * K2w * 8);
  size_t at[6];
  pool_bytes(N, D, A, Kw, cv, at);
  if (int rc = ensure_dscratch(ctx, cv.used)) return rc;
  char *base = static_cast<char *>(ctx->dscratch);
  if (int rc = stack2(ctx, base + c2, A * 8, a->clock, A * 8, b->clock, A * 8, N)) return rc;
  if (int rc = stack2(ctx, base + e2, K * A * 8, a->ec, K * A * 8, b->ec, K * A * 8, N)) return rc;
  if (int rc = stack2(ctx, base + i2, K * A * 8, a->ic, K * A * 8, b->ic, K * A * 8, N)) return rc;
  if (int rc = stack2(ctx, base + ie2, K * K2 * A * 8, a->iec, K * K2 * A * 8, b->iec, K * K2 * A * 8, N)) return rc;
  if (int rc = stack2(ctx, base + vc2, K * K2 * VS * A * 8, a->ivc, K * K2 * VS * A * 8, b->ivc, K * K2 * VS * A * 8, N))
    return rc;
  if (int rc = stack2(ctx, base + vv2, K * K2 * VS * 8, a->ivv, K * K2 * VS * 8, b->ivv, K * K2 * VS * 8, N)) return rc;
  if (int rc = stage_h2d(ctx, base + io, ioff.data(), ioff.size() * 8)) return rc;
  if (Di) {
    hipLaunchKernelGGL(vmm_csr_kernel, dim3((unsigned)(N * 2 * K)), dim3(64), 0, ctx->stream, (unsigned long long)N,
                       (unsigned long long)K, (unsigned long long)A, (unsigned long long)K2w, a->id_n, (const u64 *)a->id_clock,
                       (const u64 *)a->id_keys, b->id_n, (const u64 *)b->id_clock, (const u64 *)b->id_keys,
                       reinterpret_cast<const u64 *>(base + io), reinterpret_cast<u64 *>(base + ic),
                       reinterpret_cast<u64 *>(base + ik), (unsigned long long)Ia, (unsigned long long)Ib);
    CRDT_HIP(ctx, hipGetLastError());
  }
  Pool pl;
  if (int rc = build_pool(ctx, base, at, off, N, A, Kw, ad, bd, pl)) return rc;
  crdt_map_nested_batch in{};
  in.G = N;
  in.R = 2;
  in.K = K;
  in.K2 = K2;
  in.V = VS;
  in.A = A;
  in.clock = reinterpret_cast<const uint64_t *>(base + c2);
  in.ec = reinterpret_cast<const uint64_t *>(base + e2);
  in.ic = reinterpret_cast<const uint64_t *>(base + i2);
  in.iec = reinterpret_cast<const uint64_t *>(base + ie2);
  in.ivc = reinterpret_cast<const uint64_t *>(base + vc2);
  in.ivv = reinterpret_cast<const uint64_t *>(base + vv2);
  in.id_off = reinterpret_cast<const uint64_t *>(base + io);
  in.id_clock = Di ? reinterpret_cast<const uint64_t *>(base + ic) : nullptr;
  in.id_keys = Di ? reinterpret_cast<const uint64_t *>(base + ik) : nullptr;
  in.Di = Di;
  in.def_off = D ? off.data() : nullptr;
  in.def_row = pl.row;
  in.def_clock = reinterpret_cast<const uint64_t *>(pl.clk);
  in.def_keys = reinterpret_cast<const uint64_t *>(pl.key);
  crdt_map_nested_out out{};  // (the packed state layout is the fold's output layout: straight into self)
  out.clock = a->clock;
  out.ec = a->ec;
  out.ic = a->ic;
  out.iec = a->iec;
  out.ivc = a->ivc;
  out.ivv = a->ivv;
  out.nval = a->nval;
  out.id_n = a->id_n;
  out.id_clock = a->id_clock;
  out.id_keys = a->id_keys;
  out.Id = Ia;  // (self's slots: other's lists merge into them, bit 3 past Ia)
  out.Vs = VS;
  out.flags = reinterpret_cast<uint32_t *>(base + of);
  out.def_keep = pl.keep;
  out.def_keys = reinterpret_cast<uint64_t *>(pl.kout);
  if (int rc = crdt_map_nested_lub_many(ctx, &in, &out)) return rc;
  return survive(ctx, pl, N, A, Kw, ad, out.flags, status);
}
