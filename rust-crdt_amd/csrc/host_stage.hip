// Host-memory mode (crdt_mem_kind, SURVEY §6 ABI row): with crdt_ctx_set_mem_kind(ctx,
// CRDT_MEM_HOST) the lattice and LWWReg entry points take HOST pointers — the form a Rust
// `lub_many(replicas: Vec<Self>)` / `merge_batch(&mut [Self], Vec<Self>)` starts from — and stage
// them through two ctx-owned device chunk buffers:
//
//   copy stream:  H2D chunk k -> buf[k&1]          (waits until the fold of chunk k-2 left it)
//   ctx stream:   fold / merge of chunk k with CRDT_ACCUMULATE into a device accumulator
//                 (waits for the copy), then the D2H of results
//
// so PCIe transfers of chunk k+1 overlap the HBM pass over chunk k, and inputs larger than the
// device's free memory stream through a bounded window.  A chunked lattice fold is the same fold
// (max / or are associative and commutative, vclock.rs:130-136, gset.rs:38-40); the chunked LWW
// fold continues the exact left fold with CRDT_ACCUMULATE (lwwreg.rs:43-45 -> update :84-98) and
// keeps the FIRST conflicting merge over the whole group by offsetting each chunk's index.
// Host-mode calls are synchronous: results are in the caller's host memory on return.
// Pinned host memory (crdt_host_alloc) is DMA'd directly; pageable memory goes through the HIP
// runtime's own staging.  Entry points without a host path fail with CRDT_EUNSUPPORTED in this
// mode (CRDT_DEVICE_MEM_ONLY in each).
#include "common.hpp"

namespace crdt {

__global__ void lww_fc_combine_kernel(u64 *glob, const u64 *chunk, u64 r0, unsigned long long n) {
  const unsigned long long g = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const u64 c = chunk[g];
  if (glob[g] == ~0ull && c != ~0ull) glob[g] = c + r0;
}

static size_t stage_budget(crdt_ctx *ctx) { return (size_t)ctx->tune.stage_kb << 10; }

// dst row i <- src row i (rows of `width` u64 words at pitches dpitch / spitch; src may be NULL: zeros),
// as a kernel on the ctx stream so it is ordered with the kernels around it
__global__ void copy_rows_kernel(u64 *dst, size_t dpitch, const u64 *src, size_t spitch, size_t width, size_t rows) {
  const size_t n = width * rows;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / width, c = i % width;
    dst[r * dpitch + c] = src ? src[r * spitch + c] : 0;
  }
}
static int dev_rows(crdt_ctx *ctx, u64 *dst, size_t dpitch, const u64 *src, size_t spitch, size_t width, size_t rows) {
  const size_t n = width * rows;
  if (n == 0) return CRDT_OK;
  size_t blocks = (n + kBlock - 1) / kBlock;
  const size_t cap = (size_t)ctx->cu_count * 8;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(copy_rows_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, ctx->stream, dst, dpitch, src, spitch,
                     width, rows);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

// Two chunk buffers of >= bytes each, the copy stream and its events; plus `acc` bytes of
// accumulator (ctx->hacc).
static int ensure_stage(crdt_ctx *ctx, size_t bytes, size_t acc) {
  if (!ctx->hstream) {
    CRDT_HIP(ctx, hipStreamCreateWithFlags(&ctx->hstream, hipStreamNonBlocking));
    for (int b = 0; b < 2; ++b) {
      CRDT_HIP(ctx, hipEventCreateWithFlags(&ctx->hcopied[b], hipEventDisableTiming));
      CRDT_HIP(ctx, hipEventCreateWithFlags(&ctx->hfree[b], hipEventDisableTiming));
    }
  }
  if (bytes > ctx->hbuf_bytes) {
    CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    CRDT_HIP(ctx, hipStreamSynchronize(ctx->hstream));
    for (auto &b : ctx->hbuf)
      if (b) {
        (void)hipFree(b);
        b = nullptr;
      }
    ctx->hbuf_bytes = 0;
    for (auto &b : ctx->hbuf)
      if (hipMalloc(&b, bytes) != hipSuccess) {
        b = nullptr;
        return fail(ctx, CRDT_ENOMEM, "host staging: hipMalloc(%zu) failed", bytes);
      }
    ctx->hbuf_bytes = bytes;
  }
  if (acc > ctx->hacc_bytes) {
    CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->hacc) (void)hipFree(ctx->hacc);
    ctx->hacc = nullptr;
    ctx->hacc_bytes = 0;
    if (hipMalloc(&ctx->hacc, acc) != hipSuccess) {
      ctx->hacc = nullptr;
      return fail(ctx, CRDT_ENOMEM, "host staging: accumulator hipMalloc(%zu) failed", acc);
    }
    ctx->hacc_bytes = acc;
  }
  return CRDT_OK;
}

// A device pointer passed in host mode is a caller error (the copies would read device memory
// as if it were host memory): reject it.  Unregistered (pageable) and pinned host memory pass.
static int check_host(crdt_ctx *ctx, const void *p, const char *what) {
  if (!p) return CRDT_OK;
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return CRDT_OK;
  }
  if (a.type == hipMemoryTypeDevice)
    return fail(ctx, CRDT_EINVAL, "CRDT_MEM_HOST: %s is a device pointer", what);
  return CRDT_OK;
}

// rows x width bytes from a pitched source to a pitched destination (pitch ignored for 1 row).
static hipError_t copy_rows(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width,
                            size_t rows, hipMemcpyKind kind, hipStream_t s) {
  if (rows == 0 || width == 0) return hipSuccess;
  if (rows == 1 || (dpitch == width && spitch == width))
    return hipMemcpyAsync(dst, src, width * rows, kind, s);
  return hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, kind, s);
}

#define STAGE_HIP(expr)                                      \
  do {                                                       \
    hipError_t _e = (expr);                                  \
    if (_e != hipSuccess) return hip_fail(ctx, _e, #expr);   \
  } while (0)

// Chunk k may start copying once the kernel that read buffer k&1 two chunks ago has finished.
static int begin_chunk(crdt_ctx *ctx, int b) {
  STAGE_HIP(hipStreamWaitEvent(ctx->hstream, ctx->hfree[b], 0));
  return CRDT_OK;
}
static int copied_chunk(crdt_ctx *ctx, int b) {
  STAGE_HIP(hipEventRecord(ctx->hcopied[b], ctx->hstream));
  STAGE_HIP(hipStreamWaitEvent(ctx->stream, ctx->hcopied[b], 0));
  return CRDT_OK;
}
static int end_chunk(crdt_ctx *ctx, int b) {
  STAGE_HIP(hipEventRecord(ctx->hfree[b], ctx->stream));
  return CRDT_OK;
}

// Wait for both streams whatever happened, so no queued copy still reads caller memory.
static int finish(crdt_ctx *ctx, int rc) {
  const hipError_t a = hipStreamSynchronize(ctx->hstream);
  const hipError_t b = hipStreamSynchronize(ctx->stream);
  if (rc) return rc;
  if (a != hipSuccess) return hip_fail(ctx, a, "hipStreamSynchronize(copy stream)");
  if (b != hipSuccess) return hip_fail(ctx, b, "hipStreamSynchronize(ctx stream)");
  return CRDT_OK;
}

static int lattice_lub_host_body(crdt_ctx *ctx, Op op, const u64 *in, size_t G, size_t R, size_t W,
                                 size_t row_stride, size_t group_stride, u64 *out, size_t out_stride,
                                 unsigned flags) {
  const bool accumulate = flags & CRDT_ACCUMULATE;
  const size_t rowb = W * 8, budget = stage_budget(ctx);
  const size_t Gc = std::min(G, std::max<size_t>(1, budget / rowb));
  const size_t Rc = R ? std::min(R, std::max<size_t>(1, budget / (Gc * rowb))) : 0;
  if (int rc = ensure_stage(ctx, std::max<size_t>(1, Gc * Rc) * rowb, Gc * rowb)) return rc;
  u64 *acc = static_cast<u64 *>(ctx->hacc);
  const size_t ostride = G > 1 ? out_stride : W;
  size_t k = 0;
  for (size_t g0 = 0; g0 < G; g0 += Gc) {
    const size_t gn = std::min(Gc, G - g0);
    if (accumulate)
      STAGE_HIP(copy_rows(acc, rowb, out + g0 * ostride, ostride * 8, rowb, gn, hipMemcpyHostToDevice, ctx->stream));
    if (R == 0) {
      if (int rc = lattice_lub_many(ctx, op, nullptr, gn, 0, W, W, 0, acc, W, flags)) return rc;
    }
    for (size_t r0 = 0; r0 < R; r0 += Rc, ++k) {
      const size_t rn = std::min(Rc, R - r0);
      const int b = (int)(k & 1);
      u64 *buf = static_cast<u64 *>(ctx->hbuf[b]);
      if (int rc = begin_chunk(ctx, b)) return rc;
      const u64 *src = in + g0 * group_stride + r0 * row_stride;
      if (row_stride == W || rn == 1) {  // each group's chunk is one contiguous run of rn rows
        STAGE_HIP(copy_rows(buf, rn * rowb, src, group_stride * 8, rn * rowb, gn, hipMemcpyHostToDevice, ctx->hstream));
      } else {
        for (size_t g = 0; g < gn; ++g)
          STAGE_HIP(copy_rows(buf + g * rn * W, rowb, src + g * group_stride, row_stride * 8, rowb, rn,
                              hipMemcpyHostToDevice, ctx->hstream));
      }
      if (int rc = copied_chunk(ctx, b)) return rc;
      const unsigned f = (r0 > 0 || accumulate) ? CRDT_ACCUMULATE : 0u;
      if (int rc = lattice_lub_many(ctx, op, buf, gn, rn, W, W, rn * W, acc, W, f)) return rc;
      if (int rc = end_chunk(ctx, b)) return rc;
    }
    STAGE_HIP(copy_rows(out + g0 * ostride, ostride * 8, acc, rowb, rowb, gn, hipMemcpyDeviceToHost, ctx->stream));
  }
  return CRDT_OK;
}

int lattice_lub_many_host(crdt_ctx *ctx, Op op, const u64 *in, size_t G, size_t R, size_t W,
                          size_t row_stride, size_t group_stride, u64 *out, size_t out_stride,
                          unsigned flags) {
  if (G == 0 || W == 0) return CRDT_OK;
  if (!out) return fail(ctx, CRDT_EINVAL, "lub_many: out is NULL");
  if (G > 1 && out_stride < W)
    return fail(ctx, CRDT_EINVAL, "lub_many: out_stride %zu < row width %zu", out_stride, W);
  if (R > 0 && !in) return fail(ctx, CRDT_EINVAL, "lub_many: in is NULL");
  if (R > 1 && row_stride < W)
    return fail(ctx, CRDT_EINVAL, "lub_many: row_stride %zu < row width %zu", row_stride, W);
  if (G > 1 && R > 0 && group_stride < (R - 1) * row_stride + W)
    return fail(ctx, CRDT_EINVAL, "lub_many: group_stride %zu overlaps the previous group", group_stride);
  if (int rc = check_host(ctx, in, "in")) return rc;
  if (int rc = check_host(ctx, out, "out")) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  return finish(ctx, lattice_lub_host_body(ctx, op, in, G, R, W, row_stride, group_stride, out, out_stride, flags));
}

static int lattice_merge_host_body(crdt_ctx *ctx, Op op, u64 *self, const u64 *other, size_t N, size_t W,
                                   size_t self_stride, size_t other_stride) {
  const size_t rowb = W * 8;
  const size_t Nc = std::min(N, std::max<size_t>(1, stage_budget(ctx) / (2 * rowb)));
  if (int rc = ensure_stage(ctx, 2 * Nc * rowb, 8)) return rc;
  const size_t ss = N > 1 ? self_stride : W, os = N > 1 ? other_stride : W;
  size_t k = 0;
  for (size_t i0 = 0; i0 < N; i0 += Nc, ++k) {
    const size_t n = std::min(Nc, N - i0);
    const int b = (int)(k & 1);
    u64 *ds = static_cast<u64 *>(ctx->hbuf[b]), *dO = ds + n * W;
    if (int rc = begin_chunk(ctx, b)) return rc;
    STAGE_HIP(copy_rows(ds, rowb, self + i0 * ss, ss * 8, rowb, n, hipMemcpyHostToDevice, ctx->hstream));
    STAGE_HIP(copy_rows(dO, rowb, other + i0 * os, os * 8, rowb, n, hipMemcpyHostToDevice, ctx->hstream));
    if (int rc = copied_chunk(ctx, b)) return rc;
    if (int rc = lattice_merge_batch(ctx, op, ds, dO, n, W, W, W)) return rc;
    STAGE_HIP(copy_rows(self + i0 * ss, ss * 8, ds, rowb, rowb, n, hipMemcpyDeviceToHost, ctx->stream));
    if (int rc = end_chunk(ctx, b)) return rc;
  }
  return CRDT_OK;
}

int lattice_merge_batch_host(crdt_ctx *ctx, Op op, u64 *self, const u64 *other, size_t N, size_t W,
                             size_t self_stride, size_t other_stride) {
  if (N == 0 || W == 0) return CRDT_OK;
  if (!self || !other) return fail(ctx, CRDT_EINVAL, "merge_batch: NULL buffer");
  if (N > 1 && (self_stride < W || other_stride < W))
    return fail(ctx, CRDT_EINVAL, "merge_batch: stride < row width %zu", W);
  if (int rc = check_host(ctx, self, "self")) return rc;
  if (int rc = check_host(ctx, other, "other")) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  return finish(ctx, lattice_merge_host_body(ctx, op, self, other, N, W, self_stride, other_stride));
}

static int lww_lub_host_body(crdt_ctx *ctx, const u64 *marker, const u64 *val, size_t G, size_t R,
                             size_t group_stride, u64 *out_marker, u64 *out_val, u64 *first_conflict,
                             unsigned flags) {
  const bool accumulate = flags & CRDT_ACCUMULATE;
  const size_t budget = stage_budget(ctx);
  const size_t Gc = std::min(G, std::max<size_t>(1, budget / 16));
  const size_t Rc = std::min(R, std::max<size_t>(1, budget / (Gc * 16)));
  if (int rc = ensure_stage(ctx, Gc * Rc * 16, Gc * 32)) return rc;
  u64 *am = static_cast<u64 *>(ctx->hacc), *av = am + Gc, *fc = av + Gc, *fcc = fc + Gc;
  const size_t gs = G > 1 ? group_stride : R;
  size_t k = 0;
  for (size_t g0 = 0; g0 < G; g0 += Gc) {
    const size_t gn = std::min(Gc, G - g0);
    if (accumulate) {
      STAGE_HIP(hipMemcpyAsync(am, out_marker + g0, gn * 8, hipMemcpyHostToDevice, ctx->stream));
      STAGE_HIP(hipMemcpyAsync(av, out_val + g0, gn * 8, hipMemcpyHostToDevice, ctx->stream));
    }
    for (size_t r0 = 0; r0 < R; r0 += Rc, ++k) {
      const size_t rn = std::min(Rc, R - r0);
      const int b = (int)(k & 1);
      u64 *bm = static_cast<u64 *>(ctx->hbuf[b]), *bv = bm + gn * rn;
      if (int rc = begin_chunk(ctx, b)) return rc;
      STAGE_HIP(copy_rows(bm, rn * 8, marker + g0 * gs + r0, gs * 8, rn * 8, gn, hipMemcpyHostToDevice, ctx->hstream));
      STAGE_HIP(copy_rows(bv, rn * 8, val + g0 * gs + r0, gs * 8, rn * 8, gn, hipMemcpyHostToDevice, ctx->hstream));
      if (int rc = copied_chunk(ctx, b)) return rc;
      const bool first = r0 == 0;
      const unsigned f = (!first || accumulate) ? CRDT_ACCUMULATE : 0u;
      if (int rc = lww_lub_many_dev(ctx, bm, bv, gn, rn, rn, am, av, first_conflict ? (first ? fc : fcc) : nullptr, f))
        return rc;
      if (first_conflict && !first) {
        hipLaunchKernelGGL(lww_fc_combine_kernel, dim3((unsigned)((gn + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           ctx->stream, fc, fcc, (u64)r0, (unsigned long long)gn);
        STAGE_HIP(hipGetLastError());
      }
      if (int rc = end_chunk(ctx, b)) return rc;
    }
    STAGE_HIP(hipMemcpyAsync(out_marker + g0, am, gn * 8, hipMemcpyDeviceToHost, ctx->stream));
    STAGE_HIP(hipMemcpyAsync(out_val + g0, av, gn * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (first_conflict)
      STAGE_HIP(hipMemcpyAsync(first_conflict + g0, fc, gn * 8, hipMemcpyDeviceToHost, ctx->stream));
  }
  return CRDT_OK;
}

int lww_lub_many_host(crdt_ctx *ctx, const u64 *marker, const u64 *val, size_t G, size_t R, size_t group_stride,
                      u64 *out_marker, u64 *out_val, u64 *first_conflict, unsigned flags) {
  if (G == 0) return CRDT_OK;
  const bool accumulate = flags & CRDT_ACCUMULATE;
  if (accumulate && (!out_marker || !out_val))
    return fail(ctx, CRDT_EINVAL, "lwwreg_lub_many: CRDT_ACCUMULATE needs out_marker and out_val");
  if (R == 0 && accumulate) {  // nothing merged: state unchanged, no conflict
    if (first_conflict) std::memset(first_conflict, 0xFF, G * 8);
    return CRDT_OK;
  }
  if (R == 0) return fail(ctx, CRDT_EINVAL, "lwwreg_lub_many: R == 0 (LWWReg has no identity; the fold starts at replica 0)");
  if (!marker || !val) return fail(ctx, CRDT_EINVAL, "lwwreg_lub_many: NULL input");
  if (G > 1 && group_stride < R)
    return fail(ctx, CRDT_EINVAL, "lwwreg_lub_many: group_stride %zu < R %zu", group_stride, R);
  if (!out_marker || !out_val)  // host mode stages whole results: both state outputs are required
    return fail(ctx, CRDT_EINVAL, "lwwreg_lub_many: CRDT_MEM_HOST needs out_marker and out_val");
  for (auto [p, w] : {std::pair<const void *, const char *>{marker, "marker"}, {val, "val"}, {out_marker, "out_marker"},
                      {out_val, "out_val"}, {first_conflict, "first_conflict"}})
    if (int rc = check_host(ctx, p, w)) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  return finish(ctx, lww_lub_host_body(ctx, marker, val, G, R, group_stride, out_marker, out_val, first_conflict, flags));
}

static int lww_merge_host_body(crdt_ctx *ctx, u64 *sm, u64 *sv, const u64 *om, const u64 *ov, size_t N,
                               uint8_t *conflict) {
  const size_t Nc = std::min(N, std::max<size_t>(1, stage_budget(ctx) / 40));
  if (int rc = ensure_stage(ctx, Nc * 40, 8)) return rc;
  size_t k = 0;
  for (size_t i0 = 0; i0 < N; i0 += Nc, ++k) {
    const size_t n = std::min(Nc, N - i0);
    const int b = (int)(k & 1);
    u64 *dsm = static_cast<u64 *>(ctx->hbuf[b]), *dsv = dsm + n, *dom = dsv + n, *dov = dom + n;
    uint8_t *dc = reinterpret_cast<uint8_t *>(dov + n);
    if (int rc = begin_chunk(ctx, b)) return rc;
    STAGE_HIP(hipMemcpyAsync(dsm, sm + i0, n * 8, hipMemcpyHostToDevice, ctx->hstream));
    STAGE_HIP(hipMemcpyAsync(dsv, sv + i0, n * 8, hipMemcpyHostToDevice, ctx->hstream));
    STAGE_HIP(hipMemcpyAsync(dom, om + i0, n * 8, hipMemcpyHostToDevice, ctx->hstream));
    STAGE_HIP(hipMemcpyAsync(dov, ov + i0, n * 8, hipMemcpyHostToDevice, ctx->hstream));
    if (int rc = copied_chunk(ctx, b)) return rc;
    if (int rc = lww_merge_batch_dev(ctx, dsm, dsv, dom, dov, n, conflict ? dc : nullptr)) return rc;
    STAGE_HIP(hipMemcpyAsync(sm + i0, dsm, n * 8, hipMemcpyDeviceToHost, ctx->stream));
    STAGE_HIP(hipMemcpyAsync(sv + i0, dsv, n * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (conflict) STAGE_HIP(hipMemcpyAsync(conflict + i0, dc, n, hipMemcpyDeviceToHost, ctx->stream));
    if (int rc = end_chunk(ctx, b)) return rc;
  }
  return CRDT_OK;
}

int lww_merge_batch_host(crdt_ctx *ctx, u64 *sm, u64 *sv, const u64 *om, const u64 *ov, size_t N, uint8_t *conflict) {
  if (N == 0) return CRDT_OK;
  if (!sm || !sv || !om || !ov) return fail(ctx, CRDT_EINVAL, "lwwreg_merge_batch: NULL buffer");
  for (auto [p, w] : {std::pair<const void *, const char *>{sm, "self_marker"}, {sv, "self_val"}, {om, "other_marker"},
                      {ov, "other_val"}, {conflict, "conflict"}})
    if (int rc = check_host(ctx, p, w)) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  return finish(ctx, lww_merge_host_body(ctx, sm, sv, om, ov, N, conflict));
}

// ---- Orswot: whole-batch staging -----------------------------------------------------------------
// The Orswot join needs every replica of a group before the deferred removes are settled (the
// survival test and the forget ceiling read the final clock), so its host form stages the whole
// batch into device buffers (packed), runs the device entry point, and copies the outputs back.
struct DevScratch {  // device allocations of one host-mode call, freed on every return path
  std::vector<void *> p;
  ~DevScratch() {
    for (void *x : p) (void)hipFree(x);
  }
  template <typename T>
  int get(crdt_ctx *ctx, size_t n, T **out) {
    *out = nullptr;
    if (n == 0) return CRDT_OK;
    void *x = nullptr;
    if (hipMalloc(&x, n * sizeof(T)) != hipSuccess) return fail(ctx, CRDT_ENOMEM, "host staging: hipMalloc(%zu)", n * sizeof(T));
    p.push_back(x);
    *out = static_cast<T *>(x);
    return CRDT_OK;
  }
};

// Run the device-pointer form of an entry point on this ctx (host mode switched off for the call).
struct DeviceModeScope {
  crdt_ctx *c;
  int saved;
  explicit DeviceModeScope(crdt_ctx *x) : c(x), saved(x->mem_kind) { c->mem_kind = CRDT_MEM_DEVICE; }
  ~DeviceModeScope() { c->mem_kind = saved; }
};

static int h2d_async(crdt_ctx *ctx, void *dst, const void *src, size_t bytes) {
  if (!bytes) return CRDT_OK;
  STAGE_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  return CRDT_OK;
}
static int zero_async(crdt_ctx *ctx, void *dst, size_t bytes) {
  if (!bytes) return CRDT_OK;
  STAGE_HIP(hipMemsetAsync(dst, 0, bytes, ctx->stream));
  return CRDT_OK;
}
static int d2h_async(crdt_ctx *ctx, void *dst, const void *src, size_t bytes) {
  if (!bytes || !dst) return CRDT_OK;
  STAGE_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  return CRDT_OK;
}

static int orswot_lub_host_body(crdt_ctx *ctx, const crdt_orswot_batch *in, crdt_orswot_out *out, DevScratch &ds) {
  const size_t G = in->G, R = in->R, M = in->M, A = in->A, Mw = (M + 63) / 64;
  const size_t D = in->def_off ? in->def_off[G] : 0;
  uint64_t *c = nullptr, *e = nullptr, *dc = nullptr, *dm = nullptr, *oc = nullptr, *oe = nullptr, *om = nullptr;
  uint8_t *ok = nullptr;
  if (int rc = ds.get(ctx, G * R * A, &c)) return rc;
  if (int rc = ds.get(ctx, G * R * M * A, &e)) return rc;
  if (int rc = ds.get(ctx, D * A, &dc)) return rc;
  if (int rc = ds.get(ctx, D * Mw, &dm)) return rc;
  if (int rc = ds.get(ctx, G * A, &oc)) return rc;
  if (int rc = ds.get(ctx, G * M * A, &oe)) return rc;
  if (out->def_keep && (int)ds.get(ctx, D, &ok)) return CRDT_ENOMEM;
  if (out->def_members && (int)ds.get(ctx, D * Mw, &om)) return CRDT_ENOMEM;
  const uint64_t *hc = in->clock, *he = in->entries;
  for (size_t g = 0; g < G && R; ++g) {
    STAGE_HIP(copy_rows(c + g * R * A, A * 8, hc + g * in->clock_gstride, in->clock_rstride * 8, A * 8, R,
                        hipMemcpyHostToDevice, ctx->stream));
    if (in->entry_mstride == A || M == 1) {
      STAGE_HIP(copy_rows(e + g * R * M * A, M * A * 8, he + g * in->entry_gstride, in->entry_rstride * 8, M * A * 8, R,
                          hipMemcpyHostToDevice, ctx->stream));
    } else {
      for (size_t r = 0; r < R; ++r)
        STAGE_HIP(copy_rows(e + (g * R + r) * M * A, A * 8, he + g * in->entry_gstride + r * in->entry_rstride,
                            in->entry_mstride * 8, A * 8, M, hipMemcpyHostToDevice, ctx->stream));
    }
  }
  if (int rc = h2d_async(ctx, dc, in->def_clock, D * A * 8)) return rc;
  if (int rc = h2d_async(ctx, dm, in->def_members, D * Mw * 8)) return rc;
  crdt_orswot_batch b = *in;
  b.clock = c;
  b.clock_rstride = A;
  b.clock_gstride = R * A;
  b.entries = e;
  b.entry_mstride = A;
  b.entry_rstride = M * A;
  b.entry_gstride = R * M * A;
  b.def_clock = dc;
  b.def_members = dm;
  crdt_orswot_out o{oc, oe, ok, om};
  {
    DeviceModeScope dev(ctx);
    if (int rc = crdt_orswot_lub_many(ctx, &b, &o)) return rc;
  }
  if (int rc = d2h_async(ctx, out->clock, oc, G * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->entries, oe, G * M * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->def_keep, ok, D)) return rc;
  if (int rc = d2h_async(ctx, out->def_members, om, D * Mw * 8)) return rc;
  return CRDT_OK;
}

// ---- Orswot: replica chunks streamed through the two device chunk buffers ---------------------------
// The join without deferred removes is a left fold (exact for any input: a chunk holding a cell with
// e > c is re-folded in replica order by the join kernel, behind the running join), so the batch
// streams: chunk k's
// replicas are copied (copy stream) into buffer k&1 behind slot 0 of every group, slot 0 holds the
// running join of the chunks before (device-to-device from the accumulator, or zeros: the join's
// identity), and the chunk is joined into the accumulator on the ctx stream while chunk k+1 copies.
// The deferred removes (few: rm clock + member bitmap each) are staged whole and settled once, by
// a last lub_many over the accumulator alone (R = 1: the join of one replica is itself), whose
// survival test and forget ceiling then read the final clock (orswot.rs:141-147, :240-249).
// Device memory: two chunk buffers (tune key stage_kb) + the accumulator + the outputs.
static int orswot_lub_host_stream(crdt_ctx *ctx, const crdt_orswot_batch *in, crdt_orswot_out *out, DevScratch &ds,
                                  size_t Rc) {
  const size_t G = in->G, R = in->R, M = in->M, A = in->A, Mw = (M + 63) / 64;
  const size_t D = in->def_off ? in->def_off[G] : 0;
  const size_t S = Rc + 1;  // replica slots per group in a chunk buffer (slot 0 = the running join)
  const size_t cwords = G * S * A, ewords = G * S * M * A;
  if (int rc = ensure_stage(ctx, (cwords + ewords) * 8, G * (A + M * A) * 8)) return rc;
  uint64_t *acc_c = static_cast<uint64_t *>(ctx->hacc), *acc_e = acc_c + G * A;
  uint64_t *dc = nullptr, *dm = nullptr, *oc = nullptr, *oe = nullptr, *om = nullptr;
  uint8_t *ok = nullptr;
  if (int rc = ds.get(ctx, D * A, &dc)) return rc;
  if (int rc = ds.get(ctx, D * Mw, &dm)) return rc;
  if (int rc = ds.get(ctx, G * A, &oc)) return rc;
  if (int rc = ds.get(ctx, G * M * A, &oe)) return rc;
  if (out->def_keep && (int)ds.get(ctx, D, &ok)) return CRDT_ENOMEM;
  if (out->def_members && (int)ds.get(ctx, D * Mw, &om)) return CRDT_ENOMEM;
  const size_t nch = (R + Rc - 1) / Rc;
  const bool trace = getenv("CRDT_STAGE_TRACE") != nullptr;  // (diagnosis: one stderr line per step)
  for (size_t k = 0; k < nch; ++k) {
    const int b = (int)(k & 1);
    uint64_t *bc = static_cast<uint64_t *>(ctx->hbuf[b]), *be = bc + cwords;
    if (trace) fprintf(stderr, "orswot stream: chunk %zu/%zu Rc %zu S %zu\n", k, nch, Rc, S);
    const size_t r0 = k * Rc, n = std::min(Rc, R - r0);
    if (int rc = begin_chunk(ctx, b)) return rc;
    for (size_t g = 0; g < G; ++g) {  // replicas r0 .. r0+n of group g behind its slot 0
      STAGE_HIP(copy_rows(bc + (g * S + 1) * A, A * 8, in->clock + g * in->clock_gstride + r0 * in->clock_rstride,
                          in->clock_rstride * 8, A * 8, n, hipMemcpyHostToDevice, ctx->hstream));
      STAGE_HIP(copy_rows(be + (g * S + 1) * M * A, M * A * 8,
                          in->entries + g * in->entry_gstride + r0 * in->entry_rstride, in->entry_rstride * 8,
                          M * A * 8, n, hipMemcpyHostToDevice, ctx->hstream));
    }
    if (int rc = copied_chunk(ctx, b)) return rc;
    // slot 0: the join so far, or for the first chunk the join's identity (no dot, zero clock)
    if (int rc = dev_rows(ctx, (u64 *)bc, S * A, k ? (const u64 *)acc_c : nullptr, A, A, G)) return rc;
    if (int rc = dev_rows(ctx, (u64 *)be, S * M * A, k ? (const u64 *)acc_e : nullptr, M * A, M * A, G)) return rc;
    crdt_orswot_batch cb{};
    cb.G = G;
    cb.R = n + 1;
    cb.M = M;
    cb.A = A;
    cb.clock = bc;
    cb.clock_rstride = A;
    cb.clock_gstride = S * A;
    cb.entries = be;
    cb.entry_mstride = A;
    cb.entry_rstride = M * A;
    cb.entry_gstride = S * M * A;
    crdt_orswot_out co{acc_c, acc_e, nullptr, nullptr};
    {
      DeviceModeScope dev(ctx);
      if (int rc = crdt_orswot_lub_many(ctx, &cb, &co)) return rc;
    }
    if (int rc = end_chunk(ctx, b)) return rc;
    if (trace) {
      fprintf(stderr, "orswot stream: chunk %zu queued, syncing\n", k);
      if (int rc = finish(ctx, CRDT_OK)) return rc;
      fprintf(stderr, "orswot stream: chunk %zu done\n", k);
    }
  }
  if (trace) fprintf(stderr, "orswot stream: settling %zu deferred\n", D);
  // the deferred removes, settled once against the final join
  if (int rc = h2d_async(ctx, dc, in->def_clock, D * A * 8)) return rc;
  if (int rc = h2d_async(ctx, dm, in->def_members, D * Mw * 8)) return rc;
  crdt_orswot_batch fb{};
  fb.G = G;
  fb.R = 1;
  fb.M = M;
  fb.A = A;
  fb.clock = acc_c;
  fb.clock_rstride = A;
  fb.clock_gstride = A;
  fb.entries = acc_e;
  fb.entry_mstride = A;
  fb.entry_rstride = M * A;
  fb.entry_gstride = M * A;
  fb.def_off = in->def_off;
  fb.def_clock = dc;
  fb.def_members = dm;
  crdt_orswot_out o{oc, oe, ok, om};
  {
    DeviceModeScope dev(ctx);
    if (int rc = crdt_orswot_lub_many(ctx, &fb, &o)) return rc;
  }
  if (int rc = d2h_async(ctx, out->clock, oc, G * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->entries, oe, G * M * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->def_keep, ok, D)) return rc;
  return d2h_async(ctx, out->def_members, om, D * Mw * 8);
}

int orswot_lub_many_host(crdt_ctx *ctx, const crdt_orswot_batch *in, crdt_orswot_out *out) {
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "orswot_lub_many: NULL batch/out");
  if (in->G == 0 || in->M == 0 || in->A == 0) return CRDT_OK;
  if (!out->clock || !out->entries) return fail(ctx, CRDT_EINVAL, "orswot_lub_many: NULL output");
  if (in->R && (!in->clock || !in->entries)) return fail(ctx, CRDT_EINVAL, "orswot_lub_many: NULL input");
  if (in->R > 1 && (in->clock_rstride < in->A || in->entry_rstride < in->M * in->entry_mstride))
    return fail(ctx, CRDT_EINVAL, "orswot_lub_many: replica strides smaller than a replica");
  if (in->M > 1 && in->entry_mstride < in->A) return fail(ctx, CRDT_EINVAL, "orswot_lub_many: entry_mstride < A");
  for (auto [p, w] : {std::pair<const void *, const char *>{in->clock, "clock"}, {in->entries, "entries"},
                      {in->def_clock, "def_clock"}, {in->def_members, "def_members"}, {out->clock, "out.clock"},
                      {out->entries, "out.entries"}, {out->def_keep, "out.def_keep"}, {out->def_members, "out.def_members"}})
    if (int rc = check_host(ctx, p, w)) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  DevScratch ds;
  // streamed in replica chunks when a chunk of >= 2 replicas per group fits a stage buffer and the
  // member rows are packed; the whole batch staged otherwise
  const size_t rb = (in->A + in->M * in->A) * 8, per = in->G * rb;
  const size_t slots = per ? stage_budget(ctx) / per : 0;
  if (ctx->tune.host_stream && in->R > 1 && slots >= 3 && (in->entry_mstride == in->A || in->M == 1))
    return finish(ctx, orswot_lub_host_stream(ctx, in, out, ds, std::min(slots - 1, in->R)));
  return finish(ctx, orswot_lub_host_body(ctx, in, out, ds));
}

static int orswot_merge_host_body(crdt_ctx *ctx, const crdt_orswot_states *a, const crdt_orswot_states *b,
                                  uint32_t *status, DevScratch &ds) {
  const size_t N = a->N, M = a->M, A = a->A, Mw = (M + 63) / 64;
  crdt_orswot_states d[2] = {*a, *b};
  const crdt_orswot_states *h[2] = {a, b};
  for (int i = 0; i < 2; ++i) {
    const crdt_orswot_states &x = *h[i];
    crdt_orswot_states &y = d[i];
    if (int rc = ds.get(ctx, N * A, &y.clock)) return rc;
    if (int rc = ds.get(ctx, N * M * A, &y.entries)) return rc;
    if (int rc = ds.get(ctx, N * x.Dcap * A, &y.def_clock)) return rc;
    if (int rc = ds.get(ctx, N * x.Dcap * Mw, &y.def_members)) return rc;
    if (int rc = ds.get(ctx, N, &y.def_count)) return rc;
    y.clock_stride = A;
    y.entry_mstride = A;
    y.entry_sstride = M * A;
    STAGE_HIP(copy_rows(y.clock, A * 8, x.clock, x.clock_stride * 8, A * 8, N, hipMemcpyHostToDevice, ctx->stream));
    if (x.entry_mstride == A || M == 1) {
      STAGE_HIP(copy_rows(y.entries, M * A * 8, x.entries, x.entry_sstride * 8, M * A * 8, N, hipMemcpyHostToDevice,
                          ctx->stream));
    } else {
      for (size_t s = 0; s < N; ++s)
        STAGE_HIP(copy_rows(y.entries + s * M * A, A * 8, x.entries + s * x.entry_sstride, x.entry_mstride * 8, A * 8, M,
                            hipMemcpyHostToDevice, ctx->stream));
    }
    if (int rc = h2d_async(ctx, y.def_clock, x.def_clock, N * x.Dcap * A * 8)) return rc;
    if (int rc = h2d_async(ctx, y.def_members, x.def_members, N * x.Dcap * Mw * 8)) return rc;
    if (x.def_count && (int)h2d_async(ctx, y.def_count, x.def_count, N * 4)) return CRDT_EHIP;
    if (!x.def_count) y.def_count = nullptr;
  }
  uint32_t *dst = nullptr;
  if (int rc = ds.get(ctx, N, &dst)) return rc;
  {
    DeviceModeScope dev(ctx);
    if (int rc = crdt_orswot_merge_batch(ctx, &d[0], &d[1], dst)) return rc;
  }
  STAGE_HIP(copy_rows(a->clock, a->clock_stride * 8, d[0].clock, A * 8, A * 8, N, hipMemcpyDeviceToHost, ctx->stream));
  if (a->entry_mstride == A || M == 1) {
    STAGE_HIP(copy_rows(a->entries, a->entry_sstride * 8, d[0].entries, M * A * 8, M * A * 8, N, hipMemcpyDeviceToHost,
                        ctx->stream));
  } else {
    for (size_t s = 0; s < N; ++s)
      STAGE_HIP(copy_rows(a->entries + s * a->entry_sstride, a->entry_mstride * 8, d[0].entries + s * M * A, A * 8, A * 8,
                          M, hipMemcpyDeviceToHost, ctx->stream));
  }
  if (int rc = d2h_async(ctx, a->def_clock, d[0].def_clock, N * a->Dcap * A * 8)) return rc;
  if (int rc = d2h_async(ctx, a->def_members, d[0].def_members, N * a->Dcap * Mw * 8)) return rc;
  if (int rc = d2h_async(ctx, a->def_count, d[0].def_count, N * 4)) return rc;
  return d2h_async(ctx, status, dst, N * 4);
}

int orswot_merge_batch_host(crdt_ctx *ctx, const crdt_orswot_states *self, const crdt_orswot_states *other,
                            uint32_t *status) {
  if (!self || !other || !status) return fail(ctx, CRDT_EINVAL, "orswot_merge_batch: NULL argument");
  const crdt_orswot_states &a = *self, &b = *other;
  if (a.N != b.N || a.M != b.M || a.A != b.A)
    return fail(ctx, CRDT_EINVAL, "orswot_merge_batch: self and other differ in N, M or A");
  if (a.N == 0) return CRDT_OK;
  if (!a.clock || !b.clock || !a.def_count || (a.M && (!a.entries || !b.entries)))
    return fail(ctx, CRDT_EINVAL, "orswot_merge_batch: NULL buffer");
  if (a.clock_stride < a.A || b.clock_stride < b.A || (a.M && (a.entry_mstride < a.A || b.entry_mstride < b.A ||
                                                             a.entry_sstride < a.M * a.entry_mstride ||
                                                             b.entry_sstride < b.M * b.entry_mstride)))
    return fail(ctx, CRDT_EINVAL, "orswot_merge_batch: strides smaller than the rows they hold");
  for (const crdt_orswot_states *x : {self, other})
    for (auto [p, w] : {std::pair<const void *, const char *>{x->clock, "clock"}, {x->entries, "entries"},
                        {x->def_clock, "def_clock"}, {x->def_members, "def_members"}, {x->def_count, "def_count"}})
      if (int rc = check_host(ctx, p, w)) return rc;
  if (int rc = check_host(ctx, status, "status")) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  DevScratch ds;
  return finish(ctx, orswot_merge_host_body(ctx, self, other, status, ds));
}

// ---- Map<K, MVReg<u64>>: whole-batch staging (the fold reads every replica of a key in order) ------
// rows x width words of a (possibly strided) host block into a packed device block
static int h2d_rows(crdt_ctx *ctx, uint64_t *dst, const uint64_t *src, size_t pitch, size_t width, size_t rows) {
  STAGE_HIP(copy_rows(dst, width * 8, src, pitch * 8, width * 8, rows, hipMemcpyHostToDevice, ctx->stream));
  return CRDT_OK;
}
static int d2h_rows(crdt_ctx *ctx, uint64_t *dst, const uint64_t *src, size_t pitch, size_t width, size_t rows) {
  STAGE_HIP(copy_rows(dst, pitch * 8, src, width * 8, width * 8, rows, hipMemcpyDeviceToHost, ctx->stream));
  return CRDT_OK;
}

static int map_lub_host_body(crdt_ctx *ctx, const crdt_map_batch *in, crdt_map_out *out, DevScratch &ds) {
  const size_t G = in->G, R = in->R, K = in->K, A = in->A, V = in->V, Kw = (K + 63) / 64, Vo = out->Vout;
  const size_t D = in->def_off ? in->def_off[G] : 0;
  uint64_t *c, *ec, *vc, *vv, *dc, *dk, *oc, *oec, *ovc, *ovv, *odk = nullptr;
  uint32_t *drow, *onv = nullptr, *ofl;
  uint8_t *okp = nullptr;
  if (int rc = ds.get(ctx, G * R * A, &c)) return rc;
  if (int rc = ds.get(ctx, G * R * K * A, &ec)) return rc;
  if (int rc = ds.get(ctx, G * R * K * V * A, &vc)) return rc;
  if (int rc = ds.get(ctx, G * R * K * V, &vv)) return rc;
  if (int rc = ds.get(ctx, D, &drow)) return rc;
  if (int rc = ds.get(ctx, D * A, &dc)) return rc;
  if (int rc = ds.get(ctx, D * Kw, &dk)) return rc;
  if (int rc = ds.get(ctx, G * A, &oc)) return rc;
  if (int rc = ds.get(ctx, G * K * A, &oec)) return rc;
  if (int rc = ds.get(ctx, G * K * Vo * A, &ovc)) return rc;
  if (int rc = ds.get(ctx, G * K * Vo, &ovv)) return rc;
  if (out->nval)
    if (int rc = ds.get(ctx, G * K, &onv)) return rc;
  if (int rc = ds.get(ctx, G, &ofl)) return rc;
  if (out->def_keep)
    if (int rc = ds.get(ctx, D, &okp)) return rc;
  if (out->def_keys)
    if (int rc = ds.get(ctx, D * Kw, &odk)) return rc;
  for (size_t g = 0; g < G && R; ++g) {  // per replica: one contiguous block of each plane (packed rows)
    if (int rc = h2d_rows(ctx, c + g * R * A, in->clock + g * in->clock_gstride, in->clock_rstride, A, R)) return rc;
    if (int rc = h2d_rows(ctx, ec + g * R * K * A, in->ec + g * in->ec_gstride, in->ec_rstride, K * A, R)) return rc;
    if (int rc = h2d_rows(ctx, vc + g * R * K * V * A, in->vclk + g * in->vclk_gstride, in->vclk_rstride, K * V * A, R))
      return rc;
    if (int rc = h2d_rows(ctx, vv + g * R * K * V, in->vval + g * in->vval_gstride, in->vval_rstride, K * V, R)) return rc;
  }
  if (D) {
    STAGE_HIP(hipMemcpyAsync(drow, in->def_row, D * 4, hipMemcpyHostToDevice, ctx->stream));
    if (int rc = h2d_async(ctx, dc, in->def_clock, D * A * 8)) return rc;
    if (int rc = h2d_async(ctx, dk, in->def_keys, D * Kw * 8)) return rc;
  }
  crdt_map_batch b = *in;
  b.clock = c, b.clock_rstride = A, b.clock_gstride = R * A;
  b.ec = ec, b.ec_rstride = K * A, b.ec_gstride = R * K * A;
  b.vclk = vc, b.vclk_rstride = K * V * A, b.vclk_gstride = R * K * V * A;
  b.vval = vv, b.vval_rstride = K * V, b.vval_gstride = R * K * V;
  b.def_row = D ? drow : nullptr, b.def_clock = D ? dc : nullptr, b.def_keys = D ? dk : nullptr;
  crdt_map_out o{Vo, out->Vstate, oc, oec, ovc, ovv, onv, ofl, okp, odk};
  {
    DeviceModeScope dev(ctx);
    if (int rc = crdt_map_lub_many(ctx, &b, &o)) return rc;
  }
  if (int rc = d2h_async(ctx, out->clock, oc, G * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->ec, oec, G * K * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->vclk, ovc, G * K * Vo * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->vval, ovv, G * K * Vo * 8)) return rc;
  if (int rc = d2h_async(ctx, out->nval, onv, G * K * 4)) return rc;
  if (int rc = d2h_async(ctx, out->flags, ofl, G * 4)) return rc;
  if (int rc = d2h_async(ctx, out->def_keep, okp, D)) return rc;
  return d2h_async(ctx, out->def_keys, odk, D * Kw * 8);
}

// Value planes of n replicas widened from V to Vi slots: key row (r, key) of dw words at
// dst + r*dslot + key*dw = the packed source row (sw words, at src + (r*K + key)*sw), then zeros.
__global__ void widen_planes_kernel(u64 *dst, size_t dslot, const u64 *src, size_t K, size_t n, size_t dw, size_t sw) {
  const size_t total = n * K * dw;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / (K * dw), rem = i % (K * dw), key = rem / dw, c = rem % dw;
    dst[r * dslot + key * dw + c] = c < sw ? src[(r * K + key) * sw + c] : 0;
  }
}

// ---- Map<K, MVReg>: replica chunks, the running fold as replica 0 --------------------------------
// The fold is an exact left fold for any input, and Map::new().merge(acc) == acc for a fold result
// acc (its deferred removes are already applied to it and stay undominated), so
//   fold(r_0 .. r_{n-1}) == fold(acc_k, r_k .. r_{n-1}),  acc_k = fold(r_0 .. r_{k-1})
// (checked on the oracle's Map over op-replay histories: tests/test_oracle_map_assoc.py).  Chunk k is
// copied (copy stream) behind slot 0 of every group, slot 0 holds acc_k (its value slots widened to
// Vi), the chunk's deferred pool = acc_k's surviving removes (held by replica 0) + the removes the
// chunk's replicas hold, and the fold writes acc_{k+1}.  The host reads each chunk's surviving
// removes (a few rows) while the next chunk copies.  A key needing more than Vi value slots sets
// *retry (the caller widens Vi or stages the whole batch).
static int map_lub_host_stream(crdt_ctx *ctx, const crdt_map_batch *in, crdt_map_out *out, DevScratch &ds, size_t Rc,
                               size_t Vi, bool *retry) {
  const size_t G = in->G, R = in->R, K = in->K, A = in->A, V = in->V, Kw = (K + 63) / 64, Vo = out->Vout;
  const size_t D = in->def_off ? in->def_off[G] : 0;
  const size_t S = Rc + 1;
  *retry = false;
  // chunk buffer per group: S slots of [clock A | ec K*A | vclk K*Vi*A | vval K*Vi], then (Vi > V)
  // the chunk's raw value planes [Rc][K*V*A | K*V] widened by a kernel
  const size_t wc = A, we = K * A, wv = K * Vi * A, wvv = K * Vi, slot = wc + we + wv + wvv;
  const bool widen = Vi > V;
  const size_t raw = widen ? Rc * K * V * (A + 1) : 0;
  if (int rc = ensure_stage(ctx, (G * (S * slot + raw)) * 8, (G * slot) * 8)) return rc;
  uint64_t *acc = static_cast<uint64_t *>(ctx->hacc);
  uint64_t *a_c = acc, *a_ec = a_c + G * wc, *a_vc = a_ec + G * we, *a_vv = a_vc + G * wv;
  // the chunk pools: at most the carried survivors (<= D) + the chunk's own removes (<= D)
  const size_t P = 2 * D + 1;
  uint64_t *p_pack = nullptr;  // [P u32 rows, padded | P*A clocks | P*Kw keys]
  uint64_t *p_keys_out = nullptr, *fl_nv = nullptr;
  uint8_t *p_keep = nullptr;
  const size_t rw = (P + 1) / 2;
  if (int rc = ds.get(ctx, rw + P * (A + Kw), &p_pack)) return rc;
  if (int rc = ds.get(ctx, P * Kw, &p_keys_out)) return rc;
  if (int rc = ds.get(ctx, P, &p_keep)) return rc;
  if (int rc = ds.get(ctx, (G + G * K + 1) / 2 + 1, &fl_nv)) return rc;  // flags [G] | nval [G*K] (u32)
  uint32_t *d_flags = reinterpret_cast<uint32_t *>(fl_nv), *d_nval = d_flags + G;
  // carried survivors per group: (original pool index, rm clock, key union)
  struct Carry {
    size_t orig;
    std::vector<uint64_t> clock, keys;
  };
  std::vector<std::vector<Carry>> carry(G);
  std::vector<size_t> dpos(G, 0);  // next of each group's removes (in replica order) not yet pooled
  for (size_t g = 0; g < G; ++g) dpos[g] = in->def_off ? in->def_off[g] : 0;
  const size_t nch = (R + Rc - 1) / Rc;
  auto copy_chunk = [&](size_t k) -> int {
    const int b = (int)(k & 1);
    uint64_t *buf = static_cast<uint64_t *>(ctx->hbuf[b]);
    const size_t r0 = k * Rc, n = std::min(Rc, R - r0);
    if (int rc = begin_chunk(ctx, b)) return rc;
    for (size_t g = 0; g < G; ++g) {
      uint64_t *gb = buf + g * S * slot;  // slot s of group g at gb + s*slot
      STAGE_HIP(copy_rows(gb + slot, slot * 8, in->clock + g * in->clock_gstride + r0 * in->clock_rstride,
                          in->clock_rstride * 8, wc * 8, n, hipMemcpyHostToDevice, ctx->hstream));
      STAGE_HIP(copy_rows(gb + slot + wc, slot * 8, in->ec + g * in->ec_gstride + r0 * in->ec_rstride,
                          in->ec_rstride * 8, we * 8, n, hipMemcpyHostToDevice, ctx->hstream));
      const uint64_t *hv = in->vclk + g * in->vclk_gstride + r0 * in->vclk_rstride;
      const uint64_t *hvv = in->vval + g * in->vval_gstride + r0 * in->vval_rstride;
      if (!widen) {
        STAGE_HIP(copy_rows(gb + slot + wc + we, slot * 8, hv, in->vclk_rstride * 8, wv * 8, n, hipMemcpyHostToDevice,
                            ctx->hstream));
        STAGE_HIP(copy_rows(gb + slot + wc + we + wv, slot * 8, hvv, in->vval_rstride * 8, wvv * 8, n,
                            hipMemcpyHostToDevice, ctx->hstream));
      } else {
        uint64_t *rg = buf + G * S * slot + g * Rc * K * V * (A + 1);
        STAGE_HIP(copy_rows(rg, K * V * A * 8, hv, in->vclk_rstride * 8, K * V * A * 8, n, hipMemcpyHostToDevice,
                            ctx->hstream));
        STAGE_HIP(copy_rows(rg + n * K * V * A, K * V * 8, hvv, in->vval_rstride * 8, K * V * 8, n,
                            hipMemcpyHostToDevice, ctx->hstream));
      }
    }
    STAGE_HIP(hipEventRecord(ctx->hcopied[b], ctx->hstream));
    return CRDT_OK;
  };
  if (nch > 0)
    if (int rc = copy_chunk(0)) return rc;
  std::vector<uint8_t> hkeep;
  std::vector<uint64_t> hkeys;
  std::vector<uint64_t> pack;
  for (size_t k = 0; k < nch; ++k) {
    const int b = (int)(k & 1);
    uint64_t *buf = static_cast<uint64_t *>(ctx->hbuf[b]);
    const size_t r0 = k * Rc, n = std::min(Rc, R - r0);
    if (k + 1 < nch)  // the next chunk copies while this one folds (its buffer: freed by fold k-1)
      if (int rc = copy_chunk(k + 1)) return rc;
    STAGE_HIP(hipStreamWaitEvent(ctx->stream, ctx->hcopied[b], 0));
    for (size_t g = 0; g < G; ++g) {
      uint64_t *gb = buf + g * S * slot;
      if (widen) {  // the raw V-slot planes into the chunk's Vi-slot rows (replicas 1..n)
        const uint64_t *rg = buf + G * S * slot + g * Rc * K * V * (A + 1);
        const size_t blocks = std::min<size_t>((n * K * Vi * A + kBlock - 1) / kBlock, (size_t)ctx->cu_count * 8);
        hipLaunchKernelGGL(widen_planes_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, ctx->stream,
                           (u64 *)(gb + slot + wc + we), slot, (const u64 *)rg, K, n, (size_t)(Vi * A), (size_t)(V * A));
        hipLaunchKernelGGL(widen_planes_kernel, dim3((unsigned)std::max<size_t>(1, blocks / A)), dim3(kBlock), 0,
                           ctx->stream, (u64 *)(gb + slot + wc + we + wv), slot, (const u64 *)(rg + n * K * V * A), K,
                           n, (size_t)Vi, (size_t)V);
        CRDT_HIP(ctx, hipGetLastError());
      }
      // slot 0: acc_k, or the empty Map for the first chunk
      if (int rc = dev_rows(ctx, (u64 *)gb, slot, k ? (const u64 *)(a_c + g * wc) : nullptr, wc, wc, 1)) return rc;
      if (int rc = dev_rows(ctx, (u64 *)(gb + wc), slot, k ? (const u64 *)(a_ec + g * we) : nullptr, we, we, 1)) return rc;
      if (int rc = dev_rows(ctx, (u64 *)(gb + wc + we), slot, k ? (const u64 *)(a_vc + g * wv) : nullptr, wv, wv, 1))
        return rc;
      if (int rc = dev_rows(ctx, (u64 *)(gb + wc + we + wv), slot, k ? (const u64 *)(a_vv + g * wvv) : nullptr, wvv, wvv,
                            1))
        return rc;
    }
    // the chunk's deferred pool, group by group: carried survivors (replica 0), then the removes
    // held by replicas r0 .. r0+n-1 (at rows 1..n)
    std::vector<size_t> poff(G + 1, 0);
    std::vector<size_t> porig;
    std::vector<uint32_t> prow;
    std::vector<uint64_t> pclk, pkeys;
    for (size_t g = 0; g < G; ++g) {
      for (auto &c : carry[g]) {
        porig.push_back(c.orig);
        prow.push_back(0);
        pclk.insert(pclk.end(), c.clock.begin(), c.clock.end());
        pkeys.insert(pkeys.end(), c.keys.begin(), c.keys.end());
      }
      const size_t dend = in->def_off ? in->def_off[g + 1] : 0;
      while (dpos[g] < dend && in->def_row[dpos[g]] < r0 + n) {
        const size_t d = dpos[g]++;
        if (in->def_row[d] < r0) return fail(ctx, CRDT_EINVAL, "map_lub_many: def_row not non-decreasing");
        porig.push_back(d);
        prow.push_back((uint32_t)(in->def_row[d] - r0 + 1));
        pclk.insert(pclk.end(), in->def_clock + d * A, in->def_clock + (d + 1) * A);
        pkeys.insert(pkeys.end(), in->def_keys + d * Kw, in->def_keys + (d + 1) * Kw);
      }
      poff[g + 1] = porig.size();
    }
    const size_t np = porig.size();
    if (np > P) return fail(ctx, CRDT_EINVAL, "map_lub_many: deferred pool past its bound");
    if (np) {
      pack.assign(rw + np * (A + Kw), 0);
      std::memcpy(pack.data(), prow.data(), np * 4);
      std::memcpy(pack.data() + rw, pclk.data(), np * A * 8);
      std::memcpy(pack.data() + rw + np * A, pkeys.data(), np * Kw * 8);
      if (int rc = stage_h2d(ctx, p_pack, pack.data(), pack.size() * 8)) return rc;
    }
    crdt_map_batch cb{};
    cb.G = G;
    cb.R = n + 1;
    cb.K = K;
    cb.A = A;
    cb.V = Vi;
    cb.clock = buf, cb.clock_rstride = slot, cb.clock_gstride = S * slot;
    cb.ec = buf + wc, cb.ec_rstride = slot, cb.ec_gstride = S * slot;
    cb.vclk = buf + wc + we, cb.vclk_rstride = slot, cb.vclk_gstride = S * slot;
    cb.vval = buf + wc + we + wv, cb.vval_rstride = slot, cb.vval_gstride = S * slot;
    if (np) {
      cb.def_off = poff.data();
      cb.def_row = reinterpret_cast<const uint32_t *>(p_pack);
      cb.def_clock = p_pack + rw;
      cb.def_keys = p_pack + rw + np * A;
    }
    size_t vstate = out->Vstate;
    for (;;) {  // a fold state that ran out of value slots reruns this chunk (slot 0 still holds acc_k)
      crdt_map_out co{Vi, vstate, a_c, a_ec, a_vc, a_vv, d_nval, d_flags, np ? p_keep : nullptr,
                      np ? p_keys_out : nullptr};
      {
        DeviceModeScope dev(ctx);
        if (int rc = crdt_map_lub_many(ctx, &cb, &co)) return rc;
      }
      std::vector<uint32_t> hf(G);
      STAGE_HIP(hipMemcpyAsync(hf.data(), d_flags, G * 4, hipMemcpyDeviceToHost, ctx->stream));
      STAGE_HIP(hipStreamSynchronize(ctx->stream));
      uint32_t f = 0;
      for (uint32_t x : hf) f |= x;
      if (f & 2u) return fail(ctx, CRDT_EINVAL, "map_lub_many: def_row not non-decreasing or >= R");
      if ((f & 4u) && vstate < 16) {
        vstate = vstate < 8 ? 8 : 16;
        continue;
      }
      if (f & 5u) {  // a key needs more than Vi slots (or than the state holds): widen / stage whole
        *retry = true;
        return CRDT_OK;
      }
      break;
    }
    STAGE_HIP(hipEventRecord(ctx->hfree[b], ctx->stream));
    // the surviving removes of this chunk's pool are carried into the next (representatives with
    // the union of their clock's key sets)
    if (np) {
      hkeep.resize(np);
      hkeys.resize(np * Kw);
      STAGE_HIP(hipMemcpyAsync(hkeep.data(), p_keep, np, hipMemcpyDeviceToHost, ctx->stream));
      STAGE_HIP(hipMemcpyAsync(hkeys.data(), p_keys_out, np * Kw * 8, hipMemcpyDeviceToHost, ctx->stream));
      STAGE_HIP(hipStreamSynchronize(ctx->stream));
    }
    for (size_t g = 0; g < G; ++g) {
      std::vector<Carry> next;
      for (size_t j = poff[g]; j < poff[g + 1]; ++j)
        if (hkeep[j])
          next.push_back(Carry{porig[j], std::vector<uint64_t>(pclk.begin() + j * A, pclk.begin() + (j + 1) * A),
                               std::vector<uint64_t>(hkeys.begin() + j * Kw, hkeys.begin() + (j + 1) * Kw)});
      carry[g] = std::move(next);
    }
  }
  // outputs: acc (Vi slots) -> the caller's Vout slots; the survivors at their original indices
  std::vector<uint32_t> nv(G * K, 0), hf(G, 0);
  if (nch) {
    STAGE_HIP(hipMemcpyAsync(nv.data(), d_nval, G * K * 4, hipMemcpyDeviceToHost, ctx->stream));
    STAGE_HIP(hipMemcpyAsync(hf.data(), d_flags, G * 4, hipMemcpyDeviceToHost, ctx->stream));
  } else {
    if (int rc = device_fill(ctx, acc, G * slot * 8, 0)) return rc;
  }
  STAGE_HIP(copy_rows(out->clock, A * 8, a_c, A * 8, A * 8, G, hipMemcpyDeviceToHost, ctx->stream));
  STAGE_HIP(copy_rows(out->ec, K * A * 8, a_ec, K * A * 8, K * A * 8, G, hipMemcpyDeviceToHost, ctx->stream));
  const size_t vc = std::min(Vi, Vo);  // value slots per key that reach the caller
  STAGE_HIP(copy_rows(out->vclk, Vo * A * 8, a_vc, Vi * A * 8, vc * A * 8, G * K, hipMemcpyDeviceToHost, ctx->stream));
  STAGE_HIP(copy_rows(out->vval, Vo * 8, a_vv, Vi * 8, vc * 8, G * K, hipMemcpyDeviceToHost, ctx->stream));
  STAGE_HIP(hipStreamSynchronize(ctx->stream));
  for (size_t i = 0; i < G * K; ++i)
    for (size_t s = vc; s < Vo; ++s) {  // slots past the acc's are empty
      std::memset(out->vclk + (i * Vo + s) * A, 0, A * 8);
      out->vval[i * Vo + s] = 0;
    }
  for (size_t g = 0; g < G; ++g) {
    uint32_t f = hf[g] & ~1u;
    for (size_t kk = 0; kk < K; ++kk) f |= nv[g * K + kk] > Vo ? 1u : 0u;
    // a remove held by no replica (def_row >= R) was never pooled: flags bit 1, as the device fold
    // reports it, never a silently dropped remove
    if (in->def_off && dpos[g] != in->def_off[g + 1]) f |= 2u;
    out->flags[g] = f;
  }
  if (out->nval) std::memcpy(out->nval, nv.data(), G * K * 4);
  if (out->def_keep) std::memset(out->def_keep, 0, D);
  if (out->def_keys) std::memset(out->def_keys, 0, D * Kw * 8);
  for (size_t g = 0; g < G; ++g)
    for (auto &c : carry[g]) {
      if (out->def_keep) out->def_keep[c.orig] = 1;
      if (out->def_keys) std::memcpy(out->def_keys + c.orig * Kw, c.keys.data(), Kw * 8);
    }
  return CRDT_OK;
}

// ---- the value-typed Maps (round 5): whole-batch staging ------------------------------------------
// Map<K, GCounter / PNCounter>, Map<K, Orswot> and Map<K, Map<K2, MVReg>> fold every key in replica
// order, so their host form stages the whole batch (packed) into device buffers, runs the device
// entry point and copies the outputs back (synchronous on return, as every host-mode call).
static int map_counter_lub_host_body(crdt_ctx *ctx, const crdt_map_counter_batch *in, crdt_map_counter_out *out,
                                     DevScratch &ds) {
  const size_t G = in->G, R = in->R, K = in->K, A = in->A, W = in->W, Kw = (K + 63) / 64;
  const size_t D = in->def_off ? in->def_off[G] : 0;
  uint64_t *c = nullptr, *e = nullptr, *v = nullptr, *dc = nullptr, *dk = nullptr, *oc = nullptr, *oe = nullptr,
           *ov = nullptr, *ok2 = nullptr;
  uint32_t *dr = nullptr, *of = nullptr;
  uint8_t *okp = nullptr;
  if (int rc = ds.get(ctx, G * R * A, &c)) return rc;
  if (int rc = ds.get(ctx, G * R * K * A, &e)) return rc;
  if (int rc = ds.get(ctx, G * R * K * W * A, &v)) return rc;
  if (int rc = ds.get(ctx, D, &dr)) return rc;
  if (int rc = ds.get(ctx, D * A, &dc)) return rc;
  if (int rc = ds.get(ctx, D * Kw, &dk)) return rc;
  if (int rc = ds.get(ctx, G * A, &oc)) return rc;
  if (int rc = ds.get(ctx, G * K * A, &oe)) return rc;
  if (int rc = ds.get(ctx, G * K * W * A, &ov)) return rc;
  if (int rc = ds.get(ctx, G, &of)) return rc;
  if (out->def_keep)
    if (int rc = ds.get(ctx, D, &okp)) return rc;
  if (out->def_keys)
    if (int rc = ds.get(ctx, D * Kw, &ok2)) return rc;
  for (size_t g = 0; g < G && R; ++g) {
    STAGE_HIP(copy_rows(c + g * R * A, A * 8, in->clock + g * in->clock_gstride, in->clock_rstride * 8, A * 8, R,
                        hipMemcpyHostToDevice, ctx->stream));
    STAGE_HIP(copy_rows(e + g * R * K * A, K * A * 8, in->ec + g * in->ec_gstride, in->ec_rstride * 8, K * A * 8, R,
                        hipMemcpyHostToDevice, ctx->stream));
    STAGE_HIP(copy_rows(v + g * R * K * W * A, K * W * A * 8, in->val + g * in->val_gstride, in->val_rstride * 8,
                        K * W * A * 8, R, hipMemcpyHostToDevice, ctx->stream));
  }
  if (int rc = h2d_async(ctx, dr, in->def_row, D * 4)) return rc;
  if (int rc = h2d_async(ctx, dc, in->def_clock, D * A * 8)) return rc;
  if (int rc = h2d_async(ctx, dk, in->def_keys, D * Kw * 8)) return rc;
  crdt_map_counter_batch b = *in;
  b.clock = c;
  b.clock_rstride = A;
  b.clock_gstride = R * A;
  b.ec = e;
  b.ec_rstride = K * A;
  b.ec_gstride = R * K * A;
  b.val = v;
  b.val_rstride = K * W * A;
  b.val_gstride = R * K * W * A;
  b.def_row = dr;
  b.def_clock = dc;
  b.def_keys = dk;
  crdt_map_counter_out o{oc, oe, ov, of, okp, ok2};
  {
    DeviceModeScope dev(ctx);
    if (int rc = crdt_map_counter_lub_many(ctx, &b, &o)) return rc;
  }
  if (int rc = d2h_async(ctx, out->clock, oc, G * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->ec, oe, G * K * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->val, ov, G * K * W * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->flags, of, G * 4)) return rc;
  if (int rc = d2h_async(ctx, out->def_keep, okp, D)) return rc;
  if (int rc = d2h_async(ctx, out->def_keys, ok2, D * Kw * 8)) return rc;
  return CRDT_OK;
}

int map_counter_lub_many_host(crdt_ctx *ctx, const crdt_map_counter_batch *in, crdt_map_counter_out *out) {
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: NULL batch/out");
  if (in->G == 0 || in->K == 0 || in->A == 0) return CRDT_OK;
  if (in->W != 1 && in->W != 2) return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: W = %zu (1 GCounter, 2 PNCounter)", in->W);
  if (!out->clock || !out->ec || !out->val || !out->flags) return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: NULL output");
  if (in->R && (!in->clock || !in->ec || !in->val)) return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: NULL input");
  const size_t K = in->K, A = in->A, W = in->W;
  if (in->R > 1 && (in->clock_rstride < A || in->ec_rstride < K * A || in->val_rstride < K * W * A))
    return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: replica strides smaller than a replica");
  if (in->def_off && in->def_off[0] != 0) return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: def_off[0] must be 0");
  for (size_t i = 0; in->def_off && i < in->G; ++i)
    if (in->def_off[i + 1] < in->def_off[i]) return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: def_off not non-decreasing");
  if (in->def_off && in->def_off[in->G] && (!in->def_row || !in->def_clock || !in->def_keys))
    return fail(ctx, CRDT_EINVAL, "map_counter_lub_many: NULL deferred input");
  for (auto [p, w] : {std::pair<const void *, const char *>{in->clock, "clock"}, {in->ec, "ec"}, {in->val, "val"},
                      {in->def_row, "def_row"}, {in->def_clock, "def_clock"}, {in->def_keys, "def_keys"},
                      {out->clock, "out.clock"}, {out->ec, "out.ec"}, {out->val, "out.val"}, {out->flags, "out.flags"},
                      {out->def_keep, "out.def_keep"}, {out->def_keys, "out.def_keys"}})
    if (int rc = check_host(ctx, p, w)) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  DevScratch ds;
  return finish(ctx, map_counter_lub_host_body(ctx, in, out, ds));
}

static int map_orswot_lub_host_body(crdt_ctx *ctx, const crdt_map_orswot_batch *in, crdt_map_orswot_out *out,
                                    DevScratch &ds) {
  const size_t G = in->G, R = in->R, K = in->K, M = in->M, A = in->A, Kw = (K + 63) / 64, Dv = in->Dv;
  const size_t D = in->def_off ? in->def_off[G] : 0, N = G * R * K;
  const size_t VD = out->Vd ? out->Vd : 16;  // nested deferred slots per key in the output (crdt_gpu.h)
  const size_t Mw = M > 64 ? (M + 63) / 64 : 1;  // member-mask words
  uint64_t *c, *e, *o, *m, *vo, *vc, *vm, *dc, *dk, *oc, *oe, *oo, *om, *ovc, *ovm, *ok2 = nullptr;
  uint32_t *dr, *ovn, *of;
  uint8_t *okp = nullptr;
  if (int rc = ds.get(ctx, G * R * A, &c)) return rc;
  if (int rc = ds.get(ctx, N * A, &e)) return rc;
  if (int rc = ds.get(ctx, N * A, &o)) return rc;
  if (int rc = ds.get(ctx, N * M * A, &m)) return rc;
  if (int rc = ds.get(ctx, N + 1, &vo)) return rc;
  if (int rc = ds.get(ctx, Dv * A, &vc)) return rc;
  if (int rc = ds.get(ctx, Dv * Mw, &vm)) return rc;
  if (int rc = ds.get(ctx, D, &dr)) return rc;
  if (int rc = ds.get(ctx, D * A, &dc)) return rc;
  if (int rc = ds.get(ctx, D * Kw, &dk)) return rc;
  if (int rc = ds.get(ctx, G * A, &oc)) return rc;
  if (int rc = ds.get(ctx, G * K * A, &oe)) return rc;
  if (int rc = ds.get(ctx, G * K * A, &oo)) return rc;
  if (int rc = ds.get(ctx, G * K * M * A, &om)) return rc;
  if (int rc = ds.get(ctx, G * K * VD * A, &ovc)) return rc;
  if (int rc = ds.get(ctx, G * K * VD * Mw, &ovm)) return rc;
  if (int rc = ds.get(ctx, G * K, &ovn)) return rc;
  if (int rc = ds.get(ctx, G, &of)) return rc;
  if (out->def_keep)
    if (int rc = ds.get(ctx, D, &okp)) return rc;
  if (out->def_keys)
    if (int rc = ds.get(ctx, D * Kw, &ok2)) return rc;
  if (int rc = h2d_async(ctx, c, in->clock, G * R * A * 8)) return rc;
  if (int rc = h2d_async(ctx, e, in->ec, N * A * 8)) return rc;
  if (int rc = h2d_async(ctx, o, in->oc, N * A * 8)) return rc;
  if (int rc = h2d_async(ctx, m, in->ent, N * M * A * 8)) return rc;
  // (vd_off may be NULL when R == 0, as on the device path: the one offset word is then 0)
  if (int rc = in->vd_off ? h2d_async(ctx, vo, in->vd_off, (N + 1) * 8) : zero_async(ctx, vo, (N + 1) * 8)) return rc;
  if (int rc = h2d_async(ctx, vc, in->vd_clock, Dv * A * 8)) return rc;
  if (int rc = h2d_async(ctx, vm, in->vd_mem, Dv * Mw * 8)) return rc;
  if (int rc = h2d_async(ctx, dr, in->def_row, D * 4)) return rc;
  if (int rc = h2d_async(ctx, dc, in->def_clock, D * A * 8)) return rc;
  if (int rc = h2d_async(ctx, dk, in->def_keys, D * Kw * 8)) return rc;
  crdt_map_orswot_batch b = *in;
  b.clock = c;
  b.ec = e;
  b.oc = o;
  b.ent = m;
  b.vd_off = vo;
  b.vd_clock = vc;
  b.vd_mem = vm;
  b.def_row = dr;
  b.def_clock = dc;
  b.def_keys = dk;
  crdt_map_orswot_out ob{oc, oe, oo, om, ovn, ovc, ovm, of, okp, ok2, VD};
  {
    DeviceModeScope dev(ctx);
    if (int rc = crdt_map_orswot_lub_many(ctx, &b, &ob)) return rc;
  }
  if (int rc = d2h_async(ctx, out->clock, oc, G * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->ec, oe, G * K * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->oc, oo, G * K * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->ent, om, G * K * M * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->vd_n, ovn, G * K * 4)) return rc;
  if (int rc = d2h_async(ctx, out->vd_clock, ovc, G * K * VD * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->vd_mem, ovm, G * K * VD * Mw * 8)) return rc;
  if (int rc = d2h_async(ctx, out->flags, of, G * 4)) return rc;
  if (int rc = d2h_async(ctx, out->def_keep, okp, D)) return rc;
  if (int rc = d2h_async(ctx, out->def_keys, ok2, D * Kw * 8)) return rc;
  return CRDT_OK;
}

int map_orswot_lub_many_host(crdt_ctx *ctx, const crdt_map_orswot_batch *in, crdt_map_orswot_out *out) {
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: NULL batch/out");
  if (in->G == 0 || in->K == 0 || in->A == 0) return CRDT_OK;
  if (!out->clock || !out->ec || !out->oc || (in->M && !out->ent) || !out->vd_n || !out->vd_clock || !out->vd_mem ||
      !out->flags)
    return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: NULL output");
  if (in->R && (!in->clock || !in->ec || !in->oc || (in->M && !in->ent) || !in->vd_off))
    return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: NULL input");
  if (in->R && in->Dv && (!in->vd_clock || !in->vd_mem)) return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: NULL vd rows");
  if (in->def_off && in->def_off[0] != 0) return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: def_off[0] must be 0");
  for (size_t i = 0; in->def_off && i < in->G; ++i)
    if (in->def_off[i + 1] < in->def_off[i]) return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: def_off not non-decreasing");
  if (in->def_off && in->def_off[in->G] && (!in->def_row || !in->def_clock || !in->def_keys))
    return fail(ctx, CRDT_EINVAL, "map_orswot_lub_many: NULL deferred input");
  for (auto [p, w] : {std::pair<const void *, const char *>{in->clock, "clock"}, {in->ec, "ec"}, {in->oc, "oc"},
                      {in->ent, "ent"}, {in->vd_off, "vd_off"}, {in->vd_clock, "vd_clock"}, {in->vd_mem, "vd_mem"},
                      {in->def_row, "def_row"}, {in->def_clock, "def_clock"}, {in->def_keys, "def_keys"},
                      {out->clock, "out.clock"}, {out->ec, "out.ec"}, {out->oc, "out.oc"}, {out->ent, "out.ent"},
                      {out->vd_n, "out.vd_n"}, {out->vd_clock, "out.vd_clock"}, {out->vd_mem, "out.vd_mem"},
                      {out->flags, "out.flags"}, {out->def_keep, "out.def_keep"}, {out->def_keys, "out.def_keys"}})
    if (int rc = check_host(ctx, p, w)) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  DevScratch ds;
  return finish(ctx, map_orswot_lub_host_body(ctx, in, out, ds));
}

static int map_nested_lub_host_body(crdt_ctx *ctx, const crdt_map_nested_batch *in, crdt_map_nested_out *out,
                                    DevScratch &ds) {
  const size_t G = in->G, R = in->R, K = in->K, K2 = in->K2, V = in->V, A = in->A, Kw = (K + 63) / 64, Di = in->Di;
  const size_t D = in->def_off ? in->def_off[G] : 0, N = G * R * K;
  const size_t VS = out->Vs ? out->Vs : 8;  // output slots per inner key (crdt_gpu.h)
  const size_t ID = out->Id ? out->Id : 16;  // inner deferred slots per key in the output
  uint64_t *c, *e, *ic, *iec, *ivc, *ivv, *io, *idc, *idk, *dc, *dk, *oc, *oe, *oic, *oiec, *oivc, *oivv, *oidc, *oidk,
      *ok2 = nullptr;
  uint32_t *dr, *onv, *oidn, *of;
  uint8_t *okp = nullptr;
  if (int rc = ds.get(ctx, G * R * A, &c)) return rc;
  if (int rc = ds.get(ctx, N * A, &e)) return rc;
  if (int rc = ds.get(ctx, N * A, &ic)) return rc;
  if (int rc = ds.get(ctx, N * K2 * A, &iec)) return rc;
  if (int rc = ds.get(ctx, N * K2 * V * A, &ivc)) return rc;
  if (int rc = ds.get(ctx, N * K2 * V, &ivv)) return rc;
  if (int rc = ds.get(ctx, N + 1, &io)) return rc;
  if (int rc = ds.get(ctx, Di * A, &idc)) return rc;
  const size_t K2w = K2 > 64 ? (K2 + 63) / 64 : 1;  // inner key-set mask words
  if (int rc = ds.get(ctx, Di * K2w, &idk)) return rc;
  if (int rc = ds.get(ctx, D, &dr)) return rc;
  if (int rc = ds.get(ctx, D * A, &dc)) return rc;
  if (int rc = ds.get(ctx, D * Kw, &dk)) return rc;
  if (int rc = ds.get(ctx, G * A, &oc)) return rc;
  if (int rc = ds.get(ctx, G * K * A, &oe)) return rc;
  if (int rc = ds.get(ctx, G * K * A, &oic)) return rc;
  if (int rc = ds.get(ctx, G * K * K2 * A, &oiec)) return rc;
  if (int rc = ds.get(ctx, G * K * K2 * VS * A, &oivc)) return rc;
  if (int rc = ds.get(ctx, G * K * K2 * VS, &oivv)) return rc;
  if (int rc = ds.get(ctx, G * K * K2, &onv)) return rc;
  if (int rc = ds.get(ctx, G * K, &oidn)) return rc;
  if (int rc = ds.get(ctx, G * K * ID * A, &oidc)) return rc;
  if (int rc = ds.get(ctx, G * K * ID * K2w, &oidk)) return rc;
  if (int rc = ds.get(ctx, G, &of)) return rc;
  if (out->def_keep)
    if (int rc = ds.get(ctx, D, &okp)) return rc;
  if (out->def_keys)
    if (int rc = ds.get(ctx, D * Kw, &ok2)) return rc;
  if (int rc = h2d_async(ctx, c, in->clock, G * R * A * 8)) return rc;
  if (int rc = h2d_async(ctx, e, in->ec, N * A * 8)) return rc;
  if (int rc = h2d_async(ctx, ic, in->ic, N * A * 8)) return rc;
  if (int rc = h2d_async(ctx, iec, in->iec, N * K2 * A * 8)) return rc;
  if (int rc = h2d_async(ctx, ivc, in->ivc, N * K2 * V * A * 8)) return rc;
  if (int rc = h2d_async(ctx, ivv, in->ivv, N * K2 * V * 8)) return rc;
  // (id_off may be NULL when R == 0, as on the device path: the one offset word is then 0)
  if (int rc = in->id_off ? h2d_async(ctx, io, in->id_off, (N + 1) * 8) : zero_async(ctx, io, (N + 1) * 8)) return rc;
  if (int rc = h2d_async(ctx, idc, in->id_clock, Di * A * 8)) return rc;
  if (int rc = h2d_async(ctx, idk, in->id_keys, Di * K2w * 8)) return rc;
  if (int rc = h2d_async(ctx, dr, in->def_row, D * 4)) return rc;
  if (int rc = h2d_async(ctx, dc, in->def_clock, D * A * 8)) return rc;
  if (int rc = h2d_async(ctx, dk, in->def_keys, D * Kw * 8)) return rc;
  crdt_map_nested_batch b = *in;
  b.clock = c;
  b.ec = e;
  b.ic = ic;
  b.iec = iec;
  b.ivc = ivc;
  b.ivv = ivv;
  b.id_off = io;
  b.id_clock = idc;
  b.id_keys = idk;
  b.def_row = dr;
  b.def_clock = dc;
  b.def_keys = dk;
  crdt_map_nested_out ob{oc, oe, oic, oiec, oivc, oivv, onv, oidn, oidc, oidk, of, okp, ok2, ID, VS};
  {
    DeviceModeScope dev(ctx);
    if (int rc = crdt_map_nested_lub_many(ctx, &b, &ob)) return rc;
  }
  if (int rc = d2h_async(ctx, out->clock, oc, G * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->ec, oe, G * K * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->ic, oic, G * K * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->iec, oiec, G * K * K2 * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->ivc, oivc, G * K * K2 * VS * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->ivv, oivv, G * K * K2 * VS * 8)) return rc;
  if (int rc = d2h_async(ctx, out->nval, onv, G * K * K2 * 4)) return rc;
  if (int rc = d2h_async(ctx, out->id_n, oidn, G * K * 4)) return rc;
  if (int rc = d2h_async(ctx, out->id_clock, oidc, G * K * ID * A * 8)) return rc;
  if (int rc = d2h_async(ctx, out->id_keys, oidk, G * K * ID * K2w * 8)) return rc;
  if (int rc = d2h_async(ctx, out->flags, of, G * 4)) return rc;
  if (int rc = d2h_async(ctx, out->def_keep, okp, D)) return rc;
  if (int rc = d2h_async(ctx, out->def_keys, ok2, D * Kw * 8)) return rc;
  return CRDT_OK;
}

int map_nested_lub_many_host(crdt_ctx *ctx, const crdt_map_nested_batch *in, crdt_map_nested_out *out) {
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: NULL batch/out");
  if (in->G == 0 || in->K == 0 || in->A == 0) return CRDT_OK;
  const size_t K2 = in->K2;
  if (!out->clock || !out->ec || !out->ic || (K2 && (!out->iec || !out->ivc || !out->ivv || !out->nval)) || !out->id_n ||
      !out->id_clock || !out->id_keys || !out->flags)
    return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: NULL output");
  if (in->R && (!in->clock || !in->ec || !in->ic || !in->id_off || (K2 && !in->iec) || (K2 && in->V && (!in->ivc || !in->ivv))))
    return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: NULL input");
  if (in->R && in->Di && (!in->id_clock || !in->id_keys)) return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: NULL id rows");
  if (in->def_off && in->def_off[0] != 0) return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: def_off[0] must be 0");
  for (size_t i = 0; in->def_off && i < in->G; ++i)
    if (in->def_off[i + 1] < in->def_off[i]) return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: def_off not non-decreasing");
  if (in->def_off && in->def_off[in->G] && (!in->def_row || !in->def_clock || !in->def_keys))
    return fail(ctx, CRDT_EINVAL, "map_nested_lub_many: NULL deferred input");
  for (auto [p, w] : {std::pair<const void *, const char *>{in->clock, "clock"}, {in->ec, "ec"}, {in->ic, "ic"},
                      {in->iec, "iec"}, {in->ivc, "ivc"}, {in->ivv, "ivv"}, {in->id_off, "id_off"},
                      {in->id_clock, "id_clock"}, {in->id_keys, "id_keys"}, {in->def_row, "def_row"},
                      {in->def_clock, "def_clock"}, {in->def_keys, "def_keys"}, {out->clock, "out.clock"},
                      {out->ec, "out.ec"}, {out->ic, "out.ic"}, {out->iec, "out.iec"}, {out->ivc, "out.ivc"},
                      {out->ivv, "out.ivv"}, {out->nval, "out.nval"}, {out->id_n, "out.id_n"},
                      {out->id_clock, "out.id_clock"}, {out->id_keys, "out.id_keys"}, {out->flags, "out.flags"},
                      {out->def_keep, "out.def_keep"}, {out->def_keys, "out.def_keys"}})
    if (int rc = check_host(ctx, p, w)) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  DevScratch ds;
  return finish(ctx, map_nested_lub_host_body(ctx, in, out, ds));
}

int map_lub_many_host(crdt_ctx *ctx, const crdt_map_batch *in, crdt_map_out *out) {
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "map_lub_many: NULL batch/out");
  if (in->G == 0) return CRDT_OK;
  if (!out->clock || !out->ec || !out->vclk || !out->vval || !out->flags)
    return fail(ctx, CRDT_EINVAL, "map_lub_many: NULL output");
  if (in->R && (!in->clock || !in->ec || !in->vclk || !in->vval))
    return fail(ctx, CRDT_EINVAL, "map_lub_many: NULL input");
  const size_t K = in->K, A = in->A, V = in->V;
  if (in->R > 1 && (in->clock_rstride < A || in->ec_rstride < K * A || in->vclk_rstride < K * V * A ||
                    in->vval_rstride < K * V))
    return fail(ctx, CRDT_EINVAL, "map_lub_many: replica strides smaller than a replica");
  if (in->def_off && in->def_off[in->G] && (!in->def_row || !in->def_clock || !in->def_keys))
    return fail(ctx, CRDT_EINVAL, "map_lub_many: NULL deferred input");
  for (auto [p, w] : {std::pair<const void *, const char *>{in->clock, "clock"}, {in->ec, "ec"}, {in->vclk, "vclk"},
                      {in->vval, "vval"}, {in->def_row, "def_row"}, {in->def_clock, "def_clock"},
                      {in->def_keys, "def_keys"}, {out->clock, "out.clock"}, {out->ec, "out.ec"},
                      {out->vclk, "out.vclk"}, {out->vval, "out.vval"}, {out->nval, "out.nval"},
                      {out->flags, "out.flags"}, {out->def_keep, "out.def_keep"}, {out->def_keys, "out.def_keys"}})
    if (int rc = check_host(ctx, p, w)) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  if (ctx->tune.host_stream && in->R > 1 && V <= 8 && out->Vout > 0) {
    // streamed replica chunks: the running fold's value slots Vi hold the caller's Vout (at most
    // 8, the fold's input limit); a key needing more widens Vi to 8, then stages the whole batch
    size_t Vi = std::max(V, std::min<size_t>(out->Vout, 8));
    for (;;) {
      const size_t slot = A + K * A + K * Vi * A + K * Vi;
      const size_t per = in->G * (slot + (Vi > V ? K * V * (A + 1) : 0)) * 8;
      const size_t slots = per ? stage_budget(ctx) / per : 0;
      if (slots < 3) break;
      DevScratch ds;
      bool retry = false;
      const int rc = finish(ctx, map_lub_host_stream(ctx, in, out, ds, std::min(slots - 1, in->R), Vi, &retry));
      if (rc || !retry) return rc;
      if (Vi >= 8) break;
      Vi = 8;
    }
  }
  DevScratch ds;
  return finish(ctx, map_lub_host_body(ctx, in, out, ds));
}

static int map_merge_host_body(crdt_ctx *ctx, const crdt_map_states *a, const crdt_map_deferred *ad,
                               const crdt_map_states *b, const crdt_map_deferred *bd, uint32_t *status,
                               DevScratch &ds) {
  const size_t N = a->N, K = a->K, A = a->A, Kw = (K + 63) / 64;
  crdt_map_states d[2] = {*a, *b};
  crdt_map_deferred dd[2] = {*ad, *bd};
  const crdt_map_states *h[2] = {a, b};
  const crdt_map_deferred *hd[2] = {ad, bd};
  for (int i = 0; i < 2; ++i) {
    const crdt_map_states &x = *h[i];
    crdt_map_states &y = d[i];
    const size_t V = x.V, Dc = hd[i]->Dcap;
    if (int rc = ds.get(ctx, N * A, &y.clock)) return rc;
    if (int rc = ds.get(ctx, N * K * A, &y.ec)) return rc;
    if (int rc = ds.get(ctx, N * K * V * A, &y.vclk)) return rc;
    if (int rc = ds.get(ctx, N * K * V, &y.vval)) return rc;
    y.clock_stride = A, y.ec_stride = K * A, y.vclk_stride = K * V * A, y.vval_stride = K * V;
    if (int rc = h2d_rows(ctx, y.clock, x.clock, x.clock_stride, A, N)) return rc;
    if (K) {
      if (int rc = h2d_rows(ctx, y.ec, x.ec, x.ec_stride, K * A, N)) return rc;
      if (int rc = h2d_rows(ctx, y.vclk, x.vclk, x.vclk_stride, K * V * A, N)) return rc;
      if (int rc = h2d_rows(ctx, y.vval, x.vval, x.vval_stride, K * V, N)) return rc;
    }
    crdt_map_deferred &z = dd[i];
    if (int rc = ds.get(ctx, N * Dc * A, &z.clock)) return rc;
    if (int rc = ds.get(ctx, N * Dc * Kw, &z.keys)) return rc;
    if (hd[i]->count) {
      if (int rc = ds.get(ctx, N, &z.count)) return rc;
      STAGE_HIP(hipMemcpyAsync(z.count, hd[i]->count, N * 4, hipMemcpyHostToDevice, ctx->stream));
    }
    if (int rc = h2d_async(ctx, z.clock, hd[i]->clock, N * Dc * A * 8)) return rc;
    if (int rc = h2d_async(ctx, z.keys, hd[i]->keys, N * Dc * Kw * 8)) return rc;
  }
  uint32_t *dst = nullptr;
  if (int rc = ds.get(ctx, N, &dst)) return rc;
  {
    DeviceModeScope dev(ctx);
    if (int rc = crdt_map_merge_batch(ctx, &d[0], &dd[0], &d[1], &dd[1], dst)) return rc;
  }
  const size_t V = a->V, Dc = ad->Dcap;
  if (int rc = d2h_rows(ctx, a->clock, d[0].clock, a->clock_stride, A, N)) return rc;
  if (K) {
    if (int rc = d2h_rows(ctx, a->ec, d[0].ec, a->ec_stride, K * A, N)) return rc;
    if (int rc = d2h_rows(ctx, a->vclk, d[0].vclk, a->vclk_stride, K * V * A, N)) return rc;
    if (int rc = d2h_rows(ctx, a->vval, d[0].vval, a->vval_stride, K * V, N)) return rc;
  }
  if (int rc = d2h_async(ctx, ad->clock, dd[0].clock, N * Dc * A * 8)) return rc;
  if (int rc = d2h_async(ctx, ad->keys, dd[0].keys, N * Dc * Kw * 8)) return rc;
  if (int rc = d2h_async(ctx, ad->count, dd[0].count, N * 4)) return rc;
  return d2h_async(ctx, status, dst, N * 4);
}

int map_merge_batch_host(crdt_ctx *ctx, const crdt_map_states *self, const crdt_map_deferred *self_def,
                         const crdt_map_states *other, const crdt_map_deferred *other_def, uint32_t *status) {
  if (!self || !other || !self_def || !other_def || !status)
    return fail(ctx, CRDT_EINVAL, "map_merge_batch: NULL argument");
  const crdt_map_states &a = *self, &b = *other;
  if (a.N != b.N || a.K != b.K || a.A != b.A)
    return fail(ctx, CRDT_EINVAL, "map_merge_batch: self and other differ in N, K or A");
  if (a.N == 0) return CRDT_OK;
  if (!a.clock || !b.clock || !self_def->count || (a.K && (!a.ec || !a.vclk || !a.vval || !b.ec || !b.vclk || !b.vval)))
    return fail(ctx, CRDT_EINVAL, "map_merge_batch: NULL buffer");
  const size_t K = a.K, A = a.A;
  if (a.clock_stride < A || b.clock_stride < A || a.ec_stride < K * A || b.ec_stride < K * A ||
      a.vclk_stride < K * a.V * A || b.vclk_stride < K * b.V * A || a.vval_stride < K * a.V || b.vval_stride < K * b.V)
    return fail(ctx, CRDT_EINVAL, "map_merge_batch: strides smaller than the rows they hold");
  for (const crdt_map_states *x : {self, other})
    for (auto [p, w] : {std::pair<const void *, const char *>{x->clock, "clock"}, {x->ec, "ec"}, {x->vclk, "vclk"},
                        {x->vval, "vval"}})
      if (int rc = check_host(ctx, p, w)) return rc;
  for (const crdt_map_deferred *x : {self_def, other_def})
    for (auto [p, w] : {std::pair<const void *, const char *>{x->clock, "def.clock"}, {x->keys, "def.keys"},
                        {x->count, "def.count"}})
      if (int rc = check_host(ctx, p, w)) return rc;
  if (int rc = check_host(ctx, status, "status")) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  DevScratch ds;
  return finish(ctx, map_merge_host_body(ctx, self, self_def, other, other_def, status, ds));
}

void free_stage(crdt_ctx *ctx) {
  if (ctx->hstream) (void)hipStreamSynchronize(ctx->hstream);
  for (auto &b : ctx->hbuf)
    if (b) (void)hipFree(b);
  if (ctx->hacc) (void)hipFree(ctx->hacc);
  for (int b = 0; b < 2; ++b) {
    if (ctx->hcopied[b]) (void)hipEventDestroy(ctx->hcopied[b]);
    if (ctx->hfree[b]) (void)hipEventDestroy(ctx->hfree[b]);
  }
  if (ctx->hstream) (void)hipStreamDestroy(ctx->hstream);
}

}  // namespace crdt

extern "C" {

int crdt_ctx_set_mem_kind(crdt_ctx *ctx, int kind) {
  CRDT_CHECK_CTX(ctx);
  if (kind != CRDT_MEM_DEVICE && kind != CRDT_MEM_HOST)
    return crdt::fail(ctx, CRDT_EINVAL, "crdt_ctx_set_mem_kind: unknown kind %d", kind);
  ctx->mem_kind = kind;
  return CRDT_OK;
}

int crdt_ctx_mem_kind(const crdt_ctx *ctx) { return ctx ? ctx->mem_kind : CRDT_EINVAL; }

int crdt_host_alloc(size_t bytes, void **out) {
  if (!out) return crdt::fail(nullptr, CRDT_EINVAL, "crdt_host_alloc: out is NULL");
  *out = nullptr;
  if (bytes == 0) return CRDT_OK;
  hipError_t e = hipHostMalloc(out, bytes, hipHostMallocDefault);
  if (e != hipSuccess) {
    *out = nullptr;
    return crdt::fail(nullptr, CRDT_ENOMEM, "crdt_host_alloc(%zu): %s", bytes, hipGetErrorString(e));
  }
  return CRDT_OK;
}

int crdt_host_free(void *p) {
  if (!p) return CRDT_OK;
  hipError_t e = hipHostFree(p);
  return e == hipSuccess ? CRDT_OK : crdt::hip_fail(nullptr, e, "hipHostFree");
}

int crdt_device_alloc(crdt_ctx *ctx, size_t bytes, void **out) {
  CRDT_CHECK_CTX(ctx);
  if (!out) return crdt::fail(ctx, CRDT_EINVAL, "crdt_device_alloc: out is NULL");
  *out = nullptr;
  if (bytes == 0) return CRDT_OK;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  hipError_t e = hipExtMallocWithFlags(out, bytes, hipDeviceMallocContiguous);
  if (e != hipSuccess) {
    *out = nullptr;
    (void)hipGetLastError();  // (not sticky: the caller may fall back)
    return crdt::fail(ctx, CRDT_ENOMEM, "crdt_device_alloc(%zu): %s", bytes, hipGetErrorString(e));
  }
  return CRDT_OK;
}

int crdt_device_free(crdt_ctx *ctx, void *p) {  // (ctx may be NULL: the block knows its device)
  if (!p) return CRDT_OK;
  if (ctx) CRDT_HIP(ctx, hipSetDevice(ctx->device));
  hipError_t e = hipFree(p);
  return e == hipSuccess ? CRDT_OK : crdt::hip_fail(ctx, e, "hipFree");
}

}  // extern "C"
