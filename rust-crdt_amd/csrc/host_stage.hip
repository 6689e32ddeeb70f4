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

}  // extern "C"
