// Context lifecycle, error reporting, scratch and event timing for libcrdt_gpu.
#include <cstdarg>
#include <cstdlib>

#include "common.hpp"

namespace crdt {

static thread_local std::string g_orphan_error;  // errors raised with ctx == NULL

int fail(crdt_ctx *ctx, int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (ctx) ctx->last_error = buf;
  else g_orphan_error = buf;
  return code;
}

int hip_fail(crdt_ctx *ctx, hipError_t e, const char *what) {
  return fail(ctx, CRDT_EHIP, "%s failed: %s (%d)", what, hipGetErrorString(e), (int)e);
}

int ensure_scratch(crdt_ctx *ctx, size_t bytes) {
  if (bytes <= ctx->scratch_bytes) return CRDT_OK;
  if (ctx->scratch) {
    // The old scratch may still be read by queued kernels: drain the stream first.
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->scratch);
    ctx->scratch = nullptr;
    ctx->scratch_bytes = 0;
  }
  size_t want = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
  hipError_t e = hipMalloc(&ctx->scratch, want);
  if (e != hipSuccess) {
    ctx->scratch = nullptr;
    return fail(ctx, CRDT_ENOMEM, "scratch hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
  }
  ctx->scratch_bytes = want;
  return CRDT_OK;
}

int ensure_dscratch(crdt_ctx *ctx, size_t bytes) {
  if (bytes <= ctx->dscratch_bytes) return CRDT_OK;
  if (ctx->dscratch) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->dscratch);
    ctx->dscratch = nullptr;
    ctx->dscratch_bytes = 0;
  }
  size_t want = bytes < (1u << 16) ? (1u << 16) : bytes + bytes / 4;
  hipError_t e = hipMalloc(&ctx->dscratch, want);
  if (e != hipSuccess) {
    ctx->dscratch = nullptr;
    return fail(ctx, CRDT_ENOMEM, "dscratch hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
  }
  ctx->dscratch_bytes = want;
  return CRDT_OK;
}

int ensure_counters(crdt_ctx *ctx, size_t n) {
  if (n <= ctx->counters_n) return CRDT_OK;
  if (ctx->counters) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->counters);
    ctx->counters = nullptr;
    ctx->counters_n = 0;
  }
  size_t want = n < 16384 ? 16384 : n * 2;
  hipError_t e = hipMalloc(&ctx->counters, want * sizeof(unsigned));
  if (e != hipSuccess) {
    ctx->counters = nullptr;
    return fail(ctx, CRDT_ENOMEM, "counter hipMalloc failed: %s", hipGetErrorString(e));
  }
  ctx->counters_n = want;
  return device_fill(ctx, ctx->counters, want * sizeof(unsigned), 0);
}

int stage_h2d(crdt_ctx *ctx, void *dst, const void *src, size_t bytes) {
  if (bytes == 0) return CRDT_OK;
  if (ctx->pinned_done) {  // the previous staged copy must have left the buffer
    hipError_t e = hipEventSynchronize(ctx->pinned_done);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipEventSynchronize(pinned)");
  } else {
    hipError_t e = hipEventCreateWithFlags(&ctx->pinned_done, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipEventCreate(pinned)");
  }
  if (bytes > ctx->pinned_bytes) {
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    ctx->pinned = nullptr;
    ctx->pinned_bytes = 0;
    size_t want = bytes < 65536 ? 65536 : bytes * 2;
    hipError_t e = hipHostMalloc(&ctx->pinned, want, hipHostMallocDefault);
    if (e != hipSuccess) return fail(ctx, CRDT_ENOMEM, "hipHostMalloc(%zu) failed", want);
    ctx->pinned_bytes = want;
  }
  std::memcpy(ctx->pinned, src, bytes);
  hipError_t e = hipMemcpyAsync(dst, ctx->pinned, bytes, hipMemcpyHostToDevice, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMemcpyAsync(staged)");
  e = hipEventRecord(ctx->pinned_done, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipEventRecord(pinned)");
  return CRDT_OK;
}

// Kernel-based fill: ordered with the kernels around it on the ctx stream like any launch.
// (Small hipMemsetAsync calls were observed to race with the kernels that consume their
// result on the legacy null stream, so nothing a later kernel reads is zeroed by a memset.)
__global__ void fill_u64_kernel(unsigned long long *p, size_t n, unsigned long long v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}
__global__ void fill_u8_kernel(unsigned char *p, size_t n, unsigned char v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

int device_fill(crdt_ctx *ctx, void *dst, size_t bytes, unsigned char byte) {
  if (bytes == 0) return CRDT_OK;
  const bool wide = (reinterpret_cast<uintptr_t>(dst) % 8 == 0) && bytes % 8 == 0;
  const size_t n = wide ? bytes / 8 : bytes;
  size_t blocks = (n + kBlock - 1) / kBlock;
  const size_t cap = (size_t)ctx->cu_count * 8;
  if (blocks > cap) blocks = cap;
  if (wide)
    hipLaunchKernelGGL(fill_u64_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, ctx->stream,
                       (unsigned long long *)dst, n, 0x0101010101010101ULL * byte);
  else
    hipLaunchKernelGGL(fill_u8_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, ctx->stream,
                       (unsigned char *)dst, n, byte);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e, "device_fill");
}

static hipEvent_t take_event(crdt_ctx *ctx) {
  if (!ctx->free_events.empty()) {
    hipEvent_t e = ctx->free_events.back();
    ctx->free_events.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

void timing_begin(crdt_ctx *ctx, const char *name) {
  if (!ctx->timing) return;
  PendingTiming p;
  p.name = name;
  p.start = take_event(ctx);
  p.stop = take_event(ctx);
  (void)hipEventRecord(p.start, ctx->stream);
  ctx->pending.push_back(p);
}

void timing_end(crdt_ctx *ctx) {
  if (!ctx->timing || ctx->pending.empty()) return;
  (void)hipEventRecord(ctx->pending.back().stop, ctx->stream);
}

void timing_add_host(crdt_ctx *ctx, const char *name, double ms) {
  if (!ctx->timing) return;
  auto &t = ctx->timers[name];
  t.total_ms += ms;
  t.launches += 1;
}

static void drain_timings(crdt_ctx *ctx) {
  for (auto &p : ctx->pending) {
    (void)hipEventSynchronize(p.stop);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, p.start, p.stop) == hipSuccess) {
      auto &t = ctx->timers[p.name];
      t.total_ms += ms;
      t.launches += 1;
    }
    ctx->free_events.push_back(p.start);
    ctx->free_events.push_back(p.stop);
  }
  ctx->pending.clear();
}

}  // namespace crdt

using namespace crdt;

extern "C" {

// Launch-geometry knobs "key=value,..." (DESIGN.md §3); unknown keys / values are ignored.
static void apply_tune(crdt_ctx *ctx, const char *t) {
  std::string spec(t);
  size_t pos = 0;
  while (pos < spec.size()) {
    size_t end = spec.find(',', pos);
    if (end == std::string::npos) end = spec.size();
    std::string kv = spec.substr(pos, end - pos);
    size_t eq = kv.find('=');
    if (eq != std::string::npos) {
      std::string k = kv.substr(0, eq);
      int v = atoi(kv.c_str() + eq + 1);
      if (k == "bpc" && v > 0) ctx->tune.lub_blocks_per_cu = v;
      else if (k == "minsteps" && v > 0) ctx->tune.lub_min_steps = v;
      else if (k == "interleave") ctx->tune.lub_interleave = v != 0;
      else if (k == "unroll" && (v == 4 || v == 8 || v == 16 || v == 32)) ctx->tune.lub_unroll = v;
      else if (k == "nt") ctx->tune.lub_nt = v != 0;
      else if (k == "grid" && v > 0) ctx->tune.lub_grid = v;
      else if (k == "mbpc" && v > 0) ctx->tune.merge_blocks_per_cu = v;
      else if (k == "mrows" && (v == 0 || v == 1)) ctx->tune.merge_rows = v;
      else if (k == "obpc" && v > 0) ctx->tune.orswot_blocks_per_cu = v;
      else if (k == "ounroll" && (v == 1 || v == 2 || v == 4)) ctx->tune.orswot_unroll = v;
      else if (k == "ompt" && (v == 4 || v == 8 || v == 16)) ctx->tune.orswot_mpt = v;
      else if (k == "mglds") ctx->tune.map_glds = v != 0;
      else if (k == "mchunk" && (v == 8 || v == 16)) ctx->tune.map_chunk = v;
      else if (k == "mring" && v >= 2 && v <= 4) ctx->tune.map_ring = v;
      else if (k == "mspec") ctx->tune.map_spec = v != 0;
      else if (k == "mnt") ctx->tune.map_nt = v != 0;
      else if (k == "mscan2") ctx->tune.map_scan2 = v != 0;
      else if (k == "mscan3") ctx->tune.map_scan3 = v != 0;
      else if (k == "mrs") ctx->tune.map_rs = v != 0;
      else if (k == "msh") ctx->tune.map_sh = v != 0;
      else if (k == "mst") ctx->tune.map_st = v != 0;
      else if (k == "shagree") ctx->tune.shagree = v != 0;
      else if (k == "mbatch") ctx->tune.map_batch = v != 0;
      else if (k == "mlazyv") ctx->tune.map_lazyv = v != 0;
      else if (k == "mdiag" && v >= 0) ctx->tune.map_diag = v;
      else if (k == "wwalk") ctx->tune.wire_walk = v != 0;
      else if (k == "hstream") ctx->tune.host_stream = v != 0;
      else if (k == "wfill") ctx->tune.wire_fill = v != 0;
      else if (k == "afence") ctx->tune.apply_fence = v != 0;
      else if (k == "alane") ctx->tune.apply_lane = v != 0;
      else if (k == "mfu" && (v == 1 || v == 2 || v == 4)) ctx->tune.merge_flat_u = v;
      else if (k == "mpnt") ctx->tune.map_pair_nt = v != 0;
      else if (k == "mppf") ctx->tune.map_pair_pf = v != 0;
      else if (k == "ohpf") ctx->tune.orswot_apply_hpf = v != 0;
      else if (k == "oal2") ctx->tune.orswot_apply_l2pf = v != 0;
      else if (k == "oameta") ctx->tune.orswot_apply_meta = v != 0;
      else if (k == "oastg") ctx->tune.orswot_apply_stg = v != 0;
      else if (k == "oapf") ctx->tune.orswot_apply_pf = v != 0;
      else if (k == "mcdep") ctx->tune.map_counter_depth = v >= 16 ? 16 : (v <= 4 ? 4 : 8);
      else if (k == "mckpw") ctx->tune.map_counter_kpw = v >= 4 ? 4 : (v >= 2 ? 2 : (v == 1 ? 1 : 0));
      else if (k == "mccs") ctx->tune.map_counter_cs = v ? 1 : 0;
      else if (k == "mccl") ctx->tune.map_counter_cl = v ? 1 : 0;
      else if (k == "mocs") ctx->tune.map_orswot_cs = v ? 1 : 0;
      else if (k == "mowide") ctx->tune.map_orswot_wide = v ? 1 : 0;
      else if (k == "nmlds") ctx->tune.map_nested_lds = v ? 1 : 0;
      else if (k == "mcdma") ctx->tune.map_counter_dma = v >= 16 ? 16 : (v > 0 ? 8 : 0);
      else if (k == "mapf") ctx->tune.map_apply_pf = v != 0;
      else if (k == "mameta") ctx->tune.map_apply_meta = v != 0;
      else if (k == "rbpc" && v > 0) ctx->tune.rows_blocks_per_cu = v;
      else if (k == "hot" && v >= 0 && v <= 64) ctx->tune.apply_hot_slots = v;
      else if (k == "mhot" && v >= 0) ctx->tune.map_apply_hot = v;
      else if (k == "mfv2") ctx->tune.map_forget_vec2 = v != 0;
      else if (k == "stage_kb" && v >= 4) ctx->tune.stage_kb = v;
      else if (k == "mpreg" && v >= 0 && v <= 2) ctx->tune.map_pair_reg = v;
      else if (k == "prows" && (v == 64 || v == 128 || v == 256)) ctx->tune.pair_rows = v;
      else if (k == "pur" && (v == 2 || v == 4 || v == 8)) ctx->tune.pair_ur = v;
      else if (k == "pocc" && v >= 0 && v <= 8) ctx->tune.pair_occ = v;
      else if (k == "mppl" && v >= 1 && v <= 64) ctx->tune.merge_ppl = v;
      else if (k == "mflat" && v >= 0 && v <= 16) ctx->tune.merge_flat = v;
      else if (k == "mpbpc" && v >= 1 && v <= 4096) ctx->tune.map_pair_bpc = v;
      else if (k == "mfbpc" && v >= 1 && v <= 64) ctx->tune.map_forget_bpc = v;
    }
    pos = end + 1;
  }
}

int crdt_ctx_create(int device, crdt_ctx **out) {
  if (!out) return fail(nullptr, CRDT_EINVAL, "crdt_ctx_create: out is NULL");
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return fail(nullptr, CRDT_EHIP, "crdt_ctx_create: no HIP device (%s)", hipGetErrorString(e));
  if (device < 0 || device >= n)
    return fail(nullptr, CRDT_EINVAL, "crdt_ctx_create: device %d out of range [0,%d)", device, n);
  e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(nullptr, e, "hipSetDevice");
  auto *ctx = new crdt_ctx();
  ctx->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    ctx->cu_count = prop.multiProcessorCount;
  if (const char *t = getenv("CRDT_TUNE")) apply_tune(ctx, t);
  *out = ctx;
  return CRDT_OK;
}

int crdt_ctx_destroy(crdt_ctx *ctx) {
  if (!ctx) return CRDT_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (auto &p : ctx->pending) {
    (void)hipEventDestroy(p.start);
    (void)hipEventDestroy(p.stop);
  }
  for (auto e : ctx->free_events) (void)hipEventDestroy(e);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->counters) (void)hipFree(ctx->counters);
  if (ctx->dscratch) (void)hipFree(ctx->dscratch);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
  if (ctx->pinned_done) (void)hipEventDestroy(ctx->pinned_done);
  free_stage(ctx);
  if (ctx->comm && ctx->comm_destroy) ctx->comm_destroy(ctx->comm);
  if (ctx->comm_release) ctx->comm_release(ctx);
  for (void *b : ctx->sbuf)
    if (b) (void)hipFree(b);
  delete ctx;
  return CRDT_OK;
}

int crdt_ctx_set_stream(crdt_ctx *ctx, void *hip_stream) {
  CRDT_CHECK_CTX(ctx);
  ctx->stream = reinterpret_cast<hipStream_t>(hip_stream);
  return CRDT_OK;
}

int crdt_ctx_synchronize(crdt_ctx *ctx) {
  CRDT_CHECK_CTX(ctx);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  // a sharded call on an agreed plan verifies its check words here or at the next sharded call
  if (ctx->comm_check) return ctx->comm_check(ctx);
  return CRDT_OK;
}

const char *crdt_last_error(const crdt_ctx *ctx) {
  return ctx ? ctx->last_error.c_str() : g_orphan_error.c_str();
}

const char *crdt_version(void) { return "0.8.0"; }
int crdt_abi_version(void) { return CRDT_ABI_VERSION; }
const char *crdt_build_target(void) { return "gfx950"; }

int crdt_ctx_set_timing(crdt_ctx *ctx, int enable) {
  CRDT_CHECK_CTX(ctx);
  ctx->timing = enable != 0;
  return CRDT_OK;
}

int crdt_ctx_timing(crdt_ctx *ctx, const char *name, double *total_ms, uint64_t *launches) {
  CRDT_CHECK_CTX(ctx);
  if (!name) return fail(ctx, CRDT_EINVAL, "crdt_ctx_timing: name is NULL");
  drain_timings(ctx);
  auto it = ctx->timers.find(name);
  if (total_ms) *total_ms = it == ctx->timers.end() ? 0.0 : it->second.total_ms;
  if (launches) *launches = it == ctx->timers.end() ? 0 : it->second.launches;
  return CRDT_OK;
}

int crdt_ctx_timing_reset(crdt_ctx *ctx) {
  CRDT_CHECK_CTX(ctx);
  drain_timings(ctx);
  ctx->timers.clear();
  return CRDT_OK;
}

}  // extern "C"

int crdt_ctx_tune(crdt_ctx *ctx, const char *spec) {
  CRDT_CHECK_CTX(ctx);
  if (!spec) return fail(ctx, CRDT_EINVAL, "crdt_ctx_tune: spec is NULL");
  apply_tune(ctx, spec);
  return CRDT_OK;
}
