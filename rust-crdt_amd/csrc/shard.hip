// Replica-sharded lub across the GPUs of a node through the C ABI: one process
// (one crdt_ctx) per GPU, joined into an RCCL communicator by a unique id the caller distributes
// (a Rust caller over its own transport; the Python host over torch.distributed), or into the
// caller's own collectives (crdt_ctx_comm_init_ops: host callbacks, e.g. MPI, TCP or gloo).
//
//   VClock / GCounter / PNCounter: local lub of the rank's replica shard, then ONE in-place
//       all-reduce MAX of the G x W partials over xGMI: max is the join.
//   GSet: local lub, all-gather of the partial bitmaps, OR-fold of the world partials by the
//       same lattice kernel (RCCL has no bitwise-OR reduction).
//   Orswot: each rank joins its shard WITHOUT deferred removes (the dot-store join is associative
//       under the reference invariants), the partial (clock, entries) are all-gathered and every
//       rank re-merges the world partials together with ALL ranks' deferred removes (the forget
//       ceiling and the survival test need the global clock: orswot.rs:141-147, :240-249).
//   LWWReg: the rank states are all-gathered, every rank continues its shard from the fold of the
//       lower ranks' states (the error of lwwreg.rs:84-98 is order-dependent), MIN all-reduce.
//   Map<K, MVReg>: key shards (each rank's keys are an exact left fold), SUM all-reduce of the
//       surviving removes' key bitmaps.
// Every rank ends with the same global result.
//
// Collective discipline (VERDICT r2 / ADVICE r2): every call validates locally and runs its local
// fold, then ONE header all-gather (status + the call's rank-uniform dims) decides for all ranks at
// once whether the data collectives run; every branch around a collective depends on rank-uniform
// values only, so a bad argument or an empty shard on one rank never leaves the others blocked.
// The header exchange runs on a side stream that waits only for the work issued BEFORE the call,
// so it overlaps the local fold instead of adding a host round trip after it.
// RCCL is bound at run time, not at link time: rccl.h supplies only the types and
// enum values (stable across RCCL 2.x), and the nine entry points used here are resolved by dlsym
// from ONE librccl.so.1 chosen in this order:
//   1. $CRDT_RCCL_LIB, when set (an explicit path: the caller names the RCCL it wants);
//   2. the librccl.so.1 the process has already loaded (RTLD_NOLOAD) — inside a torch process that is
//      torch's own RCCL, so the library and torch.distributed share one RCCL;
//   3. librccl.so.1 through the library's RUNPATH (/opt/rocm/lib), for a caller without torch.
// A library loaded by step 3 owns the soname, so a torch imported later binds the same copy.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <mutex>
#include <string>

#include "common.hpp"
#include "shard_host.hpp"

namespace crdt {

static_assert(CRDT_UNIQUE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

// The oldest RCCL whose ABI for these calls this file was checked against (ncclUint64 / ncclMax
// exist since 2.x; the version code is major*10000 + minor*100 + patch since 2.9).
constexpr int kRcclMinVersion = 21800;

struct RcclApi {
  bool ok = false;
  int version = 0;
  std::string path, origin, err;
  ncclResult_t (*GetVersion)(int *) = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char *(*GetErrorString)(ncclResult_t) = nullptr;
};

static bool rccl_bind(RcclApi &a, void *h) {
  auto sym = [&](const char *n) { return dlsym(h, n); };
#define CRDT_RCCL_SYM(field, name) a.field = reinterpret_cast<decltype(a.field)>(sym(name))
  CRDT_RCCL_SYM(GetVersion, "ncclGetVersion");
  CRDT_RCCL_SYM(GetUniqueId, "ncclGetUniqueId");
  CRDT_RCCL_SYM(CommInitRank, "ncclCommInitRank");
  CRDT_RCCL_SYM(CommDestroy, "ncclCommDestroy");
  CRDT_RCCL_SYM(AllReduce, "ncclAllReduce");
  CRDT_RCCL_SYM(AllGather, "ncclAllGather");
  CRDT_RCCL_SYM(GroupStart, "ncclGroupStart");
  CRDT_RCCL_SYM(GroupEnd, "ncclGroupEnd");
  CRDT_RCCL_SYM(GetErrorString, "ncclGetErrorString");
#undef CRDT_RCCL_SYM
  if (!a.GetVersion || !a.GetUniqueId || !a.CommInitRank || !a.CommDestroy || !a.AllReduce || !a.AllGather ||
      !a.GroupStart || !a.GroupEnd || !a.GetErrorString) {
    a.err = "an RCCL entry point is missing from the loaded library";
    return false;
  }
  return true;
}

// Loaded once per process; never unloaded (communicators may outlive any one ctx).
static const RcclApi &rccl() {
  static RcclApi a;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = nullptr;
    const char *env = std::getenv("CRDT_RCCL_LIB");
    if (env && *env) {
      h = dlopen(env, RTLD_NOW | RTLD_LOCAL);
      a.origin = "CRDT_RCCL_LIB";
      if (!h) {
        a.err = std::string("dlopen($CRDT_RCCL_LIB=") + env + "): " + dlerror();
        return;
      }
    } else if ((h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD))) {
      a.origin = "already loaded by the process (shared with torch.distributed when torch is imported)";
    } else if ((h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL))) {
      a.origin = "loaded by libcrdt_gpu (RUNPATH)";
    } else {
      a.err = std::string("dlopen(librccl.so.1): ") + dlerror();
      return;
    }
    if (!rccl_bind(a, h)) return;
    Dl_info info{};
    if (dladdr(reinterpret_cast<void *>(a.GetVersion), &info) && info.dli_fname) a.path = info.dli_fname;
    if (a.GetVersion(&a.version) != ncclSuccess) a.version = 0;
    if (a.version < kRcclMinVersion) {
      a.err = "RCCL version " + std::to_string(a.version) + " at " + a.path + " is older than " +
              std::to_string(kRcclMinVersion);
      return;
    }
    a.ok = true;
  });
  return a;
}

static int need_rccl(crdt_ctx *ctx) {
  const RcclApi &a = rccl();
  if (!a.ok) return fail(ctx, CRDT_ECOMM, "RCCL unavailable: %s", a.err.c_str());
  return CRDT_OK;
}

static int nccl_fail(crdt_ctx *ctx, ncclResult_t r, const char *what) {
  return fail(ctx, CRDT_ECOMM, "%s: %s", what, rccl().GetErrorString(r));
}

#define CRDT_NCCL(ctx, expr)                                   \
  do {                                                         \
    ncclResult_t _r = (expr);                                  \
    if (_r != ncclSuccess) return crdt::nccl_fail((ctx), _r, #expr); \
  } while (0)

#define CRDT_TRY(expr)             \
  do {                             \
    int _s = (expr);               \
    if (_s != CRDT_OK) return _s;  \
  } while (0)

static void destroy_comm(void *c) { (void)rccl().CommDestroy((ncclComm_t)c); }

// ctx-owned exchange buffer slot i (grown on demand, stream drained before a re-allocation)
static int sbuf(crdt_ctx *ctx, int i, size_t bytes, void **out) {
  if (bytes > ctx->sbuf_bytes[i]) {
    if (ctx->sbuf[i]) {
      (void)hipStreamSynchronize(ctx->stream);
      (void)hipFree(ctx->sbuf[i]);
      ctx->sbuf[i] = nullptr;
      ctx->sbuf_bytes[i] = 0;
    }
    const size_t want = bytes < 4096 ? 4096 : bytes + bytes / 8;
    hipError_t e = hipMalloc(&ctx->sbuf[i], want);
    if (e != hipSuccess) {
      ctx->sbuf[i] = nullptr;
      return fail(ctx, CRDT_ENOMEM, "shard buffer hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
    }
    ctx->sbuf_bytes[i] = want;
  }
  *out = ctx->sbuf[i];
  return CRDT_OK;
}

// The check words of the last call on an agreed plan (shard_host.hpp PlanCache): every rank holds the
// same reduced words, so every rank fails the same call here, before any collective of it, and forgets
// its agreed plans (the next calls agree again).  Run after the call's local fold is issued (the
// wait for the earlier call's exchange then overlaps this call's fold).
static int check_pending(crdt_ctx *ctx) {
  if (!ctx->chk_pending) return CRDT_OK;
  ctx->chk_pending = false;
  CRDT_HIP(ctx, hipEventSynchronize(ctx->chk_ev));
  const uint64_t *r = ctx->chk_host + 3;
  if (shard_host::check_ok(r, ctx->chk_key)) return CRDT_OK;
  ctx->plans.clear();
  return fail(ctx, CRDT_ECOMM, "an earlier sharded call on an agreed plan failed: %s; its outputs are unspecified "
              "(every rank reports this at its next sharded call or crdt_ctx_synchronize)",
              r[0] ? "some rank failed its validation (see that rank's crdt_last_error)"
                   : "the ranks called different plans");
}

static int need_comm(crdt_ctx *ctx) {
  if (!ctx->comm && !ctx->has_ops)
    return fail(ctx, CRDT_EINVAL, "sharded call without crdt_ctx_comm_init / crdt_ctx_comm_init_ops");
  return CRDT_OK;
}

// ---- collectives over the ctx's backend: device buffers, ordered on the ctx stream --------------
enum class Red : int { Max = CRDT_RED_MAX, Min = CRDT_RED_MIN, Sum = CRDT_RED_SUM };

static int coll_group_begin(crdt_ctx *ctx) {
  if (ctx->comm) CRDT_NCCL(ctx, rccl().GroupStart());
  return CRDT_OK;
}
static int coll_group_end(crdt_ctx *ctx) {
  if (ctx->comm) CRDT_NCCL(ctx, rccl().GroupEnd());
  return CRDT_OK;
}

static int ops_fail(crdt_ctx *ctx, int rc, const char *what) {
  return fail(ctx, CRDT_ECOMM, "%s: the caller's collective callback returned %d", what, rc);
}

// dst[i] = op over the ranks of src[i] (u64; dst may equal src)
static int coll_allreduce(crdt_ctx *ctx, const u64 *src, u64 *dst, size_t n, Red op) {
  if (n == 0) return CRDT_OK;
  if (ctx->comm) {
    const ncclRedOp_t r = op == Red::Max ? ncclMax : (op == Red::Min ? ncclMin : ncclSum);
    CRDT_NCCL(ctx, rccl().AllReduce(src, dst, n, ncclUint64, r, (ncclComm_t)ctx->comm, ctx->stream));
    return CRDT_OK;
  }
  std::vector<uint64_t> h(n);
  CRDT_HIP(ctx, hipMemcpyAsync(h.data(), src, n * 8, hipMemcpyDeviceToHost, ctx->stream));
  CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (int rc = ctx->ops.allreduce_u64(ctx->ops.user, h.data(), n, (int)op)) return ops_fail(ctx, rc, "allreduce_u64");
  CRDT_HIP(ctx, hipMemcpyAsync(dst, h.data(), n * 8, hipMemcpyHostToDevice, ctx->stream));
  CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return CRDT_OK;
}

// recv[r*bytes ..] = rank r's send bytes
static int coll_allgather(crdt_ctx *ctx, const void *send, void *recv, size_t bytes) {
  if (bytes == 0) return CRDT_OK;
  if (ctx->comm) {
    if (bytes % 8 == 0)
      CRDT_NCCL(ctx, rccl().AllGather(send, recv, bytes / 8, ncclUint64, (ncclComm_t)ctx->comm, ctx->stream));
    else
      CRDT_NCCL(ctx, rccl().AllGather(send, recv, bytes, ncclUint8, (ncclComm_t)ctx->comm, ctx->stream));
    return CRDT_OK;
  }
  std::vector<uint8_t> hs(bytes), hr(bytes * (size_t)ctx->nranks);
  CRDT_HIP(ctx, hipMemcpyAsync(hs.data(), send, bytes, hipMemcpyDeviceToHost, ctx->stream));
  CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (int rc = ctx->ops.allgather(ctx->ops.user, hs.data(), hr.data(), bytes)) return ops_fail(ctx, rc, "allgather");
  CRDT_HIP(ctx, hipMemcpyAsync(recv, hr.data(), hr.size(), hipMemcpyHostToDevice, ctx->stream));
  CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return CRDT_OK;
}

// ---- validation agreement ------------------------------------------------------------------
// Header row of every rank: [failed, tag, d0..d4, hash(all dims)] (shard_host.hpp); tag names the
// entry point.
using shard_host::Hdr;
using shard_host::kHdr;
enum : uint64_t { kTagMax = 1, kTagOr, kTagOrswot, kTagMulti, kTagLww, kTagMap, kTagMapCounter, kTagMapOrswot,
                  kTagMapNested };

static Hdr make_hdr(int st, uint64_t tag, std::initializer_list<uint64_t> dims) {
  return shard_host::make_hdr(st != CRDT_OK, tag, dims);
}

static void comm_release(crdt_ctx *ctx) {
  if (ctx->chk_ev) (void)hipEventSynchronize(ctx->chk_ev);
  if (ctx->chk_dev) (void)hipFree(ctx->chk_dev);
  if (ctx->chk_host) (void)hipHostFree(ctx->chk_host);
  if (ctx->chk_ev) (void)hipEventDestroy(ctx->chk_ev);
  ctx->chk_dev = nullptr;
  ctx->chk_host = nullptr;
  ctx->chk_ev = nullptr;
  ctx->chk_pending = false;
  ctx->plans.clear();
  if (ctx->astream) (void)hipStreamSynchronize(ctx->astream);
  if (ctx->a_dev) (void)hipFree(ctx->a_dev);
  if (ctx->a_host) (void)hipHostFree(ctx->a_host);
  if (ctx->a_main) (void)hipEventDestroy(ctx->a_main);
  if (ctx->a_done) (void)hipEventDestroy(ctx->a_done);
  if (ctx->astream) (void)hipStreamDestroy(ctx->astream);
  ctx->a_dev = ctx->a_host = nullptr;
  ctx->a_main = ctx->a_done = nullptr;
  ctx->astream = nullptr;
  ctx->a_rows = 0;
}

static int agree_setup(crdt_ctx *ctx) {
  const size_t rows = (size_t)ctx->nranks + 1;  // nranks gathered rows + this rank's send row
  if (ctx->a_rows >= rows) return CRDT_OK;
  comm_release(ctx);
  ctx->comm_release = comm_release;
  CRDT_HIP(ctx, hipHostMalloc(&ctx->a_host, rows * kHdr * 8, hipHostMallocDefault));
  CRDT_HIP(ctx, hipMalloc(&ctx->chk_dev, 3 * 8));
  CRDT_HIP(ctx, hipHostMalloc(reinterpret_cast<void **>(&ctx->chk_host), 6 * 8, hipHostMallocDefault));
  CRDT_HIP(ctx, hipEventCreateWithFlags(&ctx->chk_ev, hipEventDisableTiming));
  ctx->comm_check = check_pending;
  if (ctx->comm) {
    CRDT_HIP(ctx, hipMalloc(&ctx->a_dev, rows * kHdr * 8));
    CRDT_HIP(ctx, hipStreamCreateWithFlags(&ctx->astream, hipStreamNonBlocking));
    CRDT_HIP(ctx, hipEventCreateWithFlags(&ctx->a_main, hipEventDisableTiming));
    CRDT_HIP(ctx, hipEventCreateWithFlags(&ctx->a_done, hipEventDisableTiming));
  }
  ctx->a_rows = rows;
  return CRDT_OK;
}

// Call first: marks the work issued before the call (the header exchange waits for it, not for
// the local fold the call issues next).
static int agree_mark(crdt_ctx *ctx) {
  CRDT_TRY(agree_setup(ctx));
  if (ctx->comm) CRDT_HIP(ctx, hipEventRecord(ctx->a_main, ctx->stream));
  return CRDT_OK;
}

// Exchange the headers; CRDT_OK on every rank iff every rank validated and the dims agree.
static int agree_exchange(crdt_ctx *ctx, const Hdr &mine);
// Host wall time of the header round trip is recorded as "shard_agree" (bench.py reports it).
static int agree(crdt_ctx *ctx, int st, const Hdr &mine, const char *what) {
  CRDT_TRY(check_pending(ctx));
  const auto t0 = std::chrono::steady_clock::now();
  const int xr = agree_exchange(ctx, mine);
  timing_add_host(ctx, "shard_agree",
                  std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  if (xr != CRDT_OK) return xr;
  const size_t W = (size_t)ctx->nranks;
  const uint64_t *h = static_cast<const uint64_t *>(ctx->a_host);
  long bad_rank, odd_rank;
  if (shard_host::check_headers(h, W, mine, &bad_rank, &odd_rank)) {
    ctx->plans.add(shard_host::plan_key(mine));
    return CRDT_OK;
  }
  ctx->plans.clear();
  if (bad_rank >= 0) {
    if (st != CRDT_OK) return st;  // this rank's own error text is in last_error
    return fail(ctx, CRDT_ECOMM, "%s: another rank (%ld) failed its validation (see that rank's "
                "crdt_last_error); no data was exchanged", what, bad_rank);
  }
  const uint64_t *o = h + (size_t)odd_rank * kHdr;
  return fail(ctx, CRDT_EINVAL, "%s: the ranks disagree on the call (rank %ld: tag %llu dims %llu %llu %llu %llu "
              "%llu; rank %d: tag %llu dims %llu %llu %llu %llu %llu); no data was exchanged", what, odd_rank,
              (unsigned long long)o[1], (unsigned long long)o[2], (unsigned long long)o[3], (unsigned long long)o[4],
              (unsigned long long)o[5], (unsigned long long)o[6], ctx->rank, (unsigned long long)mine.w[1],
              (unsigned long long)mine.w[2], (unsigned long long)mine.w[3], (unsigned long long)mine.w[4],
              (unsigned long long)mine.w[5], (unsigned long long)mine.w[6]);
}

// The header all-gather itself: rows [0, W) of ctx->a_host <- every rank's header.
static int agree_exchange(crdt_ctx *ctx, const Hdr &mine) {
  const size_t W = (size_t)ctx->nranks;
  uint64_t *h = static_cast<uint64_t *>(ctx->a_host);
  uint64_t *send_h = h + W * kHdr;
  std::memcpy(send_h, mine.w, sizeof mine.w);
  if (ctx->comm) {
    uint64_t *d = static_cast<uint64_t *>(ctx->a_dev);
    CRDT_HIP(ctx, hipStreamWaitEvent(ctx->astream, ctx->a_main, 0));
    CRDT_HIP(ctx, hipMemcpyAsync(d + W * kHdr, send_h, kHdr * 8, hipMemcpyHostToDevice, ctx->astream));
    CRDT_NCCL(ctx, rccl().AllGather(d + W * kHdr, d, kHdr, ncclUint64, (ncclComm_t)ctx->comm, ctx->astream));
    CRDT_HIP(ctx, hipMemcpyAsync(h, d, W * kHdr * 8, hipMemcpyDeviceToHost, ctx->astream));
    CRDT_HIP(ctx, hipEventRecord(ctx->a_done, ctx->astream));
    CRDT_HIP(ctx, hipEventSynchronize(ctx->a_done));
    return CRDT_OK;
  }
  if (int rc = ctx->ops.allgather(ctx->ops.user, send_h, h, kHdr * 8)) return ops_fail(ctx, rc, "allgather");
  return CRDT_OK;
}

// The agreed-plan path (shard_host.hpp PlanCache): this rank's plan was agreed by an earlier call and
// the exchange is MAX all-reduces.  No header exchange; the data collectives run whatever this rank's
// own status (a rank that failed its validation joins with zero partials), and the check words go in
// the same group.  Their copy back is verified at the next sharded call (check_pending).
static bool plan_agreed(crdt_ctx *ctx, const Hdr &mine) {
  return !ctx->tune.shagree && ctx->chk_dev && ctx->plans.has(shard_host::plan_key(mine));
}

static int check_issue(crdt_ctx *ctx, int st, const Hdr &mine) {
  const uint64_t key = shard_host::plan_key(mine);
  shard_host::check_words(st != CRDT_OK, key, ctx->chk_host);
  CRDT_HIP(ctx, hipMemcpyAsync(ctx->chk_dev, ctx->chk_host, 3 * 8, hipMemcpyHostToDevice, ctx->stream));
  return CRDT_OK;
}

static int check_finish(crdt_ctx *ctx, const Hdr &mine) {
  CRDT_HIP(ctx, hipMemcpyAsync(ctx->chk_host + 3, ctx->chk_dev, 3 * 8, hipMemcpyDeviceToHost, ctx->stream));
  CRDT_HIP(ctx, hipEventRecord(ctx->chk_ev, ctx->stream));
  ctx->chk_key = shard_host::plan_key(mine);
  ctx->chk_pending = true;
  return CRDT_OK;
}

static int device_mem_only(crdt_ctx *ctx, const char *what) {
  if (ctx->mem_kind != CRDT_MEM_DEVICE)
    return fail(ctx, CRDT_EUNSUPPORTED, "%s: device pointers only (CRDT_MEM_HOST is supported by the lattice "
                "and lwwreg lub_many / merge_batch)", what);
  return CRDT_OK;
}

// dst row i <- src row idx[i] (rows of W u64 words)
__global__ __launch_bounds__(kBlock) void gather_rows_kernel(u64 *dst, const u64 *src, const uint32_t *idx,
                                                             unsigned long long n, unsigned long long W) {
  const unsigned long long total = n * W;
  for (unsigned long long i = blockIdx.x * (unsigned long long)kBlock + threadIdx.x; i < total;
       i += (unsigned long long)gridDim.x * kBlock) {
    const unsigned long long r = i / W, c = i % W;
    dst[i] = src[(unsigned long long)idx[r] * W + c];
  }
}

static int gather_rows(crdt_ctx *ctx, u64 *dst, const u64 *src, const uint32_t *idx_dev, size_t n, size_t W) {
  if (n == 0 || W == 0) return CRDT_OK;
  const unsigned long long want = (n * W + kBlock - 1) / kBlock;
  const unsigned long long cap = (unsigned long long)ctx->cu_count * 8;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)(want < cap ? want : cap)), dim3(kBlock), 0, ctx->stream,
                     dst, src, idx_dev, (unsigned long long)n, (unsigned long long)W);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

static int lattice_sharded(crdt_ctx *ctx, Op op, const u64 *in, size_t G, size_t R, size_t W, size_t row_stride,
                           size_t group_stride, u64 *out, const char *what) {
  CRDT_CHECK_CTX(ctx);
  CRDT_TRY(need_comm(ctx));
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  CRDT_TRY(agree_mark(ctx));
  const size_t n = G * W;
  int st = device_mem_only(ctx, what);
  void *part = nullptr, *all = nullptr;
  if (!st && n && !out) st = fail(ctx, CRDT_EINVAL, "%s: out is NULL", what);
  if (!st && n) {
    if (op == Op::Max) {
      st = lattice_lub_many(ctx, op, in, G, R, W, row_stride, group_stride, out, W, 0);
    } else {
      st = sbuf(ctx, 0, n * 8, &part);
      if (!st) st = sbuf(ctx, 1, n * 8 * ctx->nranks, &all);
      if (!st) st = lattice_lub_many(ctx, op, in, G, R, W, row_stride, group_stride, (u64 *)part, W, 0);
    }
  }
  const Hdr hd = make_hdr(st, op == Op::Max ? kTagMax : kTagOr, {G, W});
  if (op == Op::Max && n && plan_agreed(ctx, hd)) {  // an agreed plan: the data all-reduce + check words
    CRDT_TRY(check_pending(ctx));
    u64 *buf = out;
    if (st != CRDT_OK || !out) {  // (this rank failed its validation: it joins with a zero partial)
      void *z = nullptr;
      CRDT_TRY(sbuf(ctx, 0, n * 8, &z));
      CRDT_HIP(ctx, hipMemsetAsync(z, 0, n * 8, ctx->stream));
      buf = (u64 *)z;
    }
    CRDT_TRY(check_issue(ctx, st, hd));
    timing_begin(ctx, "shard_exchange");
    CRDT_TRY(coll_group_begin(ctx));
    CRDT_TRY(coll_allreduce(ctx, buf, buf, n, Red::Max));
    CRDT_TRY(coll_allreduce(ctx, (const u64 *)ctx->chk_dev, (u64 *)ctx->chk_dev, 3, Red::Max));
    CRDT_TRY(coll_group_end(ctx));
    timing_end(ctx);
    CRDT_TRY(check_finish(ctx, hd));
    return st;
  }
  CRDT_TRY(agree(ctx, st, hd, what));
  if (n == 0) return CRDT_OK;
  if (op == Op::Max) {
    timing_begin(ctx, "shard_exchange");
    CRDT_TRY(coll_allreduce(ctx, out, out, n, Red::Max));
    timing_end(ctx);
    return CRDT_OK;
  }
  // GSet: partial -> all-gather [nranks][G][W] -> OR over the nranks "replicas" of each group
  timing_begin(ctx, "shard_exchange");
  CRDT_TRY(coll_allgather(ctx, part, all, n * 8));
  timing_end(ctx);
  return lattice_lub_many(ctx, op, (const u64 *)all, G, ctx->nranks, W, n, W, out, W, 0);
}

// LWWReg exchange: tm[g*n + j] / tv[g*n + j] <- marker / val of group g of rank ranks[j] in the
// gathered [nranks][2G+1] buffer (so the world states of a group are one contiguous "replica" row)
__global__ __launch_bounds__(kBlock) void lww_world_rows_kernel(u64 *tm, u64 *tv, const u64 *all,
                                                                const uint32_t *ranks, unsigned long long n,
                                                                unsigned long long G) {
  for (unsigned long long i = blockIdx.x * (unsigned long long)kBlock + threadIdx.x; i < G * n;
       i += (unsigned long long)gridDim.x * kBlock) {
    const unsigned long long g = i / n, j = i % n;
    const u64 *row = all + (unsigned long long)ranks[j] * (2 * G + 1);
    tm[i] = row[g];
    tv[i] = row[G + g];
  }
}

// local first-conflict index -> global (UINT64_MAX stays "none")
__global__ __launch_bounds__(kBlock) void lww_rebase_kernel(u64 *fc, unsigned long long G, u64 base) {
  for (unsigned long long g = blockIdx.x * (unsigned long long)kBlock + threadIdx.x; g < G;
       g += (unsigned long long)gridDim.x * kBlock)
    if (fc[g] != ~0ull) fc[g] += base;
}

// Map key shards: 64 bits of a key bitmap starting at bit `pos` (may be negative or run past
// `nbits`: those bits read as 0)
__device__ __forceinline__ u64 bits64(const u64 *b, long long pos, long long nbits) {
  u64 v = 0;
  for (int t = 0; t < 64; t += 1) {
    const long long q = pos + t;
    if (q >= 0 && q < nbits && ((b[q >> 6] >> (q & 63)) & 1ull)) v |= 1ull << t;
  }
  return v;
}
// dst[d][w] (dw words) = bits [off + 64w, off + 64w + 64) of src[d] (sw words, nbits valid bits),
// i.e. a key range re-indexed from `off` (off < 0: placing a local range at -off)
__global__ __launch_bounds__(kBlock) void bitmap_shift_kernel(u64 *dst, const u64 *src, unsigned long long D,
                                                              unsigned long long dw, unsigned long long sw,
                                                              long long off, long long nbits) {
  for (unsigned long long i = blockIdx.x * (unsigned long long)kBlock + threadIdx.x; i < D * dw;
       i += (unsigned long long)gridDim.x * kBlock) {
    const unsigned long long d = i / dw, w = i % dw;
    dst[i] = bits64(src + d * sw, off + (long long)(w * 64), nbits);
  }
}

static unsigned small_grid(crdt_ctx *ctx, unsigned long long n) {
  const unsigned long long want = (n + kBlock - 1) / kBlock;
  const unsigned long long cap = (unsigned long long)ctx->cu_count * 4;
  return (unsigned)(want == 0 ? 1 : (want < cap ? want : cap));
}

__global__ void widen_u32_kernel(u64 *dst, const uint32_t *src, unsigned long long n, u64 extra) {
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i <= n;
       i += (unsigned long long)gridDim.x * blockDim.x)
    dst[i] = i < n ? (u64)src[i] : extra;
}

}  // namespace crdt

using namespace crdt;

extern "C" {

int crdt_comm_unique_id(uint8_t *id) {
  if (!id) return CRDT_EINVAL;
  if (!rccl().ok) return CRDT_ECOMM;
  ncclUniqueId u;
  if (rccl().GetUniqueId(&u) != ncclSuccess) return CRDT_ECOMM;
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return CRDT_OK;
}

int crdt_ctx_comm_init(crdt_ctx *ctx, const uint8_t *id, int nranks, int rank) {
  CRDT_CHECK_CTX(ctx);
  if (!id || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(ctx, CRDT_EINVAL, "crdt_ctx_comm_init: bad id / nranks %d / rank %d", nranks, rank);
  if (ctx->comm || ctx->has_ops) return fail(ctx, CRDT_EINVAL, "crdt_ctx_comm_init: ctx already has a communicator");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  CRDT_TRY(need_rccl(ctx));
  // which RCCL this communicator runs on (one copy per process: see the binding order above)
  const RcclApi &api = rccl();
  ctx->comm_note = "RCCL " + std::to_string(api.version / 10000) + "." + std::to_string(api.version / 100 % 100) +
                   "." + std::to_string(api.version % 100) + " (" + std::to_string(api.version) + ") at " + api.path +
                   ", " + api.origin;
  ncclUniqueId u;
  std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  CRDT_NCCL(ctx, api.CommInitRank(&c, nranks, u, rank));
  ctx->comm = c;
  ctx->nranks = nranks;
  ctx->rank = rank;
  ctx->comm_destroy = destroy_comm;
  return CRDT_OK;
}

int crdt_ctx_comm_init_ops(crdt_ctx *ctx, const crdt_comm_ops *ops, int nranks, int rank) {
  CRDT_CHECK_CTX(ctx);
  if (!ops || !ops->allgather || !ops->allreduce_u64 || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(ctx, CRDT_EINVAL, "crdt_ctx_comm_init_ops: NULL callbacks / nranks %d / rank %d", nranks, rank);
  if (ctx->comm || ctx->has_ops)
    return fail(ctx, CRDT_EINVAL, "crdt_ctx_comm_init_ops: ctx already has a communicator");
  ctx->ops = *ops;
  ctx->has_ops = true;
  ctx->nranks = nranks;
  ctx->rank = rank;
  ctx->comm_note.clear();
  return CRDT_OK;
}

int crdt_ctx_comm_destroy(crdt_ctx *ctx) {
  CRDT_CHECK_CTX(ctx);
  (void)hipStreamSynchronize(ctx->stream);
  comm_release(ctx);
  if (ctx->comm) CRDT_NCCL(ctx, rccl().CommDestroy((ncclComm_t)ctx->comm));
  ctx->comm = nullptr;
  ctx->has_ops = false;
  ctx->ops = crdt_comm_ops{};
  ctx->nranks = 1;
  ctx->rank = 0;
  return CRDT_OK;
}

int crdt_ctx_comm_info(const crdt_ctx *ctx, int *nranks, int *rank) {
  if (!ctx) return CRDT_EINVAL;
  const bool up = ctx->comm || ctx->has_ops;
  if (nranks) *nranks = up ? ctx->nranks : 0;
  if (rank) *rank = up ? ctx->rank : -1;
  return CRDT_OK;
}

const char *crdt_ctx_comm_note(const crdt_ctx *ctx, int *runtime, int *header) {
  const RcclApi &api = rccl();
  if (runtime) *runtime = api.ok ? api.version : 0;
  if (header) *header = NCCL_VERSION_CODE;
  return ctx ? ctx->comm_note.c_str() : "";
}

int crdt_vclock_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A, size_t row_stride,
                                 size_t group_stride, uint64_t *out) {
  return lattice_sharded(ctx, Op::Max, (const u64 *)in, G, R, A, row_stride, group_stride, (u64 *)out,
                         "vclock_lub_many_sharded");
}
int crdt_gcounter_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                                   size_t row_stride, size_t group_stride, uint64_t *out) {
  return lattice_sharded(ctx, Op::Max, (const u64 *)in, G, R, A, row_stride, group_stride, (u64 *)out,
                         "gcounter_lub_many_sharded");
}
int crdt_pncounter_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                                    size_t row_stride, size_t group_stride, uint64_t *out) {
  return lattice_sharded(ctx, Op::Max, (const u64 *)in, G, R, 2 * A, row_stride, group_stride, (u64 *)out,
                         "pncounter_lub_many_sharded");
}
int crdt_gset_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t words,
                               size_t row_stride, size_t group_stride, uint64_t *out) {
  return lattice_sharded(ctx, Op::Or, (const u64 *)in, G, R, words, row_stride, group_stride, (u64 *)out,
                         "gset_lub_many_sharded");
}

}  // extern "C"

// The per-group deferred counts of device offsets, checked as def_off_check_kernel does: row[g] =
// clamp(off[g+1]) - clamp(off[g]) (g < G), row[G] = D, and *bad |= 1 for an invalid entry
// (off[0] != 0, off[G] != D, an entry past D or below its predecessor).
__global__ __launch_bounds__(kBlock) void def_counts_kernel(const u64 *off, u64 *row, unsigned long long G,
                                                            unsigned long long D, u64 *bad) {
  bool b = false;
  for (unsigned long long i = blockIdx.x * (unsigned long long)kBlock + threadIdx.x; i <= G;
       i += (unsigned long long)gridDim.x * kBlock) {
    const u64 v = off[i];
    b |= i == 0 ? v != 0 : (i == G ? v != D : v > D);
    if (i > 0 && off[i - 1] > v) b = true;
    if (i < G) {
      const u64 lo = v > D ? D : v, hi0 = off[i + 1], hi = hi0 > D ? D : hi0;
      row[i] = hi > lo ? hi - lo : 0;
    } else {
      row[G] = D;
    }
  }
  if (b) atomicOr(bad, 1ull);
}

// Position-aware, order-free hash of device offsets (the sum of a mix of (i, off[i]); u64 wrap):
// the ranks of a key-sharded Map call compare it after their flags exchange.
__global__ __launch_bounds__(kBlock) void def_hash_kernel(const u64 *off, unsigned long long n, u64 *out) {
  u64 h = 0;
  for (unsigned long long i = blockIdx.x * (unsigned long long)kBlock + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * kBlock) {
    u64 z = off[i] ^ (0x9e3779b97f4a7c15ull * (i + 1));
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    h += z ^ (z >> 31);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o);
  if (threadIdx.x % kWave == 0 && h) atomicAdd(out, h);
}

static int orswot_sharded_impl(crdt_ctx *ctx, const crdt_orswot_batch *in, const u64 *doff, size_t Ddev,
                               crdt_orswot_sharded_out *out, const char *what) {
  CRDT_CHECK_CTX(ctx);
  CRDT_TRY(need_comm(ctx));
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  CRDT_TRY(agree_mark(ctx));
  const size_t W = (size_t)ctx->nranks;
  int st = device_mem_only(ctx, what);
  if (!st && (!in || !out || !out->clock || !out->entries || !out->ndef))
    st = fail(ctx, CRDT_EINVAL, "%s: NULL argument", what);
  if (!st && doff && in->def_off) st = fail(ctx, CRDT_EINVAL, "%s: in->def_off must be NULL", what);
  if (!st && !doff && Ddev) st = fail(ctx, CRDT_EINVAL, "%s: D > 0 without def_off", what);
  const size_t G = st ? 0 : in->G, M = st ? 0 : in->M, A = st ? 0 : in->A, Mw = (M + 63) / 64;
  const bool work = G > 0 && A > 0 && M > 0;
  // deferred removes of this rank: per-group counts (device offsets: counted on the device into
  // the exchanged row below, their check travels in that row)
  std::vector<uint64_t> head(G + 1, 0);
  size_t Dk = 0;
  if (!st && work && doff) {
    Dk = Ddev;
    if (Dk && (!in->def_clock || !in->def_members))
      st = fail(ctx, CRDT_EINVAL, "%s: deferred removes without their buffers", what);
    if (!st && Dk > 0xffffffffULL) st = fail(ctx, CRDT_EUNSUPPORTED, "%s: too many deferred removes", what);
  }
  if (!st && work && in->def_off) {
    if (in->def_off[0] != 0) st = fail(ctx, CRDT_EINVAL, "%s: def_off[0] must be 0", what);
    for (size_t g = 0; !st && g < G; ++g) {
      if (in->def_off[g + 1] < in->def_off[g]) st = fail(ctx, CRDT_EINVAL, "%s: def_off not non-decreasing", what);
      else head[g] = in->def_off[g + 1] - in->def_off[g];
    }
    if (!st) Dk = in->def_off[G];
    if (!st && Dk && (!in->def_clock || !in->def_members))
      st = fail(ctx, CRDT_EINVAL, "%s: deferred removes without their buffers", what);
    if (!st && Dk > 0xffffffffULL) st = fail(ctx, CRDT_EUNSUPPORTED, "%s: too many deferred removes", what);
  }
  head[G] = Dk;
  // 1. local join of the shard without deferred removes -> partial (clock, entries); every
  //    buffer of the exchange whose size is known here is allocated before the agreement.  The
  //    exchanged row per rank: [G+1 deferred counts | G "an input cell had E > C" flags | device
  //    offsets invalid].
  const size_t crow = 2 * G + 2;
  void *pc = nullptr, *pe = nullptr, *gc = nullptr, *ge = nullptr, *lcnt = nullptr, *acnt = nullptr;
  crdt_orswot_batch loc{};
  crdt_orswot_out po{};
  OrswotJoinExtra ex{};
  if (!st && work) {
    st = sbuf(ctx, 0, G * A * 8 + G * 4 + 64, &pc);
    if (!st) st = sbuf(ctx, 1, G * M * A * 8, &pe);
    if (!st) st = sbuf(ctx, 2, W * G * A * 8, &gc);
    if (!st) st = sbuf(ctx, 3, W * G * M * A * 8, &ge);
    if (!st) st = sbuf(ctx, 4, crow * 8, &lcnt);
    if (!st) st = sbuf(ctx, 5, W * crow * 8, &acnt);
    if (!st) {
      loc = *in;
      loc.def_off = nullptr;
      po = crdt_orswot_out{(uint64_t *)pc, (uint64_t *)pe, nullptr, nullptr};
      ex.viol = reinterpret_cast<unsigned *>((u64 *)pc + G * A);
      st = orswot_lub_many_ex(ctx, &loc, &po, ex);
    }
    if (!st) {  // the G flags, then word 2G+1 = 0 (widen writes G+1 words: the last is `extra`)
      hipLaunchKernelGGL(widen_u32_kernel, dim3(small_grid(ctx, G + 1)), dim3(kBlock), 0, ctx->stream,
                         (u64 *)lcnt + G + 1, (const unsigned *)ex.viol, (unsigned long long)G, (u64)0);
      if (hipGetLastError() != hipSuccess) st = fail(ctx, CRDT_EHIP, "%s: widen_u32_kernel launch", what);
    }
    if (!st && doff) {  // counts and the offsets' check (into word 2G+1) on the device, after widen
      hipLaunchKernelGGL(def_counts_kernel, dim3(small_grid(ctx, G + 1)), dim3(kBlock), 0, ctx->stream, doff,
                         (u64 *)lcnt, (unsigned long long)G, (unsigned long long)Dk, (u64 *)lcnt + 2 * G + 1);
      if (hipGetLastError() != hipSuccess) st = fail(ctx, CRDT_EHIP, "%s: def_counts_kernel launch", what);
    } else if (!st) {
      st = stage_h2d(ctx, lcnt, head.data(), (G + 1) * 8);  // (host offsets were checked above)
    }
  }
  CRDT_TRY(agree(ctx, st, make_hdr(st, kTagOrswot, {G, M, A}), what));
  if (!work) {
    *out->ndef = 0;
    return CRDT_OK;
  }
  // 2. all-gather the partials: replica (g, r) of the re-merge at r*G*A + g*A (+ m*A), and the
  //    per-group deferred counts of every rank
  timing_begin(ctx, "shard_exchange");
  CRDT_TRY(coll_group_begin(ctx));
  CRDT_TRY(coll_allgather(ctx, pc, gc, G * A * 8));
  CRDT_TRY(coll_allgather(ctx, pe, ge, G * M * A * 8));
  CRDT_TRY(coll_allgather(ctx, lcnt, acnt, crow * 8));
  CRDT_TRY(coll_group_end(ctx));
  std::vector<uint64_t> rows(crow * W), all((G + 1) * W);
  CRDT_HIP(ctx, hipMemcpyAsync(rows.data(), acnt, rows.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  bool chain = false;  // some rank's shard holds a cell with E > C (rank-uniform: gathered flags)
  long bad_off = -1;   // the first rank whose device offsets failed their check
  for (size_t r = 0; r < W; ++r) {
    std::copy(rows.begin() + r * crow, rows.begin() + r * crow + G + 1, all.begin() + r * (G + 1));
    for (size_t g = 0; g < G; ++g) chain = chain || (rows[r * crow + G + 1 + g] & 1);
    if (bad_off < 0 && rows[r * crow + 2 * G + 1]) bad_off = (long)r;
  }
  timing_end(ctx);
  if (bad_off >= 0) {  // every rank saw the same rows: all return here, before any deferred row moves
    if (bad_off == (long)ctx->rank)
      return fail(ctx, CRDT_EINVAL, "%s: invalid def_off (entry 0 must be 0, entry G must be D, "
                  "non-decreasing)", what);
    return fail(ctx, CRDT_ECOMM, "%s: rank %ld passed invalid def_off; no deferred removes were exchanged", what,
                bad_off);
  }
  timing_begin(ctx, "shard_exchange");
  chain = chain && W > 1;
  size_t Dmax = 0, Dtot = 0;
  for (size_t r = 0; r < W; ++r) {
    Dmax = std::max<size_t>(Dmax, all[r * (G + 1) + G]);
    Dtot += all[r * (G + 1) + G];
  }
  // Such a cell makes the join non-associative, so the partials may not be joined as a tree: the
  // ranks fold in rank order instead — rank k continues from rank k-1's state (its shard re-folded
  // with that state as the start), each step published by one more all-gather — and the re-merge
  // below then reads the last rank's state alone (W-1 extra exchanges; exact for any input).
  for (size_t k = 1; chain && k < W; ++k) {
    if ((size_t)ctx->rank == k) {
      ex.init_clock = (const u64 *)gc + (k - 1) * G * A;
      ex.init_entries = (const u64 *)ge + (k - 1) * G * M * A;
      CRDT_TRY(orswot_lub_many_ex(ctx, &loc, &po, ex));
    }
    CRDT_TRY(coll_group_begin(ctx));
    CRDT_TRY(coll_allgather(ctx, pc, gc, G * A * 8));
    CRDT_TRY(coll_allgather(ctx, pe, ge, G * M * A * 8));
    CRDT_TRY(coll_group_end(ctx));
  }
  crdt_orswot_batch fin{};
  fin.G = G;
  fin.R = chain ? 1 : W;
  fin.M = M;
  fin.A = A;
  fin.clock = (const uint64_t *)gc + (chain ? (W - 1) * G * A : 0);
  fin.clock_rstride = G * A;
  fin.clock_gstride = A;
  fin.entries = (const uint64_t *)ge + (chain ? (W - 1) * G * M * A : 0);
  fin.entry_mstride = A;
  fin.entry_rstride = G * M * A;
  fin.entry_gstride = M * A;
  std::vector<size_t> goff(G + 1, 0);
  void *dcl = nullptr, *dmb = nullptr, *keep = nullptr, *kmb = nullptr, *idx = nullptr;
  if (Dtot) {  // rank-uniform: every rank saw the same gathered counts
    // padded send rows: [Dmax][A | Mw]
    void *sendc, *sendm, *allc, *allm;
    CRDT_TRY(sbuf(ctx, 6, Dmax * (A + Mw) * 8, &sendc));
    sendm = (u64 *)sendc + Dmax * A;
    CRDT_TRY(sbuf(ctx, 7, W * Dmax * (A + Mw) * 8 + Dtot * (A + 2 * Mw) * 8 + Dtot + Dtot * 4 + 64, &allc));
    allm = (u64 *)allc + W * Dmax * A;
    dcl = (u64 *)allm + W * Dmax * Mw;  // grouped pool [Dtot][A]
    dmb = (u64 *)dcl + Dtot * A;        // grouped pool [Dtot][Mw]
    kmb = (u64 *)dmb + Dtot * Mw;       // survivors' member unions [Dtot][Mw]
    idx = (u64 *)kmb + Dtot * Mw;       // gather index [Dtot] u32
    keep = (uint32_t *)idx + Dtot;      // [Dtot] u8
    if (Dk) {
      CRDT_HIP(ctx, hipMemcpyAsync(sendc, in->def_clock, Dk * A * 8, hipMemcpyDeviceToDevice, ctx->stream));
      CRDT_HIP(ctx, hipMemcpyAsync(sendm, in->def_members, Dk * Mw * 8, hipMemcpyDeviceToDevice, ctx->stream));
    }
    CRDT_TRY(coll_group_begin(ctx));
    CRDT_TRY(coll_allgather(ctx, sendc, allc, Dmax * A * 8));
    CRDT_TRY(coll_allgather(ctx, sendm, allm, Dmax * Mw * 8));
    CRDT_TRY(coll_group_end(ctx));
    std::vector<uint32_t> gi;
    shard_host::orswot_regroup(all.data(), W, G, Dmax, gi, goff);
    CRDT_TRY(stage_h2d(ctx, idx, gi.data(), Dtot * 4));
    CRDT_TRY(gather_rows(ctx, (u64 *)dcl, (const u64 *)allc, (const uint32_t *)idx, Dtot, A));
    CRDT_TRY(gather_rows(ctx, (u64 *)dmb, (const u64 *)allm, (const uint32_t *)idx, Dtot, Mw));
    fin.def_off = goff.data();
    fin.def_clock = (const uint64_t *)dcl;
    fin.def_members = (const uint64_t *)dmb;
  }
  timing_end(ctx);
  // 3. re-merge of the world partials with every deferred remove (no collective from here on)
  crdt_orswot_out fo{out->clock, out->entries, (uint8_t *)keep, (uint64_t *)kmb};
  CRDT_TRY(crdt_orswot_lub_many(ctx, &fin, &fo));
  // 4. surviving deferred removes, compacted: (rm clock, member union, group)
  size_t nkeep = 0;
  if (Dtot) {
    std::vector<uint8_t> hk(Dtot);
    CRDT_HIP(ctx, hipMemcpyAsync(hk.data(), keep, Dtot, hipMemcpyDeviceToHost, ctx->stream));
    CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<uint32_t> ki;
    std::vector<uint32_t> kg;
    for (size_t g = 0; g < G; ++g)
      for (size_t d = goff[g]; d < goff[g + 1]; ++d)
        if (hk[d]) {
          ki.push_back((uint32_t)d);
          kg.push_back((uint32_t)g);
        }
    nkeep = ki.size();
    const size_t nw = std::min(nkeep, out->def_cap);
    if (nw) {
      if (!out->def_clock || !out->def_members || !out->def_group)
        return fail(ctx, CRDT_EINVAL, "%s: def_cap > 0 without output buffers", what);
      CRDT_TRY(stage_h2d(ctx, idx, ki.data(), nw * 4));
      CRDT_TRY(gather_rows(ctx, (u64 *)out->def_clock, (const u64 *)dcl, (const uint32_t *)idx, nw, A));
      CRDT_TRY(gather_rows(ctx, (u64 *)out->def_members, (const u64 *)kmb, (const uint32_t *)idx, nw, Mw));
      CRDT_TRY(stage_h2d(ctx, out->def_group, kg.data(), nw * 4));
    }
  }
  *out->ndef = nkeep;
  return CRDT_OK;
}

extern "C" {

int crdt_orswot_lub_many_sharded(crdt_ctx *ctx, const crdt_orswot_batch *in, crdt_orswot_sharded_out *out) {
  return orswot_sharded_impl(ctx, in, nullptr, 0, out, "orswot_lub_many_sharded");
}

int crdt_orswot_lub_many_sharded_doff(crdt_ctx *ctx, const crdt_orswot_batch *in, const uint64_t *def_off, size_t D,
                                      crdt_orswot_sharded_out *out) {
  return orswot_sharded_impl(ctx, in, (const u64 *)def_off, D, out, "orswot_lub_many_sharded_doff");
}

int crdt_lub_many_multi_sharded(crdt_ctx *ctx, const crdt_lub_segment *segs, size_t nseg) {
  static const char *what = "lub_many_multi_sharded";
  CRDT_CHECK_CTX(ctx);
  CRDT_TRY(need_comm(ctx));
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  CRDT_TRY(agree_mark(ctx));
  int st = device_mem_only(ctx, what);
  std::vector<LubReq> reqs;
  if (!st) st = lub_reqs_from_segments(ctx, segs, nseg, reqs);
  const bool parsed = reqs.size() == nseg;
  std::vector<LubReq> maxr;
  uint64_t dh = 0x9e3779b97f4a7c15ull;  // hash of every segment's (op, G, W)
  for (auto &q : reqs) {
    if (!st && q.G > 1 && q.out_stride != q.W) st = fail(ctx, CRDT_EINVAL, "%s: out_stride must equal the row width", what);
    if (!st && q.flags) st = fail(ctx, CRDT_EINVAL, "%s: flags must be 0", what);
    if (!st && q.G && q.W && !q.out) st = fail(ctx, CRDT_EINVAL, "%s: a segment's out is NULL", what);
    if (q.op == Op::Max) maxr.push_back(q);
    for (uint64_t d : {(uint64_t)q.op, (uint64_t)q.G, (uint64_t)q.W}) dh = (dh ^ d) * 0x100000001b3ull;
  }
  if (!st) st = lattice_lub_many_multi(ctx, maxr.data(), maxr.size());
  const Hdr hd = make_hdr(st, kTagMulti, {(uint64_t)reqs.size(), dh});
  if (parsed && maxr.size() == reqs.size() && plan_agreed(ctx, hd)) {  // an agreed plan (max segments only)
    CRDT_TRY(check_pending(ctx));
    std::vector<u64 *> bufs;
    if (st != CRDT_OK) {  // (this rank failed its validation: it joins with zero partials of the same sizes)
      size_t tot = 0;
      for (auto &q : maxr) tot += q.G * q.W;
      void *z = nullptr;
      CRDT_TRY(sbuf(ctx, 0, (tot ? tot : 1) * 8, &z));
      CRDT_HIP(ctx, hipMemsetAsync(z, 0, tot * 8, ctx->stream));
      size_t o = 0;
      for (auto &q : maxr) {
        bufs.push_back((u64 *)z + o);
        o += q.G * q.W;
      }
    } else {
      for (auto &q : maxr) bufs.push_back(q.out);
    }
    CRDT_TRY(check_issue(ctx, st, hd));
    timing_begin(ctx, "shard_exchange");
    CRDT_TRY(coll_group_begin(ctx));
    for (size_t i = 0; i < maxr.size(); ++i)
      CRDT_TRY(coll_allreduce(ctx, bufs[i], bufs[i], maxr[i].G * maxr[i].W, Red::Max));
    CRDT_TRY(coll_allreduce(ctx, (const u64 *)ctx->chk_dev, (u64 *)ctx->chk_dev, 3, Red::Max));
    CRDT_TRY(coll_group_end(ctx));
    timing_end(ctx);
    CRDT_TRY(check_finish(ctx, hd));
    return st;
  }
  CRDT_TRY(agree(ctx, st, hd, what));
  timing_begin(ctx, "shard_exchange");
  CRDT_TRY(coll_group_begin(ctx));
  for (auto &q : maxr) CRDT_TRY(coll_allreduce(ctx, q.out, q.out, q.G * q.W, Red::Max));
  CRDT_TRY(coll_group_end(ctx));
  timing_end(ctx);
  for (auto &q : reqs)  // GSet segments: every rank reaches each of them (same segment list)
    if (q.op == Op::Or) CRDT_TRY(lattice_sharded(ctx, q.op, q.in, q.G, q.R, q.W, q.row_stride, q.group_stride, q.out, what));
  return CRDT_OK;
}

int crdt_lwwreg_lub_many_sharded(crdt_ctx *ctx, const uint64_t *marker, const uint64_t *val, size_t G, size_t R,
                                 size_t group_stride, uint64_t base, uint64_t *out_marker, uint64_t *out_val,
                                 uint64_t *first_conflict) {
  static const char *what = "lwwreg_lub_many_sharded";
  CRDT_CHECK_CTX(ctx);
  CRDT_TRY(need_comm(ctx));
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  CRDT_TRY(agree_mark(ctx));
  const size_t W = (size_t)ctx->nranks, row = 2 * G + 1;
  int st = device_mem_only(ctx, what);
  if (!st && G && (!out_marker || !out_val)) st = fail(ctx, CRDT_EINVAL, "%s: NULL output", what);
  if (!st && G && R && (!marker || !val)) st = fail(ctx, CRDT_EINVAL, "%s: NULL input", what);
  void *send = nullptr, *all = nullptr, *tmv = nullptr, *pst = nullptr;
  if (!st && G) {
    st = sbuf(ctx, 0, row * 8, &send);
    if (!st) st = sbuf(ctx, 1, W * row * 8, &all);
    if (!st) st = sbuf(ctx, 2, 2 * G * W * 8, &tmv);
    if (!st) st = sbuf(ctx, 3, 3 * G * 8 + W * 4 + 64, &pst);
  }
  uint64_t *lm = (uint64_t *)send, *lv = lm + G;
  uint64_t *tm = (uint64_t *)tmv, *tv = tm + G * W;
  uint64_t *pm = (uint64_t *)pst, *pv = pm + G, *fc = pv + G;
  uint32_t *ranks = (uint32_t *)(fc + G);
  // 1. local fold of the shard (acc = shard[0]; conflicts indexed locally); R_k travels along
  if (!st && G && R) st = crdt_lwwreg_lub_many(ctx, marker, val, G, R, group_stride, lm, lv, fc, 0);
  const uint64_t rk = R;
  if (!st && G) st = stage_h2d(ctx, lm + 2 * G, &rk, 8);
  CRDT_TRY(agree(ctx, st, make_hdr(st, kTagLww, {G}), what));
  if (G == 0) return CRDT_OK;
  // 2. all-gather the rank states
  timing_begin(ctx, "shard_exchange");
  CRDT_TRY(coll_allgather(ctx, send, all, row * 8));
  timing_end(ctx);
  std::vector<uint64_t> hall(W * row);
  CRDT_HIP(ctx, hipMemcpyAsync(hall.data(), all, hall.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  std::vector<uint32_t> nz;
  const size_t before = shard_host::lww_nonempty(hall.data(), W, row, G, ctx->rank, nz);
  const size_t n = nz.size();
  if (n == 0) {  // no replica anywhere (rank-uniform): the zero register, no conflict
    CRDT_TRY(device_fill(ctx, out_marker, G * 8, 0));
    CRDT_TRY(device_fill(ctx, out_val, G * 8, 0));
    if (first_conflict) CRDT_TRY(device_fill(ctx, first_conflict, G * 8, 0xFF));
    return CRDT_OK;
  }
  CRDT_TRY(stage_h2d(ctx, ranks, nz.data(), n * 4));
  hipLaunchKernelGGL(lww_world_rows_kernel, dim3(small_grid(ctx, G * n)), dim3(kBlock), 0, ctx->stream, (u64 *)tm,
                     (u64 *)tv, (const u64 *)all, (const uint32_t *)ranks, (unsigned long long)n, (unsigned long long)G);
  CRDT_HIP(ctx, hipGetLastError());
  // 3. the shard continues the GLOBAL fold from the fold of the lower ranks' states, so its
  //    conflicts are those of the global left fold (lwwreg.rs:84-98 is order-dependent).  A local
  //    failure here still joins the MIN all-reduce below (with "no conflict") so no rank blocks.
  int st2 = CRDT_OK;
  if (!R) {
    st2 = device_fill(ctx, fc, G * 8, 0xFF);
  } else if (before > 0) {
    st2 = crdt_lwwreg_lub_many(ctx, tm, tv, G, before, n, pm, pv, nullptr, 0);
    if (!st2) st2 = crdt_lwwreg_lub_many(ctx, marker, val, G, R, group_stride, pm, pv, fc, CRDT_ACCUMULATE);
  }
  if (st2) (void)device_fill(ctx, fc, G * 8, 0xFF);
  hipLaunchKernelGGL(lww_rebase_kernel, dim3(small_grid(ctx, G)), dim3(kBlock), 0, ctx->stream, (u64 *)fc,
                     (unsigned long long)G, (u64)base);
  CRDT_HIP(ctx, hipGetLastError());
  CRDT_TRY(coll_allreduce(ctx, (const u64 *)fc, first_conflict ? (u64 *)first_conflict : (u64 *)fc, G, Red::Min));
  if (st2) return st2;
  // 4. the global state: the fold of the world's rank states
  return crdt_lwwreg_lub_many(ctx, tm, tv, G, n, n, out_marker, out_val, nullptr, 0);
}

}  // extern "C"

// doff: device offsets (in->def_off NULL, Ddev the pool length): checked on the device (flags bit
// 1), and their hash travels in the flags row, compared on every rank after that exchange.
static int map_sharded_impl(crdt_ctx *ctx, const crdt_map_batch *in, const u64 *doff, size_t Ddev, size_t k0,
                            size_t K, crdt_map_out *out, const char *what) {
  CRDT_CHECK_CTX(ctx);
  CRDT_TRY(need_comm(ctx));
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  CRDT_TRY(agree_mark(ctx));
  const size_t W = (size_t)ctx->nranks;
  int st = device_mem_only(ctx, what);
  if (!st && (!in || !out)) st = fail(ctx, CRDT_EINVAL, "%s: NULL argument", what);
  if (!st && doff && in->def_off) st = fail(ctx, CRDT_EINVAL, "%s: in->def_off must be NULL", what);
  if (!st && !doff && Ddev) st = fail(ctx, CRDT_EINVAL, "%s: D > 0 without def_off", what);
  const size_t G = st ? 0 : in->G, Kk = st ? 0 : in->K, A = st ? 0 : in->A, R = st ? 0 : in->R;
  if (!st && k0 + Kk > K) st = fail(ctx, CRDT_EINVAL, "%s: key range [%zu, %zu) past K = %zu", what, k0, k0 + Kk, K);
  if (!st && G && A && (!out->clock || !out->flags)) st = fail(ctx, CRDT_EINVAL, "%s: NULL output", what);
  if (!st && in->def_off && G && in->def_off[0] != 0) st = fail(ctx, CRDT_EINVAL, "%s: def_off[0] must be 0", what);
  const size_t D = st ? 0 : doff ? Ddev : (in->def_off && G > 0) ? in->def_off[G] : 0;
  const size_t Kw = (K + 63) / 64, Kwl = Kk ? (Kk + 63) / 64 : 1;
  if (!st && D && (!in->def_keys || !in->def_clock || !in->def_row || !out->def_keys || !out->def_keep))
    st = fail(ctx, CRDT_EINVAL, "%s: deferred buffers missing", what);
  if (!st && D > 0xffffffffULL) st = fail(ctx, CRDT_EUNSUPPORTED, "%s: too many deferred removes", what);
  const bool work = G > 0 && A > 0;
  // the flags row per rank: [G flags | status | offsets hash (device offsets; 0 otherwise)]
  const size_t frow = G + 2;
  void *lk = nullptr, *ok = nullptr, *fl = nullptr, *fall = nullptr;
  if (!st && work) {
    st = sbuf(ctx, 2, frow * 8, &fl);
    if (!st) st = sbuf(ctx, 3, W * frow * 8, &fall);
    if (!st && D) st = sbuf(ctx, 0, D * Kwl * 8, &lk);
    if (!st && D) st = sbuf(ctx, 1, D * Kwl * 8, &ok);
  }
  crdt_map_batch loc{};
  crdt_map_out lo{};
  void *dchk = nullptr;
  // the rank's part: its keys' exact left fold (keys are independent given the clocks and the
  // deferred list: no data-path collective), or with no keys the clock lub and the
  // removes' survival alone (def_keep is a function of the clocks and the deferred list)
  auto local = [&](size_t vstate) -> int {
    if (Kk > 0) {
      lo.Vstate = vstate;
      return doff ? crdt_map_lub_many_doff(ctx, &loc, (const uint64_t *)doff, D, &lo) : crdt_map_lub_many(ctx, &loc, &lo);
    }
    if (int rc = device_fill(ctx, out->flags, G * 4, 0)) return rc;
    if (doff) {  // the offsets' check alone (flags bit 1), as the fold would make it
      if (int rc = sbuf(ctx, 4, (G + 1) * 8, &dchk)) return rc;
      if (int rc = stage_def_off_dev(ctx, doff, (size_t *)dchk, G, D, nullptr, out->flags)) return rc;
    }
    if (int rc = lattice_lub_many(ctx, Op::Max, (const u64 *)in->clock, G, R, A, in->clock_rstride,
                                  in->clock_gstride, (u64 *)out->clock, A, 0))
      return rc;
    if (!D) return CRDT_OK;
    DefPlan q{};
    q.G = G;
    q.D = D;
    q.M = 64;
    q.A = A;
    q.Mw = 1;
    q.def_clock = (const u64 *)in->def_clock;
    q.def_members = (const u64 *)lk;  // all-zero: no key of this rank
    q.out_clock = (const u64 *)out->clock;
    q.apply_ceiling = 0;
    q.out_keep = out->def_keep;
    q.out_members = (u64 *)ok;
    return launch_deferred(ctx, in->def_off, q, doff);
  };
  if (!st && work) {
    loc = *in;
    lo = *out;
    if (D) {  // the key bitmaps restricted to this rank's keys [k0, k0 + Kk), re-indexed from 0
      hipLaunchKernelGGL(bitmap_shift_kernel, dim3(small_grid(ctx, D * Kwl)), dim3(kBlock), 0, ctx->stream, (u64 *)lk,
                         (const u64 *)in->def_keys, (unsigned long long)D, (unsigned long long)Kwl,
                         (unsigned long long)Kw, (long long)k0, (long long)(k0 + Kk));
      if (hipGetLastError() != hipSuccess) st = fail(ctx, CRDT_EHIP, "%s: bitmap_shift_kernel launch", what);
      loc.def_keys = (const uint64_t *)lk;
      lo.def_keys = (uint64_t *)ok;
    }
    if (!st) st = local(std::min<size_t>(out->Vstate, 16));
  }
  const uint64_t offh = (!st && in->def_off && G) ? shard_host::hash_offsets(in->def_off, G + 1) : 0;
  // the retry below branches on vstate: its start is part of the agreed call, so ranks
  // passing different Vstate values all return EINVAL instead of meeting in different collectives
  const size_t vst0 = st ? 0 : std::min<size_t>(out->Vstate, 16);
  CRDT_TRY(agree(ctx, st, make_hdr(st, kTagMap, {G, K, A, D, st ? 0 : (uint64_t)out->Vout, offh, vst0}), what));
  if (!work) return CRDT_OK;
  // flags of every rank (+ its status) -> the OR over the ranks, written back on every rank; a
  // fold state that ran out of value slots (bit 2) on ANY rank reruns the fold with a larger state
  // on EVERY rank (each key's result is independent of the state size), so the ranks take the same
  // branches and meet in the same collectives
  size_t vstate = vst0;
  std::vector<uint64_t> hf(W * frow);
  std::vector<uint32_t> gflags(G);
  for (;;) {
    hipLaunchKernelGGL(widen_u32_kernel, dim3(small_grid(ctx, G + 1)), dim3(kBlock), 0, ctx->stream, (u64 *)fl,
                       (const uint32_t *)out->flags, (unsigned long long)G, (u64)(st ? 1 : 0));
    CRDT_HIP(ctx, hipGetLastError());
    CRDT_TRY(device_fill(ctx, (u64 *)fl + G + 1, 8, 0));
    if (doff) {
      hipLaunchKernelGGL(def_hash_kernel, dim3(small_grid(ctx, G + 1)), dim3(kBlock), 0, ctx->stream, doff,
                         (unsigned long long)(G + 1), (u64 *)fl + G + 1);
      CRDT_HIP(ctx, hipGetLastError());
    }
    CRDT_TRY(coll_allgather(ctx, fl, fall, frow * 8));
    CRDT_HIP(ctx, hipMemcpyAsync(hf.data(), fall, hf.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    bool bad, grow;
    shard_host::map_flags_or(hf.data(), W, G, gflags.data(), &bad, &grow, frow);
    if (bad) {
      if (st) return st;
      return fail(ctx, CRDT_ECOMM, "%s: another rank failed its local fold; no key sets were exchanged", what);
    }
    for (size_t r = 1; r < W; ++r)
      if (hf[r * frow + G + 1] != hf[G + 1])
        return fail(ctx, CRDT_EINVAL, "%s: the ranks hold different deferred offsets (device offsets' hash "
                    "differs between rank 0 and rank %zu); no key sets were exchanged", what, r);

    if (!grow || vstate >= 16) break;
    vstate = vstate < 8 ? 8 : 16;
    st = Kk > 0 ? local(vstate) : CRDT_OK;
  }
  CRDT_TRY(stage_h2d(ctx, out->flags, gflags.data(), G * 4));
  if (!D) return CRDT_OK;
  // surviving removes' key sets over all K keys: this rank's bits placed at k0, then a SUM
  // all-reduce (disjoint key ranges: the sum is the union)
  hipLaunchKernelGGL(bitmap_shift_kernel, dim3(small_grid(ctx, D * Kw)), dim3(kBlock), 0, ctx->stream,
                     (u64 *)out->def_keys, (const u64 *)ok, (unsigned long long)D, (unsigned long long)Kw,
                     (unsigned long long)Kwl, -(long long)k0, (long long)Kk);
  CRDT_HIP(ctx, hipGetLastError());
  timing_begin(ctx, "shard_exchange");
  CRDT_TRY(coll_allreduce(ctx, (const u64 *)out->def_keys, (u64 *)out->def_keys, D * Kw, Red::Sum));
  timing_end(ctx);
  return CRDT_OK;
}

// ---- the value-typed Maps sharded by KEYS (round 5): Map<K, GCounter / PNCounter>, Map<K, Orswot>,
// Map<K, Map<K2, MVReg>>.  As map_sharded_impl: rank k holds keys [k0, k0 + Kk) of every replica,
// every replica's clock and the group's whole deferred list with key bitmaps over all K keys; its
// fold of its keys is the exact left fold (keys are independent given the clocks and the deferred
// list), the flags are ORed over the ranks and the surviving removes' key sets assembled by one
// SUM all-reduce (disjoint key ranges).  `fold(loc_def_keys, loc_out_def_keys)` runs the local
// fold of the rank's keys with the key bitmaps restricted to them (Kw of Kk words).
struct VMapShard {
  size_t G, R, A, Kk, k0, K;
  const size_t *def_off;  // host, G+1 (NULL: no deferred removes)
  const uint32_t *def_row;
  const uint64_t *def_clock, *def_keys;  // def_keys [D][ceil(K/64)]
  const uint64_t *clock;
  size_t c_rs, c_gs;
  uint64_t *out_clock;
  uint32_t *out_flags;
  uint8_t *out_def_keep;
  uint64_t *out_def_keys;  // [D][ceil(K/64)]
};

template <class Fold>
static int vmap_sharded_impl(crdt_ctx *ctx, int st0, const VMapShard &v, uint64_t tag, uint64_t dimx, Fold &&fold,
                             const char *what) {
  CRDT_CHECK_CTX(ctx);
  CRDT_TRY(need_comm(ctx));
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  CRDT_TRY(agree_mark(ctx));
  const size_t W = (size_t)ctx->nranks;
  int st = device_mem_only(ctx, what);
  if (!st) st = st0;
  const size_t G = st ? 0 : v.G, Kk = st ? 0 : v.Kk, A = st ? 0 : v.A, R = st ? 0 : v.R, K = st ? 0 : v.K;
  const size_t k0 = st ? 0 : v.k0;
  if (!st && k0 + Kk > K) st = fail(ctx, CRDT_EINVAL, "%s: key range [%zu, %zu) past K = %zu", what, k0, k0 + Kk, K);
  if (!st && G && A && (!v.out_clock || !v.out_flags)) st = fail(ctx, CRDT_EINVAL, "%s: NULL output", what);
  if (!st && v.def_off && G && v.def_off[0] != 0) st = fail(ctx, CRDT_EINVAL, "%s: def_off[0] must be 0", what);
  const size_t D = (st || !v.def_off || G == 0) ? 0 : v.def_off[G];
  const size_t Kw = (K + 63) / 64, Kwl = Kk ? (Kk + 63) / 64 : 1;
  if (!st && D && (!v.def_keys || !v.def_clock || !v.def_row || !v.out_def_keys || !v.out_def_keep))
    st = fail(ctx, CRDT_EINVAL, "%s: deferred buffers missing", what);
  if (!st && D > 0xffffffffULL) st = fail(ctx, CRDT_EUNSUPPORTED, "%s: too many deferred removes", what);
  const bool work = !st && G > 0 && A > 0;
  const size_t frow = G + 2;  // [G flags | status | 0]
  void *lk = nullptr, *ok = nullptr, *fl = nullptr, *fall = nullptr;
  if (work) {
    st = sbuf(ctx, 2, frow * 8, &fl);
    if (!st) st = sbuf(ctx, 3, W * frow * 8, &fall);
    if (!st && D) st = sbuf(ctx, 0, D * Kwl * 8, &lk);
    if (!st && D) st = sbuf(ctx, 1, D * Kwl * 8, &ok);
  }
  if (!st && work) {
    if (D) {  // the key bitmaps restricted to this rank's keys [k0, k0 + Kk), re-indexed from 0
      hipLaunchKernelGGL(bitmap_shift_kernel, dim3(small_grid(ctx, D * Kwl)), dim3(kBlock), 0, ctx->stream, (u64 *)lk,
                         (const u64 *)v.def_keys, (unsigned long long)D, (unsigned long long)Kwl,
                         (unsigned long long)Kw, (long long)k0, (long long)(k0 + Kk));
      if (hipGetLastError() != hipSuccess) st = fail(ctx, CRDT_EHIP, "%s: bitmap_shift_kernel launch", what);
    }
    if (!st && Kk > 0) {
      st = fold((const uint64_t *)lk, (uint64_t *)ok);
    } else if (!st) {  // no keys here: the clock lub and the removes' survival alone
      st = device_fill(ctx, v.out_flags, G * 4, 0);
      if (!st) st = lattice_lub_many(ctx, Op::Max, (const u64 *)v.clock, G, R, A, v.c_rs, v.c_gs, (u64 *)v.out_clock, A, 0);
      if (!st && D) {
        DefPlan q{};
        q.G = G;
        q.D = D;
        q.M = 64;
        q.A = A;
        q.Mw = 1;
        q.def_clock = (const u64 *)v.def_clock;
        q.def_members = (const u64 *)lk;  // all-zero: no key of this rank
        q.out_clock = (const u64 *)v.out_clock;
        q.apply_ceiling = 0;
        q.out_keep = v.out_def_keep;
        q.out_members = (u64 *)ok;
        st = launch_deferred(ctx, v.def_off, q, nullptr);
      }
    }
  }
  const uint64_t offh = (!st && v.def_off && G) ? shard_host::hash_offsets(v.def_off, G + 1) : 0;
  CRDT_TRY(agree(ctx, st, make_hdr(st, tag, {G, K, A, D, dimx, offh}), what));
  if (!work) return st;
  hipLaunchKernelGGL(widen_u32_kernel, dim3(small_grid(ctx, G + 1)), dim3(kBlock), 0, ctx->stream, (u64 *)fl,
                     (const uint32_t *)v.out_flags, (unsigned long long)G, (u64)(st ? 1 : 0));
  CRDT_HIP(ctx, hipGetLastError());
  CRDT_TRY(device_fill(ctx, (u64 *)fl + G + 1, 8, 0));
  CRDT_TRY(coll_allgather(ctx, fl, fall, frow * 8));
  std::vector<uint64_t> hf(W * frow);
  std::vector<uint32_t> gflags(G);
  CRDT_HIP(ctx, hipMemcpyAsync(hf.data(), fall, hf.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  bool bad, grow;
  shard_host::map_flags_or(hf.data(), W, G, gflags.data(), &bad, &grow, frow);
  if (bad) {
    if (st) return st;
    return fail(ctx, CRDT_ECOMM, "%s: another rank failed its local fold; no key sets were exchanged", what);
  }
  CRDT_TRY(stage_h2d(ctx, v.out_flags, gflags.data(), G * 4));
  if (!D) return CRDT_OK;
  hipLaunchKernelGGL(bitmap_shift_kernel, dim3(small_grid(ctx, D * Kw)), dim3(kBlock), 0, ctx->stream,
                     (u64 *)v.out_def_keys, (const u64 *)ok, (unsigned long long)D, (unsigned long long)Kw,
                     (unsigned long long)Kwl, -(long long)k0, (long long)Kk);
  CRDT_HIP(ctx, hipGetLastError());
  timing_begin(ctx, "shard_exchange");
  CRDT_TRY(coll_allreduce(ctx, (const u64 *)v.out_def_keys, (u64 *)v.out_def_keys, D * Kw, Red::Sum));
  timing_end(ctx);
  return CRDT_OK;
}

extern "C" {

int crdt_map_counter_lub_many_sharded(crdt_ctx *ctx, const crdt_map_counter_batch *in, size_t k0, size_t K,
                                      crdt_map_counter_out *out) {
  const int st0 = (!in || !out) ? fail(ctx, CRDT_EINVAL, "map_counter_lub_many_sharded: NULL argument") : CRDT_OK;
  VMapShard v{};
  if (!st0) v = VMapShard{in->G, in->R, in->A, in->K, k0, K, in->def_off, in->def_row, in->def_clock, in->def_keys,
                          in->clock, in->clock_rstride, in->clock_gstride, out->clock, out->flags, out->def_keep,
                          out->def_keys};
  return vmap_sharded_impl(ctx, st0, v, kTagMapCounter, st0 ? 0 : in->W, [&](const uint64_t *lk, uint64_t *ok) {
    crdt_map_counter_batch loc = *in;
    crdt_map_counter_out lo = *out;
    if (lk) loc.def_keys = lk, lo.def_keys = ok;
    return crdt_map_counter_lub_many(ctx, &loc, &lo);
  }, "map_counter_lub_many_sharded");
}

int crdt_map_orswot_lub_many_sharded(crdt_ctx *ctx, const crdt_map_orswot_batch *in, size_t k0, size_t K,
                                     crdt_map_orswot_out *out) {
  const int st0 = (!in || !out) ? fail(ctx, CRDT_EINVAL, "map_orswot_lub_many_sharded: NULL argument") : CRDT_OK;
  VMapShard v{};
  if (!st0) v = VMapShard{in->G, in->R, in->A, in->K, k0, K, in->def_off, in->def_row, in->def_clock, in->def_keys,
                          in->clock, in->A, in->R * in->A, out->clock, out->flags, out->def_keep, out->def_keys};
  return vmap_sharded_impl(ctx, st0, v, kTagMapOrswot, st0 ? 0 : in->M, [&](const uint64_t *lk, uint64_t *ok) {
    crdt_map_orswot_batch loc = *in;
    crdt_map_orswot_out lo = *out;
    if (lk) loc.def_keys = lk, lo.def_keys = ok;
    return crdt_map_orswot_lub_many(ctx, &loc, &lo);
  }, "map_orswot_lub_many_sharded");
}

int crdt_map_nested_lub_many_sharded(crdt_ctx *ctx, const crdt_map_nested_batch *in, size_t k0, size_t K,
                                     crdt_map_nested_out *out) {
  const int st0 = (!in || !out) ? fail(ctx, CRDT_EINVAL, "map_nested_lub_many_sharded: NULL argument") : CRDT_OK;
  VMapShard v{};
  if (!st0) v = VMapShard{in->G, in->R, in->A, in->K, k0, K, in->def_off, in->def_row, in->def_clock, in->def_keys,
                          in->clock, in->A, in->R * in->A, out->clock, out->flags, out->def_keep, out->def_keys};
  return vmap_sharded_impl(ctx, st0, v, kTagMapNested, st0 ? 0 : (in->K2 << 8 | in->V),
                           [&](const uint64_t *lk, uint64_t *ok) {
    crdt_map_nested_batch loc = *in;
    crdt_map_nested_out lo = *out;
    if (lk) loc.def_keys = lk, lo.def_keys = ok;
    return crdt_map_nested_lub_many(ctx, &loc, &lo);
  }, "map_nested_lub_many_sharded");
}

int crdt_map_lub_many_sharded(crdt_ctx *ctx, const crdt_map_batch *in, size_t k0, size_t K, crdt_map_out *out) {
  return map_sharded_impl(ctx, in, nullptr, 0, k0, K, out, "map_lub_many_sharded");
}

int crdt_map_lub_many_sharded_doff(crdt_ctx *ctx, const crdt_map_batch *in, const uint64_t *def_off, size_t D,
                                   size_t k0, size_t K, crdt_map_out *out) {
  return map_sharded_impl(ctx, in, (const u64 *)def_off, D, k0, K, out, "map_lub_many_sharded_doff");
}

}  // extern "C"
