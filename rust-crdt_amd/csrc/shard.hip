// Replica-sharded lub across the GPUs of a node through the C ABI: one process
// (one crdt_ctx) per GPU, joined into an RCCL communicator by a unique id the caller distributes
// (a Rust caller over its own transport; the Python host over torch.distributed).
//
//   VClock / GCounter / PNCounter: local lub of the rank's replica shard, then ONE in-place
//       ncclAllReduce(ncclUint64, ncclMax) of the G x W partials over xGMI: max is the join.
//   GSet: local lub, ncclAllGather of the partial bitmaps, OR-fold of the world partials by the
//       same lattice kernel (RCCL has no bitwise-OR reduction).
//   Orswot: each rank joins its shard WITHOUT deferred removes (the dot-store join is associative
//       under the reference invariants), the partial (clock, entries) are all-gathered and every
//       rank re-merges the world partials together with ALL ranks' deferred removes (the forget
//       ceiling and the survival test need the global clock: orswot.rs:141-147, :240-249).
// Every rank ends with the same global result.  Multi-GPU tests without several GPUs: the
// Python host path (crdts_gpu/dist.py) runs the same exchange under gloo on CPU; this file is
// exercised at world size 1 on one MI355X (tests/test_gpu_shard_abi.py).
#include <rccl/rccl.h>

#include <algorithm>

#include "common.hpp"

namespace crdt {

static_assert(CRDT_UNIQUE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

static int nccl_fail(crdt_ctx *ctx, ncclResult_t r, const char *what) {
  return fail(ctx, CRDT_ECOMM, "%s: %s", what, ncclGetErrorString(r));
}

#define CRDT_NCCL(ctx, expr)                                   \
  do {                                                         \
    ncclResult_t _r = (expr);                                  \
    if (_r != ncclSuccess) return crdt::nccl_fail((ctx), _r, #expr); \
  } while (0)

static void destroy_comm(void *c) { (void)ncclCommDestroy((ncclComm_t)c); }

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

#define CRDT_TRY(expr)             \
  do {                             \
    int _s = (expr);               \
    if (_s != CRDT_OK) return _s;  \
  } while (0)

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

static int need_comm(crdt_ctx *ctx) {
  if (!ctx->comm) return fail(ctx, CRDT_EINVAL, "sharded call without crdt_ctx_comm_init");
  return CRDT_OK;
}

static int lattice_sharded(crdt_ctx *ctx, Op op, const u64 *in, size_t G, size_t R, size_t W, size_t row_stride,
                           size_t group_stride, u64 *out) {
  CRDT_CHECK_CTX(ctx);
  CRDT_TRY(need_comm(ctx));
  if (G == 0 || W == 0) return CRDT_OK;
  if (!out) return fail(ctx, CRDT_EINVAL, "lub_many_sharded: out is NULL");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  auto comm = (ncclComm_t)ctx->comm;
  const size_t n = G * W;
  if (op == Op::Max) {
    CRDT_TRY(lattice_lub_many(ctx, op, in, G, R, W, row_stride, group_stride, out, W, 0));
    timing_begin(ctx, "shard_exchange");
    CRDT_NCCL(ctx, ncclAllReduce(out, out, n, ncclUint64, ncclMax, comm, ctx->stream));
    timing_end(ctx);
    return CRDT_OK;
  }
  // GSet: partial -> all-gather [nranks][G][W] -> OR over the nranks "replicas" of each group
  void *part = nullptr, *all = nullptr;
  CRDT_TRY(sbuf(ctx, 0, n * 8, &part));
  CRDT_TRY(sbuf(ctx, 1, n * 8 * ctx->nranks, &all));
  CRDT_TRY(lattice_lub_many(ctx, op, in, G, R, W, row_stride, group_stride, (u64 *)part, W, 0));
  timing_begin(ctx, "shard_exchange");
  CRDT_NCCL(ctx, ncclAllGather(part, all, n, ncclUint64, comm, ctx->stream));
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

}  // namespace crdt

using namespace crdt;

extern "C" {

int crdt_comm_unique_id(uint8_t *id) {
  if (!id) return CRDT_EINVAL;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return CRDT_ECOMM;
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return CRDT_OK;
}

int crdt_ctx_comm_init(crdt_ctx *ctx, const uint8_t *id, int nranks, int rank) {
  CRDT_CHECK_CTX(ctx);
  if (!id || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(ctx, CRDT_EINVAL, "crdt_ctx_comm_init: bad id / nranks %d / rank %d", nranks, rank);
  if (ctx->comm) return fail(ctx, CRDT_EINVAL, "crdt_ctx_comm_init: ctx already has a communicator");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  ncclUniqueId u;
  std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  CRDT_NCCL(ctx, ncclCommInitRank(&c, nranks, u, rank));
  ctx->comm = c;
  ctx->nranks = nranks;
  ctx->rank = rank;
  ctx->comm_destroy = destroy_comm;
  return CRDT_OK;
}

int crdt_ctx_comm_destroy(crdt_ctx *ctx) {
  CRDT_CHECK_CTX(ctx);
  if (ctx->comm) {
    (void)hipStreamSynchronize(ctx->stream);
    CRDT_NCCL(ctx, ncclCommDestroy((ncclComm_t)ctx->comm));
  }
  ctx->comm = nullptr;
  ctx->nranks = 1;
  ctx->rank = 0;
  return CRDT_OK;
}

int crdt_ctx_comm_info(const crdt_ctx *ctx, int *nranks, int *rank) {
  if (!ctx) return CRDT_EINVAL;
  if (nranks) *nranks = ctx->comm ? ctx->nranks : 0;
  if (rank) *rank = ctx->comm ? ctx->rank : -1;
  return CRDT_OK;
}

int crdt_vclock_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A, size_t row_stride,
                                 size_t group_stride, uint64_t *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return lattice_sharded(ctx, Op::Max, (const u64 *)in, G, R, A, row_stride, group_stride, (u64 *)out);
}
int crdt_gcounter_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                                   size_t row_stride, size_t group_stride, uint64_t *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return lattice_sharded(ctx, Op::Max, (const u64 *)in, G, R, A, row_stride, group_stride, (u64 *)out);
}
int crdt_pncounter_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                                    size_t row_stride, size_t group_stride, uint64_t *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return lattice_sharded(ctx, Op::Max, (const u64 *)in, G, R, 2 * A, row_stride, group_stride, (u64 *)out);
}
int crdt_gset_lub_many_sharded(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t words,
                               size_t row_stride, size_t group_stride, uint64_t *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return lattice_sharded(ctx, Op::Or, (const u64 *)in, G, R, words, row_stride, group_stride, (u64 *)out);
}

int crdt_orswot_lub_many_sharded(crdt_ctx *ctx, const crdt_orswot_batch *in, crdt_orswot_sharded_out *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  CRDT_TRY(need_comm(ctx));
  if (!in || !out || !out->clock || !out->entries || !out->ndef)
    return fail(ctx, CRDT_EINVAL, "orswot_lub_many_sharded: NULL argument");
  const size_t G = in->G, M = in->M, A = in->A, Mw = (M + 63) / 64;
  const size_t W = (size_t)ctx->nranks;
  if (G == 0 || A == 0) {
    *out->ndef = 0;
    return CRDT_OK;
  }
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  auto comm = (ncclComm_t)ctx->comm;
  // 1. local join of the shard without deferred removes -> partial (clock, entries)
  void *pc, *pe, *gc, *ge;
  CRDT_TRY(sbuf(ctx, 0, G * A * 8, &pc));
  CRDT_TRY(sbuf(ctx, 1, G * M * A * 8, &pe));
  CRDT_TRY(sbuf(ctx, 2, W * G * A * 8, &gc));
  CRDT_TRY(sbuf(ctx, 3, W * G * M * A * 8, &ge));
  crdt_orswot_batch loc = *in;
  loc.def_off = nullptr;
  crdt_orswot_out po{(uint64_t *)pc, (uint64_t *)pe, nullptr, nullptr};
  CRDT_TRY(crdt_orswot_lub_many(ctx, &loc, &po));
  // 2. all-gather the partials: replica (g, r) of the re-merge at r*G*A + g*A (+ m*A)
  timing_begin(ctx, "shard_exchange");
  CRDT_NCCL(ctx, ncclGroupStart());
  CRDT_NCCL(ctx, ncclAllGather(pc, gc, G * A, ncclUint64, comm, ctx->stream));
  CRDT_NCCL(ctx, ncclAllGather(pe, ge, G * M * A, ncclUint64, comm, ctx->stream));
  CRDT_NCCL(ctx, ncclGroupEnd());
  // 3. deferred removes: per-group counts of every rank, then the padded rows
  std::vector<uint64_t> cnt(G, 0);
  size_t Dk = 0;
  if (in->def_off) {
    for (size_t g = 0; g < G; ++g) {
      if (in->def_off[g + 1] < in->def_off[g])
        return fail(ctx, CRDT_EINVAL, "orswot_lub_many_sharded: def_off not non-decreasing");
      cnt[g] = in->def_off[g + 1] - in->def_off[g];
    }
    Dk = in->def_off[G] - in->def_off[0];
    if (Dk && (!in->def_clock || !in->def_members))
      return fail(ctx, CRDT_EINVAL, "orswot_lub_many_sharded: deferred removes without their buffers");
  }
  void *lcnt, *acnt;
  CRDT_TRY(sbuf(ctx, 4, (G + 1) * 8, &lcnt));
  CRDT_TRY(sbuf(ctx, 5, W * (G + 1) * 8, &acnt));
  std::vector<uint64_t> head(G + 1);
  for (size_t g = 0; g < G; ++g) head[g] = cnt[g];
  head[G] = Dk;
  CRDT_TRY(stage_h2d(ctx, lcnt, head.data(), (G + 1) * 8));
  CRDT_NCCL(ctx, ncclAllGather(lcnt, acnt, G + 1, ncclUint64, comm, ctx->stream));
  std::vector<uint64_t> all((G + 1) * W);
  CRDT_HIP(ctx, hipMemcpyAsync(all.data(), acnt, all.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  size_t Dmax = 0, Dtot = 0;
  for (size_t r = 0; r < W; ++r) {
    Dmax = std::max<size_t>(Dmax, all[r * (G + 1) + G]);
    Dtot += all[r * (G + 1) + G];
  }
  crdt_orswot_batch fin{};
  fin.G = G;
  fin.R = W;
  fin.M = M;
  fin.A = A;
  fin.clock = (const uint64_t *)gc;
  fin.clock_rstride = G * A;
  fin.clock_gstride = A;
  fin.entries = (const uint64_t *)ge;
  fin.entry_mstride = A;
  fin.entry_rstride = G * M * A;
  fin.entry_gstride = M * A;
  std::vector<size_t> goff(G + 1, 0);
  void *dcl = nullptr, *dmb = nullptr, *keep = nullptr, *kmb = nullptr, *idx = nullptr;
  if (Dtot) {
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
      const size_t d0 = in->def_off[0];
      CRDT_HIP(ctx, hipMemcpyAsync(sendc, in->def_clock + d0 * A, Dk * A * 8, hipMemcpyDeviceToDevice, ctx->stream));
      CRDT_HIP(ctx, hipMemcpyAsync(sendm, in->def_members + d0 * Mw, Dk * Mw * 8, hipMemcpyDeviceToDevice,
                                   ctx->stream));
    }
    CRDT_NCCL(ctx, ncclGroupStart());
    CRDT_NCCL(ctx, ncclAllGather(sendc, allc, Dmax * A, ncclUint64, comm, ctx->stream));
    CRDT_NCCL(ctx, ncclAllGather(sendm, allm, Dmax * Mw, ncclUint64, comm, ctx->stream));
    CRDT_NCCL(ctx, ncclGroupEnd());
    // regroup: group g gathers rank 0's rows of g, then rank 1's, ... (rank order, local order)
    std::vector<uint32_t> gi;
    gi.reserve(Dtot);
    std::vector<uint64_t> base(W, 0);
    for (size_t g = 0; g < G; ++g) {
      for (size_t r = 0; r < W; ++r) {
        const uint64_t c = all[r * (G + 1) + g];
        for (uint64_t j = 0; j < c; ++j) gi.push_back((uint32_t)(r * Dmax + base[r] + j));
        base[r] += c;
      }
      goff[g + 1] = gi.size();
    }
    CRDT_TRY(stage_h2d(ctx, idx, gi.data(), Dtot * 4));
    CRDT_TRY(gather_rows(ctx, (u64 *)dcl, (const u64 *)allc, (const uint32_t *)idx, Dtot, A));
    CRDT_TRY(gather_rows(ctx, (u64 *)dmb, (const u64 *)allm, (const uint32_t *)idx, Dtot, Mw));
    fin.def_off = goff.data();
    fin.def_clock = (const uint64_t *)dcl;
    fin.def_members = (const uint64_t *)dmb;
  }
  timing_end(ctx);
  // 4. re-merge of the world partials with every deferred remove
  crdt_orswot_out fo{out->clock, out->entries, (uint8_t *)keep, (uint64_t *)kmb};
  CRDT_TRY(crdt_orswot_lub_many(ctx, &fin, &fo));
  // 5. surviving deferred removes, compacted: (rm clock, member union, group)
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
        return fail(ctx, CRDT_EINVAL, "orswot_lub_many_sharded: def_cap > 0 without output buffers");
      CRDT_TRY(stage_h2d(ctx, idx, ki.data(), nw * 4));
      CRDT_TRY(gather_rows(ctx, (u64 *)out->def_clock, (const u64 *)dcl, (const uint32_t *)idx, nw, A));
      CRDT_TRY(gather_rows(ctx, (u64 *)out->def_members, (const u64 *)kmb, (const uint32_t *)idx, nw, Mw));
      CRDT_TRY(stage_h2d(ctx, out->def_group, kg.data(), nw * 4));
    }
  }
  *out->ndef = nkeep;
  return CRDT_OK;
}

int crdt_lub_many_multi_sharded(crdt_ctx *ctx, const crdt_lub_segment *segs, size_t nseg) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  CRDT_TRY(need_comm(ctx));
  std::vector<LubReq> reqs;
  CRDT_TRY(lub_reqs_from_segments(ctx, segs, nseg, reqs));
  std::vector<LubReq> maxr;
  for (auto &q : reqs) {
    if (q.G > 1 && q.out_stride != q.W)
      return fail(ctx, CRDT_EINVAL, "lub_many_multi_sharded: out_stride must equal the row width");
    if (q.flags) return fail(ctx, CRDT_EINVAL, "lub_many_multi_sharded: flags must be 0");
    if (q.op == Op::Max) maxr.push_back(q);
  }
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  CRDT_TRY(lattice_lub_many_multi(ctx, maxr.data(), maxr.size()));
  auto comm = (ncclComm_t)ctx->comm;
  timing_begin(ctx, "shard_exchange");
  CRDT_NCCL(ctx, ncclGroupStart());
  for (auto &q : maxr)
    if (q.G && q.W) CRDT_NCCL(ctx, ncclAllReduce(q.out, q.out, q.G * q.W, ncclUint64, ncclMax, comm, ctx->stream));
  CRDT_NCCL(ctx, ncclGroupEnd());
  timing_end(ctx);
  for (auto &q : reqs)
    if (q.op == Op::Or) CRDT_TRY(lattice_sharded(ctx, q.op, q.in, q.G, q.R, q.W, q.row_stride, q.group_stride, q.out));
  return CRDT_OK;
}

int crdt_lwwreg_lub_many_sharded(crdt_ctx *ctx, const uint64_t *marker, const uint64_t *val, size_t G, size_t R,
                                 size_t group_stride, uint64_t base, uint64_t *out_marker, uint64_t *out_val,
                                 uint64_t *first_conflict) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  CRDT_TRY(need_comm(ctx));
  if (G == 0) return CRDT_OK;
  if (!out_marker || !out_val) return fail(ctx, CRDT_EINVAL, "lwwreg_lub_many_sharded: NULL output");
  if (R && (!marker || !val)) return fail(ctx, CRDT_EINVAL, "lwwreg_lub_many_sharded: NULL input");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  auto comm = (ncclComm_t)ctx->comm;
  const size_t W = (size_t)ctx->nranks, row = 2 * G + 1;
  void *send, *all, *tmv, *pst;
  CRDT_TRY(sbuf(ctx, 0, row * 8, &send));
  CRDT_TRY(sbuf(ctx, 1, W * row * 8, &all));
  CRDT_TRY(sbuf(ctx, 2, 2 * G * W * 8, &tmv));
  CRDT_TRY(sbuf(ctx, 3, 3 * G * 8 + W * 4 + 64, &pst));
  uint64_t *lm = (uint64_t *)send, *lv = lm + G;
  uint64_t *tm = (uint64_t *)tmv, *tv = tm + G * W;
  uint64_t *pm = (uint64_t *)pst, *pv = pm + G, *fc = pv + G;
  uint32_t *ranks = (uint32_t *)(fc + G);
  // 1. local fold of the shard (acc = shard[0]; conflicts indexed locally); R_k travels along
  if (R) CRDT_TRY(crdt_lwwreg_lub_many(ctx, marker, val, G, R, group_stride, lm, lv, fc, 0));
  const uint64_t rk = R;
  CRDT_TRY(stage_h2d(ctx, lm + 2 * G, &rk, 8));
  // 2. all-gather the rank states
  timing_begin(ctx, "shard_exchange");
  CRDT_NCCL(ctx, ncclAllGather(send, all, row, ncclUint64, comm, ctx->stream));
  timing_end(ctx);
  std::vector<uint64_t> counts(W);
  for (size_t r = 0; r < W; ++r)
    CRDT_HIP(ctx, hipMemcpyAsync(&counts[r], (u64 *)all + r * row + 2 * G, 8, hipMemcpyDeviceToHost, ctx->stream));
  CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
  std::vector<uint32_t> nz;
  size_t before = 0;  // non-empty ranks before this one
  for (size_t r = 0; r < W; ++r)
    if (counts[r]) {
      if ((int)r < ctx->rank) ++before;
      nz.push_back((uint32_t)r);
    }
  const size_t n = nz.size();
  if (n == 0) {  // no replica anywhere: the zero register, no conflict
    CRDT_TRY(device_fill(ctx, out_marker, G * 8, 0));
    CRDT_TRY(device_fill(ctx, out_val, G * 8, 0));
    if (first_conflict) CRDT_TRY(device_fill(ctx, first_conflict, G * 8, 0xFF));
    return CRDT_OK;
  }
  CRDT_TRY(stage_h2d(ctx, ranks, nz.data(), n * 4));
  hipLaunchKernelGGL(lww_world_rows_kernel, dim3(small_grid(ctx, G * n)), dim3(kBlock), 0, ctx->stream, (u64 *)tm, (u64 *)tv,
                     (const u64 *)all, (const uint32_t *)ranks, (unsigned long long)n, (unsigned long long)G);
  CRDT_HIP(ctx, hipGetLastError());
  // 3. the shard continues the GLOBAL fold from the fold of the lower ranks' states, so its
  //    conflicts are those of the global left fold (lwwreg.rs:84-98 is order-dependent)
  if (!R) {
    CRDT_TRY(device_fill(ctx, fc, G * 8, 0xFF));
  } else if (before > 0) {
    CRDT_TRY(crdt_lwwreg_lub_many(ctx, tm, tv, G, before, n, pm, pv, nullptr, 0));
    CRDT_TRY(crdt_lwwreg_lub_many(ctx, marker, val, G, R, group_stride, pm, pv, fc, CRDT_ACCUMULATE));
  }
  hipLaunchKernelGGL(lww_rebase_kernel, dim3(small_grid(ctx, G)), dim3(kBlock), 0, ctx->stream, (u64 *)fc,
                     (unsigned long long)G, (u64)base);
  CRDT_HIP(ctx, hipGetLastError());
  CRDT_NCCL(ctx, ncclAllReduce(fc, first_conflict ? (void *)first_conflict : (void *)fc, G, ncclUint64, ncclMin, comm,
                               ctx->stream));
  // 4. the global state: the fold of the world's rank states
  return crdt_lwwreg_lub_many(ctx, tm, tv, G, n, n, out_marker, out_val, nullptr, 0);
}

int crdt_map_lub_many_sharded(crdt_ctx *ctx, const crdt_map_batch *in, size_t k0, size_t K, crdt_map_out *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  CRDT_TRY(need_comm(ctx));
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "map_lub_many_sharded: NULL argument");
  const size_t G = in->G, Kk = in->K, A = in->A;
  if (k0 + Kk > K) return fail(ctx, CRDT_EINVAL, "map_lub_many_sharded: key range [%zu, %zu) past K = %zu", k0, k0 + Kk, K);
  const size_t D = (in->def_off && G > 0) ? in->def_off[G] - in->def_off[0] : 0;
  const size_t Kw = (K + 63) / 64, Kwl = (Kk + 63) / 64;
  if (D == 0 || Kk == 0 || A == 0) return crdt_map_lub_many(ctx, in, out);
  if (!in->def_keys || !out->def_keys || !out->def_keep)
    return fail(ctx, CRDT_EINVAL, "map_lub_many_sharded: deferred buffers missing");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  auto comm = (ncclComm_t)ctx->comm;
  // the key bitmaps restricted to this rank's keys [k0, k0 + Kk), re-indexed from 0
  void *lk, *ok;
  CRDT_TRY(sbuf(ctx, 0, D * Kwl * 8, &lk));
  CRDT_TRY(sbuf(ctx, 1, D * Kwl * 8, &ok));
  hipLaunchKernelGGL(bitmap_shift_kernel, dim3(small_grid(ctx, D * Kwl)), dim3(kBlock), 0, ctx->stream, (u64 *)lk,
                     (const u64 *)in->def_keys, (unsigned long long)D, (unsigned long long)Kwl,
                     (unsigned long long)Kw, (long long)k0, (long long)(k0 + Kk));
  CRDT_HIP(ctx, hipGetLastError());
  crdt_map_batch loc = *in;
  loc.def_keys = (const uint64_t *)lk;
  crdt_map_out lo = *out;
  lo.def_keys = (uint64_t *)ok;
  // keys are independent given the clocks and the deferred list: the exact left fold of the
  // rank's keys, with no data-path collective
  CRDT_TRY(crdt_map_lub_many(ctx, &loc, &lo));
  // surviving removes' key sets over all K keys: this rank's bits placed at k0, then a SUM
  // all-reduce (disjoint key ranges: the sum is the union)
  hipLaunchKernelGGL(bitmap_shift_kernel, dim3(small_grid(ctx, D * Kw)), dim3(kBlock), 0, ctx->stream,
                     (u64 *)out->def_keys, (const u64 *)ok, (unsigned long long)D, (unsigned long long)Kw,
                     (unsigned long long)Kwl, -(long long)k0, (long long)Kk);
  CRDT_HIP(ctx, hipGetLastError());
  timing_begin(ctx, "shard_exchange");
  CRDT_NCCL(ctx, ncclAllReduce(out->def_keys, out->def_keys, D * Kw, ncclUint64, ncclSum, comm, ctx->stream));
  timing_end(ctx);
  return CRDT_OK;
}

}  // extern "C"
