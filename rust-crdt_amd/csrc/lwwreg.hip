// LWWReg<u64 val, u64 marker> batched merge.
//
// Reference: FunkyCvRDT::merge (lwwreg.rs:43-45) -> update (lwwreg.rs:84-98):
//     if self.marker < marker            { self = (val, marker); Ok }
//     elif self.marker == marker && val != self.val { Err(ConflictingMarker), self unchanged }
//     else Ok (no-op)
// A fold acc = r[0]; for i in 1..R: acc.merge(r[i]) therefore ends in
//     (max marker, val of the FIRST replica holding it)      — argmax over (marker, -index)
// and merge i returns Err exactly when
//     marker_i == P(i-1).marker  &&  val_i != val[P(i-1).idx]
// where P(i-1) = inclusive prefix of (marker, first index) over r[0..i-1]: the state acc has
// just before merge i.  That prefix is an associative scan, so the fold is computed as
//   pass 1  lww_chunk_reduce : per chunk of CH replicas, (max marker, first index)
//   pass 2  lww_chunk_scan   : per group, exclusive scan over chunks + the final winner
//   pass 3  lww_conflict     : per chunk, in-chunk scan seeded by the chunk prefix, flags
//                              errors, atomicMin of the first erroring index per group.
#include "common.hpp"

namespace crdt {

constexpr u64 kNone = ~0ULL;
constexpr u64 kPrior = ~0ULL - 1;  // index of the caller's state under CRDT_ACCUMULATE (before replica 0)
constexpr int kLwwPer = 8;                      // replicas per thread
constexpr int kLwwChunk = kBlock * kLwwPer;     // replicas per chunk (one workgroup)

struct MI {
  u64 m, i;  // marker, first index holding it (kNone = empty)
};

__device__ __forceinline__ MI mi_join(MI a, MI b) {  // a precedes b in fold order
  if (a.i == kNone) return b;
  if (b.i == kNone) return a;
  return (a.m >= b.m) ? a : b;  // ties keep the earlier index
}

__device__ __forceinline__ MI wave_inclusive_scan(MI x) {
  const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    MI y;
    y.m = __shfl_up(x.m, d, kWave);
    y.i = __shfl_up(x.i, d, kWave);
    if (lane >= d) x = mi_join(y, x);
  }
  return x;
}

// Exclusive block scan of one MI per thread; returns this thread's exclusive prefix.
__device__ __forceinline__ MI block_exclusive_scan(MI x, MI *wave_tot) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  MI inc = wave_inclusive_scan(x);
  if (lane == kWave - 1) wave_tot[wid] = inc;
  __syncthreads();
  MI pre{0, kNone};
  for (int w = 0; w < wid; ++w) pre = mi_join(pre, wave_tot[w]);
  MI up;
  up.m = __shfl_up(inc.m, 1, kWave);
  up.i = __shfl_up(inc.i, 1, kWave);
  if (lane == 0) up = MI{0, kNone};
  __syncthreads();
  return mi_join(pre, up);
}

__device__ __forceinline__ MI block_reduce(MI x, MI *wave_tot) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    MI y;
    y.m = __shfl_down(x.m, d, kWave);
    y.i = __shfl_down(x.i, d, kWave);
    if (lane + d < kWave) x = mi_join(x, y);
  }
  if (lane == 0) wave_tot[wid] = x;
  __syncthreads();
  MI t{0, kNone};
  for (int w = 0; w < kBlock / kWave; ++w) t = mi_join(t, wave_tot[w]);
  __syncthreads();
  return t;
}

struct LwwPlan {
  const u64 *marker, *val;
  unsigned long long G, R, gstride, nch;
  MI *part;  // [G][nch]
  MI *pre;   // [G][nch] exclusive chunk prefixes
  u64 *prior_val;  // [G] the caller's val under CRDT_ACCUMULATE
  u64 *out_marker, *out_val, *first_conflict;
  int accumulate;
  bool vec;  // 16-byte aligned group rows: coalesced u64x2 staging
};

// Stage a chunk's markers in LDS with coalesced loads (16 B per lane when aligned); thread t
// then owns replicas c*CH + t*kLwwPer .. +kLwwPer (contiguous, fold order) from LDS.
__device__ __forceinline__ void stage_chunk(const u64 *__restrict__ mk, unsigned long long c0,
                                            unsigned long long R, bool vec, u64 *sm) {
  if (vec && c0 + kLwwChunk <= R) {
    const u64x2 *src = reinterpret_cast<const u64x2 *>(mk + c0);
#pragma unroll
    for (int k = 0; k < kLwwPer / 2; ++k) {
      const int j = k * kBlock + threadIdx.x;
      reinterpret_cast<u64x2 *>(sm)[j] = __builtin_nontemporal_load(src + j);
    }
  } else {
#pragma unroll
    for (int k = 0; k < kLwwPer; ++k) {
      const int j = k * kBlock + threadIdx.x;
      sm[j] = c0 + j < R ? mk[c0 + j] : 0;
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(kBlock) void lww_chunk_reduce(LwwPlan p) {
  __shared__ MI wt[kBlock / kWave];
  __shared__ u64 sm[kLwwChunk];
  const unsigned long long c = blockIdx.x % p.nch;
  const unsigned long long g = blockIdx.x / p.nch;
  const unsigned long long c0 = c * kLwwChunk;
  stage_chunk(p.marker + g * p.gstride, c0, p.R, p.vec, sm);
  const unsigned long long r0 = c0 + (unsigned long long)threadIdx.x * kLwwPer;
  MI x{0, kNone};
#pragma unroll
  for (int k = 0; k < kLwwPer; ++k) {
    const unsigned long long r = r0 + k;
    if (r < p.R) x = mi_join(x, MI{sm[threadIdx.x * kLwwPer + k], r});
  }
  x = block_reduce(x, wt);
  if (threadIdx.x == 0) p.part[g * p.nch + c] = x;
}

// One thread per group: exclusive scan over its chunks, and the folded winner.
__global__ __launch_bounds__(kBlock) void lww_chunk_scan(LwwPlan p) {
  const unsigned long long g = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= p.G) return;
  MI run{0, kNone};
  if (p.accumulate) {  // the caller's state precedes replica 0 (ties keep it: it is earlier)
    run = MI{p.out_marker[g], kPrior};
    p.prior_val[g] = p.out_val[g];
  }
  for (unsigned long long c = 0; c < p.nch; ++c) {
    p.pre[g * p.nch + c] = run;
    run = mi_join(run, p.part[g * p.nch + c]);
  }
  if (p.out_marker) p.out_marker[g] = run.m;
  if (p.out_val) p.out_val[g] = run.i == kPrior ? p.prior_val[g] : p.val[g * p.gstride + run.i];
}

// One workgroup per group (many chunks): the same exclusive scan, 256 chunk aggregates per step.
__global__ __launch_bounds__(kBlock) void lww_chunk_scan_block(LwwPlan p) {
  __shared__ MI wt[kBlock / kWave];
  __shared__ MI s_carry;
  const unsigned long long g = blockIdx.x;
  if (threadIdx.x == 0) {
    s_carry = MI{0, kNone};
    if (p.accumulate) {
      s_carry = MI{p.out_marker[g], kPrior};
      p.prior_val[g] = p.out_val[g];
    }
  }
  __syncthreads();
  for (unsigned long long c0 = 0; c0 < p.nch; c0 += kBlock) {
    const unsigned long long c = c0 + threadIdx.x;
    const MI x = c < p.nch ? p.part[g * p.nch + c] : MI{0, kNone};
    const MI carry = s_carry;
    const MI excl = block_exclusive_scan(x, wt);
    if (c < p.nch) p.pre[g * p.nch + c] = mi_join(carry, excl);
    if (threadIdx.x == kBlock - 1) s_carry = mi_join(carry, mi_join(excl, x));
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const MI run = s_carry;
    if (p.out_marker) p.out_marker[g] = run.m;
    if (p.out_val) p.out_val[g] = run.i == kPrior ? p.prior_val[g] : p.val[g * p.gstride + run.i];
  }
}

__global__ __launch_bounds__(kBlock) void lww_conflict(LwwPlan p) {
  __shared__ MI wt[kBlock / kWave];
  __shared__ unsigned long long s_first;
  __shared__ u64 sm[kLwwChunk];
  const unsigned long long c = blockIdx.x % p.nch;
  const unsigned long long g = blockIdx.x / p.nch;
  const MI pre = p.pre[g * p.nch + c];
  // A merge can only err on a marker equal to the running max; if every marker of the chunk is
  // below the incoming prefix max, none can (block-uniform early exit, no loads).
  if (pre.i != kNone && p.part[g * p.nch + c].m < pre.m) return;
  const u64 *vl = p.val + g * p.gstride;
  const unsigned long long c0 = c * kLwwChunk;
  if (threadIdx.x == 0) s_first = kNone;
  stage_chunk(p.marker + g * p.gstride, c0, p.R, p.vec, sm);
  const unsigned long long r0 = c0 + (unsigned long long)threadIdx.x * kLwwPer;
  u64 m[kLwwPer];
  MI agg{0, kNone};
#pragma unroll
  for (int k = 0; k < kLwwPer; ++k) {
    const unsigned long long r = r0 + k;
    m[k] = sm[threadIdx.x * kLwwPer + k];
    if (r < p.R) agg = mi_join(agg, MI{m[k], r});
  }
  MI run = mi_join(pre, block_exclusive_scan(agg, wt));
  unsigned long long first = kNone;
#pragma unroll
  for (int k = 0; k < kLwwPer; ++k) {
    const unsigned long long r = r0 + k;
    if (r < p.R) {
      if (run.i != kNone && m[k] == run.m && first == kNone) {
        const u64 held = run.i == kPrior ? p.prior_val[g] : vl[run.i];
        if (vl[r] != held) first = r;
      }
      run = mi_join(run, MI{m[k], r});
    }
  }
  if (first != kNone) atomicMin(&s_first, first);
  __syncthreads();
  if (threadIdx.x == 0 && s_first != kNone) atomicMin(p.first_conflict + g, s_first);
}

__global__ __launch_bounds__(kBlock) void lww_merge_pairs(u64 *sm, u64 *sv, const u64 *om,
                                                          const u64 *ov, unsigned long long N,
                                                          uint8_t *conflict) {
  const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const u64 a = sm[i], b = om[i];
  uint8_t err = 0;
  if (a < b) {
    sm[i] = b;
    sv[i] = ov[i];
  } else if (a == b) {
    err = sv[i] != ov[i];
  }
  if (conflict) conflict[i] = err;
}

int lww_lub_many_dev(crdt_ctx *ctx, const u64 *marker, const u64 *val, size_t G, size_t R, size_t group_stride,
                     u64 *out_marker, u64 *out_val, u64 *first_conflict, unsigned flags) {
  CRDT_CHECK_CTX(ctx);
  if (G == 0) return CRDT_OK;
  const bool accumulate = flags & CRDT_ACCUMULATE;
  if (accumulate && (!out_marker || !out_val))
    return fail(ctx, CRDT_EINVAL, "lwwreg_lub_many: CRDT_ACCUMULATE needs out_marker and out_val");
  if (R == 0 && accumulate) {
    if (first_conflict)
      if (int rc = device_fill(ctx, first_conflict, G * 8, 0xFF)) return rc;
    return CRDT_OK;
  }
  if (R == 0) return fail(ctx, CRDT_EINVAL, "lwwreg_lub_many: R == 0 (LWWReg has no identity; the fold starts at replica 0)");
  if (!marker || !val) return fail(ctx, CRDT_EINVAL, "lwwreg_lub_many: NULL input");
  if (G > 1 && group_stride < R)
    return fail(ctx, CRDT_EINVAL, "lwwreg_lub_many: group_stride %zu < R %zu", group_stride, R);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  LwwPlan p{};
  p.marker = (const u64 *)marker;
  p.val = (const u64 *)val;
  p.G = G;
  p.R = R;
  p.gstride = group_stride;
  p.nch = (R + kLwwChunk - 1) / kLwwChunk;
  p.out_marker = (u64 *)out_marker;
  p.out_val = (u64 *)out_val;
  p.first_conflict = (u64 *)first_conflict;
  const size_t nparts = G * p.nch;
  if (G * p.nch > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "lwwreg_lub_many: grid too large");
  p.accumulate = accumulate ? 1 : 0;
  p.vec = (reinterpret_cast<uintptr_t>(marker) & 15) == 0 && (G == 1 || group_stride % 2 == 0);
  int rc = ensure_scratch(ctx, 2 * nparts * sizeof(MI) + G * sizeof(u64));
  if (rc) return rc;
  p.part = static_cast<MI *>(ctx->scratch);
  p.pre = p.part + nparts;
  p.prior_val = reinterpret_cast<u64 *>(p.pre + nparts);
  timing_begin(ctx, "lww_reduce");
  hipLaunchKernelGGL(lww_chunk_reduce, dim3((unsigned)nparts), dim3(kBlock), 0, ctx->stream, p);
  timing_end(ctx);
  if (p.nch > 16)  // long groups: a workgroup scans each group's chunk aggregates
    hipLaunchKernelGGL(lww_chunk_scan_block, dim3((unsigned)G), dim3(kBlock), 0, ctx->stream, p);
  else
    hipLaunchKernelGGL(lww_chunk_scan, dim3((unsigned)((G + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       ctx->stream, p);
  if (first_conflict) {
    if (int rc = device_fill(ctx, first_conflict, G * sizeof(uint64_t), 0xFF)) return rc;
    hipLaunchKernelGGL(lww_conflict, dim3((unsigned)nparts), dim3(kBlock), 0, ctx->stream, p);
  }
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

int lww_merge_batch_dev(crdt_ctx *ctx, u64 *self_marker, u64 *self_val, const u64 *other_marker,
                        const u64 *other_val, size_t N, uint8_t *conflict) {
  CRDT_CHECK_CTX(ctx);
  if (N == 0) return CRDT_OK;
  if (!self_marker || !self_val || !other_marker || !other_val)
    return fail(ctx, CRDT_EINVAL, "lwwreg_merge_batch: NULL buffer");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const unsigned long long nb = (N + kBlock - 1) / kBlock;
  if (nb > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "lwwreg_merge_batch: N too large");
  timing_begin(ctx, "lww_merge_pairs");
  hipLaunchKernelGGL(lww_merge_pairs, dim3((unsigned)nb), dim3(kBlock), 0, ctx->stream,
                     (u64 *)self_marker, (u64 *)self_val, (const u64 *)other_marker,
                     (const u64 *)other_val, (unsigned long long)N, conflict);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

}  // namespace crdt

using namespace crdt;

extern "C" {

int crdt_lwwreg_lub_many(crdt_ctx *ctx, const uint64_t *marker, const uint64_t *val, size_t G,
                         size_t R, size_t group_stride, uint64_t *out_marker,
                         uint64_t *out_val, uint64_t *first_conflict, unsigned flags) {
  CRDT_CHECK_CTX(ctx);
  if (ctx->mem_kind == CRDT_MEM_HOST)
    return lww_lub_many_host(ctx, (const u64 *)marker, (const u64 *)val, G, R, group_stride, (u64 *)out_marker,
                             (u64 *)out_val, (u64 *)first_conflict, flags);
  return lww_lub_many_dev(ctx, (const u64 *)marker, (const u64 *)val, G, R, group_stride, (u64 *)out_marker,
                          (u64 *)out_val, (u64 *)first_conflict, flags);
}

int crdt_lwwreg_merge_batch(crdt_ctx *ctx, uint64_t *self_marker, uint64_t *self_val,
                            const uint64_t *other_marker, const uint64_t *other_val,
                            size_t N, uint8_t *conflict) {
  CRDT_CHECK_CTX(ctx);
  if (ctx->mem_kind == CRDT_MEM_HOST)
    return lww_merge_batch_host(ctx, (u64 *)self_marker, (u64 *)self_val, (const u64 *)other_marker,
                                (const u64 *)other_val, N, conflict);
  return lww_merge_batch_dev(ctx, (u64 *)self_marker, (u64 *)self_val, (const u64 *)other_marker,
                             (const u64 *)other_val, N, conflict);
}

}  // extern "C"
