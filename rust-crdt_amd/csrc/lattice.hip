// Lattice lub kernels: elementwise max (VClock, GCounter, PNCounter) and bitwise OR (GSet).
//
// Reference semantics (crdts 3.0.0):
//   VClock::merge    vclock.rs:130-136 -> apply_dot :155-159  => out[a] = max(self[a], other[a])
//   GCounter::merge  gcounter.rs:44-48  (VClock on `inner`)
//   PNCounter::merge pncounter.rs:70-75 (P and N independently)  => max over a row of 2A words
//   GSet::merge      gset.rs:38-40 -> insert :69-71             => union = OR of interned bitmaps
// All four joins are associative, commutative and idempotent (README.md:37-47), so the fold
// `acc = T::new(); for r: acc.merge(r)` equals any tree of joins: the kernels fold a slice
// of replicas per thread in registers, combine the threads of a workgroup through LDS and
// the workgroups of a group through a two-level last-arriver combine inside the same launch.
//
// HBM layout: replica (g, r) row = in + g*gstride + r*rstride, W words contiguous.
// Loads are 16 B per lane (u64x2) and non-temporal: every input byte is read exactly once.
#include "common.hpp"

namespace crdt {

template <int V>
struct VecOf;
template <>
struct VecOf<1> {
  using T = u64;
};
template <>
struct VecOf<2> {
  using T = u64x2;
};

template <Op OP>
__device__ __forceinline__ u64 vjoin(u64 a, u64 b) {
  return join<OP>(a, b);
}
template <Op OP>
__device__ __forceinline__ u64x2 vjoin(u64x2 a, u64x2 b) {
  return join2<OP>(a, b);
}

template <typename VT>
__device__ __forceinline__ VT vzero() {
  return VT(0);
}

// Fold n rows spaced `step` vectors apart, U loads in flight per thread.
template <Op OP, typename VT, int U, bool NT>
__device__ __forceinline__ VT fold_rows(const VT *__restrict__ p, size_t n, long long step) {
  VT acc = vzero<VT>();
  size_t i = 0;
  for (; i + U <= n; i += U) {
    VT v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if constexpr (NT) v[k] = __builtin_nontemporal_load(p + k * step);
      else v[k] = p[k * step];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) acc = vjoin<OP>(acc, v[k]);
    p += U * step;
  }
  for (; i < n; ++i) {
    VT v;
    if constexpr (NT) v = __builtin_nontemporal_load(p);
    else v = *p;
    acc = vjoin<OP>(acc, v);
    p += step;
  }
  return acc;
}

// Combine the TR row-lanes of a workgroup that share a column (lane l = rsub*PW + cl).
// Result valid for rsub == 0.  Every thread of the block must call it.
template <Op OP, typename VT>
__device__ __forceinline__ VT block_rows_combine(VT acc, VT *red, int l, int PW, int TR) {
  if (TR > 1) {
    red[l] = acc;
    __syncthreads();
    if (l < PW) {
      for (int j = 1; j < TR; ++j) acc = vjoin<OP>(acc, red[l + j * PW]);
    }
    __syncthreads();
  }
  return acc;
}

struct LubPlan {
  const u64 *in;
  u64 *out;
  u64 *part;   // [units][S][PW] vectors
  u64 *cpart;  // [units][ncl][PW] vectors
  unsigned *cnt1;  // [units][ncl]
  unsigned *cnt2;  // [units]
  long long rstride, gstride, ostride;  // words
  unsigned long long R, Rs;
  int Wv, PW, TR, ncolblk, S, CL, ncl;
  int accumulate;
  int interleave;  // 1: slice s takes row-steps s, s+S, s+2S, ... (all slices sweep HBM together)
};

template <Op OP, typename VT>
__device__ __forceinline__ void store_out(const LubPlan &p, size_t g, int col, VT v) {
  VT *o = reinterpret_cast<VT *>(p.out + g * p.ostride) + col;
  if (p.accumulate) v = vjoin<OP>(v, *o);
  *o = v;
}

// Agent-scope arrival on a counter after this block's stores (MI355X_MICROARCH.md
// "Valid forms": waitcnt -> barrier -> lane-0 release fence -> waitcnt -> atomic).
// Returns (block-uniformly) whether this block is the last of `expected` arrivals; the last
// arriver resets the counter and performs the agent-scope acquire before returning.
__device__ __forceinline__ bool arrive_last(unsigned *counter, unsigned expected, int *s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = (t == expected - 1);
    if (last) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag != 0;
}

// One launch = the whole lub.  Block b -> (unit u = g*ncolblk + cb, slice s).
template <Op OP, int V, int U, bool NT, typename VT>
__device__ __forceinline__ void lub_stream_body(const LubPlan &p, unsigned b, VT *red, int &s_flag) {
  const int l = threadIdx.x;
  const int s = b % p.S;
  const unsigned u = b / p.S;
  const int cb = u % p.ncolblk;
  const size_t g = u / p.ncolblk;
  const int cl = l % p.PW;
  const int rsub = l / p.PW;
  const int col = cb * kBlock + cl;
  const bool active = rsub < p.TR && col < p.Wv;

  VT acc = vzero<VT>();
  if (active) {
    unsigned long long r0, rend, rstep;
    if (p.interleave) {
      r0 = (unsigned long long)s * p.TR + rsub;
      rend = p.R;
      rstep = (unsigned long long)p.S * p.TR;
    } else {
      const unsigned long long rbeg = (unsigned long long)s * p.Rs;
      rend = min(p.R, rbeg + p.Rs);
      r0 = rbeg + rsub;
      rstep = p.TR;
    }
    if (r0 < rend) {
      const size_t n = (rend - r0 + rstep - 1) / rstep;
      const VT *src = reinterpret_cast<const VT *>(p.in + g * p.gstride + r0 * p.rstride) + col;
      acc = fold_rows<OP, VT, U, NT>(src, n, (long long)rstep * p.rstride / V);
    }
  }
  acc = block_rows_combine<OP>(acc, red, l, p.PW, p.TR);
  const bool writer = (l < p.PW) && col < p.Wv;
  if (p.S == 1) {
    if (writer) store_out<OP>(p, g, col, acc);
    return;
  }

  // Level 1: publish this slice's partial row; the last slice of the cluster combines it.
  VT *part = reinterpret_cast<VT *>(p.part);
  if (writer) part[((size_t)u * p.S + s) * p.PW + cl] = acc;
  const int c = s / p.CL;
  const int csize = min(p.CL, p.S - c * p.CL);
  if (!arrive_last(p.cnt1 + (size_t)u * p.ncl + c, csize, &s_flag)) return;

  acc = vzero<VT>();
  {
    const int TRc = p.TR;
    if (rsub < TRc && col < p.Wv) {
      const int r0 = rsub;
      if (r0 < csize) {
        const size_t n = (csize - r0 + TRc - 1) / TRc;
        acc = fold_rows<OP, VT, 4, false>(part + ((size_t)u * p.S + c * p.CL + r0) * p.PW + cl, n,
                                          (long long)TRc * p.PW);
      }
    }
  }
  acc = block_rows_combine<OP>(acc, red, l, p.PW, p.TR);
  if (p.ncl == 1) {
    if (writer) store_out<OP>(p, g, col, acc);
    return;
  }

  // Level 2: publish the cluster partial; the last cluster combines all of them.
  VT *cpart = reinterpret_cast<VT *>(p.cpart);
  if (writer) cpart[((size_t)u * p.ncl + c) * p.PW + cl] = acc;
  if (!arrive_last(p.cnt2 + u, p.ncl, &s_flag)) return;

  acc = vzero<VT>();
  if (rsub < p.TR && col < p.Wv && rsub < p.ncl) {
    const size_t n = (p.ncl - rsub + p.TR - 1) / p.TR;
    acc = fold_rows<OP, VT, 4, false>(cpart + ((size_t)u * p.ncl + rsub) * p.PW + cl, n,
                                      (long long)p.TR * p.PW);
  }
  acc = block_rows_combine<OP>(acc, red, l, p.PW, p.TR);
  if (writer) store_out<OP>(p, g, col, acc);
}

template <Op OP, int V, int U, bool NT = true>
__global__ __launch_bounds__(kBlock) void lub_stream_kernel(LubPlan p) {
  using VT = typename VecOf<V>::T;
  __shared__ VT red[kBlock];
  __shared__ int s_flag;
  lub_stream_body<OP, V, U, NT, VT>(p, blockIdx.x, red, s_flag);
}

// Several lubs of one join op in ONE launch (crdt_lub_many_multi): segment i owns blocks
// [start[i], start[i+1]) and runs exactly the single-lub body on its own plan, so the launch pays
// one ramp and one tail instead of one per lub.
constexpr int kLubMultiMax = 8;
struct LubMulti {
  LubPlan p[kLubMultiMax];
  unsigned start[kLubMultiMax + 1];
  int n;
};

template <Op OP, int V, int U>
__global__ __launch_bounds__(kBlock) void lub_multi_kernel(LubMulti m) {
  using VT = typename VecOf<V>::T;
  __shared__ VT red[kBlock];
  __shared__ int s_flag;
  const unsigned b = blockIdx.x;
  int i = 0;
#pragma unroll
  for (int j = 1; j < kLubMultiMax; ++j)
    if (j < m.n && b >= m.start[j]) i = j;
  lub_stream_body<OP, V, U, true, VT>(m.p[i], b - m.start[i], red, s_flag);
}

// self[i] := self[i] ⊔ other[i]: three streams (2 reads, 1 write), TR rows per block step.
template <Op OP, int V>
__global__ __launch_bounds__(kBlock) void merge_pairs_kernel(u64 *__restrict__ self,
                                                             const u64 *__restrict__ other,
                                                             unsigned long long N, int Wv, int PW,
                                                             int TR, long long sstride,
                                                             long long ostride,
                                                             unsigned long long rows_per_block) {
  using VT = typename VecOf<V>::T;
  constexpr int U = 4;  // row pairs in flight per lane
  const int l = threadIdx.x;
  const int cl = l % PW;
  const int rsub = l / PW;
  const int col = blockIdx.y * kBlock + cl;
  if (rsub >= TR || col >= Wv) return;
  const unsigned long long rbeg = (unsigned long long)blockIdx.x * rows_per_block;
  const unsigned long long rend = min(N, rbeg + rows_per_block);
  unsigned long long r = rbeg + rsub;
  for (; r + (U - 1) * TR < rend; r += U * TR) {
    VT a[U], bv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      a[k] = __builtin_nontemporal_load(reinterpret_cast<const VT *>(self + (r + k * TR) * sstride) + col);
      bv[k] = __builtin_nontemporal_load(reinterpret_cast<const VT *>(other + (r + k * TR) * ostride) + col);
    }
#pragma unroll
    for (int k = 0; k < U; ++k)
      __builtin_nontemporal_store(vjoin<OP>(a[k], bv[k]), reinterpret_cast<VT *>(self + (r + k * TR) * sstride) + col);
  }
  for (; r < rend; r += TR) {
    VT *sp = reinterpret_cast<VT *>(self + r * sstride) + col;
    const VT *op = reinterpret_cast<const VT *>(other + r * ostride) + col;
    *sp = vjoin<OP>(*sp, __builtin_nontemporal_load(op));
  }
}

// merge_batch with 16-byte rows: LR-lane row groups (common.hpp ROW_GROUP_LOOP), ~8 independent
// pieces per lane, 2 workgroups per CU — the shape that measured fastest for the 2-read-1-write
// row passes (1,080 us vs 1,207 us for merge_pairs_kernel at 1M pairs x 256).
template <Op OP>
__global__ __launch_bounds__(kBlock) void merge_rows_kernel(u64 *self, const u64 *other, unsigned long long N,
                                                            unsigned long long W, long long ss, long long os,
                                                            int lr_log) {
  ROW_GROUP_LOOP(N, lr_log) {
    const unsigned long long r = rb + (lane >> lr_log);
    if (r >= N) continue;
    u64 *sr = self + r * ss;
    const u64 *orow = other + r * os;
#pragma unroll 8
    for (unsigned long long c = 2ull * gl; c < W; c += 2ull * LR) {
      const u64x2 a = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(sr + c));
      const u64x2 b = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(orow + c));
      __builtin_nontemporal_store(join2<OP>(a, b), reinterpret_cast<u64x2 *>(sr + c));
    }
  }
}

// merge_batch of packed rows (both strides == W): one flat stream of 16-byte pieces, grid-stride,
// 2 pieces per lane in flight at one workgroup per CU — the shape at which an in-place
// read-self / read-other / write-self stream peaks on this part (scripts/micro/stream_rate.hip,
// 75% vs 65-69% with more requests in flight).
template <Op OP, int U>
__global__ __launch_bounds__(kBlock) void merge_flat_kernel(u64x2 *self, const u64x2 *other, unsigned long long n) {
  const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
  unsigned long long i = (unsigned long long)blockIdx.x * kBlock + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u64x2 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = __builtin_nontemporal_load(self + i + u * stride);
      b[u] = __builtin_nontemporal_load(other + i + u * stride);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(join2<OP>(a[u], b[u]), self + i + u * stride);
  }
  for (; i < n; i += stride) __builtin_nontemporal_store(join2<OP>(self[i], other[i]), self + i);
}

static bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Validation and launch geometry of one lub (no scratch yet).  launch = false: nothing to run
// (an empty fold was already written, or G / W is 0).
struct LubSetup {
  LubPlan p;
  int V = 1;
  bool launch = false;
  size_t blocks = 0, part_b = 0, cpart_b = 0, ncnt = 0;
};

static int lub_prepare(crdt_ctx *ctx, Op op, const u64 *in, size_t G, size_t R, size_t W, size_t row_stride,
                       size_t group_stride, u64 *out, size_t out_stride, unsigned flags, LubSetup &su) {
  su = LubSetup{};
  if (G == 0 || W == 0) return CRDT_OK;
  if (!out) return fail(ctx, CRDT_EINVAL, "lub_many: out is NULL");
  if (G > 1 && out_stride < W)
    return fail(ctx, CRDT_EINVAL, "lub_many: out_stride %zu < row width %zu", out_stride, W);
  if (W > (size_t)1 << 30) return fail(ctx, CRDT_EUNSUPPORTED, "lub_many: row width %zu too large", W);
  const bool accumulate = flags & CRDT_ACCUMULATE;
  if (R == 0) {  // fold of nothing = T::new() (all zero); with ACCUMULATE: unchanged
    if (!accumulate)
      CRDT_HIP(ctx, hipMemset2DAsync(out, (G > 1 ? out_stride : W) * 8, 0, W * 8, G, ctx->stream));
    return CRDT_OK;
  }
  if (!in) return fail(ctx, CRDT_EINVAL, "lub_many: in is NULL");
  if (R > 1 && row_stride < W)
    return fail(ctx, CRDT_EINVAL, "lub_many: row_stride %zu < row width %zu", row_stride, W);

  const bool vec2 = (W % 2 == 0) && (R == 1 || row_stride % 2 == 0) &&
                    (G == 1 || (group_stride % 2 == 0 && out_stride % 2 == 0)) && aligned16(in) &&
                    aligned16(out);
  const int V = vec2 ? 2 : 1;
  LubPlan &p = su.p;
  p.in = in;
  p.out = out;
  p.rstride = (long long)row_stride;
  p.gstride = (long long)group_stride;
  p.ostride = (long long)out_stride;
  p.R = R;
  p.Wv = (int)(W / V);
  p.PW = p.Wv <= kBlock ? p.Wv : kBlock;
  p.TR = kBlock / p.PW;
  p.ncolblk = (p.Wv + kBlock - 1) / kBlock;
  p.accumulate = accumulate ? 1 : 0;

  // Slice replicas so the grid holds ~bpc workgroups per CU, each thread folding >= min_steps rows.
  const size_t units = G * (size_t)p.ncolblk;
  const size_t target = ctx->tune.lub_grid > 0 ? (size_t)ctx->tune.lub_grid
                                               : (size_t)ctx->cu_count * ctx->tune.lub_blocks_per_cu;
  const size_t steps = (R + p.TR - 1) / p.TR;
  size_t S = 1;
  if (units < target) {
    S = (target + units - 1) / units;
    size_t max_s = steps / ctx->tune.lub_min_steps;
    if (max_s < 1) max_s = 1;
    if (S > max_s) S = max_s;
  }
  size_t Rs = (R + S - 1) / S;
  Rs = (Rs + p.TR - 1) / p.TR * p.TR;  // whole block steps per slice
  S = (R + Rs - 1) / Rs;
  if ((size_t)units * S > 0x7fffffffULL)
    return fail(ctx, CRDT_EUNSUPPORTED, "lub_many: grid too large (%zu units x %zu slices)", units, S);
  p.S = (int)S;
  p.Rs = Rs;
  p.interleave = ctx->tune.lub_interleave;
  p.CL = 32;
  p.ncl = (p.S + p.CL - 1) / p.CL;
  if (p.S > 1) {
    const size_t vecb = (size_t)V * 8;
    su.part_b = units * S * p.PW * vecb;
    su.cpart_b = units * p.ncl * p.PW * vecb;
    su.ncnt = units * p.ncl + units;
  }
  su.V = V;
  su.blocks = units * S;
  su.launch = true;
  return CRDT_OK;
}

// Scratch of a prepared lub at `base` (part, then cpart) and counters at `cnt`.
static void lub_assign(LubSetup &su, char *base, unsigned *cnt) {
  if (su.p.S <= 1) return;
  const size_t units = su.blocks / su.p.S;
  su.p.cnt1 = cnt;
  su.p.cnt2 = cnt + units * su.p.ncl;
  su.p.part = reinterpret_cast<u64 *>(base);
  su.p.cpart = reinterpret_cast<u64 *>(base + su.part_b);
}

int lattice_lub_many(crdt_ctx *ctx, Op op, const u64 *in, size_t G, size_t R, size_t W,
                     size_t row_stride, size_t group_stride, u64 *out, size_t out_stride,
                     unsigned flags) {
  CRDT_CHECK_CTX(ctx);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  LubSetup su;
  if (int rc = lub_prepare(ctx, op, in, G, R, W, row_stride, group_stride, out, out_stride, flags, su)) return rc;
  if (!su.launch) return CRDT_OK;
  if (su.p.S > 1) {
    if (int rc = ensure_scratch(ctx, su.part_b + su.cpart_b)) return rc;
    if (int rc = ensure_counters(ctx, su.ncnt)) return rc;
    lub_assign(su, static_cast<char *>(ctx->scratch), ctx->counters);
  }
  const LubPlan &p = su.p;
  const int V = su.V;
  const dim3 grid((unsigned)su.blocks);
  timing_begin(ctx, "lub_stream");
  const int U = ctx->tune.lub_unroll;
#define CRDT_LAUNCH_LUB(OPV, VV, UV) \
  hipLaunchKernelGGL((lub_stream_kernel<OPV, VV, UV>), grid, dim3(kBlock), 0, ctx->stream, p)
  if (op == Op::Max) {
    if (V == 2) {
      if (!ctx->tune.lub_nt) hipLaunchKernelGGL((lub_stream_kernel<Op::Max, 2, 8, false>), grid, dim3(kBlock), 0, ctx->stream, p);
      else if (U == 4) CRDT_LAUNCH_LUB(Op::Max, 2, 4);
      else if (U == 16) CRDT_LAUNCH_LUB(Op::Max, 2, 16);
      else if (U == 32) CRDT_LAUNCH_LUB(Op::Max, 2, 32);
      else CRDT_LAUNCH_LUB(Op::Max, 2, 8);
    } else CRDT_LAUNCH_LUB(Op::Max, 1, 8);
  } else {
    if (V == 2) CRDT_LAUNCH_LUB(Op::Or, 2, 8);
    else CRDT_LAUNCH_LUB(Op::Or, 1, 8);
  }
#undef CRDT_LAUNCH_LUB
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

// Several lattice lubs, one launch per (join op, vector width) class of up to kLubMultiMax
// segments; results identical to one lattice_lub_many per segment (each segment's blocks run the
// single-lub body on its own plan and scratch).
int lattice_lub_many_multi(crdt_ctx *ctx, const LubReq *reqs, size_t n) {
  CRDT_CHECK_CTX(ctx);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  std::vector<LubSetup> su(n);
  for (size_t i = 0; i < n; ++i) {
    const LubReq &q = reqs[i];
    if (int rc = lub_prepare(ctx, q.op, q.in, q.G, q.R, q.W, q.row_stride, q.group_stride, q.out, q.out_stride,
                             q.flags, su[i]))
      return rc;
  }
  // one scratch / counter region for every segment (a later launch of this call never reuses an
  // earlier one's region, so launches need no ordering beyond the stream's)
  size_t sb = 0, nc = 0;
  for (auto &x : su)
    if (x.launch) {
      sb += (x.part_b + x.cpart_b + 255) / 256 * 256;
      nc += x.ncnt;
    }
  if (sb) {
    if (int rc = ensure_scratch(ctx, sb)) return rc;
    if (int rc = ensure_counters(ctx, nc)) return rc;
  }
  {
    char *base = static_cast<char *>(ctx->scratch);
    unsigned *cnt = ctx->counters;
    for (auto &x : su)
      if (x.launch && x.p.S > 1) {
        lub_assign(x, base, cnt);
        base += (x.part_b + x.cpart_b + 255) / 256 * 256;
        cnt += x.ncnt;
      }
  }
  std::vector<bool> done(n, false);
  for (size_t i = 0; i < n; ++i) {
    if (!su[i].launch || done[i]) continue;
    LubMulti m{};
    m.n = 0;
    size_t blocks = 0;
    const Op op = reqs[i].op;
    const int V = su[i].V;
    for (size_t j = i; j < n && m.n < kLubMultiMax; ++j) {
      if (!su[j].launch || done[j] || reqs[j].op != op || su[j].V != V) continue;
      m.p[m.n] = su[j].p;
      m.start[m.n] = (unsigned)blocks;
      blocks += su[j].blocks;
      ++m.n;
      done[j] = true;
    }
    if (blocks > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "lub_many_multi: grid too large");
    for (int k = m.n; k <= kLubMultiMax; ++k) m.start[k] = (unsigned)blocks;
    timing_begin(ctx, "lub_stream");
    if (op == Op::Max) {
      if (V == 2) hipLaunchKernelGGL((lub_multi_kernel<Op::Max, 2, 8>), dim3((unsigned)blocks), dim3(kBlock), 0, ctx->stream, m);
      else hipLaunchKernelGGL((lub_multi_kernel<Op::Max, 1, 8>), dim3((unsigned)blocks), dim3(kBlock), 0, ctx->stream, m);
    } else {
      if (V == 2) hipLaunchKernelGGL((lub_multi_kernel<Op::Or, 2, 8>), dim3((unsigned)blocks), dim3(kBlock), 0, ctx->stream, m);
      else hipLaunchKernelGGL((lub_multi_kernel<Op::Or, 1, 8>), dim3((unsigned)blocks), dim3(kBlock), 0, ctx->stream, m);
    }
    timing_end(ctx);
    CRDT_HIP(ctx, hipGetLastError());
  }
  return CRDT_OK;
}

int lattice_merge_batch(crdt_ctx *ctx, Op op, u64 *self, const u64 *other, size_t N, size_t W,
                        size_t self_stride, size_t other_stride) {
  CRDT_CHECK_CTX(ctx);
  if (N == 0 || W == 0) return CRDT_OK;
  if (!self || !other) return fail(ctx, CRDT_EINVAL, "merge_batch: NULL buffer");
  if (N > 1 && (self_stride < W || other_stride < W))
    return fail(ctx, CRDT_EINVAL, "merge_batch: stride < row width %zu", W);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const bool vec2 = W % 2 == 0 && (N == 1 || (self_stride % 2 == 0 && other_stride % 2 == 0)) &&
                    aligned16(self) && aligned16(other);
  const bool packed = N == 1 || (self_stride == W && other_stride == W);
  if (vec2 && packed && ctx->tune.merge_flat) {
    const unsigned long long n = (unsigned long long)N * W / 2;  // 16-byte pieces
    const unsigned long long want = (n + kBlock - 1) / kBlock;
    const unsigned long long cap = (unsigned long long)ctx->cu_count * ctx->tune.merge_flat;
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    timing_begin(ctx, "merge_pairs");
    u64x2 *sp = reinterpret_cast<u64x2 *>(self);
    const u64x2 *op2 = reinterpret_cast<const u64x2 *>(other);
    const int fu = ctx->tune.merge_flat_u;
#define CRDT_FLAT(OPV, UU) hipLaunchKernelGGL((merge_flat_kernel<OPV, UU>), dim3(grid), dim3(kBlock), 0, ctx->stream, sp, op2, n)
    if (op == Op::Max) {
      if (fu == 1) CRDT_FLAT(Op::Max, 1);
      else if (fu == 4) CRDT_FLAT(Op::Max, 4);
      else CRDT_FLAT(Op::Max, 2);
    } else {
      if (fu == 1) CRDT_FLAT(Op::Or, 1);
      else if (fu == 4) CRDT_FLAT(Op::Or, 4);
      else CRDT_FLAT(Op::Or, 2);
    }
#undef CRDT_FLAT
    timing_end(ctx);
    CRDT_HIP(ctx, hipGetLastError());
    return CRDT_OK;
  }
  if (vec2 && ctx->tune.merge_rows) {
    const int lr_log = row_lr_log(W / 2, ctx->tune.merge_ppl);
    const unsigned long long rpb = 4ull * (kWave >> lr_log);
    const unsigned long long want = (N + rpb - 1) / rpb;
    const unsigned long long cap = (unsigned long long)ctx->cu_count * ctx->tune.merge_blocks_per_cu;
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    timing_begin(ctx, "merge_pairs");
    if (op == Op::Max)
      hipLaunchKernelGGL(merge_rows_kernel<Op::Max>, dim3(grid), dim3(kBlock), 0, ctx->stream, self, other,
                         (unsigned long long)N, (unsigned long long)W, (long long)self_stride, (long long)other_stride, lr_log);
    else
      hipLaunchKernelGGL(merge_rows_kernel<Op::Or>, dim3(grid), dim3(kBlock), 0, ctx->stream, self, other,
                         (unsigned long long)N, (unsigned long long)W, (long long)self_stride, (long long)other_stride, lr_log);
    timing_end(ctx);
    CRDT_HIP(ctx, hipGetLastError());
    return CRDT_OK;
  }
  const int V = vec2 ? 2 : 1;
  const int Wv = (int)(W / V);
  const int PW = Wv <= kBlock ? Wv : kBlock;
  const int TR = kBlock / PW;
  const int ncolblk = (Wv + kBlock - 1) / kBlock;
  // Contiguous row ranges, ~mbpc workgroups per CU (each lane >= 16 row steps).
  const unsigned long long want = (unsigned long long)ctx->cu_count * ctx->tune.merge_blocks_per_cu;
  unsigned long long rpb = (N + want - 1) / want;
  rpb = (rpb + TR - 1) / TR * TR;
  if (rpb < (unsigned long long)TR * 16) rpb = (unsigned long long)TR * 16;
  unsigned long long nb = (N + rpb - 1) / rpb;
  if (nb > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "merge_batch: N too large");
  dim3 grid((unsigned)nb, (unsigned)ncolblk);
  timing_begin(ctx, "merge_pairs");
  if (op == Op::Max) {
    if (V == 2) hipLaunchKernelGGL((merge_pairs_kernel<Op::Max, 2>), grid, dim3(kBlock), 0, ctx->stream, self, other, N, Wv, PW, TR, (long long)self_stride, (long long)other_stride, rpb);
    else hipLaunchKernelGGL((merge_pairs_kernel<Op::Max, 1>), grid, dim3(kBlock), 0, ctx->stream, self, other, N, Wv, PW, TR, (long long)self_stride, (long long)other_stride, rpb);
  } else {
    if (V == 2) hipLaunchKernelGGL((merge_pairs_kernel<Op::Or, 2>), grid, dim3(kBlock), 0, ctx->stream, self, other, N, Wv, PW, TR, (long long)self_stride, (long long)other_stride, rpb);
    else hipLaunchKernelGGL((merge_pairs_kernel<Op::Or, 1>), grid, dim3(kBlock), 0, ctx->stream, self, other, N, Wv, PW, TR, (long long)self_stride, (long long)other_stride, rpb);
  }
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

}  // namespace crdt

using crdt::Op;
using crdt::u64;

// CRDT_MEM_HOST routes the public lattice entry points through the chunked host staging.
static int lub_dispatch(crdt_ctx *ctx, Op op, const u64 *in, size_t G, size_t R, size_t W, size_t row_stride,
                        size_t group_stride, u64 *out, size_t out_stride, unsigned flags) {
  CRDT_CHECK_CTX(ctx);
  if (ctx->mem_kind == CRDT_MEM_HOST)
    return crdt::lattice_lub_many_host(ctx, op, in, G, R, W, row_stride, group_stride, out, out_stride, flags);
  return crdt::lattice_lub_many(ctx, op, in, G, R, W, row_stride, group_stride, out, out_stride, flags);
}
static int merge_dispatch(crdt_ctx *ctx, Op op, u64 *self, const u64 *other, size_t N, size_t W, size_t self_stride,
                          size_t other_stride) {
  CRDT_CHECK_CTX(ctx);
  if (ctx->mem_kind == CRDT_MEM_HOST)
    return crdt::lattice_merge_batch_host(ctx, op, self, other, N, W, self_stride, other_stride);
  return crdt::lattice_merge_batch(ctx, op, self, other, N, W, self_stride, other_stride);
}

// crdt_lub_many_multi: the per-kind dims of each segment mapped to the lattice form
// (PNCounter rows hold 2A words; GCounter is VClock).
int crdt::lub_reqs_from_segments(crdt_ctx *ctx, const crdt_lub_segment *segs, size_t nseg,
                                 std::vector<crdt::LubReq> &reqs) {
  if (nseg && !segs) return crdt::fail(ctx, CRDT_EINVAL, "lub_many_multi: segs is NULL");
  reqs.resize(nseg);
  for (size_t i = 0; i < nseg; ++i) {
    const crdt_lub_segment &sg = segs[i];
    crdt::LubReq &q = reqs[i];
    switch (sg.kind) {
      case CRDT_KIND_VCLOCK:
      case CRDT_KIND_GCOUNTER: q.op = Op::Max; q.W = sg.A; break;
      case CRDT_KIND_PNCOUNTER: q.op = Op::Max; q.W = 2 * sg.A; break;
      case CRDT_KIND_GSET: q.op = Op::Or; q.W = sg.A; break;
      default: return crdt::fail(ctx, CRDT_EINVAL, "lub_many_multi: segment %zu has unknown kind %d", i, sg.kind);
    }
    q.in = (const u64 *)sg.in;
    q.G = sg.G;
    q.R = sg.R;
    q.row_stride = sg.row_stride;
    q.group_stride = sg.group_stride;
    q.out = (u64 *)sg.out;
    q.out_stride = sg.out_stride;
    q.flags = sg.flags;
  }
  return CRDT_OK;
}

extern "C" {

int crdt_vclock_lub_many(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                         size_t row_stride, size_t group_stride, uint64_t *out,
                         size_t out_stride, unsigned flags) {
  return lub_dispatch(ctx, Op::Max, (const u64 *)in, G, R, A, row_stride, group_stride,
                                (u64 *)out, out_stride, flags);
}
int crdt_vclock_merge_batch(crdt_ctx *ctx, uint64_t *self, const uint64_t *other, size_t N,
                            size_t A, size_t self_stride, size_t other_stride) {
  return merge_dispatch(ctx, Op::Max, (u64 *)self, (const u64 *)other, N, A,
                                   self_stride, other_stride);
}
int crdt_gcounter_lub_many(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                           size_t row_stride, size_t group_stride, uint64_t *out,
                           size_t out_stride, unsigned flags) {
  return crdt_vclock_lub_many(ctx, in, G, R, A, row_stride, group_stride, out, out_stride, flags);
}
int crdt_gcounter_merge_batch(crdt_ctx *ctx, uint64_t *self, const uint64_t *other, size_t N,
                              size_t A, size_t self_stride, size_t other_stride) {
  return crdt_vclock_merge_batch(ctx, self, other, N, A, self_stride, other_stride);
}
int crdt_pncounter_lub_many(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t A,
                            size_t row_stride, size_t group_stride, uint64_t *out,
                            size_t out_stride, unsigned flags) {
  return lub_dispatch(ctx, Op::Max, (const u64 *)in, G, R, 2 * A, row_stride,
                                group_stride, (u64 *)out, out_stride, flags);
}
int crdt_pncounter_merge_batch(crdt_ctx *ctx, uint64_t *self, const uint64_t *other,
                               size_t N, size_t A, size_t self_stride, size_t other_stride) {
  return merge_dispatch(ctx, Op::Max, (u64 *)self, (const u64 *)other, N, 2 * A,
                                   self_stride, other_stride);
}
int crdt_gset_lub_many(crdt_ctx *ctx, const uint64_t *in, size_t G, size_t R, size_t words,
                       size_t row_stride, size_t group_stride, uint64_t *out,
                       size_t out_stride, unsigned flags) {
  return lub_dispatch(ctx, Op::Or, (const u64 *)in, G, R, words, row_stride,
                                group_stride, (u64 *)out, out_stride, flags);
}
int crdt_gset_merge_batch(crdt_ctx *ctx, uint64_t *self, const uint64_t *other, size_t N,
                          size_t words, size_t self_stride, size_t other_stride) {
  return merge_dispatch(ctx, Op::Or, (u64 *)self, (const u64 *)other, N, words,
                                   self_stride, other_stride);
}

int crdt_lub_many_multi(crdt_ctx *ctx, const crdt_lub_segment *segs, size_t nseg) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  std::vector<crdt::LubReq> reqs;
  if (int rc = crdt::lub_reqs_from_segments(ctx, segs, nseg, reqs)) return rc;
  return crdt::lattice_lub_many_multi(ctx, reqs.data(), reqs.size());
}

}  // extern "C"
