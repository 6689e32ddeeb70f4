// Batched causal helpers on dense clock rows: VClock::glb,
// Causal::forget, VClock::partial_cmp (pairwise and all-pairs) and the GCounter / PNCounter
// read() sums.  All are HBM-bound elementwise / row-reduction passes (the all-pairs matrix is
// an LDS-tiled compare kernel), no MFMA.
//
// Reference: vclock.rs:68-80 (partial_cmp), :95-105 (forget), :246-259 (glb);
// gcounter.rs:51-53 (forget = inner.forget), :70-72 (read); pncounter.rs:78-81 (forget),
// :110-115 (read).  Dense convention: actor absent <=> 0 (vclock.rs:155-159 never stores 0), so
// glb's "drop zero minima" and forget's "remove the actor" are a 0 in the dense row.
#include "common.hpp"

namespace crdt {

// Row groups: a wave covers 64 / LR rows at once, LR lanes per row (a power of two, chosen so
// each lane moves ~8 pieces of its row: 16-byte pieces when every row starts 16-byte aligned
// and A is even, else words).  All of a lane's loads are independent, so they are in flight
// together; per-row reductions stay inside the LR-lane group (ballot bits / xor shuffles).
struct PairPlan {
  u64 *out;
  const u64 *x, *y;
  unsigned long long N, A, os, xs, ys;
  int op;  // CRDT_PAIR_GLB / CRDT_PAIR_FORGET / CRDT_PAIR_INTERSECTION
  int vec2;
  int lr_log;  // log2(LR)
};

__device__ __forceinline__ u64 pair_apply(int op, u64 a, u64 b) {
  // glb: min (vclock.rs:246-259); forget: keep a iff a > b (vclock.rs:98-104: counter >= own
  // removes the actor); intersection: keep a iff b holds the same counter (vclock.rs:218-227; an
  // absent actor is 0 on both sides, so it stays absent)
  if (op == CRDT_PAIR_GLB) return a < b ? a : b;
  if (op == CRDT_PAIR_FORGET) return a > b ? a : 0;
  return a == b ? a : 0;
}

__global__ __launch_bounds__(kBlock) void pair_op_kernel(PairPlan p) {
  ROW_GROUP_LOOP(p.N, p.lr_log) {
    const unsigned long long r = rb + (lane >> p.lr_log);
    if (r >= p.N) continue;
    const u64 *xr = p.x + r * p.xs, *yr = p.y + r * p.ys;
    u64 *orow = p.out + r * p.os;
    if (p.vec2) {
#pragma unroll 8
      for (unsigned long long c = 2ull * gl; c < p.A; c += 2ull * LR) {
        const u64x2 a = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(xr + c));
        const u64x2 b = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(yr + c));
        u64x2 o;
        o.x = pair_apply(p.op, a.x, b.x);
        o.y = pair_apply(p.op, a.y, b.y);
        __builtin_nontemporal_store(o, reinterpret_cast<u64x2 *>(orow + c));
      }
    } else {
#pragma unroll 8
      for (unsigned long long c = gl; c < p.A; c += LR) orow[c] = pair_apply(p.op, xr[c], yr[c]);
    }
  }
}

// Bits of the LR-lane groups of a wave: bit g*LR set iff every bit of group g is set in m.
__device__ __forceinline__ u64 group_all(u64 m, int lr_log) {
  for (int sh = 1; sh < (1 << lr_log); sh <<= 1) m &= m >> sh;
  return m;
}

// partial_cmp of row pairs: Equal 0, Greater 1, Less -1, None 2 (vclock.rs:69-80: equal first,
// then "every counter of other <= self's" = Greater, then the mirror = Less).
__global__ __launch_bounds__(kBlock) void pair_cmp_kernel(PairPlan p, int8_t *res) {
  ROW_GROUP_LOOP(p.N, p.lr_log) {
    const unsigned long long r = rb + (lane >> p.lr_log);
    const bool on = r < p.N;
    const unsigned long long rr = on ? r : p.N - 1;
    const u64 *xr = p.x + rr * p.xs, *yr = p.y + rr * p.ys;
    bool ge = true, le = true;
    if (p.vec2) {
#pragma unroll 8
      for (unsigned long long c = 2ull * gl; c < p.A; c += 2ull * LR) {
        const u64x2 a = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(xr + c));
        const u64x2 b = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(yr + c));
        ge &= (a.x >= b.x) & (a.y >= b.y);
        le &= (a.x <= b.x) & (a.y <= b.y);
      }
    } else {
#pragma unroll 8
      for (unsigned long long c = gl; c < p.A; c += LR) {
        ge &= xr[c] >= yr[c];
        le &= xr[c] <= yr[c];
      }
    }
    const u64 G = group_all(__ballot(ge), p.lr_log), L = group_all(__ballot(le), p.lr_log);
    if (on && gl == 0) {
      const bool g = (G >> lane) & 1, l = (L >> lane) & 1;
      res[r] = (int8_t)(g && l ? 0 : (g ? 1 : (l ? -1 : 2)));
    }
  }
}

// All-pairs partial_cmp matrix of N clocks: res[i*N + j] = partial_cmp(x_i, x_j).  A 64x64 tile
// of pairs per workgroup; both 64-clock blocks are staged through LDS 32 actors at a time
// (actor-major, padded), each thread owns 16 pairs (one i, 16 j) and accumulates the
// "all >=" / "all <=" bits over the actor chunks.
constexpr int kCmpT = 64;   // clocks per tile side
constexpr int kCmpK = 32;   // actors per LDS stage
__global__ __launch_bounds__(kBlock) void cmp_matrix_kernel(const u64 *x, unsigned long long N,
                                                            unsigned long long A, unsigned long long xs,
                                                            int8_t *res) {
  __shared__ u64 ti[kCmpK][kCmpT + 1];
  __shared__ u64 tj[kCmpK][kCmpT + 1];
  const unsigned long long i0 = (unsigned long long)blockIdx.y * kCmpT;
  const unsigned long long j0 = (unsigned long long)blockIdx.x * kCmpT;
  const int t = threadIdx.x;
  const int ii = t % kCmpT;          // this thread's i within the tile
  const int jb = (t / kCmpT) * 16;   // its 16 j's
  unsigned ge = 0xffffu, le = 0xffffu;  // bit q: pair (ii, jb + q)
  for (unsigned long long a0 = 0; a0 < A; a0 += kCmpK) {
    // stage: 64 clocks x 32 actors per block, 8 words per thread per block
    for (int e = t; e < kCmpT * kCmpK; e += kBlock) {
      const int c = e / kCmpK, k = e % kCmpK;  // consecutive threads walk one clock's actors
      const unsigned long long a = a0 + k;
      const unsigned long long gi = i0 + c, gj = j0 + c;
      ti[k][c] = (gi < N && a < A) ? x[gi * xs + a] : 0;
      tj[k][c] = (gj < N && a < A) ? x[gj * xs + a] : 0;
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < kCmpK; ++k) {
      const u64 vi = ti[k][ii];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const u64 vj = tj[k][jb + q];
        ge &= ~((unsigned)(vi < vj) << q);
        le &= ~((unsigned)(vi > vj) << q);
      }
    }
    __syncthreads();
  }
  const unsigned long long gi = i0 + ii;
  if (gi >= N) return;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const unsigned long long gj = j0 + jb + q;
    if (gj < N) {
      const bool G = (ge >> q) & 1, L = (le >> q) & 1;
      res[gi * N + gj] = (int8_t)(G && L ? 0 : (G ? 1 : (L ? -1 : 2)));
    }
  }
}

// 128-bit exact row sums (GCounter::read, BigUint sum of u64 counters; A < 2^64 terms fit in
// 128 bits).  PNCounter: P - N of the row's two halves as a two's-complement 128-bit integer
// (|sum| < 2^126 for A < 2^62).  One wave per row: per-lane (lo, hi) accumulators, then a
// butterfly reduction with carries.
struct ReadPlan {
  const u64 *in;
  unsigned long long N, A, rs;
  int pn;  // 0: GCounter (A words), 1: PNCounter (P in [0, A), N in [A, 2A))
  u64 *out;  // [N][2] (lo, hi)
  int vec2;
  int lr_log;
};

__device__ __forceinline__ void add128(u64 &lo, u64 &hi, u64 blo, u64 bhi) {
  const u64 l = lo + blo;
  hi += bhi + (l < lo ? 1 : 0);
  lo = l;
}

// Sum over the aligned LR-lane group of each lane (xor offsets < LR stay inside the group).
__device__ __forceinline__ void group_sum128(u64 &lo, u64 &hi, int LR) {
  for (int off = LR >> 1; off >= 1; off >>= 1) {
    const u64 olo = __shfl_xor(lo, off, kWave);
    const u64 ohi = __shfl_xor(hi, off, kWave);
    add128(lo, hi, olo, ohi);
  }
}

__global__ __launch_bounds__(kBlock) void read_sum_kernel(ReadPlan p) {
  ROW_GROUP_LOOP(p.N, p.lr_log) {
    const unsigned long long r = rb + (lane >> p.lr_log);
    const bool on = r < p.N;
    const u64 *row = p.in + (on ? r : p.N - 1) * p.rs;
    u64 plo = 0, phi = 0, nlo = 0, nhi = 0;
    if (p.vec2) {  // 16-byte loads
#pragma unroll 8
      for (unsigned long long c = 2ull * gl; c < p.A; c += 2ull * LR) {
        const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(row + c));
        add128(plo, phi, v.x, 0);
        add128(plo, phi, v.y, 0);
      }
      if (p.pn) {
#pragma unroll 8
        for (unsigned long long c = 2ull * gl; c < p.A; c += 2ull * LR) {
          const u64x2 w = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(row + p.A + c));
          add128(nlo, nhi, w.x, 0);
          add128(nlo, nhi, w.y, 0);
        }
      }
    } else {
#pragma unroll 8
      for (unsigned long long c = gl; c < p.A; c += LR) {
        add128(plo, phi, __builtin_nontemporal_load(row + c), 0);
        if (p.pn) add128(nlo, nhi, __builtin_nontemporal_load(row + p.A + c), 0);
      }
    }
    group_sum128(plo, phi, LR);
    if (p.pn) {
      group_sum128(nlo, nhi, LR);
      // P - N = P + ~N + 1
      add128(plo, phi, ~nlo, ~nhi);
      add128(plo, phi, 1, 0);
    }
    if (on && gl == 0) {
      p.out[2 * r] = plo;
      p.out[2 * r + 1] = phi;
    }
  }
}

// Workgroups per CU measured on MI355X at 1M rows x 256 (scripts/bench_causal.py, CRDT_TUNE=rbpc):
// two-read-one-write passes prefer few (2: 72% vs 16: 69%), partial_cmp 4 (84%), read many (32: 79%).
constexpr int kRbpcPair = 2, kRbpcCmp = 4, kRbpcRead = 32;

static unsigned rows_grid(const crdt_ctx *ctx, unsigned long long N, int lr_log, int bpc) {
  // 64 / LR rows per wave, 4 waves per workgroup; enough workgroups to fill the chip
  // (tune rows_wpc: workgroups per CU)
  const unsigned long long rpb = 4ull * (kWave >> lr_log);
  const unsigned long long want = (N + rpb - 1) / rpb;
  const unsigned long long cap =
      (unsigned long long)ctx->cu_count * (ctx->tune.rows_blocks_per_cu > 0 ? ctx->tune.rows_blocks_per_cu : bpc);
  return (unsigned)(want < cap ? (want ? want : 1) : cap);
}

static bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_vclock_pair_op(crdt_ctx *ctx, int op, uint64_t *out, const uint64_t *x, const uint64_t *y,
                                   size_t N, size_t A, size_t out_stride, size_t x_stride, size_t y_stride) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (op != CRDT_PAIR_GLB && op != CRDT_PAIR_FORGET && op != CRDT_PAIR_INTERSECTION) return fail(ctx, CRDT_EINVAL, "vclock_pair_op: op %d", op);
  if (N == 0 || A == 0) return CRDT_OK;
  if (!out || !x || !y) return fail(ctx, CRDT_EINVAL, "vclock_pair_op: NULL buffer");
  if (N > 1 && (out_stride < A || x_stride < A || y_stride < A)) return fail(ctx, CRDT_EINVAL, "vclock_pair_op: stride < A");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  PairPlan p{(u64 *)out, (const u64 *)x, (const u64 *)y, N, A, out_stride, x_stride, y_stride, op, 0};
  p.vec2 = (A % 2 == 0) && ((out_stride | x_stride | y_stride) % 2 == 0) && al16(out) && al16(x) && al16(y);
  p.lr_log = row_lr_log(p.vec2 ? A / 2 : A);
  timing_begin(ctx, "pair_op");
  hipLaunchKernelGGL(pair_op_kernel, dim3(rows_grid(ctx, N, p.lr_log, kRbpcPair)), dim3(kBlock), 0, ctx->stream, p);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

extern "C" int crdt_vclock_partial_cmp(crdt_ctx *ctx, const uint64_t *x, const uint64_t *y, size_t N, size_t A,
                                       size_t x_stride, size_t y_stride, int8_t *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (N == 0) return CRDT_OK;
  if (!out || (A > 0 && (!x || !y))) return fail(ctx, CRDT_EINVAL, "vclock_partial_cmp: NULL buffer");
  if (N > 1 && A > 0 && (x_stride < A || y_stride < A)) return fail(ctx, CRDT_EINVAL, "vclock_partial_cmp: stride < A");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  PairPlan p{nullptr, (const u64 *)x, (const u64 *)y, N, A, 0, x_stride, y_stride, 0, 0};
  p.vec2 = (A % 2 == 0) && ((x_stride | y_stride) % 2 == 0) && al16(x) && al16(y);
  p.lr_log = row_lr_log(p.vec2 ? A / 2 : A);
  timing_begin(ctx, "pair_cmp");
  hipLaunchKernelGGL(pair_cmp_kernel, dim3(rows_grid(ctx, N, p.lr_log, kRbpcCmp)), dim3(kBlock), 0, ctx->stream, p, out);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

extern "C" int crdt_vclock_cmp_matrix(crdt_ctx *ctx, const uint64_t *x, size_t N, size_t A, size_t x_stride,
                                      int8_t *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (N == 0) return CRDT_OK;
  if (!out || (A > 0 && !x)) return fail(ctx, CRDT_EINVAL, "vclock_cmp_matrix: NULL buffer");
  if (A > 0 && x_stride < A) return fail(ctx, CRDT_EINVAL, "vclock_cmp_matrix: stride < A");
  const unsigned long long tiles = (N + kCmpT - 1) / kCmpT;
  if (tiles > 65535) return fail(ctx, CRDT_EUNSUPPORTED, "vclock_cmp_matrix: N = %zu too large", N);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  timing_begin(ctx, "cmp_matrix");
  hipLaunchKernelGGL(cmp_matrix_kernel, dim3((unsigned)tiles, (unsigned)tiles), dim3(kBlock), 0, ctx->stream,
                     (const u64 *)x, (unsigned long long)N, (unsigned long long)A, (unsigned long long)x_stride,
                     out);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

static int read_rows(crdt_ctx *ctx, int pn, const uint64_t *in, size_t N, size_t A, size_t stride, uint64_t *out) {
  CRDT_CHECK_CTX(ctx);
  if (N == 0) return CRDT_OK;
  if (!out || (A > 0 && !in)) return fail(ctx, CRDT_EINVAL, "read: NULL buffer");
  if (N > 1 && A > 0 && stride < (pn ? 2 : 1) * A) return fail(ctx, CRDT_EINVAL, "read: row stride too small");
  if (A >= (1ull << 62)) return fail(ctx, CRDT_EUNSUPPORTED, "read: A too large for 128-bit sums");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  ReadPlan p{(const u64 *)in, N, A, stride, pn, (u64 *)out, 0, 0};
  p.vec2 = (A % 2 == 0) && (stride % 2 == 0) && al16(in);
  p.lr_log = row_lr_log(p.vec2 ? A / 2 : A);
  timing_begin(ctx, "read_sum");
  hipLaunchKernelGGL(read_sum_kernel, dim3(rows_grid(ctx, N, p.lr_log, kRbpcRead)), dim3(kBlock), 0, ctx->stream, p);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

extern "C" int crdt_gcounter_read(crdt_ctx *ctx, const uint64_t *in, size_t N, size_t A, size_t row_stride,
                                  uint64_t *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return read_rows(ctx, 0, in, N, A, row_stride, out);
}

extern "C" int crdt_pncounter_read(crdt_ctx *ctx, const uint64_t *in, size_t N, size_t A, size_t row_stride,
                                   uint64_t *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return read_rows(ctx, 1, in, N, A, row_stride, out);
}
