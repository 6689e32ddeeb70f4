// Batched CmRDT::apply of op streams to many dense states.
//
// Reference: VClock::apply (vclock.rs:125-127) -> apply_dot (vclock.rs:155-159): the counter of
// the dot's actor becomes max(own, dot.counter); GCounter::apply (gcounter.rs:39-41) is the same
// on `inner`; PNCounter::apply (pncounter.rs:62-67) applies the dot to P (Dir::Pos) or N
// (Dir::Neg); GSet::apply (gset.rs:46-48) inserts the element.  All of these are per-cell joins
// (max / set-bit), so ops commute: a batch is applied by one thread per op with a 64-bit
// atomic max (global_atomic_umax_x2) or atomic OR into the state row, in any order, exactly as
// applying the ops one by one in the reference.  Out-of-range ops are skipped and counted.
#include "common.hpp"

namespace crdt {

struct ApplyPlan {
  u64 *states;
  unsigned long long N, W, stride;  // W: row width in words (A, 2A for PNCounter, ceil(U/64) for GSet)
  const uint32_t *state_idx;
  const uint32_t *col;   // actor (VClock / GCounter / PNCounter) or element (GSet)
  const u64 *counter;    // dot counters (not GSet)
  const uint8_t *dir;    // PNCounter: 0 = Pos (P), 1 = Neg (N); nullptr otherwise
  unsigned long long n_ops, A;
  int kind;              // 0 max (vclock / gcounter / pncounter), 1 GSet bit
  unsigned *bad;         // count of skipped (out-of-range) ops, may be null
};

__global__ __launch_bounds__(kBlock) void apply_kernel(ApplyPlan p) {
  const unsigned long long i0 = blockIdx.x * (unsigned long long)kBlock + threadIdx.x;
  const unsigned long long step = (unsigned long long)gridDim.x * kBlock;
  unsigned nbad = 0;
  for (unsigned long long i = i0; i < p.n_ops; i += step) {
    const unsigned long long s = p.state_idx[i];
    const unsigned long long c = p.col[i];
    if (s >= p.N) {
      ++nbad;
      continue;
    }
    u64 *row = p.states + s * p.stride;
    if (p.kind == 1) {  // GSet insert: element c -> bit c of the bitmap row
      if (c >= p.A) {
        ++nbad;
        continue;
      }
      atomicOr(row + c / 64, 1ull << (c % 64));
    } else {
      if (c >= p.A) {
        ++nbad;
        continue;
      }
      const unsigned long long w = (p.dir && p.dir[i]) ? p.A + c : c;
      atomicMax(row + w, p.counter[i]);
    }
  }
  if (p.bad) {
    // one atomic per wave with anything to report
    const unsigned long long m = __ballot(nbad != 0);
    if (m) {
      unsigned tot = nbad;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) tot += __shfl_xor(tot, off, kWave);
      if ((threadIdx.x % kWave) == (unsigned)__builtin_ctzll(m)) atomicAdd(p.bad, tot);
    }
  }
}

static int apply_ops(crdt_ctx *ctx, int kind, bool pn, uint64_t *states, size_t N, size_t A, size_t stride,
                     const uint32_t *state_idx, const uint32_t *col, const uint64_t *counter, const uint8_t *dir,
                     size_t n_ops, uint32_t *bad) {
  CRDT_CHECK_CTX(ctx);
  if (n_ops == 0) return CRDT_OK;
  if (!states || !state_idx || !col || (kind == 0 && !counter) || (pn && !dir))
    return fail(ctx, CRDT_EINVAL, "apply: NULL buffer");
  const size_t W = kind == 1 ? (A + 63) / 64 : (pn ? 2 * A : A);
  if (stride < W) return fail(ctx, CRDT_EINVAL, "apply: row stride %zu < row width %zu", stride, W);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  ApplyPlan p{(u64 *)states, N, W, stride, state_idx, col, (const u64 *)counter, pn ? dir : nullptr,
              n_ops, A, kind, bad};
  const unsigned long long want = (n_ops + kBlock - 1) / kBlock;
  const unsigned long long cap = (unsigned long long)ctx->cu_count * 16;
  timing_begin(ctx, "apply");
  hipLaunchKernelGGL(apply_kernel, dim3((unsigned)(want < cap ? want : cap)), dim3(kBlock), 0, ctx->stream, p);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_vclock_apply_batch(crdt_ctx *ctx, uint64_t *states, size_t N, size_t A, size_t row_stride,
                                       const uint32_t *state_idx, const uint32_t *actor, const uint64_t *counter,
                                       size_t n_ops, uint32_t *bad) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return apply_ops(ctx, 0, false, states, N, A, row_stride, state_idx, actor, counter, nullptr, n_ops, bad);
}

extern "C" int crdt_gcounter_apply_batch(crdt_ctx *ctx, uint64_t *states, size_t N, size_t A, size_t row_stride,
                                         const uint32_t *state_idx, const uint32_t *actor, const uint64_t *counter,
                                         size_t n_ops, uint32_t *bad) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return apply_ops(ctx, 0, false, states, N, A, row_stride, state_idx, actor, counter, nullptr, n_ops, bad);
}

extern "C" int crdt_pncounter_apply_batch(crdt_ctx *ctx, uint64_t *states, size_t N, size_t A, size_t row_stride,
                                          const uint32_t *state_idx, const uint32_t *actor,
                                          const uint64_t *counter, const uint8_t *dir, size_t n_ops,
                                          uint32_t *bad) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return apply_ops(ctx, 0, true, states, N, A, row_stride, state_idx, actor, counter, dir, n_ops, bad);
}

extern "C" int crdt_gset_apply_batch(crdt_ctx *ctx, uint64_t *states, size_t N, size_t U, size_t row_stride,
                                     const uint32_t *state_idx, const uint32_t *element, size_t n_ops,
                                     uint32_t *bad) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return apply_ops(ctx, 1, false, states, N, U, row_stride, state_idx, element, nullptr, nullptr, n_ops, bad);
}
