// Counter-based synthetic replica states, generated directly in HBM.
//
// Bench and parity inputs are far larger than what is worth shipping over PCIe (config 2 is
// 6 GiB), so they are generated on device from a stateless hash that the CPU restates
// bit-for-bit (tests/golden/make_golden.py, oracle/oracle.py: synth_*).
//   h(seed, idx) = splitmix64 finaliser of (seed + (idx + 1) * 0x9E3779B97F4A7C15)
//   kind 0, counters : (h & 3) == 0 -> 0 (actor absent, 1/4);  ((h >> 2) & 63) == 0 -> h
//                      (full-range u64, 3/256);  else h >> 16 (48-bit)
//   kind 1, GSet     : h & mix(h ^ K1)          (~25% of bits set)
//   kind 2, LWW mark : ((h >> 58) == 0) ? 0xFFFFFFFFFFFF (shared top marker, 1/64) : h >> 20
//   kind 3, LWW val  : (h & 1) ? 42 : mix(h ^ K2)
#include "common.hpp"

namespace crdt {

__host__ __device__ __forceinline__ u64 mix64(u64 z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ u64 synth_value(u64 seed, u64 idx, int kind) {
  const u64 h = mix64(seed + (idx + 1) * 0x9E3779B97F4A7C15ULL);
  switch (kind) {
    case 0:
      if ((h & 3) == 0) return 0;
      if (((h >> 2) & 63) == 0) return h;
      return h >> 16;
    case 1:
      return h & mix64(h ^ 0x5851F42D4C957F2DULL);
    case 2:
      return (h >> 58) == 0 ? 0xFFFFFFFFFFFFULL : (h >> 20);
    default:
      return (h & 1) ? 42ULL : mix64(h ^ 0x14057B7EF767814FULL);
  }
}

__global__ __launch_bounds__(kBlock) void synth_fill_kernel(u64 *out, unsigned long long rows,
                                                            unsigned long long width,
                                                            unsigned long long row_stride,
                                                            unsigned long long first_row, u64 seed,
                                                            int kind) {
  const unsigned long long total = rows * width;
  const unsigned long long nthreads = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += nthreads) {
    const unsigned long long r = i / width;
    const unsigned long long c = i - r * width;
    out[r * row_stride + c] = synth_value(seed, i + first_row * width, kind);
  }
}

}  // namespace crdt

extern "C" int crdt_synth_fill(crdt_ctx *ctx, uint64_t *out, size_t rows, size_t width,
                               size_t row_stride, size_t first_row, uint64_t seed, int kind) {
  CRDT_CHECK_CTX(ctx);
  if (rows == 0 || width == 0) return CRDT_OK;
  if (!out) return crdt::fail(ctx, CRDT_EINVAL, "synth_fill: out is NULL");
  if (rows > 1 && row_stride < width)
    return crdt::fail(ctx, CRDT_EINVAL, "synth_fill: row_stride < width");
  if (kind < 0 || kind > 3) return crdt::fail(ctx, CRDT_EINVAL, "synth_fill: bad kind %d", kind);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const unsigned long long total = (unsigned long long)rows * width;
  unsigned long long blocks = (total + crdt::kBlock - 1) / crdt::kBlock;
  const unsigned long long cap = (unsigned long long)ctx->cu_count * 16;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(crdt::synth_fill_kernel, dim3((unsigned)blocks), dim3(crdt::kBlock), 0,
                     ctx->stream, (crdt::u64 *)out, (unsigned long long)rows,
                     (unsigned long long)width, (unsigned long long)row_stride,
                     (unsigned long long)first_row, (crdt::u64)seed,
                     kind);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}
