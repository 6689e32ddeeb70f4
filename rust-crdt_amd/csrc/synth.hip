// Counter-based synthetic replica states, generated directly in HBM.
//
// Bench and parity inputs are far larger than what is worth shipping over PCIe (config 2 is
// 6 GiB), so they are generated on device from a stateless hash that the CPU restates
// bit-for-bit (oracle/oracle.py: synth_*; tests/golden/make_golden.py writes small fixtures).
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
  CRDT_DEVICE_MEM_ONLY(ctx);
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

// ---- Orswot replicas ----------------------------------------------------------------------
// Well-formed by construction (the invariants the dot-store join relies on: every dot (a, k)
// adds exactly one member, and every entry counter is <= the replica clock):
//   clock[r][a]      = synth(seed, r*A + a) % (kmax + 1)
//   actor a's k-th add targets member mem(a, k) = (a*P + k) mod M, so for member m the only
//   candidate event is k(m, a) = (m - a*P) mod M (kmax < M keeps it unique);
//   entries[r][m][a] = k(m, a) if 1 <= k(m, a) <= clock[r][a] and replica r has not observed a
//                      remove of that dot, else 0.  A quarter of the dots are removed (the dot's
//                      hash hd(m, a) & 3 == 0); the remove is observed by the replicas that have
//                      seen actor a advance past it: clock[r][a] >= k + 1 + ((hd >> 8) & 7).
//   So the fold keeps exactly the dots nobody has observed removed (a non-empty set), as a
//   remove that propagates with the actor's history would leave it.
namespace crdt {

constexpr u64 kOrswotP = 0x9E3779B1ULL;
constexpr u64 kObsSalt = 0xD1B54A32D192ED03ULL;

__global__ __launch_bounds__(kBlock) void synth_orswot_kernel(u64 *clock, u64 *entries,
                                                              unsigned long long R,
                                                              unsigned long long M,
                                                              unsigned long long A,
                                                              unsigned long long first_row,
                                                              u64 seed, u64 kmax, int which) {
  const unsigned long long nthreads = (unsigned long long)gridDim.x * blockDim.x;
  if (which == 0) {
    const unsigned long long total = R * A;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += nthreads)
      clock[i] = mix64(seed + (i + first_row * A + 1) * 0x9E3779B97F4A7C15ULL) % (kmax + 1);
    return;
  }
  const unsigned long long total = R * M * A;
  const u64 pm = kOrswotP % M;
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += nthreads) {
    const unsigned long long a = i % A;
    const unsigned long long rm = i / A;
    const unsigned long long m = rm % M;
    const unsigned long long r = rm / M;
    const unsigned long long gr = r + first_row;
    const u64 c = mix64(seed + (gr * A + a + 1) * 0x9E3779B97F4A7C15ULL) % (kmax + 1);
    const u64 k = (m + M - (a * pm) % M) % M;
    u64 e = (k >= 1 && k <= c) ? k : 0;
    const u64 hd = mix64(kObsSalt + (m * A + a));
    if (e && (hd & 3) == 0 && c >= k + 1 + ((hd >> 8) & 7)) e = 0;
    entries[i] = e;
  }
}

// forget(rm) on the listed members of each replica's own entries: what apply_rm
// (orswot.rs:230-238) leaves behind for a deferred remove the replica holds.
__global__ __launch_bounds__(kBlock) void synth_orswot_rm_kernel(u64 *entries, unsigned long long M,
                                                                 unsigned long long A,
                                                                 const unsigned *def_row,
                                                                 const u64 *def_clock,
                                                                 const u64 *def_members,
                                                                 unsigned long long Mw) {
  const unsigned long long d = blockIdx.x;
  const unsigned long long r = def_row[d];
  const u64 *rm = def_clock + d * A;
  const u64 *bits = def_members + d * Mw;
  for (unsigned long long w = 0; w < Mw; ++w) {
    u64 word = bits[w];
    while (word) {
      const int b = __builtin_ctzll(word);
      word &= word - 1;
      const unsigned long long m = w * 64 + b;
      if (m >= M) break;
      u64 *row = entries + (r * M + m) * A;
      for (unsigned long long a = threadIdx.x; a < A; a += kBlock)
        if (row[a] <= rm[a]) row[a] = 0;
    }
  }
}

}  // namespace crdt

extern "C" int crdt_synth_orswot(crdt_ctx *ctx, uint64_t *clock, uint64_t *entries, size_t R,
                                 size_t M, size_t A, size_t first_row, uint64_t seed,
                                 uint64_t kmax) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (R == 0 || M == 0 || A == 0) return CRDT_OK;
  if (!clock || !entries) return crdt::fail(ctx, CRDT_EINVAL, "synth_orswot: NULL output");
  if (kmax >= M) return crdt::fail(ctx, CRDT_EINVAL, "synth_orswot: kmax must be < M");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  const unsigned blocks = (unsigned)ctx->cu_count * 16;
  hipLaunchKernelGGL(crdt::synth_orswot_kernel, dim3(blocks), dim3(crdt::kBlock), 0, ctx->stream,
                     (crdt::u64 *)clock, (crdt::u64 *)entries, (unsigned long long)R,
                     (unsigned long long)M, (unsigned long long)A, (unsigned long long)first_row,
                     (crdt::u64)seed, (crdt::u64)kmax, 0);
  hipLaunchKernelGGL(crdt::synth_orswot_kernel, dim3(blocks), dim3(crdt::kBlock), 0, ctx->stream,
                     (crdt::u64 *)clock, (crdt::u64 *)entries, (unsigned long long)R,
                     (unsigned long long)M, (unsigned long long)A, (unsigned long long)first_row,
                     (crdt::u64)seed, (crdt::u64)kmax, 1);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

extern "C" int crdt_synth_orswot_rm(crdt_ctx *ctx, uint64_t *entries, size_t M, size_t A,
                                    size_t D, const uint32_t *def_row, const uint64_t *def_clock,
                                    const uint64_t *def_members) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (D == 0) return CRDT_OK;
  if (!entries || !def_row || !def_clock || !def_members)
    return crdt::fail(ctx, CRDT_EINVAL, "synth_orswot_rm: NULL buffer");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  hipLaunchKernelGGL(crdt::synth_orswot_rm_kernel, dim3((unsigned)D), dim3(crdt::kBlock), 0,
                     ctx->stream, (crdt::u64 *)entries, (unsigned long long)M,
                     (unsigned long long)A, (const unsigned *)def_row,
                     (const crdt::u64 *)def_clock, (const crdt::u64 *)def_members,
                     (unsigned long long)((M + 63) / 64));
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

// ---- Map<K, MVReg<u64>> replicas (BASELINE config 4) ----------------------------------------
// Restated bit-for-bit by oracle.synth_map / synth_map_deferred (model in their docstrings):
//   clock[r][a] = synth(seed, r*A + a) % (kmax + 1)  (ops 1..clock[r][a] of actor a seen)
//   key k is written by w0 = k % A and w1 = (k + 1) % A; actor a's n-th op targets the
//   ((n-1) mod M_a)-th of its keys (k % A == a in key order, then k % A == a-1), and is a
//   remove iff mix(seed ^ KIND, a << 32 | n) % 8 == 0, else an update with MVReg clock {a: n}
//   and value mix(seed ^ VAL, a << 32 | n).
//   Entry (r, k): per writer w (w0 then w1), w's latest op n <= clock[r][w] on k, if an update
//   whose dot survives the replica's own deferred removes naming k (n > max rm[w]):
//   ec[w] = n and the next value slot = ({w: n}, value).
namespace crdt {

constexpr u64 kSaltKind = 0xA5A5A5A55A5A5A5AULL;
constexpr u64 kSaltVal = 0x5EED5EED0B57AC1EULL;

__device__ __forceinline__ u64 key_count(u64 K, u64 A, u64 res) {
  return res < K ? (K - res + A - 1) / A : 0;
}

struct SynthMapPlan {
  u64 *clock, *ec, *vclk, *vval;
  unsigned long long R, K, A, V, first_row, kmax;
  u64 seed;
  const u64 *def_off;  // local replica CSR [R+1] or null
  const u64 *def_clock, *def_keys;
  unsigned long long Kw;
};

__device__ __forceinline__ u64 synth_map_c(const SynthMapPlan &p, u64 r, u64 a) {
  return mix64(p.seed + ((p.first_row + r) * p.A + a + 1) * 0x9E3779B97F4A7C15ULL) % (p.kmax + 1);
}

// Latest op n <= c of writer w on key k (0 if none).
__device__ __forceinline__ u64 synth_map_latest(const SynthMapPlan &p, u64 w, u64 k, u64 c) {
  u64 M, j;
  if (p.A == 1) {
    M = p.K;
    j = k;
  } else {
    const u64 P = key_count(p.K, p.A, w);
    M = P + key_count(p.K, p.A, (w + p.A - 1) % p.A);
    j = (k % p.A == w) ? k / p.A : P + k / p.A;
  }
  if (c < j + 1) return 0;
  return j + 1 + M * ((c - j - 1) / M);
}

__global__ __launch_bounds__(kBlock) void synth_map_kernel(SynthMapPlan p) {
  const unsigned long long total = p.R * p.K * p.A;
  const unsigned long long nthreads = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long idx = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += nthreads) {
    const u64 a = idx % p.A;
    const u64 rk = idx / p.A;
    const u64 k = rk % p.K;
    const u64 r = rk / p.K;
    if (k == 0) p.clock[r * p.A + a] = synth_map_c(p, r, a);
    const int nw = p.A == 1 ? 1 : 2;
    u64 wv[2], nv[2];
    bool live[2];
    for (int i = 0; i < nw; ++i) {
      const u64 w = (k + i) % p.A;
      const u64 n = synth_map_latest(p, w, k, synth_map_c(p, r, w));
      const bool upd = n > 0 && (mix64((p.seed ^ kSaltKind) + (w << 32) + n) & 7) != 0;
      u64 ceil = 0;
      if (p.def_off)
        for (u64 d = p.def_off[r]; d < p.def_off[r + 1]; ++d)
          if ((p.def_keys[d * p.Kw + k / 64] >> (k % 64)) & 1) {
            const u64 x = p.def_clock[d * p.A + w];
            ceil = x > ceil ? x : ceil;
          }
      wv[i] = w;
      nv[i] = n;
      live[i] = upd && n > ceil;
    }
    u64 e = 0;
    int slot = 0;
    u64 *vc = p.vclk + rk * p.V * p.A;
    u64 *vv = p.vval + rk * p.V;
    for (u64 s = 0; s < p.V; ++s) vc[s * p.A + a] = 0;
    for (int i = 0; i < nw; ++i) {
      if (!live[i]) continue;
      if (wv[i] == a) e = nv[i];
      if ((u64)slot < p.V) {
        if (wv[i] == a) vc[slot * p.A + a] = nv[i];
        if (a == 0) vv[slot] = mix64((p.seed ^ kSaltVal) + (wv[i] << 32) + nv[i]);
      }
      ++slot;
    }
    if (a == 0)
      for (u64 s = slot; s < p.V; ++s) vv[s] = 0;
    p.ec[rk * p.A + a] = e;
  }
}

}  // namespace crdt

extern "C" int crdt_synth_map(crdt_ctx *ctx, uint64_t *clock, uint64_t *ec, uint64_t *vclk,
                              uint64_t *vval, size_t R, size_t K, size_t A, size_t V,
                              size_t first_row, uint64_t seed, uint64_t kmax,
                              const uint64_t *def_off, const uint64_t *def_clock,
                              const uint64_t *def_keys) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (R == 0 || K == 0 || A == 0) return CRDT_OK;
  if (!clock || !ec || (V > 0 && (!vclk || !vval)))
    return crdt::fail(ctx, CRDT_EINVAL, "synth_map: NULL output");
  if (def_off && (!def_clock || !def_keys))
    return crdt::fail(ctx, CRDT_EINVAL, "synth_map: deferred buffers missing");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  crdt::SynthMapPlan p{};
  p.clock = (crdt::u64 *)clock;
  p.ec = (crdt::u64 *)ec;
  p.vclk = (crdt::u64 *)vclk;
  p.vval = (crdt::u64 *)vval;
  p.R = R;
  p.K = K;
  p.A = A;
  p.V = V;
  p.first_row = first_row;
  p.kmax = kmax;
  p.seed = seed;
  p.def_off = (const crdt::u64 *)def_off;
  p.def_clock = (const crdt::u64 *)def_clock;
  p.def_keys = (const crdt::u64 *)def_keys;
  p.Kw = (K + 63) / 64;
  const unsigned long long total = (unsigned long long)R * K * A;
  unsigned long long blocks = (total + crdt::kBlock - 1) / crdt::kBlock;
  const unsigned long long cap = (unsigned long long)ctx->cu_count * 16;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(crdt::synth_map_kernel, dim3((unsigned)blocks), dim3(crdt::kBlock), 0, ctx->stream, p);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}
