// Shared pieces of the serde wire kernels (wire.hip: the reference types and Map<K, MVReg>;
// wire_vmap.hip: the value-typed Maps): frame access, dictionary lookups, VClock parse / write.
// The encoding (bincode 1.x, default options) is restated at the top of wire.hip.
#pragma once
#include "common.hpp"

namespace crdt {

constexpr int kScanItems = 1024;  // items per block of the exclusive scan (wire.hip)

constexpr unsigned kWireBad = 1u, kWireMissing = 2u, kWireCap = 4u;
constexpr int kWireRowLds = 4096;  // u64 words of the LDS row per wave (A or bitmap words)

struct Frame {
  const uint32_t *w;  // 4-aligned base
  unsigned long long nw;  // words in the frame
};

__device__ __forceinline__ u64 rd64(const uint32_t *w, unsigned long long k) {
  return (u64)w[k] | ((u64)w[k + 1] << 32);
}

__device__ __forceinline__ long long find_u32(const uint32_t *dict, unsigned long long n, uint32_t id,
                                              unsigned long long hint) {
  if (hint < n && dict[hint] == id) return (long long)hint;  // the dense, in-order case
  unsigned long long lo = 0, hi = n;
  while (lo < hi) {
    const unsigned long long mid = (lo + hi) / 2;
    if (dict[mid] < id) lo = mid + 1;
    else hi = mid;
  }
  return (lo < n && dict[lo] == id) ? (long long)lo : -1;
}
__device__ __forceinline__ long long find_u64(const u64 *dict, unsigned long long n, u64 id, unsigned long long hint) {
  if (hint < n && dict[hint] == id) return (long long)hint;
  unsigned long long lo = 0, hi = n;
  while (lo < hi) {
    const unsigned long long mid = (lo + hi) / 2;
    if (dict[mid] < id) lo = mid + 1;
    else hi = mid;
  }
  return (lo < n && dict[lo] == id) ? (long long)lo : -1;
}

__device__ __forceinline__ void wfence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup"); }

// Parse the VClock at word k of frame f into the LDS row (A u64, zeroed here); returns the word
// after it (or ~0 on a truncated clock).  st |= kWireMissing for an actor not in the dictionary.
__device__ inline unsigned long long parse_vclock(const Frame &f, unsigned long long k, const uint32_t *actors,
                                           unsigned long long A, u64 *row, int lane, unsigned &st) {
  for (unsigned long long a = lane; a < A; a += kWave) row[a] = 0;
  wfence();
  if (k + 2 > f.nw) {
    st |= kWireBad;
    return ~0ull;
  }
  const u64 n = rd64(f.w, k);
  if (n > (f.nw - k - 2) / 3) {
    st |= kWireBad;
    return ~0ull;
  }
  const uint32_t *rec = f.w + k + 2;
  bool miss = false;
  for (unsigned long long i = lane; i < n; i += kWave) {
    const uint32_t id = rec[3 * i];
    const u64 cnt = rd64(rec, 3 * i + 1);
    const long long col = find_u32(actors, A, id, i);
    if (col < 0) miss = true;
    else row[col] = cnt;
  }
  if (__ballot(miss)) st |= kWireMissing;
  wfence();
  return k + 2 + 3 * n;
}

template <typename T>
__device__ __forceinline__ void store_row(u64 *dst, const u64 *row, unsigned long long W, int lane) {
  for (unsigned long long a = lane; a < W; a += kWave) dst[a] = row[a];
}

// nonzero words of a row: one ballot per 64 words (no shuffle-reduction chain; the count is uniform)
__device__ __forceinline__ u64 nnz_row(const u64 *r, unsigned long long A, int lane) {
  unsigned long long c = 0;
  for (unsigned long long a0 = 0; a0 < A; a0 += kWave) {
    const unsigned long long a = a0 + lane;
    c += __popcll(__ballot(a < A && r[a] != 0));
  }
  return c;
}
__device__ __forceinline__ u64 popc_row(const u64 *r, unsigned long long W, int lane) {
  unsigned long long c = 0;
  for (unsigned long long w = lane; w < W; w += kWave) c += __popcll(r[w]);
  for (int off = kWave / 2; off > 0; off >>= 1) c += __shfl_xor(c, off, kWave);
  return c;
}
__device__ __forceinline__ void wr64(uint32_t *w, unsigned long long k, u64 v) {
  w[k] = (uint32_t)v;
  w[k + 1] = (uint32_t)(v >> 32);
}

// Write a dense row as a VClock at word k (len, then (actor, counter) ascending); returns the
// next word.  Lanes take columns; a wave prefix count gives every nonzero its record slot.
__device__ inline unsigned long long write_vclock(uint32_t *w, unsigned long long k, const u64 *r, unsigned long long A,
                                           const uint32_t *actors, int lane) {
  const u64 n = nnz_row(r, A, lane);
  if (lane == 0) wr64(w, k, n);
  unsigned long long base = 0;
  for (unsigned long long a0 = 0; a0 < A; a0 += kWave) {
    const unsigned long long a = a0 + lane;
    const u64 v = a < A ? r[a] : 0;
    const u64 m = __ballot(v != 0);
    if (v != 0) {
      const unsigned long long i = base + __popcll(m & ((1ull << lane) - 1));
      w[k + 2 + 3 * i] = actors[a];
      wr64(w, k + 3 + 3 * i, v);
    }
    base += __popcll(m);
  }
  return k + 2 + 3 * n;
}

inline unsigned wave_grid(crdt_ctx *ctx, unsigned long long waves, int wpb, int per_cu) {
  const unsigned long long want = (waves + wpb - 1) / wpb;
  const unsigned long long cap = (unsigned long long)ctx->cu_count * per_cu;
  return (unsigned)(want == 0 ? 1 : (want < cap ? want : cap));
}

// frame sizes -> frame_off (device, N+1) -> *total (wire.hip; launches the scan kernels)
int egress_layout(crdt_ctx *ctx, u64 *sizes, u64 *frame_off, unsigned long long N, size_t *total);

inline int wire_scratch(crdt_ctx *ctx, unsigned long long N, u64 **sizes) {
  const unsigned long long nb = (N + kScanItems - 1) / kScanItems + 2;
  int rc = ensure_scratch(ctx, (N + nb + 8) * 8);
  if (rc) return rc;
  *sizes = reinterpret_cast<u64 *>(ctx->scratch);
  return CRDT_OK;
}

inline int check_frames(crdt_ctx *ctx, const void *bytes, const uint64_t *frame_off, size_t N, uint32_t *status) {
  if (N && (!frame_off || !status)) return fail(ctx, CRDT_EINVAL, "ingest: NULL frame_off / status");
  (void)bytes;
  return CRDT_OK;
}

}  // namespace crdt
