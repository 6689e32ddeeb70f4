// Lane groups for the ordered apply kernels: 16 lanes (one DPP row) run one state's op stream, 4
// states per wave.  Lane g of a group holds actors a = g + 16j, j < KJ (A <= 16 KJ), so a clock row
// is KJ registers per lane and a row access moves 128 contiguous bytes per group.  All control
// flow that feeds these helpers is group-uniform: votes are ballots masked to the group, the
// minimum is four DPP moves inside the row.
#pragma once
#include "common.hpp"

namespace crdt {
namespace grp {

constexpr int kG = 16;
constexpr unsigned kMask = 0xFFFFu;
constexpr unsigned kNone = 0xFFu;  // no actor (a witness value)

__device__ __forceinline__ unsigned bits(u64 ballot, int lane) { return (unsigned)(ballot >> (lane & ~(kG - 1))) & kMask; }
__device__ __forceinline__ bool any(bool x, int lane) { return bits(__ballot(x), lane) != 0; }
__device__ __forceinline__ bool all(bool x, int lane) { return bits(__ballot(x), lane) == kMask; }

// min over the 16 lanes of the row: xor 1, xor 2 (quad_perm), then the mirrors within 8 and 16
// lanes pair every lane with one of the other half (VALU moves, no LDS round trip)
__device__ __forceinline__ unsigned min(unsigned x) {
  unsigned y = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  x = y < x ? y : x;
  y = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  x = y < x ? y : x;
  y = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
  x = y < x ? y : x;
  y = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);  // row_mirror
  return y < x ? y : x;
}
__device__ __forceinline__ u64 orx(u64 x) {
#pragma unroll
  for (int o = 1; o < kG; o <<= 1) x |= __shfl_xor(x, o);
  return x;
}

template <int KJ>
__device__ __forceinline__ void load_row(u64 (&x)[KJ], const u64 *row, int g, unsigned long long A) {
#pragma unroll
  for (int j = 0; j < KJ; ++j) {
    const unsigned a = g + kG * j;
    x[j] = a < A ? row[a] : 0;
  }
}
template <int KJ>
__device__ __forceinline__ void store_row(u64 *row, const u64 (&x)[KJ], int g, unsigned long long A) {
#pragma unroll
  for (int j = 0; j < KJ; ++j) {
    const unsigned a = g + kG * j;
    if (a < A) row[a] = x[j];
  }
}
template <int KJ>
__device__ __forceinline__ bool any_nz(const u64 (&x)[KJ], int lane) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < KJ; ++j) b |= x[j] != 0;
  return any(b, lane);
}
// x <= y on every actor (padding words are 0 on both sides)
template <int KJ>
__device__ __forceinline__ bool all_le(const u64 (&x)[KJ], const u64 (&y)[KJ], int lane) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < KJ; ++j) b |= x[j] > y[j];
  return !any(b, lane);
}
template <int KJ>
__device__ __forceinline__ bool rows_eq(const u64 (&x)[KJ], const u64 (&y)[KJ], int lane) {
  bool b = false;
#pragma unroll
  for (int j = 0; j < KJ; ++j) b |= x[j] != y[j];
  return !any(b, lane);
}

// The group's first actor a >= from with x[a] > c[a] (kNone if none).
template <int KJ>
__device__ __forceinline__ unsigned witness(const u64 (&x)[KJ], const u64 (&c)[KJ], int g, unsigned from,
                                            unsigned long long A) {
  unsigned f = kNone;
#pragma unroll
  for (int j = KJ - 1; j >= 0; --j) {
    const unsigned a = g + kG * j;
    if (a < A && a >= from && x[j] > c[j]) f = a;
  }
  return min(f);
}

// c[a] of the clock held by the group (owner lane a % 16, register a / 16), in every lane
template <int KJ>
__device__ __forceinline__ u64 clock_at(const u64 (&c)[KJ], unsigned a, int lane) {
  u64 mine = c[0];
#pragma unroll
  for (int j = 1; j < KJ; ++j)
    if ((unsigned)j == a / kG) mine = c[j];
  return __shfl(mine, (lane & ~(kG - 1)) | (int)(a % kG));
}
template <int KJ>
__device__ __forceinline__ void clock_set(u64 (&c)[KJ], unsigned a, u64 v, int g) {
  if ((unsigned)g == a % kG) {
#pragma unroll
    for (int j = 0; j < KJ; ++j)
      if ((unsigned)j == a / kG) c[j] = v;
  }
}

}  // namespace grp
}  // namespace crdt
