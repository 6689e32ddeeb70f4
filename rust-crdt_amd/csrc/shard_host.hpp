// Host-side bookkeeping of the sharded entry points (csrc/shard.hip), kept free of HIP so the
// CPU suite compiles it with g++ -fsanitize=address,undefined and unit-tests it
// (tests/cpp/test_shard_host.cpp, run by tests/test_sanitizers.py).  Pure functions of the
// gathered exchange data; every rank calls them on the same data and takes the same branches.
#pragma once

#include <cstddef>
#include <cstdint>
#include <initializer_list>
#include <vector>

namespace crdt {
namespace shard_host {

// Agreement header of one rank: [failed, tag, d0..d4, hash(all dims)].
constexpr int kHdr = 8;
struct Hdr {
  uint64_t w[kHdr];
};

inline Hdr make_hdr(bool failed, uint64_t tag, std::initializer_list<uint64_t> dims) {
  Hdr h{};
  h.w[0] = failed ? 1 : 0;
  h.w[1] = tag;
  uint64_t hash = 0xcbf29ce484222325ull;  // FNV-1a over every byte of every dim
  uint64_t i = 0;
  for (uint64_t d : dims) {
    if (i < (uint64_t)(kHdr - 3)) h.w[2 + i] = d;
    ++i;
    for (int b = 0; b < 8; ++b) hash = (hash ^ ((d >> (8 * b)) & 0xff)) * 0x100000001b3ull;
  }
  h.w[kHdr - 1] = hash ^ i;
  return h;
}

// The gathered headers rows[W][kHdr] against this rank's: *failed_rank = the first rank that
// failed validation (-1 if none), *mismatch_rank = the first rank whose tag / dims differ from
// `mine` (-1 if none).  Returns true iff both are -1 (the data collectives may run).
inline bool check_headers(const uint64_t *rows, size_t W, const Hdr &mine, long *failed_rank, long *mismatch_rank) {
  *failed_rank = -1;
  *mismatch_rank = -1;
  for (size_t r = 0; r < W && *failed_rank < 0; ++r)
    if (rows[r * kHdr]) *failed_rank = (long)r;
  for (size_t r = 0; r < W && *mismatch_rank < 0; ++r)
    for (int k = 1; k < kHdr; ++k)
      if (rows[r * kHdr + k] != mine.w[k]) {
        *mismatch_rank = (long)r;
        break;
      }
  return *failed_rank < 0 && *mismatch_rank < 0;
}

// Agreed plans (round 6).  A plan is an entry point with its dims: the key of a header hashes its tag
// and dims hash.  Once the ranks agreed a plan (the header all-gather above found every rank valid
// and equal), later calls with that plan skip the header exchange: they all-reduce (MAX) three check
// words [failed, key, ~key] beside their data instead, and every rank verifies the reduced words at
// its next sharded call (or crdt_ctx_synchronize).  All ranks see the same reduced words, so all reach
// the same verdict at the same call: any rank failed, or ranks sent different keys (max(key) == key
// and max(~key) == ~key on a rank only if every rank sent that key).
inline uint64_t plan_key(const Hdr &h) { return (h.w[1] * 0x9E3779B97F4A7C15ull) ^ h.w[kHdr - 1]; }

struct PlanCache {
  static constexpr int kCap = 16;
  uint64_t key[kCap] = {};
  int n = 0;
  bool has(uint64_t k) const {
    for (int i = 0; i < n; ++i)
      if (key[i] == k) return true;
    return false;
  }
  void add(uint64_t k) {
    if (has(k)) return;
    if (n == kCap) {  // oldest out
      for (int i = 1; i < kCap; ++i) key[i - 1] = key[i];
      --n;
    }
    key[n++] = k;
  }
  void clear() { n = 0; }
};

inline void check_words(bool failed, uint64_t key, uint64_t *w) {
  w[0] = failed ? 1 : 0;
  w[1] = key;
  w[2] = ~key;
}
inline bool check_ok(const uint64_t *reduced, uint64_t key) {
  return reduced[0] == 0 && reduced[1] == key && reduced[2] == ~key;
}

// Orswot deferred regrouping: cnt[W][G+1] are the gathered per-group counts (entry G = the rank's
// total), the all-gathered rows sit rank-major with rank r's rows of group g at
// r*Dmax + (r's rows of the groups before g) + j.  Group g gathers rank 0's rows of g, then rank
// 1's, ... (rank order, then local order): gi = the source row of each regrouped row, goff[g] =
// group g's first regrouped row (G+1 entries).
inline void orswot_regroup(const uint64_t *cnt, size_t W, size_t G, size_t Dmax, std::vector<uint32_t> &gi,
                           std::vector<size_t> &goff) {
  gi.clear();
  goff.assign(G + 1, 0);
  std::vector<uint64_t> base(W, 0);
  for (size_t g = 0; g < G; ++g) {
    for (size_t r = 0; r < W; ++r) {
      const uint64_t c = cnt[r * (G + 1) + g];
      for (uint64_t j = 0; j < c; ++j) gi.push_back((uint32_t)(r * Dmax + base[r] + j));
      base[r] += c;
    }
    goff[g + 1] = gi.size();
  }
}

// LWWReg: the ranks holding replicas (R_k at word 2G of each gathered row of `row` words), in rank
// order, and how many of them sit below `rank` (the states this rank's shard continues from).
inline size_t lww_nonempty(const uint64_t *rows, size_t W, size_t row, size_t G, int rank,
                           std::vector<uint32_t> &nz) {
  nz.clear();
  size_t before = 0;
  for (size_t r = 0; r < W; ++r)
    if (rows[r * row + 2 * G]) {
      if ((long)r < (long)rank) ++before;
      nz.push_back((uint32_t)r);
    }
  return before;
}

// Map key shards: rows[W][G+1] = every rank's per-group flags and (word G) its local status.
// gflags[g] = OR of the ranks' flags; *bad = some rank failed; *grow = some key's fold state ran
// out of value slots (flags bit 2) on some rank.
inline void map_flags_or(const uint64_t *rows, size_t W, size_t G, uint32_t *gflags, bool *bad, bool *grow,
                         size_t stride = 0) {
  if (stride == 0) stride = G + 1;  // row r: [G flags | status | ...] at rows + r * stride
  *bad = false;
  *grow = false;
  for (size_t g = 0; g < G; ++g) {
    uint32_t f = 0;
    for (size_t r = 0; r < W; ++r) f |= (uint32_t)rows[r * stride + g];
    gflags[g] = f;
    *grow = *grow || (f & 4u) != 0;
  }
  for (size_t r = 0; r < W; ++r) *bad = *bad || rows[r * stride + G] != 0;
}

// Order-sensitive hash of a host offset array (def_off must be identical on every rank of a
// key-sharded Map call).
inline uint64_t hash_offsets(const size_t *off, size_t n) {
  uint64_t h = 0x84222325cbf29ce4ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ (uint64_t)off[i]) * 0x100000001b3ull;
  return h;
}

}  // namespace shard_host
}  // namespace crdt
