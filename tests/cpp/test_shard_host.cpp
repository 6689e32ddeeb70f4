// Unit tests of the host-side bookkeeping of the sharded entry points (csrc/shard_host.hpp), built
// with g++ -fsanitize=address,undefined by tests/test_sanitizers.py.  Every function is checked
// against a brute-force restatement on random inputs; any failed check aborts with a message.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "shard_host.hpp"

using namespace crdt::shard_host;

#define CHECK(x)                                                        \
  do {                                                                  \
    if (!(x)) {                                                         \
      std::fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #x); \
      std::abort();                                                     \
    }                                                                   \
  } while (0)

static void test_regroup(std::mt19937_64 &rng) {
  for (int it = 0; it < 200; ++it) {
    const size_t W = 1 + rng() % 8, G = rng() % 9;
    std::vector<uint64_t> cnt(W * (G + 1), 0);
    size_t Dmax = 0, Dtot = 0;
    for (size_t r = 0; r < W; ++r) {
      uint64_t tot = 0;
      for (size_t g = 0; g < G; ++g) {
        cnt[r * (G + 1) + g] = (rng() % 3 == 0) ? rng() % 4 : 0;
        tot += cnt[r * (G + 1) + g];
      }
      cnt[r * (G + 1) + G] = tot;
      Dmax = std::max<size_t>(Dmax, tot);
      Dtot += tot;
    }
    std::vector<uint32_t> gi;
    std::vector<size_t> goff;
    orswot_regroup(cnt.data(), W, G, Dmax, gi, goff);
    CHECK(gi.size() == Dtot && goff.size() == G + 1 && goff[0] == 0 && goff[G] == Dtot);
    // brute force: rank r's rows are r*Dmax + [0, tot_r) in group order; group g takes rank 0's
    // rows of g, then rank 1's, ...
    size_t pos = 0;
    for (size_t g = 0; g < G; ++g) {
      CHECK(goff[g] == pos);
      for (size_t r = 0; r < W; ++r) {
        uint64_t before = 0;
        for (size_t h = 0; h < g; ++h) before += cnt[r * (G + 1) + h];
        for (uint64_t j = 0; j < cnt[r * (G + 1) + g]; ++j) {
          CHECK(gi[pos] == r * Dmax + before + j);
          CHECK(gi[pos] < W * Dmax);
          ++pos;
        }
      }
    }
    CHECK(pos == Dtot);
  }
}

static void test_headers(std::mt19937_64 &rng) {
  for (int it = 0; it < 200; ++it) {
    const size_t W = 1 + rng() % 8;
    const uint64_t G = rng() % 5, A = rng() % 300;
    const Hdr mine = make_hdr(false, 3, {G, A, 7, 8, 9, 10, 11});
    std::vector<uint64_t> rows(W * kHdr);
    long bad_exp = -1, odd_exp = -1;
    for (size_t r = 0; r < W; ++r) {
      const bool fail = rng() % 5 == 0;
      const bool odd = rng() % 6 == 0;
      // a difference past the 5 raw dims is caught by the hash word
      const Hdr h = make_hdr(fail, 3, {G, A, 7, 8, 9, 10, odd ? 12ull : 11ull});
      for (int k = 0; k < kHdr; ++k) rows[r * kHdr + k] = h.w[k];
      if (fail && bad_exp < 0) bad_exp = (long)r;
      if (odd && odd_exp < 0) odd_exp = (long)r;
    }
    long bad, odd;
    const bool ok = check_headers(rows.data(), W, mine, &bad, &odd);
    CHECK(bad == bad_exp && odd == odd_exp && ok == (bad < 0 && odd < 0));
  }
  // the same dims in another entry point (tag) disagree; dims order matters
  const Hdr a = make_hdr(false, 1, {4, 5}), b = make_hdr(false, 2, {4, 5}), c = make_hdr(false, 1, {5, 4});
  long bad, odd;
  std::vector<uint64_t> rows(2 * kHdr);
  for (int k = 0; k < kHdr; ++k) rows[k] = a.w[k], rows[kHdr + k] = b.w[k];
  CHECK(!check_headers(rows.data(), 2, a, &bad, &odd) && bad == -1 && odd == 1);
  for (int k = 0; k < kHdr; ++k) rows[kHdr + k] = c.w[k];
  CHECK(!check_headers(rows.data(), 2, a, &bad, &odd) && odd == 1);
}

static void test_lww_nonempty(std::mt19937_64 &rng) {
  for (int it = 0; it < 200; ++it) {
    const size_t W = 1 + rng() % 8, G = 1 + rng() % 4, row = 2 * G + 1;
    std::vector<uint64_t> rows(W * row, 0);
    for (size_t r = 0; r < W; ++r) rows[r * row + 2 * G] = rng() % 3 == 0 ? 0 : 1 + rng() % 100;
    const int rank = (int)(rng() % W);
    std::vector<uint32_t> nz;
    const size_t before = lww_nonempty(rows.data(), W, row, G, rank, nz);
    size_t b = 0, n = 0;
    for (size_t r = 0; r < W; ++r)
      if (rows[r * row + 2 * G]) {
        CHECK(nz[n] == r);
        ++n;
        if ((int)r < rank) ++b;
      }
    CHECK(n == nz.size() && b == before);
  }
}

static void test_map_flags(std::mt19937_64 &rng) {
  for (int it = 0; it < 200; ++it) {
    const size_t W = 1 + rng() % 8, G = rng() % 6;
    std::vector<uint64_t> rows(W * (G + 1));
    for (auto &x : rows) x = rng() % 8 == 0 ? rng() % 8 : 0;
    std::vector<uint32_t> f(G + 1, 0xdead);
    bool bad, grow;
    map_flags_or(rows.data(), W, G, f.data(), &bad, &grow);
    bool b2 = false, g2 = false;
    for (size_t g = 0; g < G; ++g) {
      uint32_t o = 0;
      for (size_t r = 0; r < W; ++r) o |= (uint32_t)rows[r * (G + 1) + g];
      CHECK(f[g] == o);
      g2 = g2 || (o & 4);
    }
    for (size_t r = 0; r < W; ++r) b2 = b2 || rows[r * (G + 1) + G];
    CHECK(bad == b2 && grow == g2 && f[G] == 0xdead);  // nothing written past G
  }
  size_t off1[3] = {0, 4, 9}, off2[3] = {0, 5, 9};
  CHECK(hash_offsets(off1, 3) != hash_offsets(off2, 3) && hash_offsets(off1, 3) == hash_offsets(off1, 3));
}

// Agreed-plan cache and the cached path's check words: the MAX over ranks of [failed, key, ~key] passes
// on every rank iff every rank sent the same key and none failed.
static void test_plan_cache(std::mt19937_64 &rng) {
  PlanCache c;
  for (uint64_t k = 0; k < 40; ++k) {
    c.add(k * 7 + 1);
    CHECK(c.has(k * 7 + 1) && c.n <= PlanCache::kCap);
  }
  CHECK(!c.has(1) && c.has(39 * 7 + 1));  // the oldest plans left the full cache
  c.add(39 * 7 + 1);
  CHECK(c.n == PlanCache::kCap);  // no duplicate
  c.clear();
  CHECK(c.n == 0 && !c.has(39 * 7 + 1));
  const Hdr a = make_hdr(false, 1, {4, 256}), b = make_hdr(true, 1, {4, 256}), d = make_hdr(false, 1, {4, 254});
  CHECK(plan_key(a) == plan_key(b) && plan_key(a) != plan_key(d));  // a rank's own status is not in the key
  CHECK(plan_key(a) != plan_key(make_hdr(false, 2, {4, 256})));
  for (int it = 0; it < 500; ++it) {
    const size_t W = 1 + rng() % 8;
    const uint64_t key = rng();
    std::vector<uint64_t> red(3, 0), w(3);
    bool failed = false, odd = false;
    for (size_t r = 0; r < W; ++r) {
      const bool f = rng() % 5 == 0;
      const uint64_t k = rng() % 4 == 0 ? rng() : key;
      failed = failed || f;
      odd = odd || k != key;
      check_words(f, k, w.data());
      for (int j = 0; j < 3; ++j) red[j] = std::max(red[j], w[j]);
    }
    CHECK(check_ok(red.data(), key) == (!failed && !odd));
  }
}

int main() {
  std::mt19937_64 rng(0x5EED);
  test_plan_cache(rng);
  test_regroup(rng);
  test_headers(rng);
  test_lww_nonempty(rng);
  test_map_flags(rng);
  std::printf("shard_host: all checks passed\n");
  return 0;
}
