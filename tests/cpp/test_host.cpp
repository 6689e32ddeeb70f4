// C++ host-mirror tests (rust-crdt_amd/host/crdts.hpp): the reference's own tests, restated
// with every merge executed by libcrdt_gpu on the GPU.  Run by tests/test_gpu_host_cpp.py.
//   test/vclock.rs:104-231, src/vclock.rs:231-245 (glb doctest), src/gcounter.rs:79-92,
//   src/pncounter.rs:135-184,
//   src/gset.rs:29-37, src/lwwreg.rs:36-42,112-138, src/orswot.rs:294-394, test/orswot.rs:33-236
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

#include "crdts.hpp"

using namespace crdts;
using S = std::string;

static int g_fail = 0, g_checks = 0;
#define CHECK(cond)                                                        \
  do {                                                                     \
    ++g_checks;                                                            \
    if (!(cond)) {                                                         \
      ++g_fail;                                                            \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                      \
  } while (0)

template <class A>
static VClock<A> vc(std::initializer_list<std::pair<A, uint64_t>> ds) {
  VClock<A> v;
  for (auto &d : ds) v.apply(Dot<A>{d.first, d.second});
  return v;
}

// ---- test/vclock.rs -----------------------------------------------------------------------
static void test_merge(Gpu &g) {  // :118-130
  auto a = vc<uint8_t>({{1, 1}, {4, 4}});
  auto b = vc<uint8_t>({{3, 3}, {4, 3}});
  a.merge(g, b);
  CHECK(a == vc<uint8_t>({{1, 1}, {3, 3}, {4, 4}}));
}
static void test_merge_less_left(Gpu &g) {  // :132-144
  VClock<int> a, b;
  a.apply({5, 5});
  b.apply({6, 6});
  b.apply({7, 7});
  a.merge(g, b);
  CHECK(a.get(5) == 5 && a.get(6) == 6 && a.get(7) == 7);
}
static void test_merge_less_right(Gpu &g) {  // :146-158
  VClock<int> a, b;
  a.apply({6, 6});
  a.apply({7, 7});
  b.apply({5, 5});
  a.merge(g, b);
  CHECK(a.get(5) == 5 && a.get(6) == 6 && a.get(7) == 7);
}
static void test_merge_same_id(Gpu &g) {  // :160-173
  VClock<int> a, b;
  a.apply({1, 1});
  a.apply({2, 1});
  b.apply({1, 1});
  b.apply({3, 1});
  a.merge(g, b);
  CHECK(a.get(1) == 1 && a.get(2) == 1 && a.get(3) == 1);
}
static void test_vclock_ordering() {  // :175-231 (PartialOrd, host)
  CHECK(VClock<int8_t>() == VClock<int8_t>());
  VClock<S> a, b;
  a.apply({"A", 1});
  a.apply({"A", 2});
  a.apply({"A", 0});
  b.apply({"A", 1});
  CHECK(a.gt(b) && b.lt(a) && a != b);
  b.apply({"A", 3});
  CHECK(b.gt(a) && a.lt(b) && a != b);
  a.apply({"B", 1});
  CHECK(a != b && !a.gt(b) && !b.gt(a));
  a.apply({"A", 3});
  CHECK(a.gt(b) && b.lt(a) && a != b);
  b.apply({"B", 2});
  CHECK(b.gt(a) && a.lt(b) && a != b);
  a.apply({"B", 2});
  CHECK(!b.gt(a) && !a.gt(b) && a == b);
}
static void test_vclock_lub_many_and_batch(Gpu &g) {
  std::mt19937_64 rng(7);
  std::vector<VClock<uint32_t>> reps(300), others(300);
  VClock<uint32_t> expect;
  for (auto *vs : {&reps, &others})
    for (auto &v : *vs)
      for (int k = 0; k < 20; ++k) v.apply({uint32_t(rng() % 50), rng() % 1000 + 1});
  for (auto &r : reps)  // host expectation of the fold: per-actor max (apply_dot)
    for (auto &kv : r.dots) expect.apply({kv.first, kv.second});
  CHECK(lub_many(g, reps) == expect);
  auto selves = reps;
  merge_batch(g, selves, others);
  bool ok = true;
  for (size_t i = 0; i < reps.size(); ++i) {
    auto e = reps[i];
    for (auto &kv : others[i].dots) e.apply({kv.first, kv.second});
    ok = ok && selves[i] == e;
  }
  CHECK(ok);
  CHECK(lub_many(g, std::vector<VClock<uint32_t>>{}) == VClock<uint32_t>());
}

static void test_forget_gpu(Gpu &g) {  // test/vclock.rs:104-116, forget on the GPU
  std::vector<VClock<uint8_t>> a{vc<uint8_t>({{1, 4}, {2, 3}, {5, 9}})};
  std::vector<VClock<uint8_t>> b{vc<uint8_t>({{1, 5}, {2, 3}, {5, 8}})};
  forget_batch(g, a, b);
  CHECK(a[0] == vc<uint8_t>({{5, 9}}));
}
static void doctest_glb_gpu(Gpu &g) {  // src/vclock.rs:231-245, glb on the GPU
  VClock<int> c;
  c.apply({23, 6});
  c.apply({89, 14});
  auto c2 = c;
  std::vector<VClock<int>> cs{c}, c2s{c2};
  glb_batch(g, cs, c2s);  // no-op: glb { c, c } = c
  CHECK(cs[0] == c2);
  cs[0].apply({43, 1});
  CHECK(cs[0].get(43) == 1);
  glb_batch(g, cs, c2s);  // removes the 43 => 1 entry
  CHECK(cs[0].get(43) == 0);
}
static void test_causal_batches_gpu(Gpu &g) {  // GPU vs host on random clocks
  std::mt19937_64 rng(11);
  std::vector<VClock<uint32_t>> xs(400), ys(400);
  for (size_t i = 0; i < xs.size(); ++i) {
    for (int k = 0; k < 12; ++k) xs[i].apply({uint32_t(rng() % 20), rng() % 5 + 1});
    ys[i] = (i % 4 == 0) ? xs[i] : VClock<uint32_t>();  // equal, dominated, dominating, concurrent
    if (i % 4 == 1)
      for (auto &kv : xs[i].dots) ys[i].apply({kv.first, kv.second > 1 ? kv.second - 1 : 0});
    if (i % 4 == 2) {
      ys[i] = xs[i];
      ys[i].apply({uint32_t(rng() % 20), 9});
    }
    if (i % 4 == 3)
      for (int k = 0; k < 12; ++k) ys[i].apply({uint32_t(rng() % 20), rng() % 5 + 1});
  }
  auto cmp = partial_cmp_batch(g, xs, ys);
  bool ok = cmp.size() == xs.size();
  for (size_t i = 0; ok && i < xs.size(); ++i) ok = cmp[i] == xs[i].partial_cmp(ys[i]);
  CHECK(ok);
  auto in = intersection_batch(g, xs, ys);  // vclock.rs:218-227, restated on the host
  ok = in.size() == xs.size();
  for (size_t i = 0; ok && i < xs.size(); ++i) {
    VClock<uint32_t> e;
    for (auto &kv : xs[i].dots)
      if (ys[i].get(kv.first) == kv.second) e.dots[kv.first] = kv.second;
    ok = in[i] == e;
  }
  CHECK(ok);
  auto m = cmp_matrix(g, xs);
  ok = m.size() == xs.size() * xs.size();
  for (size_t i = 0; ok && i < xs.size(); i += 7)
    for (size_t j = 0; ok && j < xs.size(); j += 3) ok = m[i * xs.size() + j] == xs[i].partial_cmp(xs[j]);
  CHECK(ok);
  auto states = xs;
  std::vector<std::pair<size_t, Dot<uint32_t>>> ops;
  for (int k = 0; k < 5000; ++k) ops.push_back({rng() % states.size(), {uint32_t(rng() % 30), rng() % 9}});
  apply_batch(g, states, ops);
  auto host = xs;
  for (auto &o : ops) host[o.first].apply(o.second);
  CHECK(states == host);
  std::vector<GCounter<uint32_t>> gcs(xs.size());
  for (size_t i = 0; i < xs.size(); ++i) gcs[i].inner = xs[i];
  gcs[0].inner.apply({99, ~0ull});  // sum beyond 2^64
  gcs[0].inner.apply({98, ~0ull});
  auto rd = read_batch(g, gcs);
  ok = true;
  for (size_t i = 0; i < gcs.size(); ++i) ok = ok && rd[i] == gcs[i].read();
  CHECK(ok);
}

// ---- src/gcounter.rs / src/pncounter.rs -------------------------------------------------------
static void gcounter_test_basic(Gpu &g) {  // gcounter.rs:79-92
  GCounter<S> a, b;
  a.apply(a.inc("A"));
  b.apply(b.inc("B"));
  CHECK(a.read() == b.read());
  CHECK(a != b);
  a.apply(a.inc("A"));
  CHECK(a.read() == b.read() + 1);
  a.merge(g, b);
  CHECK(a.read() == 3);
}
static void pncounter_test_basic() {  // pncounter.rs:168-184
  PNCounter<S> a;
  CHECK(a.read() == 0);
  a.apply(a.inc("A"));
  CHECK(a.read() == 1);
  a.apply(a.inc("A"));
  CHECK(a.read() == 2);
  a.apply(a.dec("A"));
  CHECK(a.read() == 1);
  a.apply(a.inc("A"));
  CHECK(a.read() == 2);
}
static void pncounter_prop_merge_converges(Gpu &g) {  // pncounter.rs:135-166
  for (int seed = 0; seed < 5; ++seed) {
    std::mt19937_64 rng(100 + seed);
    std::vector<PNOp<uint8_t>> ops;
    for (int k = 0; k < 60; ++k)
      ops.push_back({{uint8_t(rng() % 11), rng() % 20}, (rng() & 1) ? Dir::Pos : Dir::Neg});
    std::set<long long> results;
    for (int i = 2; i < 11; ++i) {
      std::vector<PNCounter<uint8_t>> w(i);
      for (auto &op : ops) w[op.dot.actor % i].apply(op);
      results.insert((long long)lub_many(g, w).read());
    }
    CHECK(results.size() == 1);
  }
}

// ---- src/gset.rs, src/lwwreg.rs -------------------------------------------------------------
static void gset_doctest_merge(Gpu &g) {  // gset.rs:29-37
  GSet<int> a, b;
  a.insert(1);
  b.insert(2);
  a.merge(g, b);
  CHECK(a.contains(1) && a.contains(2));
  std::vector<GSet<int>> reps(70);
  for (int r = 0; r < 70; ++r) reps[r].insert(r * 3);
  CHECK(lub_many(g, reps).value.size() == 70);
}
static void lwwreg_test_update() {  // lwwreg.rs:112-138 (host update)
  LWWReg<int> reg(123, 0);
  CHECK(!reg.update(32, 2));
  CHECK(reg == LWWReg<int>(32, 2));
  CHECK(!reg.update(57, 1));
  CHECK(reg == LWWReg<int>(32, 2));
  CHECK(!reg.update(32, 2));
  CHECK(reg == LWWReg<int>(32, 2));
  CHECK(reg.update(4000, 2) == Error::ConflictingMarker);
  CHECK(reg == LWWReg<int>(32, 2));
}
static void lwwreg_merge_gpu(Gpu &g) {  // lwwreg.rs:36-42 + fold semantics
  LWWReg<int> l1(1, 2), l2(3, 2);
  CHECK(l1.merge(g, l2) == Error::ConflictingMarker);
  CHECK(l1 == LWWReg<int>(1, 2));
  LWWReg<S> r("a", 1);
  CHECK(!r.merge(g, LWWReg<S>("b", 5)));
  CHECK(r == LWWReg<S>("b", 5));
  CHECK(!r.merge(g, LWWReg<S>("z", 4)));
  CHECK(r == LWWReg<S>("b", 5));
  auto lub = lub_many(g, std::vector<LWWReg<int>>{{1, 3}, {2, 7}, {3, 5}, {4, 7}, {2, 7}, {5, 9}});
  CHECK(lub.reg == LWWReg<int>(5, 9));
  CHECK(lub.first_conflict && *lub.first_conflict == 3);  // (4,7) vs held (2,7)
}

// ---- src/orswot.rs, test/orswot.rs ------------------------------------------------------------
using OS = Orswot<S, S>;
using OI = Orswot<int, S>;

template <class M>
static void add(Orswot<M, S> &o, const M &m, const S &actor) {
  o.apply(o.add(m, o.read().derive_add_ctx(actor)));
}
template <class M>
static void rm(Orswot<M, S> &o, const M &m) {
  o.apply(o.rm(m, o.contains(m).derive_rm_ctx()));
}

static void ensure_deferred_merges(Gpu &g) {  // orswot.rs:294-330
  OS a, b;
  add<S>(b, "element 1", "A");
  b.apply(b.rm("element 1", RmCtx<S>{vc<S>({{"A", 4}})}));
  add<S>(a, "element 4", "B");
  b.apply(b.rm("element 9", RmCtx<S>{vc<S>({{"C", 4}})}));
  OS merged;
  merged.merge(g, a);
  merged.merge(g, b);
  merged.merge(g, OS());
  CHECK(merged.deferred.size() == 2);
}
static void preserve_deferred_across_merges(Gpu &g) {  // orswot.rs:334-361
  OI a, b, c;
  add<int>(a, 5, "A");
  b.apply(b.rm(5, RmCtx<S>{vc<S>({{"A", 3}, {"B", 8}})}));
  CHECK(b.deferred.size() == 1);
  c.merge(g, b);
  CHECK(c.deferred.size() == 1);
  a.merge(g, c);
  CHECK(a.read().val.empty());
}
static void test_present_but_removed(Gpu &g) {  // orswot.rs:366-394
  OI a, b;
  add<int>(a, 0, "A");
  OI c = a;
  rm<int>(a, 0);
  CHECK(a.deferred.empty());
  add<int>(b, 0, "B");
  a.merge(g, b);
  rm<int>(b, 0);
  a.merge(g, b);
  a.merge(g, c);
  CHECK(a.read().val.empty());
}
static void weird_highlight_1(Gpu &g) {  // test/orswot.rs:74-83
  OI a, b;
  add<int>(a, 1, "A");
  add<int>(b, 2, "A");
  a.merge(g, b);
  CHECK(a.read().val.empty());
}
static void adds_dont_destroy_causality(Gpu &g) {  // test/orswot.rs:86-114
  OS a, b, c;
  auto c_ctx = c.read();
  c.apply(c.add("element", c_ctx.derive_add_ctx("A")));
  c.apply(c.add("element", c_ctx.derive_add_ctx("B")));
  auto c_element_ctx = c.contains("element");
  CHECK(c_element_ctx.rm_clock == vc<S>({{"A", 1}, {"B", 1}}));
  add<S>(a, "element", "C");
  b.apply(c.rm("element", c_element_ctx.derive_rm_ctx()));
  add<S>(a, "element", "A");
  a.merge(g, b);
  CHECK(a.read().val == std::set<S>{"element"});
}
static void merge_clocks_of_identical_entries(Gpu &g) {  // test/orswot.rs:119-135
  OI a, b;
  add<int>(a, 1, "A");
  add<int>(b, 1, "B");
  a.merge(g, b);
  CHECK(a.read().val == std::set<int>{1});
  CHECK(a.contains(1).val);
  CHECK(a.contains(1).rm_clock == vc<S>({{"A", 1}, {"B", 1}}));
}
static void test_disjoint_merge(Gpu &g) {  // test/orswot.rs:138-158
  OI a, b;
  add<int>(a, 0, "A");
  CHECK(a.read().val == std::set<int>{0});
  add<int>(b, 1, "B");
  CHECK(b.read().val == std::set<int>{1});
  OI c = a;
  c.merge(g, b);
  CHECK((c.read().val == std::set<int>{0, 1}));
  rm<int>(a, 0);
  OI d = a;
  d.merge(g, c);
  CHECK(d.read().val == std::set<int>{1});
}
static void test_no_dots_left_test(Gpu &g) {  // test/orswot.rs:163-194
  OI a, b;
  add<int>(a, 0, "A");
  add<int>(b, 0, "B");
  OI c = a;
  rm<int>(a, 0);
  a.merge(g, b);
  CHECK(a.read().val == std::set<int>{0});
  CHECK(a.read().add_clock == vc<S>({{"A", 1}, {"B", 1}}));
  rm<int>(b, 0);
  CHECK(b.read().val.empty());
  b.merge(g, c);
  CHECK(b.read().val == std::set<int>{0});
  b.merge(g, a);
  b.merge(g, c);
  CHECK(b.read().val.empty());
}
static void test_dead_node_update(Gpu &g) {  // test/orswot.rs:209-236
  OI a;
  auto a_op = a.add(0, a.read().derive_add_ctx("A"));
  CHECK(a_op.is_add && a_op.dot == (Dot<S>{"A", 1}) && a_op.members == std::set<int>{0});
  a.apply(a_op);
  CHECK(a.contains(0).rm_clock == vc<S>({{"A", 1}}));
  OI b = a;
  add<int>(b, 1, "B");
  auto bctx = b.read();
  CHECK(bctx.add_clock == vc<S>({{"A", 1}, {"B", 1}}));
  a.apply(a.rm(0, bctx.derive_rm_ctx()));
  CHECK(a.read().val.empty());
  (void)g;
}
static void orswot_prop_merge_converges(Gpu &g) {  // test/orswot.rs:33-68
  for (int seed = 0; seed < 8; ++seed) {
    std::mt19937_64 rng(1000 + seed);
    std::vector<std::pair<uint8_t, OrswotOp<uint8_t, uint8_t>>> ops;
    for (int k = 0; k < 40; ++k) {  // build_opvec (test/orswot.rs:15-31)
      uint8_t actor = rng() % 11;
      std::set<uint8_t> members;
      for (int j = 0, n = 1 + rng() % 3; j < n; ++j) members.insert(rng() % 8);
      uint64_t counter = rng() % 8 + 1;
      OrswotOp<uint8_t, uint8_t> op;
      op.is_add = (rng() % 2) == 0;
      op.members = members;
      if (op.is_add) op.dot = Dot<uint8_t>{actor, counter};
      else op.clock.apply(Dot<uint8_t>{actor, counter});
      ops.push_back({actor, op});
    }
    std::optional<Orswot<uint8_t, uint8_t>> result;
    bool ok = true;
    for (int i = 2; i < 11; ++i) {
      std::vector<Orswot<uint8_t, uint8_t>> w(i);
      for (auto &p : ops) w[p.first % i].apply(p.second);
      auto merged = lub_many(g, w);  // == Orswot::new() merged with every witness
      if (!result) result = merged;
      else if (!(merged == *result)) {
        if (ok) {
          std::fprintf(stderr, "seed %d i %d mismatch\n", seed, i);
          for (auto *o : {&*result, &merged}) {
            std::fprintf(stderr, "  clock:");
            for (auto &kv : o->clock.dots) std::fprintf(stderr, " %d:%llu", kv.first, (unsigned long long)kv.second);
            std::fprintf(stderr, "\n  entries:");
            for (auto &e : o->entries) {
              std::fprintf(stderr, " m%d{", e.first);
              for (auto &kv : e.second.dots) std::fprintf(stderr, "%d:%llu ", kv.first, (unsigned long long)kv.second);
              std::fprintf(stderr, "}");
            }
            std::fprintf(stderr, "\n  deferred:");
            for (auto &d : o->deferred) {
              std::fprintf(stderr, " {");
              for (auto &kv : d.first.dots) std::fprintf(stderr, "%d:%llu ", kv.first, (unsigned long long)kv.second);
              std::fprintf(stderr, "}->[");
              for (auto m : d.second) std::fprintf(stderr, "%d ", m);
              std::fprintf(stderr, "]");
            }
            std::fprintf(stderr, "\n");
          }
        }
        ok = false;
      }
    }
    CHECK(ok);
  }
}

int main() {
  Gpu g(0);
  test_merge(g);
  test_merge_less_left(g);
  test_merge_less_right(g);
  test_merge_same_id(g);
  test_vclock_ordering();
  test_vclock_lub_many_and_batch(g);
  test_forget_gpu(g);
  doctest_glb_gpu(g);
  test_causal_batches_gpu(g);
  gcounter_test_basic(g);
  pncounter_test_basic();
  pncounter_prop_merge_converges(g);
  gset_doctest_merge(g);
  lwwreg_test_update();
  lwwreg_merge_gpu(g);
  ensure_deferred_merges(g);
  preserve_deferred_across_merges(g);
  test_present_but_removed(g);
  weird_highlight_1(g);
  adds_dont_destroy_causality(g);
  merge_clocks_of_identical_entries(g);
  test_disjoint_merge(g);
  test_no_dots_left_test(g);
  test_dead_node_update(g);
  orswot_prop_merge_converges(g);
  std::printf("%d checks, %d failed\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
