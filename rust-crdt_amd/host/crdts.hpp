// crdts.hpp — C++ host mirror of the `crdts` 3.0.0 (rust-crdt) merge surface over
// libcrdt_gpu.so (include/crdt_gpu.h).  Header-only, C++17.
//
// The reference is Rust; this image has no Rust toolchain, so the host side above the C ABI is
// C++ (INTEGRATION.md shows the Rust binding the ABI is designed for).  Types keep the
// reference's shapes and names: VClock<A> (vclock.rs:56-60, BTreeMap -> std::map), GCounter,
// PNCounter, GSet<T>, LWWReg<V, u64>, Orswot<M, A> (orswot.rs:20-25) with ReadCtx / AddCtx /
// RmCtx (ctx.rs).  Every MERGE runs on the GPU:
//
//   x.merge(gpu, other)             CvRDT::merge (traits.rs:4-7) == lub_many of {x, other}
//   lub_many(gpu, replicas)         acc = T::new(); for r in replicas { acc.merge(r) }
//   merge_batch(gpu, selves, others)  for i: selves[i].merge(others[i])
//
// Ingest interns actors / members / elements to dense indices (sorted, so results are
// deterministic), egress drops zero counters (apply_dot never stores 0, vclock.rs:155-159).
// Op application (`apply`, CmRDT, traits.rs:10-36) is host-side: it is how tests and callers
// BUILD states one op at a time and is not part of the batched merge path.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <functional>
#include <map>
#include <optional>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "crdt_gpu.h"

namespace crdts {

// error.rs:8-15 — Error::ConflictingMarker (LWWReg); returned, never thrown, like Result.
enum class Error { ConflictingMarker };

struct GpuError : std::runtime_error {
  int code;
  GpuError(const std::string &what, int c) : std::runtime_error(what), code(c) {}
};

// ---- device context ------------------------------------------------------------------------
class Gpu {
 public:
  explicit Gpu(int device = 0) : device_(device) {
    check(crdt_ctx_create(device, &ctx_), "crdt_ctx_create");
  }
  ~Gpu() { crdt_ctx_destroy(ctx_); }
  Gpu(const Gpu &) = delete;
  Gpu &operator=(const Gpu &) = delete;
  crdt_ctx *ctx() const { return ctx_; }
  int device() const { return device_; }
  void check(int rc, const char *what) const {
    if (rc != CRDT_OK) throw GpuError(std::string(what) + ": " + crdt_last_error(ctx_), rc);
  }
  void sync() const { check(crdt_ctx_synchronize(ctx_), "crdt_ctx_synchronize"); }

 private:
  int device_;
  crdt_ctx *ctx_ = nullptr;
};

template <class T>
class DeviceBuf {
 public:
  explicit DeviceBuf(size_t n) : n_(n) {
    if (n_ && hipMalloc(reinterpret_cast<void **>(&p_), n_ * sizeof(T)) != hipSuccess)
      throw GpuError("hipMalloc failed", CRDT_ENOMEM);
  }
  explicit DeviceBuf(const std::vector<T> &v) : DeviceBuf(v.size()) { upload(v); }
  ~DeviceBuf() {
    if (p_) (void)hipFree(p_);
  }
  DeviceBuf(const DeviceBuf &) = delete;
  DeviceBuf &operator=(const DeviceBuf &) = delete;
  T *get() const { return p_; }
  void upload(const std::vector<T> &v) {
    if (n_ && hipMemcpy(p_, v.data(), n_ * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
      throw GpuError("hipMemcpy H2D failed", CRDT_EHIP);
  }
  std::vector<T> download() const {
    std::vector<T> v(n_);
    if (n_ && hipMemcpy(v.data(), p_, n_ * sizeof(T), hipMemcpyDeviceToHost) != hipSuccess)
      throw GpuError("hipMemcpy D2H failed", CRDT_EHIP);
    return v;
  }

 private:
  T *p_ = nullptr;
  size_t n_;
};

// Dense interning of ids, in sorted order (deterministic column assignment).
template <class K>
class Interner {
 public:
  void add(const K &k) { pos_.emplace(k, 0); }
  void freeze() {
    ids_.clear();
    uint32_t i = 0;
    for (auto &kv : pos_) {
      kv.second = i++;
      ids_.push_back(kv.first);
    }
  }
  uint32_t at(const K &k) const { return pos_.at(k); }
  const K &id(size_t i) const { return ids_[i]; }
  size_t size() const { return ids_.size(); }

 private:
  std::map<K, uint32_t> pos_;
  std::vector<K> ids_;
};

// ---- VClock (vclock.rs) ------------------------------------------------------------------
template <class A>
struct Dot {  // vclock.rs:32-38
  A actor;
  uint64_t counter;
  bool operator==(const Dot &o) const { return actor == o.actor && counter == o.counter; }
};

enum class Ordering { Less, Equal, Greater };

template <class A>
class VClock {
 public:
  std::map<A, uint64_t> dots;  // vclock.rs:59

  VClock() = default;
  VClock(std::initializer_list<Dot<A>> ds) {
    for (auto &d : ds) apply(d);
  }
  uint64_t get(const A &a) const {  // vclock.rs:207-209
    auto it = dots.find(a);
    return it == dots.end() ? 0 : it->second;
  }
  bool is_empty() const { return dots.empty(); }
  Dot<A> inc(const A &a) const { return Dot<A>{a, get(a) + 1}; }  // vclock.rs:183-189
  void apply(const Dot<A> &d) {  // CmRDT::apply -> apply_dot, vclock.rs:125-127, 155-159
    if (get(d.actor) < d.counter) dots[d.actor] = d.counter;
  }
  bool operator==(const VClock &o) const { return dots == o.dots; }
  bool operator!=(const VClock &o) const { return !(*this == o); }
  bool operator<(const VClock &o) const { return dots < o.dots; }  // container key only
  // PartialOrd (vclock.rs:68-80); nullopt = concurrent.
  std::optional<Ordering> partial_cmp(const VClock &o) const {
    if (*this == o) return Ordering::Equal;
    if (std::all_of(o.dots.begin(), o.dots.end(), [&](auto &kv) { return get(kv.first) >= kv.second; }))
      return Ordering::Greater;
    if (std::all_of(dots.begin(), dots.end(), [&](auto &kv) { return o.get(kv.first) >= kv.second; }))
      return Ordering::Less;
    return std::nullopt;
  }
  bool gt(const VClock &o) const { return partial_cmp(o) == Ordering::Greater; }
  bool lt(const VClock &o) const { return partial_cmp(o) == Ordering::Less; }
  bool concurrent(const VClock &o) const { return !partial_cmp(o).has_value(); }

  void merge(Gpu &gpu, const VClock &other);  // CvRDT::merge on the GPU
};

namespace detail {

template <class A>
void intern_clock(Interner<A> &ix, const VClock<A> &c) {
  for (auto &kv : c.dots) ix.add(kv.first);
}
template <class A>
void write_row(const Interner<A> &ix, const VClock<A> &c, uint64_t *row) {
  for (auto &kv : c.dots) row[ix.at(kv.first)] = kv.second;
}
template <class A>
VClock<A> read_row(const Interner<A> &ix, const uint64_t *row, size_t n) {
  VClock<A> c;
  for (size_t a = 0; a < n; ++a)
    if (row[a]) c.dots.emplace_hint(c.dots.end(), ix.id(a), row[a]);
  return c;
}

// Shared body of the max-lattice lubs: rows (R x W) -> one row, through `fn`.
using LubFn = int (*)(crdt_ctx *, const uint64_t *, size_t, size_t, size_t, size_t, size_t,
                      uint64_t *, size_t, unsigned);
inline std::vector<uint64_t> lattice_lub(Gpu &gpu, LubFn fn, const char *name,
                                         const std::vector<uint64_t> &rows, size_t R, size_t W,
                                         size_t Wcall) {
  std::vector<uint64_t> out(W, 0);
  if (R == 0 || W == 0) return out;
  DeviceBuf<uint64_t> din(rows), dout(W);
  gpu.check(fn(gpu.ctx(), din.get(), 1, R, Wcall, W, 0, dout.get(), W, 0), name);
  gpu.sync();
  return dout.download();
}

}  // namespace detail

// acc = VClock::new(); for r in replicas { acc.merge(r) }   (vclock.rs:130-136)
template <class A>
VClock<A> lub_many(Gpu &gpu, const std::vector<VClock<A>> &replicas) {
  Interner<A> ix;
  for (auto &r : replicas) detail::intern_clock(ix, r);
  ix.freeze();
  const size_t R = replicas.size(), W = ix.size();
  std::vector<uint64_t> rows(R * W, 0);
  for (size_t r = 0; r < R; ++r) detail::write_row(ix, replicas[r], rows.data() + r * W);
  auto out = detail::lattice_lub(gpu, crdt_vclock_lub_many, "crdt_vclock_lub_many", rows, R, W, W);
  return detail::read_row(ix, out.data(), W);
}

template <class A>
void VClock<A>::merge(Gpu &gpu, const VClock<A> &other) {
  *this = lub_many<A>(gpu, {*this, other});
}

// for i: selves[i].merge(others[i])
template <class A>
void merge_batch(Gpu &gpu, std::vector<VClock<A>> &selves, const std::vector<VClock<A>> &others) {
  if (selves.size() != others.size()) throw std::invalid_argument("merge_batch: size mismatch");
  Interner<A> ix;
  for (auto &r : selves) detail::intern_clock(ix, r);
  for (auto &r : others) detail::intern_clock(ix, r);
  ix.freeze();
  const size_t N = selves.size(), W = ix.size();
  if (N == 0 || W == 0) return;
  std::vector<uint64_t> s(N * W, 0), o(N * W, 0);
  for (size_t i = 0; i < N; ++i) {
    detail::write_row(ix, selves[i], s.data() + i * W);
    detail::write_row(ix, others[i], o.data() + i * W);
  }
  DeviceBuf<uint64_t> ds(s), dod(o);
  gpu.check(crdt_vclock_merge_batch(gpu.ctx(), ds.get(), dod.get(), N, W, W, W), "crdt_vclock_merge_batch");
  gpu.sync();
  auto res = ds.download();
  for (size_t i = 0; i < N; ++i) selves[i] = detail::read_row(ix, res.data() + i * W, W);
}

// ---- causal helpers on the GPU (crdt_vclock_pair_op / partial_cmp / cmp_matrix) ------------
namespace detail {
// Pairs -> two dense (N x W) row blocks over one interner.
template <class A>
size_t pair_rows(const std::vector<VClock<A>> &xs, const std::vector<VClock<A>> &ys, Interner<A> &ix,
                 std::vector<uint64_t> &x, std::vector<uint64_t> &y) {
  if (xs.size() != ys.size()) throw std::invalid_argument("pair op: size mismatch");
  for (auto &r : xs) intern_clock(ix, r);
  for (auto &r : ys) intern_clock(ix, r);
  ix.freeze();
  const size_t N = xs.size(), W = ix.size();
  x.assign(N * W, 0);
  y.assign(N * W, 0);
  for (size_t i = 0; i < N; ++i) {
    write_row(ix, xs[i], x.data() + i * W);
    write_row(ix, ys[i], y.data() + i * W);
  }
  return W;
}
template <class A>
void pair_op(Gpu &gpu, int op, std::vector<VClock<A>> &selves, const std::vector<VClock<A>> &others) {
  Interner<A> ix;
  std::vector<uint64_t> x, y;
  const size_t W = pair_rows(selves, others, ix, x, y), N = selves.size();
  if (N == 0 || W == 0) return;
  DeviceBuf<uint64_t> dx(x), dy(y);
  gpu.check(crdt_vclock_pair_op(gpu.ctx(), op, dx.get(), dx.get(), dy.get(), N, W, W, W, W), "crdt_vclock_pair_op");
  gpu.sync();
  auto res = dx.download();
  for (size_t i = 0; i < N; ++i) selves[i] = read_row(ix, res.data() + i * W, W);
}
inline std::optional<Ordering> ordering_of(int8_t c) {
  if (c == 0) return Ordering::Equal;
  if (c == 1) return Ordering::Greater;
  if (c == -1) return Ordering::Less;
  return std::nullopt;
}
}  // namespace detail

// for i: selves[i].glb(&others[i])      (vclock.rs:246-259)
template <class A>
void glb_batch(Gpu &gpu, std::vector<VClock<A>> &selves, const std::vector<VClock<A>> &others) {
  detail::pair_op(gpu, CRDT_PAIR_GLB, selves, others);
}
// for i: selves[i].forget(&others[i])   (Causal::forget, vclock.rs:95-105)
template <class A>
void forget_batch(Gpu &gpu, std::vector<VClock<A>> &selves, const std::vector<VClock<A>> &others) {
  detail::pair_op(gpu, CRDT_PAIR_FORGET, selves, others);
}
// VClock::intersection(&lefts[i], &rights[i]): the common dots   (vclock.rs:218-227)
template <class A>
std::vector<VClock<A>> intersection_batch(Gpu &gpu, const std::vector<VClock<A>> &lefts,
                                          const std::vector<VClock<A>> &rights) {
  std::vector<VClock<A>> out(lefts);
  detail::pair_op(gpu, CRDT_PAIR_INTERSECTION, out, rights);
  return out;
}
// xs[i].partial_cmp(&ys[i])               (vclock.rs:68-80; nullopt = concurrent)
template <class A>
std::vector<std::optional<Ordering>> partial_cmp_batch(Gpu &gpu, const std::vector<VClock<A>> &xs,
                                                        const std::vector<VClock<A>> &ys) {
  Interner<A> ix;
  std::vector<uint64_t> x, y;
  const size_t W = detail::pair_rows(xs, ys, ix, x, y), N = xs.size();
  std::vector<std::optional<Ordering>> out;
  if (N == 0) return out;
  if (W == 0) return std::vector<std::optional<Ordering>>(N, Ordering::Equal);
  DeviceBuf<uint64_t> dx(x), dy(y);
  DeviceBuf<int8_t> dc(N);
  gpu.check(crdt_vclock_partial_cmp(gpu.ctx(), dx.get(), dy.get(), N, W, W, W, dc.get()), "crdt_vclock_partial_cmp");
  gpu.sync();
  for (int8_t c : dc.download()) out.push_back(detail::ordering_of(c));
  return out;
}
// every clocks[i].partial_cmp(&clocks[j]), row-major N x N
template <class A>
std::vector<std::optional<Ordering>> cmp_matrix(Gpu &gpu, const std::vector<VClock<A>> &clocks) {
  Interner<A> ix;
  for (auto &c : clocks) detail::intern_clock(ix, c);
  ix.freeze();
  const size_t N = clocks.size(), W = ix.size();
  std::vector<std::optional<Ordering>> out;
  if (N == 0) return out;
  if (W == 0) return std::vector<std::optional<Ordering>>(N * N, Ordering::Equal);
  std::vector<uint64_t> x(N * W, 0);
  for (size_t i = 0; i < N; ++i) detail::write_row(ix, clocks[i], x.data() + i * W);
  DeviceBuf<uint64_t> dx(x);
  DeviceBuf<int8_t> dc(N * N);
  gpu.check(crdt_vclock_cmp_matrix(gpu.ctx(), dx.get(), N, W, W, dc.get()), "crdt_vclock_cmp_matrix");
  gpu.sync();
  for (int8_t c : dc.download()) out.push_back(detail::ordering_of(c));
  return out;
}
// for (i, dot) in ops { states[i].apply(dot) }   (CmRDT::apply, vclock.rs:125-127, 155-159)
template <class A>
void apply_batch(Gpu &gpu, std::vector<VClock<A>> &states, const std::vector<std::pair<size_t, Dot<A>>> &ops) {
  Interner<A> ix;
  for (auto &s : states) detail::intern_clock(ix, s);
  for (auto &o : ops) ix.add(o.second.actor);
  ix.freeze();
  const size_t N = states.size(), W = ix.size();
  if (N == 0 || W == 0 || ops.empty()) return;
  std::vector<uint64_t> rows(N * W, 0), ctr;
  std::vector<uint32_t> si, ac;
  for (size_t i = 0; i < N; ++i) detail::write_row(ix, states[i], rows.data() + i * W);
  for (auto &o : ops) {
    if (o.first >= N) throw std::out_of_range("apply_batch: state index");
    si.push_back((uint32_t)o.first);
    ac.push_back(ix.at(o.second.actor));
    ctr.push_back(o.second.counter);
  }
  DeviceBuf<uint64_t> drows(rows), dctr(ctr);
  DeviceBuf<uint32_t> dsi(si), dac(ac), bad(std::vector<uint32_t>{0});
  gpu.check(crdt_vclock_apply_batch(gpu.ctx(), drows.get(), N, W, W, dsi.get(), dac.get(), dctr.get(), ops.size(),
                                    bad.get()),
            "crdt_vclock_apply_batch");
  gpu.sync();
  auto res = drows.download();
  for (size_t i = 0; i < N; ++i) states[i] = detail::read_row(ix, res.data() + i * W, W);
}

// ---- GCounter (gcounter.rs) / PNCounter (pncounter.rs) ------------------------------------
template <class A>
class GCounter {
 public:
  VClock<A> inner;  // gcounter.rs:27
  Dot<A> inc(const A &a) const { return inner.inc(a); }
  void apply(const Dot<A> &d) { inner.apply(d); }
  unsigned __int128 read() const {  // gcounter.rs:70-72 (BigUint sum; exact to 2^128)
    unsigned __int128 s = 0;
    for (auto &kv : inner.dots) s += kv.second;
    return s;
  }
  bool operator==(const GCounter &o) const { return inner == o.inner; }
  bool operator!=(const GCounter &o) const { return !(*this == o); }
  void merge(Gpu &gpu, const GCounter &other) {  // gcounter.rs:44-48
    *this = lub_many<A>(gpu, std::vector<GCounter>{*this, other});
  }
};

template <class A>
GCounter<A> lub_many(Gpu &gpu, const std::vector<GCounter<A>> &replicas) {
  Interner<A> ix;
  for (auto &r : replicas) detail::intern_clock(ix, r.inner);
  ix.freeze();
  const size_t R = replicas.size(), W = ix.size();
  std::vector<uint64_t> rows(R * W, 0);
  for (size_t r = 0; r < R; ++r) detail::write_row(ix, replicas[r].inner, rows.data() + r * W);
  auto out = detail::lattice_lub(gpu, crdt_gcounter_lub_many, "crdt_gcounter_lub_many", rows, R, W, W);
  GCounter<A> g;
  g.inner = detail::read_row(ix, out.data(), W);
  return g;
}

// GCounter::read of many counters on the GPU (crdt_gcounter_read, exact 128-bit sums).
template <class A>
std::vector<unsigned __int128> read_batch(Gpu &gpu, const std::vector<GCounter<A>> &cs) {
  Interner<A> ix;
  for (auto &c : cs) detail::intern_clock(ix, c.inner);
  ix.freeze();
  const size_t N = cs.size(), W = ix.size();
  std::vector<unsigned __int128> out(N, 0);
  if (N == 0 || W == 0) return out;
  std::vector<uint64_t> rows(N * W, 0);
  for (size_t i = 0; i < N; ++i) detail::write_row(ix, cs[i].inner, rows.data() + i * W);
  DeviceBuf<uint64_t> d(rows), w(2 * N);
  gpu.check(crdt_gcounter_read(gpu.ctx(), d.get(), N, W, W, w.get()), "crdt_gcounter_read");
  gpu.sync();
  auto h = w.download();
  for (size_t i = 0; i < N; ++i) out[i] = ((unsigned __int128)h[2 * i + 1] << 64) | h[2 * i];
  return out;
}

enum class Dir { Pos, Neg };  // pncounter.rs:36-41
template <class A>
struct PNOp {  // pncounter.rs:46-51
  Dot<A> dot;
  Dir dir;
};

template <class A>
class PNCounter {
 public:
  GCounter<A> p, n;  // pncounter.rs:30-31
  PNOp<A> inc(const A &a) const { return {p.inc(a), Dir::Pos}; }
  PNOp<A> dec(const A &a) const { return {n.inc(a), Dir::Neg}; }
  void apply(const PNOp<A> &op) { (op.dir == Dir::Pos ? p : n).apply(op.dot); }  // :59-68
  __int128 read() const { return (__int128)p.read() - (__int128)n.read(); }  // :110-115
  bool operator==(const PNCounter &o) const { return p == o.p && n == o.n; }
  void merge(Gpu &gpu, const PNCounter &other) {  // pncounter.rs:70-75
    *this = lub_many<A>(gpu, std::vector<PNCounter>{*this, other});
  }
};

// Rows of 2W words: P counters in [0, W), N counters in [W, 2W).
template <class A>
PNCounter<A> lub_many(Gpu &gpu, const std::vector<PNCounter<A>> &replicas) {
  Interner<A> ix;
  for (auto &r : replicas) {
    detail::intern_clock(ix, r.p.inner);
    detail::intern_clock(ix, r.n.inner);
  }
  ix.freeze();
  const size_t R = replicas.size(), W = ix.size();
  std::vector<uint64_t> rows(R * 2 * W, 0);
  for (size_t r = 0; r < R; ++r) {
    detail::write_row(ix, replicas[r].p.inner, rows.data() + r * 2 * W);
    detail::write_row(ix, replicas[r].n.inner, rows.data() + r * 2 * W + W);
  }
  auto out = detail::lattice_lub(gpu, crdt_pncounter_lub_many, "crdt_pncounter_lub_many", rows, R,
                                 2 * W, W);
  PNCounter<A> pn;
  if (W) {
    pn.p.inner = detail::read_row(ix, out.data(), W);
    pn.n.inner = detail::read_row(ix, out.data() + W, W);
  }
  return pn;
}

// ---- GSet (gset.rs) ---------------------------------------------------------------------------
template <class T>
class GSet {
 public:
  std::set<T> value;  // gset.rs:9
  void insert(const T &e) { value.insert(e); }  // gset.rs:69-71
  void apply(const T &e) { insert(e); }
  bool contains(const T &e) const { return value.count(e) != 0; }
  std::set<T> read() const { return value; }
  bool operator==(const GSet &o) const { return value == o.value; }
  void merge(Gpu &gpu, const GSet &other) {  // gset.rs:38-40
    *this = lub_many<T>(gpu, std::vector<GSet>{*this, other});
  }
};

template <class T>
GSet<T> lub_many(Gpu &gpu, const std::vector<GSet<T>> &replicas) {
  Interner<T> ix;
  for (auto &r : replicas)
    for (auto &e : r.value) ix.add(e);
  ix.freeze();
  const size_t R = replicas.size(), U = ix.size(), W = (U + 63) / 64;
  std::vector<uint64_t> rows(R * W, 0);
  for (size_t r = 0; r < R; ++r)
    for (auto &e : replicas[r].value) {
      const uint32_t p = ix.at(e);
      rows[r * W + p / 64] |= 1ull << (p % 64);
    }
  auto out = detail::lattice_lub(gpu, crdt_gset_lub_many, "crdt_gset_lub_many", rows, R, W, W);
  GSet<T> s;
  for (size_t w = 0; w < W; ++w)
    for (uint64_t x = out[w]; x; x &= x - 1) s.value.insert(ix.id(w * 64 + __builtin_ctzll(x)));
  return s;
}

// ---- LWWReg<V, u64 marker> (lwwreg.rs) ------------------------------------------------------
template <class V>
class LWWReg {
 public:
  V val{};
  uint64_t marker = 0;
  LWWReg() = default;
  LWWReg(V v, uint64_t m) : val(std::move(v)), marker(m) {}
  bool operator==(const LWWReg &o) const { return val == o.val && marker == o.marker; }
  // lwwreg.rs:84-98 (host; single update, not the batched path)
  std::optional<Error> update(V v, uint64_t m) {
    if (marker < m) {
      val = std::move(v);
      marker = m;
      return std::nullopt;
    }
    if (marker == m && !(v == val)) return Error::ConflictingMarker;
    return std::nullopt;
  }
  // FunkyCvRDT::merge (lwwreg.rs:43-45) on the GPU; on Err the register is unchanged.
  std::optional<Error> merge(Gpu &gpu, const LWWReg &other);
};

template <class V>
struct LwwLub {
  LWWReg<V> reg;
  std::optional<size_t> first_conflict;  // index of the first merge returning Err
};

// acc = replicas[0]; for r in replicas[1..] { acc.merge(r) } (errors leave acc unchanged)
template <class V>
LwwLub<V> lub_many(Gpu &gpu, const std::vector<LWWReg<V>> &replicas) {
  if (replicas.empty()) throw std::invalid_argument("LWWReg lub_many of no replicas");
  Interner<V> vals;
  for (auto &r : replicas) vals.add(r.val);
  vals.freeze();
  const size_t R = replicas.size();
  std::vector<uint64_t> m(R), v(R);
  for (size_t r = 0; r < R; ++r) {
    m[r] = replicas[r].marker;
    v[r] = vals.at(replicas[r].val);
  }
  DeviceBuf<uint64_t> dm(m), dv(v), om(1), ov(1), fc(1);
  gpu.check(crdt_lwwreg_lub_many(gpu.ctx(), dm.get(), dv.get(), 1, R, R, om.get(), ov.get(), fc.get(), 0),
            "crdt_lwwreg_lub_many");
  gpu.sync();
  LwwLub<V> out;
  out.reg = LWWReg<V>(vals.id(ov.download()[0]), om.download()[0]);
  const uint64_t f = fc.download()[0];
  if (f != UINT64_MAX) out.first_conflict = (size_t)f;
  return out;
}

template <class V>
std::optional<Error> LWWReg<V>::merge(Gpu &gpu, const LWWReg<V> &other) {
  Interner<V> vals;
  vals.add(val);
  vals.add(other.val);
  vals.freeze();
  std::vector<uint64_t> sm{marker}, sv{vals.at(val)}, om{other.marker}, ov{vals.at(other.val)};
  DeviceBuf<uint64_t> dsm(sm), dsv(sv), dom(om), dov(ov);
  DeviceBuf<uint8_t> conflict(1);
  gpu.check(crdt_lwwreg_merge_batch(gpu.ctx(), dsm.get(), dsv.get(), dom.get(), dov.get(), 1, conflict.get()),
            "crdt_lwwreg_merge_batch");
  gpu.sync();
  if (conflict.download()[0]) return Error::ConflictingMarker;
  marker = dsm.download()[0];
  val = vals.id(dsv.download()[0]);
  return std::nullopt;
}

// ---- ctx.rs + Orswot (orswot.rs) ------------------------------------------------------------
template <class A>
struct AddCtx {  // ctx.rs:19-26
  VClock<A> clock;
  Dot<A> dot;
};
template <class A>
struct RmCtx {  // ctx.rs:29-33
  VClock<A> clock;
};
template <class V, class A>
struct ReadCtx {  // ctx.rs:12-21
  VClock<A> add_clock, rm_clock;
  V val;
  AddCtx<A> derive_add_ctx(const A &actor) const {  // ctx.rs:42-48
    VClock<A> clock = add_clock;
    Dot<A> dot = clock.inc(actor);
    clock.apply(dot);
    return {clock, dot};
  }
  RmCtx<A> derive_rm_ctx() const { return {rm_clock}; }  // ctx.rs:50-54
};

template <class M, class A>
struct OrswotOp {  // orswot.rs:32-47
  bool is_add;
  Dot<A> dot;          // Add
  VClock<A> clock;     // Rm
  std::set<M> members;
};

template <class M, class A>
class Orswot {
 public:
  VClock<A> clock;                                 // orswot.rs:22
  std::unordered_map<M, VClock<A>> entries;        // orswot.rs:23
  std::map<VClock<A>, std::set<M>> deferred;       // orswot.rs:24

  bool operator==(const Orswot &o) const {
    return clock == o.clock && entries == o.entries && deferred == o.deferred;
  }

  // op builders (orswot.rs:196-227)
  OrswotOp<M, A> add(const M &m, const AddCtx<A> &ctx) const { return {true, ctx.dot, {}, {m}}; }
  OrswotOp<M, A> rm(const M &m, const RmCtx<A> &ctx) const { return {false, {}, ctx.clock, {m}}; }

  // CmRDT::apply (orswot.rs:55-79) — host-side op application
  void apply(const OrswotOp<M, A> &op) {
    if (op.is_add) {
      if (clock.get(op.dot.actor) >= op.dot.counter) return;
      for (auto &m : op.members) entries[m].apply(op.dot);
      clock.apply(op.dot);
      apply_deferred();
    } else {
      apply_rm(op.members, op.clock);
    }
  }
  ReadCtx<bool, A> contains(const M &m) const {  // orswot.rs:253-261
    auto it = entries.find(m);
    return {clock, it == entries.end() ? VClock<A>() : it->second, it != entries.end()};
  }
  ReadCtx<std::set<M>, A> read() const {  // orswot.rs:264-270
    std::set<M> v;
    for (auto &kv : entries) v.insert(kv.first);
    return {clock, clock, v};
  }

  void merge(Gpu &gpu, const Orswot &other);  // CvRDT::merge (orswot.rs:81-149) on the GPU

 private:
  void apply_rm(std::set<M> members, const VClock<A> &rm) {  // orswot.rs:230-250
    for (auto &m : members) {
      auto it = entries.find(m);
      if (it == entries.end()) continue;
      for (auto &kv : rm.dots)  // VClock::forget (vclock.rs:95-105)
        if (kv.second >= it->second.get(kv.first)) it->second.dots.erase(kv.first);
      if (it->second.is_empty()) entries.erase(it);
    }
    auto c = rm.partial_cmp(clock);
    if (!c.has_value() || *c == Ordering::Greater) deferred[rm].insert(members.begin(), members.end());
  }
  void apply_deferred() {  // orswot.rs:281-286
    auto d = std::move(deferred);
    deferred.clear();
    for (auto &kv : d) apply_rm(kv.second, kv.first);
  }
};

// acc = Orswot::new(); for r in replicas { acc.merge(r) }   — on the GPU
template <class M, class A>
Orswot<M, A> lub_many(Gpu &gpu, const std::vector<Orswot<M, A>> &replicas) {
  Interner<A> ax;
  Interner<M> mx;
  for (auto &r : replicas) {
    detail::intern_clock(ax, r.clock);
    for (auto &kv : r.entries) {
      mx.add(kv.first);
      detail::intern_clock(ax, kv.second);
    }
    for (auto &kv : r.deferred) {
      detail::intern_clock(ax, kv.first);
      for (auto &m : kv.second) mx.add(m);
    }
  }
  ax.freeze();
  mx.freeze();
  Orswot<M, A> out;
  const size_t R = replicas.size(), A_ = ax.size(), M_ = mx.size();
  if (R == 0 || A_ == 0) return out;
  const size_t Mm = M_ ? M_ : 1, Mw = (Mm + 63) / 64;
  std::vector<uint64_t> clock(R * A_, 0), entries(R * Mm * A_, 0), dcl, dmem;
  for (size_t r = 0; r < R; ++r) {
    detail::write_row(ax, replicas[r].clock, clock.data() + r * A_);
    for (auto &kv : replicas[r].entries)
      detail::write_row(ax, kv.second, entries.data() + (r * Mm + mx.at(kv.first)) * A_);
    for (auto &kv : replicas[r].deferred) {
      dcl.resize(dcl.size() + A_, 0);
      detail::write_row(ax, kv.first, dcl.data() + dcl.size() - A_);
      dmem.resize(dmem.size() + Mw, 0);
      for (auto &m : kv.second) {
        const uint32_t p = mx.at(m);
        dmem[dmem.size() - Mw + p / 64] |= 1ull << (p % 64);
      }
    }
  }
  const size_t D = dcl.size() / A_;
  DeviceBuf<uint64_t> dc(clock), de(entries), ddc(dcl), ddm(dmem), oc(A_), oe(Mm * A_), odm(D * Mw);
  DeviceBuf<uint8_t> okeep(D);
  const size_t off[2] = {0, D};
  crdt_orswot_batch in{1, R, Mm, A_, dc.get(), A_, R * A_, de.get(), A_, Mm * A_, R * Mm * A_,
                       D ? off : nullptr, ddc.get(), ddm.get()};
  crdt_orswot_out o{oc.get(), oe.get(), okeep.get(), odm.get()};
  gpu.check(crdt_orswot_lub_many(gpu.ctx(), &in, &o), "crdt_orswot_lub_many");
  gpu.sync();
  auto hc = oc.download(), he = oe.download();
  out.clock = detail::read_row(ax, hc.data(), A_);
  for (size_t m = 0; m < M_; ++m) {
    VClock<A> e = detail::read_row(ax, he.data() + m * A_, A_);
    if (!e.is_empty()) out.entries.emplace(mx.id(m), std::move(e));
  }
  if (D) {
    auto keep = okeep.download();
    auto mem = odm.download();
    for (size_t d = 0; d < D; ++d) {
      if (!keep[d]) continue;
      std::set<M> ms;
      for (size_t w = 0; w < Mw; ++w)
        for (uint64_t x = mem[d * Mw + w]; x; x &= x - 1) ms.insert(mx.id(w * 64 + __builtin_ctzll(x)));
      out.deferred[detail::read_row(ax, dcl.data() + d * A_, A_)] = ms;
    }
  }
  return out;
}

template <class M, class A>
void Orswot<M, A>::merge(Gpu &gpu, const Orswot<M, A> &other) {
  *this = lub_many<M, A>(gpu, {*this, other});
}

}  // namespace crdts
