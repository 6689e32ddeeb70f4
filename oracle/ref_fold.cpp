// ORACLE — test infrastructure only.  Not part of the product and never linked into it.
//
// A CPU restatement of the reference `crdts` 3.0.0 merge paths (rust-crdt; the Rust crate
// cannot be built here: no cargo/rustc, see DESIGN.md "Oracle").  The containers mirror the
// reference's: VClock = ordered map actor -> counter (BTreeMap, vclock.rs:56-60), Orswot
// entries = hash map member -> VClock, deferred = map VClock -> member set (orswot.rs:20-25).
// Every function follows the cited reference lines statement by statement.  It is pinned by
// the reference's own known-answer tests (tests/golden/kat_*.json via oracle/oracle.py, whose
// pure-Python twin is cross-checked against this file) and is used by tests/ as the parity
// checker and by bench.py as the `cpu_baseline` (kind "port").
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library.
#include <atomic>
#include <chrono>
#include <thread>
#include <cstdint>
#include <cstring>
#include <map>
#include <set>
#include <unordered_map>
#include <vector>

namespace oracle {

using Actor = uint32_t;
using Member = uint32_t;
using u64 = uint64_t;

// ---- VClock (vclock.rs) ---------------------------------------------------------------
struct VClock {
  std::map<Actor, u64> dots;  // vclock.rs:59

  u64 get(Actor a) const {  // vclock.rs:207-209
    auto it = dots.find(a);
    return it == dots.end() ? 0 : it->second;
  }
  void apply_dot(Actor a, u64 counter) {  // vclock.rs:155-159
    if (get(a) < counter) dots[a] = counter;
  }
  void merge(VClock &&other) {  // vclock.rs:130-136 (consumes other)
    for (auto &kv : other.dots) apply_dot(kv.first, kv.second);
    other.dots.clear();
  }
  void forget(const VClock &other) {  // vclock.rs:95-105
    for (auto &kv : other.dots)
      if (kv.second >= get(kv.first)) dots.erase(kv.first);
  }
  bool empty() const { return dots.empty(); }
  bool operator==(const VClock &o) const { return dots == o.dots; }
  bool operator<(const VClock &o) const { return dots < o.dots; }  // map key only
  // partial_cmp (vclock.rs:68-80): 0 Equal, 1 Greater, -1 Less, 2 None
  int partial_cmp(const VClock &other) const {
    if (*this == other) return 0;
    bool ge = true;
    for (auto &kv : other.dots)
      if (!(get(kv.first) >= kv.second)) { ge = false; break; }
    if (ge) return 1;
    bool le = true;
    for (auto &kv : dots)
      if (!(other.get(kv.first) >= kv.second)) { le = false; break; }
    if (le) return -1;
    return 2;
  }
  // self >= other  <=>  partial_cmp(self, other) in {Greater, Equal}
  bool geq(const VClock &other) const {
    int c = partial_cmp(other);
    return c == 0 || c == 1;
  }
  static VClock intersection(const VClock &left, const VClock &right) {  // vclock.rs:218-227
    VClock out;
    for (auto &kv : left.dots)
      if (right.get(kv.first) == kv.second) out.dots.insert(kv);
    return out;
  }
  VClock clone_without(const VClock &base) const {  // vclock.rs:148-152
    VClock c = *this;
    c.forget(base);
    return c;
  }
};

static VClock vclock_from_row(const u64 *row, size_t A) {
  VClock v;
  for (size_t a = 0; a < A; ++a)
    if (row[a]) v.dots.emplace_hint(v.dots.end(), (Actor)a, row[a]);
  return v;
}
static void vclock_to_row(const VClock &v, u64 *row, size_t A) {
  std::memset(row, 0, A * 8);
  for (auto &kv : v.dots) row[kv.first] = kv.second;
}

// ---- LWWReg (lwwreg.rs) --------------------------------------------------------------
struct LWWReg {
  u64 val, marker;
  int update(u64 v, u64 m) {  // lwwreg.rs:84-98; returns 1 on Err(ConflictingMarker)
    if (marker < m) {
      val = v;
      marker = m;
      return 0;
    } else if (marker == m && v != val) {
      return 1;
    }
    return 0;
  }
};

// ---- Orswot (orswot.rs) --------------------------------------------------------------
struct Orswot {
  VClock clock;                                   // orswot.rs:22
  std::unordered_map<Member, VClock> entries;     // orswot.rs:23
  std::map<VClock, std::set<Member>> deferred;    // orswot.rs:24 (keyed by whole clock)

  void apply_rm(std::set<Member> members, VClock clock_rm) {  // orswot.rs:230-250
    for (Member m : members) {
      auto it = entries.find(m);
      if (it != entries.end()) {
        it->second.forget(clock_rm);
        if (it->second.empty()) entries.erase(it);
      }
    }
    int c = clock_rm.partial_cmp(clock);
    if (c == 2 /*None*/ || c == 1 /*Greater*/) {
      auto it = deferred.find(clock_rm);
      if (it != deferred.end()) it->second.insert(members.begin(), members.end());
      else deferred.emplace(std::move(clock_rm), std::move(members));
    }
  }
  void apply_deferred() {  // orswot.rs:281-286
    auto d = std::move(deferred);
    deferred.clear();
    for (auto &kv : d) apply_rm(kv.second, kv.first);
  }
  void apply_add(Actor a, u64 counter, const std::set<Member> &members) {  // orswot.rs:59-72
    if (clock.get(a) >= counter) return;  // we've already seen this op
    for (Member m : members) entries[m].apply_dot(a, counter);
    clock.apply_dot(a, counter);
    apply_deferred();
  }
  void merge(Orswot &&other) {  // orswot.rs:81-149
    // :84-106 rebuild self.entries
    std::unordered_map<Member, VClock> kept;
    kept.reserve(entries.size());
    for (auto &kv : entries) {
      if (other.entries.find(kv.first) == other.entries.end()) {
        if (other.clock.geq(kv.second)) {
          // other has seen this entry and dropped it
        } else {
          VClock c = std::move(kv.second);
          c.forget(other.clock);
          kept.emplace(kv.first, std::move(c));
        }
      } else {
        kept.emplace(kv.first, std::move(kv.second));
      }
    }
    entries = std::move(kept);
    // :108-138
    for (auto &kv : other.entries) {
      auto it = entries.find(kv.first);
      if (it != entries.end()) {
        VClock common = VClock::intersection(kv.second, it->second);
        common.merge(kv.second.clone_without(clock));
        common.merge(it->second.clone_without(other.clock));
        if (common.empty()) entries.erase(it);
        else it->second = std::move(common);
      } else {
        if (clock.geq(kv.second)) {
          // we've seen this entry and dropped it
        } else {
          VClock c = std::move(kv.second);
          c.forget(clock);
          entries.emplace(kv.first, std::move(c));
        }
      }
    }
    // :141-143 merge deferred removals
    for (auto &kv : other.deferred) apply_rm(kv.second, kv.first);
    // :145
    clock.merge(std::move(other.clock));
    // :147
    apply_deferred();
  }
};

// ---- MVReg<u64, A> (mvreg.rs) ------------------------------------------------------------
struct MVReg {
  std::vector<std::pair<VClock, u64>> vals;  // mvreg.rs:34 (ordered Vec)

  static bool lt(const VClock &x, const VClock &y) { return x.partial_cmp(y) == -1; }
  void forget(const VClock &clock) {  // mvreg.rs:88-104
    std::vector<std::pair<VClock, u64>> out;
    out.reserve(vals.size());
    for (auto &cv : vals) {
      VClock c = cv.first;  // .clone().into_iter()
      c.forget(clock);
      if (!c.empty()) out.emplace_back(std::move(c), cv.second);
    }
    vals = std::move(out);
  }
  void merge(MVReg &&other) {  // mvreg.rs:112-128
    std::vector<std::pair<VClock, u64>> kept;
    for (auto &cv : vals) {
      size_t n = 0;
      for (auto &o : other.vals) n += lt(cv.first, o.first);
      if (n == 0) kept.push_back(std::move(cv));
    }
    vals = std::move(kept);
    std::vector<std::pair<VClock, u64>> add;
    for (auto &o : other.vals) {
      size_t n = 0;
      for (auto &s : vals) n += lt(o.first, s.first);
      if (n != 0) continue;
      bool all_ne = true;
      for (auto &s : vals) all_ne &= !(o.first == s.first);
      if (all_ne) add.push_back(std::move(o));
    }
    for (auto &x : add) vals.push_back(std::move(x));
  }
};

// ---- Map<u32, MVReg<u64>, A> (map.rs) ---------------------------------------------------------
struct MapEntry {
  VClock clock;  // map.rs:42
  MVReg val;     // map.rs:45
};

struct MapMV {
  VClock clock;                                      // map.rs:35
  std::map<uint32_t, MapEntry> entries;              // map.rs:36 (BTreeMap)
  std::map<VClock, std::set<uint32_t>> deferred;     // map.rs:37 (keyed by whole clock)
  uint64_t *peak = nullptr;  // test instrumentation: max values per key after each entry join

  void apply_keyset_rm(std::set<uint32_t> keyset, VClock clock_rm) {  // map.rs:318-348
    for (uint32_t key : keyset) {
      auto it = entries.find(key);
      if (it != entries.end()) {
        it->second.clock.forget(clock_rm);
        if (it->second.clock.empty()) entries.erase(it);
        else it->second.val.forget(clock_rm);
      }
    }
    int c = clock.partial_cmp(clock_rm);
    if (c == 2 /*None*/ || c == -1 /*Less*/) {
      auto it = deferred.find(clock_rm);
      if (it != deferred.end()) it->second.insert(keyset.begin(), keyset.end());
      else deferred.emplace(std::move(clock_rm), std::move(keyset));
    }
  }
  void apply_deferred() {  // map.rs:311-316
    auto d = std::move(deferred);
    deferred.clear();
    for (auto &kv : d) apply_keyset_rm(kv.second, kv.first);
  }
  void merge(MapMV &&other) {  // map.rs:140-220
    // :142-165 rebuild self.entries
    for (auto it = entries.begin(); it != entries.end();) {
      if (other.entries.find(it->first) == other.entries.end()) {
        MapEntry &e = it->second;
        if (other.clock.geq(e.clock)) {
          it = entries.erase(it);  // other has seen this entry and dropped it
          continue;
        }
        e.clock.forget(other.clock);
        VClock removed_information = other.clock;
        removed_information.forget(e.clock);
        e.val.forget(removed_information);
      }
      ++it;
    }
    // :167-210
    for (auto &kv : other.entries) {
      MapEntry &entry = kv.second;
      auto it = entries.find(kv.first);
      if (it != entries.end()) {
        MapEntry &our = it->second;
        VClock common = VClock::intersection(entry.clock, our.clock);
        common.merge(entry.clock.clone_without(clock));
        common.merge(our.clock.clone_without(other.clock));
        if (common.empty()) {
          entries.erase(it);
        } else {
          our.val.merge(std::move(entry.val));
          VClock deleted = entry.clock;
          deleted.merge(VClock(our.clock));
          deleted.forget(common);
          our.val.forget(deleted);
          our.clock = std::move(common);
        }
      } else {
        if (clock.geq(entry.clock)) {
          // we've seen this entry and dropped it
        } else {
          entry.clock.forget(clock);
          VClock we_deleted = clock;
          we_deleted.forget(entry.clock);
          entry.val.forget(we_deleted);
          entries.emplace(kv.first, std::move(entry));
        }
      }
    }
    if (peak)
      for (auto &kv : entries)
        if (kv.second.val.vals.size() > peak[kv.first]) peak[kv.first] = kv.second.val.vals.size();
    // :213-215
    for (auto &kv : other.deferred) apply_keyset_rm(kv.second, kv.first);
    clock.merge(std::move(other.clock));  // :217
    apply_deferred();                     // :219
  }
};

}  // namespace oracle

using namespace oracle;

static double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

extern "C" {

// ---- VClock / GCounter / PNCounter ----------------------------------------------------
// Left fold from VClock::new() over R dense rows (W counters each); returns fold seconds
// (ingest into maps is outside the timed region, as the reference receives map states).
double oracle_vclock_fold(const uint64_t *rows, size_t R, size_t W, size_t stride,
                          uint64_t *out) {
  std::vector<VClock> reps;
  reps.reserve(R);
  for (size_t r = 0; r < R; ++r) reps.push_back(vclock_from_row(rows + r * stride, W));
  double t0 = now_s();
  VClock acc;
  for (auto &r : reps) acc.merge(std::move(r));  // GCounter::merge gcounter.rs:44-48
  double t1 = now_s();
  vclock_to_row(acc, out, W);
  return t1 - t0;
}

// PNCounter rows hold P in [0,A) and N in [A,2A) (pncounter.rs:70-75 merges p then n).
double oracle_pncounter_fold(const uint64_t *rows, size_t R, size_t A, size_t stride,
                             uint64_t *out) {
  std::vector<std::pair<VClock, VClock>> reps;
  reps.reserve(R);
  for (size_t r = 0; r < R; ++r)
    reps.emplace_back(vclock_from_row(rows + r * stride, A), vclock_from_row(rows + r * stride + A, A));
  double t0 = now_s();
  VClock p, n;
  for (auto &r : reps) {
    p.merge(std::move(r.first));
    n.merge(std::move(r.second));
  }
  double t1 = now_s();
  vclock_to_row(p, out, A);
  vclock_to_row(n, out + A, A);
  return t1 - t0;
}

// The same left fold split over `threads` host threads (SURVEY §8d CPU timing (2)): thread t
// folds rows [t*R/T, (t+1)*R/T) from T::new(), then the T partials are merged in thread order
// (merge is a join: any split gives the same result).  pn = 1: rows are PNCounter P | N halves
// of W/2 counters each.  Ingest into maps runs before the clock starts; the timed region is
// the parallel fold plus the final combine.  Returns seconds.
double oracle_counter_fold_mt(const uint64_t *rows, size_t R, size_t W, size_t stride, int pn, int threads,
                              uint64_t *out) {
  const size_t T = threads < 1 ? 1 : (size_t)threads;
  const size_t H = pn ? W / 2 : W;
  std::vector<std::vector<VClock>> in_p(T), in_n(T);
  std::vector<VClock> acc_p(T), acc_n(T);
  std::atomic<int> ready{0}, go{0};
  std::vector<std::thread> pool;
  for (size_t t = 0; t < T; ++t)
    pool.emplace_back([&, t] {
      const size_t lo = t * R / T, hi = (t + 1) * R / T;
      for (size_t r = lo; r < hi; ++r) {
        in_p[t].push_back(vclock_from_row(rows + r * stride, H));
        if (pn) in_n[t].push_back(vclock_from_row(rows + r * stride + H, H));
      }
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (size_t i = 0; i < in_p[t].size(); ++i) {
        acc_p[t].merge(std::move(in_p[t][i]));  // gcounter.rs:44-48 / vclock.rs:130-136
        if (pn) acc_n[t].merge(std::move(in_n[t][i]));  // pncounter.rs:70-75
      }
    });
  while (ready.load() < (int)T) std::this_thread::yield();
  double t0 = now_s();
  go.store(1, std::memory_order_release);
  for (auto &th : pool) th.join();
  VClock p, n;
  for (size_t t = 0; t < T; ++t) {
    p.merge(std::move(acc_p[t]));
    if (pn) n.merge(std::move(acc_n[t]));
  }
  double t1 = now_s();
  vclock_to_row(p, out, H);
  if (pn) vclock_to_row(n, out + H, H);
  return t1 - t0;
}

// SURVEY §8d CPU timing (3), "the honest CPU roofline": the same fold on the DENSE SoA rows
// (elementwise max of u64 rows, the restatement of vclock.rs:130-136 under the dense convention),
// split over `threads` host threads by row ranges, partials maxed at the end.  Returns seconds.
double oracle_dense_max_mt(const uint64_t *rows, size_t R, size_t W, size_t stride, int threads, uint64_t *out) {
  const size_t T = threads < 1 ? 1 : (size_t)threads;
  std::vector<std::vector<uint64_t>> part(T, std::vector<uint64_t>(W, 0));
  std::atomic<int> ready{0}, go{0};
  std::vector<std::thread> pool;
  for (size_t t = 0; t < T; ++t)
    pool.emplace_back([&, t] {
      const size_t lo = t * R / T, hi = (t + 1) * R / T;
      uint64_t *acc = part[t].data();
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (size_t r = lo; r < hi; ++r) {
        const uint64_t *row = rows + r * stride;
        for (size_t a = 0; a < W; ++a) acc[a] = row[a] > acc[a] ? row[a] : acc[a];
      }
    });
  while (ready.load() < (int)T) std::this_thread::yield();
  double t0 = now_s();
  go.store(1, std::memory_order_release);
  for (auto &th : pool) th.join();
  for (size_t a = 0; a < W; ++a) out[a] = 0;
  for (size_t t = 0; t < T; ++t)
    for (size_t a = 0; a < W; ++a) out[a] = part[t][a] > out[a] ? part[t][a] : out[a];
  double t1 = now_s();
  return t1 - t0;
}

// Pairwise: self[i].merge(other[i]) on dense rows (A counters), in place.
void oracle_vclock_merge_pairs(uint64_t *self, const uint64_t *other, size_t N, size_t A) {
  for (size_t i = 0; i < N; ++i) {
    VClock s = vclock_from_row(self + i * A, A);
    s.merge(vclock_from_row(other + i * A, A));
    vclock_to_row(s, self + i * A, A);
  }
}

// VClock::forget (vclock.rs:95-105) and partial_cmp (vclock.rs:68-80) on dense rows.
void oracle_vclock_forget(uint64_t *self, const uint64_t *other, size_t A) {
  VClock s = vclock_from_row(self, A);
  s.forget(vclock_from_row(other, A));
  vclock_to_row(s, self, A);
}
int oracle_vclock_partial_cmp(const uint64_t *a, const uint64_t *b, size_t A) {
  return vclock_from_row(a, A).partial_cmp(vclock_from_row(b, A));
}

// ---- GSet (gset.rs:38-40): union of ordered sets, dense bitmap in/out -------------------
double oracle_gset_fold(const uint64_t *rows, size_t R, size_t words, size_t stride,
                        uint64_t *out) {
  std::vector<std::set<uint64_t>> reps(R);
  for (size_t r = 0; r < R; ++r)
    for (size_t w = 0; w < words; ++w) {
      uint64_t x = rows[r * stride + w];
      while (x) {
        int b = __builtin_ctzll(x);
        x &= x - 1;
        reps[r].insert(w * 64 + b);
      }
    }
  double t0 = now_s();
  std::set<uint64_t> acc;
  for (auto &s : reps)
    for (uint64_t e : s) acc.insert(e);  // other.value.into_iter().for_each(insert)
  double t1 = now_s();
  std::memset(out, 0, words * 8);
  for (uint64_t e : acc) out[e / 64] |= 1ull << (e % 64);
  return t1 - t0;
}

// ---- LWWReg fold: acc = r[0]; acc.merge(r[i]) ignoring (but recording) Err ------------------
double oracle_lwwreg_fold(const uint64_t *marker, const uint64_t *val, size_t R,
                          uint64_t *out_marker, uint64_t *out_val, uint64_t *first_conflict) {
  double t0 = now_s();
  LWWReg acc{val[0], marker[0]};
  uint64_t first = ~0ull;
  for (size_t i = 1; i < R; ++i)
    if (acc.update(val[i], marker[i]) && first == ~0ull) first = i;
  double t1 = now_s();
  *out_marker = acc.marker;
  *out_val = acc.val;
  *first_conflict = first;
  return t1 - t0;
}

// ---- Orswot fold from Orswot::new() over R dense replicas ----------------------------------
// Replica r: clock[r*A + a], entries[r*M*A + m*A + a]; deferred of replica r are
// d in [def_off[r], def_off[r+1]) with rm clock def_clock[d*A..] and member bitmap
// def_members[d*Mw..].  Output: out_clock[A], out_entries[M*A]; surviving deferred removes
// are written as out_def_clock[k*A..], out_def_members[k*Mw..] for k < *out_ndef (caller
// provides room for max_def).  Returns fold seconds (ingest excluded).
double oracle_orswot_fold(const uint64_t *clock, const uint64_t *entries, size_t R, size_t M,
                          size_t A, const uint64_t *def_off, const uint64_t *def_clock,
                          const uint64_t *def_members, uint64_t *out_clock, uint64_t *out_entries,
                          uint64_t *out_def_clock, uint64_t *out_def_members, size_t max_def,
                          size_t *out_ndef) {
  const size_t Mw = (M + 63) / 64;
  std::vector<Orswot> reps(R);
  for (size_t r = 0; r < R; ++r) {
    Orswot &o = reps[r];
    o.clock = vclock_from_row(clock + r * A, A);
    for (size_t m = 0; m < M; ++m) {
      VClock e = vclock_from_row(entries + (r * M + m) * A, A);
      if (!e.empty()) o.entries.emplace((Member)m, std::move(e));
    }
    if (def_off)
      for (uint64_t d = def_off[r]; d < def_off[r + 1]; ++d) {
        VClock rm = vclock_from_row(def_clock + d * A, A);
        std::set<Member> mem;
        for (size_t w = 0; w < Mw; ++w) {
          uint64_t x = def_members[d * Mw + w];
          while (x) {
            int b = __builtin_ctzll(x);
            x &= x - 1;
            mem.insert((Member)(w * 64 + b));
          }
        }
        auto it = o.deferred.find(rm);
        if (it != o.deferred.end()) it->second.insert(mem.begin(), mem.end());
        else o.deferred.emplace(std::move(rm), std::move(mem));
      }
  }
  double t0 = now_s();
  Orswot acc;
  for (auto &r : reps) acc.merge(std::move(r));
  double t1 = now_s();
  vclock_to_row(acc.clock, out_clock, A);
  std::memset(out_entries, 0, M * A * 8);
  for (auto &kv : acc.entries) vclock_to_row(kv.second, out_entries + (size_t)kv.first * A, A);
  size_t k = 0;
  for (auto &kv : acc.deferred) {
    if (k < max_def) {
      vclock_to_row(kv.first, out_def_clock + k * A, A);
      std::memset(out_def_members + k * Mw, 0, Mw * 8);
      for (Member m : kv.second) out_def_members[k * Mw + m / 64] |= 1ull << (m % 64);
    }
    ++k;
  }
  *out_ndef = k;
  return t1 - t0;
}

// ---- Orswot CmRDT::apply streams (orswot.rs:55-79) from Orswot::new() -----------------------
// State s applies ops [op_off[s], op_off[s+1]): kind 0 = Op::Add { dot (actor, counter) },
// 1 = Op::Rm { clock rm_clock[rm_row*A..] }, members mem[mem_off[o]..mem_off[o+1]) (the layout
// of crdt_orswot_ops).  Output per state: clock[s*A..], entries[(s*M + m)*A..] and the number of
// deferred removes ndef[s].  Returns apply seconds (op ingest into sets / maps excluded).
double oracle_orswot_apply_streams(size_t N, size_t M, size_t A, const uint64_t *op_off, const uint8_t *kind,
                                   const uint32_t *actor, const uint64_t *counter, const uint32_t *rm_row,
                                   const uint64_t *rm_clock, const uint64_t *mem_off, const uint32_t *mem,
                                   uint64_t *out_clock, uint64_t *out_entries, uint64_t *out_ndef) {
  struct OpIn {
    int kind;
    Actor a;
    u64 k;
    VClock rm;
    std::set<Member> ms;
  };
  std::vector<std::vector<OpIn>> streams(N);
  for (size_t s = 0; s < N; ++s)
    for (uint64_t o = op_off[s]; o < op_off[s + 1]; ++o) {
      OpIn op{kind[o], actor ? actor[o] : 0, counter ? counter[o] : 0, {}, {}};
      if (op.kind == 1) op.rm = vclock_from_row(rm_clock + (size_t)rm_row[o] * A, A);
      for (uint64_t j = mem_off[o]; j < mem_off[o + 1]; ++j) op.ms.insert(mem[j]);
      streams[s].push_back(std::move(op));
    }
  std::vector<Orswot> st(N);
  double t0 = now_s();
  for (size_t s = 0; s < N; ++s)
    for (auto &op : streams[s]) {
      if (op.kind == 0) st[s].apply_add(op.a, op.k, op.ms);
      else st[s].apply_rm(std::move(op.ms), std::move(op.rm));  // orswot.rs:74-76
    }
  double t1 = now_s();
  for (size_t s = 0; s < N; ++s) {
    vclock_to_row(st[s].clock, out_clock + s * A, A);
    std::memset(out_entries + s * M * A, 0, M * A * 8);
    for (auto &kv : st[s].entries) vclock_to_row(kv.second, out_entries + (s * M + kv.first) * A, A);
    out_ndef[s] = st[s].deferred.size();
  }
  return t1 - t0;
}

// ---- Map<u32, MVReg<u64>> fold from Map::new() over R dense replicas ------------------------
// Replica r: clock[r*A + a]; entry clock ec[(r*K + k)*A + a] (key absent <=> row all 0); val
// slots s < V: clock vclk[((r*K + k)*V + s)*A + a] (slot empty <=> row all 0, used slots come
// first, in Vec order) and value vval[(r*K + k)*V + s].  Deferred removes of replica r are
// d in [def_off[r], def_off[r+1]): rm clock def_clock[d*A..], key bitmap def_keys[d*Kw..].
// Output (dense, Vout slots per key): out_clock[A], out_ec[K*A], out_vclk[K*Vout*A],
// out_vval[K*Vout], out_nval[K] (true number of vals; > Vout means the slots overflowed), and
// the surviving deferred removes as in oracle_orswot_fold; out_peak[K] (may be NULL) = the most
// values a key held after any step's entry join.  Returns fold seconds.
double oracle_map_fold(const uint64_t *clock, const uint64_t *ec, const uint64_t *vclk,
                       const uint64_t *vval, size_t R, size_t K, size_t A, size_t V,
                       const uint64_t *def_off, const uint64_t *def_clock, const uint64_t *def_keys,
                       size_t Vout, uint64_t *out_clock, uint64_t *out_ec, uint64_t *out_vclk,
                       uint64_t *out_vval, uint64_t *out_nval, uint64_t *out_def_clock,
                       uint64_t *out_def_keys, size_t max_def, size_t *out_ndef,
                       uint64_t *out_peak) {
  const size_t Kw = (K + 63) / 64;
  std::vector<MapMV> reps(R);
  for (size_t r = 0; r < R; ++r) {
    MapMV &m = reps[r];
    m.clock = vclock_from_row(clock + r * A, A);
    for (size_t k = 0; k < K; ++k) {
      VClock e = vclock_from_row(ec + (r * K + k) * A, A);
      if (e.empty()) continue;
      MapEntry ent;
      ent.clock = std::move(e);
      for (size_t s = 0; s < V; ++s) {
        VClock c = vclock_from_row(vclk + ((r * K + k) * V + s) * A, A);
        if (!c.empty()) ent.val.vals.emplace_back(std::move(c), vval[(r * K + k) * V + s]);
      }
      m.entries.emplace((uint32_t)k, std::move(ent));
    }
    if (def_off)
      for (uint64_t d = def_off[r]; d < def_off[r + 1]; ++d) {
        VClock rm = vclock_from_row(def_clock + d * A, A);
        std::set<uint32_t> keys;
        for (size_t w = 0; w < Kw; ++w) {
          uint64_t x = def_keys[d * Kw + w];
          while (x) {
            int b = __builtin_ctzll(x);
            x &= x - 1;
            keys.insert((uint32_t)(w * 64 + b));
          }
        }
        auto it = m.deferred.find(rm);
        if (it != m.deferred.end()) it->second.insert(keys.begin(), keys.end());
        else m.deferred.emplace(std::move(rm), std::move(keys));
      }
  }
  if (out_peak) std::memset(out_peak, 0, K * 8);
  double t0 = now_s();
  MapMV acc;
  acc.peak = out_peak;
  for (auto &r : reps) acc.merge(std::move(r));
  double t1 = now_s();
  vclock_to_row(acc.clock, out_clock, A);
  std::memset(out_ec, 0, K * A * 8);
  std::memset(out_vclk, 0, K * Vout * A * 8);
  std::memset(out_vval, 0, K * Vout * 8);
  std::memset(out_nval, 0, K * 8);
  for (auto &kv : acc.entries) {
    const size_t k = kv.first;
    vclock_to_row(kv.second.clock, out_ec + k * A, A);
    out_nval[k] = kv.second.val.vals.size();
    size_t s = 0;
    for (auto &cv : kv.second.val.vals) {
      if (s >= Vout) break;
      vclock_to_row(cv.first, out_vclk + (k * Vout + s) * A, A);
      out_vval[k * Vout + s] = cv.second;
      ++s;
    }
  }
  size_t k = 0;
  for (auto &kv : acc.deferred) {
    if (k < max_def) {
      vclock_to_row(kv.first, out_def_clock + k * A, A);
      std::memset(out_def_keys + k * Kw, 0, Kw * 8);
      for (uint32_t key : kv.second) out_def_keys[k * Kw + key / 64] |= 1ull << (key % 64);
    }
    ++k;
  }
  *out_ndef = k;
  return t1 - t0;
}


// ---- Multi-threaded CPU baselines (SURVEY §8d CPU timing (2), configs 3 and 4) ----------------
// Orswot: thread t ingests and folds replicas [t*R/T, (t+1)*R/T) from Orswot::new(), then the T
// partial states are merged in thread order (orswot.rs:81-149 is a join on the states a fold
// produces: tests/test_oracle_twins.py checks tree == left fold, tests/test_oracle_mt.py this
// split).  Timed: the parallel folds plus the final merges.  Output as oracle_orswot_fold.
double oracle_orswot_fold_mt(const uint64_t *clock, const uint64_t *entries, size_t R, size_t M, size_t A,
                             const uint64_t *def_off, const uint64_t *def_clock, const uint64_t *def_members,
                             int threads, uint64_t *out_clock, uint64_t *out_entries, uint64_t *out_def_clock,
                             uint64_t *out_def_members, size_t max_def, size_t *out_ndef) {
  const size_t T = threads < 1 ? 1 : (size_t)threads, Mw = (M + 63) / 64;
  std::vector<Orswot> part(T);
  std::atomic<int> ready{0}, go{0};
  std::vector<std::thread> pool;
  for (size_t t = 0; t < T; ++t)
    pool.emplace_back([&, t] {
      const size_t lo = t * R / T, hi = (t + 1) * R / T;
      std::vector<Orswot> reps(hi - lo);
      for (size_t r = lo; r < hi; ++r) {  // ingest, as oracle_orswot_fold
        Orswot &o = reps[r - lo];
        o.clock = vclock_from_row(clock + r * A, A);
        for (size_t m = 0; m < M; ++m) {
          VClock e = vclock_from_row(entries + (r * M + m) * A, A);
          if (!e.empty()) o.entries.emplace((Member)m, std::move(e));
        }
        if (def_off)
          for (uint64_t d = def_off[r]; d < def_off[r + 1]; ++d) {
            VClock rm = vclock_from_row(def_clock + d * A, A);
            std::set<Member> mem;
            for (size_t w = 0; w < Mw; ++w)
              for (uint64_t x = def_members[d * Mw + w]; x; x &= x - 1) mem.insert((Member)(w * 64 + __builtin_ctzll(x)));
            auto it = o.deferred.find(rm);
            if (it != o.deferred.end()) it->second.insert(mem.begin(), mem.end());
            else o.deferred.emplace(std::move(rm), std::move(mem));
          }
      }
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (auto &r : reps) part[t].merge(std::move(r));
    });
  while (ready.load() < (int)T) std::this_thread::yield();
  const double t0 = now_s();
  go.store(1, std::memory_order_release);
  for (auto &th : pool) th.join();
  Orswot acc = std::move(part[0]);
  for (size_t t = 1; t < T; ++t) acc.merge(std::move(part[t]));
  const double t1 = now_s();
  vclock_to_row(acc.clock, out_clock, A);
  std::memset(out_entries, 0, M * A * 8);
  for (auto &kv : acc.entries) vclock_to_row(kv.second, out_entries + (size_t)kv.first * A, A);
  size_t k = 0;
  for (auto &kv : acc.deferred) {
    if (k < max_def) {
      vclock_to_row(kv.first, out_def_clock + k * A, A);
      std::memset(out_def_members + k * Mw, 0, Mw * 8);
      for (Member m : kv.second) out_def_members[k * Mw + m / 64] |= 1ull << (m % 64);
    }
    ++k;
  }
  *out_ndef = k;
  return t1 - t0;
}

// Map<u32, MVReg<u64>>: the fold is not associative, so the threads split KEYS, not
// replicas — keys are independent given the replica clocks and the deferred list (map.rs:140-220:
// the entry loop is per key, the clock merge and the removes' survival see only clocks).  Thread t
// folds every replica restricted to keys [t*K/T, (t+1)*K/T), with every deferred remove restricted
// to those keys (possibly to none: its clock still joins acc.deferred as the reference's does).
// Timed: the parallel folds.  Output as oracle_map_fold (the survivors' key sets are the union of
// the threads' restrictions; every thread keeps the same surviving clocks).
double oracle_map_fold_mt(const uint64_t *clock, const uint64_t *ec, const uint64_t *vclk, const uint64_t *vval,
                          size_t R, size_t K, size_t A, size_t V, const uint64_t *def_off, const uint64_t *def_clock,
                          const uint64_t *def_keys, size_t Vout, int threads, uint64_t *out_clock, uint64_t *out_ec,
                          uint64_t *out_vclk, uint64_t *out_vval, uint64_t *out_nval, uint64_t *out_def_clock,
                          uint64_t *out_def_keys, size_t max_def, size_t *out_ndef) {
  const size_t T = threads < 1 ? 1 : (size_t)threads, Kw = (K + 63) / 64;
  std::vector<MapMV> part(T);
  std::atomic<int> ready{0}, go{0};
  std::vector<std::thread> pool;
  for (size_t t = 0; t < T; ++t)
    pool.emplace_back([&, t] {
      const size_t k0 = t * K / T, k1 = (t + 1) * K / T;
      std::vector<MapMV> reps(R);
      for (size_t r = 0; r < R; ++r) {  // ingest of the thread's keys, as oracle_map_fold
        MapMV &m = reps[r];
        m.clock = vclock_from_row(clock + r * A, A);
        for (size_t k = k0; k < k1; ++k) {
          VClock e = vclock_from_row(ec + (r * K + k) * A, A);
          if (e.empty()) continue;
          MapEntry ent;
          ent.clock = std::move(e);
          for (size_t s = 0; s < V; ++s) {
            VClock c = vclock_from_row(vclk + ((r * K + k) * V + s) * A, A);
            if (!c.empty()) ent.val.vals.emplace_back(std::move(c), vval[(r * K + k) * V + s]);
          }
          m.entries.emplace((uint32_t)k, std::move(ent));
        }
        if (def_off)
          for (uint64_t d = def_off[r]; d < def_off[r + 1]; ++d) {
            VClock rm = vclock_from_row(def_clock + d * A, A);
            std::set<uint32_t> keys;
            for (size_t w = 0; w < Kw; ++w)
              for (uint64_t x = def_keys[d * Kw + w]; x; x &= x - 1) {
                const size_t key = w * 64 + __builtin_ctzll(x);
                if (key >= k0 && key < k1) keys.insert((uint32_t)key);
              }
            auto it = m.deferred.find(rm);
            if (it != m.deferred.end()) it->second.insert(keys.begin(), keys.end());
            else m.deferred.emplace(std::move(rm), std::move(keys));
          }
      }
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (auto &r : reps) part[t].merge(std::move(r));
    });
  while (ready.load() < (int)T) std::this_thread::yield();
  const double t0 = now_s();
  go.store(1, std::memory_order_release);
  for (auto &th : pool) th.join();
  const double t1 = now_s();
  vclock_to_row(part[0].clock, out_clock, A);
  std::memset(out_ec, 0, K * A * 8);
  std::memset(out_vclk, 0, K * Vout * A * 8);
  std::memset(out_vval, 0, K * Vout * 8);
  std::memset(out_nval, 0, K * 8);
  std::map<VClock, std::set<uint32_t>> dfr;
  for (size_t t = 0; t < T; ++t) {
    for (auto &kv : part[t].entries) {
      const size_t k = kv.first;
      vclock_to_row(kv.second.clock, out_ec + k * A, A);
      out_nval[k] = kv.second.val.vals.size();
      size_t s = 0;
      for (auto &cv : kv.second.val.vals) {
        if (s >= Vout) break;
        vclock_to_row(cv.first, out_vclk + (k * Vout + s) * A, A);
        out_vval[k * Vout + s] = cv.second;
        ++s;
      }
    }
    for (auto &kv : part[t].deferred) dfr[kv.first].insert(kv.second.begin(), kv.second.end());
  }
  size_t k = 0;
  for (auto &kv : dfr) {
    if (k < max_def) {
      vclock_to_row(kv.first, out_def_clock + k * A, A);
      std::memset(out_def_keys + k * Kw, 0, Kw * 8);
      for (uint32_t key : kv.second) out_def_keys[k * Kw + key / 64] |= 1ull << (key % 64);
    }
    ++k;
  }
  *out_ndef = k;
  return t1 - t0;
}

}  // extern "C"
