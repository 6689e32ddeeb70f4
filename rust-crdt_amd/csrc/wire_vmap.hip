// Serde wire format <-> dense state layouts of the value-typed Maps (round 5, SURVEY §8f row 1 for
// the Map value types the library folds, applies and forgets): Map<u32, GCounter<u32>, u32>,
// Map<u32, PNCounter<u32>, u32> (the crdt_map_counter_states layout) and Map<u32, Orswot<u64, u32>,
// u32> (the crdt_map_orswot_states layout — the value type of the reference's merge_error KAT,
// map.rs:435-494) and Map<u32, Map<u32, MVReg<u64, u32>, u32>, u32> (the crdt_map_nested_states
// layout — the reference's own Map test type, test/map.rs:10), with the Map's deferred removes as
// per-state slots (crdt_map_deferred).
//
// bincode 1.x of the derives (map.rs:31-47 Map { clock, entries: BTreeMap<K, Entry { clock, val }>,
// deferred: HashMap<VClock, BTreeSet<K>> }; gcounter.rs:25-28, pncounter.rs:28-32, orswot.rs:20-25):
//   VClock clock; u64 n, n x (u32 key, VClock entry clock, value);   keys ascending (BTreeMap)
//   u64 d, d x (VClock rm, u64 k, k x u32 key)                       keys ascending (BTreeSet)
// with value = GCounter: VClock | PNCounter: VClock p, VClock n |
//   Orswot: VClock clock; u64 m, m x (u64 member, VClock) (HashMap: any order);
//           u64 e, e x (VClock rm, u64 j, j x u64 member)   (HashMap<VClock, HashSet<M>>: any order) |
//   Map<K2, MVReg>: the same Map layout one level down, its value u64 m, m x (VClock, u64 val)
//           (mvreg.rs:32-35, Vec order), inner key sets u32 ascending
// Ingest is one wave per state (the record loop of every VClock across lanes, rows assembled in LDS,
// written with coalesced stores), as map_ingest_kernel (wire.hip); egress is count -> exclusive scan
// -> write, present keys / members / key sets in ascending dictionary order (the HashMaps' order is
// unspecified in the reference: any order decodes to the same state).
// A key is present iff its entry clock row is nonzero, a member iff its dot row is (the fold
// layouts' convention); a nested Orswot's deferred removes are slots 0 .. vd_n of its key.
#include "wire_common.hpp"

namespace crdt {

constexpr int kVwVd = 16;  // nested deferred removes per key (crdt_map_orswot_states / crdt_map_nested_states)
constexpr int kVwVs = 8;   // MVReg slots per inner key (crdt_map_nested_states)

struct VMapWirePlan {
  const uint8_t *bytes;
  const u64 *frame_off;
  unsigned long long N, A, K, Kw, W, M, Mw, Dcap;
  int vt;  // value type: 0 = W counter VClocks (GCounter W = 1, PNCounter W = 2), 1 = Orswot, 2 = Map<K2, MVReg>
  const uint32_t *actors, *keys, *ikeys;
  const u64 *members;
  unsigned long long K2, K2w;  // inner keys; inner key-set mask words (1 up to K2 = 64)
  unsigned long long Vs;       // MVReg slots per inner key (crdt_map_nested_states.Vs; 8 if 0)
  u64 *ic, *iec, *ivc, *ivv, *id_clock, *id_keys;  // nested Map [N][K][A], [N][K][K2][A], [N][K][K2][8][A],
  uint32_t *nval, *id_n;                           // [N][K][K2][8], [N][K][16][A], [N][K][16][K2w]; [N][K][K2], [N][K]
  u64 *clock, *ec, *val;           // [N][A], [N][K][A], counter [N][K][W][A]
  u64 *oc, *ent;                   // Orswot [N][K][A], [N][K][M][A]
  uint32_t *vd_n;                  // [N][K]
  u64 *vd_clock, *vd_mem;          // [N][K][Vd][A], [N][K][Vd][Mw]
  unsigned long long Vd;           // nested slots per key: the Orswot's Vd or the inner Map's Id (16 if 0)
  u64 *def_clock, *def_keys;       // [N][Dcap][A], [N][Dcap][Kw]
  uint32_t *def_count;             // [N]
  uint32_t *status;
  int stage;                       // dictionaries staged in LDS
  // egress
  u64 *sizes;
  const u64 *frame_out;
  uint8_t *out;
};

// Parse a set of ids (u64 members when wide, else u32 keys) at word k into the LDS bitmap `bits`
// (nw words, zeroed here); returns the word after it, or ~0 on a truncated / lying count.
__device__ __forceinline__ unsigned long long parse_idset(const Frame &f, unsigned long long k, bool wide,
                                                          const uint32_t *d32, const u64 *d64, unsigned long long nd,
                                                          u64 *bits, unsigned long long nw, int lane, unsigned &st) {
  for (unsigned long long w = lane; w < nw; w += kWave) bits[w] = 0;
  wfence();
  if (k == ~0ull || k + 2 > f.nw) return ~0ull;
  const u64 n = rd64(f.w, k);
  k += 2;
  const unsigned long long per = wide ? 2 : 1;
  if (n > (f.nw - k) / per) return ~0ull;
  bool miss = false;
  for (unsigned long long i = lane; i < n; i += kWave) {
    const long long b = wide ? find_u64(d64, nd, rd64(f.w, k + 2 * i), i) : find_u32(d32, nd, f.w[k + i], i);
    if (b < 0) miss = true;
    else atomicOr(bits + b / 64, 1ull << (b % 64));
  }
  if (__ballot(miss)) st |= kWireMissing;
  wfence();
  return k + per * n;
}

__host__ __device__ __forceinline__ unsigned long long max3(unsigned long long a, unsigned long long b,
                                                            unsigned long long c) {
  const unsigned long long m = a > b ? a : b;
  return m > c ? m : c;
}

__global__ __launch_bounds__(kBlock) void vmap_ingest_kernel(VMapWirePlan p) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x % kWave, wib = threadIdx.x / kWave;
  const int wpb = blockDim.x / kWave;
  const uint32_t *actors = p.actors, *keys = p.keys, *ikeys = p.ikeys;
  const u64 *members = p.members;
  u64 *base = lds;
  if (p.stage) {  // [actors u32 | keys u32 | members u64 or inner keys u32], the u32 arrays padded to 8 bytes
    uint32_t *la = reinterpret_cast<uint32_t *>(lds);
    const unsigned long long aw = (p.A + 1) / 2, kw = (p.K + 1) / 2;
    for (unsigned long long i = threadIdx.x; i < p.A; i += blockDim.x) la[i] = p.actors[i];
    uint32_t *lk = reinterpret_cast<uint32_t *>(lds + aw);
    for (unsigned long long i = threadIdx.x; i < p.K; i += blockDim.x) lk[i] = p.keys[i];
    u64 *lm = lds + aw + kw;
    const unsigned long long nm = p.vt == 1 ? p.M : (p.vt == 2 ? (p.K2 + 1) / 2 : 0);
    if (p.vt == 1)
      for (unsigned long long i = threadIdx.x; i < p.M; i += blockDim.x) lm[i] = p.members[i];
    if (p.vt == 2)
      for (unsigned long long i = threadIdx.x; i < p.K2; i += blockDim.x) reinterpret_cast<uint32_t *>(lm)[i] = p.ikeys[i];
    __syncthreads();
    actors = la;
    keys = lk;
    if (p.vt == 1) members = lm;
    if (p.vt == 2) ikeys = reinterpret_cast<const uint32_t *>(lm);
    base = lds + aw + kw + nm;
  }
  const unsigned long long bw = max3(p.Kw, p.Mw, p.K2w);
  u64 *row = base + (unsigned long long)wib * (p.A + bw);
  u64 *bits = row + p.A;
  for (unsigned long long s = (unsigned long long)blockIdx.x * wpb + wib; s < p.N;
       s += (unsigned long long)gridDim.x * wpb) {
    unsigned st = 0;
    unsigned long long nd = 0;
    Frame f;
    const u64 b = p.frame_off[s], e = p.frame_off[s + 1];
    unsigned long long k = ~0ull;
    if ((b & 3) || (e & 3) || e < b) {
      st = kWireBad;
    } else {
      f.w = reinterpret_cast<const uint32_t *>(p.bytes + b);
      f.nw = (e - b) / 4;
      k = parse_vclock(f, 0, actors, p.A, row, lane, st);
      store_row<u64>(p.clock + s * p.A, row, p.A, lane);
      wfence();
      const u64 n = (k == ~0ull || k + 2 > f.nw) ? 0 : rd64(f.w, k);
      if (k == ~0ull || k + 2 > f.nw) k = ~0ull;
      else k += 2;
      for (u64 en = 0; en < n && k != ~0ull; ++en) {
        if (k + 1 > f.nw) {
          k = ~0ull;
          break;
        }
        const long long ki = find_u32(keys, p.K, f.w[k], en);
        if (ki < 0) st |= kWireMissing;
        const unsigned long long sk = s * p.K + (unsigned long long)(ki < 0 ? 0 : ki);
        k = parse_vclock(f, k + 1, actors, p.A, row, lane, st);
        if (k == ~0ull) break;
        if (ki >= 0) store_row<u64>(p.ec + sk * p.A, row, p.A, lane);
        wfence();
        if (p.vt == 2) {  // the inner Map<K2, MVReg>: clock, entries, deferred removes
          k = parse_vclock(f, k, actors, p.A, row, lane, st);
          if (k == ~0ull || k + 2 > f.nw) {
            k = ~0ull;
            break;
          }
          if (ki >= 0) store_row<u64>(p.ic + sk * p.A, row, p.A, lane);
          wfence();
          const u64 n2 = rd64(f.w, k);
          k += 2;
          for (u64 j = 0; j < n2 && k != ~0ull; ++j) {
            if (k + 1 > f.nw) {
              k = ~0ull;
              break;
            }
            const long long ji = find_u32(ikeys, p.K2, f.w[k], j);
            if (ji < 0) st |= kWireMissing;
            const bool on = ki >= 0 && ji >= 0;
            const unsigned long long skj = sk * p.K2 + (unsigned long long)(ji < 0 ? 0 : ji);
            k = parse_vclock(f, k + 1, actors, p.A, row, lane, st);
            if (k == ~0ull || k + 2 > f.nw) {
              k = ~0ull;
              break;
            }
            if (on) store_row<u64>(p.iec + skj * p.A, row, p.A, lane);
            wfence();
            const u64 m = rd64(f.w, k);
            k += 2;
            unsigned long long nv = 0;
            for (u64 v = 0; v < m && k != ~0ull; ++v) {
              k = parse_vclock(f, k, actors, p.A, row, lane, st);
              if (k == ~0ull || k + 2 > f.nw) {
                k = ~0ull;
                break;
              }
              const u64 val = rd64(f.w, k);
              k += 2;
              if (on) {
                if (nv < p.Vs) {
                  store_row<u64>(p.ivc + (skj * p.Vs + nv) * p.A, row, p.A, lane);
                  if (lane == 0) p.ivv[skj * p.Vs + nv] = val;
                  ++nv;
                } else {
                  st |= kWireCap;
                }
              }
              wfence();
            }
            if (on && lane == 0) p.nval[skj] = (uint32_t)nv;
          }
          if (k == ~0ull || k + 2 > f.nw) {
            k = ~0ull;
            break;
          }
          const u64 d2 = rd64(f.w, k);
          k += 2;
          unsigned long long dn = 0;
          for (u64 j = 0; j < d2 && k != ~0ull; ++j) {
            k = parse_vclock(f, k, actors, p.A, row, lane, st);
            k = parse_idset(f, k, false, ikeys, nullptr, p.K2, bits, p.K2w, lane, st);
            if (k == ~0ull) break;
            if (ki >= 0) {
              if (dn < p.Vd) {
                store_row<u64>(p.id_clock + (sk * p.Vd + dn) * p.A, row, p.A, lane);
                for (unsigned long long x = lane; x < p.K2w; x += kWave) p.id_keys[(sk * p.Vd + dn) * p.K2w + x] = bits[x];
                ++dn;
              } else {
                st |= kWireCap;
              }
            }
            wfence();
          }
          if (ki >= 0 && lane == 0) p.id_n[sk] = (uint32_t)dn;
          continue;
        }
        if (p.vt == 0) {
          for (unsigned long long w = 0; w < p.W && k != ~0ull; ++w) {
            k = parse_vclock(f, k, actors, p.A, row, lane, st);
            if (k != ~0ull && ki >= 0) store_row<u64>(p.val + (sk * p.W + w) * p.A, row, p.A, lane);
            wfence();
          }
          continue;
        }
        // the nested Orswot: clock, member dots, deferred removes
        k = parse_vclock(f, k, actors, p.A, row, lane, st);
        if (k == ~0ull || k + 2 > f.nw) {
          k = ~0ull;
          break;
        }
        if (ki >= 0) store_row<u64>(p.oc + sk * p.A, row, p.A, lane);
        wfence();
        const u64 nm = rd64(f.w, k);
        k += 2;
        for (u64 j = 0; j < nm && k != ~0ull; ++j) {
          if (k + 2 > f.nw) {
            k = ~0ull;
            break;
          }
          const long long mi = find_u64(members, p.M, rd64(f.w, k), p.M);
          k = parse_vclock(f, k + 2, actors, p.A, row, lane, st);
          if (k == ~0ull) break;
          if (mi < 0) st |= kWireMissing;
          else if (ki >= 0) store_row<u64>(p.ent + (sk * p.M + (unsigned long long)mi) * p.A, row, p.A, lane);
          wfence();
        }
        if (k == ~0ull || k + 2 > f.nw) {
          k = ~0ull;
          break;
        }
        const u64 nv = rd64(f.w, k);
        k += 2;
        unsigned long long vn = 0;
        for (u64 j = 0; j < nv && k != ~0ull; ++j) {
          k = parse_vclock(f, k, actors, p.A, row, lane, st);
          k = parse_idset(f, k, true, nullptr, members, p.M, bits, p.Mw, lane, st);
          if (k == ~0ull) break;
          if (ki >= 0) {
            if (vn < p.Vd) {
              store_row<u64>(p.vd_clock + (sk * p.Vd + vn) * p.A, row, p.A, lane);
              store_row<u64>(p.vd_mem + (sk * p.Vd + vn) * p.Mw, bits, p.Mw, lane);
              ++vn;
            } else {
              st |= kWireCap;
            }
          }
          wfence();
        }
        if (ki >= 0 && lane == 0) p.vd_n[sk] = (uint32_t)vn;
      }
      if (k != ~0ull && k + 2 <= f.nw) {
        const u64 d = rd64(f.w, k);
        k += 2;
        for (u64 j = 0; j < d && k != ~0ull; ++j) {
          k = parse_vclock(f, k, actors, p.A, row, lane, st);
          k = parse_idset(f, k, false, keys, nullptr, p.K, bits, p.Kw, lane, st);
          if (k == ~0ull) break;
          if (nd < p.Dcap) {
            store_row<u64>(p.def_clock + (s * p.Dcap + nd) * p.A, row, p.A, lane);
            store_row<u64>(p.def_keys + (s * p.Dcap + nd) * p.Kw, bits, p.Kw, lane);
            ++nd;
          } else {
            st |= kWireCap;
          }
          wfence();
        }
      } else {
        k = ~0ull;
      }
      if (k != f.nw) st |= kWireBad;  // truncated, lying counts or trailing bytes
    }
    if (lane == 0) {
      p.status[s] = st;
      p.def_count[s] = (uint32_t)nd;
    }
  }
}

// Write the ids of bitmap `bits` (nw words) ascending at word k: u64 count, then u64 members (wide)
// or u32 keys.  Lanes take bitmap words; a wave prefix sum places their ids.  Returns the next word.
__device__ __forceinline__ unsigned long long write_idset(uint32_t *w, unsigned long long k, const u64 *bits,
                                                          unsigned long long nw, bool wide, const uint32_t *d32,
                                                          const u64 *d64, int lane) {
  const u64 n = popc_row(bits, nw, lane);
  if (lane == 0) wr64(w, k, n);
  const unsigned long long per = wide ? 2 : 1;
  unsigned long long basei = 0;
  for (unsigned long long x0 = 0; x0 < nw; x0 += kWave) {
    const unsigned long long x = x0 + lane;
    u64 word = x < nw ? bits[x] : 0;
    const unsigned cnt = __popcll(word);
    unsigned long long pre = cnt;
    for (int off = 1; off < kWave; off <<= 1) {
      const unsigned long long t = __shfl_up(pre, off, kWave);
      if (lane >= off) pre += t;
    }
    unsigned long long i = basei + pre - cnt;
    while (word) {
      const int b = __builtin_ctzll(word);
      word &= word - 1;
      if (wide) wr64(w, k + 2 + 2 * i, d64[x * 64 + b]);
      else w[k + 2 + i] = d32[x * 64 + b];
      ++i;
    }
    basei += __shfl(pre, kWave - 1, kWave);
  }
  return k + 2 + per * n;
}

__device__ __forceinline__ u64 vclock_bytes(const u64 *r, unsigned long long A, int lane) {
  return 8 + 12 * nnz_row(r, A, lane);
}

// (4 waves per SIMD: the K2w key sets of round 6 took the kernel past 128 VGPRs, 3 waves, 25% slower)
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void vmap_egress_kernel(VMapWirePlan p, int write) {
  const int lane = threadIdx.x % kWave;
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;
  const unsigned long long nwv = (unsigned long long)gridDim.x * (kBlock / kWave);
  for (unsigned long long s = w0; s < p.N; s += nwv) {
    uint32_t *w = write ? reinterpret_cast<uint32_t *>(p.out + p.frame_out[s]) : nullptr;
    const u64 *c = p.clock + s * p.A;
    u64 sz = vclock_bytes(c, p.A, lane);
    unsigned long long k = write ? write_vclock(w, 0, c, p.A, p.actors, lane) : 0;
    u64 ne = 0;
    for (unsigned long long key = 0; key < p.K; ++key) ne += nnz_row(p.ec + (s * p.K + key) * p.A, p.A, lane) != 0;
    sz += 8;
    if (write) {
      if (lane == 0) wr64(w, k, ne);
      k += 2;
    }
    for (unsigned long long key = 0; key < p.K; ++key) {
      const unsigned long long sk = s * p.K + key;
      const u64 *er = p.ec + sk * p.A;
      if (nnz_row(er, p.A, lane) == 0) continue;
      sz += 4 + vclock_bytes(er, p.A, lane);
      if (write) {
        if (lane == 0) w[k] = p.keys[key];
        k = write_vclock(w, k + 1, er, p.A, p.actors, lane);
      }
      if (p.vt == 2) {
        const u64 *ic = p.ic + sk * p.A;
        sz += vclock_bytes(ic, p.A, lane) + 8;
        if (write) k = write_vclock(w, k, ic, p.A, p.actors, lane);
        u64 n2 = 0;
        for (unsigned long long j = 0; j < p.K2; ++j) n2 += nnz_row(p.iec + (sk * p.K2 + j) * p.A, p.A, lane) != 0;
        if (write) {
          if (lane == 0) wr64(w, k, n2);
          k += 2;
        }
        for (unsigned long long j = 0; j < p.K2; ++j) {
          const unsigned long long skj = sk * p.K2 + j;
          const u64 *er2 = p.iec + skj * p.A;
          if (nnz_row(er2, p.A, lane) == 0) continue;
          const unsigned long long m = p.nval[skj] < p.Vs ? p.nval[skj] : p.Vs;
          sz += 4 + vclock_bytes(er2, p.A, lane) + 8;
          if (write) {
            if (lane == 0) w[k] = p.ikeys[j];
            k = write_vclock(w, k + 1, er2, p.A, p.actors, lane);
            if (lane == 0) wr64(w, k, m);
            k += 2;
          }
          for (unsigned long long v = 0; v < m; ++v) {
            const u64 *vr = p.ivc + (skj * p.Vs + v) * p.A;
            sz += vclock_bytes(vr, p.A, lane) + 8;
            if (write) {
              k = write_vclock(w, k, vr, p.A, p.actors, lane);
              if (lane == 0) wr64(w, k, p.ivv[skj * p.Vs + v]);
              k += 2;
            }
          }
        }
        const unsigned long long dn = p.id_n[sk] < p.Vd ? p.id_n[sk] : p.Vd;
        sz += 8;
        if (write) {
          if (lane == 0) wr64(w, k, dn);
          k += 2;
        }
        for (unsigned long long i = 0; i < dn; ++i) {
          const u64 *rm = p.id_clock + (sk * p.Vd + i) * p.A, *kb = p.id_keys + (sk * p.Vd + i) * p.K2w;
          sz += vclock_bytes(rm, p.A, lane) + 8 + 4 * popc_row(kb, p.K2w, lane);
          if (write) {
            k = write_vclock(w, k, rm, p.A, p.actors, lane);
            k = write_idset(w, k, kb, p.K2w, false, p.ikeys, nullptr, lane);
          }
        }
        continue;
      }
      if (p.vt == 0) {
        for (unsigned long long x = 0; x < p.W; ++x) {
          const u64 *vr = p.val + (sk * p.W + x) * p.A;
          sz += vclock_bytes(vr, p.A, lane);
          if (write) k = write_vclock(w, k, vr, p.A, p.actors, lane);
        }
        continue;
      }
      const u64 *oc = p.oc + sk * p.A;
      sz += vclock_bytes(oc, p.A, lane) + 8;
      if (write) k = write_vclock(w, k, oc, p.A, p.actors, lane);
      u64 nm = 0;
      for (unsigned long long m = 0; m < p.M; ++m) nm += nnz_row(p.ent + (sk * p.M + m) * p.A, p.A, lane) != 0;
      if (write) {
        if (lane == 0) wr64(w, k, nm);
        k += 2;
      }
      for (unsigned long long m = 0; m < p.M; ++m) {
        const u64 *mr = p.ent + (sk * p.M + m) * p.A;
        if (nnz_row(mr, p.A, lane) == 0) continue;
        sz += 8 + vclock_bytes(mr, p.A, lane);
        if (write) {
          if (lane == 0) wr64(w, k, p.members[m]);
          k = write_vclock(w, k + 2, mr, p.A, p.actors, lane);
        }
      }
      const unsigned long long vn = p.vd_n[sk] < p.Vd ? p.vd_n[sk] : p.Vd;
      sz += 8;
      if (write) {
        if (lane == 0) wr64(w, k, vn);
        k += 2;
      }
      for (unsigned long long i = 0; i < vn; ++i) {
        const u64 *rm = p.vd_clock + (sk * p.Vd + i) * p.A, *mb = p.vd_mem + (sk * p.Vd + i) * p.Mw;
        sz += vclock_bytes(rm, p.A, lane) + 8 + 8 * popc_row(mb, p.Mw, lane);
        if (write) {
          k = write_vclock(w, k, rm, p.A, p.actors, lane);
          k = write_idset(w, k, mb, p.Mw, true, nullptr, p.members, lane);
        }
      }
    }
    const unsigned long long nd = p.def_count[s] < p.Dcap ? p.def_count[s] : p.Dcap;
    sz += 8;
    if (write) {
      if (lane == 0) wr64(w, k, nd);
      k += 2;
    }
    for (unsigned long long d = 0; d < nd; ++d) {
      const u64 *rm = p.def_clock + (s * p.Dcap + d) * p.A, *kb = p.def_keys + (s * p.Dcap + d) * p.Kw;
      sz += vclock_bytes(rm, p.A, lane) + 8 + 4 * popc_row(kb, p.Kw, lane);
      if (write) {
        k = write_vclock(w, k, rm, p.A, p.actors, lane);
        k = write_idset(w, k, kb, p.Kw, false, p.keys, nullptr, lane);
      }
    }
    if (!write && lane == 0) p.sizes[s] = sz;
  }
}

static int vmap_deferred_plan(crdt_ctx *ctx, const crdt_map_deferred *df, size_t N, VMapWirePlan &p, const char *what) {
  if (!df) return fail(ctx, CRDT_EINVAL, "%s: NULL deferred slots", what);
  if (N && (!df->count || (df->Dcap && (!df->clock || !df->keys))))
    return fail(ctx, CRDT_EINVAL, "%s: NULL deferred slot buffer", what);
  p.Dcap = df->Dcap;
  p.def_clock = (u64 *)df->clock;
  p.def_keys = (u64 *)df->keys;
  p.def_count = df->count;
  return CRDT_OK;
}

static int vmap_counter_plan(crdt_ctx *ctx, const crdt_map_counter_states *st, const crdt_map_deferred *df,
                             const uint32_t *actors, const uint32_t *keys, VMapWirePlan &p, const char *what) {
  if (!st || !actors || !keys) return fail(ctx, CRDT_EINVAL, "%s: NULL states / dictionaries", what);
  const size_t N = st->N, K = st->K, A = st->A, W = st->W;
  if (A == 0 || K == 0 || (W != 1 && W != 2)) return fail(ctx, CRDT_EINVAL, "%s: need A, K >= 1 and W in {1, 2}", what);
  if (N && (!st->clock || !st->ec || !st->val)) return fail(ctx, CRDT_EINVAL, "%s: NULL state buffer", what);
  if (N > 1 && (st->clock_stride != A || st->ec_stride != K * A || st->val_stride != K * W * A))
    return fail(ctx, CRDT_EUNSUPPORTED, "%s: states must be packed (strides A, K*A, K*W*A)", what);
  const size_t Kw = (K + 63) / 64;
  if (A + Kw > (size_t)kWireRowLds) return fail(ctx, CRDT_EUNSUPPORTED, "%s: A + K/64 too large", what);
  p = VMapWirePlan{};
  if (int rc = vmap_deferred_plan(ctx, df, N, p, what)) return rc;
  p.N = N;
  p.A = A;
  p.K = K;
  p.Kw = Kw;
  p.W = W;
  p.actors = actors;
  p.keys = keys;
  p.clock = (u64 *)st->clock;
  p.ec = (u64 *)st->ec;
  p.val = (u64 *)st->val;
  return CRDT_OK;
}

static int vmap_orswot_plan(crdt_ctx *ctx, const crdt_map_orswot_states *st, const crdt_map_deferred *df,
                            const uint32_t *actors, const uint32_t *keys, const uint64_t *members, VMapWirePlan &p,
                            const char *what) {
  if (!st || !actors || !keys || !members) return fail(ctx, CRDT_EINVAL, "%s: NULL states / dictionaries", what);
  const size_t N = st->N, K = st->K, M = st->M, A = st->A;
  if (A == 0 || K == 0 || M == 0) return fail(ctx, CRDT_EINVAL, "%s: need A, K, M >= 1", what);
  if (N && (!st->clock || !st->ec || !st->oc || !st->ent || !st->vd_n || !st->vd_clock || !st->vd_mem))
    return fail(ctx, CRDT_EINVAL, "%s: NULL state buffer", what);
  const size_t Kw = (K + 63) / 64, Mw = (M + 63) / 64;
  if (A + (Kw > Mw ? Kw : Mw) > (size_t)kWireRowLds)
    return fail(ctx, CRDT_EUNSUPPORTED, "%s: A + max(K, M)/64 too large", what);
  p = VMapWirePlan{};
  if (int rc = vmap_deferred_plan(ctx, df, N, p, what)) return rc;
  p.N = N;
  p.A = A;
  p.K = K;
  p.Kw = Kw;
  p.M = M;
  p.Mw = Mw;
  p.vt = 1;
  p.actors = actors;
  p.keys = keys;
  p.members = (const u64 *)members;
  p.clock = (u64 *)st->clock;
  p.ec = (u64 *)st->ec;
  p.oc = (u64 *)st->oc;
  p.ent = (u64 *)st->ent;
  p.vd_n = st->vd_n;
  p.vd_clock = (u64 *)st->vd_clock;
  p.vd_mem = (u64 *)st->vd_mem;
  p.Vd = st->Vd ? st->Vd : (size_t)kVwVd;
  return CRDT_OK;
}

static int vmap_nested_plan(crdt_ctx *ctx, const crdt_map_nested_states *st, const crdt_map_deferred *df,
                            const uint32_t *actors, const uint32_t *keys, const uint32_t *ikeys, VMapWirePlan &p,
                            const char *what) {
  if (!st || !actors || !keys || !ikeys) return fail(ctx, CRDT_EINVAL, "%s: NULL states / dictionaries", what);
  const size_t N = st->N, K = st->K, K2 = st->K2, A = st->A;
  if (A == 0 || K == 0 || K2 == 0) return fail(ctx, CRDT_EINVAL, "%s: need A, K, K2 >= 1", what);
  if (K2 > 256) return fail(ctx, CRDT_EUNSUPPORTED, "%s: K2 = %zu > 256", what, K2);
  if (N && (!st->clock || !st->ec || !st->ic || !st->iec || !st->ivc || !st->ivv || !st->nval || !st->id_n ||
            !st->id_clock || !st->id_keys))
    return fail(ctx, CRDT_EINVAL, "%s: NULL state buffer", what);
  const size_t Kw = (K + 63) / 64, K2w = K2 > 64 ? (K2 + 63) / 64 : 1;
  if (A + (Kw > K2w ? Kw : K2w) > (size_t)kWireRowLds)
    return fail(ctx, CRDT_EUNSUPPORTED, "%s: A + K/64 too large", what);
  p = VMapWirePlan{};
  if (int rc = vmap_deferred_plan(ctx, df, N, p, what)) return rc;
  p.N = N;
  p.A = A;
  p.K = K;
  p.Kw = Kw;
  p.K2 = K2;
  p.K2w = K2 > 64 ? (K2 + 63) / 64 : 1;
  p.Vd = st->Id ? st->Id : (size_t)kVwVd;
  p.Vs = st->Vs ? st->Vs : (size_t)kVwVs;
  if (p.Vs > 64) return fail(ctx, CRDT_EUNSUPPORTED, "%s: Vs = %zu > 64", what, (size_t)p.Vs);
  p.vt = 2;
  p.actors = actors;
  p.keys = keys;
  p.ikeys = ikeys;
  p.clock = (u64 *)st->clock;
  p.ec = (u64 *)st->ec;
  p.ic = (u64 *)st->ic;
  p.iec = (u64 *)st->iec;
  p.ivc = (u64 *)st->ivc;
  p.ivv = (u64 *)st->ivv;
  p.nval = st->nval;
  p.id_n = st->id_n;
  p.id_clock = (u64 *)st->id_clock;
  p.id_keys = (u64 *)st->id_keys;
  return CRDT_OK;
}

static int vmap_ingest(crdt_ctx *ctx, VMapWirePlan &p, const uint8_t *bytes, const uint64_t *frame_off,
                       uint32_t *status) {
  const size_t N = p.N;
  if (N == 0) return CRDT_OK;
  if (int rc = check_frames(ctx, bytes, frame_off, N, status)) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  // absent keys / members / nested removes are zero rows
  if (int rc = device_fill(ctx, p.ec, N * p.K * p.A * 8, 0)) return rc;
  if (p.vt == 0) {
    if (int rc = device_fill(ctx, p.val, N * p.K * p.W * p.A * 8, 0)) return rc;
  } else if (p.vt == 2) {
    if (int rc = device_fill(ctx, p.ic, N * p.K * p.A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, p.iec, N * p.K * p.K2 * p.A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, p.ivc, N * p.K * p.K2 * p.Vs * p.A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, p.ivv, N * p.K * p.K2 * p.Vs * 8, 0)) return rc;
    if (int rc = device_fill(ctx, p.nval, N * p.K * p.K2 * 4, 0)) return rc;
    if (int rc = device_fill(ctx, p.id_n, N * p.K * 4, 0)) return rc;
    if (int rc = device_fill(ctx, p.id_clock, N * p.K * p.Vd * p.A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, p.id_keys, N * p.K * p.Vd * p.K2w * 8, 0)) return rc;
  } else {
    if (int rc = device_fill(ctx, p.oc, N * p.K * p.A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, p.ent, N * p.K * p.M * p.A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, p.vd_n, N * p.K * 4, 0)) return rc;
    if (int rc = device_fill(ctx, p.vd_clock, N * p.K * p.Vd * p.A * 8, 0)) return rc;
    if (int rc = device_fill(ctx, p.vd_mem, N * p.K * p.Vd * p.Mw * 8, 0)) return rc;
  }
  p.bytes = bytes;
  p.frame_off = (const u64 *)frame_off;
  p.status = status;
  const size_t bw = max3(p.Kw, p.Mw, p.K2w);
  const size_t per_wave = p.A + bw;
  int wpb = 4;
  while (wpb > 1 && (size_t)wpb * per_wave * 8 > 64 * 1024) --wpb;
  const size_t dw = (p.A + 1) / 2 + (p.K + 1) / 2 + (p.vt == 1 ? p.M : (p.vt == 2 ? (p.K2 + 1) / 2 : 0));
  p.stage = (dw + wpb * per_wave) * 8 <= 64 * 1024;
  const size_t lds = ((p.stage ? dw : 0) + wpb * per_wave) * 8;
  timing_begin(ctx, "wire_ingest");
  hipLaunchKernelGGL(vmap_ingest_kernel, dim3(wave_grid(ctx, N, wpb, 32)), dim3(wpb * kWave), lds, ctx->stream, p);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

static int vmap_egress(crdt_ctx *ctx, VMapWirePlan &p, uint64_t *frame_off, uint8_t *bytes, size_t cap, size_t *total,
                       const char *what) {
  const size_t N = p.N;
  if (N == 0) return CRDT_OK;
  if (!frame_off || !total) return fail(ctx, CRDT_EINVAL, "%s: need frame_off and total", what);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  u64 *sizes = nullptr;
  if (int rc = wire_scratch(ctx, N, &sizes)) return rc;
  p.sizes = sizes;
  const unsigned grid = wave_grid(ctx, N, 4, 32);
  timing_begin(ctx, "wire_egress");
  hipLaunchKernelGGL(vmap_egress_kernel, dim3(grid), dim3(kBlock), 0, ctx->stream, p, 0);
  CRDT_HIP(ctx, hipGetLastError());
  if (int rc = egress_layout(ctx, sizes, (u64 *)frame_off, N, total)) return rc;
  if (bytes && cap >= *total) {
    p.frame_out = (const u64 *)frame_off;
    p.out = bytes;
    hipLaunchKernelGGL(vmap_egress_kernel, dim3(grid), dim3(kBlock), 0, ctx->stream, p, 1);
    CRDT_HIP(ctx, hipGetLastError());
  }
  timing_end(ctx);
  return CRDT_OK;
}

}  // namespace crdt

using namespace crdt;

extern "C" {

int crdt_map_counter_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, const uint32_t *actors,
                            const uint32_t *keys, const crdt_map_counter_states *out, const crdt_map_deferred *out_def,
                            uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  VMapWirePlan p;
  if (int rc = vmap_counter_plan(ctx, out, out_def, actors, keys, p, "map_counter_ingest")) return rc;
  return vmap_ingest(ctx, p, bytes, frame_off, status);
}

int crdt_map_counter_egress(crdt_ctx *ctx, const crdt_map_counter_states *states, const crdt_map_deferred *def,
                            const uint32_t *actors, const uint32_t *keys, uint64_t *frame_off, uint8_t *bytes,
                            size_t cap, size_t *total) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (total) *total = 0;
  VMapWirePlan p;
  if (int rc = vmap_counter_plan(ctx, states, def, actors, keys, p, "map_counter_egress")) return rc;
  return vmap_egress(ctx, p, frame_off, bytes, cap, total, "map_counter_egress");
}

int crdt_map_orswot_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, const uint32_t *actors,
                           const uint32_t *keys, const uint64_t *members, const crdt_map_orswot_states *out,
                           const crdt_map_deferred *out_def, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  VMapWirePlan p;
  if (int rc = vmap_orswot_plan(ctx, out, out_def, actors, keys, members, p, "map_orswot_ingest")) return rc;
  return vmap_ingest(ctx, p, bytes, frame_off, status);
}

int crdt_map_orswot_egress(crdt_ctx *ctx, const crdt_map_orswot_states *states, const crdt_map_deferred *def,
                           const uint32_t *actors, const uint32_t *keys, const uint64_t *members, uint64_t *frame_off,
                           uint8_t *bytes, size_t cap, size_t *total) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (total) *total = 0;
  VMapWirePlan p;
  if (int rc = vmap_orswot_plan(ctx, states, def, actors, keys, members, p, "map_orswot_egress")) return rc;
  return vmap_egress(ctx, p, frame_off, bytes, cap, total, "map_orswot_egress");
}

int crdt_map_nested_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, const uint32_t *actors,
                           const uint32_t *keys, const uint32_t *ikeys, const crdt_map_nested_states *out,
                           const crdt_map_deferred *out_def, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  VMapWirePlan p;
  if (int rc = vmap_nested_plan(ctx, out, out_def, actors, keys, ikeys, p, "map_nested_ingest")) return rc;
  return vmap_ingest(ctx, p, bytes, frame_off, status);
}

int crdt_map_nested_egress(crdt_ctx *ctx, const crdt_map_nested_states *states, const crdt_map_deferred *def,
                           const uint32_t *actors, const uint32_t *keys, const uint32_t *ikeys, uint64_t *frame_off,
                           uint8_t *bytes, size_t cap, size_t *total) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (total) *total = 0;
  VMapWirePlan p;
  if (int rc = vmap_nested_plan(ctx, states, def, actors, keys, ikeys, p, "map_nested_egress")) return rc;
  return vmap_egress(ctx, p, frame_off, bytes, cap, total, "map_nested_egress");
}

}  // extern "C"
