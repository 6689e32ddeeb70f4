// Serde wire format <-> dense SoA, on the device (the step before the path).
//
// Replicas ship whole states (the crate is transport-agnostic, README.md:12-16), serialized with
// the serde derives of the reference types (vclock.rs:56, gcounter.rs:25, pncounter.rs:28,
// gset.rs:7, lwwreg.rs:13, orswot.rs:20).  The crate does not pick an encoding; this file reads and
// writes the one `bincode::serialize` (bincode 1.x, default options) produces, restated here:
//   integers little-endian at fixed width (u32 = 4 B, u64 = 8 B); a struct is its fields in
//   declaration order; a map / set / Vec is a u64 length followed by its entries (key then value);
//   no padding, no field names.
// So, for the instantiations the kernels take (actors A = u32, members / elements M = u64):
//   VClock<u32>      = u64 n, then n x (u32 actor, u64 counter), actors ascending (BTreeMap)
//   GCounter<u32>    = VClock                               (struct { inner })
//   PNCounter<u32>   = GCounter p, GCounter n               (struct { p, n })
//   GSet<u64>        = u64 n, then n x u64, ascending       (BTreeSet)
//   LWWReg<u64, u64> = u64 val, u64 marker                  (struct { val, marker })
//   Orswot<u64, u32> = VClock clock; u64 n, n x (u64 member, VClock) (HashMap: any order);
//                      u64 d, d x (VClock rm, u64 k, k x u64 member) (HashMap<VClock, HashSet>)
//   Map<u32, MVReg<u64, u32>, u32> (map.rs:31-47, mvreg.rs:32-35)
//                    = VClock clock; u64 n, n x (u32 key, VClock entry clock, u64 m,
//                      m x (VClock value clock, u64 value)) (BTreeMap: keys ascending; MVReg vals in
//                      Vec order); u64 d, d x (VClock rm, u64 k, k x u32 key) (BTreeSet: ascending)
// Every field is 4 or 8 bytes, so with 4-byte-aligned frame offsets every field is 4-aligned and
// is read / written as 32-bit words (a u64 as two).
//
// Frames: state s = bytes[frame_off[s] .. frame_off[s+1]).  Ids are interned through sorted
// dictionaries (device): the dense column of an actor / bit of an element / row of a member is its
// position in the dictionary.  Ingest is one wave per state: the record loop runs across lanes
// (lane i parses record i), rows are assembled in LDS and written out with coalesced stores.
// Egress is count -> exclusive scan -> write.
#include "wire_common.hpp"

namespace crdt {

struct IngestPlan {
  const uint8_t *bytes;
  const u64 *frame_off;
  unsigned long long N;
  const uint32_t *actors;  // sorted dictionaries
  unsigned long long A;
  const u64 *elems;
  unsigned long long U;
  u64 *out;  // rows
  unsigned long long row_stride;
  int nclocks;  // VClocks per frame: 1 (VClock / GCounter) or 2 (PNCounter: p then n)
  uint32_t *status;
  // Orswot
  const u64 *members;
  unsigned long long M, Mw;
  u64 *entries;  // [N][M][A]
  u64 *dpos;     // [N] word index of the deferred section
  u64 *dcount;   // [N]
  u64 *def_off;  // [N+1] exclusive scan of dcount
  u64 *def_clock, *def_members;
  unsigned long long def_cap;
  unsigned long long dict_words;  // > 0: the dictionaries are staged in LDS (this many u64 words)
};

// Stage the block's dictionaries in LDS (dependent binary-search loads then hit LDS, not L2):
// layout [actors u32 (A, padded to 8 B) | elems or members u64].  Returns the row area.
__device__ __forceinline__ u64 *stage_dicts(const IngestPlan &p, u64 *lds, const uint32_t *&actors, const u64 *&elems,
                                            const u64 *&members) {
  if (!p.dict_words) return lds;
  uint32_t *la = reinterpret_cast<uint32_t *>(lds);
  const unsigned long long aw = p.actors ? (p.A + 1) / 2 : 0;
  for (unsigned long long i = threadIdx.x; i < (p.actors ? p.A : 0); i += blockDim.x) la[i] = p.actors[i];
  u64 *lu = lds + aw;
  const u64 *src = p.members ? p.members : p.elems;
  const unsigned long long nu = p.members ? p.M : (p.elems ? p.U : 0);
  for (unsigned long long i = threadIdx.x; i < nu; i += blockDim.x) lu[i] = src[i];
  __syncthreads();
  if (p.actors) actors = la;
  if (p.members) members = lu;
  else if (p.elems) elems = lu;
  return lds + p.dict_words;
}

__device__ __forceinline__ bool frame_of(const IngestPlan &p, unsigned long long s, Frame &f) {
  const u64 b = p.frame_off[s], e = p.frame_off[s + 1];
  if ((b & 3) || (e & 3) || e < b) return false;
  f.w = reinterpret_cast<const uint32_t *>(p.bytes + b);
  f.nw = (e - b) / 4;
  return true;
}

// VClock / GCounter / PNCounter frames -> rows of nclocks*A counters.
__global__ __launch_bounds__(kBlock) void vclock_ingest_kernel(IngestPlan p) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x % kWave, wib = threadIdx.x / kWave;
  const int wpb = blockDim.x / kWave;
  const uint32_t *actors = p.actors;
  const u64 *elems = p.elems, *members = p.members;
  u64 *row = stage_dicts(p, lds, actors, elems, members) + (unsigned long long)wib * p.A;
  for (unsigned long long s = (unsigned long long)blockIdx.x * wpb + wib; s < p.N;
       s += (unsigned long long)gridDim.x * wpb) {
    unsigned st = 0;
    Frame f;
    u64 *dst = p.out + s * p.row_stride;
    if (!frame_of(p, s, f)) {
      st = kWireBad;
      for (unsigned long long a = lane; a < (unsigned long long)p.nclocks * p.A; a += kWave) dst[a] = 0;
    } else {
      unsigned long long k = 0;
      for (int c = 0; c < p.nclocks; ++c) {
        if (k != ~0ull) {
          k = parse_vclock(f, k, actors, p.A, row, lane, st);
        } else {  // after a truncated clock: the remaining clocks are empty
          for (unsigned long long a = lane; a < p.A; a += kWave) row[a] = 0;
          wfence();
        }
        store_row<u64>(dst + c * p.A, row, p.A, lane);
        wfence();
      }
      if (k != f.nw) st |= kWireBad;  // trailing bytes or a truncated frame
    }
    if (lane == 0) p.status[s] = st;
  }
}

// GSet<u64> frames -> bitmap rows of ceil(U/64) words.
__global__ __launch_bounds__(kBlock) void gset_ingest_kernel(IngestPlan p) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x % kWave, wib = threadIdx.x / kWave;
  const int wpb = blockDim.x / kWave;
  const unsigned long long W = (p.U + 63) / 64;
  const uint32_t *actors = p.actors;
  const u64 *elems = p.elems, *members = p.members;
  u64 *row = stage_dicts(p, lds, actors, elems, members) + (unsigned long long)wib * W;
  for (unsigned long long s = (unsigned long long)blockIdx.x * wpb + wib; s < p.N;
       s += (unsigned long long)gridDim.x * wpb) {
    unsigned st = 0;
    Frame f;
    for (unsigned long long w = lane; w < W; w += kWave) row[w] = 0;
    wfence();
    if (!frame_of(p, s, f) || f.nw < 2) {
      st = kWireBad;
    } else {
      const u64 n = rd64(f.w, 0);
      if (2 + 2 * n != f.nw) st |= kWireBad;
      const u64 nn = n < (f.nw - 2) / 2 ? n : (f.nw - 2) / 2;
      bool miss = false;
      for (unsigned long long i = lane; i < nn; i += kWave) {
        const long long b = find_u64(elems, p.U, rd64(f.w, 2 + 2 * i), i);
        if (b < 0) miss = true;
        else atomicOr(row + b / 64, 1ull << (b % 64));
      }
      if (__ballot(miss)) st |= kWireMissing;
    }
    wfence();
    store_row<u64>(p.out + s * p.row_stride, row, W, lane);
    if (lane == 0) p.status[s] = st;
    wfence();
  }
}

// LWWReg<u64, u64> frames (16 B: val, marker) -> the two planes.
__global__ __launch_bounds__(kBlock) void lwwreg_ingest_kernel(IngestPlan p, u64 *marker, u64 *val) {
  for (unsigned long long s = blockIdx.x * (unsigned long long)kBlock + threadIdx.x; s < p.N;
       s += (unsigned long long)gridDim.x * kBlock) {
    Frame f;
    unsigned st = 0;
    if (!frame_of(p, s, f) || f.nw != 4) {
      st = kWireBad;
      marker[s] = 0;
      val[s] = 0;
    } else {
      val[s] = rd64(f.w, 0);
      marker[s] = rd64(f.w, 2);
    }
    p.status[s] = st;
  }
}

// Orswot<u64, u32> pass 1: clock and entries (the entries were zero-filled before), the deferred
// section's position and count.
__global__ __launch_bounds__(kBlock) void orswot_ingest_kernel(IngestPlan p) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x % kWave, wib = threadIdx.x / kWave;
  const int wpb = blockDim.x / kWave;
  const uint32_t *actors = p.actors;
  const u64 *elems = p.elems, *members = p.members;
  u64 *row = stage_dicts(p, lds, actors, elems, members) + (unsigned long long)wib * p.A;
  for (unsigned long long s = (unsigned long long)blockIdx.x * wpb + wib; s < p.N;
       s += (unsigned long long)gridDim.x * wpb) {
    unsigned st = 0;
    Frame f;
    u64 dpos = 0, dcnt = 0;
    if (!frame_of(p, s, f)) {
      st = kWireBad;
      for (unsigned long long a = lane; a < p.A; a += kWave) p.out[s * p.row_stride + a] = 0;
    } else {
      unsigned long long k = parse_vclock(f, 0, actors, p.A, row, lane, st);
      store_row<u64>(p.out + s * p.row_stride, row, p.A, lane);
      wfence();
      if (k != ~0ull && k + 2 <= f.nw) {
        const u64 n = rd64(f.w, k);
        k += 2;
        for (u64 e = 0; e < n && k != ~0ull; ++e) {
          if (k + 2 > f.nw) {
            st |= kWireBad;
            k = ~0ull;
            break;
          }
          const long long mi = find_u64(members, p.M, rd64(f.w, k), p.M);
          k = parse_vclock(f, k + 2, actors, p.A, row, lane, st);
          if (mi < 0) {
            st |= kWireMissing;
          } else {
            store_row<u64>(p.entries + (s * p.M + (unsigned long long)mi) * p.A, row, p.A, lane);
          }
          wfence();
        }
        if (k != ~0ull && k + 2 <= f.nw) {
          dcnt = rd64(f.w, k);
          dpos = k + 2;
          // every remove record takes at least 4 words (its clock's length and its member
          // count): a larger count is a lying frame, and it must not reach the exclusive scan of
          // def_off (it would shift or wrap every later state's pooled rows) -> this frame only
          if (dcnt > (f.nw - dpos) / 4) {
            st |= kWireBad;
            dcnt = 0;
          }
        } else {
          st |= kWireBad;
        }
      } else {
        st |= kWireBad;
      }
    }
    if (lane == 0) {
      p.status[s] = st;
      p.dpos[s] = dpos;
      p.dcount[s] = (st & kWireBad) ? 0 : dcnt;
    }
  }
}

// Orswot pass 3: deferred removes -> pooled rows at def_off[s] (rm clock row, member bitmap).
__global__ __launch_bounds__(kBlock) void orswot_ingest_deferred_kernel(IngestPlan p) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x % kWave, wib = threadIdx.x / kWave;
  const int wpb = blockDim.x / kWave;
  const uint32_t *actors = p.actors;
  const u64 *elems = p.elems, *members = p.members;
  u64 *row = stage_dicts(p, lds, actors, elems, members) + (unsigned long long)wib * (p.A + p.Mw);
  u64 *bits = row + p.A;
  for (unsigned long long s = (unsigned long long)blockIdx.x * wpb + wib; s < p.N;
       s += (unsigned long long)gridDim.x * wpb) {
    const u64 n = p.dcount[s];
    if (n == 0) continue;
    unsigned st = p.status[s];
    Frame f;
    frame_of(p, s, f);
    unsigned long long k = p.dpos[s];
    const u64 d0 = p.def_off[s];
    for (u64 j = 0; j < n && k != ~0ull; ++j) {
      k = parse_vclock(f, k, actors, p.A, row, lane, st);
      for (unsigned long long w = lane; w < p.Mw; w += kWave) bits[w] = 0;
      wfence();
      if (k == ~0ull || k + 2 > f.nw) {
        st |= kWireBad;
        break;
      }
      const u64 m = rd64(f.w, k);
      k += 2;
      if (m > (f.nw - k) / 2) {
        st |= kWireBad;
        break;
      }
      bool miss = false;
      for (unsigned long long i = lane; i < m; i += kWave) {
        const long long b = find_u64(members, p.M, rd64(f.w, k + 2 * i), p.M);
        if (b < 0) miss = true;
        else atomicOr(bits + b / 64, 1ull << (b % 64));
      }
      if (__ballot(miss)) st |= kWireMissing;
      k += 2 * m;
      wfence();
      const u64 d = d0 + j;
      if (d < p.def_cap) {
        store_row<u64>(p.def_clock + d * p.A, row, p.A, lane);
        store_row<u64>(p.def_members + d * p.Mw, bits, p.Mw, lane);
      } else {
        st |= kWireCap;
      }
      wfence();
    }
    if (k != f.nw) st |= kWireBad;
    if (lane == 0) p.status[s] = st;
  }
}

// ---- exclusive scan of u64 counts (frame sizes, deferred counts) ----------------------------------

__global__ __launch_bounds__(kBlock) void scan_block_kernel(const u64 *in, u64 *out, u64 *block_sums,
                                                            unsigned long long n) {
  __shared__ u64 sh[kScanItems];
  const unsigned long long base = (unsigned long long)blockIdx.x * kScanItems;
  for (int i = threadIdx.x; i < kScanItems; i += kBlock) sh[i] = base + i < n ? in[base + i] : 0;
  __syncthreads();
  if (threadIdx.x == 0) {  // 1024 adds: negligible next to the passes it serves
    u64 run = 0;
    for (int i = 0; i < kScanItems; ++i) {
      const u64 v = sh[i];
      sh[i] = run;
      run += v;
    }
    block_sums[blockIdx.x] = run;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kScanItems; i += kBlock)
    if (base + i < n) out[base + i] = sh[i];
}

__global__ void scan_sums_kernel(u64 *block_sums, unsigned long long nb, u64 *total) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    u64 run = 0;
    for (unsigned long long i = 0; i < nb; ++i) {
      const u64 v = block_sums[i];
      block_sums[i] = run;
      run += v;
    }
    *total = run;
  }
}

__global__ __launch_bounds__(kBlock) void scan_add_kernel(u64 *out, const u64 *block_sums, unsigned long long n,
                                                          const u64 *total) {
  const unsigned long long i = blockIdx.x * (unsigned long long)kBlock + threadIdx.x;
  if (i < n) out[i] += block_sums[i / kScanItems];
  if (i == n) out[n] = *total;  // out has n+1 entries: the last is the sum
}

// out[0..n] = exclusive scan of in[0..n), out[n] = sum; *host_total = sum (synchronises).
static int exclusive_scan(crdt_ctx *ctx, const u64 *in, u64 *out, unsigned long long n, u64 *scratch,
                          unsigned long long *host_total) {
  const unsigned long long nb = (n + kScanItems - 1) / kScanItems;
  u64 *sums = scratch, *total = scratch + (nb ? nb : 1);
  if (n) hipLaunchKernelGGL(scan_block_kernel, dim3((unsigned)nb), dim3(kBlock), 0, ctx->stream, in, out, sums, n);
  hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(64), 0, ctx->stream, sums, nb, total);
  hipLaunchKernelGGL(scan_add_kernel, dim3((unsigned)((n + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                     out, sums, n, total);
  CRDT_HIP(ctx, hipGetLastError());
  if (host_total) {
    u64 t = 0;
    CRDT_HIP(ctx, hipMemcpyAsync(&t, total, 8, hipMemcpyDeviceToHost, ctx->stream));
    CRDT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *host_total = t;
  }
  return CRDT_OK;
}

// ---- egress ---------------------------------------------------------------------------------------
struct EgressPlan {
  const u64 *rows;
  unsigned long long N, A, row_stride;
  int nclocks;
  const uint32_t *actors;
  const u64 *elems;
  unsigned long long U;
  u64 *sizes;      // [N] bytes of each frame
  const u64 *frame_off;
  uint8_t *bytes;
  // Orswot
  const u64 *entries;  // [N][M][A]
  unsigned long long M, Mw;
  const u64 *members;
  const u64 *def_off;  // [N+1] device: state s owns pooled removes [def_off[s], def_off[s+1])
  const u64 *def_clock, *def_members;
  const uint8_t *def_keep;  // may be NULL (all kept)
};

__global__ __launch_bounds__(kBlock) void vclock_egress_kernel(EgressPlan p, int write) {
  const int lane = threadIdx.x % kWave;
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;
  const unsigned long long nw = (unsigned long long)gridDim.x * (kBlock / kWave);
  for (unsigned long long s = w0; s < p.N; s += nw) {
    const u64 *r = p.rows + s * p.row_stride;
    if (!write) {
      u64 sz = 0;
      for (int c = 0; c < p.nclocks; ++c) sz += 8 + 12 * nnz_row(r + c * p.A, p.A, lane);
      if (lane == 0) p.sizes[s] = sz;
      continue;
    }
    uint32_t *w = reinterpret_cast<uint32_t *>(p.bytes + p.frame_off[s]);
    unsigned long long k = 0;
    for (int c = 0; c < p.nclocks; ++c) k = write_vclock(w, k, r + c * p.A, p.A, p.actors, lane);
  }
}

__global__ __launch_bounds__(kBlock) void gset_egress_kernel(EgressPlan p, int write) {
  const int lane = threadIdx.x % kWave;
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;
  const unsigned long long nw = (unsigned long long)gridDim.x * (kBlock / kWave);
  const unsigned long long W = (p.U + 63) / 64;
  for (unsigned long long s = w0; s < p.N; s += nw) {
    const u64 *r = p.rows + s * p.row_stride;
    const u64 n = popc_row(r, W, lane);
    if (!write) {
      if (lane == 0) p.sizes[s] = 8 + 8 * n;
      continue;
    }
    uint32_t *w = reinterpret_cast<uint32_t *>(p.bytes + p.frame_off[s]);
    if (lane == 0) wr64(w, 0, n);
    unsigned long long base = 0;  // elements ascending = dictionary order = bit order
    for (unsigned long long w0b = 0; w0b < W; w0b += kWave) {
      const unsigned long long wi = w0b + lane;
      u64 x = wi < W ? r[wi] : 0;
      const unsigned c = __popcll(x);
      unsigned long long pre = c;  // inclusive prefix of the lane counts
      for (int off = 1; off < kWave; off <<= 1) {
        const unsigned long long t = __shfl_up(pre, off, kWave);
        if (lane >= off) pre += t;
      }
      unsigned long long i = base + pre - c;
      while (x) {
        const int b = __builtin_ctzll(x);
        x &= x - 1;
        wr64(w, 2 + 2 * i, p.elems[wi * 64 + b]);
        ++i;
      }
      base += __shfl(pre, kWave - 1, kWave);
    }
  }
}

__global__ __launch_bounds__(kBlock) void lwwreg_egress_kernel(const u64 *marker, const u64 *val, unsigned long long N,
                                                               uint8_t *bytes) {
  for (unsigned long long s = blockIdx.x * (unsigned long long)kBlock + threadIdx.x; s < N;
       s += (unsigned long long)gridDim.x * kBlock) {
    uint32_t *w = reinterpret_cast<uint32_t *>(bytes + 16 * s);
    wr64(w, 0, val[s]);
    wr64(w, 2, marker[s]);
  }
}

constexpr int kEgRows = 16;  // entry rows in flight per wave (egress, A <= 64)
constexpr int kEgKeys = 8;   // Map egress: keys in flight per wave (A <= 64, V <= kEgMaxV)
constexpr int kEgMaxV = 4;

// kEgRows rows m0.. of a [M][A] block, lane = actor: every load unconditional (rows past M and
// lanes past A re-read valid cells, then masked to 0), so all of them issue before the first wait.
__device__ __forceinline__ void eg_rows(u64 (&v)[kEgRows], const u64 *E, unsigned long long m0, unsigned long long M,
                                        unsigned long long A, bool on, int lane) {
  const unsigned long long a = on ? (unsigned long long)lane : 0;
#pragma unroll
  for (int j = 0; j < kEgRows; ++j) {
    const unsigned long long m = m0 + j < M ? m0 + j : M - 1;
    v[j] = E[m * A + a];
  }
#pragma unroll
  for (int j = 0; j < kEgRows; ++j)
    if (!on || m0 + j >= M) v[j] = 0;
}

// Orswot: clock; entries of every present member (index order); surviving removes.
__global__ __launch_bounds__(kBlock) void orswot_egress_kernel(EgressPlan p, int write) {
  const int lane = threadIdx.x % kWave;
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;
  const unsigned long long nw = (unsigned long long)gridDim.x * (kBlock / kWave);
  for (unsigned long long s = w0; s < p.N; s += nw) {
    const u64 *c = p.rows + s * p.row_stride;
    const u64 *E = p.entries + s * p.M * p.A;
    const u64 d0 = p.def_off ? p.def_off[s] : 0, d1 = p.def_off ? p.def_off[s + 1] : 0;
    uint32_t *w = write ? reinterpret_cast<uint32_t *>(p.bytes + p.frame_off[s]) : nullptr;
    u64 sz = 8 + 12 * nnz_row(c, p.A, lane);
    unsigned long long k = write ? write_vclock(w, 0, c, p.A, p.actors, lane) : 0;
    u64 ne = 0;
    if (p.A <= kWave) {
      // lane = actor: a row is one coalesced load, its nonzeros one ballot; kEgRows rows are
      // loaded before the first is examined (the rows are independent: a chain of one dependent
      // load per row was what bound this pass)
      const bool on = (unsigned long long)lane < p.A;
      const uint32_t act = on ? p.actors[lane] : 0u;
      u64 esz = 0;
      for (unsigned long long m0 = 0; m0 < (write ? 0 : p.M); m0 += kEgRows) {
        u64 v[kEgRows];
        eg_rows(v, E, m0, p.M, p.A, on, lane);
#pragma unroll
        for (int j = 0; j < kEgRows; ++j) {
          const u64 bm = __ballot(v[j] != 0);
          if (bm) {
            ++ne;
            esz += 16 + 12 * (u64)__popcll(bm);
          }
        }
      }
      sz += 8 + esz;
      if (write) {  // (the count sweep above is skipped when writing: ne goes to its slot at the end)
        const unsigned long long kne = k;
        ne = 0;
        k += 2;
        for (unsigned long long m0 = 0; m0 < p.M; m0 += kEgRows) {
          u64 v[kEgRows];
          eg_rows(v, E, m0, p.M, p.A, on, lane);
#pragma unroll
          for (int j = 0; j < kEgRows; ++j) {
            const u64 bm = __ballot(v[j] != 0);
            if (!bm) continue;
            const u64 n = __popcll(bm);
            if (lane == 0) {  // member, then the VClock: len, (actor, counter) ascending
              wr64(w, k, p.members[m0 + j]);
              wr64(w, k + 2, n);
            }
            if (v[j] != 0) {
              const unsigned long long i = __popcll(bm & ((1ull << lane) - 1));
              w[k + 4 + 3 * i] = act;
              wr64(w, k + 5 + 3 * i, v[j]);
            }
            k += 4 + 3 * n;
            ++ne;
          }
        }
        if (lane == 0) wr64(w, kne, ne);
      }
    } else {
      for (unsigned long long m = 0; m < p.M; ++m) ne += nnz_row(E + m * p.A, p.A, lane) != 0;
      sz += 8;
      if (write) {
        if (lane == 0) wr64(w, k, ne);
        k += 2;
      }
      for (unsigned long long m = 0; m < p.M; ++m) {
        const u64 n = nnz_row(E + m * p.A, p.A, lane);
        if (n == 0) continue;
        sz += 8 + 8 + 12 * n;
        if (write) {
          if (lane == 0) wr64(w, k, p.members[m]);
          k = write_vclock(w, k + 2, E + m * p.A, p.A, p.actors, lane);
        }
      }
    }
    u64 nd = 0;
    for (u64 d = d0; d < d1; ++d) nd += (!p.def_keep || p.def_keep[d]) ? 1 : 0;
    sz += 8;
    if (write) {
      if (lane == 0) wr64(w, k, nd);
      k += 2;
    }
    for (u64 d = d0; d < d1; ++d) {
      if (p.def_keep && !p.def_keep[d]) continue;
      const u64 *rm = p.def_clock + d * p.A, *mb = p.def_members + d * p.Mw;
      const u64 nm = popc_row(mb, p.Mw, lane);
      sz += 8 + 12 * nnz_row(rm, p.A, lane) + 8 + 8 * nm;
      if (!write) continue;
      k = write_vclock(w, k, rm, p.A, p.actors, lane);
      if (lane == 0) {
        wr64(w, k, nm);
        unsigned long long i = 0;
        for (unsigned long long x = 0; x < p.Mw; ++x) {
          u64 word = mb[x];
          while (word) {
            const int b = __builtin_ctzll(word);
            word &= word - 1;
            wr64(w, k + 2 + 2 * i, p.members[x * 64 + b]);
            ++i;
          }
        }
      }
      k += 2 + 2 * nm;
    }
    if (!write && lane == 0) p.sizes[s] = sz;
  }
}

// ---- Map<u32, MVReg<u64>> ------------------------------------------------------------------------
struct MapWirePlan {
  const uint8_t *bytes;
  const u64 *frame_off;
  unsigned long long N, A, K, Kw, V, Dcap;
  const uint32_t *actors, *keys;  // sorted dictionaries
  u64 *clock, *ec, *vclk, *vval;  // [N][A], [N][K][A], [N][K][V][A], [N][K][V] (zero-filled before ingest)
  u64 *def_clock, *def_keys;      // [N][Dcap][A], [N][Dcap][Kw]
  uint32_t *def_count;            // [N]
  uint32_t *status;
  int stage;                      // dictionaries staged in LDS
  // egress
  u64 *sizes;
  const u64 *frame_out;
  uint8_t *out;
};

// One wave per state: the entries in frame order (the record loop of each VClock across lanes),
// value clocks into the key's slots in Vec order, the deferred removes into the state's slots.
// status: kWireBad (malformed / trailing bytes), kWireMissing (an actor or key not in the
// dictionaries: skipped), kWireCap (more values than V for a key, or removes than Dcap: dropped).
__global__ __launch_bounds__(kBlock) void map_ingest_kernel(MapWirePlan p) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x % kWave, wib = threadIdx.x / kWave;
  const int wpb = blockDim.x / kWave;
  const uint32_t *actors = p.actors, *keys = p.keys;
  u64 *base = lds;
  if (p.stage) {  // [actors u32 | keys u32], each padded to 8 bytes
    uint32_t *la = reinterpret_cast<uint32_t *>(lds);
    const unsigned long long aw = (p.A + 1) / 2, kw = (p.K + 1) / 2;
    for (unsigned long long i = threadIdx.x; i < p.A; i += blockDim.x) la[i] = p.actors[i];
    uint32_t *lk = reinterpret_cast<uint32_t *>(lds + aw);
    for (unsigned long long i = threadIdx.x; i < p.K; i += blockDim.x) lk[i] = p.keys[i];
    __syncthreads();
    actors = la;
    keys = lk;
    base = lds + aw + kw;
  }
  u64 *row = base + (unsigned long long)wib * (p.A + p.Kw);
  u64 *bits = row + p.A;
  for (unsigned long long s = (unsigned long long)blockIdx.x * wpb + wib; s < p.N;
       s += (unsigned long long)gridDim.x * wpb) {
    unsigned st = 0;
    unsigned long long nd = 0;
    Frame f;
    const u64 b = p.frame_off[s], e = p.frame_off[s + 1];
    if ((b & 3) || (e & 3) || e < b) {
      st = kWireBad;
    } else {
      f.w = reinterpret_cast<const uint32_t *>(p.bytes + b);
      f.nw = (e - b) / 4;
      unsigned long long k = parse_vclock(f, 0, actors, p.A, row, lane, st);
      store_row<u64>(p.clock + s * p.A, row, p.A, lane);
      wfence();
      if (k == ~0ull || k + 2 > f.nw) {
        st |= kWireBad;
        k = ~0ull;
      }
      const u64 n = k == ~0ull ? 0 : rd64(f.w, k);
      if (k != ~0ull) k += 2;
      for (u64 en = 0; en < n && k != ~0ull; ++en) {
        if (k + 1 > f.nw) {
          st |= kWireBad;
          k = ~0ull;
          break;
        }
        const long long ki = find_u32(keys, p.K, f.w[k], en);
        if (ki < 0) st |= kWireMissing;
        k = parse_vclock(f, k + 1, actors, p.A, row, lane, st);
        if (k == ~0ull || k + 2 > f.nw) {
          st |= kWireBad;
          k = ~0ull;
          break;
        }
        if (ki >= 0) store_row<u64>(p.ec + (s * p.K + (unsigned long long)ki) * p.A, row, p.A, lane);
        wfence();
        const u64 m = rd64(f.w, k);
        k += 2;
        for (u64 v = 0; v < m && k != ~0ull; ++v) {
          k = parse_vclock(f, k, actors, p.A, row, lane, st);
          if (k == ~0ull || k + 2 > f.nw) {
            st |= kWireBad;
            k = ~0ull;
            break;
          }
          const u64 val = rd64(f.w, k);
          k += 2;
          if (ki >= 0) {
            if (v < p.V) {
              const unsigned long long slot = (s * p.K + (unsigned long long)ki) * p.V + v;
              store_row<u64>(p.vclk + slot * p.A, row, p.A, lane);
              if (lane == 0) p.vval[slot] = val;
            } else {
              st |= kWireCap;
            }
          }
          wfence();
        }
      }
      if (k != ~0ull && k + 2 <= f.nw) {
        const u64 d = rd64(f.w, k);
        k += 2;
        for (u64 j = 0; j < d && k != ~0ull; ++j) {
          k = parse_vclock(f, k, actors, p.A, row, lane, st);
          for (unsigned long long w = lane; w < p.Kw; w += kWave) bits[w] = 0;
          wfence();
          if (k == ~0ull || k + 2 > f.nw) {
            st |= kWireBad;
            k = ~0ull;
            break;
          }
          const u64 nk = rd64(f.w, k);
          k += 2;
          if (nk > f.nw - k) {
            st |= kWireBad;
            k = ~0ull;
            break;
          }
          bool miss = false;
          for (unsigned long long i = lane; i < nk; i += kWave) {
            const long long kb = find_u32(keys, p.K, f.w[k + i], i);
            if (kb < 0) miss = true;
            else atomicOr(bits + kb / 64, 1ull << (kb % 64));
          }
          if (__ballot(miss)) st |= kWireMissing;
          k += nk;
          wfence();
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
        st |= kWireBad;
        k = ~0ull;
      }
      if (k != f.nw) st |= kWireBad;
    }
    if (lane == 0) {
      p.status[s] = st;
      p.def_count[s] = (uint32_t)nd;
    }
  }
}

// ---- Map ingest, round 3: walk + batched parse ---------------------------------------------------
// map_ingest_kernel above is one dependent chain per state: every VClock waits for its length, then
// for its records, then fences its LDS row out (3 x 1,024 VClocks per config-4 state).  Here a state
// is parsed in two roles by the same wave:
//   the walk (scalar): only the lengths, keys, value counts and values — the positions of the
//     VClocks and where each one goes — read from a 256-word register window of the frame; the
//     frame streams through a per-wave LDS ring of kWalkRing windows by LDS-DMA, issued
//     kWalkRing windows ahead of the walk, so a length costs a readlane, not a memory round trip;
//   the parse (lane = VClock): every 64 VClocks found, lane i parses VClock i's records (loads in
//     flight together, L2 hits behind the DMA) and stores each counter straight into its
//     zero-filled destination row (no LDS row, no fence).
// Deferred removes (a few per state, at the end of the frame) keep the row-staged parse.
constexpr int kWalkWin = 256;  // words per window (one per lane per register, 4 registers)
constexpr int kWalkRing = 8;   // LDS ring windows per wave

template <int N>
__device__ __forceinline__ void wire_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// A wave-uniform 64-bit value the compiler cannot prove uniform (the walk's positions): made so, so
// that the walk's arithmetic and branches stay scalar instead of EXEC-masked vector code.
__device__ __forceinline__ unsigned long long uni64(unsigned long long x) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)x), hi = __builtin_amdgcn_readfirstlane((unsigned)(x >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

template <int RING = kWalkRing>
struct MapWalk {
  const uint32_t *fw;
  unsigned long long nw, nwin, issued, cur;
  uint32_t *ring;
  uint32_t r0, r1, r2, r3;

  __device__ void dma(unsigned long long wi, int lane) {
    uint32_t *dst = ring + (wi % RING) * kWalkWin;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned long long w = wi * kWalkWin + 64 * j + lane;
      __builtin_amdgcn_global_load_lds(fw + (w < nw ? w : nw - 1),
                                       (__attribute__((address_space(3))) void *)(dst + 64 * j), 4, 0, 0);
    }
  }
  __device__ void start(int lane) {
    nw = uni64(nw);
    nwin = uni64(nwin);
    issued = 0;
    cur = ~0ull;
    while (issued < nwin && issued < (unsigned long long)RING) {
      dma(issued, lane);
      issued = uni64(issued + 1);
    }
  }
  // window wi into registers (wi > cur); then keep the ring full
  __device__ void load(unsigned long long wi, int lane) {
    // windows issued after wi: every vector-memory op issued since wi's DMA counts too, so this
    // waits at least for wi (in-order counter)
    switch ((int)(issued - 1 - wi)) {
      case 0: wire_vmcnt<0>(); break;
      case 1: wire_vmcnt<4>(); break;
      case 2: wire_vmcnt<8>(); break;
      case 3: wire_vmcnt<12>(); break;
      case 4: wire_vmcnt<16>(); break;
      case 5: wire_vmcnt<20>(); break;
      case 6: wire_vmcnt<24>(); break;
      default: wire_vmcnt<28>(); break;
    }
    const uint32_t *src = ring + (wi % RING) * kWalkWin + lane;
    r0 = src[0];
    r1 = src[64];
    r2 = src[128];
    r3 = src[192];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is read: it may be refilled
    cur = uni64(wi);
    while (issued < nwin && issued <= wi + RING) {
      dma(issued, lane);
      issued = uni64(issued + 1);
    }
  }
  __device__ uint32_t get(unsigned long long k, int lane) {
    k = uni64(k);
    const unsigned long long wi = k / kWalkWin;
    if (wi != uni64(cur)) load(wi, lane);
    const int off = (int)(k % kWalkWin), l = off & 63, q = off >> 6;
    // four readlanes and scalar selects: a switch over r0..r3 may be lowered as an indexed access
    // to a stack copy of them (scratch: a memory round trip per word read)
    const uint32_t a = __builtin_amdgcn_readlane(r0, l), b = __builtin_amdgcn_readlane(r1, l);
    const uint32_t c = __builtin_amdgcn_readlane(r2, l), d = __builtin_amdgcn_readlane(r3, l);
    return q == 0 ? a : (q == 1 ? b : (q == 2 ? c : d));
  }
  __device__ u64 get64(unsigned long long k, int lane) { return (u64)get(k, lane) | ((u64)get(k + 1, lane) << 32); }
};

// The batched parse: lane i < cnt parses the VClock at word pos of n records into row dst.
__device__ __forceinline__ bool walk_parse(const uint32_t *fw, const uint32_t *actors, unsigned long long A,
                                           int lane, int cnt, unsigned long long pos, unsigned long long n, u64 *dst) {
  bool miss = false;
  if (lane < cnt) {
    const uint32_t *rec = fw + pos + 2;
    for (unsigned long long r = 0; r < n; r += 4) {
      uint32_t id[4];
      u64 c[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // all loads of the group in flight before the first lookup
        const unsigned long long i = r + u < n ? r + u : n - 1;
        id[u] = rec[3 * i];
        c[u] = (u64)rec[3 * i + 1] | ((u64)rec[3 * i + 2] << 32);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (r + u < n) {
          const long long col = find_u32(actors, A, id[u], r + u);
          if (col < 0) miss = true;
          else dst[col] = c[u];
        }
    }
  }
  return miss;
}

__global__ __launch_bounds__(kBlock) void map_ingest_walk_kernel(MapWirePlan p) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x % kWave, wib = threadIdx.x / kWave;
  const int wpb = blockDim.x / kWave;
  const uint32_t *actors = p.actors, *keys = p.keys;
  u64 *base = lds;
  if (p.stage) {  // [actors u32 | keys u32], each padded to 8 bytes
    uint32_t *la = reinterpret_cast<uint32_t *>(lds);
    const unsigned long long aw = (p.A + 1) / 2, kw = (p.K + 1) / 2;
    for (unsigned long long i = threadIdx.x; i < p.A; i += blockDim.x) la[i] = p.actors[i];
    uint32_t *lk = reinterpret_cast<uint32_t *>(lds + aw);
    for (unsigned long long i = threadIdx.x; i < p.K; i += blockDim.x) lk[i] = p.keys[i];
    __syncthreads();
    actors = la;
    keys = lk;
    base = lds + aw + kw;
  }
  const unsigned long long per_wave = kWalkRing * kWalkWin / 2 + p.A + p.Kw;  // u64 words
  u64 *mine = base + (unsigned long long)wib * per_wave;
  uint32_t *ring = reinterpret_cast<uint32_t *>(mine);
  u64 *row = mine + kWalkRing * kWalkWin / 2;
  u64 *bits = row + p.A;
  for (unsigned long long s = (unsigned long long)blockIdx.x * wpb + wib; s < p.N;
       s += (unsigned long long)gridDim.x * wpb) {
    unsigned st = 0;
    unsigned long long nd = 0;
    const u64 b = p.frame_off[s], e = p.frame_off[s + 1];
    if ((b & 3) || (e & 3) || e < b || e - b < 16) {
      st = kWireBad;  // (a valid frame holds at least the clock and entry counts)
    } else {
      MapWalk<> w;
      w.fw = reinterpret_cast<const uint32_t *>(p.bytes + b);
      w.nw = (e - b) / 4;
      w.nwin = (w.nw + kWalkWin - 1) / kWalkWin;
      w.ring = ring;
      w.start(lane);
      // the batch of VClocks the lanes parse next: lane i holds entry i
      int cnt = 0;
      unsigned long long dpos = 0, dn = 0;
      u64 *ddst = nullptr;
      bool miss = false;
      auto push = [&](unsigned long long pos, unsigned long long n, u64 *dst) {
        if (lane == cnt) {
          dpos = pos;
          dn = n;
          ddst = dst;
        }
        if (++cnt == kWave) {
          miss |= walk_parse(w.fw, actors, p.A, lane, cnt, dpos, dn, ddst);
          cnt = 0;
        }
      };
      // a VClock's record count at k, checked against the frame (~0: malformed)
      auto clock_len = [&](unsigned long long k) -> unsigned long long {
        if (k + 2 > w.nw) return ~0ull;
        const u64 n = w.get64(k, lane);
        return n > (w.nw - k - 2) / 3 ? ~0ull : n;
      };
      unsigned long long k = 0;
      unsigned long long n = clock_len(0);
      if (n == ~0ull) {
        st |= kWireBad;
        k = ~0ull;
      } else {
        n = uni64(n);
        push(0, n, p.clock + s * p.A);
        k = uni64(2 + 3 * n);
      }
      if (k != ~0ull && k + 2 > w.nw) {
        st |= kWireBad;
        k = ~0ull;
      }
      const u64 ne = k == ~0ull ? 0 : w.get64(k, lane);
      if (k != ~0ull) k += 2;
      long long hint = 0;
      for (u64 en = 0; en < ne && k != ~0ull; ++en) {
        if (k + 1 > w.nw) {
          st |= kWireBad;
          k = ~0ull;
          break;
        }
        const long long ki = find_u32(keys, p.K, w.get(k, lane), (unsigned long long)hint);
        if (ki < 0) st |= kWireMissing;
        else hint = ki + 1;
        n = uni64(clock_len(k + 1));
        if (n == ~0ull) {
          st |= kWireBad;
          k = ~0ull;
          break;
        }
        if (ki >= 0) push(k + 1, n, p.ec + (s * p.K + (unsigned long long)ki) * p.A);
        k = uni64(k + 3 + 3 * n);
        if (k + 2 > w.nw) {
          st |= kWireBad;
          k = ~0ull;
          break;
        }
        const u64 m = w.get64(k, lane);
        k = uni64(k + 2);
        for (u64 v = 0; v < m && k != ~0ull; ++v) {
          n = uni64(clock_len(k));
          if (n == ~0ull || k + 2 + 3 * n + 2 > w.nw) {
            st |= kWireBad;
            k = ~0ull;
            break;
          }
          const unsigned long long pos = k;
          k = uni64(k + 2 + 3 * n);
          const u64 val = w.get64(k, lane);
          k = uni64(k + 2);
          if (ki >= 0) {
            if (v < p.V) {
              const unsigned long long slot = (s * p.K + (unsigned long long)ki) * p.V + v;
              push(pos, n, p.vclk + slot * p.A);
              if (lane == 0) p.vval[slot] = val;
            } else {
              st |= kWireCap;
            }
          }
        }
      }
      if (cnt) miss |= walk_parse(w.fw, actors, p.A, lane, cnt, dpos, dn, ddst);
      if (__ballot(miss)) st |= kWireMissing;
      // deferred removes: the row-staged parse (rare; global reads)
      Frame f{w.fw, w.nw};
      if (k != ~0ull && k + 2 <= f.nw) {
        const u64 d = w.get64(k, lane);
        k += 2;
        for (u64 j = 0; j < d && k != ~0ull; ++j) {
          k = parse_vclock(f, k, actors, p.A, row, lane, st);
          for (unsigned long long x = lane; x < p.Kw; x += kWave) bits[x] = 0;
          wfence();
          if (k == ~0ull || k + 2 > f.nw) {
            st |= kWireBad;
            k = ~0ull;
            break;
          }
          const u64 nk = rd64(f.w, k);
          k += 2;
          if (nk > f.nw - k) {
            st |= kWireBad;
            k = ~0ull;
            break;
          }
          bool dmiss = false;
          for (unsigned long long i = lane; i < nk; i += kWave) {
            const long long kb = find_u32(keys, p.K, f.w[k + i], i);
            if (kb < 0) dmiss = true;
            else atomicOr(bits + kb / 64, 1ull << (kb % 64));
          }
          if (__ballot(dmiss)) st |= kWireMissing;
          k += nk;
          wfence();
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
        st |= kWireBad;
        k = ~0ull;
      }
      if (k != f.nw) st |= kWireBad;
      wire_vmcnt<0>();  // no DMA of this frame may land in the ring after the next state starts
    }
    if (lane == 0) {
      p.status[s] = st;
      p.def_count[s] = (uint32_t)nd;
    }
  }
}

// ---- Orswot ingest, round 3: walk + batched parse (pass 1) ----------------------------------------
// The same two roles as map_ingest_walk_kernel: the walk reads only the member ids and record counts
// (a readlane from the frame window the LDS ring holds), every 64 entries found the lanes parse one
// entry each — member lookup (binary search in the LDS dictionary), then its records straight into
// the zero-filled entry row.  Pass 3 (the deferred removes) is unchanged.
__device__ __forceinline__ bool walk_parse_members(const uint32_t *fw, const uint32_t *actors, unsigned long long A,
                                                   const u64 *members, unsigned long long M, int lane, int cnt,
                                                   unsigned long long pos, unsigned long long n, u64 id, u64 *ent) {
  if (lane >= cnt) return false;
  const long long mi = find_u64(members, M, id, M);
  if (mi < 0) return true;
  return walk_parse(fw, actors, A, lane, cnt, pos, n, ent + (unsigned long long)mi * A);
}

// 16 waves per block share one copy of the dictionaries, each with a 4-window frame ring: the walk is
// a dependent scalar chain per state, so its speed is the states in flight per SIMD (4 here; 2 with
// 4 waves per block and 8-window rings, which the 33-KiB member dictionary capped at 2 blocks/CU).
constexpr int kOrWalkRing = 4, kOrWalkWaves = 16;
__global__ __launch_bounds__(kOrWalkWaves * kWave) void orswot_ingest_walk_kernel(IngestPlan p) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x % kWave, wib = threadIdx.x / kWave;
  const int wpb = blockDim.x / kWave;
  const uint32_t *actors = p.actors;
  const u64 *elems = p.elems, *members = p.members;
  u64 *mine = stage_dicts(p, lds, actors, elems, members) + (unsigned long long)wib * (kOrWalkRing * kWalkWin / 2);
  uint32_t *ring = reinterpret_cast<uint32_t *>(mine);
  for (unsigned long long s = (unsigned long long)blockIdx.x * wpb + wib; s < p.N;
       s += (unsigned long long)gridDim.x * wpb) {
    unsigned st = 0;
    u64 dpos = 0, dcnt = 0;
    u64 *crow = p.out + s * p.row_stride;
    for (unsigned long long a = lane; a < p.A; a += kWave) crow[a] = 0;
    const u64 b = p.frame_off[s], e = p.frame_off[s + 1];
    if ((b & 3) || (e & 3) || e < b || e - b < 16) {
      st = kWireBad;  // (a valid frame holds at least the clock and entry counts)
    } else {
      MapWalk<kOrWalkRing> w;
      w.fw = reinterpret_cast<const uint32_t *>(p.bytes + b);
      w.nw = (e - b) / 4;
      w.nwin = (w.nw + kWalkWin - 1) / kWalkWin;
      w.ring = ring;
      w.start(lane);
      u64 *ent = p.entries + s * p.M * p.A;
#ifdef WIRE_STATS
      u64 t_all = __builtin_amdgcn_s_memtime(), t_parse = 0, t0 = 0, n_ent = 0, n_win = 0;
#define WS_T0() (t0 = __builtin_amdgcn_s_memtime())
#define WS_T1() (t_parse += __builtin_amdgcn_s_memtime() - t0)
#else
#define WS_T0() ((void)0)
#define WS_T1() ((void)0)
#endif
      int cnt = 0;  // the batch the lanes parse next: lane i holds entry i
      unsigned long long bpos = 0, bn = 0;
      u64 bid = 0;
      bool miss = false;
      auto clock_len = [&](unsigned long long k) -> unsigned long long {
        if (k + 2 > w.nw) return ~0ull;
        const u64 n = w.get64(k, lane);
        return n > (w.nw - k - 2) / 3 ? ~0ull : n;
      };
      unsigned long long k = 0;
      unsigned long long n = clock_len(0);
      if (n == ~0ull) {
        st |= kWireBad;
        k = ~0ull;
      } else {
        miss |= walk_parse(w.fw, actors, p.A, lane, 1, 0, n, crow);
        k = 2 + 3 * n;
      }
      if (k != ~0ull && k + 2 > w.nw) {
        st |= kWireBad;
        k = ~0ull;
      }
      const u64 ne = k == ~0ull ? 0 : w.get64(k, lane);
      if (k != ~0ull) k += 2;
      for (u64 en = 0; en < ne && k != ~0ull; ++en) {
        if (k + 2 > w.nw) {
          st |= kWireBad;
          k = ~0ull;
          break;
        }
        const u64 id = w.get64(k, lane);
        n = clock_len(k + 2);
        if (n == ~0ull) {
          st |= kWireBad;
          k = ~0ull;
          break;
        }
        n = uni64(n);
        if (lane == cnt) {
          bpos = k + 2;
          bn = n;
          bid = id;
        }
        if (++cnt == kWave) {
          WS_T0();
          miss |= walk_parse_members(w.fw, actors, p.A, members, p.M, lane, cnt, bpos, bn, bid, ent);
          WS_T1();
          cnt = 0;
        }
        k = uni64(k + 4 + 3 * n);
#ifdef WIRE_STATS
        ++n_ent;
#endif
      }
      if (cnt) miss |= walk_parse_members(w.fw, actors, p.A, members, p.M, lane, cnt, bpos, bn, bid, ent);
#ifdef WIRE_STATS
      if (lane == 0 && s % 509 == 0)
        printf("s=%llu entries=%llu windows=%llu cyc all=%llu parse=%llu\n", s, n_ent, w.nwin,
               __builtin_amdgcn_s_memtime() - t_all, t_parse);
#endif
      if (__ballot(miss)) st |= kWireMissing;
      if (k != ~0ull && k + 2 <= w.nw) {
        dcnt = w.get64(k, lane);
        dpos = k + 2;
        if (dcnt > (w.nw - dpos) / 4) {  // a lying count (see orswot_ingest_kernel)
          st |= kWireBad;
          dcnt = 0;
        }
      } else {
        st |= kWireBad;
      }
      wire_vmcnt<0>();  // no DMA of this frame may land in the ring after the next state starts
    }
    if (lane == 0) {
      p.status[s] = st;
      p.dpos[s] = dpos;
      p.dcount[s] = (st & kWireBad) ? 0 : dcnt;
    }
  }
}

// ---- Orswot ingest, round 4: rows zeroed by filler waves while the walk runs ----------------------
// The dense entries of a state are ~60x its frame (config 3: 2 MiB of rows per 35 KiB frame), and a
// separate zero-fill pass before the walk costs as much HBM time as the walk itself.  Here the block
// holds kOfWalk walker waves and kOfFill filler waves: a filler zeroes its walkers' entry blocks with
// 16-byte non-temporal stores while the walkers walk (the walk is a scalar chain, latency-bound; the
// zeroing is write-bandwidth-bound, so the two overlap), then publishes "state zeroed" in LDS after
// its stores completed (vmcnt(0) + release).  A walker only records the entries it finds — the word
// position of each, in a per-state scratch list of up to M — and parses them once its state is
// zeroed (acquire), in batches of 64 as before: every present member's counters land in a zeroed
// row, no row is written before it is zero.  (Separate waves: a walker's own stores would enter the
// in-order vmcnt its window DMA waits on.)  A frame with more than M entries parses the overflow at
// once, after the wait: the same order of row writes as the one-pass kernel.
constexpr int kOfWalk = 8, kOfFill = 2;
__global__ __launch_bounds__((kOfWalk + kOfFill) * kWave) void orswot_ingest_walk_fill_kernel(IngestPlan p,
                                                                                             uint32_t *epos) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x % kWave, wib = threadIdx.x / kWave;
  const uint32_t *actors = p.actors;
  const u64 *elems = p.elems, *members = p.members;
  u64 *base = stage_dicts(p, lds, actors, elems, members);
  unsigned *zeroed = reinterpret_cast<unsigned *>(base);  // [kOfWalk]: iterations zeroed, per walker
  u64 *rings = base + (kOfWalk + 1) / 2;
  if (threadIdx.x < kOfWalk) zeroed[threadIdx.x] = 0;
  __syncthreads();  // (the last barrier: walkers and fillers part here)
  const unsigned long long MA = p.M * p.A;
  if (wib >= kOfWalk) {  // ---- filler: walkers f, f + kOfFill, ... of every iteration
    const int f = wib - kOfWalk;
    unsigned it = 0;
    for (unsigned long long s0 = (unsigned long long)blockIdx.x * kOfWalk; s0 < p.N;
         s0 += (unsigned long long)gridDim.x * kOfWalk, ++it) {
      for (int w = f; w < kOfWalk; w += kOfFill) {
        const unsigned long long s = s0 + w;
        if (s >= p.N) break;
        u64 *ent = p.entries + s * MA;
        if ((reinterpret_cast<uintptr_t>(ent) & 15) == 0 && MA % 2 == 0) {
          u64x2 *e2 = reinterpret_cast<u64x2 *>(ent);
          u64x2 z;
          z.x = 0;
          z.y = 0;
          for (unsigned long long i = lane; i < MA / 2; i += kWave) __builtin_nontemporal_store(z, e2 + i);
        } else {
          for (unsigned long long i = lane; i < MA; i += kWave) __builtin_nontemporal_store(0ull, ent + i);
        }
        wire_vmcnt<0>();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (lane == 0) __hip_atomic_store(zeroed + w, it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    return;
  }
  // ---- walker
  u64 *mine = rings + (unsigned long long)wib * (kOrWalkRing * kWalkWin / 2);
  uint32_t *ring = reinterpret_cast<uint32_t *>(mine);
  unsigned it = 0;
  for (unsigned long long s = (unsigned long long)blockIdx.x * kOfWalk + wib; s < p.N;
       s += (unsigned long long)gridDim.x * kOfWalk, ++it) {
    unsigned st = 0;
    u64 dpos = 0, dcnt = 0;
    u64 *crow = p.out + s * p.row_stride;
    for (unsigned long long a = lane; a < p.A; a += kWave) crow[a] = 0;
    uint32_t *ep = epos + s * p.M;  // this state's entry positions (up to M)
    bool ready = false;             // this state's rows are zeroed (waited for)
    auto wait_zeroed = [&]() {
      if (ready) return;
      while (__builtin_amdgcn_readfirstlane(
                 __hip_atomic_load(zeroed + wib, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < it + 1)
        __builtin_amdgcn_s_sleep(2);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      ready = true;
    };
    const u64 b = p.frame_off[s], e = p.frame_off[s + 1];
    if ((b & 3) || (e & 3) || e < b || e - b < 16) {
      st = kWireBad;
    } else {
      MapWalk<kOrWalkRing> w;
      w.fw = reinterpret_cast<const uint32_t *>(p.bytes + b);
      w.nw = (e - b) / 4;
      w.nwin = (w.nw + kWalkWin - 1) / kWalkWin;
      w.ring = ring;
      w.start(lane);
      u64 *ent = p.entries + s * MA;
      bool miss = false;
      // parse the entries recorded at ep[e0 .. e1) (lane = entry)
      auto parse_stash = [&](unsigned long long e0, unsigned long long e1) {
        for (unsigned long long x = e0; x < e1; x += kWave) {
          const int cnt = (int)(e1 - x < (unsigned long long)kWave ? e1 - x : kWave);
          unsigned long long k = 0, n = 0;
          u64 id = 0;
          if (lane < cnt) {
            k = ep[x + lane];
            id = (u64)w.fw[k] | ((u64)w.fw[k + 1] << 32);
            n = (u64)w.fw[k + 2] | ((u64)w.fw[k + 3] << 32);
          }
          miss |= walk_parse_members(w.fw, actors, p.A, members, p.M, lane, cnt, k + 2, n, id, ent);
        }
      };
      auto clock_len = [&](unsigned long long k) -> unsigned long long {
        if (k + 2 > w.nw) return ~0ull;
        const u64 n = w.get64(k, lane);
        return n > (w.nw - k - 2) / 3 ? ~0ull : n;
      };
      unsigned long long k = 0;
      unsigned long long n = clock_len(0);
      if (n == ~0ull) {
        st |= kWireBad;
        k = ~0ull;
      } else {
        miss |= walk_parse(w.fw, actors, p.A, lane, 1, 0, n, crow);
        k = 2 + 3 * n;
      }
      if (k != ~0ull && k + 2 > w.nw) {
        st |= kWireBad;
        k = ~0ull;
      }
      const u64 ne = k == ~0ull ? 0 : w.get64(k, lane);
      if (k != ~0ull) k += 2;
      unsigned long long stashed = 0;  // entries recorded in ep[], not parsed yet
      int cnt = 0;                     // entries of the current 64-batch; lane i holds entry i's start
      uint32_t bk = 0;
      for (u64 en = 0; en < ne && k != ~0ull; ++en) {
        if (k + 2 > w.nw) {
          st |= kWireBad;
          k = ~0ull;
          break;
        }
        n = clock_len(k + 2);
        if (n == ~0ull) {
          st |= kWireBad;
          k = ~0ull;
          break;
        }
        n = uni64(n);
        if (lane == cnt) bk = (uint32_t)k;
        if (++cnt == kWave) {
          if (stashed + kWave <= p.M) {  // record the batch's positions (one 256-byte store)
            ep[stashed + lane] = bk;
            stashed += kWave;
          } else {  // more entries than M: the stash first, then this batch, at once
            wait_zeroed();
            parse_stash(0, stashed);
            stashed = 0;
            ep[lane] = bk;
            parse_stash(0, kWave);
          }
          cnt = 0;
        }
        k = uni64(k + 4 + 3 * n);
      }
      if (k != ~0ull && k + 2 <= w.nw) {
        dcnt = w.get64(k, lane);
        dpos = k + 2;
        if (dcnt > (w.nw - dpos) / 4) {  // a lying count (see orswot_ingest_kernel)
          st |= kWireBad;
          dcnt = 0;
        }
      } else {
        st |= kWireBad;
      }
      wire_vmcnt<0>();  // no DMA of this frame may land in the ring after the next state starts
      // the rows: zeroed by the filler by now (the walk outlasts the zeroing), then parsed in order
      if (cnt && stashed + (unsigned long long)cnt <= p.M) {
        if (lane < cnt) ep[stashed + lane] = bk;
        stashed += cnt;
        cnt = 0;
      }
      wait_zeroed();
      parse_stash(0, stashed);
      if (cnt) {  // (the M-overflow case: the last partial batch)
        if (lane < cnt) ep[lane] = bk;
        parse_stash(0, cnt);
      }
      if (__ballot(miss)) st |= kWireMissing;
    }
    wait_zeroed();  // (a bad frame too: the filler zeroed its rows, the output of a bad frame is zero)
    if (lane == 0) {
      p.status[s] = st;
      p.dpos[s] = dpos;
      p.dcount[s] = (st & kWireBad) ? 0 : dcnt;
    }
  }
}

// Egress, count (write = 0: frame sizes) or write pass: clock; present keys ascending with their
// occupied value slots in slot (Vec) order; the state's deferred slots.
__global__ __launch_bounds__(kBlock) void map_egress_kernel(MapWirePlan p, int write) {
  const int lane = threadIdx.x % kWave;
  const unsigned long long w0 = (blockIdx.x * (unsigned long long)kBlock + threadIdx.x) / kWave;
  const unsigned long long nw = (unsigned long long)gridDim.x * (kBlock / kWave);
  for (unsigned long long s = w0; s < p.N; s += nw) {
    const u64 *c = p.clock + s * p.A;
    uint32_t *w = write ? reinterpret_cast<uint32_t *>(p.out + p.frame_out[s]) : nullptr;
    u64 sz = 8 + 12 * nnz_row(c, p.A, lane);
    unsigned long long k = write ? write_vclock(w, 0, c, p.A, p.actors, lane) : 0;
    u64 ne = 0;
    if (p.A <= kWave && p.V <= kEgMaxV) {
      // lane = actor: every row of kEgKeys keys (entry clock + V value clocks) is loaded before the
      // first is examined, nonzeros are ballots (the plain loop below was a chain of one dependent
      // load and a shuffle reduction per row)
      const bool on = (unsigned long long)lane < p.A;
      const uint32_t act = on ? p.actors[lane] : 0u;
      {
        const int pass = write ? 1 : 0;  // count sweep, or write sweep (ne to its slot at the end)
        u64 esz = 0;
        const unsigned long long kne = k;
        if (pass == 1) k += 2;
        ne = 0;
        for (unsigned long long k0 = 0; k0 < p.K; k0 += kEgKeys) {
          u64 e[kEgKeys], vc[kEgKeys][kEgMaxV];
          {  // every load unconditional (clamped to valid cells), then masked: all issue before a wait
            const unsigned long long al = on ? (unsigned long long)lane : 0;
#pragma unroll
            for (int j = 0; j < kEgKeys; ++j) {
              const unsigned long long sk = s * p.K + (k0 + j < p.K ? k0 + j : p.K - 1);
              e[j] = p.ec[sk * p.A + al];
#pragma unroll
              for (int t = 0; t < kEgMaxV; ++t)
                vc[j][t] = p.vclk[(sk * p.V + ((unsigned long long)t < p.V ? t : p.V - 1)) * p.A + al];
            }
#pragma unroll
            for (int j = 0; j < kEgKeys; ++j) {
              const bool kon = on && k0 + j < p.K;
              if (!kon) e[j] = 0;
#pragma unroll
              for (int t = 0; t < kEgMaxV; ++t)
                if (!kon || (unsigned long long)t >= p.V) vc[j][t] = 0;
            }
          }
          // the batch's values: lane j * V + t holds key k0 + j's slot t
          u64 vv = 0;
          if (pass == 1 && (unsigned long long)lane < kEgKeys * p.V) {
            const unsigned long long j = lane / p.V, t = lane % p.V;
            if (k0 + j < p.K) vv = p.vval[(s * p.K + k0 + j) * p.V + t];
          }
#pragma unroll
          for (int j = 0; j < kEgKeys; ++j) {
            const u64 be = __ballot(e[j] != 0);
            if (!be) continue;
            ++ne;
            const u64 n = __popcll(be);
            u64 bv[kEgMaxV], m = 0, vsz = 0;
#pragma unroll
            for (int t = 0; t < kEgMaxV; ++t) {
              bv[t] = __ballot(vc[j][t] != 0);
              if (bv[t]) {
                ++m;
                vsz += 8 + 12 * (u64)__popcll(bv[t]) + 8;
              }
            }
            esz += 4 + 8 + 12 * n + 8 + vsz;
            if (pass == 0) continue;
            const unsigned long long below = (1ull << lane) - 1;
            if (lane == 0) {  // key, entry clock length
              w[k] = p.keys[k0 + j];
              wr64(w, k + 1, n);
            }
            if (e[j] != 0) {
              const unsigned long long i = __popcll(be & below);
              w[k + 3 + 3 * i] = act;
              wr64(w, k + 4 + 3 * i, e[j]);
            }
            k += 3 + 3 * n;
            if (lane == 0) wr64(w, k, m);
            k += 2;
#pragma unroll
            for (int t = 0; t < kEgMaxV; ++t) {
              if (!bv[t]) continue;
              const u64 nv = __popcll(bv[t]);
              const u64 val = __shfl(vv, j * (int)p.V + t, kWave);
              if (lane == 0) {
                wr64(w, k, nv);
                wr64(w, k + 2 + 3 * nv, val);
              }
              if (vc[j][t] != 0) {
                const unsigned long long i = __popcll(bv[t] & below);
                w[k + 2 + 3 * i] = act;
                wr64(w, k + 3 + 3 * i, vc[j][t]);
              }
              k += 2 + 3 * nv + 2;
            }
          }
        }
        if (pass == 0) sz += 8 + esz;
        else if (lane == 0) wr64(w, kne, ne);
      }
    } else {
    for (unsigned long long key = 0; key < p.K; ++key) ne += nnz_row(p.ec + (s * p.K + key) * p.A, p.A, lane) != 0;
    sz += 8;
    if (write) {
      if (lane == 0) wr64(w, k, ne);
      k += 2;
    }
    for (unsigned long long key = 0; key < p.K; ++key) {
      const u64 *er = p.ec + (s * p.K + key) * p.A;
      const u64 n = nnz_row(er, p.A, lane);
      if (n == 0) continue;
      const unsigned long long slot0 = (s * p.K + key) * p.V;
      u64 m = 0, vsz = 0;
      for (unsigned long long v = 0; v < p.V; ++v) {
        const u64 nv = nnz_row(p.vclk + (slot0 + v) * p.A, p.A, lane);
        if (nv) {
          ++m;
          vsz += 8 + 12 * nv + 8;
        }
      }
      sz += 4 + 8 + 12 * n + 8 + vsz;
      if (!write) continue;
      if (lane == 0) w[k] = p.keys[key];
      k = write_vclock(w, k + 1, er, p.A, p.actors, lane);
      if (lane == 0) wr64(w, k, m);
      k += 2;
      for (unsigned long long v = 0; v < p.V; ++v) {
        const u64 *vr = p.vclk + (slot0 + v) * p.A;
        if (nnz_row(vr, p.A, lane) == 0) continue;
        k = write_vclock(w, k, vr, p.A, p.actors, lane);
        if (lane == 0) wr64(w, k, p.vval[slot0 + v]);
        k += 2;
      }
    }
    }
    const unsigned long long nd = p.def_count ? p.def_count[s] : 0;
    sz += 8;
    if (write) {
      if (lane == 0) wr64(w, k, nd);
      k += 2;
    }
    for (unsigned long long d = 0; d < nd && d < p.Dcap; ++d) {
      const u64 *rm = p.def_clock + (s * p.Dcap + d) * p.A, *kb = p.def_keys + (s * p.Dcap + d) * p.Kw;
      const u64 nk = popc_row(kb, p.Kw, lane);
      sz += 8 + 12 * nnz_row(rm, p.A, lane) + 8 + 4 * nk;
      if (!write) continue;
      k = write_vclock(w, k, rm, p.A, p.actors, lane);
      if (lane == 0) wr64(w, k, nk);
      // keys ascending = bit order: lanes take bitmap words, a wave prefix sum places them
      unsigned long long basei = 0;
      for (unsigned long long x0 = 0; x0 < p.Kw; x0 += kWave) {
        const unsigned long long x = x0 + lane;
        u64 word = x < p.Kw ? kb[x] : 0;
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
          w[k + 2 + i] = p.keys[x * 64 + b];
          ++i;
        }
        basei += __shfl(pre, kWave - 1, kWave);
      }
      k += 2 + nk;
    }
    if (!write && lane == 0) p.sizes[s] = sz;
  }
}

// frame sizes -> frame_off (device, N+1) -> *total; returns CRDT_OK
int egress_layout(crdt_ctx *ctx, u64 *sizes, u64 *frame_off, unsigned long long N, size_t *total) {
  unsigned long long t = 0;
  u64 *sc = sizes + N;
  int rc = exclusive_scan(ctx, sizes, frame_off, N, sc, &t);
  if (rc) return rc;
  if (total) *total = t;
  return CRDT_OK;
}

}  // namespace crdt

using namespace crdt;

extern "C" {

static int vclock_ingest_common(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, size_t N,
                                const uint32_t *actors, size_t A, uint64_t *out, size_t row_stride, uint32_t *status,
                                int nclocks, const char *what) {
  CRDT_CHECK_CTX(ctx);
  if (N == 0) return CRDT_OK;
  if (int rc = check_frames(ctx, bytes, frame_off, N, status)) return rc;
  if (A == 0 || !actors || !out) return fail(ctx, CRDT_EINVAL, "%s: need actors (A >= 1) and out", what);
  if (A > (size_t)kWireRowLds) return fail(ctx, CRDT_EUNSUPPORTED, "%s: A = %zu > %d", what, A, kWireRowLds);
  if (row_stride < (size_t)nclocks * A) return fail(ctx, CRDT_EINVAL, "%s: row_stride < %d*A", what, nclocks);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  int wpb = 4;
  while (wpb > 1 && (size_t)wpb * A * 8 > 64 * 1024) --wpb;
  IngestPlan p{};
  p.bytes = bytes;
  p.frame_off = (const u64 *)frame_off;
  p.N = N;
  p.actors = actors;
  p.A = A;
  p.out = (u64 *)out;
  p.row_stride = row_stride;
  p.nclocks = nclocks;
  p.status = status;
  const size_t dw = (A + 1) / 2;
  if ((dw + wpb * A) * 8 <= 64 * 1024) p.dict_words = dw;
  timing_begin(ctx, "wire_ingest");
  hipLaunchKernelGGL(vclock_ingest_kernel, dim3(wave_grid(ctx, N, wpb, 32)), dim3(wpb * kWave),
                     (p.dict_words + wpb * A) * 8, ctx->stream, p);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

int crdt_vclock_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, size_t N, const uint32_t *actors,
                       size_t A, uint64_t *out, size_t row_stride, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return vclock_ingest_common(ctx, bytes, frame_off, N, actors, A, out, row_stride, status, 1, "vclock_ingest");
}

int crdt_pncounter_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, size_t N,
                          const uint32_t *actors, size_t A, uint64_t *out, size_t row_stride, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  return vclock_ingest_common(ctx, bytes, frame_off, N, actors, A, out, row_stride, status, 2, "pncounter_ingest");
}

int crdt_gset_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, size_t N, const uint64_t *elems,
                     size_t U, uint64_t *out, size_t row_stride, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (N == 0) return CRDT_OK;
  if (int rc = check_frames(ctx, bytes, frame_off, N, status)) return rc;
  const size_t W = (U + 63) / 64;
  if (U == 0 || !elems || !out) return fail(ctx, CRDT_EINVAL, "gset_ingest: need elems (U >= 1) and out");
  if (W > (size_t)kWireRowLds) return fail(ctx, CRDT_EUNSUPPORTED, "gset_ingest: U = %zu too large", U);
  if (row_stride < W) return fail(ctx, CRDT_EINVAL, "gset_ingest: row_stride < ceil(U/64)");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  int wpb = 4;
  while (wpb > 1 && (size_t)wpb * W * 8 > 64 * 1024) --wpb;
  IngestPlan p{};
  p.bytes = bytes;
  p.frame_off = (const u64 *)frame_off;
  p.N = N;
  p.elems = (const u64 *)elems;
  p.U = U;
  p.out = (u64 *)out;
  p.row_stride = row_stride;
  p.status = status;
  if ((U + wpb * W) * 8 <= 64 * 1024) p.dict_words = U;
  timing_begin(ctx, "wire_ingest");
  hipLaunchKernelGGL(gset_ingest_kernel, dim3(wave_grid(ctx, N, wpb, 32)), dim3(wpb * kWave),
                     (p.dict_words + wpb * W) * 8, ctx->stream, p);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

int crdt_lwwreg_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, size_t N, uint64_t *marker,
                       uint64_t *val, uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (N == 0) return CRDT_OK;
  if (int rc = check_frames(ctx, bytes, frame_off, N, status)) return rc;
  if (!marker || !val) return fail(ctx, CRDT_EINVAL, "lwwreg_ingest: NULL output");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  IngestPlan p{};
  p.bytes = bytes;
  p.frame_off = (const u64 *)frame_off;
  p.N = N;
  p.status = status;
  hipLaunchKernelGGL(lwwreg_ingest_kernel, dim3(wave_grid(ctx, N, 4, 16)), dim3(kBlock), 0, ctx->stream, p,
                     (u64 *)marker, (u64 *)val);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

int crdt_orswot_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, size_t N, const uint32_t *actors,
                       size_t A, const uint64_t *members, size_t M, uint64_t *clock, uint64_t *entries,
                       uint64_t *def_off, uint64_t *def_clock, uint64_t *def_members, size_t def_cap, size_t *n_def,
                       uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (n_def) *n_def = 0;
  if (N == 0) return CRDT_OK;
  if (int rc = check_frames(ctx, bytes, frame_off, N, status)) return rc;
  if (A == 0 || M == 0 || !actors || !members || !clock || !entries || !def_off)
    return fail(ctx, CRDT_EINVAL, "orswot_ingest: need actors, members, clock, entries, def_off");
  if (def_cap && (!def_clock || !def_members)) return fail(ctx, CRDT_EINVAL, "orswot_ingest: NULL deferred output");
  const size_t Mw = (M + 63) / 64;
  if (A + Mw > (size_t)kWireRowLds) return fail(ctx, CRDT_EUNSUPPORTED, "orswot_ingest: A + M/64 too large");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  // scratch: deferred positions + counts [2N], scan block sums
  const unsigned long long nb = (N + kScanItems - 1) / kScanItems + 2;
  if (int rc = ensure_scratch(ctx, (2 * N + nb + 8) * 8)) return rc;
  u64 *dpos = reinterpret_cast<u64 *>(ctx->scratch), *dcount = dpos + N, *sc = dcount + N;
  int wpb = 4;
  while (wpb > 1 && (size_t)wpb * (A + Mw) * 8 > 64 * 1024) --wpb;
  IngestPlan p{};
  p.bytes = bytes;
  p.frame_off = (const u64 *)frame_off;
  p.N = N;
  p.actors = actors;
  p.A = A;
  p.out = (u64 *)clock;
  p.row_stride = A;
  p.status = status;
  p.members = (const u64 *)members;
  p.M = M;
  p.Mw = Mw;
  p.entries = (u64 *)entries;
  p.dpos = dpos;
  p.dcount = dcount;
  p.def_off = (u64 *)def_off;
  p.def_clock = (u64 *)def_clock;
  p.def_members = (u64 *)def_members;
  p.def_cap = def_cap;
  const size_t dw = (A + 1) / 2 + M;
  if ((dw + wpb * (A + Mw)) * 8 <= 64 * 1024) p.dict_words = dw;
  const unsigned grid = wave_grid(ctx, N, wpb, 32);
  timing_begin(ctx, "wire_ingest");
  // pass 1: walk + batched parse (wwalk=1, default), the dictionaries in LDS when they fit beside
  // sixteen 4-KiB frame rings; else the one-chain kernel
  const size_t ring_w = (size_t)kOrWalkRing * kWalkWin / 2;
  const size_t walk_lds = (dw + kOrWalkWaves * ring_w) * 8;
  const size_t fill_lds = (dw + (kOfWalk + 1) / 2 + kOfWalk * ring_w) * 8;
  if (ctx->tune.wire_walk && ctx->tune.wire_fill && fill_lds <= 80 * 1024 && N * M <= 0xffffffffffull &&
      N * M * A * 8 > 0) {
    // zero rows by filler waves beside the walk (no separate fill pass); two blocks per CU
    if (int rc = ensure_scratch(ctx, (2 * N + nb + 8) * 8 + N * M * 4)) return rc;
    dpos = reinterpret_cast<u64 *>(ctx->scratch), dcount = dpos + N, sc = dcount + N;
    p.dpos = dpos;
    p.dcount = dcount;
    IngestPlan q = p;
    q.dict_words = dw;
    uint32_t *epos = reinterpret_cast<uint32_t *>(sc + nb + 8);
    CRDT_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(&orswot_ingest_walk_fill_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)fill_lds));
    hipLaunchKernelGGL(orswot_ingest_walk_fill_kernel, dim3((unsigned)((N + kOfWalk - 1) / kOfWalk)),
                       dim3((kOfWalk + kOfFill) * kWave), fill_lds, ctx->stream, q, epos);
  } else if (ctx->tune.wire_walk && walk_lds <= 160 * 1024) {
    if (int rc = device_fill(ctx, entries, N * M * A * 8, 0)) return rc;
    IngestPlan q = p;
    q.dict_words = dw;
    CRDT_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void *>(&orswot_ingest_walk_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)walk_lds));
    hipLaunchKernelGGL(orswot_ingest_walk_kernel, dim3(wave_grid(ctx, N, kOrWalkWaves, 8)),
                       dim3(kOrWalkWaves * kWave), walk_lds, ctx->stream, q);
  } else {
    if (int rc = device_fill(ctx, entries, N * M * A * 8, 0)) return rc;
    hipLaunchKernelGGL(orswot_ingest_kernel, dim3(grid), dim3(wpb * kWave), (p.dict_words + wpb * A) * 8, ctx->stream, p);
  }
  CRDT_HIP(ctx, hipGetLastError());
  unsigned long long D = 0;
  if (int rc = exclusive_scan(ctx, dcount, (u64 *)def_off, N, sc, &D)) return rc;
  if (D)
    hipLaunchKernelGGL(orswot_ingest_deferred_kernel, dim3(grid), dim3(wpb * kWave),
                       (p.dict_words + wpb * (A + Mw)) * 8, ctx->stream, p);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  if (n_def) *n_def = D;
  return CRDT_OK;
}

// Map<u32, MVReg<u64>>: states packed (clock_stride A, ec_stride K*A, vclk_stride K*V*A,
// vval_stride K*V), deferred as per-state slots (crdt_map_deferred).
static int map_wire_plan(crdt_ctx *ctx, const crdt_map_states *st, const crdt_map_deferred *df, const uint32_t *actors,
                         const uint32_t *keys, MapWirePlan &p, const char *what) {
  if (!st || !df || !actors || !keys) return fail(ctx, CRDT_EINVAL, "%s: NULL states / deferred / dictionaries", what);
  const size_t N = st->N, K = st->K, A = st->A, V = st->V;
  if (A == 0 || K == 0 || V == 0) return fail(ctx, CRDT_EINVAL, "%s: need A, K, V >= 1", what);
  if (N && (!st->clock || !st->ec || !st->vclk || !st->vval || !df->count || (df->Dcap && (!df->clock || !df->keys))))
    return fail(ctx, CRDT_EINVAL, "%s: NULL state buffer", what);
  if ((N > 1 && st->clock_stride != A) || (N > 1 && st->ec_stride != K * A) || (N > 1 && st->vclk_stride != K * V * A) ||
      (N > 1 && st->vval_stride != K * V))
    return fail(ctx, CRDT_EUNSUPPORTED, "%s: states must be packed (strides A, K*A, K*V*A, K*V)", what);
  const size_t Kw = (K + 63) / 64;
  if (A + Kw > (size_t)kWireRowLds) return fail(ctx, CRDT_EUNSUPPORTED, "%s: A + K/64 too large", what);
  p = MapWirePlan{};
  p.N = N;
  p.A = A;
  p.K = K;
  p.Kw = Kw;
  p.V = V;
  p.Dcap = df->Dcap;
  p.actors = actors;
  p.keys = keys;
  p.clock = (u64 *)st->clock;
  p.ec = (u64 *)st->ec;
  p.vclk = (u64 *)st->vclk;
  p.vval = (u64 *)st->vval;
  p.def_clock = (u64 *)df->clock;
  p.def_keys = (u64 *)df->keys;
  p.def_count = df->count;
  return CRDT_OK;
}

int crdt_map_ingest(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *frame_off, const uint32_t *actors,
                    const uint32_t *keys, const crdt_map_states *out, const crdt_map_deferred *out_def,
                    uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  MapWirePlan p;
  if (int rc = map_wire_plan(ctx, out, out_def, actors, keys, p, "map_ingest")) return rc;
  const size_t N = p.N;
  if (N == 0) return CRDT_OK;
  if (int rc = check_frames(ctx, bytes, frame_off, N, status)) return rc;
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  // absent keys / values are zero rows
  if (int rc = device_fill(ctx, p.ec, N * p.K * p.A * 8, 0)) return rc;
  if (int rc = device_fill(ctx, p.vclk, N * p.K * p.V * p.A * 8, 0)) return rc;
  if (int rc = device_fill(ctx, p.vval, N * p.K * p.V * 8, 0)) return rc;
  p.bytes = bytes;
  p.frame_off = (const u64 *)frame_off;
  p.status = status;
  {  // walk + batched parse when a wave's frame ring and rows fit beside the dictionaries
    const size_t per_wave = kWalkRing * kWalkWin / 2 + p.A + p.Kw;
    const size_t dw = (p.A + 1) / 2 + (p.K + 1) / 2;
    int wpb = 4;
    while (wpb > 1 && (dw + wpb * per_wave) * 8 > 64 * 1024) --wpb;
    p.stage = (dw + wpb * per_wave) * 8 <= 64 * 1024;
    if (ctx->tune.wire_walk && ((p.stage ? dw : 0) + wpb * per_wave) * 8 <= 64 * 1024) {
      if (int rc = device_fill(ctx, p.clock, N * p.A * 8, 0)) return rc;  // the parse writes nonzeros only
      const size_t lds = ((p.stage ? dw : 0) + wpb * per_wave) * 8;
      timing_begin(ctx, "wire_ingest");
      hipLaunchKernelGGL(map_ingest_walk_kernel, dim3(wave_grid(ctx, N, wpb, 32)), dim3(wpb * kWave), lds,
                         ctx->stream, p);
      timing_end(ctx);
      CRDT_HIP(ctx, hipGetLastError());
      return CRDT_OK;
    }
  }
  int wpb = 4;
  while (wpb > 1 && (size_t)wpb * (p.A + p.Kw) * 8 > 64 * 1024) --wpb;
  const size_t dw = (p.A + 1) / 2 + (p.K + 1) / 2;
  p.stage = (dw + wpb * (p.A + p.Kw)) * 8 <= 64 * 1024;
  const size_t lds = ((p.stage ? dw : 0) + wpb * (p.A + p.Kw)) * 8;
  const unsigned grid = wave_grid(ctx, N, wpb, 32);
  timing_begin(ctx, "wire_ingest");
  hipLaunchKernelGGL(map_ingest_kernel, dim3(grid), dim3(wpb * kWave), lds, ctx->stream, p);
  timing_end(ctx);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

int crdt_map_egress(crdt_ctx *ctx, const crdt_map_states *states, const crdt_map_deferred *def, const uint32_t *actors,
                    const uint32_t *keys, uint64_t *frame_off, uint8_t *bytes, size_t cap, size_t *total) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (total) *total = 0;
  MapWirePlan p;
  if (int rc = map_wire_plan(ctx, states, def, actors, keys, p, "map_egress")) return rc;
  const size_t N = p.N;
  if (N == 0) return CRDT_OK;
  if (!frame_off || !total) return fail(ctx, CRDT_EINVAL, "map_egress: need frame_off and total");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  u64 *sizes = nullptr;
  if (int rc = wire_scratch(ctx, N, &sizes)) return rc;
  p.sizes = sizes;
  const unsigned grid = wave_grid(ctx, N, 4, 32);
  timing_begin(ctx, "wire_egress");
  hipLaunchKernelGGL(map_egress_kernel, dim3(grid), dim3(kBlock), 0, ctx->stream, p, 0);
  CRDT_HIP(ctx, hipGetLastError());
  if (int rc = egress_layout(ctx, sizes, (u64 *)frame_off, N, total)) return rc;
  if (bytes && cap >= *total) {
    p.frame_out = (const u64 *)frame_off;
    p.out = bytes;
    hipLaunchKernelGGL(map_egress_kernel, dim3(grid), dim3(kBlock), 0, ctx->stream, p, 1);
    CRDT_HIP(ctx, hipGetLastError());
  }
  timing_end(ctx);
  return CRDT_OK;
}

static int egress_common(crdt_ctx *ctx, EgressPlan p, size_t N, uint64_t *frame_off, uint8_t *bytes, size_t cap,
                         size_t *total, void (*kern)(EgressPlan, int), const char *what) {
  CRDT_CHECK_CTX(ctx);
  if (total) *total = 0;
  if (N == 0) return CRDT_OK;
  if (!frame_off || !total) return fail(ctx, CRDT_EINVAL, "%s: need frame_off and total", what);
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  u64 *sizes = nullptr;
  if (int rc = wire_scratch(ctx, N, &sizes)) return rc;
  p.sizes = sizes;
  const unsigned grid = wave_grid(ctx, N, 4, 32);
  timing_begin(ctx, "wire_egress");
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, ctx->stream, p, 0);
  CRDT_HIP(ctx, hipGetLastError());
  if (int rc = egress_layout(ctx, sizes, (u64 *)frame_off, N, total)) return rc;
  if (bytes && cap >= *total) {
    p.frame_off = (const u64 *)frame_off;
    p.bytes = bytes;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, ctx->stream, p, 1);
    CRDT_HIP(ctx, hipGetLastError());
  }
  timing_end(ctx);
  return CRDT_OK;
}

int crdt_vclock_egress(crdt_ctx *ctx, const uint64_t *rows, size_t N, size_t A, size_t row_stride,
                       const uint32_t *actors, uint64_t *frame_off, uint8_t *bytes, size_t cap, size_t *total) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  if (ctx && N && (!rows || !actors || A == 0)) return fail(ctx, CRDT_EINVAL, "vclock_egress: NULL rows / actors");
  EgressPlan p{};
  p.rows = (const u64 *)rows;
  p.N = N;
  p.A = A;
  p.row_stride = row_stride;
  p.nclocks = 1;
  p.actors = actors;
  return egress_common(ctx, p, N, frame_off, bytes, cap, total, vclock_egress_kernel, "vclock_egress");
}

int crdt_pncounter_egress(crdt_ctx *ctx, const uint64_t *rows, size_t N, size_t A, size_t row_stride,
                          const uint32_t *actors, uint64_t *frame_off, uint8_t *bytes, size_t cap, size_t *total) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  if (ctx && N && (!rows || !actors || A == 0)) return fail(ctx, CRDT_EINVAL, "pncounter_egress: NULL rows / actors");
  EgressPlan p{};
  p.rows = (const u64 *)rows;
  p.N = N;
  p.A = A;
  p.row_stride = row_stride;
  p.nclocks = 2;
  p.actors = actors;
  return egress_common(ctx, p, N, frame_off, bytes, cap, total, vclock_egress_kernel, "pncounter_egress");
}

int crdt_gset_egress(crdt_ctx *ctx, const uint64_t *rows, size_t N, size_t U, size_t row_stride, const uint64_t *elems,
                     uint64_t *frame_off, uint8_t *bytes, size_t cap, size_t *total) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  if (ctx && N && (!rows || !elems || U == 0)) return fail(ctx, CRDT_EINVAL, "gset_egress: NULL rows / elems");
  EgressPlan p{};
  p.rows = (const u64 *)rows;
  p.N = N;
  p.U = U;
  p.row_stride = row_stride;
  p.elems = (const u64 *)elems;
  return egress_common(ctx, p, N, frame_off, bytes, cap, total, gset_egress_kernel, "gset_egress");
}

int crdt_lwwreg_egress(crdt_ctx *ctx, const uint64_t *marker, const uint64_t *val, size_t N, uint8_t *bytes) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (N == 0) return CRDT_OK;
  if (!marker || !val || !bytes) return fail(ctx, CRDT_EINVAL, "lwwreg_egress: NULL buffer");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  hipLaunchKernelGGL(lwwreg_egress_kernel, dim3(wave_grid(ctx, N, 4, 16)), dim3(kBlock), 0, ctx->stream,
                     (const u64 *)marker, (const u64 *)val, (unsigned long long)N, bytes);
  CRDT_HIP(ctx, hipGetLastError());
  return CRDT_OK;
}

int crdt_orswot_egress(crdt_ctx *ctx, const uint64_t *clock, const uint64_t *entries, size_t N, size_t M, size_t A,
                       const uint32_t *actors, const uint64_t *members, const uint64_t *def_off,
                       const uint64_t *def_clock, const uint64_t *def_members, const uint8_t *def_keep,
                       uint64_t *frame_off, uint8_t *bytes, size_t cap, size_t *total) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  if (ctx && N && (!clock || !entries || !actors || !members || A == 0 || M == 0))
    return fail(ctx, CRDT_EINVAL, "orswot_egress: NULL state / dictionaries");
  if (ctx && def_off && (!def_clock || !def_members)) return fail(ctx, CRDT_EINVAL, "orswot_egress: NULL deferred");
  EgressPlan p{};
  p.rows = (const u64 *)clock;
  p.N = N;
  p.A = A;
  p.row_stride = A;
  p.actors = actors;
  p.entries = (const u64 *)entries;
  p.M = M;
  p.Mw = (M + 63) / 64;
  p.members = (const u64 *)members;
  p.def_off = (const u64 *)def_off;
  p.def_clock = (const u64 *)def_clock;
  p.def_members = (const u64 *)def_members;
  p.def_keep = def_keep;
  return egress_common(ctx, p, N, frame_off, bytes, cap, total, orswot_egress_kernel, "orswot_egress");
}

}  // extern "C"
