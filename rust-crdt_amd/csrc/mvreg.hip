// Batched MVReg<u64, A> (the multi-value register, src/mvreg.rs) on its own, outside a Map:
//   crdt_mvreg_lub_many    G left folds  acc = MVReg::new(); for r: acc.merge(replica[g][r])
//   crdt_mvreg_merge_batch N pairwise    self[i].merge(other[i])                 (mvreg.rs:112-128)
//   crdt_mvreg_apply_batch N op streams  for op in ops[i]: reg[i].apply(op)      (mvreg.rs:130-166)
// Exact for ANY input in the dense layout (no associativity assumed: each register is folded in
// order), so the reference's own MVReg tests (test/mvreg.rs:11-105) replay on it bit for bit.
//
// Dense register: value slots in Vec order, slot s = (clock row vclk[s*A ..], value vval[s]); an
// empty slot is an all-zero clock row (a stored value never has an empty clock: apply returns on
// one, mvreg.rs:138-140, merge keeps what it gets, forget drops what it empties).
//
// One wave per register, lane = actor (APL clock words per lane, A <= 64 * APL).  The working
// register lives in registers as VS slots with insertion sequence numbers: `merge` keeps own
// values not strictly below another's (mvreg.rs:113-117), then appends other's values not below
// or equal to a kept one (:119-126: lt || eq == le); `apply` drops values <= the Put clock and
// appends unless a remaining value dominates it (:143-163).  Removal only clears a slot bit, an
// append takes a free slot with the next sequence number, and the Vec order is the sequence order
// (own kept values keep their relative order, appended ones follow in theirs), ranked once when
// the register is written.  Every vote is a wave ballot, so all control flow is wave-uniform.
//
// Past one wave's shapes (A > 256 actors or more than 8 value slots, round 4: the reference's
// MVReg is unbounded, mvreg.rs:33-35) the same code runs with BLK = true: a workgroup of
// ceil(A / 64) waves per register, thread t = actor t (one clock word per thread), every vote a
// workgroup vote (__syncthreads_or), value slots up to 16 in and 16 in the working register.
#include "common.hpp"

namespace crdt {

constexpr int kMvMaxState = 16;  // values a working register holds (flags bit 2 past it)

// "some thread holds x": a wave ballot, or with BLK a workgroup vote
template <bool BLK>
__device__ __forceinline__ bool mv_any(bool x) {
  if constexpr (BLK) return __syncthreads_or(x) != 0;
  else return __ballot(x) != 0;
}
template <int APL, bool BLK = false>
__device__ __forceinline__ bool mv_le(const u64 (&x)[APL], const u64 (&y)[APL]) {
  bool gt = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) gt |= x[j] > y[j];
  return !mv_any<BLK>(gt);
}
template <int APL, bool BLK = false>
__device__ __forceinline__ bool mv_eq(const u64 (&x)[APL], const u64 (&y)[APL]) {
  bool ne = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) ne |= x[j] != y[j];
  return !mv_any<BLK>(ne);
}
// x < y as VClock's PartialOrd: x <= y everywhere and x != y (vclock.rs:68-80)
template <int APL, bool BLK = false>
__device__ __forceinline__ bool mv_lt(const u64 (&x)[APL], const u64 (&y)[APL]) {
  bool gt = false, ne = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    gt |= x[j] > y[j];
    ne |= x[j] != y[j];
  }
  return !mv_any<BLK>(gt) && mv_any<BLK>(ne);
}
template <int APL, bool BLK = false>
__device__ __forceinline__ bool mv_zero(const u64 (&x)[APL]) {
  bool nz = false;
#pragma unroll
  for (int j = 0; j < APL; ++j) nz |= x[j] != 0;
  return !mv_any<BLK>(nz);
}

// lane = the thread's index in its wave (BLK: in its workgroup); nt = 64 (BLK: the workgroup size)
template <int APL>
__device__ __forceinline__ void mv_load_row(u64 (&x)[APL], const u64 *row, unsigned long long A, int lane,
                                            unsigned nt = 64) {
#pragma unroll
  for (int j = 0; j < APL; ++j) {
    const unsigned long long a = lane + (unsigned long long)nt * j;
    x[j] = a < A ? row[a] : 0;
  }
}

// The working register: VS slots, `used` bit mask and insertion sequence numbers (wave-uniform).
template <int APL, int VS, bool BLK = false>
struct MvReg {
  u64 c[VS][APL];
  u64 v[VS];
  unsigned seq[VS];
  unsigned used;
  unsigned next;
  bool ovf;

  __device__ void clear() {
    used = 0;
    next = 0;
    ovf = false;
#pragma unroll
    for (int s = 0; s < VS; ++s) {
      seq[s] = 0;
      v[s] = 0;
#pragma unroll
      for (int j = 0; j < APL; ++j) c[s][j] = 0;
    }
  }

  __device__ int count() const { return __builtin_popcount(used); }

  // push (clock, val) at the end of the Vec: the first free slot, the next sequence number
  __device__ void push(const u64 (&x)[APL], u64 val) {
    bool placed = false;
#pragma unroll
    for (int s = 0; s < VS; ++s)
      if (!placed && !((used >> s) & 1u)) {
        placed = true;
#pragma unroll
        for (int j = 0; j < APL; ++j) c[s][j] = x[j];
        v[s] = val;
        seq[s] = next;
        used |= 1u << s;
      }
    if (placed) ++next;
    else ovf = true;
  }

  // Load V slots of a register (Vec order = slot order, empty slots skipped).
  __device__ void load(const u64 *vclk, const u64 *vval, unsigned long long V, unsigned long long A, int lane,
                       unsigned nt = 64) {
    clear();
    for (unsigned long long s = 0; s < V; ++s) {
      u64 x[APL];
      mv_load_row<APL>(x, vclk + s * A, A, lane, nt);
      if (!mv_zero<APL, BLK>(x)) push(x, vval[s]);
    }
  }

  // self.merge(other) for other's VI slots (mvreg.rs:112-128)
  template <int VI>
  __device__ void merge(const u64 (&oc)[VI][APL], const u64 (&ov)[VI], unsigned opres) {
    // own values not strictly below any of other's
#pragma unroll
    for (int i = 0; i < VS; ++i)
      if ((used >> i) & 1u) {
        bool dom = false;
#pragma unroll
        for (int k = 0; k < VI; ++k)
          if (!dom && ((opres >> k) & 1u)) dom = mv_lt<APL, BLK>(c[i], oc[k]);
        if (dom) used &= ~(1u << i);
      }
    // other's values not below or equal to a KEPT own value (collected before any is appended)
    const unsigned kept = used;
    unsigned add = 0;
#pragma unroll
    for (int k = 0; k < VI; ++k)
      if ((opres >> k) & 1u) {
        bool drop = false;
#pragma unroll
        for (int i = 0; i < VS; ++i)
          if (!drop && ((kept >> i) & 1u)) drop = mv_le<APL, BLK>(oc[k], c[i]);
        if (!drop) add |= 1u << k;
      }
#pragma unroll
    for (int k = 0; k < VI; ++k)
      if ((add >> k) & 1u) push(oc[k], ov[k]);
  }

  // self.apply(Op::Put { clock: x, val }) (mvreg.rs:133-163)
  __device__ void apply(const u64 (&x)[APL], u64 val) {
    if (mv_zero<APL, BLK>(x)) return;  // an empty clock is a no-op
    // retain values whose clock is concurrent with or above the Put clock
#pragma unroll
    for (int i = 0; i < VS; ++i)
      if ((used >> i) & 1u)
        if (mv_le<APL, BLK>(c[i], x)) used &= ~(1u << i);
    bool add = true;
#pragma unroll
    for (int i = 0; i < VS; ++i)
      if (add && ((used >> i) & 1u)) add = !mv_lt<APL, BLK>(x, c[i]);
    if (add) push(x, val);
  }

  // Write the register to `Vout` slots in Vec order (empty slots zeroed); returns the count.
  __device__ int store(u64 *vclk, u64 *vval, unsigned long long Vout, unsigned long long A, int lane,
                       unsigned nt = 64) const {
    const int n = count();
#pragma unroll
    for (int i = 0; i < VS; ++i)
      if ((used >> i) & 1u) {
        int rank = 0;
#pragma unroll
        for (int k = 0; k < VS; ++k) rank += (((used >> k) & 1u) && seq[k] < seq[i]) ? 1 : 0;
        if ((unsigned long long)rank < Vout) {
          u64 *row = vclk + (unsigned long long)rank * A;
#pragma unroll
          for (int j = 0; j < APL; ++j) {
            const unsigned long long a = lane + (unsigned long long)nt * j;
            if (a < A) row[a] = c[i][j];
          }
          if (lane == 0) vval[rank] = v[i];
        }
      }
    for (unsigned long long s = (unsigned long long)n; s < Vout; ++s) {
      for (unsigned long long a = lane; a < A; a += nt) vclk[s * A + a] = 0;
      if (lane == 0) vval[s] = 0;
    }
    return n;
  }
};

struct MvFoldPlan {
  const u64 *vclk, *vval;
  unsigned long long G, R, A, V;
  unsigned long long c_rs, c_gs, v_rs, v_gs;
  u64 *o_vclk, *o_vval;
  unsigned long long Vout;
  uint32_t *o_nval, *o_flags;
};

// One group's left fold (one wave per group); the next replica's slots are loaded while this
// one merges.
template <int APL, int VS, int VI, bool BLK = false>
__global__ __launch_bounds__(BLK ? 1024 : 64) void mvreg_fold_kernel(MvFoldPlan p) {
  const int lane = threadIdx.x;
  const unsigned nt = blockDim.x;
  const unsigned long long g = blockIdx.x;
  MvReg<APL, VS, BLK> acc;
  acc.clear();
  u64 nc[VI][APL], nv[VI];
  auto fetch = [&](unsigned long long r) {
    const u64 *cb = p.vclk + g * p.c_gs + r * p.c_rs;
    const u64 *vb = p.vval + g * p.v_gs + r * p.v_rs;
#pragma unroll
    for (int k = 0; k < VI; ++k) {
      if ((unsigned long long)k < p.V) {
        mv_load_row<APL>(nc[k], cb + k * p.A, p.A, lane, nt);
        nv[k] = vb[k];
      } else {
#pragma unroll
        for (int j = 0; j < APL; ++j) nc[k][j] = 0;
        nv[k] = 0;
      }
    }
  };
  if (p.R > 0) fetch(0);
  for (unsigned long long r = 0; r < p.R; ++r) {
    u64 oc[VI][APL], ov[VI];
#pragma unroll
    for (int k = 0; k < VI; ++k) {
      ov[k] = nv[k];
#pragma unroll
      for (int j = 0; j < APL; ++j) oc[k][j] = nc[k][j];
    }
    if (r + 1 < p.R) fetch(r + 1);
    unsigned opres = 0;
#pragma unroll
    for (int k = 0; k < VI; ++k)
      if (!mv_zero<APL, BLK>(oc[k])) opres |= 1u << k;
    acc.template merge<VI>(oc, ov, opres);
  }
  const int n = acc.store(p.o_vclk + g * p.Vout * p.A, p.o_vval + g * p.Vout, p.Vout, p.A, lane, nt);
  if (lane == 0) {
    if (p.o_nval) p.o_nval[g] = (uint32_t)n;
    p.o_flags[g] = ((unsigned long long)n > p.Vout ? 1u : 0u) | (acc.ovf ? 4u : 0u);
  }
}

struct MvPairPlan {
  u64 *s_vclk, *s_vval;
  unsigned long long s_cs, s_vs, Vs;
  const u64 *o_vclk, *o_vval;
  unsigned long long o_cs, o_vs, Vo;
  unsigned long long N, A;
  uint32_t *status;
};

template <int APL, int VS, int VI, bool BLK = false>
__global__ __launch_bounds__(BLK ? 1024 : 64) void mvreg_pair_kernel(MvPairPlan p) {
  const int lane = threadIdx.x;
  const unsigned nt = blockDim.x;
  const unsigned long long i = blockIdx.x;
  MvReg<APL, VS, BLK> acc;
  acc.load(p.s_vclk + i * p.s_cs, p.s_vval + i * p.s_vs, p.Vs, p.A, lane, nt);
  u64 oc[VI][APL], ov[VI];
  unsigned opres = 0;
#pragma unroll
  for (int k = 0; k < VI; ++k) {
    if ((unsigned long long)k < p.Vo) {
      mv_load_row<APL>(oc[k], p.o_vclk + i * p.o_cs + k * p.A, p.A, lane, nt);
      ov[k] = p.o_vval[i * p.o_vs + k];
    } else {
#pragma unroll
      for (int j = 0; j < APL; ++j) oc[k][j] = 0;
      ov[k] = 0;
    }
    if (!mv_zero<APL, BLK>(oc[k])) opres |= 1u << k;
  }
  acc.template merge<VI>(oc, ov, opres);
  const int n = acc.store(p.s_vclk + i * p.s_cs, p.s_vval + i * p.s_vs, p.Vs, p.A, lane, nt);
  if (lane == 0) p.status[i] = ((unsigned long long)n > p.Vs || acc.ovf) ? 16u : 0u;
}

struct MvApplyPlan {
  u64 *vclk, *vval;
  unsigned long long cs, vs, V, N, A;
  const u64 *op_off;
  const uint32_t *clk_row;
  const u64 *clk_pool, *val;
  unsigned long long n_ops, n_clk_rows;
  uint32_t *status;
};

template <int APL, int VS, bool BLK = false>
__global__ __launch_bounds__(BLK ? 1024 : 64) void mvreg_apply_kernel(MvApplyPlan p) {
  const int lane = threadIdx.x;
  const unsigned nt = blockDim.x;
  const unsigned long long i = blockIdx.x;
  const unsigned long long o0 = p.op_off[i], o1 = p.op_off[i + 1];
  if (o1 < o0 || o1 > p.n_ops) {  // invalid range: register untouched
    if (lane == 0) p.status[i] = 8u;
    return;
  }
  MvReg<APL, VS, BLK> acc;
  acc.load(p.vclk + i * p.cs, p.vval + i * p.vs, p.V, p.A, lane, nt);
  unsigned st = 0;
  for (unsigned long long o = o0; o < o1; ++o) {
    const unsigned long long row = p.clk_row[o];
    if (row >= p.n_clk_rows) {
      st |= 2u;  // malformed op: skipped
      continue;
    }
    u64 x[APL];
    mv_load_row<APL>(x, p.clk_pool + row * p.A, p.A, lane, nt);
    acc.apply(x, p.val[o]);
  }
  const int n = acc.store(p.vclk + i * p.cs, p.vval + i * p.vs, p.V, p.A, lane, nt);
  if ((unsigned long long)n > p.V || acc.ovf) st |= 16u;
  if (lane == 0) p.status[i] = st;
}

static int mv_apl(size_t A) { return A <= 64 ? 1 : (A <= 128 ? 2 : 4); }
static int mv_vi(size_t V) { return V <= 1 ? 1 : (V <= 2 ? 2 : (V <= 4 ? 4 : 8)); }
static int mv_vs(size_t want) { return want <= 4 ? 4 : (want <= 8 ? 8 : 16); }

template <int APL, int VS>
static hipError_t launch_fold_vi(const MvFoldPlan &p, int VI, hipStream_t s) {
  const dim3 grid((unsigned)p.G);
  switch (VI) {
    case 1: hipLaunchKernelGGL((mvreg_fold_kernel<APL, VS, 1>), grid, dim3(64), 0, s, p); break;
    case 2: hipLaunchKernelGGL((mvreg_fold_kernel<APL, VS, 2>), grid, dim3(64), 0, s, p); break;
    case 4: hipLaunchKernelGGL((mvreg_fold_kernel<APL, VS, 4>), grid, dim3(64), 0, s, p); break;
    default: hipLaunchKernelGGL((mvreg_fold_kernel<APL, VS, 8>), grid, dim3(64), 0, s, p); break;
  }
  return hipGetLastError();
}
template <int APL>
static hipError_t launch_fold(const MvFoldPlan &p, int VS, int VI, hipStream_t s) {
  if (VS == 4) return launch_fold_vi<APL, 4>(p, VI, s);
  if (VS == 8) return launch_fold_vi<APL, 8>(p, VI, s);
  return launch_fold_vi<APL, 16>(p, VI, s);
}

template <int APL, int VS>
static hipError_t launch_pair_vi(const MvPairPlan &p, int VI, hipStream_t s) {
  const dim3 grid((unsigned)p.N);
  switch (VI) {
    case 1: hipLaunchKernelGGL((mvreg_pair_kernel<APL, VS, 1>), grid, dim3(64), 0, s, p); break;
    case 2: hipLaunchKernelGGL((mvreg_pair_kernel<APL, VS, 2>), grid, dim3(64), 0, s, p); break;
    case 4: hipLaunchKernelGGL((mvreg_pair_kernel<APL, VS, 4>), grid, dim3(64), 0, s, p); break;
    default: hipLaunchKernelGGL((mvreg_pair_kernel<APL, VS, 8>), grid, dim3(64), 0, s, p); break;
  }
  return hipGetLastError();
}
template <int APL>
static hipError_t launch_pair(const MvPairPlan &p, int VS, int VI, hipStream_t s) {
  if (VS == 4) return launch_pair_vi<APL, 4>(p, VI, s);
  if (VS == 8) return launch_pair_vi<APL, 8>(p, VI, s);
  return launch_pair_vi<APL, 16>(p, VI, s);
}

// Wide shapes (A > 256 or V > 8): one workgroup of ceil(A / 64) waves per register, one actor per
// thread, VI / VS up to 16.
static unsigned mv_wide_nt(size_t A) { return (unsigned)std::max<size_t>(64, (A + 63) / 64 * 64); }
static bool mv_wide(size_t A, size_t V) { return A > 256 || V > 8; }
static int mv_vi_wide(size_t V) { return V <= 8 ? mv_vi(V) : 16; }

template <int VS, int VI>
static void launch_fold_w(const MvFoldPlan &p, hipStream_t s) {
  hipLaunchKernelGGL((mvreg_fold_kernel<1, VS, VI, true>), dim3((unsigned)p.G), dim3(mv_wide_nt(p.A)), 0, s, p);
}
template <int VS>
static void launch_fold_wvi(const MvFoldPlan &p, int VI, hipStream_t s) {
  switch (VI) {
    case 1: launch_fold_w<VS, 1>(p, s); break;
    case 2: launch_fold_w<VS, 2>(p, s); break;
    case 4: launch_fold_w<VS, 4>(p, s); break;
    case 8: launch_fold_w<VS, 8>(p, s); break;
    default: launch_fold_w<VS, 16>(p, s); break;
  }
}
static hipError_t launch_fold_wide(const MvFoldPlan &p, int VS, int VI, hipStream_t s) {
  if (VS == 4) launch_fold_wvi<4>(p, VI, s);
  else if (VS == 8) launch_fold_wvi<8>(p, VI, s);
  else launch_fold_wvi<16>(p, VI, s);
  return hipGetLastError();
}
template <int VS, int VI>
static void launch_pair_w(const MvPairPlan &p, hipStream_t s) {
  hipLaunchKernelGGL((mvreg_pair_kernel<1, VS, VI, true>), dim3((unsigned)p.N), dim3(mv_wide_nt(p.A)), 0, s, p);
}
template <int VS>
static void launch_pair_wvi(const MvPairPlan &p, int VI, hipStream_t s) {
  switch (VI) {
    case 1: launch_pair_w<VS, 1>(p, s); break;
    case 2: launch_pair_w<VS, 2>(p, s); break;
    case 4: launch_pair_w<VS, 4>(p, s); break;
    case 8: launch_pair_w<VS, 8>(p, s); break;
    default: launch_pair_w<VS, 16>(p, s); break;
  }
}
static hipError_t launch_pair_wide(const MvPairPlan &p, int VS, int VI, hipStream_t s) {
  if (VS == 4) launch_pair_wvi<4>(p, VI, s);
  else if (VS == 8) launch_pair_wvi<8>(p, VI, s);
  else launch_pair_wvi<16>(p, VI, s);
  return hipGetLastError();
}
static hipError_t launch_apply_wide(const MvApplyPlan &p, int VS, hipStream_t s) {
  const dim3 grid((unsigned)p.N), blk(mv_wide_nt(p.A));
  if (VS == 4) hipLaunchKernelGGL((mvreg_apply_kernel<1, 4, true>), grid, blk, 0, s, p);
  else if (VS == 8) hipLaunchKernelGGL((mvreg_apply_kernel<1, 8, true>), grid, blk, 0, s, p);
  else hipLaunchKernelGGL((mvreg_apply_kernel<1, 16, true>), grid, blk, 0, s, p);
  return hipGetLastError();
}

template <int APL>
static hipError_t launch_apply(const MvApplyPlan &p, int VS, hipStream_t s) {
  const dim3 grid((unsigned)p.N);
  if (VS == 4) hipLaunchKernelGGL((mvreg_apply_kernel<APL, 4>), grid, dim3(64), 0, s, p);
  else if (VS == 8) hipLaunchKernelGGL((mvreg_apply_kernel<APL, 8>), grid, dim3(64), 0, s, p);
  else hipLaunchKernelGGL((mvreg_apply_kernel<APL, 16>), grid, dim3(64), 0, s, p);
  return hipGetLastError();
}

}  // namespace crdt

using namespace crdt;

extern "C" {

int crdt_mvreg_lub_many(crdt_ctx *ctx, const crdt_mvreg_batch *in, crdt_mvreg_out *out) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!in || !out) return fail(ctx, CRDT_EINVAL, "mvreg_lub_many: NULL batch/out");
  const size_t G = in->G, R = in->R, A = in->A, V = in->V, Vout = out->Vout;
  if (G == 0 || A == 0) return CRDT_OK;
  if (!out->vclk || !out->vval || !out->flags) return fail(ctx, CRDT_EINVAL, "mvreg_lub_many: NULL output");
  if (Vout == 0 || Vout > (size_t)kMvMaxState)
    return fail(ctx, CRDT_EUNSUPPORTED, "mvreg_lub_many: Vout = %zu not in [1, %d]", Vout, kMvMaxState);
  if (R > 0 && V > 0 && (!in->vclk || !in->vval)) return fail(ctx, CRDT_EINVAL, "mvreg_lub_many: NULL input");
  if (A > 1024) return fail(ctx, CRDT_EUNSUPPORTED, "mvreg_lub_many: A = %zu > 1024 actors", A);
  if (V > 16) return fail(ctx, CRDT_EUNSUPPORTED, "mvreg_lub_many: V = %zu > 16 value slots", V);
  if (G > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "mvreg_lub_many: G too large");
  if (R > 0 && V > 0 && (in->vclk_rstride < V * A || in->vval_rstride < V))
    return fail(ctx, CRDT_EINVAL, "mvreg_lub_many: replica strides below the register size");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  MvFoldPlan p{};
  p.vclk = (const u64 *)in->vclk;
  p.vval = (const u64 *)in->vval;
  p.G = G;
  p.R = V > 0 ? R : 0;  // replicas without value slots are empty registers: merging them is a no-op
  p.A = A;
  p.V = V;
  p.c_rs = in->vclk_rstride;
  p.c_gs = in->vclk_gstride;
  p.v_rs = in->vval_rstride;
  p.v_gs = in->vval_gstride;
  p.o_vclk = (u64 *)out->vclk;
  p.o_vval = (u64 *)out->vval;
  p.Vout = Vout;
  p.o_nval = out->nval;
  p.o_flags = out->flags;
  const int VS = mv_vs(std::max<size_t>({Vout, out->Vstate, 2 * std::max<size_t>(V, 1)}));
  const bool wide = mv_wide(A, V);
  const int VI = wide ? mv_vi_wide(V) : mv_vi(V);
  timing_begin(ctx, "mvreg_fold");
  const int apl = mv_apl(A);
  hipError_t e = wide ? launch_fold_wide(p, VS, VI, ctx->stream)
                 : apl == 1 ? launch_fold<1>(p, VS, VI, ctx->stream)
                          : (apl == 2 ? launch_fold<2>(p, VS, VI, ctx->stream) : launch_fold<4>(p, VS, VI, ctx->stream));
  timing_end(ctx);
  if (e != hipSuccess) return hip_fail(ctx, e, "mvreg_fold_kernel launch");
  return CRDT_OK;
}

int crdt_mvreg_merge_batch(crdt_ctx *ctx, const crdt_mvreg_states *self, const crdt_mvreg_states *other,
                           uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!self || !other || !status) return fail(ctx, CRDT_EINVAL, "mvreg_merge_batch: NULL argument");
  const size_t N = self->N, A = self->A;
  if (other->N != N || other->A != A) return fail(ctx, CRDT_EINVAL, "mvreg_merge_batch: self and other differ in N or A");
  if (N == 0 || A == 0) return CRDT_OK;
  if (self->V == 0 || self->V > 16 || other->V > 16)
    return fail(ctx, CRDT_EUNSUPPORTED, "mvreg_merge_batch: V must be in [1, 16] (self %zu, other %zu)", self->V,
                other->V);
  if (A > 1024) return fail(ctx, CRDT_EUNSUPPORTED, "mvreg_merge_batch: A = %zu > 1024 actors", A);
  if (!self->vclk || !self->vval || (other->V && (!other->vclk || !other->vval)))
    return fail(ctx, CRDT_EINVAL, "mvreg_merge_batch: NULL register buffers");
  if (N > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "mvreg_merge_batch: N too large");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  MvPairPlan p{};
  p.s_vclk = (u64 *)self->vclk;
  p.s_vval = (u64 *)self->vval;
  p.s_cs = self->vclk_stride;
  p.s_vs = self->vval_stride;
  p.Vs = self->V;
  p.o_vclk = (const u64 *)other->vclk;
  p.o_vval = (const u64 *)other->vval;
  p.o_cs = other->vclk_stride;
  p.o_vs = other->vval_stride;
  p.Vo = other->V;
  p.N = N;
  p.A = A;
  p.status = status;
  const int VS = mv_vs(self->V + std::max<size_t>(other->V, 1));
  const bool wide = mv_wide(A, std::max(self->V, other->V));
  const int VI = wide ? mv_vi_wide(other->V) : mv_vi(other->V);
  timing_begin(ctx, "mvreg_pair");
  const int apl = mv_apl(A);
  hipError_t e = wide ? launch_pair_wide(p, VS, VI, ctx->stream)
                 : apl == 1 ? launch_pair<1>(p, VS, VI, ctx->stream)
                          : (apl == 2 ? launch_pair<2>(p, VS, VI, ctx->stream) : launch_pair<4>(p, VS, VI, ctx->stream));
  timing_end(ctx);
  if (e != hipSuccess) return hip_fail(ctx, e, "mvreg_pair_kernel launch");
  return CRDT_OK;
}

int crdt_mvreg_apply_batch(crdt_ctx *ctx, const crdt_mvreg_states *states, const crdt_mvreg_ops *ops,
                           uint32_t *status) {
  CRDT_DEVICE_MEM_ONLY(ctx);
  CRDT_CHECK_CTX(ctx);
  if (!states || !ops || !status) return fail(ctx, CRDT_EINVAL, "mvreg_apply_batch: NULL argument");
  const size_t N = states->N, A = states->A, V = states->V;
  if (N == 0 || A == 0) return CRDT_OK;
  if (V == 0 || V > 16) return fail(ctx, CRDT_EUNSUPPORTED, "mvreg_apply_batch: V = %zu not in [1, 16]", V);
  if (A > 1024) return fail(ctx, CRDT_EUNSUPPORTED, "mvreg_apply_batch: A = %zu > 1024 actors", A);
  if (!states->vclk || !states->vval || !ops->op_off)
    return fail(ctx, CRDT_EINVAL, "mvreg_apply_batch: NULL register / op_off buffers");
  if (ops->n_ops && (!ops->clk_row || !ops->clk_pool || !ops->val))
    return fail(ctx, CRDT_EINVAL, "mvreg_apply_batch: NULL op buffers");
  if (N > 0x7fffffffULL) return fail(ctx, CRDT_EUNSUPPORTED, "mvreg_apply_batch: N too large");
  CRDT_HIP(ctx, hipSetDevice(ctx->device));
  MvApplyPlan p{};
  p.vclk = (u64 *)states->vclk;
  p.vval = (u64 *)states->vval;
  p.cs = states->vclk_stride;
  p.vs = states->vval_stride;
  p.V = V;
  p.N = N;
  p.A = A;
  p.op_off = (const u64 *)ops->op_off;
  p.clk_row = ops->clk_row;
  p.clk_pool = (const u64 *)ops->clk_pool;
  p.val = (const u64 *)ops->val;
  p.n_ops = ops->n_ops;
  p.n_clk_rows = ops->n_clk_rows;
  p.status = status;
  const int VS = mv_vs(V + 1);
  timing_begin(ctx, "mvreg_apply");
  const int apl = mv_apl(A);
  hipError_t e = mv_wide(A, V) ? launch_apply_wide(p, VS, ctx->stream)
                 : apl == 1 ? launch_apply<1>(p, VS, ctx->stream)
                          : (apl == 2 ? launch_apply<2>(p, VS, ctx->stream) : launch_apply<4>(p, VS, ctx->stream));
  timing_end(ctx);
  if (e != hipSuccess) return hip_fail(ctx, e, "mvreg_apply_kernel launch");
  return CRDT_OK;
}

}  // extern "C"
