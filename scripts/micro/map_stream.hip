// Microbenchmark: the HBM ceiling of the config-4 Map fold's ACCESS PATTERN, without its test.
// Layout and sizes as BASELINE config 4 (R = 16,384 replicas, K = 1,024 keys, A = 32 actors, V = 2):
// entry clocks EC[R][K][A], value clocks VC[R][K][2][A], replica clocks CL[R][A], chunk clock maxima
// CM[R/16][A], all u64.  Each key's fold streams, per replica step, a 1-KiB image (its entry-clock row,
// two value-clock rows, the replica-clock row) through LDS-DMA in 16-step chunks with two chunks in
// flight, exactly as map_fold_kernel's RS path; per chunk the slot is copied into registers and the
// wave then burns `work` dependent VALU iterations (a stand-in for the chunk test).
//   SPLIT = 1: one wave per key (1,024 waves, the RS path's grid);
//   SPLIT = 2: two waves per key, wave h moving actors 16h .. 16h+15 (512 B per step, two steps per
//              1-KiB instruction), optionally handing a per-chunk vote to its partner through LDS
//              (`sync`), i.e. the split-actor design the round-5 verdict proposed.
// Prints kernel time and the config-4 algorithmic rate (13,159,852,256 B per fold) as % of 8 TB/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

constexpr int R = 16384, K = 1024, A = 32, C = 16;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void glds16(const void *g, u64 *lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
}

template <int SPLIT>
__global__ __launch_bounds__(64 * SPLIT) void mstream(const char *ec, const char *vc, const char *cl, const char *cm,
                                                       int work, int sync, u64 *out, u64 *cyc) {
  extern __shared__ u64 lds[];
  constexpr int PIECES = 16 / SPLIT;           // step-image instructions per chunk
  constexpr unsigned SLOT = 16 * 128 / SPLIT;  // u64 words per chunk slot (per wave)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u64 k = blockIdx.x;
  u64 *my = lds + w * (2 * SLOT + 64);
  u64 *cms = my + 2 * SLOT;  // 2 x 32 words: staged clock max (this wave's actors)
  volatile unsigned *flag = reinterpret_cast<volatile unsigned *>(lds + SPLIT * (2 * SLOT + 64));
  // per-lane source of its 16 bytes of a piece and the replica stride
  const char *src0;
  u64 stride;
  if (SPLIT == 1) {
    const int o = 2 * lane;  // word of the step image
    if (o < A) { src0 = ec + (k * A + o) * 8; stride = (u64)K * A * 8; }
    else if (o < 3 * A) { src0 = vc + (k * 2 * A + (o - A)) * 8; stride = (u64)K * 2 * A * 8; }
    else { src0 = cl + (o - 3 * A) * 8; stride = A * 8; }
  } else {
    const int l = lane & 31, step = lane >> 5;  // two steps per instruction
    const int a0 = 16 * w;
    if (l < 8) { src0 = ec + (k * A + a0 + 2 * l) * 8; stride = (u64)K * A * 8; }
    else if (l < 24) {
      const int t = (l - 8) / 8;
      src0 = vc + (k * 2 * A + t * A + a0 + 2 * ((l - 8) % 8)) * 8;
      stride = (u64)K * 2 * A * 8;
    } else { src0 = cl + (a0 + 2 * (l - 24)) * 8; stride = A * 8; }
    src0 += step * stride;
    stride *= 2;  // piece j moves steps 2j, 2j+1
  }
  const int nch = R / C;
  const int cml = A / SPLIT / 2;  // lanes moving the clock max
  auto issue = [&](int c, int sl) {
    const char *s = src0 + (u64)c * C * (SPLIT == 1 ? stride : stride / 2);
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      glds16(s, my + sl * SLOT + j * 128);
      s += stride;
    }
    if (lane < cml) glds16(cm + ((u64)c * A + w * (A / SPLIT) + 2 * lane) * 8, cms + sl * 32);
  };
  if (SPLIT == 2 && threadIdx.x < 4) flag[threadIdx.x] = 0;
  if (SPLIT == 2) __syncthreads();
  issue(0, 0);
  issue(1, 1);
  u64 acc = 0, cw = 0;
  const u64 t0 = __builtin_amdgcn_s_memtime();
  for (int ch = 0; ch < nch; ++ch) {
    const int sl = ch & 1;
    if (ch + 1 < nch) wait_vmcnt<PIECES + 1>();
    else wait_vmcnt<0>();
    // copy the slot into registers (the RS path's reload: 8 x 16 B per lane at SPLIT 1)
    u64x2 r[8 / SPLIT];
    const u64 *img = my + sl * SLOT;
#pragma unroll
    for (int m = 0; m < 8 / SPLIT; ++m) r[m] = *reinterpret_cast<const u64x2 *>(img + (m * 64 + lane) * 2);
    const u64 cmv = cms[sl * 32 + (lane & 31)];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (ch + 2 < nch) issue(ch + 2, sl);
    const u64 tw = __builtin_amdgcn_s_memtime();
    unsigned x = (unsigned)cmv;
#pragma unroll
    for (int m = 0; m < 8 / SPLIT; ++m) x ^= (unsigned)(r[m].x ^ r[m].y);
    for (int i = 0; i < work; ++i) x = x * 2654435761u + (unsigned)i;
    acc += x;
    if (SPLIT == 2 && sync) {  // hand this chunk's "vote" to the partner and wait for its own
      if (lane == 0) flag[2 * (ch & 1) + w] = (unsigned)ch + 1;
      unsigned spins = 0;
      while (__builtin_amdgcn_readfirstlane(flag[2 * (ch & 1) + (w ^ 1)]) < (unsigned)ch + 1 && ++spins < (1u << 22)) {
      }
    }
    cw += __builtin_amdgcn_s_memtime() - tw;
  }
  const u64 t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    cyc[2 * (blockIdx.x * SPLIT + w)] = t1 - t0;
    cyc[2 * (blockIdx.x * SPLIT + w) + 1] = cw;
  }
  if (acc == 0x1234567ull) out[0] = acc;
}

template <int SPLIT>
void run(const char *ec, const char *vc, const char *cl, const char *cm, int work, int sync, u64 *out, u64 *cyc) {
  const size_t lds = SPLIT * (2 * (16 * 128 / SPLIT) + 64) * 8 + 64;
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  hipLaunchKernelGGL(mstream<SPLIT>, dim3(K), dim3(64 * SPLIT), lds, 0, ec, vc, cl, cm, work, sync, out, cyc);
  float best = 1e30f, sum = 0;
  const int reps = 5;
  for (int rep = 0; rep < reps; ++rep) {
    hipEventRecord(s);
    hipLaunchKernelGGL(mstream<SPLIT>, dim3(K), dim3(64 * SPLIT), lds, 0, ec, vc, cl, cm, work, sync, out, cyc);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    best = ms < best ? ms : best;
    sum += ms;
  }
  static u64 h[2 * 2 * K];
  hipMemcpy(h, cyc, sizeof(u64) * 2 * SPLIT * K, hipMemcpyDeviceToHost);
  double tot = 0, wk = 0;
  for (int i = 0; i < SPLIT * K; ++i) {
    tot += h[2 * i];
    wk += h[2 * i + 1];
  }
  tot /= SPLIT * K;
  wk /= SPLIT * K;
  const double alg = 13159852256.0;
  printf("split %d work %5d sync %d: best %.3f ms avg %.3f ms  %.1f%% of 8 TB/s (best)  per chunk: %.0f clk total, %.0f clk in work\n",
         SPLIT, work, sync, best, sum / reps, alg / (best * 1e-3) / 8e12 * 100, tot / (R / C), wk / (R / C));
  fflush(stdout);
  hipEventDestroy(s);
  hipEventDestroy(e);
}

int main(int argc, char **argv) {
  const size_t bec = (size_t)R * K * A * 8, bvc = 2 * bec, bcl = (size_t)R * A * 8, bcm = (size_t)(R / C) * A * 8;
  char *ec, *vc, *cl, *cm;
  u64 *out, *cyc;
  if (hipMalloc(&ec, bec) || hipMalloc(&vc, bvc) || hipMalloc(&cl, bcl) || hipMalloc(&cm, bcm) ||
      hipMalloc(&out, 64) || hipMalloc(&cyc, sizeof(u64) * 4 * K)) {
    printf("hipMalloc failed\n");
    return 1;
  }
  hipMemset(ec, 1, bec);
  hipMemset(vc, 2, bvc);
  hipMemset(cl, 3, bcl);
  hipMemset(cm, 4, bcm);
  hipDeviceSynchronize();
  for (int work : {0, 100, 200, 300, 400, 600}) run<1>(ec, vc, cl, cm, work, 0, out, cyc);
  for (int work : {0, 50, 100, 150, 200, 300}) run<2>(ec, vc, cl, cm, work, 0, out, cyc);
  for (int work : {0, 50, 100, 150, 200, 300}) run<2>(ec, vc, cl, cm, work, 1, out, cyc);
  return 0;
}
