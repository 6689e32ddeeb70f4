// Probe: issue cost of the Map fold's chunk-test pattern on gfx950 — a VALU compare writing a lane
// mask to SGPRs, AND-ed into a scalar accumulator — for 64-bit vs 32-bit compares, one and two waves
// per SIMD.  Build: hipcc --offload-arch=gfx950 -O3 scripts/probe_cmp.hip -o probe_cmp
// Prints cycles (s_memtime) per compare+and pair per wave, and the kernel time.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kIt = 4096;

template <int MODE>
__global__ __launch_bounds__(64) void probe(const unsigned long long *in, unsigned long long *out,
                                            unsigned long long *cyc) {
  const int lane = threadIdx.x;
  unsigned long long a[16], b[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    a[j] = in[(blockIdx.x * 16 + j) * 64 + lane];
    b[j] = in[(blockIdx.x * 16 + j) * 64 + lane] + 1;
  }
  unsigned long long acc = ~0ull;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIt; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      unsigned long long m;
      if constexpr (MODE == 0) {  // 64-bit compare -> SGPR mask, and-ed at once
        asm volatile("v_cmp_le_u64_e64 %0, %2, %3\n\ts_and_b64 %1, %1, %0" : "=&s"(m), "+s"(acc) : "v"(a[j]), "v"(b[j]) : "scc");
      } else if constexpr (MODE == 1) {  // 32-bit compare on the low words
        const unsigned lo = (unsigned)a[j], lb = (unsigned)b[j];
        asm volatile("v_cmp_le_u32_e64 %0, %2, %3\n\ts_and_b64 %1, %1, %0" : "=&s"(m), "+s"(acc) : "v"(lo), "v"(lb) : "scc");
      } else if constexpr (MODE == 2) {  // 64-bit compare only (results or-ed into VCC-free SGPRs later)
        asm volatile("v_cmp_le_u64_e64 %0, %1, %2" : "=s"(m) : "v"(a[j]), "v"(b[j]));
        acc &= m;
      } else if constexpr (MODE == 3) {  // 32-bit compare only
        const unsigned lo = (unsigned)a[j], lb = (unsigned)b[j];
        asm volatile("v_cmp_le_u32_e64 %0, %1, %2" : "=s"(m) : "v"(lo), "v"(lb));
        acc &= m;
      }
    }
    if constexpr (MODE == 4) {  // all 16 compares issued before the first scalar consumer
      unsigned long long mm[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) mm[j] = __ballot(a[j] <= b[j]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 16; ++j) acc &= mm[j];
    }
    if constexpr (MODE == 5) {  // two batches of 8
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        unsigned long long mm[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) mm[j] = __ballot(a[8 * h + j] <= b[8 * h + j]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc &= mm[j];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (MODE == 6) {  // per-lane AND in a VGPR, one ballot at the end
      unsigned ok = 1;
#pragma unroll
      for (int j = 0; j < 16; ++j) ok &= (a[j] <= b[j]) ? 1u : 0u;
      acc &= __ballot(ok != 0);
    }
    if constexpr (MODE == 8) {  // 16 independent u64 max (compare + two selects), the compiler's form
#pragma unroll
      for (int j = 0; j < 16; ++j) a[j] = a[j] > b[j] ? a[j] : b[j];
    }
    if constexpr (MODE == 9) {  // 16 independent u64 max: all compares first, then all selects
      unsigned long long mm[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) mm[j] = __ballot(a[j] > b[j]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        unsigned lo, hi;
        asm volatile("v_cndmask_b32_e64 %0, %2, %3, %4\n\tv_cndmask_b32_e64 %1, %5, %6, %4"
                     : "=&v"(lo), "=&v"(hi)
                     : "v"((unsigned)b[j]), "v"((unsigned)a[j]), "s"(mm[j]), "v"((unsigned)(b[j] >> 32)),
                       "v"((unsigned)(a[j] >> 32)));
        a[j] = ((unsigned long long)hi << 32) | lo;
      }
    }
    if constexpr (MODE == 7) {  // the plain C++ form the kernel uses (ballot per test, and-ed)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc &= __ballot(a[j] <= b[j]);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(a[j]), "+v"(b[j]));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
  unsigned long long x = acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) x += a[j];
  out[blockIdx.x * 64 + lane] = x;
}

template <int MODE>
static void run(int blocks, const unsigned long long *din, unsigned long long *dout, unsigned long long *dcyc,
                const char *name) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(64), 0, 0, din, dout, dcyc);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(64), 0, 0, din, dout, dcyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long *h = (unsigned long long *)malloc(blocks * 8);
  hipMemcpy(h, dcyc, blocks * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < blocks; ++i) s += (double)h[i];
  s /= blocks;
  const double pairs = (double)kIt * 16;
  printf("%-28s blocks %5d  %.3f ms  %.2f memtime-cycles per op per wave  %.3f ns per op per wave\n", name, blocks, ms,
         s / pairs, ms * 1e6 / pairs);
  free(h);
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int maxb = 4096;
  unsigned long long *din, *dout, *dcyc;
  hipMalloc(&din, (size_t)maxb * 16 * 64 * 8);
  hipMalloc(&dout, (size_t)maxb * 64 * 8);
  hipMalloc(&dcyc, (size_t)maxb * 8);
  hipMemset(din, 0, (size_t)maxb * 16 * 64 * 8);
  for (int blocks : {1024, 2048}) {
    run<0>(blocks, din, dout, dcyc, "u64 cmp + s_and (paired)");
    run<1>(blocks, din, dout, dcyc, "u32 cmp + s_and (paired)");
    run<2>(blocks, din, dout, dcyc, "u64 cmp, compiler and");
    run<3>(blocks, din, dout, dcyc, "u32 cmp, compiler and");
    run<4>(blocks, din, dout, dcyc, "16 cmps, then 16 ands");
    run<5>(blocks, din, dout, dcyc, "2 x (8 cmps, then 8 ands)");
    run<6>(blocks, din, dout, dcyc, "per-lane and, 1 ballot");
    run<7>(blocks, din, dout, dcyc, "ballot per test (kernel form)");
    run<8>(blocks, din, dout, dcyc, "u64 max, compiler form");
    run<9>(blocks, din, dout, dcyc, "u64 max, compares batched");
  }
  return 0;
}
