// Microbenchmark: cost per wave of one global_load_lds_dwordx4 (LDS-DMA) piece on gfx950 as a
// function of the active lanes (64 = 1 KiB, 48 = 768 B, 32, 16) and of the source (an L2-resident
// 64 KiB window or a streamed 2 GiB buffer), one wave per SIMD (the Map fold's occupancy), 16 pieces
// per batch and two batches in flight (the RS path's ring).  Answers: is the ~60-cycle issue cost
// of a Map chunk piece per instruction or per byte?
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned long long u64;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ __launch_bounds__(64) void glds_kernel(const char *src, u64 mask, int iters, int active, u64 *out) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x;
  const u64 wave = blockIdx.x;
  u64 off = (wave * 16 * 1024) & mask;
  for (int i = 0; i < iters; ++i) {
    u64 *slot = lds + (i & 1) * 16 * 128;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      // active < 0: the SH path's first packing, lane l moving 16 bytes of row (l % 4), the rows
      // 4 KiB apart (every quad of lanes touches 4 lines); active == 65: rows of 256 B, lanes
      // 16 j .. 16 j + 15 contiguous in row j (every quad one 64-byte run)
      // active == 66: quad-interleaved (quad t = step t % 4, pairs 4 (t / 4) ..), active == 67: 16 lanes
      // per row, the row's pairs rotated by 4 * row
      const u64 lo = active < 0    ? (u64)(lane & 3) * 4096 + (u64)(lane >> 2) * 16
                     : active == 65 ? (u64)(lane >> 4) * 4096 + (u64)(lane & 15) * 16
                     : active == 66 ? (u64)((lane >> 2) & 3) * 4096 + (u64)(4 * (lane >> 4) + (lane & 3)) * 16
                     : active == 67 ? (u64)(lane >> 4) * 4096 + (u64)(((lane & 15) + 4 * (lane >> 4)) & 15) * 16
                                    : (u64)lane * 16;
      if (active < 0 || active >= 65 || lane < active)
        __builtin_amdgcn_global_load_lds(src + ((off + s * 1024 + lo) & mask),
                                         (__attribute__((address_space(3))) void *)(slot + s * 128), 16, 0, 0);
    }
    off += (u64)gridDim.x * 16 * 1024;
    wait_vmcnt<16>();
  }
  wait_vmcnt<0>();
  if (lane == 0) out[wave] = lds[lane];
}

float run(const char *src, u64 mask, int blocks, int iters, int active, u64 *out) {
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  const size_t lds = 2 * 16 * 128 * 8;
  hipLaunchKernelGGL(glds_kernel, dim3(blocks), dim3(64), lds, 0, src, mask, iters, active, out);
  hipEventRecord(s);
  hipLaunchKernelGGL(glds_kernel, dim3(blocks), dim3(64), lds, 0, src, mask, iters, active, out);
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms;
  hipEventElapsedTime(&ms, s, e);
  return ms;
}

int main() {
  const size_t big = 2ull << 30;
  char *src;
  u64 *out;
  hipMalloc(&src, big);
  hipMemset(src, 1, big);
  hipMalloc(&out, 8192 * 8);
  const int iters = 2000;
  for (int blocks : {1024}) {
    for (int act : {64, -1, 65, 66, 67}) {
      for (int which = 0; which < 2; ++which) {
        const u64 mask = which ? big - 1 : (64 << 10) - 1;
        const float ms = run(src, mask, blocks, iters, act, out);
        const double pieces = (double)iters * 16;
        const double ns = ms * 1e6 / pieces;
        const double bytes = (double)blocks * pieces * (act < 0 || act >= 65 ? 64 : act) * 16;
        printf("waves %5d lanes %2d src %-6s: %.2f ns (%.0f cycles @2.4GHz) per piece per wave, %.2f TB/s\n", blocks,
               act, which ? "stream" : "L2", ns, ns * 2.4, bytes / (ms * 1e-3) / 1e12);
      }
    }
  }
  return 0;
}
