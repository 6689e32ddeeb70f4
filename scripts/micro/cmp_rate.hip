// Microbenchmark: issue cost of 64-bit vs 32-bit integer compares feeding ballots on gfx950,
// one wave per SIMD (the Map fold's occupancy).  Prints ns per compare+ballot per wave.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T>
__global__ __launch_bounds__(64) void cmp_kernel(const T *in, unsigned long long *out, int iters) {
  T a = in[threadIdx.x], b = in[64 + threadIdx.x], c = in[128 + threadIdx.x], d = in[192 + threadIdx.x];
  unsigned long long m0 = ~0ull, m1 = ~0ull, m2 = 0, m3 = ~0ull;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      m0 &= __ballot(a <= b);
      m1 &= __ballot(c - 1 >= d);
      m2 |= __ballot(a != c);
      m3 &= __ballot(b <= d);
      a += (T)1; b += (T)1; c += (T)1; d += (T)1;
    }
  }
  if (threadIdx.x == 0) out[blockIdx.x] = m0 ^ m1 ^ m2 ^ m3;
}

template <typename T>
float run(int blocks, int iters) {
  T *in; unsigned long long *out;
  hipMalloc(&in, 256 * sizeof(T));
  hipMemset(in, 1, 256 * sizeof(T));
  hipMalloc(&out, blocks * 8);
  hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
  hipLaunchKernelGGL(cmp_kernel<T>, dim3(blocks), dim3(64), 0, 0, in, out, iters);
  hipEventRecord(s);
  hipLaunchKernelGGL(cmp_kernel<T>, dim3(blocks), dim3(64), 0, 0, in, out, iters);
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms; hipEventElapsedTime(&ms, s, e);
  hipFree(in); hipFree(out);
  return ms;
}

int main() {
  const int blocks = 1024, iters = 20000;  // one wave per SIMD on 256 CUs
  const double cmps = (double)iters * 16 * 4;
  float t64 = run<unsigned long long>(blocks, iters);
  float t32 = run<unsigned>(blocks, iters);
  printf("u64: %.3f ms, %.3f ns per compare+ballot per wave\n", t64, t64 * 1e6 / cmps);
  printf("u32: %.3f ms, %.3f ns per compare+ballot per wave\n", t32, t32 * 1e6 / cmps);
  return 0;
}
