// Microbenchmark: the HBM stream ceilings the pairwise merge / forget kernels run against on gfx950.
//   copy   : out[i] = a[i]                      (1 read, 1 write: the whole-state forget's shape)
//   max_oop: out[i] = max(a[i], b[i])           (2 reads, 1 write to a third array)
//   max_ip : a[i]   = max(a[i], b[i])           (2 reads, 1 write back over a read: merge_batch)
//   read   : acc ^= a[i]                        (read only)
// 16-byte lanes, U pieces in flight per lane before the first store, grid = CUs x blocks-per-CU of
// 256 threads (grid-stride), optional non-temporal loads / stores.  Bytes counted: every read and
// every write once (the algorithmic bytes of DESIGN.md 3.5).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

template <int MODE, int U, bool NT>
__global__ __launch_bounds__(256) void stream_kernel(u64x2 *a, const u64x2 *b, u64x2 *out, size_t n, u64 *sink) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  u64x2 acc = {0, 0};
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u64x2 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = NT ? __builtin_nontemporal_load(a + i + u * stride) : a[i + u * stride];
      if (MODE == 1 || MODE == 2) y[u] = NT ? __builtin_nontemporal_load(b + i + u * stride) : b[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      u64x2 r = x[u];
      if (MODE == 1 || MODE == 2) {
        r.x = x[u].x > y[u].x ? x[u].x : y[u].x;
        r.y = x[u].y > y[u].y ? x[u].y : y[u].y;
      }
      if (MODE == 3) {
        acc ^= r;
        continue;
      }
      u64x2 *dst = (MODE == 2 ? a : out) + i + u * stride;
      if (NT) __builtin_nontemporal_store(r, dst);
      else *dst = r;
    }
  }
  for (; i < n; i += stride) {  // tail
    u64x2 r = a[i];
    if (MODE == 1 || MODE == 2) {
      const u64x2 y = b[i];
      r.x = r.x > y.x ? r.x : y.x;
      r.y = r.y > y.y ? r.y : y.y;
    }
    if (MODE == 3) acc ^= r;
    else (MODE == 2 ? a : out)[i] = r;
  }
  if (MODE == 3 && (acc.x ^ acc.y) == 0x123456789ULL) sink[0] = acc.x;  // keep the reads alive
}

template <int MODE, int U, bool NT>
float run(u64x2 *a, u64x2 *b, u64x2 *o, size_t n, int blocks, u64 *sink) {
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  hipLaunchKernelGGL((stream_kernel<MODE, U, NT>), dim3(blocks), dim3(256), 0, 0, a, b, o, n, sink);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(s);
    hipLaunchKernelGGL((stream_kernel<MODE, U, NT>), dim3(blocks), dim3(256), 0, 0, a, b, o, n, sink);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    if (ms < best) best = ms;
  }
  hipEventDestroy(s);
  hipEventDestroy(e);
  return best;
}

static const char *kName[] = {"copy", "max_oop", "max_ip", "read"};
static const int kArrays[] = {2, 3, 3, 1};  // bytes moved = arrays x array bytes

template <int MODE, int U, bool NT>
void sweep(u64x2 *a, u64x2 *b, u64x2 *o, size_t n, int cus, u64 *sink) {
  for (int bpc : {1, 2, 3, 4, 8}) {
    const float ms = run<MODE, U, NT>(a, b, o, n, cus * bpc, sink);
    const double bytes = (double)kArrays[MODE] * n * 16;
    printf("%-8s U=%d nt=%d blocks/CU=%d: %.3f ms  %.2f TB/s  (%.1f%% of 8 TB/s)\n", kName[MODE], U, NT ? 1 : 0, bpc,
           ms, bytes / (ms * 1e-3) / 1e12, bytes / (ms * 1e-3) / 8e12 * 100);
    fflush(stdout);
  }
}

int main(int argc, char **argv) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  // per array: far past the 256 MB of last-level cache (argv[2]: GiB per array, default 4)
  const size_t bytes = (argc > 2 ? (size_t)atoi(argv[2]) : 4ull) << 30;
  const size_t n = bytes / 16;
  u64x2 *a, *b, *o;
  u64 *sink;
  if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&o, bytes) || hipMalloc(&sink, 64)) {
    printf("hipMalloc failed\n");
    return 1;
  }
  hipMemset(a, 1, bytes);
  hipMemset(b, 2, bytes);
  hipMemset(o, 0, bytes);
  printf("CUs %d, %zu MiB per array\n", cus, bytes >> 20);
  const int which = argc > 1 ? atoi(argv[1]) : 0;
  if (which == 0) {
    sweep<3, 4, true>(a, b, o, n, cus, sink);
    sweep<0, 4, true>(a, b, o, n, cus, sink);
    sweep<0, 4, false>(a, b, o, n, cus, sink);
    sweep<0, 8, true>(a, b, o, n, cus, sink);
    sweep<1, 4, true>(a, b, o, n, cus, sink);
    sweep<2, 4, true>(a, b, o, n, cus, sink);
    sweep<2, 4, false>(a, b, o, n, cus, sink);
    sweep<2, 8, true>(a, b, o, n, cus, sink);
    sweep<2, 1, true>(a, b, o, n, cus, sink);
  } else if (which == 2) {  // the in-place merge at 1-4 pieces per lane, few workgroups (array size sweep)
    for (int pass = 0; pass < 2; ++pass) {
      sweep<2, 1, true>(a, b, o, n, cus, sink);
      sweep<2, 2, true>(a, b, o, n, cus, sink);
      sweep<2, 4, true>(a, b, o, n, cus, sink);
    }
  } else {  // the in-place merge and the copy at few pieces in flight, three passes (run-to-run spread)
    for (int pass = 0; pass < 3; ++pass) {
      sweep<2, 1, true>(a, b, o, n, cus, sink);
      sweep<2, 2, true>(a, b, o, n, cus, sink);
      sweep<2, 1, false>(a, b, o, n, cus, sink);
      sweep<0, 1, true>(a, b, o, n, cus, sink);
      sweep<0, 2, true>(a, b, o, n, cus, sink);
    }
  }
  return 0;
}
