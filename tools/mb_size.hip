// HBM stream rate against buffer size: copy (read + write) and read-only sum over 128 MiB ..
// 8 GiB per buffer, fresh random data, contiguous-per-workgroup order.  Does the read+write
// ceiling measured on the 2-16 GB solver shapes (5.4-5.5 TB/s) depend on the footprint?
// Not part of the library.   hipcc --offload-arch=gfx950 -O3 tools/mb_size.hip -o tools/mb_size
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

__global__ void fill(d2 *p, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    unsigned long long x = (i + 7) * 6364136223846793005ULL;
    x ^= x >> 31;
    p[i] = d2{(double)(x & 0xFFFF), (double)((x >> 16) & 0xFFFF)};
  }
}
template <int U, bool WRITE>
__global__ __launch_bounds__(256) void k_stream(const d2 *__restrict__ a, d2 *b, long long n, double *sink) {
  const long long tile = 256LL * U, ntile = n / tile;
  const long long t0 = ntile * blockIdx.x / gridDim.x, t1 = ntile * (blockIdx.x + 1) / gridDim.x;
  d2 acc = {0, 0};
  for (long long t = t0; t < t1; ++t) {
    const long long base = t * tile + threadIdx.x;
    d2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = a[base + (long long)u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (WRITE) b[base + (long long)u * 256] = v[u];
      else acc += v[u];
    }
  }
  if (!WRITE && acc.x == 12345.678) sink[0] = acc.y;
}
template <class F> float timeit(F f, int reps) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a)); for (int i = 0; i < reps; ++i) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}
int main() {
  int dev = 0, ncu = 0; CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const long long maxn = 1LL << 29;  // 8 GiB of d2
  d2 *a, *b; double *sink;
  CK(hipMalloc(&a, 16 * maxn)); CK(hipMalloc(&b, 16 * maxn)); CK(hipMalloc(&sink, 64));
  fill<<<4096, 256>>>(a, maxn); fill<<<4096, 256>>>(b, maxn); CK(hipDeviceSynchronize());
  for (long long n = 1LL << 23; n <= maxn; n <<= 2) {
    const double gb = 16.0 * n / 1e9;
    for (int wg : {4, 8}) {
      const int grid = wg * ncu;
      const int reps = n < (1LL << 26) ? 50 : 8;
      float c = timeit([&] { k_stream<4, true><<<grid, 256>>>(a, b, n, sink); }, reps);
      float r = timeit([&] { k_stream<4, false><<<grid, 256>>>(a, b, n, sink); }, reps);
      float r8 = timeit([&] { k_stream<8, false><<<grid, 256>>>(a, b, n, sink); }, reps);
      printf("buffer %7.3f GB  wg/CU %d  copy %6.0f GB/s (r+w)  read U4 %6.0f GB/s  read U8 %6.0f GB/s\n", gb, wg,
             2 * gb / (c * 1e-3), gb / (r * 1e-3), gb / (r8 * 1e-3));
    }
  }
  return 0;
}
