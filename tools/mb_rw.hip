// Read/write mix probe: stream L columns (+ the k columns of X) and write the k columns of X
// in the update kernels' pattern (thread per row pair, 16-B accesses, grid-stride), with
// the stores plain, non-temporal, or off; plus a copy kernel.  Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

template <int MODE, int K>  // MODE 0: no store, 1: plain store, 2: nontemporal store, 3: sc1, 4: sc0 sc1,
                            // 5: X not read, plain store into X, 6: X read, store into a separate Y
__global__ __launch_bounds__(256) void k_rw(const double *__restrict__ Q, double *X, long long ld, int L, long long nrows,
                                            double *__restrict__ out) {
  d2 acc[K];
#pragma unroll
  for (int c = 0; c < K; ++c) acc[c] = d2{0, 0};
  for (long long r = 2LL * ((long long)blockIdx.x * 256 + threadIdx.x); r < nrows; r += 2LL * gridDim.x * 256) {
    int j = 0;
    for (; j + 4 <= L; j += 4) {
      d2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(const d2 *)(Q + (long long)(j + u) * ld + r);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += v[u];
    }
#pragma unroll
    for (int c = 0; c < K; ++c) {
      double *xp = X + (long long)c * ld + r;
      d2 x = MODE == 5 ? d2{0.0, 0.0} : *(const d2 *)xp;
      x += acc[c];
      if (MODE == 1) *(d2 *)xp = x;
      if (MODE == 2) __builtin_nontemporal_store(x, (d2 *)xp);
      if (MODE == 3) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(xp), "v"(x) : "memory");
      if (MODE == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(xp), "v"(x) : "memory");
      if (MODE == 5) *(d2 *)xp = x;
      if (MODE == 6) *(d2 *)(xp + 16 * ld) = x;
      if (MODE == 0 && x.x == 1234.5) out[threadIdx.x] = x.y;
    }
  }
}

__global__ __launch_bounds__(256) void k_copy(const d2 *__restrict__ a, d2 *__restrict__ b, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) b[i] = a[i];
}

template <class F> float timeit(F f) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < 5; ++i) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / 5;
}

int main() {
  const long long n = 1LL << 24, ld = n + 64;
  const int k = 8;
  double *V, *o;
  CK(hipMalloc(&V, sizeof(double) * ld * 232));
  CK(hipMalloc(&o, 8192));
  CK(hipMemset(V, 0, sizeof(double) * ld * 232));
  for (int grid : {1024, 4096}) {
    for (int L : {64, 104, 200}) {
      double *X = V + (long long)L * ld;
      const double by_r = 8.0 * n * (L + k), by_rw = 8.0 * n * (L + 2 * k);
      float t0 = timeit([&] { k_rw<0, 8><<<grid, 256>>>(V, X, ld, L, n, o); });
      float t1 = timeit([&] { k_rw<1, 8><<<grid, 256>>>(V, X, ld, L, n, o); });
      float t2 = timeit([&] { k_rw<2, 8><<<grid, 256>>>(V, X, ld, L, n, o); });
      float t5 = timeit([&] { k_rw<5, 8><<<grid, 256>>>(V, X, ld, L, n, o); });
      float t6 = timeit([&] { k_rw<6, 8><<<grid, 256>>>(V, X, ld, L, n, o); });
      const double by_w = 8.0 * n * (L + k);
      printf("grid %4d L=%3d read-only %6.0f GB/s | in-place store %6.0f | nt %6.0f | X not read %6.0f | store to Y %6.0f GB/s\n",
             grid, L, by_r / t0 / 1e6, by_rw / t1 / 1e6, by_rw / t2 / 1e6, by_w / t5 / 1e6, by_rw / t6 / 1e6);
    }
  }
  const long long nc = n * 8 / 2;
  float tc = timeit([&] { k_copy<<<4096, 256>>>((const d2 *)V, (d2 *)(V + 8 * ld), nc); });
  printf("copy 1 GB: %6.0f GB/s\n", 2.0 * 16 * nc / tc / 1e6);
  return 0;
}
