// Write-path ceiling probe: where does a read+write stream top out on
// this chip, and which store/launch shape gets there?  Copy and in-place-update variants
// (loads in flight per thread, grid size, contiguous-per-workgroup vs grid-stride order,
// plain vs nontemporal stores), then the closing-update shape (read L columns + k columns,
// write k columns in place) in the same variants.  Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

// copy n d2 elements a -> b; U elements per thread in flight; CONTIG: workgroup owns a
// contiguous range of 16 B x NT x U tiles; NTS: nontemporal stores; INPLACE: b == a, scaled
template <int U, int NT, bool CONTIG, bool NTS, bool INPLACE>
__global__ __launch_bounds__(NT) void k_copy(const d2 *__restrict__ a, d2 *b, long long n) {
  const long long tile = (long long)NT * U, ntile = n / tile;
  long long t0, t1, st;
  if (CONTIG) { t0 = ntile * blockIdx.x / gridDim.x; t1 = ntile * (blockIdx.x + 1) / gridDim.x; st = 1; }
  else { t0 = blockIdx.x; t1 = ntile; st = gridDim.x; }
  for (long long t = t0; t < t1; t += st) {
    const long long base = t * tile + threadIdx.x;
    d2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = a[base + (long long)u * NT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      d2 x = INPLACE ? v[u] * 1.0000001 : v[u];
      if (NTS) __builtin_nontemporal_store(x, b + base + (long long)u * NT);
      else b[base + (long long)u * NT] = x;
    }
  }
}

// closing-update shape: thread per row pair; L columns of Q and K columns of X read, X
// written in place (X - sum Q); CONTIG: workgroup owns a contiguous row range
template <int K, int NB, bool CONTIG, bool NTS>
__global__ __launch_bounds__(256) void k_upd(const double *__restrict__ Q, double *X, long long ld, int L,
                                             long long nrows) {
  const long long np = nrows / 2;
  long long p0, p1, st;
  if (CONTIG) {
    const long long nt = np / 256;
    p0 = nt * blockIdx.x / gridDim.x * 256 + threadIdx.x; p1 = nt * (blockIdx.x + 1) / gridDim.x * 256; st = 256;
  } else { p0 = (long long)blockIdx.x * 256 + threadIdx.x; p1 = np; st = (long long)gridDim.x * 256; }
  for (long long p = p0; p < p1; p += st) {
    const long long r = 2 * p;
    d2 acc[K];
#pragma unroll
    for (int c = 0; c < K; ++c) acc[c] = d2{0, 0};
    int j = 0;
    for (; j + NB <= L; j += NB) {
      d2 v[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) v[u] = *(const d2 *)(Q + (long long)(j + u) * ld + r);
#pragma unroll
      for (int u = 0; u < NB; ++u) acc[u % K] += v[u];
    }
#pragma unroll
    for (int c = 0; c < K; ++c) {
      double *xp = X + (long long)c * ld + r;
      const d2 x = *(const d2 *)xp - acc[c];
      if (NTS) __builtin_nontemporal_store(x, (d2 *)xp);
      else *(d2 *)xp = x;
    }
  }
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

int cus() { int d = 0, c = 0; CK(hipGetDevice(&d)); CK(hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d)); return c; }

#define COPY(U, NT, C, N, I, label)                                                                       \
  for (int wgcu : {1, 2, 4, 8}) {                                                                         \
    const int grid = wgcu * ncu * (1024 / NT);                                                              \
    float ms = timeit([&] { k_copy<U, NT, C, N, I><<<grid, NT>>>(src, I ? src : dst, n); });                \
    printf("copy %-26s U=%d NT=%4d grid=%5d %6.3f ms %6.0f GB/s\n", label, U, NT, grid, ms, 32.0 * n / ms / 1e6); \
  }

int main() {
  const int ncu = cus();
  const long long n = 1LL << 27;  // 2 GiB of d2 each way
  d2 *src, *dst;
  CK(hipMalloc(&src, 16 * n));
  CK(hipMalloc(&dst, 16 * n));
  CK(hipMemset(src, 0, 16 * n));
  CK(hipMemset(dst, 0, 16 * n));
  COPY(1, 256, false, false, false, "stride")
  COPY(4, 256, false, false, false, "stride")
  COPY(8, 256, false, false, false, "stride")
  COPY(4, 256, true, false, false, "contig")
  COPY(8, 256, true, false, false, "contig")
  COPY(4, 1024, true, false, false, "contig")
  COPY(4, 256, false, true, false, "stride nt")
  COPY(4, 256, true, true, false, "contig nt")
  COPY(4, 256, false, false, true, "stride in-place")
  COPY(4, 256, true, false, true, "contig in-place")
  COPY(8, 256, true, false, true, "contig in-place")
  CK(hipFree(dst));
  const long long nr = 1LL << 24, ld = nr + 64;
  double *V;
  CK(hipMalloc(&V, sizeof(double) * ld * 232));
  CK(hipMemset(V, 0, sizeof(double) * ld * 232));
  for (int L : {104, 200}) {
    double *X = V + (long long)L * ld;
    const double by = 8.0 * nr * (L + 16);
    for (int wgcu : {1, 2, 4, 8}) {
      const int grid = wgcu * ncu * 4;
      float a = timeit([&] { k_upd<8, 8, false, false><<<grid, 256>>>(V, X, ld, L, nr); });
      float b = timeit([&] { k_upd<8, 8, true, false><<<grid, 256>>>(V, X, ld, L, nr); });
      float c = timeit([&] { k_upd<8, 16, true, false><<<grid, 256>>>(V, X, ld, L, nr); });
      float d = timeit([&] { k_upd<8, 8, true, true><<<grid, 256>>>(V, X, ld, L, nr); });
      printf("upd L=%3d grid=%5d stride %6.0f | contig %6.0f | contig NB16 %6.0f | contig nt %6.0f GB/s\n", L, grid,
             by / a / 1e6, by / b / 1e6, by / c / 1e6, by / d / 1e6);
    }
  }
  return 0;
}
