// Shape sweep of the ICGS streaming kernels at k = 8 and k = 16 over the projection widths of
// a Num Blocks 25 cycle (links build/csrc/kernels.o, icgs.o): ms per launch and GB/s of the
// algorithmic bytes.  Not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_k16.cpp build/csrc/kernels.o build/csrc/icgs.o -o tools/mb_k16
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../trilinos_amd/csrc/icgs.h"
#include "../trilinos_amd/csrc/internal.h"

using namespace migmres;

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

__global__ void fill(double *p, long long n, unsigned seed) {
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    unsigned long long x = (i + 1) * 6364136223846793005ULL + seed;
    x ^= x >> 29;
    p[i] = (double)(x % 100000) / 100000.0 - 0.5;
  }
}

template <class F>
double timeit(F f, int reps = 5) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char **argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 256;
  const long long n = (long long)m * m * m;
  const long long ld = (n + 63) / 64 * 64 + 64;
  const int Lmax = 416;
  double *V, *P, *R, *SINK;
  CK(hipMalloc(&V, sizeof(double) * ld * Lmax + 256));
  CK(hipMalloc(&P, sizeof(double) * 1024 * 512 * 16));
  CK(hipMalloc(&R, sizeof(double) * 512 * 16));
  CK(hipMalloc(&SINK, sizeof(double) * 1024 * 2048));
  fill<<<(ld * Lmax + 255) / 256, 256>>>(V, ld * Lmax, 1);
  for (int c = 0; c < Lmax; ++c) CK(hipMemset(V + (long long)c * ld + n, 0, sizeof(double) * (ld - n)));
  fill<<<(512 * 16 + 255) / 256, 256>>>(R, 512 * 16, 3);
  CK(hipDeviceSynchronize());
  hipStream_t s = 0;
  const int nblk = gemm_tn_blocks((int)n);
  for (int k : {8, 16}) {
    for (int L : {8, 16, 24, 32, 40, 48, 56, 64, 96, 128, 144, 160, 192, 208, 224, 256, 272, 320, 336, 352, 400}) {
      if (L + k > Lmax) continue;
      MvDesc A{V, ld, nullptr, L + k};
      MvDesc X{V + (long long)L * ld, ld, nullptr, k};
      MvDesc Q{V, ld, nullptr, L};
      const double by1 = 8.0 * n * (L + k), by2 = 8.0 * n * (L + 2 * k);
      double t_tn = timeit([&] { launch_gemm_tn_partial(s, A, L + k, X, k, (int)n, P, nblk); });
      double t_nn = timeit([&] { launch_gemm_nn(s, Q, L, R, L + k, X, (int)n, -1.0, 1.0); });
      double t_f = -1;
      int nbf = 0;
      if (nn_tn_supported(L, k)) {
        nbf = nn_tn_blocks((int)n, L, k);
        t_f = timeit([&] { launch_nn_tn(s, Q, L, R, L + k, X, (int)n, P, nbf, SINK, false); });
      }
      printf("k=%2d L=%3d  tn %7.3f ms %5.0f GB/s | nn %7.3f ms %5.0f GB/s | nn_tn %7.3f ms %5.0f GB/s (%d wg)\n", k, L,
             t_tn, by1 / t_tn / 1e6, t_nn, by2 / t_nn / 1e6, t_f, by1 / t_f / 1e6, nbf);
    }
  }
  return 0;
}
