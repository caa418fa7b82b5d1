// Shape sweep of the library's own kernels (links build/csrc/kernels.o, icgs.o): GB/s of
// algorithmic bytes per launch at the Block GMRES shapes.  Not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_lib.cpp build/csrc/kernels.o build/csrc/icgs.o
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

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
double timeit(F f, int reps = 10) {
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
  const long long ld = (n + 63) / 64 * 64 + (argc > 2 ? atoi(argv[2]) : 0);
  const int k = 8, Lmax = 216;
  double *V, *P, *R, *S;
  CK(hipMalloc(&V, sizeof(double) * ld * Lmax + 256));
  CK(hipMalloc(&P, sizeof(double) * 4096 * 512 * 16 + sizeof(double) * 2048 * 256 * 16));
  CK(hipMalloc(&R, sizeof(double) * 512 * 16));
  double *SINK;
  CK(hipMalloc(&SINK, sizeof(double) * 256 * 4096));
  CK(hipMalloc(&S, sizeof(double) * ld));
  fill<<<(ld * Lmax + 255) / 256, 256>>>(V, ld * Lmax, 1);
  CK(hipMemset(R, 0, sizeof(double) * 512 * 16));
  CK(hipDeviceSynchronize());
  hipStream_t s = 0;
  const int nblk = gemm_tn_blocks((int)n);
  printf("n=%lld gemm_tn blocks=%d\n", n, nblk);
  for (int L : {8, 16, 32, 64, 104, 128, 160, 200}) {
    MvDesc A{V, ld, nullptr, L + k};
    MvDesc X{V + (long long)L * ld, ld, nullptr, k};
    const double by_tn = 8.0 * n * (L + k + k);
    double t_tn = timeit([&] { launch_gemm_tn_partial(s, A, L + k, X, k, (int)n, P, nblk); });
    double t_red = timeit([&] { launch_reduce_partials_ld(s, P, nblk, L + k, k, L + k, 1.0, R); });
    MvDesc Q{V, ld, nullptr, L};
    double t_nn = timeit([&] { launch_gemm_nn(s, Q, L, R, L + k, X, (int)n, -1.0, 1.0); });
    const int nb2 = icgs_blocks((int)n);
    double t_nnd = timeit([&] { launch_gemm_nn_dot(s, Q, L, R, L + k, X, (int)n, -1.0, 1.0, 1, X, P, nb2); });
    const double by_nn = 8.0 * n * (L + 2 * k);
    const int nbf = nn_tn_blocks((int)n, L, k);
    double t_f = timeit([&] { launch_nn_tn(s, Q, L, R, L + k, X, (int)n, P, nbf, SINK); });
    printf("L=%3d  tn %7.3f ms %6.0f GB/s | reduce %6.1f us | nn %7.3f ms %6.0f GB/s | nn_dot %7.3f ms %6.0f GB/s"
           " | nn_tn %7.3f ms %6.0f GB/s (%d wg)\n", L,
           t_tn, by_tn / t_tn / 1e6, t_red * 1e3, t_nn, by_nn / t_nn / 1e6, t_nnd, by_nn / t_nnd / 1e6, t_f,
           by_nn / t_f / 1e6, nbf);
  }
  // correctness of the fused update+projection against nn followed by tn (L = 200, 40, 13)
  for (int L : {200, 40, 13}) {
    double *Xb, *R2a, *R2b;
    CK(hipMalloc(&Xb, sizeof(double) * ld * k));
    CK(hipMalloc(&R2a, sizeof(double) * L * k));
    CK(hipMalloc(&R2b, sizeof(double) * L * k));
    MvDesc Q{V, ld, nullptr, L};
    MvDesc X{V + (long long)L * ld, ld, nullptr, k};
    MvDesc XB{Xb, ld, nullptr, k};
    fill<<<(ld * Lmax + 255) / 256, 256>>>(V, ld * Lmax, 7);
    for (int c = 0; c < Lmax; ++c) CK(hipMemset(V + (long long)c * ld + n, 0, sizeof(double) * (ld - n)));
    fill<<<((L + k) * k + 255) / 256, 256>>>(R, (long long)(L + k) * k, 3);
    CK(hipMemcpy(Xb, X.base, sizeof(double) * ld * k, hipMemcpyDeviceToDevice));
    launch_gemm_nn(s, Q, L, R, L + k, X, (int)n, -1.0, 1.0);
    launch_gemm_tn_partial(s, Q, L, X, k, (int)n, P, nblk);
    launch_reduce_partials_ld(s, P, nblk, L, k, L, 1.0, R2a);
    const int nbf = nn_tn_blocks((int)n, L, k);
    launch_nn_tn(s, Q, L, R, L + k, XB, (int)n, P, nbf, SINK);
    launch_reduce_partials_ld(s, P, nbf, L, k, L, 1.0, R2b);
    CK(hipDeviceSynchronize());
    std::vector<double> xa((size_t)ld * k), xb((size_t)ld * k), ra(L * k), rb(L * k);
    CK(hipMemcpy(xa.data(), X.base, sizeof(double) * ld * k, hipMemcpyDeviceToHost));
    CK(hipMemcpy(xb.data(), Xb, sizeof(double) * ld * k, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ra.data(), R2a, sizeof(double) * L * k, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rb.data(), R2b, sizeof(double) * L * k, hipMemcpyDeviceToHost));
    double dx = 0, mx = 0, dr = 0, mr = 0;
    for (size_t i = 0; i < xa.size(); ++i) dx = fmax(dx, fabs(xa[i] - xb[i])), mx = fmax(mx, fabs(xa[i]));
    for (size_t i = 0; i < ra.size(); ++i) dr = fmax(dr, fabs(ra[i] - rb[i])), mr = fmax(mr, fabs(ra[i]));
    printf("check nn_tn L=%d: X1 maxdiff %.3e (max %.3e)  R2 maxdiff %.3e (max %.3e)  %s\n", L, dx, mx, dr, mr,
           (dx <= 1e-12 * mx && dr <= 1e-10 * mr) ? "OK" : "MISMATCH");
    CK(hipFree(Xb));
    CK(hipFree(R2a));
    CK(hipFree(R2b));
  }
  // findBasis column kernels on the k-block
  IcgsState *st;
  CK(hipMalloc(&st, sizeof(IcgsState)));
  CK(hipMemset(st, 0, sizeof(IcgsState)));
  MvDesc X{V, ld, nullptr, k};
  for (int nb2 : {icgs_blocks((int)n), 1024, 2048, 4096})
  for (int j : {1, 3, 7}) {
    printf("nb=%d ", nb2);
    double ta = timeit([&] { launch_fb_a(s, X, j, st, (int)n, P, nb2); });
    double tb = j ? timeit([&] { launch_fb_b(s, X, j, st, S, (int)n, P, nb2); }) : 0;
    double tc = j ? timeit([&] { launch_fb_c(s, X, j, st, S, (int)n, P, nb2); }) : 0;
    printf("fb j=%d  a %6.3f ms %6.0f GB/s  b %6.3f ms %6.0f GB/s  c %6.3f ms %6.0f GB/s\n", j, ta,
           8.0 * n * (j + 1 + (j > 0)) / ta / 1e6, tb, tb ? 8.0 * n * (j + 2) / tb / 1e6 : 0, tc,
           tc ? 8.0 * n * (j + 3) / tc / 1e6 : 0);
  }
  // SpMM on the 7-point stencil (CSR built on the host)
  {
    std::vector<int> rp(n + 1), ci;
    std::vector<double> vv;
    ci.reserve(n * 7);
    vv.reserve(n * 7);
    const long long m2 = (long long)m * m;
    for (long long g = 0; g < n; ++g) {
      const long long ix = g % m, iy = (g / m) % m, iz = g / m2;
      if (iz > 0) { ci.push_back(g - m2); vv.push_back(-1); }
      if (iy > 0) { ci.push_back(g - m); vv.push_back(-1); }
      if (ix > 0) { ci.push_back(g - 1); vv.push_back(-1); }
      ci.push_back(g); vv.push_back(6);
      if (ix < m - 1) { ci.push_back(g + 1); vv.push_back(-1); }
      if (iy < m - 1) { ci.push_back(g + m); vv.push_back(-1); }
      if (iz < m - 1) { ci.push_back(g + m2); vv.push_back(-1); }
      rp[g + 1] = (int)ci.size();
    }
    int *drp, *dci;
    double *dvv;
    CK(hipMalloc(&drp, sizeof(int) * (n + 1)));
    CK(hipMalloc(&dci, sizeof(int) * ci.size()));
    CK(hipMalloc(&dvv, sizeof(double) * vv.size()));
    CK(hipMemcpy(drp, rp.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(dci, ci.data(), sizeof(int) * ci.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dvv, vv.data(), sizeof(double) * vv.size(), hipMemcpyHostToDevice));
    for (int kk : {1, 8, 16}) {
      MvDesc Xs{V, ld, nullptr, kk};
      MvDesc Ys{V + (long long)16 * ld, ld, nullptr, kk};
      double t = timeit([&] { launch_spmm(s, 0, (int)n, drp, dci, dvv, Xs, (int)n, nullptr, 0, Ys, 1.0, 0.0); });
      const double by = 12.0 * ci.size() + 4.0 * (n + 1) + 16.0 * n * kk;
      printf("spmm k=%2d %7.3f ms %6.0f GB/s\n", kk, t, by / t / 1e6);
    }
  }
  return 0;
}
