// Diagnostic builds of the fused update+projection kernel (icgs.hip) with parts switched
// off (NT_DIAG_MASK, see icgs.hip), timed at the Block GMRES shapes.  Not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DNT_DIAG_MASK=<m> [-DMB_K=16] -I trilinos_amd/csrc tools/mb_nntn.hip
#include "../trilinos_amd/csrc/icgs.hip"

#include <cstdio>
#include <initializer_list>
#ifndef LD_PAD
#define LD_PAD 0
#endif
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main() {
  using namespace migmres;
  const long long n = 1LL << 24;
  const long long ld = n + LD_PAD;
#ifndef MB_K
#define MB_K 8
#endif
  const int k = MB_K, Lmax = MB_K > 8 ? 352 : 216;
  double *V, *P, *R;
  CK(hipMalloc(&V, sizeof(double) * ld * Lmax));
  CK(hipMalloc(&P, sizeof(double) * 2048 * 256 * 16));
  CK(hipMalloc(&R, sizeof(double) * 512 * 16));
  double *SINK;
  CK(hipMalloc(&SINK, sizeof(double) * 256 * 4096));
  CK(hipMemset(V, 0, sizeof(double) * ld * Lmax));
  CK(hipMemset(R, 0, sizeof(double) * 512 * 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int L : (MB_K > 8 ? std::initializer_list<int>{160, 208, 256, 320} : std::initializer_list<int>{64, 104, 200})) {
    MvDesc Q{V, ld, nullptr, L};
    MvDesc X{V + (long long)L * ld, ld, nullptr, k};
    const int nb = nn_tn_blocks((int)n, L, k);
    launch_nn_tn(0, Q, L, R, L + k, X, (int)n, P, nb, SINK, k <= 8);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < 5; ++i) launch_nn_tn(0, Q, L, R, L + k, X, (int)n, P, nb, SINK, k <= 8);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 5;
    printf("k=%d pad %d mask %2d L=%3d nn_tn %7.3f ms %6.0f GB/s (%d wg)\n", k, (int)LD_PAD, NT_DIAG_MASK, L, ms, 8.0 * n * (L + 2 * k) / ms / 1e6, nb);
  }
  return 0;
}
