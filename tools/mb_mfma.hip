// fp64 MFMA and VALU FMA throughput on one launch filling the chip (calibration for the
// ICGS kernels' compute budget).  Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ __launch_bounds__(256) void mfma_loop(double *out, int iters, double a0, double b0) {
  d4 acc[CH];
  for (int i = 0; i < CH; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = a0 + threadIdx.x, b = b0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < CH; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CH>
__global__ __launch_bounds__(256) void mfma4_loop(double *out, int iters, double a0, double b0) {
  double acc[CH];
  for (int i = 0; i < CH; ++i) acc[i] = 0;
  double a = a0 + threadIdx.x, b = b0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < CH; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// probe of the 4x4x4 f64 layout: lane l supplies a = A-code, b = B-code; output per lane
__global__ void probe4(double *out, int mode, int sel) {
  const int l = threadIdx.x;
  double a = 0, b = 0;
  if (mode == 0) { a = (l == sel) ? 1.0 : 0.0; b = 1.0; }
  else { a = 1.0; b = (l == sel) ? 1.0 : 0.0; }
  out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
}

template <int CH>
__global__ __launch_bounds__(256) void fma_loop(double *out, int iters, double a0, double b0) {
  double acc[CH];
  for (int i = 0; i < CH; ++i) acc[i] = i;
  double a = a0 + threadIdx.x, b = b0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) acc[i] = fma(a, acc[i], b);
  }
  double s = 0;
  for (int i = 0; i < CH; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class K>
float run(K k, int blocks, int iters, double *out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<<<blocks, 256>>>(out, iters, 1.0, 1e-9);
  hipEventRecord(e0);
  k<<<blocks, 256>>>(out, iters, 1.0, 1e-9);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  double *out;
  hipMalloc(&out, sizeof(double) * 4096 * 256);
  const int iters = 4000;
  for (int bpc : {1, 2, 4}) {
    const int blocks = 256 * bpc;
    float t1 = run(mfma_loop<1>, blocks, iters, out);
    float t4 = run(mfma_loop<4>, blocks, iters, out);
    const double n1 = (double)blocks * 4 * iters * 1, n4 = (double)blocks * 4 * iters * 4;
    printf("mfma f64 16x16x4: %d WG/CU  1 chain %.2f TF (%.0f clk/MFMA/SIMD)  4 chains %.2f TF (%.0f clk)\n", bpc,
           n1 * 2048 / t1 / 1e9, t1 * 1e-3 * 2.4e9 / (n1 / 1024), n4 * 2048 / t4 / 1e9, t4 * 1e-3 * 2.4e9 / (n4 / 1024));
    float m4 = run(mfma4_loop<8>, blocks, iters, out);
    const double n44 = (double)blocks * 4 * iters * 8;
    printf("mfma f64 4x4x4 (4 blocks): %d WG/CU  8 chains %.2f TF (%.0f clk/MFMA/SIMD)\n", bpc,
           n44 * 512 / m4 / 1e9, m4 * 1e-3 * 2.4e9 / (n44 / 1024));
    float f8 = run(fma_loop<8>, blocks, iters, out);
    const double nf = (double)blocks * 256 * iters * 8;
    printf("v_fma_f64: %d WG/CU  8 chains %.2f TF\n", bpc, nf * 2 / f8 / 1e9);
  }
  // layout probe: which output lanes does input lane `sel` reach (A side / B side)
  double *po;
  hipMalloc(&po, 64 * sizeof(double));
  double h[64];
  for (int mode = 0; mode < 2; ++mode)
    for (int sel : {0, 1, 2, 3, 4, 5, 15, 16, 17, 20, 32, 48}) {
      probe4<<<1, 64>>>(po, mode, sel);
      hipMemcpy(h, po, sizeof(h), hipMemcpyDeviceToHost);
      printf("%s lane %2d ->", mode ? "B" : "A", sel);
      for (int l = 0; l < 64; ++l) if (h[l] != 0.0) printf(" %d", l);
      printf("\n");
    }
  return 0;
}
