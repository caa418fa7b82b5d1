// Access-pattern probe for the fused update+projection: read an nrows x L column-major
// block in RW-row chunks (every thread 16-B loads, pure streaming, no LDS) with the chunk
// order grid-stride or contiguous per workgroup.  Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

template <int RW, int NT, bool CONTIG>
__global__ __launch_bounds__(NT) void k_stream(const double *__restrict__ Q, long long ld, int L, long long nrows,
                                              double *__restrict__ out) {
  constexpr int LPC = RW / 2;          // threads per column per chunk
  constexpr int CPI = NT / LPC;        // columns per pass
  const int t = threadIdx.x, lrow = 2 * (t % LPC), lcol = t / LPC;
  const long long nch = nrows / RW;
  long long c0, c1, step;
  if (CONTIG) { c0 = nch * blockIdx.x / gridDim.x; c1 = nch * (blockIdx.x + 1) / gridDim.x; step = 1; }
  else { c0 = blockIdx.x; c1 = nch; step = gridDim.x; }
  d2 acc = {0, 0};
  for (long long ch = c0; ch < c1; ch += step) {
    const double *b = Q + ch * RW + lrow;
    d2 v[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int col = lcol + CPI * m;
      v[m] = col < L ? *(const d2 *)(b + col * ld) : d2{0, 0};
    }
    for (int m0 = 8; m0 * CPI < L; m0 += 8) {
#pragma unroll
      for (int m = 0; m < 8; ++m) acc += v[m];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int col = lcol + CPI * (m0 + m);
        v[m] = col < L ? *(const d2 *)(b + col * ld) : d2{0, 0};
      }
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) acc += v[m];
  }
  if (acc.x == 1234.5) out[t] = acc.y;
}

template <int RW, int NT, bool CONTIG>
void run(const double *Q, long long ld, long long n, double *o, int wgcu) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int L : {64, 104, 200}) {
    const int grid = 256 * wgcu;
    k_stream<RW, NT, CONTIG><<<grid, NT>>>(Q, ld, L, n, o);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < 5; ++i) k_stream<RW, NT, CONTIG><<<grid, NT>>>(Q, ld, L, n, o);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 5;
    printf("RW=%3d NT=%4d %s wg/cu=%d L=%3d %7.3f ms %6.0f GB/s\n", RW, NT, CONTIG ? "contig" : "stride", wgcu, L, ms,
           8.0 * n * L / ms / 1e6);
  }
}

int main() {
  const long long n = 1LL << 24, ld = n + 64;
  double *Q, *o;
  CK(hipMalloc(&Q, sizeof(double) * ld * 216));
  CK(hipMalloc(&o, 8192));
  CK(hipMemset(Q, 0, sizeof(double) * ld * 216));
  run<16, 256, false>(Q, ld, n, o, 4);
  run<32, 512, false>(Q, ld, n, o, 2);
  run<32, 512, true>(Q, ld, n, o, 2);
  run<64, 512, false>(Q, ld, n, o, 2);
  run<64, 512, true>(Q, ld, n, o, 2);
  run<64, 1024, false>(Q, ld, n, o, 1);
  run<128, 512, false>(Q, ld, n, o, 2);
  run<128, 512, true>(Q, ld, n, o, 2);
  run<32, 256, false>(Q, ld, n, o, 4);
  run<32, 256, true>(Q, ld, n, o, 4);
  run<64, 256, false>(Q, ld, n, o, 4);
  return 0;
}
