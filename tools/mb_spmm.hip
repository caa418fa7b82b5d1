// SpMM x8 variants on the 256^3 7-point Laplacian (CSR, column-major X/Y with ld = n
// rounded to 64).  Bytes = 12 nnz + 4 (n + 1) + 16 n k.  Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

// V0: library kernel shape (thread per row, 8 entries per batch, 8 columns)
template <bool XCD>
__global__ __launch_bounds__(256) void v0(const int *__restrict__ rp, const int *__restrict__ ci,
                                          const double *__restrict__ vv, const double *__restrict__ X, long long ld,
                                          double *__restrict__ Y, int n) {
#pragma clang fp contract(off)
  int b = blockIdx.x;
  if (XCD) {  // contiguous row slabs per XCD (workgroups go round-robin over the 8 XCDs)
    const int nb = gridDim.x, per = (nb + 7) / 8;
    const int x = b & 7, i = b >> 3;
    b = x * per + i;
    if (b >= nb) return;
  }
  const int r = b * 256 + threadIdx.x;
  if (r >= n) return;
  double sum[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) sum[c] = 0.0;
  const int e0 = rp[r], e1 = rp[r + 1];
  for (int eb = e0; eb < e1; eb += 8) {
    int col[8];
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = (eb + j < e1) ? eb + j : e0;
      col[j] = ci[e];
      v[j] = vv[e];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = eb + j < e1;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const double p = v[j] * X[c * ld + col[j]];
        sum[c] = sum[c] + (ok ? p : 0.0);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) Y[c * ld + r] = sum[c];
}

// V2: CSR of the workgroup's 256 rows staged in LDS with 16-B loads; thread per row.
template <int MAXE>
__global__ __launch_bounds__(256) void v2(const int *__restrict__ rp, const int *__restrict__ ci,
                                          const double *__restrict__ vv, const double *__restrict__ X, long long ld,
                                          double *__restrict__ Y, int n) {
#pragma clang fp contract(off)
  __shared__ int scol[256 * MAXE + 8];
  __shared__ double sval[256 * MAXE + 4];
  const int r0 = blockIdx.x * 256;
  const int r = r0 + threadIdx.x;
  const int rend = min(r0 + 256, n);
  const int E0 = rp[r0], E1 = rp[rend];
  const int a0 = E0 & ~3;  // 16-B aligned start for both arrays (ints: 4, doubles: 2 per 16 B)
  const int cnt = E1 - a0;
  for (int e = threadIdx.x * 4; e < cnt; e += 1024) {
    if (e + 4 <= cnt + 3) {
      const int4 cc = *(const int4 *)(ci + a0 + e);
      scol[e] = cc.x; scol[e + 1] = cc.y; scol[e + 2] = cc.z; scol[e + 3] = cc.w;
    }
  }
  for (int e = threadIdx.x * 2; e < cnt; e += 512) {
    const d2 w = *(const d2 *)(vv + a0 + e);
    sval[e] = w.x; sval[e + 1] = w.y;
  }
  __syncthreads();
  if (r >= n) return;
  double sum[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) sum[c] = 0.0;
  const int e0 = rp[r] - a0, e1 = rp[r + 1] - a0;
  for (int eb = e0; eb < e1; eb += 8) {
    int col[8];
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = (eb + j < e1) ? eb + j : e0;
      col[j] = scol[e];
      v[j] = sval[e];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = eb + j < e1;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const double p = v[j] * X[c * ld + col[j]];
        sum[c] = sum[c] + (ok ? p : 0.0);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) Y[c * ld + r] = sum[c];
}

// V3: two rows per thread (rows 2t, 2t+1 of the block), 16-B Y stores.
__global__ __launch_bounds__(256) void v3(const int *__restrict__ rp, const int *__restrict__ ci,
                                          const double *__restrict__ vv, const double *__restrict__ X, long long ld,
                                          double *__restrict__ Y, int n) {
#pragma clang fp contract(off)
  const int r = 2 * (blockIdx.x * 256 + threadIdx.x);
  if (r >= n) return;
  double s0[8], s1[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) s0[c] = s1[c] = 0.0;
  const int e0 = rp[r], e1 = rp[r + 1], e2 = rp[r + 2];
  // both rows in lockstep batches of 8 entries
  const int n0 = e1 - e0, n1 = e2 - e1, nmax = n0 > n1 ? n0 : n1;
  for (int b = 0; b < nmax; b += 8) {
    int c0[8], c1[8];
    double v0_[8], v1_[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ea = (b + j < n0) ? e0 + b + j : e0;
      const int eb = (b + j < n1) ? e1 + b + j : e1;
      c0[j] = ci[ea]; v0_[j] = vv[ea];
      c1[j] = ci[eb]; v1_[j] = vv[eb];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok0 = b + j < n0, ok1 = b + j < n1;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const double p0 = v0_[j] * X[c * ld + c0[j]];
        const double p1 = v1_[j] * X[c * ld + c1[j]];
        s0[c] = s0[c] + (ok0 ? p0 : 0.0);
        s1[c] = s1[c] + (ok1 ? p1 : 0.0);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) *(d2 *)(Y + c * ld + r) = d2{s0[c], s1[c]};
}

// V4: 8 lanes per row (lane = entry slot), products transposed through LDS so lane c
// sums column c's products in stored order.  Rows with > 8 entries loop with carry.
__global__ __launch_bounds__(256) void v4(const int *__restrict__ rp, const int *__restrict__ ci,
                                          const double *__restrict__ vv, const double *__restrict__ X, long long ld,
                                          double *__restrict__ Y, int n) {
#pragma clang fp contract(off)
  __shared__ double pr[32][8][9];  // [row in block][entry][column] (+1 pad)
  const int lane8 = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int r = blockIdx.x * 32 + rl;
  const bool live = r < n;
  const int e0 = live ? rp[r] : 0, e1 = live ? rp[r + 1] : 0;
  double sum = 0.0;  // lane8 = column c
  for (int eb = e0; eb < e1 || eb == e0; eb += 8) {
    const int e = eb + lane8;
    const bool ok = e < e1;
    const int col = ci[ok ? e : e0];
    const double v = vv[ok ? e : e0];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const double p = v * X[c * ld + col];
      pr[rl][lane8][c] = ok ? p : 0.0;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 8; ++j) sum = sum + pr[rl][j][lane8];
    __builtin_amdgcn_wave_barrier();
    if (e1 - eb <= 8) break;
  }
  if (live) Y[lane8 * ld + r] = sum;
}


// V5: diagnostic - same loads as v0 but every x read is X[c][r] (coalesced, no gather)
template <int MODE>
__global__ __launch_bounds__(256) void v5(const int *__restrict__ rp, const int *__restrict__ ci,
                                          const double *__restrict__ vv, const double *__restrict__ X, long long ld,
                                          double *__restrict__ Y, int n) {
#pragma clang fp contract(off)
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  double sum[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) sum[c] = 0.0;
  const int e0 = rp[r], e1 = rp[r + 1];
  for (int eb = e0; eb < e1; eb += 8) {
    int col[8];
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = (eb + j < e1) ? eb + j : e0;
      col[j] = ci[e];
      v[j] = vv[e];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = eb + j < e1;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        double p;
        if (MODE == 0) p = v[j] * X[c * ld + (r ^ (col[j] & 1))];  // coalesced, 56 loads (r^1 < n: n even)
        else if (MODE == 1) p = v[j] * (double)col[j];            // no X loads at all
        else p = v[j] * X[c * ld + (j == 0 ? r : col[j])];          // (unused)
        sum[c] = sum[c] + (ok ? p : 0.0);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) Y[c * ld + r] = sum[c];
}

// V6: diagnostic of 16-B X loads: rows (r, r+1) of an interior 7-point stencil share 7
// aligned pairs per column (timing only; boundary rows are wrong).
__global__ __launch_bounds__(256) void v6(const int *__restrict__ rp, const int *__restrict__ ci,
                                          const double *__restrict__ vv, const double *__restrict__ X, long long ld,
                                          double *__restrict__ Y, int n, int m) {
#pragma clang fp contract(off)
  const int r = 2 * (blockIdx.x * 256 + threadIdx.x);
  if (r >= n) return;
  const long long m2 = (long long)m * m;
  long long pc[7] = {r - m2, r - m, r - 2, r, r + 2, r + m, r + m2};
#pragma unroll
  for (int i = 0; i < 7; ++i) pc[i] = pc[i] < 0 ? 0 : (pc[i] >= n ? n - 2 : pc[i]);
  const int e0 = rp[r];
  double v0[7], v1[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) { v0[i] = vv[e0 + i]; v1[i] = vv[e0 + 7 + i]; }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    d2 x[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) x[i] = *(const d2 *)(X + c * ld + pc[i]);
    double s0 = 0.0, s1 = 0.0;
    s0 = s0 + v0[0] * x[0].x; s0 = s0 + v0[1] * x[1].x; s0 = s0 + v0[2] * x[2].y; s0 = s0 + v0[3] * x[3].x;
    s0 = s0 + v0[4] * x[3].y; s0 = s0 + v0[5] * x[5].x; s0 = s0 + v0[6] * x[6].x;
    s1 = s1 + v1[0] * x[0].y; s1 = s1 + v1[1] * x[1].y; s1 = s1 + v1[2] * x[3].x; s1 = s1 + v1[3] * x[3].y;
    s1 = s1 + v1[4] * x[4].x; s1 = s1 + v1[5] * x[5].y; s1 = s1 + v1[6] * x[6].y;
    *(d2 *)(Y + c * ld + r) = d2{s0, s1};
  }
}

int main(int argc, char **argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 256;
  const long long n = (long long)m * m * m;
  const long long ld = (n + 63) / 64 * 64;
  std::vector<int> rp(n + 1), ci;
  std::vector<double> vv;
  ci.reserve(n * 7 + 8);
  vv.reserve(n * 7 + 8);
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
  const long long nnz = ci.size();
  for (int i = 0; i < 8; ++i) { ci.push_back(0); vv.push_back(0); }  // tail pad for 16-B loads
  int *drp, *dci;
  double *dvv, *X, *Y, *Yref;
  CK(hipMalloc(&drp, sizeof(int) * (n + 1)));
  CK(hipMalloc(&dci, sizeof(int) * ci.size()));
  CK(hipMalloc(&dvv, sizeof(double) * vv.size()));
  CK(hipMalloc(&X, sizeof(double) * ld * 8));
  CK(hipMalloc(&Y, sizeof(double) * ld * 8));
  CK(hipMalloc(&Yref, sizeof(double) * ld * 8));
  CK(hipMemcpy(drp, rp.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(dci, ci.data(), sizeof(int) * ci.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dvv, vv.data(), sizeof(double) * vv.size(), hipMemcpyHostToDevice));
  {
    std::vector<double> hx(ld * 8);
    unsigned long long s = 88172645463325252ULL;
    for (auto &v : hx) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; v = (double)(s % 1000003) / 1000003.0 - 0.5; }
    CK(hipMemcpy(X, hx.data(), sizeof(double) * hx.size(), hipMemcpyHostToDevice));
  }
  const double bytes = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n * 8;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timeit = [&](const char *name, auto launch) {
    CK(hipMemset(Y, 0, sizeof(double) * ld * 8));
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < 10; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 10;
    std::vector<double> y(ld * 8), yr(ld * 8);
    CK(hipMemcpy(y.data(), Y, sizeof(double) * ld * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(yr.data(), Yref, sizeof(double) * ld * 8, hipMemcpyDeviceToHost));
    long long bad = 0;
    for (int c = 0; c < 8; ++c)
      bad += memcmp(y.data() + c * ld, yr.data() + c * ld, sizeof(double) * n) != 0;
    printf("%-28s %7.3f ms %6.0f GB/s  %s\n", name, ms, bytes / ms / 1e6, bad ? "MISMATCH" : "bit-exact");
  };
  const int nb = (int)((n + 255) / 256);
  v0<false><<<nb, 256>>>(drp, dci, dvv, X, ld, Yref, (int)n);
  CK(hipDeviceSynchronize());
  timeit("v0 thread/row", [&] { v0<false><<<nb, 256>>>(drp, dci, dvv, X, ld, Y, (int)n); });
  timeit("v0 + XCD slabs", [&] { v0<true><<<nb, 256>>>(drp, dci, dvv, X, ld, Y, (int)n); });
  timeit("v2 CSR in LDS", [&] { v2<8><<<nb, 256>>>(drp, dci, dvv, X, ld, Y, (int)n); });
  timeit("v3 2 rows/thread", [&] { v3<<<(int)((n / 2 + 255) / 256), 256>>>(drp, dci, dvv, X, ld, Y, (int)n); });
  timeit("v5 diag: X[c][r] loads", [&] { v5<0><<<nb, 256>>>(drp, dci, dvv, X, ld, Y, (int)n); });
  timeit("v5 diag: no X loads", [&] { v5<1><<<nb, 256>>>(drp, dci, dvv, X, ld, Y, (int)n); });
  timeit("v6 diag: 16-B pair loads", [&] { v6<<<(int)((n / 2 + 255) / 256), 256>>>(drp, dci, dvv, X, ld, Y, (int)n, m); });
  timeit("v4 8 lanes/row", [&] { v4<<<(int)((n + 31) / 32), 256>>>(drp, dci, dvv, X, ld, Y, (int)n); });
  return 0;
}
