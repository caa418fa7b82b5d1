// SpMM x8 variants on the 27-point Brick3D stencil (config 5's operator), n = nx^3, column-
// major X/Y with ld = n rounded to 64 + 64.  Algorithmic bytes = 12 nnz + 4 (n + 1) + 16 n k.
// Not part of the library: a measurement tool for choosing the general-row SpMM kernel.
//   A   SELL-64 thread per row (the library's k_spmm_sell)
//   AX  A with contiguous row slabs per XCD
//   B   thread per row pair: keys = aligned row pairs of X (16-B loads shared by both rows),
//       per key 4 coefficients (row0 lo/hi, row1 lo/hi) and a 4-bit use mask, SELL-64 layout
//   BX  B with contiguous pair slabs per XCD
// usage: mb_spmm27 [nx]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);                \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int xcd_block(int b, int nb) {
  const int per = (nb + 7) / 8;
  return (b & 7) * per + (b >> 3);
}

template <bool XCD>
__global__ __launch_bounds__(256) void kA(const long long *__restrict__ off, const int *__restrict__ len,
                                          const int *__restrict__ sc, const double *__restrict__ sv,
                                          const double *__restrict__ X, long long ld, double *__restrict__ Y, int n) {
#pragma clang fp contract(off)
  int b = blockIdx.x;
  if (XCD) b = xcd_block(b, gridDim.x);
  const int r = b * 256 + threadIdx.x;
  if (r >= n) return;
  double sum[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) sum[c] = 0.0;
  const long long base = off[r >> 6] + (r & 63);
  const int L = len[r];
  for (int sb = 0; sb < L; sb += 8) {
    int ci[8];
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long long e = base + (long long)((sb + j < L) ? sb + j : L - 1) * 64;
      ci[j] = sc[e];
      v[j] = sv[e];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = sb + j < L;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const double p = v[j] * X[c * ld + ci[j]];
        sum[c] = sum[c] + (ok ? p : 0.0);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) Y[c * ld + r] = sum[c];
}

// A with J entries' x loads (J x 8 columns) issued together before they are consumed
// (an empty asm with a memory clobber keeps the compiler from interleaving load/wait/use).
template <int J, bool XCD>
__global__ __launch_bounds__(256) void kAJ(const long long *__restrict__ off, const int *__restrict__ len,
                                           const int *__restrict__ sc, const double *__restrict__ sv,
                                           const double *__restrict__ X, long long ld, double *__restrict__ Y, int n) {
#pragma clang fp contract(off)
  int b = blockIdx.x;
  if (XCD) b = xcd_block(b, gridDim.x);
  const int r = b * 256 + threadIdx.x;
  if (r >= n) return;
  double sum[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) sum[c] = 0.0;
  const long long base = off[r >> 6] + (r & 63);
  const int L = len[r];
  for (int sb = 0; sb < L; sb += 8) {
    int ci[8];
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long long e = base + (long long)((sb + j < L) ? sb + j : L - 1) * 64;
      ci[j] = sc[e];
      v[j] = sv[e];
    }
#pragma unroll
    for (int j0 = 0; j0 < 8; j0 += J) {
      double xv[J][8];
#pragma unroll
      for (int j = 0; j < J; ++j)
#pragma unroll
        for (int c = 0; c < 8; ++c) xv[j][c] = X[c * ld + ci[j0 + j]];
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const bool ok = sb + j0 + j < L;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const double p = v[j0 + j] * xv[j][c];
          sum[c] = sum[c] + (ok ? p : 0.0);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) Y[c * ld + r] = sum[c];
}

// B: pair p = rows (2p, 2p+1); slot u of chunk ch: key[(ch*maxk+u)*64+lane] (pair index of X),
// c0/c1[(...)] = (lo, hi) coefficients of row 0 / row 1, m = use bits (1 r0lo, 2 r0hi, 4 r1lo, 8 r1hi).
template <bool XCD>
__global__ __launch_bounds__(256) void kB(int npairs, int maxk, const int *__restrict__ nk,
                                          const int *__restrict__ key, const d2 *__restrict__ c0,
                                          const d2 *__restrict__ c1, const unsigned char *__restrict__ msk,
                                          const double *__restrict__ X, long long ld, double *__restrict__ Y) {
#pragma clang fp contract(off)
  int b = blockIdx.x;
  if (XCD) b = xcd_block(b, gridDim.x);
  const int p = b * 256 + threadIdx.x;
  if (p >= npairs) return;
  double s0[8], s1[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) s0[c] = s1[c] = 0.0;
  const long long base = (long long)(p >> 6) * maxk * 64 + (p & 63);
  const int K = nk[p];
  for (int ub = 0; ub < K; ub += 4) {
    int kk[4];
    d2 a[4], bb[4];
    unsigned m[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long e = base + (long long)((ub + j < K) ? ub + j : K - 1) * 64;
      kk[j] = key[e];
      a[j] = c0[e];
      bb[j] = c1[e];
      m[j] = (ub + j < K) ? msk[e] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const d2 x = *(const d2 *)(X + c * ld + 2LL * kk[j]);
        const double p0 = a[j].x * x.x, p1 = a[j].y * x.y, q0 = bb[j].x * x.x, q1 = bb[j].y * x.y;
        s0[c] = s0[c] + ((m[j] & 1u) ? p0 : 0.0);
        s0[c] = s0[c] + ((m[j] & 2u) ? p1 : 0.0);
        s1[c] = s1[c] + ((m[j] & 4u) ? q0 : 0.0);
        s1[c] = s1[c] + ((m[j] & 8u) ? q1 : 0.0);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) *(d2 *)(Y + c * ld + 2LL * p) = d2{s0[c], s1[c]};
}

int main(int argc, char **argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 256;
  const long long n = (long long)m * m * m;
  const long long ld = (n + 63) / 64 * 64 + 64;
  const int K = 8;
  auto t0 = std::chrono::steady_clock::now();
  // CSR (sorted columns), Brick3D: -1 off-diagonal, 26 diagonal, Dirichlet truncation
  std::vector<long long> rp(n + 1, 0);
  std::vector<int> ci;
  std::vector<double> vv;
  ci.reserve((size_t)n * 27);
  vv.reserve((size_t)n * 27);
  const long long mm = (long long)m * m;
  for (long long r = 0; r < n; ++r) {
    const long long iz = r / mm, iy = (r % mm) / m, ix = r % m;
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          if (ix + dx < 0 || ix + dx >= m || iy + dy < 0 || iy + dy >= m || iz + dz < 0 || iz + dz >= m) continue;
          ci.push_back((int)(r + dx + dy * m + dz * mm));
          vv.push_back(dx == 0 && dy == 0 && dz == 0 ? 26.0 : -1.0 - 1e-3 * ((r + dx) % 7));
        }
    rp[r + 1] = (long long)ci.size();
  }
  const long long nnz = rp[n];
  // SELL-64
  const long long nch = (n + 63) / 64;
  std::vector<long long> off(nch + 1, 0);
  std::vector<int> len(n);
  for (long long c = 0; c < nch; ++c) {
    int w = 0;
    for (long long r = 64 * c; r < std::min(n, 64 * c + 64); ++r) {
      len[r] = (int)(rp[r + 1] - rp[r]);
      w = std::max(w, len[r]);
    }
    off[c + 1] = off[c] + (long long)w * 64;
  }
  std::vector<int> sc(off[nch], 0);
  std::vector<double> sv(off[nch], 0.0);
  for (long long r = 0; r < n; ++r)
    for (int s = 0; s < len[r]; ++s) {
      const long long at = off[r >> 6] + (long long)s * 64 + (r & 63);
      sc[at] = ci[rp[r] + s];
      sv[at] = vv[rp[r] + s];
    }
  // pair plan
  const long long np = (n + 1) / 2;
  std::vector<int> nk(np);
  int maxk = 0;
  std::vector<std::vector<int>> pk(1);
  for (long long p = 0; p < np; ++p) {
    std::vector<int> ks;
    for (int h = 0; h < 2; ++h) {
      const long long r = 2 * p + h;
      if (r >= n) continue;
      for (long long e = rp[r]; e < rp[r + 1]; ++e) ks.push_back(ci[e] >> 1);
    }
    std::sort(ks.begin(), ks.end());
    ks.erase(std::unique(ks.begin(), ks.end()), ks.end());
    nk[p] = (int)ks.size();
    maxk = std::max(maxk, nk[p]);
  }
  const long long pslots = (np + 63) / 64 * 64 * maxk;
  std::vector<int> key(pslots, 0);
  std::vector<d2> c0(pslots, d2{0, 0}), c1(pslots, d2{0, 0});
  std::vector<unsigned char> msk(pslots, 0);
  for (long long p = 0; p < np; ++p) {
    std::vector<int> ks;
    for (int h = 0; h < 2; ++h) {
      const long long r = 2 * p + h;
      if (r >= n) continue;
      for (long long e = rp[r]; e < rp[r + 1]; ++e) ks.push_back(ci[e] >> 1);
    }
    std::sort(ks.begin(), ks.end());
    ks.erase(std::unique(ks.begin(), ks.end()), ks.end());
    for (size_t u = 0; u < ks.size(); ++u) {
      const long long at = ((p >> 6) * maxk + (long long)u) * 64 + (p & 63);
      key[at] = ks[u];
      for (int h = 0; h < 2; ++h) {
        const long long r = 2 * p + h;
        if (r >= n) continue;
        for (long long e = rp[r]; e < rp[r + 1]; ++e)
          if ((ci[e] >> 1) == ks[u]) {
            const int hi = ci[e] & 1;
            d2 &q = h == 0 ? c0[at] : c1[at];
            if (hi)
              q.y = vv[e];
            else
              q.x = vv[e];
            msk[at] |= (unsigned char)(1u << (2 * h + hi));
          }
      }
    }
  }
  printf("n=%lld nnz=%lld maxk=%d host build %.1f s\n", n, nnz, maxk,
         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  // device
  long long *doff;
  int *dlen, *dsc, *dnk, *dkey;
  double *dsv, *dX, *dY, *dY2;
  d2 *dc0, *dc1;
  unsigned char *dm;
  CK(hipMalloc(&doff, sizeof(long long) * off.size()));
  CK(hipMalloc(&dlen, sizeof(int) * n));
  CK(hipMalloc(&dsc, sizeof(int) * sc.size()));
  CK(hipMalloc(&dsv, sizeof(double) * sv.size()));
  CK(hipMalloc(&dnk, sizeof(int) * np));
  CK(hipMalloc(&dkey, sizeof(int) * pslots));
  CK(hipMalloc(&dc0, sizeof(d2) * pslots));
  CK(hipMalloc(&dc1, sizeof(d2) * pslots));
  CK(hipMalloc(&dm, pslots));
  CK(hipMalloc(&dX, sizeof(double) * ld * K));
  CK(hipMalloc(&dY, sizeof(double) * ld * K));
  CK(hipMalloc(&dY2, sizeof(double) * ld * K));
  CK(hipMemcpy(doff, off.data(), sizeof(long long) * off.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dlen, len.data(), sizeof(int) * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsc, sc.data(), sizeof(int) * sc.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dsv, sv.data(), sizeof(double) * sv.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dnk, nk.data(), sizeof(int) * np, hipMemcpyHostToDevice));
  CK(hipMemcpy(dkey, key.data(), sizeof(int) * pslots, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc0, c0.data(), sizeof(d2) * pslots, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc1, c1.data(), sizeof(d2) * pslots, hipMemcpyHostToDevice));
  CK(hipMemcpy(dm, msk.data(), pslots, hipMemcpyHostToDevice));
  {
    std::vector<double> hx((size_t)ld * K, 0.0);
    for (int c = 0; c < K; ++c)
      for (long long r = 0; r < n; ++r) hx[c * ld + r] = std::sin(0.001 * r + c) + 0.5;
    CK(hipMemcpy(dX, hx.data(), sizeof(double) * hx.size(), hipMemcpyHostToDevice));
  }
  const double bytes = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n * K;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, auto launch, double *out) {
    launch(out);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch(out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-4s %.3f ms  %6.0f GB/s (algorithmic)\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  const int gA = (int)((n + 255) / 256), gB = (int)((np + 255) / 256);
  timeit("A", [&](double *o) { kA<false><<<gA, 256>>>(doff, dlen, dsc, dsv, dX, ld, o, (int)n); }, dY);
  timeit("AX", [&](double *o) { kA<true><<<gA, 256>>>(doff, dlen, dsc, dsv, dX, ld, o, (int)n); }, dY2);
  auto cmp = [&](const char *name) {
    std::vector<double> a((size_t)ld * K), b((size_t)ld * K);
    CK(hipMemcpy(a.data(), dY, sizeof(double) * a.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), dY2, sizeof(double) * b.size(), hipMemcpyDeviceToHost));
    long long bad = 0;
    for (int c = 0; c < K; ++c)
      for (long long r = 0; r < n; ++r)
        if (a[c * ld + r] != b[c * ld + r]) ++bad;
    printf("  %s vs A: %lld mismatches\n", name, bad);
  };
  cmp("AX");
  CK(hipMemset(dY2, 0, sizeof(double) * ld * K));
  timeit("A1", [&](double *o) { kAJ<1, false><<<gA, 256>>>(doff, dlen, dsc, dsv, dX, ld, o, (int)n); }, dY2);
  cmp("A1");
  CK(hipMemset(dY2, 0, sizeof(double) * ld * K));
  timeit("A2", [&](double *o) { kAJ<2, false><<<gA, 256>>>(doff, dlen, dsc, dsv, dX, ld, o, (int)n); }, dY2);
  cmp("A2");
  CK(hipMemset(dY2, 0, sizeof(double) * ld * K));
  timeit("A4", [&](double *o) { kAJ<4, false><<<gA, 256>>>(doff, dlen, dsc, dsv, dX, ld, o, (int)n); }, dY2);
  cmp("A4");
  CK(hipMemset(dY2, 0, sizeof(double) * ld * K));
  timeit("A8", [&](double *o) { kAJ<8, false><<<gA, 256>>>(doff, dlen, dsc, dsv, dX, ld, o, (int)n); }, dY2);
  cmp("A8");
  CK(hipMemset(dY2, 0, sizeof(double) * ld * K));
  timeit("A2X", [&](double *o) { kAJ<2, true><<<gA, 256>>>(doff, dlen, dsc, dsv, dX, ld, o, (int)n); }, dY2);
  cmp("A2X");
  CK(hipMemset(dY2, 0, sizeof(double) * ld * K));
  timeit("B", [&](double *o) { kB<false><<<gB, 256>>>((int)np, maxk, dnk, dkey, dc0, dc1, dm, dX, ld, o); }, dY2);
  cmp("B");
  CK(hipMemset(dY2, 0, sizeof(double) * ld * K));
  timeit("BX", [&](double *o) { kB<true><<<gB, 256>>>((int)np, maxk, dnk, dkey, dc0, dc1, dm, dX, ld, o); }, dY2);
  cmp("BX");
  return 0;
}
