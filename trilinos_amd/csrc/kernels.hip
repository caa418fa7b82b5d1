// HIP/CDNA4 (gfx950) kernels for the Block GMRES hot path.
//
//  k_spmm       CSR SpMM x k  (Epetra_CrsMatrix::GeneralMM, epetra/src/Epetra_CrsMatrix.cpp:3486-3585;
//               KokkosSparse SPMV_MV_LayoutLeft_Functor, kokkos-kernels/src/sparse/impl/
//               KokkosSparse_spmv_impl.hpp:511-878)
//  k_gemm_tn    C = A^T B, tall-skinny inner products on fp64 MFMA 16x16x4 (MvTransMv ->
//               Epetra_MultiVector::Multiply('T','N'), Epetra_MultiVector.cpp:1936-2083)
//  k_gemm_nn    X = beta X + alpha A M (MvTimesMatAddMv -> Multiply('N','N'))
//  k_coldot     per-column dot / 1-norm / inf-norm (Epetra_MultiVector::Dot/Norm1/NormInf)
//  elementwise  Update / Scale / PutScalar / Random / pack for the Import exchange
//
// Layout: every multivector is column-major with an even leading dimension (rows padded
// to a multiple of 64), so a lane's 16-byte load of rows (2i, 2i+1) is aligned.
#include "internal.h"

namespace migmres {

typedef double d2 __attribute__((ext_vector_type(2)));
typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double *colp(const MvDesc &d, int c) {
  return d.base + (long long)(d.cols ? d.cols[c] : c) * d.ld;
}

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

#define LAUNCH_CHECK()                                                                      \
  do {                                                                                      \
    hipError_t e_ = hipGetLastError();                                                      \
    if (e_ != hipSuccess) throw Error(MIGMRES_EHIP, std::string("kernel launch: ") + hipGetErrorString(e_)); \
  } while (0)

// -------------------------------------------------------------------------------------
// SpMM x k: one thread per row, k accumulators, stored-order sums without FMA so the
// result is bit-identical to the reference's C loop (sum = 0; sum += v * x[col]).
// -------------------------------------------------------------------------------------
template <int KC>
__global__ __launch_bounds__(256) void k_spmm(int row_begin, int row_end,
                                              const int *__restrict__ rowptr,
                                              const int *__restrict__ cols,
                                              const double *__restrict__ vals, MvDesc X,
                                              int n_local, const double *__restrict__ ghost,
                                              long long ldg, MvDesc Y, int c0, int kc,
                                              double alpha, double beta) {
#pragma clang fp contract(off)
  const int r = row_begin + blockIdx.x * 256 + threadIdx.x;
  if (r >= row_end) return;
  const double *xc[KC];
  const double *gc[KC];
  double sum[KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    sum[c] = 0.0;
    if (c < kc) {
      xc[c] = colp(X, c0 + c);
      gc[c] = ghost + (long long)(c0 + c) * ldg;
    }
  }
  const int e0 = rowptr[r], e1 = rowptr[r + 1];
  for (int e = e0; e < e1; ++e) {
    const int col = cols[e];
    const double v = vals[e];
    if (col < n_local) {
#pragma unroll
      for (int c = 0; c < KC; ++c)
        if (c < kc) sum[c] = sum[c] + v * xc[c][col];
    } else {
      const int g = col - n_local;
#pragma unroll
      for (int c = 0; c < KC; ++c)
        if (c < kc) sum[c] = sum[c] + v * gc[c][g];
    }
  }
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    if (c < kc) {
      double *yp = colp(Y, c0 + c) + r;
      if (beta == 0.0)
        *yp = (alpha == 1.0) ? sum[c] : alpha * sum[c];
      else
        *yp = alpha * sum[c] + beta * (*yp);
    }
  }
}

void launch_spmm(hipStream_t s, int row_begin, int row_end, const int *rowptr, const int *cols,
                 const double *vals, MvDesc X, int n_local, const double *ghost, long long ldg,
                 MvDesc Y, double alpha, double beta) {
  const int n = row_end - row_begin;
  if (n <= 0) return;
  const int k = Y.ncols;
  const dim3 grid(cdiv(n, 256));
  for (int c0 = 0; c0 < k; c0 += 16) {
    const int kc = (k - c0) < 16 ? (k - c0) : 16;
    if (kc == 1)
      k_spmm<1><<<grid, 256, 0, s>>>(row_begin, row_end, rowptr, cols, vals, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta);
    else if (kc <= 2)
      k_spmm<2><<<grid, 256, 0, s>>>(row_begin, row_end, rowptr, cols, vals, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta);
    else if (kc <= 4)
      k_spmm<4><<<grid, 256, 0, s>>>(row_begin, row_end, rowptr, cols, vals, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta);
    else if (kc <= 8)
      k_spmm<8><<<grid, 256, 0, s>>>(row_begin, row_end, rowptr, cols, vals, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta);
    else
      k_spmm<16><<<grid, 256, 0, s>>>(row_begin, row_end, rowptr, cols, vals, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta);
    LAUNCH_CHECK();
  }
}

// -------------------------------------------------------------------------------------
// C = A^T B (A: nrows x L, B: nrows x kb <= 16) on v_mfma_f64_16x16x4_f64.
// MFMA M = 16 columns of A, N = 16 columns of B, K = 4 rows per instruction; the row
// reduction happens inside the matrix core.  A workgroup streams 64-row tiles: B tile
// (64x16) and A column groups (64 rows x 64 cols, 8 coalesced dwordx4 loads per thread,
// each wave-instruction = 2 full 512-B column segments) are staged through LDS; wave w
// owns column tile w of each 64-column group.  Per-workgroup partials are summed by
// k_reduce in a fixed order.
// f64 MFMA lane maps: A[i=l&15][k=l>>4], B[k=l>>4][j=l&15], D[row=(l>>4)+4r][col=l&15].
// -------------------------------------------------------------------------------------
constexpr int TN_ROWS = 64;
constexpr int TN_APITCH = 66;  // doubles; 66 = 2 mod 32 -> conflict-free ds_read_b64

template <int MAXG>
__global__ __launch_bounds__(256) void k_gemm_tn(MvDesc A, int L, MvDesc B, int kb, int nrows,
                                                 double *__restrict__ partial) {
  __shared__ __attribute__((aligned(16))) double As[64 * TN_APITCH];
  __shared__ __attribute__((aligned(16))) double Bs[TN_ROWS * 16];
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int ngroups = (L + 63) >> 6;
  d4 acc[MAXG];
#pragma unroll
  for (int g = 0; g < MAXG; ++g) acc[g] = d4{0.0, 0.0, 0.0, 0.0};

  for (long long rt = blockIdx.x; rt * TN_ROWS < nrows; rt += gridDim.x) {
    const long long r0 = rt * TN_ROWS;
    const bool full = r0 + TN_ROWS <= nrows;
    {  // stage B: thread -> column j = t>>4, rows 4*(t&15) .. +3
      const int j = t >> 4, rr = (t & 15) * 4;
      double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
      if (j < kb) {
        const double *bp = colp(B, j) + r0 + rr;
        if (full) {
          const d2 p = *(const d2 *)bp, q = *(const d2 *)(bp + 2);
          v0 = p.x; v1 = p.y; v2 = q.x; v3 = q.y;
        } else {
          v0 = (r0 + rr + 0 < nrows) ? bp[0] : 0.0;
          v1 = (r0 + rr + 1 < nrows) ? bp[1] : 0.0;
          v2 = (r0 + rr + 2 < nrows) ? bp[2] : 0.0;
          v3 = (r0 + rr + 3 < nrows) ? bp[3] : 0.0;
        }
      }
      Bs[(rr + 0) * 16 + j] = v0;
      Bs[(rr + 1) * 16 + j] = v1;
      Bs[(rr + 2) * 16 + j] = v2;
      Bs[(rr + 3) * 16 + j] = v3;
    }
#pragma unroll
    for (int g = 0; g < MAXG; ++g) {
      if (g < ngroups) {
        d2 v[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const int cl = 8 * s + (t >> 5);
          const int cg = g * 64 + cl;
          const int rr = 2 * (t & 31);
          v[s] = d2{0.0, 0.0};
          if (cg < L) {
            const double *ap = colp(A, cg) + r0 + rr;
            if (full) {
              v[s] = *(const d2 *)ap;
            } else {
              v[s].x = (r0 + rr < nrows) ? ap[0] : 0.0;
              v[s].y = (r0 + rr + 1 < nrows) ? ap[1] : 0.0;
            }
          }
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const int cl = 8 * s + (t >> 5);
          *(d2 *)&As[cl * TN_APITCH + 2 * (t & 31)] = v[s];
        }
        __syncthreads();
        if (g * 64 + 16 * w < L) {
#pragma unroll
          for (int q = 0; q < TN_ROWS / 4; ++q) {
            const double a = As[(16 * w + (l & 15)) * TN_APITCH + 4 * q + (l >> 4)];
            const double b = Bs[(4 * q + (l >> 4)) * 16 + (l & 15)];
            acc[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[g], 0, 0, 0);
          }
        }
        __syncthreads();
      }
    }
  }
  double *out = partial + (long long)blockIdx.x * L * kb;
  const int j = l & 15;
#pragma unroll
  for (int g = 0; g < MAXG; ++g) {
    if (g < ngroups && g * 64 + 16 * w < L && j < kb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = g * 64 + 16 * w + (l >> 4) + 4 * r;
        if (i < L) out[i + (long long)j * L] = acc[g][r];
      }
    }
  }
}

int gemm_tn_blocks(int nrows) {
  const int tiles = cdiv(nrows, TN_ROWS);
  return tiles < 1024 ? (tiles > 0 ? tiles : 1) : 1024;
}

void launch_gemm_tn_partial(hipStream_t s, MvDesc A, int L, MvDesc B, int kb, int nrows,
                            double *partial, int nblocks) {
  if (L > 512 || kb > 16) throw Error(MIGMRES_EINVAL, "gemm_tn: L <= 512 and kb <= 16 per launch");
  if (L <= 128)
    k_gemm_tn<2><<<nblocks, 256, 0, s>>>(A, L, B, kb, nrows, partial);
  else if (L <= 256)
    k_gemm_tn<4><<<nblocks, 256, 0, s>>>(A, L, B, kb, nrows, partial);
  else
    k_gemm_tn<8><<<nblocks, 256, 0, s>>>(A, L, B, kb, nrows, partial);
  LAUNCH_CHECK();
}

__global__ __launch_bounds__(256) void k_reduce(const double *__restrict__ partial, int nblocks,
                                                int nout, double alpha, double *__restrict__ out) {
  __shared__ double red[4][64];
  const int l = threadIdx.x & 63, s = threadIdx.x >> 6;
  const int o = blockIdx.x * 64 + l;
  double acc = 0.0;
  if (o < nout)
    for (int b = s; b < nblocks; b += 4) acc += partial[(long long)b * nout + o];
  red[s][l] = acc;
  __syncthreads();
  if (s == 0 && o < nout) out[o] = alpha * ((red[0][l] + red[1][l]) + (red[2][l] + red[3][l]));
}

void launch_reduce_partials(hipStream_t s, const double *partial, int nblocks, int nout,
                            double alpha, double *out) {
  if (nout <= 0) return;
  k_reduce<<<cdiv(nout, 64), 256, 0, s>>>(partial, nblocks, nout, alpha, out);
  LAUNCH_CHECK();
}

__global__ __launch_bounds__(256) void k_reduce_max(const double *__restrict__ partial,
                                                    int nblocks, int nout,
                                                    double *__restrict__ out) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= nout) return;
  double m = 0.0;
  for (int b = 0; b < nblocks; ++b) m = fmax(m, partial[(long long)b * nout + o]);
  out[o] = m;
}

void launch_reduce_max(hipStream_t s, const double *partial, int nblocks, int nout, double *out) {
  if (nout <= 0) return;
  k_reduce_max<<<cdiv(nout, 256), 256, 0, s>>>(partial, nblocks, nout, out);
  LAUNCH_CHECK();
}

// -------------------------------------------------------------------------------------
// X = beta X + alpha A M.  Two rows per thread (one 16-B load per column of A), the
// coefficient chunk (64 x KX) broadcast from LDS; A is streamed exactly once.
// -------------------------------------------------------------------------------------
template <int KX>
__global__ __launch_bounds__(256) void k_gemm_nn(MvDesc A, int L, const double *__restrict__ M,
                                                 int ldm, MvDesc X, int kx, int nrows,
                                                 double alpha, double beta) {
  __shared__ __attribute__((aligned(16))) double Ms[64 * KX];
  const long long r = 2LL * ((long long)blockIdx.x * 256 + threadIdx.x);
  double acc0[KX], acc1[KX];
#pragma unroll
  for (int c = 0; c < KX; ++c) acc0[c] = acc1[c] = 0.0;
  const bool two = r + 1 < nrows;
  for (int j0 = 0; j0 < L; j0 += 64) {
    const int jn = (L - j0) < 64 ? (L - j0) : 64;
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * KX; e += 256) {
      const int jj = e / KX, c = e % KX;
      Ms[e] = (jj < jn && c < kx) ? M[(j0 + jj) + (long long)c * ldm] : 0.0;
    }
    __syncthreads();
    if (r < nrows) {
#pragma unroll 4
      for (int jj = 0; jj < jn; ++jj) {
        const double *ap = colp(A, j0 + jj) + r;
        double a0, a1;
        if (two) {
          const d2 v = *(const d2 *)ap;
          a0 = v.x;
          a1 = v.y;
        } else {
          a0 = ap[0];
          a1 = 0.0;
        }
        const double *mrow = &Ms[jj * KX];
#pragma unroll
        for (int c = 0; c < KX; ++c) {
          acc0[c] += a0 * mrow[c];
          acc1[c] += a1 * mrow[c];
        }
      }
    }
  }
  if (r >= nrows) return;
#pragma unroll
  for (int c = 0; c < KX; ++c) {
    if (c < kx) {
      double *xp = colp(X, c) + r;
      if (beta == 0.0) {
        xp[0] = alpha * acc0[c];
        if (two) xp[1] = alpha * acc1[c];
      } else {
        xp[0] = beta * xp[0] + alpha * acc0[c];
        if (two) xp[1] = beta * xp[1] + alpha * acc1[c];
      }
    }
  }
}

void launch_gemm_nn(hipStream_t s, MvDesc A, int L, const double *M, int ldm, MvDesc X, int nrows,
                    double alpha, double beta) {
  if (nrows <= 0) return;
  const int kx = X.ncols;
  const dim3 grid(cdiv(nrows, 512));
  for (int c0 = 0; c0 < kx; c0 += 16) {
    const int kc = (kx - c0) < 16 ? (kx - c0) : 16;
    MvDesc Xc = X;
    Xc.ncols = kc;
    if (X.cols)
      Xc.cols = X.cols + c0;
    else
      Xc.base = X.base + (long long)c0 * X.ld;
    const double *Mc = M + (long long)c0 * ldm;
    if (kc <= 1)
      k_gemm_nn<1><<<grid, 256, 0, s>>>(A, L, Mc, ldm, Xc, kc, nrows, alpha, beta);
    else if (kc <= 2)
      k_gemm_nn<2><<<grid, 256, 0, s>>>(A, L, Mc, ldm, Xc, kc, nrows, alpha, beta);
    else if (kc <= 4)
      k_gemm_nn<4><<<grid, 256, 0, s>>>(A, L, Mc, ldm, Xc, kc, nrows, alpha, beta);
    else if (kc <= 8)
      k_gemm_nn<8><<<grid, 256, 0, s>>>(A, L, Mc, ldm, Xc, kc, nrows, alpha, beta);
    else
      k_gemm_nn<16><<<grid, 256, 0, s>>>(A, L, Mc, ldm, Xc, kc, nrows, alpha, beta);
    LAUNCH_CHECK();
  }
}

// -------------------------------------------------------------------------------------
// Per-column reductions (dot, sum|a|, max|a|), fixed-shape block tree -> partials.
// -------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_down(v, off, 64));
  return v;
}

template <int OP>
__global__ __launch_bounds__(256) void k_coldot(MvDesc A, MvDesc B, int nrows,
                                                double *__restrict__ partial) {
  __shared__ double red[4];
  const int k = A.ncols;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int c = 0; c < k; ++c) {
    const double *ap = colp(A, c);
    const double *bp = OP == 0 ? colp(B, c) : nullptr;
    double acc = 0.0;
    for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < nrows;
         r += (long long)gridDim.x * 256) {
      if (OP == 0) acc += ap[r] * bp[r];
      else if (OP == 1) acc += fabs(ap[r]);
      else acc = fmax(acc, fabs(ap[r]));
    }
    acc = OP == 2 ? wave_max(acc) : wave_sum(acc);
    if (l == 0) red[w] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      const double v = OP == 2 ? fmax(fmax(red[0], red[1]), fmax(red[2], red[3]))
                               : (red[0] + red[1]) + (red[2] + red[3]);
      partial[(long long)blockIdx.x * k + c] = v;
    }
    __syncthreads();
  }
}

int coldot_blocks(int nrows) {
  const int b = cdiv(nrows, 4096);
  return b < 1 ? 1 : (b > 1024 ? 1024 : b);
}

void launch_coldot_partial(hipStream_t s, MvDesc A, MvDesc B, int nrows, int op, double *partial,
                           int nblocks) {
  if (op == 0)
    k_coldot<0><<<nblocks, 256, 0, s>>>(A, B, nrows, partial);
  else if (op == 1)
    k_coldot<1><<<nblocks, 256, 0, s>>>(A, B, nrows, partial);
  else
    k_coldot<2><<<nblocks, 256, 0, s>>>(A, B, nrows, partial);
  LAUNCH_CHECK();
}

// -------------------------------------------------------------------------------------
// Elementwise column kernels: grid.y = column.
// -------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_axpby(double alpha, MvDesc A, double beta, MvDesc B,
                                               MvDesc Y, int nrows) {
  const int c = blockIdx.y;
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  colp(Y, c)[r] = alpha * colp(A, c)[r] + beta * colp(B, c)[r];
}

__global__ __launch_bounds__(256) void k_scale(MvDesc Y, int nrows, double alpha,
                                               const double *__restrict__ alphas) {
  const int c = blockIdx.y;
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  double *p = colp(Y, c) + r;
  *p = (alphas ? alphas[c] : alpha) * (*p);
}

__global__ __launch_bounds__(256) void k_fill(MvDesc Y, int nrows, double v) {
  const int c = blockIdx.y;
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r < nrows) colp(Y, c)[r] = v;
}

__global__ __launch_bounds__(256) void k_copy(MvDesc A, MvDesc Y, int nrows) {
  const int c = blockIdx.y;
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r < nrows) colp(Y, c)[r] = colp(A, c)[r];
}

// seed * 16807^e mod (2^31-1), e >= 1: the e-th Epetra_Util::RandomInt after `seed`.
__device__ __forceinline__ unsigned long long minstd_jump(unsigned long long seed,
                                                          unsigned long long e) {
  const unsigned long long m = 2147483647ULL;
  unsigned long long base = 16807ULL, acc = 1ULL;
  while (e) {
    if (e & 1ULL) acc = (acc * base) % m;
    base = (base * base) % m;
    e >>= 1;
  }
  return (seed * acc) % m;
}

__global__ __launch_bounds__(256) void k_random(MvDesc Y, int nrows, long long first,
                                                long long n_global, unsigned int seed) {
#pragma clang fp contract(off)
  const int c = blockIdx.y;
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  const unsigned long long p = (unsigned long long)c * (unsigned long long)n_global +
                               (unsigned long long)(first + r) + 1ULL;
  const double x = (double)minstd_jump(seed, p);
  colp(Y, c)[r] = 2.0 * (x / 2147483647.0) - 1.0;
}

__global__ __launch_bounds__(256) void k_pack(MvDesc X, const int *__restrict__ lids, int count,
                                              double *__restrict__ send) {
  const int c = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < count) send[(long long)c * count + i] = colp(X, c)[lids[i]];
}

void launch_axpby(hipStream_t s, double alpha, MvDesc A, double beta, MvDesc B, MvDesc Y, int nrows) {
  if (nrows <= 0 || Y.ncols <= 0) return;
  k_axpby<<<dim3(cdiv(nrows, 256), Y.ncols), 256, 0, s>>>(alpha, A, beta, B, Y, nrows);
  LAUNCH_CHECK();
}
void launch_scale(hipStream_t s, MvDesc Y, int nrows, double alpha, const double *alphas) {
  if (nrows <= 0 || Y.ncols <= 0) return;
  k_scale<<<dim3(cdiv(nrows, 256), Y.ncols), 256, 0, s>>>(Y, nrows, alpha, alphas);
  LAUNCH_CHECK();
}
void launch_fill(hipStream_t s, MvDesc Y, int nrows, double v) {
  if (nrows <= 0 || Y.ncols <= 0) return;
  k_fill<<<dim3(cdiv(nrows, 256), Y.ncols), 256, 0, s>>>(Y, nrows, v);
  LAUNCH_CHECK();
}
void launch_copy(hipStream_t s, MvDesc A, MvDesc Y, int nrows) {
  if (nrows <= 0 || Y.ncols <= 0) return;
  k_copy<<<dim3(cdiv(nrows, 256), Y.ncols), 256, 0, s>>>(A, Y, nrows);
  LAUNCH_CHECK();
}
void launch_random(hipStream_t s, MvDesc Y, int nrows, long long first, long long n_global,
                   unsigned int seed) {
  if (nrows <= 0 || Y.ncols <= 0) return;
  k_random<<<dim3(cdiv(nrows, 256), Y.ncols), 256, 0, s>>>(Y, nrows, first, n_global, seed);
  LAUNCH_CHECK();
}
void launch_pack(hipStream_t s, MvDesc X, const int *lids, int count, double *send, int k) {
  if (count <= 0 || k <= 0) return;
  k_pack<<<dim3(cdiv(count, 256), k), 256, 0, s>>>(X, lids, count, send);
  LAUNCH_CHECK();
}

}  // namespace migmres
