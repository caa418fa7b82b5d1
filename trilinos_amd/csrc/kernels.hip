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
                                              double alpha, double beta, const int *__restrict__ sel,
                                              int nsel, const double *__restrict__ cs,
                                              const double *__restrict__ gcs) {
#pragma clang fp contract(off)
  int r = row_begin + blockIdx.x * 256 + threadIdx.x;
  if (sel) {  // optional list of rows (interior / boundary split of the halo overlap)
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= nsel) return;
    r = sel[t];
  } else if (r >= row_end) {
    return;
  }
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
  // Entries in batches of 8: every index/value load and x-gather of a batch is issued
  // before the sums consume them.  An empty slot loads a valid address (the row's first
  // entry) and adds exactly +0.0, which leaves the stored-order sum unchanged (the sum
  // starts at +0.0 and can never become -0.0).
  for (int eb = e0; eb < e1; eb += 8) {
    int ci[8];
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = (eb + j < e1) ? eb + j : e0;
      ci[j] = cols[e];
      v[j] = vals[e];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = eb + j < e1;
      const int col = ci[j];
      const bool own = col < n_local;
      const int g = col - n_local;
      // fused right Jacobi: the operand (omega D^-1) x as k_jacobi forms it (ghost columns
      // scaled by their owner's omega d^-1, imported once)
      const double sc = cs ? (own ? cs[col] : gcs[g]) : 1.0;
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        if (c < kc) {
          double x = own ? xc[c][col] : gc[c][g];
          if (cs) x = sc * x;
          const double prod = v[j] * x;
          sum[c] = sum[c] + (ok ? prod : 0.0);
        }
      }
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
                 MvDesc Y, double alpha, double beta, const int *sel, int nsel, ColScale cs) {
  const int n = sel ? nsel : row_end - row_begin;
  if (n <= 0) return;
  const int k = Y.ncols;
  const dim3 grid(cdiv(n, 256));
  for (int c0 = 0; c0 < k; c0 += 16) {
    const int kc = (k - c0) < 16 ? (k - c0) : 16;
    if (kc == 1)
      k_spmm<1><<<grid, 256, 0, s>>>(row_begin, row_end, rowptr, cols, vals, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta, sel, nsel, cs.own, cs.ghost);
    else if (kc <= 2)
      k_spmm<2><<<grid, 256, 0, s>>>(row_begin, row_end, rowptr, cols, vals, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta, sel, nsel, cs.own, cs.ghost);
    else if (kc <= 4)
      k_spmm<4><<<grid, 256, 0, s>>>(row_begin, row_end, rowptr, cols, vals, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta, sel, nsel, cs.own, cs.ghost);
    else if (kc <= 8)
      k_spmm<8><<<grid, 256, 0, s>>>(row_begin, row_end, rowptr, cols, vals, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta, sel, nsel, cs.own, cs.ghost);
    else
      k_spmm<16><<<grid, 256, 0, s>>>(row_begin, row_end, rowptr, cols, vals, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta, sel, nsel, cs.own, cs.ghost);
    LAUNCH_CHECK();
  }
}

// -------------------------------------------------------------------------------------
// SpMM x k for rows too long for the row-pair plan (27-point stencils, unstructured
// matrices): one thread per row over a SELL-64 copy of the CSR (make_sell64), so each
// column-index / value load of a wave is one contiguous 256 / 512-byte segment.  Sums in
// stored order, products v * x, no FMA: bit-identical to k_spmm and the reference loop.
// -------------------------------------------------------------------------------------
// XR: the owned operands come from xr, a row-interleaved copy of X's columns c0 .. c0 + KC - 1
// (k_interleave): one entry's KC values are KC / 2 16-byte loads of one 8 KC-byte segment
// (one cache line) instead of KC 8-byte gathers from KC lines.  Same values, same order.
template <int KC, bool XR = false>
__global__ __launch_bounds__(256) void k_spmm_sell(int n, const long long *__restrict__ off,
                                                   const int *__restrict__ len, const int *__restrict__ scol,
                                                   const double *__restrict__ sval, MvDesc X, int n_local,
                                                   const double *__restrict__ ghost, long long ldg, MvDesc Y,
                                                   int c0, int kc, double alpha, double beta,
                                                   const int *__restrict__ sel, int nsel,
                                                   const double *__restrict__ xr, const double *__restrict__ cs,
                                                   const double *__restrict__ gcs) {
#pragma clang fp contract(off)
  // entries whose KC x loads are issued together (XR: KC / 2 16-byte loads per entry; 8
  // entries at a time there measured the same as 4 on FlanProxy)
  constexpr int J = KC >= 4 ? 4 : 8;
  const int t = blockIdx.x * 256 + threadIdx.x;
  int r;
  if (sel) {
    if (t >= nsel) return;
    r = sel[t];
  } else {
    if (t >= n) return;
    r = t;
  }
  const double *xc[KC];
  const double *gc[KC];
  double sum[KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    sum[c] = 0.0;
    xc[c] = colp(X, c0 + (c < kc ? c : 0));
    gc[c] = ghost + (long long)(c0 + (c < kc ? c : 0)) * ldg;
  }
  const long long base = off[r >> 6] + (r & 63);
  const int L = len[r];
  for (int sb = 0; sb < L; sb += 8) {
    int ci[8];
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long long e = base + (long long)((sb + j < L) ? sb + j : L - 1) * 64;
      ci[j] = scol[e];
      v[j] = sval[e];
    }
    // J entries' gathers in flight before any is consumed: left to itself the compiler
    // issues one load, waits, multiplies, and only then issues the next (latency-bound,
    // 1.4x slower on the 27-point stencil, tools/mb_spmm27.hip)
#pragma unroll
    for (int j0 = 0; j0 < 8; j0 += J) {
      double xv[J][KC];
      double sc[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int col = ci[j0 + j];
        const bool own = col < n_local;
        // fused right Jacobi: (omega d^-1) of the column (owner's value for a ghost column)
        sc[j] = cs ? (own ? cs[col] : gcs[col - n_local]) : 1.0;
        if constexpr (XR) {
          if (own) {
            const d2 *xp = (const d2 *)(xr + (long long)col * KC);
#pragma unroll
            for (int h = 0; h < KC / 2; ++h) {
              const d2 q = xp[h];
              xv[j][2 * h] = q.x;
              xv[j][2 * h + 1] = q.y;
            }
          } else {
#pragma unroll
            for (int c = 0; c < KC; ++c) xv[j][c] = gc[c][col - n_local];
          }
        } else {
#pragma unroll
          for (int c = 0; c < KC; ++c) xv[j][c] = *(own ? xc[c] + col : gc[c] + (col - n_local));
        }
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const bool ok = sb + j0 + j < L;
#pragma unroll
        for (int c = 0; c < KC; ++c) {
          const double x = cs ? sc[j] * xv[j][c] : xv[j][c];
          const double prod = v[j0 + j] * x;
          sum[c] = sum[c] + (ok ? prod : 0.0);
        }
      }
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

// xr[r][c] = X[r][c0 + c] for c < kc, 0 beyond (KC-wide rows)
template <int KC>
__global__ __launch_bounds__(256) void k_interleave(MvDesc X, int c0, int kc, int n, double *__restrict__ xr) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  double v[KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) v[c] = c < kc ? colp(X, c0 + c)[r] : 0.0;
  d2 *out = (d2 *)(xr + (long long)r * KC);
#pragma unroll
  for (int h = 0; h < KC / 2; ++h) out[h] = d2{v[2 * h], v[2 * h + 1]};
}

bool launch_spmm_sell(hipStream_t s, int n_local, const long long *off, const int *len, const int *scol,
                      const double *sval, MvDesc X, const double *ghost, long long ldg, MvDesc Y, double alpha,
                      double beta, const int *sel, int nsel, double *xr, bool xr_ready, ColScale cs) {
  const int n = sel ? nsel : n_local;
  if (n <= 0) return xr_ready;  // nothing launched: xr is as it was
  const int k = Y.ncols;
  const dim3 grid(cdiv(n, 256));
  for (int c0 = 0; c0 < k; c0 += 8) {
    const int kc = (k - c0) < 8 ? (k - c0) : 8;
    if (xr && kc >= 2) {
      const dim3 gi(cdiv(n_local, 256));
      // xr_ready: an earlier launch of the same apply (interior rows) already interleaved X;
      // only with one column chunk, since xr holds one chunk at a time
      const bool fresh = !(xr_ready && k <= 8);
#define SELL_XR(KC)                                                                                            \
  if (fresh) k_interleave<KC><<<gi, 256, 0, s>>>(X, c0, kc, n_local, xr);                                    \
  k_spmm_sell<KC, true><<<grid, 256, 0, s>>>(n_local, off, len, scol, sval, X, n_local, ghost, ldg, Y, c0, kc, \
                                             alpha, beta, sel, nsel, xr, cs.own, cs.ghost);
      if (kc <= 2) {
        SELL_XR(2)
      } else if (kc <= 4) {
        SELL_XR(4)
      } else {
        SELL_XR(8)
      }
#undef SELL_XR
      LAUNCH_CHECK();
      xr_ready = k <= 8;  // xr holds this (only) chunk now
      continue;
    }
    if (kc == 1)
      k_spmm_sell<1><<<grid, 256, 0, s>>>(n_local, off, len, scol, sval, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta, sel, nsel, nullptr, cs.own, cs.ghost);
    else if (kc <= 2)
      k_spmm_sell<2><<<grid, 256, 0, s>>>(n_local, off, len, scol, sval, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta, sel, nsel, nullptr, cs.own, cs.ghost);
    else if (kc <= 4)
      k_spmm_sell<4><<<grid, 256, 0, s>>>(n_local, off, len, scol, sval, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta, sel, nsel, nullptr, cs.own, cs.ghost);
    else
      k_spmm_sell<8><<<grid, 256, 0, s>>>(n_local, off, len, scol, sval, X, n_local, ghost, ldg, Y, c0, kc, alpha, beta, sel, nsel, nullptr, cs.own, cs.ghost);
    LAUNCH_CHECK();
  }
  return xr_ready;
}

// -------------------------------------------------------------------------------------
// SpMM x k over 3 x 3 blocks (plan: make_bsr3, plan.cpp; rows in node triples with whole
// column triples, e.g. 3-dof finite elements): one thread per block row (3 rows), SELL-64 by
// block, so per block ONE column id (instead of 9) and one contiguous 3 KC-double operand
// segment of the row-interleaved X copy (xr, KC >= 2) instead of 3 KC gathers.  Each row adds
// its three products of a block in column order, blocks in ascending order: the stored order,
// products v * x, no FMA -- bit-identical to k_spmm_sell.  cs: fused right Jacobi scale.
// -------------------------------------------------------------------------------------
// PF: the next group's column ids are loaded one group ahead, so a group's X segment loads
// wait on ids that arrived during the previous group instead of on a fresh id load (the id ->
// X dependent pair was two memory latencies per group).
template <int KC, int J, bool PF = false>
__global__ __launch_bounds__(256) void k_spmm_bsr3(int nbr, const long long *__restrict__ off,
                                                   const int *__restrict__ len, const int *__restrict__ bcol,
                                                   const double *__restrict__ bval, const double *__restrict__ xr,
                                                   MvDesc X, MvDesc Y, int c0, int kc, double alpha, double beta,
                                                   const double *__restrict__ cs) {
#pragma clang fp contract(off)
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= nbr) return;
  const int L = len[b];
  if (L == 0) return;  // a block row left to the row kernel
  const long long o = off[b >> 6];
  const int lane = b & 63;
  const int *bc = bcol + o + lane;
  const double *bv = bval + 9 * o + lane;  // + lane: the pair strips' offset 2 lane is added below
  double s[3][KC];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < KC; ++c) s[r][c] = 0.0;
  const double *x1 = colp(X, c0);  // KC == 1: X's column directly
  int jn[J];
  if constexpr (PF) {
#pragma unroll
    for (int u = 0; u < J; ++u) jn[u] = bc[64LL * (u < L ? u : L - 1)];
  }
  // J blocks' loads in flight together
  for (int q0 = 0; q0 < L; q0 += J) {
    int j[J];
    double v[J][9], x[J][3][KC], sc[J][3];
    if constexpr (PF) {
#pragma unroll
      for (int u = 0; u < J; ++u) {
        j[u] = jn[u];
        const int qn = q0 + J + u < L ? q0 + J + u : L - 1;
        jn[u] = bc[64LL * qn];
      }
    }
#pragma unroll
    for (int u = 0; u < J; ++u) {
      const int q = q0 + u < L ? q0 + u : L - 1;
      if constexpr (!PF) j[u] = bc[64LL * q];
      // values 0..7 as four 16-byte loads of pair-interleaved strips, value 8 from its own strip
      const double *vq = bv + 9 * 64LL * q;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const d2 t = *(const d2 *)(vq + 128 * m + lane);
        v[u][2 * m] = t.x;
        v[u][2 * m + 1] = t.y;
      }
      v[u][8] = vq[512];
    }
#pragma unroll
    for (int u = 0; u < J; ++u) {
      if constexpr (KC == 1) {
#pragma unroll
        for (int e = 0; e < 3; ++e) x[u][e][0] = x1[j[u] + e];
      } else {
        const d2 *xp = (const d2 *)(xr + (long long)j[u] * KC);
#pragma unroll
        for (int h = 0; h < 3 * KC / 2; ++h) {
          const d2 t = xp[h];
          x[u][(2 * h) / KC][(2 * h) % KC] = t.x;
          x[u][(2 * h + 1) / KC][(2 * h + 1) % KC] = t.y;
        }
      }
      if (cs) {
#pragma unroll
        for (int e = 0; e < 3; ++e) sc[u][e] = cs[j[u] + e];
      }
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < J; ++u) {
      if (q0 + u >= L) break;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int e = 0; e < 3; ++e)
#pragma unroll
          for (int c = 0; c < KC; ++c) {
            const double xv = cs ? sc[u][e] * x[u][e][c] : x[u][e][c];
            s[r][c] = s[r][c] + v[u][3 * r + e] * xv;
          }
    }
  }
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      if (c < kc) {
        double *yp = colp(Y, c0 + c) + 3 * b + r;
        if (beta == 0.0)
          *yp = (alpha == 1.0) ? s[r][c] : alpha * s[r][c];
        else
          *yp = alpha * s[r][c] + beta * (*yp);
      }
    }
}

// The same SpMM with H = 2 lanes per block row, lane h taking columns h KC/2 .. (h+1) KC/2 - 1
// of the row-interleaved X: a block's X segment (3 rows x KC doubles, contiguous) is read by
// the lane pair as adjacent halves, so an X load instruction touches half as many cache lines
// per block row as the one-lane form, where every lane's 16-byte piece sat in a line of its own
// (PMC, FlanProxy k = 4: TA 80 % and TD 91 % busy on those gathers, profiles/r4c_flan_pmc.txt).
// Both lanes read the block's column id and 9 values (the same addresses); each output element
// is summed in the one-lane form's order: bit-identical.
template <int KC, int J>
__global__ __launch_bounds__(256) void k_spmm_bsr3h(int nbr, const long long *__restrict__ off,
                                                    const int *__restrict__ len, const int *__restrict__ bcol,
                                                    const double *__restrict__ bval, const double *__restrict__ xr,
                                                    MvDesc Y, int c0, int kc, double alpha, double beta,
                                                    const double *__restrict__ cs) {
#pragma clang fp contract(off)
  constexpr int KH = KC / 2;  // columns per lane
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int b = t >> 1, h = t & 1;
  if (b >= nbr) return;
  const int L = len[b];
  if (L == 0) return;  // a block row left to the row kernel
  const long long o = off[b >> 6];
  const int lane = b & 63;
  const int *bc = bcol + o + lane;
  const double *bv = bval + 9 * o + lane;
  double s[3][KH];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < KH; ++c) s[r][c] = 0.0;
  for (int q0 = 0; q0 < L; q0 += J) {
    int j[J];
    double v[J][9], x[J][3][KH], sc[J][3];
#pragma unroll
    for (int u = 0; u < J; ++u) {
      const int q = q0 + u < L ? q0 + u : L - 1;
      j[u] = bc[64LL * q];
      const double *vq = bv + 9 * 64LL * q;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const d2 tt = *(const d2 *)(vq + 128 * m + lane);
        v[u][2 * m] = tt.x;
        v[u][2 * m + 1] = tt.y;
      }
      v[u][8] = vq[512];
    }
#pragma unroll
    for (int u = 0; u < J; ++u) {
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const double *xp = xr + (long long)(j[u] + e) * KC + h * KH;
#pragma unroll
        for (int p = 0; p < KH / 2; ++p) {
          const d2 tt = *(const d2 *)(xp + 2 * p);
          x[u][e][2 * p] = tt.x;
          x[u][e][2 * p + 1] = tt.y;
        }
      }
      if (cs) {
#pragma unroll
        for (int e = 0; e < 3; ++e) sc[u][e] = cs[j[u] + e];
      }
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < J; ++u) {
      if (q0 + u >= L) break;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int e = 0; e < 3; ++e)
#pragma unroll
          for (int c = 0; c < KH; ++c) {
            const double xv = cs ? sc[u][e] * x[u][e][c] : x[u][e][c];
            s[r][c] = s[r][c] + v[u][3 * r + e] * xv;
          }
    }
  }
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < KH; ++c) {
      const int col = h * KH + c;
      if (col < kc) {
        double *yp = colp(Y, c0 + col) + 3 * b + r;
        if (beta == 0.0)
          *yp = (alpha == 1.0) ? s[r][c] : alpha * s[r][c];
        else
          *yp = alpha * s[r][c] + beta * (*yp);
      }
    }
}

// Cooperative form (the default, launch_spmm_bsr3): the X segments of a wave's 64 J blocks are loaded by
// consecutive lanes as consecutive 16-byte pieces (a segment's 3 KC / 2 pieces by neighbouring
// lanes, so a load instruction covers ~64 / (3 KC / 2) whole segments instead of one piece of
// 64 scattered ones), staged in a wave-private LDS slice, and read back by their owners.  The
// column ids go through LDS the same way.  Every lane of the wave takes part in the loads until
// the wave's longest block row is done; lanes past their own row length (or past nbr) add
// nothing and store nothing.  Same products and order as k_spmm_bsr3: bit-identical.
template <int KC, int J>
__global__ __launch_bounds__(256) void k_spmm_bsr3c(int nbr, const long long *__restrict__ off,
                                                    const int *__restrict__ len, const int *__restrict__ bcol,
                                                    const double *__restrict__ bval, const double *__restrict__ xr,
                                                    MvDesc Y, int c0, int kc, double alpha, double beta,
                                                    const double *__restrict__ cs) {
#pragma clang fp contract(off)
  constexpr int S2 = 3 * KC / 2, NI = J * S2;
  __shared__ __attribute__((aligned(16))) d2 seg[4][64 * NI];
  __shared__ int jl[4][64 * J];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x * 256 + threadIdx.x;
  const bool live = b < nbr;
  const int L = live ? len[b] : 0;
  int Lw = L;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) Lw = max(Lw, __shfl_xor(Lw, o, 64));
  if (Lw == 0) return;  // the whole wave: nothing to do
  const long long o = live ? off[b >> 6] : 0;
  const int *bc = bcol + o + lane;
  const double *bv = bval + 9 * o + lane;
  d2 *sg = seg[w];
  int *jw = jl[w];
  double s[3][KC];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < KC; ++c) s[r][c] = 0.0;
  for (int q0 = 0; q0 < Lw; q0 += J) {
    int j[J];
    double v[J][9], x[J][3][KC], sc[J][3];
#pragma unroll
    for (int u = 0; u < J; ++u) {
      const bool on = q0 + u < L;
      const int q = on ? q0 + u : 0;
      j[u] = on ? bc[64LL * q] : 0;
      if (on) {
        const double *vq = bv + 9 * 64LL * q;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const d2 t = *(const d2 *)(vq + 128 * m + lane);
          v[u][2 * m] = t.x;
          v[u][2 * m + 1] = t.y;
        }
        v[u][8] = vq[512];
      } else {
#pragma unroll
        for (int e = 0; e < 9; ++e) v[u][e] = 0.0;
      }
      jw[u * 64 + lane] = j[u];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    d2 pc[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int p = i * 64 + lane, sidx = p / S2, m = p - sidx * S2;
      pc[i] = *(const d2 *)(xr + (long long)jw[sidx] * KC + 2 * m);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) sg[i * 64 + lane] = pc[i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < J; ++u) {
#pragma unroll
      for (int h = 0; h < S2; ++h) {
        const d2 t = sg[(u * 64 + lane) * S2 + h];
        x[u][(2 * h) / KC][(2 * h) % KC] = t.x;
        x[u][(2 * h + 1) / KC][(2 * h + 1) % KC] = t.y;
      }
      if (cs) {
#pragma unroll
        for (int e = 0; e < 3; ++e) sc[u][e] = cs[j[u] + e];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // the slice is rewritten by the next step
#pragma unroll
    for (int u = 0; u < J; ++u) {
      if (q0 + u >= L) break;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int e = 0; e < 3; ++e)
#pragma unroll
          for (int c = 0; c < KC; ++c) {
            const double xv = cs ? sc[u][e] * x[u][e][c] : x[u][e][c];
            s[r][c] = s[r][c] + v[u][3 * r + e] * xv;
          }
    }
  }
  if (L == 0) return;  // a block row left to the row kernel (or past nbr)
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      if (c < kc) {
        double *yp = colp(Y, c0 + c) + 3 * b + r;
        if (beta == 0.0)
          *yp = (alpha == 1.0) ? s[r][c] : alpha * s[r][c];
        else
          *yp = alpha * s[r][c] + beta * (*yp);
      }
    }
}

void launch_spmm_bsr3(hipStream_t s, int nbr, int n_local, const long long *off, const int *len, const int *bcol,
                      const double *bval, MvDesc X, MvDesc Y, double alpha, double beta, double *xr,
                      ColScale cs) {
  if (nbr <= 0) return;
  static const int jsel = [] {
    const char *e = std::getenv("MIGMRES_BSR3_J");
    return e ? std::atoi(e) : 2;
  }();
  static const bool pf = [] {  // MIGMRES_BSR3_PF=1: column ids one group ahead
    const char *e = std::getenv("MIGMRES_BSR3_PF");
    return e && e[0] == '1';
  }();
  static const int lanes = [] {  // MIGMRES_BSR3_H=2: two lanes per block row (k >= 4)
    const char *e = std::getenv("MIGMRES_BSR3_H");
    return e ? std::atoi(e) : 1;
  }();
  // Cooperative segment loads (k_spmm_bsr3c, default; MIGMRES_BSR3_C=0: k_spmm_bsr3).  Same box,
  // FlanProxy (profiles/r4_knob_sweeps.txt, sweep_r4t_*): k = 4 SpMM 0.300 -> 0.281 ms and
  // 0.291 -> 0.272 ms (two blocks per lane and step; one: equal), k = 8 0.440 -> 0.387 ms.
  static const bool coop = [] {
    const char *e = std::getenv("MIGMRES_BSR3_C");
    return !(e && e[0] == '0');
  }();
  const int k = Y.ncols;
  const dim3 grid(cdiv(nbr, 256)), gi(cdiv(n_local, 256));
  for (int c0 = 0; c0 < k; c0 += 8) {
    const int kc = (k - c0) < 8 ? (k - c0) : 8;
    if (kc == 1) {
      k_spmm_bsr3<1, 4><<<grid, 256, 0, s>>>(nbr, off, len, bcol, bval, nullptr, X, Y, c0, kc, alpha, beta, cs.own);
    } else {
#define BSR3_XR(KC)                                                                                             \
  k_interleave<KC><<<gi, 256, 0, s>>>(X, c0, kc, n_local, xr);                                                \
  if (coop && jsel == 1)                                                                                        \
    k_spmm_bsr3c<KC, 1><<<grid, 256, 0, s>>>(nbr, off, len, bcol, bval, xr, Y, c0, kc, alpha, beta, cs.own);    \
  else if (coop && KC <= 4)                                                                                     \
    k_spmm_bsr3c<KC, 2><<<grid, 256, 0, s>>>(nbr, off, len, bcol, bval, xr, Y, c0, kc, alpha, beta, cs.own);    \
  else if (coop)                                                                                                \
    k_spmm_bsr3c<KC, 1><<<grid, 256, 0, s>>>(nbr, off, len, bcol, bval, xr, Y, c0, kc, alpha, beta, cs.own);    \
  else if (lanes == 2 && KC >= 4)                                                                               \
    k_spmm_bsr3h<KC, 2><<<dim3(cdiv(2LL * nbr, 256)), 256, 0, s>>>(nbr, off, len, bcol, bval, xr, Y, c0, kc, alpha, beta, cs.own); \
  else if (pf && jsel == 4 && KC <= 4)                                                                          \
    k_spmm_bsr3<KC, 4, true><<<grid, 256, 0, s>>>(nbr, off, len, bcol, bval, xr, X, Y, c0, kc, alpha, beta, cs.own); \
  else if (pf)                                                                                                  \
    k_spmm_bsr3<KC, 2, true><<<grid, 256, 0, s>>>(nbr, off, len, bcol, bval, xr, X, Y, c0, kc, alpha, beta, cs.own); \
  else if (jsel == 4 && KC <= 4)                                                                                \
    k_spmm_bsr3<KC, 4><<<grid, 256, 0, s>>>(nbr, off, len, bcol, bval, xr, X, Y, c0, kc, alpha, beta, cs.own); \
  else if (jsel == 1)                                                                                           \
    k_spmm_bsr3<KC, 1><<<grid, 256, 0, s>>>(nbr, off, len, bcol, bval, xr, X, Y, c0, kc, alpha, beta, cs.own); \
  else                                                                                                          \
    k_spmm_bsr3<KC, 2><<<grid, 256, 0, s>>>(nbr, off, len, bcol, bval, xr, X, Y, c0, kc, alpha, beta, cs.own);
      if (kc <= 2) {
        BSR3_XR(2)
      } else if (kc <= 4) {
        BSR3_XR(4)
      } else {
        BSR3_XR(8)
      }
#undef BSR3_XR
    }
    LAUNCH_CHECK();
  }
}

// -------------------------------------------------------------------------------------
// SpMM x k over row pairs (plan: make_pair_plan, plan.cpp).  One thread per row pair; every
// X read is a 16-byte load of an aligned pair of rows shared by both rows of the pair (the
// 8-byte gathers of k_spmm were instruction-bound: tools/mb_spmm.hip measured 1.35 ms
// for 8-B gathers vs 0.79 ms for 16-B pair loads on the 256^3 stencil).  Each key's 16-bit
// map says which entry of each row takes the low / high half; the row sums still run in
// stored order with products v * x and no FMA, so the result is bit-identical to k_spmm.
// Keys past a pair's count re-read the last key with an empty map (adds nothing).
// -------------------------------------------------------------------------------------
constexpr int PAIR_MAXR = 8;

// CS: the fused right Jacobi's column scale (a template flag, so the plain form holds no scale
// registers: 154 -> fewer VGPRs, one more wave per SIMD)
template <int KC, int PAIR_MAXK, bool CS>
__global__ __launch_bounds__(256) void k_spmm_pair(int npairs, int rmax, const double *__restrict__ sv,
                                                   const int *__restrict__ sk,
                                                   const unsigned short *__restrict__ sm, MvDesc X, int n_local,
                                                   const double *__restrict__ ghost, long long ldg, MvDesc Y,
                                                   int c0, int kc, double alpha, double beta,
                                                   const int *__restrict__ sel, int nsel,
                                                   const double *__restrict__ cs, const double *__restrict__ gcs) {
#pragma clang fp contract(off)
  // sel: optional list of the pairs to compute (interior / boundary split of the halo overlap)
  int p = blockIdx.x * 256 + threadIdx.x;
  if (sel) {
    if (p >= nsel) return;
    p = sel[p];
  } else if (p >= npairs) {
    return;
  }
  const int ra = 2 * p;
  const bool hasb = ra + 1 < n_local;
  // SELL-64 plan (make_pair_sell): slot j of the 64 pairs of a wave is contiguous
  const long long chunk = p >> 6;
  const int lane = p & 63;
  const double *va_p = sv + chunk * 2 * rmax * 64 + lane;
  const double *vb_p = va_p + (long long)rmax * 64;
  // the pair's coefficients go through a per-thread LDS slot so that each (key, half, row)
  // picks its entry with one indexed read instead of an 8-way select chain
  __shared__ double vlds[256][2 * PAIR_MAXR + 1];
  double *myv = vlds[threadIdx.x];
#pragma unroll
  for (int j = 0; j < PAIR_MAXR; ++j) {
    if (j < rmax) {
      myv[j] = va_p[j * 64];
      myv[PAIR_MAXR + j] = vb_p[j * 64];
    }
  }
  myv[2 * PAIR_MAXR] = 0.0;
  const int *kp = sk + chunk * PAIR_MAXK * 64 + lane;
  const unsigned short *mp = sm + chunk * PAIR_MAXK * 64 + lane;
  int key[PAIR_MAXK];
  double cx[PAIR_MAXK][4];  // coefficient taking (row a low, row a high, row b low, row b high)
  unsigned long long use = 0;  // bit 4u + s: slot s of key u is used
#pragma unroll
  for (int u = 0; u < PAIR_MAXK; ++u) {
    key[u] = kp[u * 64];
    const unsigned m = mp[u * 64];
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {
      const int idx = (m >> (4 * sl)) & 0xF;
      const bool used = idx != 0xF;
      cx[u][sl] = myv[used ? (sl < 2 ? 0 : PAIR_MAXR) + idx : 2 * PAIR_MAXR];
      use |= (used ? 1ull : 0ull) << (4 * u + sl);
    }
  }
  // fused right Jacobi: per key the (omega d^-1) pair of its two columns (the owner's values
  // for ghost columns, imported once); zero padding past the last row / ghost
  d2 sc[CS ? PAIR_MAXK : 1];
  if constexpr (CS) {
#pragma unroll
    for (int u = 0; u < PAIR_MAXK; ++u)
      sc[u] = *(const d2 *)(key[u] >= 0 ? cs + 2LL * key[u] : gcs + 2LL * (-key[u] - 1));
  }
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    if (c >= kc) break;
    const double *xc = colp(X, c0 + c);
    const double *gc = ghost + (long long)(c0 + c) * ldg;
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int u = 0; u < PAIR_MAXK; ++u) {
      const int kk = key[u];
      const double *src = kk >= 0 ? xc + 2LL * kk : gc + 2LL * (-kk - 1);
      d2 x = *(const d2 *)src;
      if constexpr (CS) x = sc[u] * x;
      const double pa0 = cx[u][0] * x.x, pa1 = cx[u][1] * x.y;
      const double pb0 = cx[u][2] * x.x, pb1 = cx[u][3] * x.y;
      sa = sa + ((use >> (4 * u)) & 1ull ? pa0 : 0.0);
      sa = sa + ((use >> (4 * u + 1)) & 1ull ? pa1 : 0.0);
      sb = sb + ((use >> (4 * u + 2)) & 1ull ? pb0 : 0.0);
      sb = sb + ((use >> (4 * u + 3)) & 1ull ? pb1 : 0.0);
    }
    double *yp = colp(Y, c0 + c) + ra;
    if (beta == 0.0) {
      if (alpha != 1.0) {
        sa = alpha * sa;
        sb = alpha * sb;
      }
    } else {
      sa = alpha * sa + beta * yp[0];
      if (hasb) sb = alpha * sb + beta * yp[1];
    }
    if (hasb)
      *(d2 *)yp = d2{sa, sb};
    else
      yp[0] = sa;
  }
}

template <int MAXK>
static void spmm_pair_cols(hipStream_t s, int npairs, int rmax, const double *sv, const int *sk,
                           const unsigned short *sm, MvDesc X, int n_local, const double *ghost, long long ldg,
                           MvDesc Y, double alpha, double beta, const int *sel, int nsel, ColScale cs) {
  const int k = Y.ncols;
  const int units = sel ? nsel : npairs;
  if (units <= 0) return;
  const dim3 grid(cdiv(units, 256));
  for (int c0 = 0; c0 < k; c0 += 8) {
    const int kc = (k - c0) < 8 ? (k - c0) : 8;
#define PAIR_KC(KC)                                                                                              \
  if (cs.own)                                                                                                    \
    k_spmm_pair<KC, MAXK, true><<<grid, 256, 0, s>>>(npairs, rmax, sv, sk, sm, X, n_local, ghost, ldg, Y, c0, kc,  \
                                                     alpha, beta, sel, nsel, cs.own, cs.ghost);                  \
  else                                                                                                           \
    k_spmm_pair<KC, MAXK, false><<<grid, 256, 0, s>>>(npairs, rmax, sv, sk, sm, X, n_local, ghost, ldg, Y, c0, kc, \
                                                      alpha, beta, sel, nsel, nullptr, nullptr);
    if (kc == 1) {
      PAIR_KC(1)
    } else if (kc <= 2) {
      PAIR_KC(2)
    } else if (kc <= 4) {
      PAIR_KC(4)
    } else {
      PAIR_KC(8)
    }
#undef PAIR_KC
    LAUNCH_CHECK();
  }
}

void launch_spmm_pair(hipStream_t s, int n_local, int max_keys, int rmax, const double *sv, const int *sk,
                      const unsigned short *sm, MvDesc X, const double *ghost, long long ldg, MvDesc Y,
                      double alpha, double beta, const int *sel, int nsel, ColScale cs) {
  const int npairs = (n_local + 1) / 2;
  if (npairs <= 0) return;
  if (rmax > PAIR_MAXR) throw Error(MIGMRES_EINVAL, "spmm_pair: rows longer than 8 entries");
  // instantiated for the exact key count (the SELL plan is laid out with that stride)
#define PAIR_CASE(K) \
  case K:            \
    spmm_pair_cols<K>(s, npairs, rmax, sv, sk, sm, X, n_local, ghost, ldg, Y, alpha, beta, sel, nsel, cs); \
    break;
  switch (max_keys) {
    PAIR_CASE(1)
    PAIR_CASE(2)
    PAIR_CASE(3)
    PAIR_CASE(4)
    PAIR_CASE(5)
    PAIR_CASE(6)
    PAIR_CASE(7)
    PAIR_CASE(8)
    PAIR_CASE(9)
    PAIR_CASE(10)
    PAIR_CASE(11)
    PAIR_CASE(12)
    default:
      throw Error(MIGMRES_EINVAL, "spmm_pair: more than 12 keys per row pair");
  }
#undef PAIR_CASE
}

// -------------------------------------------------------------------------------------
// SpMM x k over row-pair TEMPLATES (plan: make_pair_templates, plan.cpp).  Same arithmetic
// as k_spmm_pair -- one thread per row pair, 16-byte loads of aligned X row pairs, each
// row's products added in stored order, no FMA -- but the matrix is read as one template
// byte per pair: the template's keys (offsets from the pair) and coefficient slots sit in
// LDS, the coefficients in a value dictionary (slot 255 = no entry, value 0, never added).
// For a stencil operator this removes the 12 bytes per entry of the CSR stream, leaving X
// (gathered, mostly from L2) and Y.  Pairs marked kTplNone (they read ghost columns) are
// skipped here and computed by the fallback kernel.  Grid-stride over resident workgroups,
// so the LDS tables are loaded once per workgroup.  Per key the next key's KC loads are
// issued before the current key's products (two keys' loads in flight).
// -------------------------------------------------------------------------------------
template <int KC>
__global__ __launch_bounds__(256) void k_spmm_tpl(int npairs, int n_local, const unsigned char *__restrict__ tid,
                                                  const int2 *__restrict__ rec, int maxk, int nrec,
                                                  const double *__restrict__ vals, int nvals, MvDesc X, MvDesc Y,
                                                  int c0, int kc, double alpha, double beta,
                                                  const double *__restrict__ cs) {
#pragma clang fp contract(off)
  extern __shared__ double tpl_lds[];
  double *s_val = tpl_lds;                   // 256 dictionary slots (255: none, 0.0)
  int2 *s_rec = (int2 *)(tpl_lds + 256);     // ntpl * maxk key records
  s_val[threadIdx.x] = (int)threadIdx.x < nvals ? vals[threadIdx.x] : 0.0;
  for (int i = threadIdx.x; i < nrec; i += 256) s_rec[i] = rec[i];
  __syncthreads();
  const double *xc[KC];
  double *yc[KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    xc[c] = colp(X, c0 + (c < kc ? c : 0));
    yc[c] = colp(Y, c0 + (c < kc ? c : 0));
  }
  for (int p = blockIdx.x * 256 + threadIdx.x; p < npairs; p += gridDim.x * 256) {
    const int t = tid[p];
    if (t == 0xFF) continue;
    const int2 *r = s_rec + t * maxk;
    double sa[KC], sb[KC];
#pragma unroll
    for (int c = 0; c < KC; ++c) sa[c] = sb[c] = 0.0;
    d2 xn[KC], scn = d2{1.0, 1.0};
    int2 qn = r[0];
#pragma unroll
    for (int c = 0; c < KC; ++c) xn[c] = *(const d2 *)(xc[c] + 2LL * (p + qn.x));
    if (cs) scn = *(const d2 *)(cs + 2LL * (p + qn.x));
    for (int u = 0; u < maxk; ++u) {
      d2 x[KC];
#pragma unroll
      for (int c = 0; c < KC; ++c) x[c] = xn[c];
      const d2 sc = scn;
      const unsigned sl = (unsigned)qn.y;
      if (u + 1 < maxk) {  // uniform: issue the next key's loads before these products
        qn = r[u + 1];
#pragma unroll
        for (int c = 0; c < KC; ++c) xn[c] = *(const d2 *)(xc[c] + 2LL * (p + qn.x));
        if (cs) scn = *(const d2 *)(cs + 2LL * (p + qn.x));
      }
      if (cs) {  // fused Jacobi: the operand is (omega D^-1) x, formed exactly as k_jacobi forms it
#pragma unroll
        for (int c = 0; c < KC; ++c) x[c] = sc * x[c];
      }
      const unsigned s0 = sl & 0xFF, s1 = (sl >> 8) & 0xFF, s2 = (sl >> 16) & 0xFF, s3 = sl >> 24;
      const double v0 = s_val[s0], v1 = s_val[s1], v2 = s_val[s2], v3 = s_val[s3];
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        const double pa0 = v0 * x[c].x, pa1 = v1 * x[c].y;
        const double pb0 = v2 * x[c].x, pb1 = v3 * x[c].y;
        sa[c] = sa[c] + (s0 != 0xFF ? pa0 : 0.0);
        sa[c] = sa[c] + (s1 != 0xFF ? pa1 : 0.0);
        sb[c] = sb[c] + (s2 != 0xFF ? pb0 : 0.0);
        sb[c] = sb[c] + (s3 != 0xFF ? pb1 : 0.0);
      }
    }
    const int ra = 2 * p;
    const bool hasb = ra + 1 < n_local;
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      if (c >= kc) break;
      double *yp = yc[c] + ra;
      double a = sa[c], b = sb[c];
      if (beta == 0.0) {
        if (alpha != 1.0) {
          a = alpha * a;
          b = alpha * b;
        }
      } else {
        a = alpha * a + beta * yp[0];
        if (hasb) b = alpha * b + beta * yp[1];
      }
      if (hasb)
        *(d2 *)yp = d2{a, b};
      else
        yp[0] = a;
    }
  }
}

// Short templates (at most 12 keys per pair: 5- and 7-point stencils): the pair's key
// offsets and coefficients are taken into registers once, then the KC columns are swept
// with all of a column's MAXK loads in flight (the k_spmm_pair loop without its plan
// stream).  Instantiated for the exact key count.
template <int KC, int MAXK>
__global__ __launch_bounds__(256) void k_spmm_tplr(int npairs, int n_local, const unsigned char *__restrict__ tid,
                                                   const int2 *__restrict__ rec, int nrec,
                                                   const double *__restrict__ vals, int nvals, MvDesc X, MvDesc Y,
                                                   int c0, int kc, double alpha, double beta,
                                                   const double *__restrict__ cs, int xcd_slabs) {
#pragma clang fp contract(off)
  extern __shared__ double tpl_lds[];
  double *s_val = tpl_lds;
  int2 *s_rec = (int2 *)(tpl_lds + 256);
  s_val[threadIdx.x] = (int)threadIdx.x < nvals ? vals[threadIdx.x] : 0.0;
  for (int i = threadIdx.x; i < nrec; i += 256) s_rec[i] = rec[i];
  __syncthreads();
  // grid-stride, or (xcd_slabs) each XCD a contiguous eighth of the pairs in 256-pair blocks
  int p0, p1, ps;
  if (xcd_slabs) {
    const int xcd = blockIdx.x & 7, nb = gridDim.x >> 3;
    const int blocks = (npairs + 255) / 256;
    p0 = ((int)((long long)blocks * xcd / 8) + (int)(blockIdx.x >> 3)) * 256 + threadIdx.x;
    p1 = min(npairs, (int)((long long)blocks * (xcd + 1) / 8) * 256);
    ps = nb * 256;
  } else {
    p0 = blockIdx.x * 256 + threadIdx.x;
    p1 = npairs;
    ps = gridDim.x * 256;
  }
  for (int p = p0; p < p1; p += ps) {
    const int t = tid[p];
    if (t == 0xFF) continue;
    int key[MAXK];
    double cx[MAXK][4];
    unsigned long long use = 0;
#pragma unroll
    for (int u = 0; u < MAXK; ++u) {
      const int2 q = s_rec[t * MAXK + u];
      key[u] = p + q.x;
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) {
        const unsigned s = ((unsigned)q.y >> (8 * sl)) & 0xFF;
        cx[u][sl] = s_val[s];
        use |= (s != 0xFF ? 1ull : 0ull) << (4 * u + sl);
      }
    }
    const int ra = 2 * p;
    const bool hasb = ra + 1 < n_local;
    d2 sc[MAXK];
    if (cs) {
#pragma unroll
      for (int u = 0; u < MAXK; ++u) sc[u] = *(const d2 *)(cs + 2LL * key[u]);
    }
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      if (c >= kc) break;
      const double *xc = colp(X, c0 + c);
      d2 x[MAXK];
#pragma unroll
      for (int u = 0; u < MAXK; ++u) x[u] = *(const d2 *)(xc + 2LL * key[u]);
      if (cs) {  // fused Jacobi: (omega D^-1) x exactly as k_jacobi forms it
#pragma unroll
        for (int u = 0; u < MAXK; ++u) x[u] = sc[u] * x[u];
      }
      double sa = 0.0, sb = 0.0;
#pragma unroll
      for (int u = 0; u < MAXK; ++u) {
        const double pa0 = cx[u][0] * x[u].x, pa1 = cx[u][1] * x[u].y;
        const double pb0 = cx[u][2] * x[u].x, pb1 = cx[u][3] * x[u].y;
        sa = sa + ((use >> (4 * u)) & 1ull ? pa0 : 0.0);
        sa = sa + ((use >> (4 * u + 1)) & 1ull ? pa1 : 0.0);
        sb = sb + ((use >> (4 * u + 2)) & 1ull ? pb0 : 0.0);
        sb = sb + ((use >> (4 * u + 3)) & 1ull ? pb1 : 0.0);
      }
      double *yp = colp(Y, c0 + c) + ra;
      if (beta == 0.0) {
        if (alpha != 1.0) {
          sa = alpha * sa;
          sb = alpha * sb;
        }
      } else {
        sa = alpha * sa + beta * yp[0];
        if (hasb) sb = alpha * sb + beta * yp[1];
      }
      if (hasb)
        *(d2 *)yp = d2{sa, sb};
      else
        yp[0] = sa;
    }
  }
}

// -------------------------------------------------------------------------------------
// SpMM x k over stencil-group templates (plan: make_stencil_groups, plan.cpp) -- the 27-point
// operator.  A pair's keys form G groups of three consecutive pairs (c_g - 1, c_g, c_g + 1),
// and the pair's lane loads only the centre pair p + c_g of each group: its left neighbour
// lane's centre is p - 1 + c_g (= this pair's key c_g - 1) and its right neighbour's is
// p + 1 + c_g (= key c_g + 1), so the two halves a row needs from those keys -- row 0 the high
// half of c_g - 1, row 1 the low half of c_g + 1 -- come from the adjacent lanes by DPP wave
// shifts (v_mov_b32_dpp wave_shr:1 / wave_shl:1) instead of loads: 9 X loads per column and
// pair instead of 27 (the template kernel was bound by the texture addresser: TA 82 % busy,
// 243 vector-memory instructions per 64 pairs, profiles/r3b_brick_spmm_pmc.json).  A wave
// covers 64 consecutive pairs and writes the 62 inner ones (lanes 0 and 63 only load, for
// their neighbours), so the shifts never cross a wave.  Per row the products are added group
// by group, each group's three in ascending column order -- the stored order -- with the same
// products v * x and no FMA as k_spmm: bit-identical.  With cs the centre operands are scaled
// by (omega d^-1) before they are shared, exactly as k_jacobi forms them.
// -------------------------------------------------------------------------------------
struct StencilCenters {
  int c[9];
};

__device__ __forceinline__ double dpp_from_prev_lane(double v) {  // lane i <- lane i - 1
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x138, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x138, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_from_next_lane(double v) {  // lane i <- lane i + 1
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x130, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x130, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

template <int KC, int G>
__global__ __launch_bounds__(256) void k_spmm_tpl3(int npairs, int n_local, const unsigned char *__restrict__ tid,
                                                   const unsigned long long *__restrict__ grp, int ngrp,
                                                   StencilCenters ctr, const double *__restrict__ vals, int nvals,
                                                   MvDesc X, MvDesc Y, int c0, int kc, double alpha, double beta,
                                                   const double *__restrict__ cs, int xcd_slabs) {
#pragma clang fp contract(off)
  extern __shared__ double tpl_lds[];
  double *s_val = tpl_lds;
  __shared__ int s_ctr[G + 1];
  unsigned long long *s_grp = (unsigned long long *)(tpl_lds + 256);
  s_val[threadIdx.x] = (int)threadIdx.x < nvals ? vals[threadIdx.x] : 0.0;
  for (int i = threadIdx.x; i < ngrp; i += 256) s_grp[i] = grp[i];
  if (threadIdx.x <= G) s_ctr[threadIdx.x] = threadIdx.x < G ? ctr.c[threadIdx.x] : 0;
  __syncthreads();
  const double *xc[KC];
  double *yc[KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    xc[c] = colp(X, c0 + (c < kc ? c : 0));
    yc[c] = colp(Y, c0 + (c < kc ? c : 0));
  }
  const int lane = threadIdx.x & 63;
  // wave items of 62 pairs: grid-stride over all of them, or (xcd_slabs; workgroups are
  // dealt to the 8 XCDs round-robin) each XCD walks a contiguous eighth, so the neighbouring
  // lines and planes a stencil row reads were mostly fetched into the same XCD's L2
  const int items = (npairs + 61) / 62;
  int w0, w1, ws;
  if (xcd_slabs) {
    const int xcd = blockIdx.x & 7, nb = gridDim.x >> 3;
    w0 = (int)((long long)items * xcd / 8) + (int)(blockIdx.x >> 3) * 4 + (int)(threadIdx.x >> 6);
    w1 = (int)((long long)items * (xcd + 1) / 8);
    ws = nb * 4;
  } else {
    w0 = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    w1 = items;
    ws = gridDim.x * 4;
  }
  // wave-uniform loop: every lane takes part in the shifts
  for (int w = w0; w < w1; w += ws) {
    const int p = w * 62 + lane - 1;
    const bool mine = lane >= 1 && lane <= 62 && p < npairs;
    const int t = mine ? (int)tid[p] : 0xFF;
    const int tt = t == 0xFF ? 0 : t;  // a load-only or untemplated lane follows template 0 (unused)
    const int pc = p < 0 ? 0 : (p >= npairs ? npairs - 1 : p);
    double sa[KC], sb[KC];
#pragma unroll
    for (int c = 0; c < KC; ++c) sa[c] = sb[c] = 0.0;
    d2 xn[KC], scn = d2{1.0, 1.0};
    {
      int q = pc + s_ctr[0];
      q = q < 0 ? 0 : (q >= npairs ? npairs - 1 : q);
#pragma unroll
      for (int c = 0; c < KC; ++c) xn[c] = *(const d2 *)(xc[c] + 2LL * q);
      if (cs) scn = *(const d2 *)(cs + 2LL * q);
    }
    // not unrolled: unrolled, the scheduler hoists all G groups' loads (512 VGPRs at KC = 8)
#pragma unroll 1
    for (int g = 0; g < G; ++g) {
      d2 x[KC];
#pragma unroll
      for (int c = 0; c < KC; ++c) x[c] = xn[c];
      const d2 sc = scn;
      if (g + 1 < G) {  // the next group's loads before this group's products
        int q = pc + s_ctr[g + 1];
        q = q < 0 ? 0 : (q >= npairs ? npairs - 1 : q);
#pragma unroll
        for (int c = 0; c < KC; ++c) xn[c] = *(const d2 *)(xc[c] + 2LL * q);
        if (cs) scn = *(const d2 *)(cs + 2LL * q);
      }
      if (cs) {
#pragma unroll
        for (int c = 0; c < KC; ++c) x[c] = sc * x[c];
      }
      const unsigned long long sl = s_grp[tt * G + g];
      const unsigned s0 = sl & 0xFF, s1 = (sl >> 8) & 0xFF, s2 = (sl >> 16) & 0xFF;
      const unsigned s3 = (sl >> 24) & 0xFF, s4 = (sl >> 32) & 0xFF, s5 = (sl >> 40) & 0xFF;
      const double v0 = s_val[s0], v1 = s_val[s1], v2 = s_val[s2];
      const double v3 = s_val[s3], v4 = s_val[s4], v5 = s_val[s5];
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        const double left = dpp_from_prev_lane(x[c].y);   // key c_g - 1, high half (row 0's x - 1)
        const double right = dpp_from_next_lane(x[c].x);  // key c_g + 1, low half (row 1's x + 1)
        const double pa0 = v0 * left, pa1 = v1 * x[c].x, pa2 = v2 * x[c].y;
        const double pb0 = v3 * x[c].x, pb1 = v4 * x[c].y, pb2 = v5 * right;
        sa[c] = sa[c] + (s0 != 0xFF ? pa0 : 0.0);
        sa[c] = sa[c] + (s1 != 0xFF ? pa1 : 0.0);
        sa[c] = sa[c] + (s2 != 0xFF ? pa2 : 0.0);
        sb[c] = sb[c] + (s3 != 0xFF ? pb0 : 0.0);
        sb[c] = sb[c] + (s4 != 0xFF ? pb1 : 0.0);
        sb[c] = sb[c] + (s5 != 0xFF ? pb2 : 0.0);
      }
    }
    if (t == 0xFF) continue;
    const int ra = 2 * p;
    const bool hasb = ra + 1 < n_local;
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      if (c >= kc) break;
      double *yp = yc[c] + ra;
      double a = sa[c], b = sb[c];
      if (beta == 0.0) {
        if (alpha != 1.0) {
          a = alpha * a;
          b = alpha * b;
        }
      } else {
        a = alpha * a + beta * yp[0];
        if (hasb) b = alpha * b + beta * yp[1];
      }
      if (hasb)
        *(d2 *)yp = d2{a, b};
      else
        yp[0] = a;
    }
  }
}

static int tpl_resident_blocks(const void *kern, size_t lds) {
  int dev = 0, ncu = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
    ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  return ncu * per_cu;
}

template <class K>
static void tpl_launch(K kern, hipStream_t s, size_t lds, int npairs, const void *key) {
  // resident grid per (kernel, table size): grid-stride loops load the LDS tables once per
  // workgroup
  static thread_local std::vector<std::pair<std::pair<const void *, size_t>, int>> cache;
  int resident = 0;
  for (auto &e : cache)
    if (e.first.first == key && e.first.second == lds) resident = e.second;
  if (!resident) {
    resident = tpl_resident_blocks(key, lds);
    cache.push_back({{key, lds}, resident});
  }
  kern(std::min(cdiv(npairs, 256), resident));
}

template <int KC>
static void tpl_cols(hipStream_t s, size_t lds, int npairs, int n_local, const unsigned char *tid, const int2 *rec,
                     int maxk, int nrec, const double *vals, int nvals, MvDesc X, MvDesc Y, int c0, int kc,
                     double alpha, double beta, const double *cs, int xcd_slabs) {
#define TPLR_CASE(K)                                                                                          \
  case K:                                                                                                     \
    tpl_launch([&](int grid) {                                                                                \
                 const bool slabs = xcd_slabs && grid >= 64;                                                  \
                 if (slabs) grid &= ~7;                                                                       \
                 k_spmm_tplr<KC, K><<<grid, 256, lds, s>>>(npairs, n_local, tid, rec, nrec, vals, nvals, X, Y, \
                                                           c0, kc, alpha, beta, cs, slabs ? 1 : 0);           \
               },                                                                                             \
               s, lds, npairs, (const void *)k_spmm_tplr<KC, K>);                                             \
    return;
  switch (maxk) {
    TPLR_CASE(1)
    TPLR_CASE(2)
    TPLR_CASE(3)
    TPLR_CASE(4)
    TPLR_CASE(5)
    TPLR_CASE(6)
    TPLR_CASE(7)
    TPLR_CASE(8)
    TPLR_CASE(9)
    TPLR_CASE(10)
    TPLR_CASE(11)
    TPLR_CASE(12)
    default:
      break;
  }
#undef TPLR_CASE
  tpl_launch([&](int grid) { k_spmm_tpl<KC><<<grid, 256, lds, s>>>(npairs, n_local, tid, rec, maxk, nrec, vals, nvals,
                                                                  X, Y, c0, kc, alpha, beta, cs); },
             s, lds, npairs, (const void *)k_spmm_tpl<KC>);
}

template <int KC, int G>
static void tpl3_cols(hipStream_t s, size_t lds, int npairs, int n_local, const unsigned char *tid,
                      const unsigned long long *grp, int ngrp, StencilCenters ctr, const double *vals, int nvals,
                      MvDesc X, MvDesc Y, int c0, int kc, double alpha, double beta, const double *cs,
                      int xcd_slabs) {
  const int units = cdiv(npairs, 62);  // wave iterations (62 pairs each)
  tpl_launch([&](int grid) {
               // the slab walk needs whole rounds of 8 workgroups (one per XCD)
               const bool slabs = xcd_slabs && grid >= 64;
               if (slabs) grid &= ~7;
               k_spmm_tpl3<KC, G><<<grid, 256, lds, s>>>(npairs, n_local, tid, grp, ngrp, ctr, vals, nvals, X, Y,
                                                          c0, kc, alpha, beta, cs, slabs ? 1 : 0);
             },
             s, lds, units * 64, (const void *)k_spmm_tpl3<KC, G>);
}

bool launch_spmm_tpl3(hipStream_t s, int n_local, const unsigned char *tid, const unsigned long long *grp, int ntpl,
                      int G, const int *centers, const double *vals, int nvals, MvDesc X, MvDesc Y, double alpha,
                      double beta, const double *colscale, int xcd_slabs, int kcmax) {
  const int npairs = (n_local + 1) / 2;
  if (npairs <= 0) return true;
  if (G != 9 && G != 5 && G != 3) return false;
  StencilCenters ctr{};
  for (int g = 0; g < G; ++g) ctr.c[g] = centers[g];
  const int ngrp = ntpl * G;
  const size_t lds = sizeof(double) * 256 + sizeof(unsigned long long) * (size_t)ngrp;
  const int k = Y.ncols;
  const int kstep = kcmax == 2 ? 2 : kcmax == 4 ? 4 : 8;
  for (int c0 = 0; c0 < k; c0 += kstep) {
    const int kc = (k - c0) < kstep ? (k - c0) : kstep;
#define TPL3(KC)                                                                                                   \
  if (G == 9)                                                                                                      \
    tpl3_cols<KC, 9>(s, lds, npairs, n_local, tid, grp, ngrp, ctr, vals, nvals, X, Y, c0, kc, alpha, beta, colscale, \
                     xcd_slabs);                                                                                   \
  else if (G == 5)                                                                                                 \
    tpl3_cols<KC, 5>(s, lds, npairs, n_local, tid, grp, ngrp, ctr, vals, nvals, X, Y, c0, kc, alpha, beta, colscale, \
                     xcd_slabs);                                                                                   \
  else                                                                                                             \
    tpl3_cols<KC, 3>(s, lds, npairs, n_local, tid, grp, ngrp, ctr, vals, nvals, X, Y, c0, kc, alpha, beta, colscale, \
                     xcd_slabs);
    if (kc == 1) {
      TPL3(1)
    } else if (kc <= 2) {
      TPL3(2)
    } else if (kc <= 4) {
      TPL3(4)
    } else {
      TPL3(8)
    }
#undef TPL3
    LAUNCH_CHECK();
  }
  return true;
}

// -------------------------------------------------------------------------------------
// SpMM x k over the stencil-group templates as a 2.5-D march (geometry: make_march_geometry,
// plan.cpp).  The template kernels gather every key of every pair from memory -- 7 (9 with
// lane sharing) 16-byte loads per pair and column, each X pair fetched once per pair that
// reads it; the 7-point launch kept the texture data path 96 % busy
// (profiles/r2e_spmm_cache_pmc.json).  Here a workgroup owns a tile of 64 pairs x 4 lines and
// walks a slab of planes: each plane tile, with a one-pair and one-line halo, is loaded once
// into a 4-plane LDS ring (planes z - 1, z, z + 1 read, z + 2 being written: one barrier per
// plane), the next plane's loads are in flight while the current one is computed, and every
// key of a pair is then an LDS read -- the group centre (x, y + b, z + a), the left
// neighbour's high half and the right neighbour's low half.  Products, their order and the
// zero-for-unused rule are k_spmm_tpl3's (its per-group sums in stored column order, no FMA),
// so the result is the same bits.  With cs the staged operand is (omega d^-1) x, formed once
// per X pair as k_jacobi forms it.  Tiles are dealt to the XCDs in contiguous ranges of
// consecutive lines (workgroup b runs on XCD b mod 8), so the line halo a tile loads was
// usually just loaded by its neighbour on the same XCD.
// -------------------------------------------------------------------------------------
constexpr int kMarchTX = 64, kMarchTY = 4;
constexpr int kMarchLX = kMarchTX + 2, kMarchLY = kMarchTY + 2, kMarchPl = kMarchLX * kMarchLY;

__device__ __forceinline__ void march_barrier() {  // LDS hand-off only: keeps global loads in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int KC, int G, int PD>
__global__ __launch_bounds__(256) void k_spmm_march(int npairs, int n_local, const unsigned char *__restrict__ tid,
                                                    const unsigned long long *__restrict__ grp, int ngrp,
                                                    MarchGeom mg, int txn, int tyn, int tzn, int sz,
                                                    const double *__restrict__ vals, int nvals, MvDesc X, MvDesc Y,
                                                    double alpha, double beta, const double *__restrict__ cs) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) double march_lds[];
  d2 *ring = (d2 *)march_lds;                                  // [4][KC][kMarchLY][kMarchLX]
  double *s_val = march_lds + 2 * 4 * KC * kMarchPl;           // 256 dictionary slots
  unsigned long long *s_grp = (unsigned long long *)(s_val + 256);
  __shared__ int s_gz[G], s_gl[G];  // group g: plane offset, line offset x kMarchLX
  const int t = threadIdx.x;
  s_val[t] = t < nvals ? vals[t] : 0.0;
  for (int i = t; i < ngrp; i += 256) s_grp[i] = grp[i];
  if (t < G) {
    s_gz[t] = mg.ga[t];
    s_gl[t] = mg.gb[t] * kMarchLX;
  }
  // tile of this workgroup: XCD b mod 8 takes the b-th eighth of the tiles, lines fastest
  const int ntile = txn * tyn * tzn, per = (ntile + 7) >> 3;
  const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (tile >= ntile) return;  // uniform: the whole workgroup leaves before any barrier
  const int ty = tile % tyn, tx = (tile / tyn) % txn, tz = tile / (tyn * txn);
  const int lx = t & 63, ly = t >> 6;
  // load slot 0: this thread's own pair; slot 1 (t < 140): a halo pair (two halo lines of 64,
  // then the left / right halo pair of each of the 6 tile lines)
  int sx[2], sy[2], spos[2];
  sx[0] = tx * kMarchTX + lx;
  sy[0] = ty * kMarchTY + ly;
  spos[0] = (ly + 1) * kMarchLX + lx + 1;
  {
    int line, xp;
    if (t < 128) {
      line = t < 64 ? 0 : kMarchLY - 1;
      xp = lx + 1;
    } else {
      const int e = t - 128;
      line = e >> 1;
      xp = (e & 1) ? kMarchLX - 1 : 0;
    }
    sx[1] = tx * kMarchTX + xp - 1;
    sy[1] = ty * kMarchTY + line - 1;
    spos[1] = line * kMarchLX + xp;
  }
  bool sok[2];
  int soff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    sok[h] = (h == 0 || t < 140) && sx[h] >= 0 && sx[h] < mg.nxp && sy[h] >= 0 && sy[h] < mg.nyl;
    soff[h] = sok[h] ? sy[h] * mg.nxp + sx[h] : 0;
  }
  const bool own = sok[0];
  const int z0 = tz * sz, z1 = min(z0 + sz, mg.nz);
  const int k = Y.ncols;
  __syncthreads();  // dictionary and groups

  for (int c0 = 0; c0 < k; c0 += KC) {
    const int kc = min(KC, k - c0);
    const double *xc[KC];
    double *yc[KC];
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      xc[c] = colp(X, c0 + (c < kc ? c : 0));
      yc[c] = colp(Y, c0 + (c < kc ? c : 0));
    }
    auto products = [&](int z, int tz_) __attribute__((always_inline)) {
      const long long p = (long long)z * mg.plane + soff[0];
      if (own && tz_ != 0xFF) {
        double sa[KC], sb[KC];
#pragma unroll
        for (int c = 0; c < KC; ++c) sa[c] = sb[c] = 0.0;
        // not unrolled: unrolled, all groups' operands and coefficients are hoisted (256 VGPRs)
#pragma unroll 1
        for (int g = 0; g < G; ++g) {
          const unsigned long long sl = s_grp[tz_ * G + g];
          const unsigned s0 = sl & 0xFF, s1 = (sl >> 8) & 0xFF, s2 = (sl >> 16) & 0xFF;
          const unsigned s3 = (sl >> 24) & 0xFF, s4 = (sl >> 32) & 0xFF, s5 = (sl >> 40) & 0xFF;
          const double w0 = s_val[s0], w1 = s_val[s1], w2 = s_val[s2];
          const double w3 = s_val[s3], w4 = s_val[s4], w5 = s_val[s5];
          const d2 *b = ring + ((z + s_gz[g]) & 3) * (KC * kMarchPl) + s_gl[g] + (ly + 1) * kMarchLX + lx + 1;
#pragma unroll
          for (int c = 0; c < KC; ++c) {
            const d2 x = b[c * kMarchPl];
            const double left = b[c * kMarchPl - 1].y;   // row 0's x - 1
            const double right = b[c * kMarchPl + 1].x;  // row 1's x + 1
            const double pa0 = w0 * left, pa1 = w1 * x.x, pa2 = w2 * x.y;
            const double pb0 = w3 * x.x, pb1 = w4 * x.y, pb2 = w5 * right;
            sa[c] = sa[c] + (s0 != 0xFF ? pa0 : 0.0);
            sa[c] = sa[c] + (s1 != 0xFF ? pa1 : 0.0);
            sa[c] = sa[c] + (s2 != 0xFF ? pa2 : 0.0);
            sb[c] = sb[c] + (s3 != 0xFF ? pb0 : 0.0);
            sb[c] = sb[c] + (s4 != 0xFF ? pb1 : 0.0);
            sb[c] = sb[c] + (s5 != 0xFF ? pb2 : 0.0);
          }
        }
        const long long ra = 2 * p;
        const bool hasb = ra + 1 < n_local;
#pragma unroll
        for (int c = 0; c < KC; ++c) {
          if (c >= kc) break;
          double *yp = yc[c] + ra;
          double a = sa[c], bb = sb[c];
          if (beta == 0.0) {
            if (alpha != 1.0) {
              a = alpha * a;
              bb = alpha * bb;
            }
          } else {
            a = alpha * a + beta * yp[0];
            if (hasb) bb = alpha * bb + beta * yp[1];
          }
          if (hasb)
            *(d2 *)yp = d2{a, bb};
          else
            yp[0] = a;
        }
      }
    };
    // one plane's registers: both load slots' KC operands, their column scale, the own pair's
    // template id
    struct PlaneRegs {
      d2 v[2][KC];
      d2 sc[2];
      int tid;
    };
    // loads of plane q (zeros outside the local pairs)
    auto load = [&](PlaneRegs &r, int q) __attribute__((always_inline)) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const long long pr = (long long)q * mg.plane + soff[h];
        const bool ok = sok[h] && q >= 0 && q < mg.nz && pr < npairs;
        const long long pc = ok ? pr : 0;
#pragma unroll
        for (int c = 0; c < KC; ++c) r.v[h][c] = (ok && c < kc) ? *(const d2 *)(xc[c] + 2 * pc) : d2{0.0, 0.0};
        if (cs) r.sc[h] = ok ? *(const d2 *)(cs + 2 * pc) : d2{0.0, 0.0};
      }
      const long long pr = (long long)q * mg.plane + soff[0];
      r.tid = (own && q >= 0 && q < mg.nz && pr < npairs) ? (int)tid[pr] : 0xFF;
    };
    auto stage = [&](const PlaneRegs &r, int q) __attribute__((always_inline)) {  // -> ring slot of plane q
      d2 *d = ring + (size_t)(q & 3) * KC * kMarchPl;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && t >= 140) break;
#pragma unroll
        for (int c = 0; c < KC; ++c) d[c * kMarchPl + spos[h]] = cs ? r.sc[h] * r.v[h][c] : r.v[h][c];
      }
    };
    if (c0 > 0) march_barrier();  // the previous chunk's last plane has been read
    PlaneRegs ra, rb;
    load(ra, z0 - 1);
    stage(ra, z0 - 1);
    load(ra, z0);
    stage(ra, z0);
    int tcur = ra.tid;
    load(ra, z0 + 1);
    if (PD == 2) load(rb, z0 + 2);
    // plane z: stage plane z + 1 from r, refill r with plane z + 1 + PD (in flight through this
    // plane's products and, with PD = 2, the next one's), one barrier, the products
    auto step = [&](int z, PlaneRegs &r) __attribute__((always_inline)) {
      stage(r, z + 1);
      const int tz_ = tcur;
      tcur = r.tid;
      load(r, z + 1 + PD);
      march_barrier();
      products(z, tz_);
    };
    for (int z = z0; z < z1; z += 2) {
      step(z, ra);
      if (z + 1 < z1) step(z + 1, PD == 2 ? rb : ra);
    }
  }
}

template <int KC, int G>
static void march_cols(hipStream_t s, int npairs, int n_local, const unsigned char *tid,
                       const unsigned long long *grp, int ngrp, const MarchGeom &g, int sz, int pd,
                       const double *vals, int nvals, MvDesc X, MvDesc Y, double alpha, double beta,
                       const double *cs) {
  const int txn = cdiv(g.nxp, kMarchTX), tyn = cdiv(g.nyl, kMarchTY), tzn = cdiv(g.nz, sz);
  const int ntile = txn * tyn * tzn;
  const size_t lds = sizeof(d2) * 4 * KC * kMarchPl + sizeof(double) * 256 + sizeof(unsigned long long) * ngrp;
  const int grid = 8 * ((ntile + 7) / 8);
  if (pd == 2)
    k_spmm_march<KC, G, 2><<<grid, 256, lds, s>>>(npairs, n_local, tid, grp, ngrp, g, txn, tyn, tzn, sz, vals, nvals,
                                                   X, Y, alpha, beta, cs);
  else
    k_spmm_march<KC, G, 1><<<grid, 256, lds, s>>>(npairs, n_local, tid, grp, ngrp, g, txn, tyn, tzn, sz, vals, nvals,
                                                   X, Y, alpha, beta, cs);
}

bool launch_spmm_march(hipStream_t s, int n_local, const unsigned char *tid, const unsigned long long *grp, int ntpl,
                       int G, const MarchGeom &geom, const double *vals, int nvals, MvDesc X, MvDesc Y, double alpha,
                       double beta, const double *colscale, int kcmax, int sz, int pd) {
  const int npairs = (n_local + 1) / 2;
  if (npairs <= 0 || Y.ncols <= 0) return true;
  if (G != 9 && G != 5 && G != 3) return false;
  if (geom.nxp <= 0 || geom.nyl <= 0 || geom.plane != geom.nxp * geom.nyl ||
      (long long)geom.nz * geom.plane < npairs)
    return false;
  const int ngrp = ntpl * G;
  if (sz <= 0) {
    // z slabs: about one resident round of workgroups, at least 8 planes per slab
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    }
    const int per_cu = kcmax >= 2 ? 3 : 6;
    const long long cols = (long long)cdiv(geom.nxp, kMarchTX) * cdiv(geom.nyl, kMarchTY);
    const long long slabs = std::max(1LL, std::min((long long)cus * per_cu / cols, (long long)cdiv(geom.nz, 8)));
    sz = cdiv(geom.nz, slabs);
  }
#define MARCH(KC)                                                                                                 \
  if (G == 9)                                                                                                     \
    march_cols<KC, 9>(s, npairs, n_local, tid, grp, ngrp, geom, sz, pd, vals, nvals, X, Y, alpha, beta, colscale);     \
  else if (G == 5)                                                                                                \
    march_cols<KC, 5>(s, npairs, n_local, tid, grp, ngrp, geom, sz, pd, vals, nvals, X, Y, alpha, beta, colscale);     \
  else                                                                                                            \
    march_cols<KC, 3>(s, npairs, n_local, tid, grp, ngrp, geom, sz, pd, vals, nvals, X, Y, alpha, beta, colscale);
  if (kcmax >= 2 && Y.ncols >= 2) {
    MARCH(2)
  } else {
    MARCH(1)
  }
#undef MARCH
  LAUNCH_CHECK();
  return true;
}

// -------------------------------------------------------------------------------------
// The march for the 7-point pattern (groups (z-1), (y-1), the x line, (y+1), (z+1); only the
// x line reads neighbour halves): measured, the general march is bound by its LDS reads --
// per pair and column one group word, six dictionary lookups and three operand reads per group,
// about 50 LDS instructions, more than the 7 global loads it saves.  Here:
//  * the coefficients live in registers: a template's 30 values (5 groups x 6 slots, 0 where
//    unused) are read from an LDS table only when a lane's template changes between planes
//    (interior pairs keep theirs for the whole slab);
//  * only plane z is staged (a 3-slot ring, one barrier per plane): the (z - 1) and (z + 1)
//    centres are the lane's own pair, kept in registers from its loads, so a pair and column
//    costs 4 LDS reads (the y - 1 and y + 1 centres, the left and right halves);
//  * PD planes of loads are in flight (registers), and workgroups take one column at a time.
// Products and order are k_spmm_tpl3's (the slots the host check found unused in every
// template -- the (z +- 1), (y +- 1) groups' neighbour halves -- would add +0.0, which leaves a
// running sum that starts at +0.0 unchanged): the same bits.
// -------------------------------------------------------------------------------------
template <int PD, bool CS, int NL, bool UNI>
__global__ __launch_bounds__(256) void k_spmm_march7(int npairs, int n_local, const unsigned char *__restrict__ tid,
                                                     const unsigned long long *__restrict__ grp, int ntpl,
                                                     MarchGeom mg, int txn, int tyn, int tzn, int sz,
                                                     const double *__restrict__ vals, int nvals, MvDesc X, MvDesc Y,
                                                     double alpha, double beta, const double *__restrict__ cs,
                                                     March27Coef U) {
#pragma clang fp contract(off)
  // NL lines per thread: tile of 64 pairs x 4 NL lines, staged with a one-pair / one-line halo
  constexpr int TY = 4 * NL, LY = TY + 2, PL = LY * kMarchLX, NH = 128 + 2 * LY, NS = NL + 1;
  extern __shared__ __attribute__((aligned(16))) double march_lds[];
  d2 *ring = (d2 *)march_lds;                          // [3][LY][kMarchLX]
  double *s_coef = march_lds + 2 * 3 * PL;             // [ntpl][30]
  unsigned *s_mask = (unsigned *)(s_coef + 30 * ntpl);  // [ntpl]: bit 6 g + i = slot i of group g used
  const int t = threadIdx.x;
  for (int e = t; e < 30 * ntpl; e += 256) {
    const int tt = e / 30, r = e % 30;
    const unsigned sl = (unsigned)(grp[tt * 5 + r / 6] >> (8 * (r % 6))) & 0xFF;
    s_coef[e] = (sl != 0xFF && (int)sl < nvals) ? vals[sl] : 0.0;
  }
  for (int tt = t; tt < ntpl; tt += 256) {
    unsigned m = 0;
    for (int r = 0; r < 30; ++r) m |= (((unsigned)(grp[tt * 5 + r / 6] >> (8 * (r % 6))) & 0xFF) != 0xFF ? 1u : 0u) << r;
    s_mask[tt] = m;
  }
  // work item = (column, tile): XCD b mod 8 takes the b-th eighth, lines fastest, so a tile's
  // line halo was usually just loaded by its neighbour on the same XCD
  const int ntile = txn * tyn * tzn, nwork = ntile * Y.ncols, per = (nwork + 7) >> 3;
  const int work = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (work >= nwork) return;  // uniform
  const int c = work / ntile, tile = work % ntile;
  const int ty = tile % tyn, tx = (tile / tyn) % txn, tz = tile / (tyn * txn);
  const int lx = t & 63, ly = t >> 6;
  // load slots: i < NL this thread's own pair on tile line ly + 4 i; NL: a halo pair (t < NH:
  // the two halo lines, then the left / right halo pair of each staged line)
  int spos[NS], soff[NS];
  bool sok[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    int line, xp;
    if (i < NL) {
      line = ly + 4 * i + 1;
      xp = lx + 1;
    } else if (t < 128) {
      line = t < 64 ? 0 : LY - 1;
      xp = lx + 1;
    } else {
      const int e = t - 128;
      line = e >> 1;
      xp = (e & 1) ? kMarchLX - 1 : 0;
    }
    const int gx = tx * kMarchTX + xp - 1, gy = ty * TY + line - 1;
    sok[i] = (i < NL || t < NH) && gx >= 0 && gx < mg.nxp && gy >= 0 && gy < mg.nyl;
    soff[i] = sok[i] ? gy * mg.nxp + gx : 0;
    spos[i] = line * kMarchLX + xp;
  }
  const int z0 = tz * sz, z1 = min(z0 + sz, mg.nz);
  __syncthreads();  // coefficient table

  double w[30];
  unsigned msk = 0;
  int tcoef = -1;
  struct PlaneRegs {
    d2 v[NS];
    d2 sc[CS ? NS : 1];
    int tid[NL];
  };
  const double *xc = colp(X, c);
  double *yc = colp(Y, c);
  auto load = [&](PlaneRegs &r, int q) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < NS; ++h) {
      const long long pr = (long long)q * mg.plane + soff[h];
      const bool ok = sok[h] && q >= 0 && q < mg.nz && pr < npairs;
      const long long pc = ok ? pr : 0;
      r.v[h] = ok ? *(const d2 *)(xc + 2 * pc) : d2{0.0, 0.0};
      if constexpr (CS) r.sc[h] = ok ? *(const d2 *)(cs + 2 * pc) : d2{0.0, 0.0};
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const long long pr = (long long)q * mg.plane + soff[i];
      // tid == null (uniform stencil, every pair templated): no per-pair template byte to read
      r.tid[i] = (sok[i] && q >= 0 && q < mg.nz && pr < npairs) ? (tid ? (int)tid[pr] : 0) : 0xFF;
    }
  };
  auto operand = [&](const PlaneRegs &r, int h) __attribute__((always_inline)) {
    d2 o = r.v[h];
    if constexpr (CS) o = r.sc[h] * r.v[h];
    return o;
  };
  // plane q -> ring slot s; the own lines' (scaled) operands go to o (the lanes' z +- 1 centres)
  auto stage = [&](const PlaneRegs &r, int s, d2 (&o)[NL]) __attribute__((always_inline)) {
    d2 *d = ring + s * PL;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      o[i] = operand(r, i);
      d[spos[i]] = o[i];
    }
    if (t < NH) d[spos[NL]] = operand(r, NL);
  };
  PlaneRegs rb[PD];
  d2 om[NL], oz[NL], op[NL];  // own operands of planes z - 1, z, z + 1
  int tc[NL];
  {
    PlaneRegs r0;
    load(r0, z0 - 1);
#pragma unroll
    for (int i = 0; i < NL; ++i) om[i] = operand(r0, i);
    load(r0, z0);
    stage(r0, z0 % 3, oz);
#pragma unroll
    for (int i = 0; i < NL; ++i) tc[i] = r0.tid[i];
  }
#pragma unroll
  for (int i = 0; i < PD; ++i) load(rb[i], z0 + 1 + i);
  // plane z: stage z + 1 from rb[i] into slot (z + 1) % 3, refill rb[i] with plane z + 1 + PD,
  // one barrier, then plane z's products (reading slot z % 3)
  int sz3 = z0 % 3;
  for (int z = z0; z < z1; z += PD) {
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      const int zz = z + i;
      if (zz < z1) {
        const int sn = sz3 == 2 ? 0 : sz3 + 1;
        stage(rb[i], sn, op);
        int tzz[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) {
          tzz[l] = tc[l];
          tc[l] = rb[i].tid[l];
        }
        load(rb[i], zz + 1 + PD);
        march_barrier();
#pragma unroll
        for (int l = 0; l < NL; ++l) {
          const int tl = tzz[l];
          if (tl != 0xFF) {
            if (!UNI && tl != tcoef) {  // the lines of a tile share a template away from the grid edges
#pragma unroll
              for (int r = 0; r < 30; ++r) w[r] = s_coef[tl * 30 + r];
              msk = s_mask[tl];
              tcoef = tl;
            }
            const d2 *b = ring + sz3 * PL + spos[l];
            const d2 ym = b[-kMarchLX], yp = b[kMarchLX];
            const double left = b[-1].y, right = b[1].x;
            const d2 ctr[5] = {om[l], ym, oz[l], yp, op[l]};
            double sa = 0.0, sb = 0.0;
            if constexpr (UNI) {
              // uniform stencil with the full 7-point pattern (kMarch7Used: the x line's six
              // slots, c.lo / c.hi for the y / z groups): every pair adds the full template's
              // products (absent entries read out-of-grid zeros) with the coefficients as kernel
              // constants -- no per-slot tests (measured: the runtime tests were ~95 scalar
              // instructions per 64 pairs and column, more than the VALU work)
              auto uw = [&](int g, int i) __attribute__((always_inline)) { return U.w[g][i]; };
              auto on = [&](int g, int i) __attribute__((always_inline)) { return ((kMarch7Used >> (6 * g + i)) & 1ULL) != 0; };
#pragma unroll
              for (int g = 0; g < 5; ++g) {
                const d2 x = ctr[g];
                if (g == 2 && on(2, 0)) sa = sa + uw(2, 0) * left;
                if (on(g, 1)) sa = sa + uw(g, 1) * x.x;
                if (on(g, 2)) sa = sa + uw(g, 2) * x.y;
                if (on(g, 3)) sb = sb + uw(g, 3) * x.x;
                if (on(g, 4)) sb = sb + uw(g, 4) * x.y;
                if (g == 2 && on(2, 5)) sb = sb + uw(2, 5) * right;
              }
            } else {
#pragma unroll
              for (int g = 0; g < 5; ++g) {
                const d2 x = ctr[g];
                if (g == 2) sa = sa + ((msk >> 12) & 1u ? w[12] * left : 0.0);
                sa = sa + ((msk >> (6 * g + 1)) & 1u ? w[6 * g + 1] * x.x : 0.0);
                sa = sa + ((msk >> (6 * g + 2)) & 1u ? w[6 * g + 2] * x.y : 0.0);
                sb = sb + ((msk >> (6 * g + 3)) & 1u ? w[6 * g + 3] * x.x : 0.0);
                sb = sb + ((msk >> (6 * g + 4)) & 1u ? w[6 * g + 4] * x.y : 0.0);
                if (g == 2) sb = sb + ((msk >> 17) & 1u ? w[17] * right : 0.0);
              }
            }
            const long long ra = 2 * ((long long)zz * mg.plane + soff[l]);
            double *yq = yc + ra;
            if (beta == 0.0) {
              if (alpha != 1.0) {
                sa = alpha * sa;
                sb = alpha * sb;
              }
            } else {
              sa = alpha * sa + beta * yq[0];
              if (ra + 1 < n_local) sb = alpha * sb + beta * yq[1];
            }
            if (ra + 1 < n_local)
              *(d2 *)yq = d2{sa, sb};
            else
              yq[0] = sa;
          }
          om[l] = oz[l];
          oz[l] = op[l];
        }
        sz3 = sn;
      }
    }
  }
}

bool launch_spmm_march7(hipStream_t s, int n_local, const unsigned char *tid, const unsigned long long *grp, int ntpl,
                        const MarchGeom &geom, const double *vals, int nvals, MvDesc X, MvDesc Y, double alpha,
                        double beta, const double *colscale, int sz, int pd, int nl, const March27Coef *uni,
                        bool all_templated) {
  const int npairs = (n_local + 1) / 2;
  if (npairs <= 0 || Y.ncols <= 0) return true;
  if (geom.nxp <= 0 || geom.nyl <= 0 || geom.plane != geom.nxp * geom.nyl ||
      (long long)geom.nz * geom.plane < npairs)
    return false;
  nl = nl == 2 ? 2 : 1;
  const int TY = 4 * nl;
  if (sz <= 0) {
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    }
    // slabs: about MIGMRES_MARCH_WPC (default 2) work items per CU over all (column, tile) work
    // items, at least 8 planes per slab (each slab re-reads 2 halo planes).  With 8-line tiles,
    // same box (profiles/r4_knob_sweeps.txt, sweep_r4m_* / sweep_r4n_*): 256^3 SpMM x 8 0.449 ->
    // 0.420 ms (one 256-plane slab instead of five), and the 8-GPU per-rank shapes 0.054 ->
    // 0.047 ms (256 x 256 x 32: one slab) and 0.049 ms (128^3: 32-plane slabs).
    static const int wpc = [] {
      const char *e = std::getenv("MIGMRES_MARCH_WPC");
      const int v = e ? std::atoi(e) : 2;
      return v > 0 ? v : 2;
    }();
    const long long cols = (long long)cdiv(geom.nxp, kMarchTX) * cdiv(geom.nyl, TY) * Y.ncols;
    const long long slabs = std::max(1LL, std::min((long long)cdiv((long long)wpc * cus, cols), (long long)cdiv(geom.nz, 8)));
    sz = cdiv(geom.nz, slabs);
  }
  const int txn = cdiv(geom.nxp, kMarchTX), tyn = cdiv(geom.nyl, TY), tzn = cdiv(geom.nz, sz);
  const int ntile = txn * tyn * tzn * Y.ncols;
  const size_t lds =
      sizeof(d2) * 3 * (TY + 2) * kMarchLX + sizeof(double) * 30 * ntpl + sizeof(unsigned) * ntpl;
  const int grid = 8 * ((ntile + 7) / 8);
  const March27Coef U = uni ? *uni : March27Coef{};
  // uniform stencil with every pair templated: the kernel needs no template id (the k-fold
  // re-read of the N/2-byte id array, 2.6 % of the launch's bytes at k = 8)
  static const bool keep_tid = [] {
    const char *e = std::getenv("MIGMRES_MARCH7_TID");
    return e && e[0] == '1';
  }();
  if (uni && all_templated && !keep_tid) tid = nullptr;
#define M7U(PD, NL, UNI)                                                                                              \
  if (colscale)                                                                                                       \
    k_spmm_march7<PD, true, NL, UNI><<<grid, 256, lds, s>>>(npairs, n_local, tid, grp, ntpl, geom, txn, tyn, tzn,    \
                                                            sz, vals, nvals, X, Y, alpha, beta, colscale, U);         \
  else                                                                                                                \
    k_spmm_march7<PD, false, NL, UNI><<<grid, 256, lds, s>>>(npairs, n_local, tid, grp, ntpl, geom, txn, tyn, tzn,   \
                                                             sz, vals, nvals, X, Y, alpha, beta, colscale, U)
#define M7(PD, NL)     \
  if (uni) {           \
    M7U(PD, NL, true); \
  } else {             \
    M7U(PD, NL, false);\
  }
  if (nl == 2) {
    if (pd >= 3) {
      M7(3, 2)
    } else if (pd == 2) {
      M7(2, 2)
    } else {
      M7(1, 2)
    }
  } else {
    if (pd >= 3) {
      M7(3, 1)
    } else if (pd == 2) {
      M7(2, 1)
    } else {
      M7(1, 1)
    }
  }
#undef M7
#undef M7U
  LAUNCH_CHECK();
  return true;
}

__global__ __launch_bounds__(256) void k_march_check(int npairs, const unsigned char *__restrict__ tid,
                                                     const int4 *__restrict__ tb, int nxp, int nyl,
                                                     int *__restrict__ bad) {
  int n = 0;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < npairs; p += gridDim.x * 256) {
    const int t = tid[p];
    if (t == 0xFF) continue;
    const int x = p % nxp, y = (p / nxp) % nyl;
    const int4 b = tb[t];
    n += (b.x && x == 0) || (b.y && x == nxp - 1) || y + b.z < 0 || y + b.w >= nyl;
  }
  for (int off = 32; off > 0; off >>= 1) n += __shfl_down(n, off, 64);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(bad, n);
}

// -------------------------------------------------------------------------------------
// The march for the 27-point pattern (groups: every (plane, line) offset in {-1, 0, 1}^2) when
// the stencil is UNIFORM: one coefficient table U[9][6] (the full template's) serves every
// templated pair, and each slot a template does not use reads a neighbour outside the grid,
// whose staged operand is zero (march27_check verifies both per pair).  Then every pair adds
// all 54 products in k_spmm_tpl3's order -- an absent entry contributes U * 0 = +-0, which
// leaves a running sum that starts at +0.0 unchanged -- with no per-lane coefficients or
// masks: U sits in scalar registers / the constant cache.  Planes z - 1, z and z + 1 are read
// from a 4-slot LDS ring (one barrier per plane); PD planes of loads in flight; one column per
// workgroup.  Same bits as k_spmm_tpl3.
// -------------------------------------------------------------------------------------
template <int PD, bool CS, bool TWO>
__global__ __launch_bounds__(256) void k_spmm_march27(int npairs, int n_local, const unsigned char *__restrict__ tid,
                                                      MarchGeom mg, int txn, int tyn, int tzn, int sz, March27Coef U,
                                                      MvDesc X, MvDesc Y, double alpha, double beta,
                                                      const double *__restrict__ cs) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) d2 ring[4 * kMarchPl];  // [4][kMarchLY][kMarchLX]
  const int t = threadIdx.x;
  const int ntile = txn * tyn * tzn, nwork = ntile * Y.ncols, per = (nwork + 7) >> 3;
  const int work = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (work >= nwork) return;  // uniform
  const int c = work / ntile, tile = work % ntile;
  const int ty = tile % tyn, tx = (tile / tyn) % txn, tz = tile / (tyn * txn);
  const int lx = t & 63, ly = t >> 6;
  int spos[2], soff[2];
  bool sok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int line, xp;
    if (i == 0) {
      line = ly + 1;
      xp = lx + 1;
    } else if (t < 128) {
      line = t < 64 ? 0 : kMarchLY - 1;
      xp = lx + 1;
    } else {
      const int e = t - 128;
      line = e >> 1;
      xp = (e & 1) ? kMarchLX - 1 : 0;
    }
    const int gx = tx * kMarchTX + xp - 1, gy = ty * kMarchTY + line - 1;
    sok[i] = (i == 0 || t < 140) && gx >= 0 && gx < mg.nxp && gy >= 0 && gy < mg.nyl;
    soff[i] = sok[i] ? gy * mg.nxp + gx : 0;
    spos[i] = line * kMarchLX + xp;
  }
  const int z0 = tz * sz, z1 = min(z0 + sz, mg.nz);
  struct PlaneRegs {
    d2 v[2];
    d2 sc[CS ? 2 : 1];
    int tid;
  };
  const double *xc = colp(X, c);
  double *yc = colp(Y, c);
  auto load = [&](PlaneRegs &r, int q) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const long long pr = (long long)q * mg.plane + soff[h];
      const bool ok = sok[h] && q >= 0 && q < mg.nz && pr < npairs;
      const long long pc = ok ? pr : 0;
      r.v[h] = ok ? *(const d2 *)(xc + 2 * pc) : d2{0.0, 0.0};
      if constexpr (CS) r.sc[h] = ok ? *(const d2 *)(cs + 2 * pc) : d2{0.0, 0.0};
    }
    const long long pr = (long long)q * mg.plane + soff[0];
    // tid == null (every pair templated): no per-pair template byte to read
    r.tid = (sok[0] && q >= 0 && q < mg.nz && pr < npairs) ? (tid ? (int)tid[pr] : 0) : 0xFF;
  };
  auto stage = [&](const PlaneRegs &r, int q) __attribute__((always_inline)) {
    d2 *d = ring + (q & 3) * kMarchPl;
    d2 o0 = r.v[0], o1 = r.v[1];
    if constexpr (CS) {
      o0 = r.sc[0] * r.v[0];
      o1 = r.sc[CS ? 1 : 0] * r.v[1];
    }
    d[spos[0]] = o0;
    if (t < 140) d[spos[1]] = o1;
  };
  PlaneRegs rb[PD];
  int tc;
  {
    PlaneRegs r0;
    load(r0, z0 - 1);
    stage(r0, z0 - 1);
    load(r0, z0);
    stage(r0, z0);
    tc = r0.tid;
  }
#pragma unroll
  for (int i = 0; i < PD; ++i) load(rb[i], z0 + 1 + i);
  for (int z = z0; z < z1; z += PD) {
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      const int zz = z + i;
      if (zz < z1) {
        stage(rb[i], zz + 1);
        const int tzz = tc;
        tc = rb[i].tid;
        load(rb[i], zz + 1 + PD);
        march_barrier();
        if (tzz != 0xFF) {
          double sa = 0.0, sb = 0.0;
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            const d2 *pl = ring + ((zz + a - 1) & 3) * kMarchPl + spos[0];
#pragma unroll
            for (int bq = 0; bq < 3; ++bq) {
              const int g = 3 * a + bq;
              const d2 *b = pl + (bq - 1) * kMarchLX;
              const d2 x = b[0];
              const double left = b[-1].y, right = b[1].x;
              // TWO: the Brick3D pattern (kMarch27Diag: v2[1] on the two diagonal slots, v2[0]
              // elsewhere) fixed at compile time -- no per-slot scalar selects
              auto w = [&](int i) __attribute__((always_inline)) {
                return TWO ? ((kMarch27Diag >> (6 * g + i)) & 1ULL ? U.v2[1] : U.v2[0]) : U.w[g][i];
              };
              sa = sa + w(0) * left;
              sa = sa + w(1) * x.x;
              sa = sa + w(2) * x.y;
              sb = sb + w(3) * x.x;
              sb = sb + w(4) * x.y;
              sb = sb + w(5) * right;
            }
          }
          const long long ra = 2 * ((long long)zz * mg.plane + soff[0]);
          double *yq = yc + ra;
          if (beta == 0.0) {
            if (alpha != 1.0) {
              sa = alpha * sa;
              sb = alpha * sb;
            }
          } else {
            sa = alpha * sa + beta * yq[0];
            if (ra + 1 < n_local) sb = alpha * sb + beta * yq[1];
          }
          if (ra + 1 < n_local)
            *(d2 *)yq = d2{sa, sb};
          else
            yq[0] = sa;
        }
      }
    }
  }
}

bool launch_spmm_march27(hipStream_t s, int n_local, const unsigned char *tid, const MarchGeom &geom,
                         const March27Coef &U, MvDesc X, MvDesc Y, double alpha, double beta, const double *colscale,
                         int sz, int pd, bool all_templated) {
  const int npairs = (n_local + 1) / 2;
  if (npairs <= 0 || Y.ncols <= 0) return true;
  if (geom.nxp <= 0 || geom.nyl <= 0 || geom.plane != geom.nxp * geom.nyl ||
      (long long)geom.nz * geom.plane < npairs)
    return false;
  if (sz <= 0) {
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    }
    const long long cols = (long long)cdiv(geom.nxp, kMarchTX) * cdiv(geom.nyl, kMarchTY) * Y.ncols;
    // (about 9 work items per CU; 2 or 4, which helped the 7-point march, measured equal here:
    // Brick3D + Jacobi 256^3 fused SpMM 0.574-0.581 ms either way, sweep_r4p_bj)
    const long long slabs = std::max(1LL, std::min((long long)cdiv(9LL * cus, cols), (long long)cdiv(geom.nz, 4)));
    sz = cdiv(geom.nz, slabs);
  }
  const int txn = cdiv(geom.nxp, kMarchTX), tyn = cdiv(geom.nyl, kMarchTY), tzn = cdiv(geom.nz, sz);
  static const bool keep_tid = [] {
    const char *e = std::getenv("MIGMRES_MARCH7_TID");
    return e && e[0] == '1';
  }();
  if (all_templated && !keep_tid) tid = nullptr;
  const int grid = 8 * ((txn * tyn * tzn * Y.ncols + 7) / 8);
#define M27T(PD, TWO)                                                                                             \
  if (colscale)                                                                                                   \
    k_spmm_march27<PD, true, TWO><<<grid, 256, 0, s>>>(npairs, n_local, tid, geom, txn, tyn, tzn, sz, U, X, Y,    \
                                                       alpha, beta, colscale);                                    \
  else                                                                                                            \
    k_spmm_march27<PD, false, TWO><<<grid, 256, 0, s>>>(npairs, n_local, tid, geom, txn, tyn, tzn, sz, U, X, Y,   \
                                                        alpha, beta, colscale)
#define M27(PD)          \
  if (U.two_valued) {    \
    M27T(PD, true);      \
  } else {               \
    M27T(PD, false);     \
  }
  if (pd >= 3) {
    M27(3)
  } else if (pd == 2) {
    M27(2)
  } else {
    M27(1)
  }
#undef M27
#undef M27T
  LAUNCH_CHECK();
  return true;
}

// Pairs for which the uniform 27-point form would differ: per templated pair, every slot its
// template leaves unused must read a neighbour outside the grid (a staged zero).  umask[t]: the
// template's used slots (bit 6 g + i).
__global__ __launch_bounds__(256) void k_march27_check(int npairs, const unsigned char *__restrict__ tid,
                                                       const unsigned long long *__restrict__ umask, MarchGeom mg,
                                                       int G, unsigned long long skip, int *__restrict__ bad) {
  int n = 0;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < npairs; p += gridDim.x * 256) {
    const int t = tid[p];
    if (t == 0xFF) continue;
    const unsigned long long m = umask[t] | skip;
    const int x = p % mg.nxp, y = (p / mg.nxp) % mg.nyl, z = p / mg.plane;
    for (int g = 0; g < G; ++g)
      for (int i = 0; i < 6; ++i) {
        if ((m >> (6 * g + i)) & 1ull) continue;
        const int xq = x + (i == 0 ? -1 : i == 5 ? 1 : 0), yq = y + mg.gb[g], zq = z + mg.ga[g];
        const bool inside = xq >= 0 && xq < mg.nxp && yq >= 0 && yq < mg.nyl && zq >= 0 && zq < mg.nz &&
                            (long long)zq * mg.plane + (long long)yq * mg.nxp + xq < npairs;
        n += inside ? 1 : 0;
      }
  }
  for (int off = 32; off > 0; off >>= 1) n += __shfl_down(n, off, 64);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(bad, n);
}

int march27_check(hipStream_t s, int npairs, const unsigned char *tid, const unsigned long long *umask, int ntpl,
                  const MarchGeom &geom, int G, unsigned long long skip) {
  if (npairs <= 0) return 0;
  int *d = nullptr;
  unsigned long long *dm = nullptr;
  MIG_HIP(hipMalloc(&d, sizeof(int)));
  MIG_HIP(hipMalloc(&dm, sizeof(unsigned long long) * ntpl));
  MIG_HIP(hipMemcpyAsync(dm, umask, sizeof(unsigned long long) * ntpl, hipMemcpyHostToDevice, s));
  MIG_HIP(hipMemsetAsync(d, 0, sizeof(int), s));
  k_march27_check<<<std::min(cdiv(npairs, 256), 4096), 256, 0, s>>>(npairs, tid, dm, geom, G, skip, d);
  LAUNCH_CHECK();
  int h = 0;
  MIG_HIP(hipMemcpyAsync(&h, d, sizeof(int), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  hipFree(d);
  hipFree(dm);
  return h;
}

int march_check(hipStream_t s, int npairs, const unsigned char *tid, const int4 *tbounds, int ntpl, int nxp,
                int nyl) {
  if (npairs <= 0) return 0;
  int *d = nullptr;
  int4 *dtb = nullptr;
  MIG_HIP(hipMalloc(&d, sizeof(int)));
  MIG_HIP(hipMalloc(&dtb, sizeof(int4) * ntpl));
  MIG_HIP(hipMemcpyAsync(dtb, tbounds, sizeof(int4) * ntpl, hipMemcpyHostToDevice, s));
  MIG_HIP(hipMemsetAsync(d, 0, sizeof(int), s));
  k_march_check<<<std::min(cdiv(npairs, 256), 4096), 256, 0, s>>>(npairs, tid, dtb, nxp, nyl, d);
  LAUNCH_CHECK();
  int h = 0;
  MIG_HIP(hipMemcpyAsync(&h, d, sizeof(int), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  hipFree(d);
  hipFree(dtb);
  return h;
}

void launch_spmm_tpl(hipStream_t s, int n_local, const unsigned char *tid, const int2 *rec, int ntpl, int maxk,
                     const double *vals, int nvals, MvDesc X, MvDesc Y, double alpha, double beta,
                     const double *colscale, int xcd_slabs, int kcmax) {
  const int npairs = (n_local + 1) / 2;
  if (npairs <= 0) return;
  const int nrec = ntpl * maxk;
  const size_t lds = sizeof(double) * 256 + sizeof(int2) * (size_t)nrec;
  const int k = Y.ncols;
  const int kstep = kcmax == 2 ? 2 : kcmax == 4 ? 4 : 8;
  for (int c0 = 0; c0 < k; c0 += kstep) {
    const int kc = (k - c0) < kstep ? (k - c0) : kstep;
    if (kc == 1)
      tpl_cols<1>(s, lds, npairs, n_local, tid, rec, maxk, nrec, vals, nvals, X, Y, c0, kc, alpha, beta, colscale, xcd_slabs);
    else if (kc <= 2)
      tpl_cols<2>(s, lds, npairs, n_local, tid, rec, maxk, nrec, vals, nvals, X, Y, c0, kc, alpha, beta, colscale, xcd_slabs);
    else if (kc <= 4)
      tpl_cols<4>(s, lds, npairs, n_local, tid, rec, maxk, nrec, vals, nvals, X, Y, c0, kc, alpha, beta, colscale, xcd_slabs);
    else
      tpl_cols<8>(s, lds, npairs, n_local, tid, rec, maxk, nrec, vals, nvals, X, Y, c0, kc, alpha, beta, colscale, xcd_slabs);
    LAUNCH_CHECK();
  }
}

// -------------------------------------------------------------------------------------
// C = A^T B (A: nrows x L, B: nrows x kb <= 16) on v_mfma_f64_16x16x4_f64.
// MFMA M = 16 columns of A (one column tile), N = 16 columns of B, K = rows.
// The K index of an MFMA may map to ANY row as long as A and B agree, so each lane loads
// 16 bytes = two consecutive rows of one column straight into the operand layout:
// for 64-row chunk r0 and pair p (0..7), lane l (c = l&15, g = l>>4) holds rows
// r0 + 8p + 2g and +1 of column c; MFMA 2p uses the first, MFMA 2p+1 the second.
// A wave-instruction then reads 16 columns x 64 contiguous bytes, and two consecutive
// instructions consume whole 128-byte lines -- no LDS, no barriers in the main loop.
// Waves stream 64-row chunks (grid-stride, grid sized to residency); blockIdx.y selects a
// group of MAXT column tiles; B's fragment is loaded once per chunk and reused across
// the tiles; the next tile's A fragment is loaded before the current tile's 16 MFMAs.
// The four waves' accumulators are summed through LDS, one partial per workgroup.
// f64 MFMA lane maps: A[i=l&15][k=l>>4], B[k=l>>4][j=l&15], D[row=(l>>4)+4r][col=l&15].
// -------------------------------------------------------------------------------------
constexpr int TN_ROWS = 64;

template <int MAXT>
__global__ __launch_bounds__(256) void k_gemm_tn(MvDesc A, int L, MvDesc B, int kb, int nrows,
                                                 double *__restrict__ partial, int contig) {
  // Branch-free main loop: every multivector keeps its padding rows [nrows, ld) at zero
  // (mv_create clears the allocation; kernels only write rows < nrows), so whole 64-row
  // chunks are read without row guards; columns past L / kb are clamped to a valid column,
  // and their values only reach output rows >= L / columns >= kb, which are not stored.
  __shared__ __attribute__((aligned(16))) double red[2][MAXT * 4][64];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int c = l & 15, g = l >> 4;
  const int ntiles = (L + 15) >> 4;
  const int tpg = (ntiles + gridDim.y - 1) / gridDim.y;  // tiles per group, balanced (<= MAXT)
  const int t0 = blockIdx.y * tpg;
  const int nt = (ntiles - t0) < tpg ? (ntiles - t0) : tpg;
  const long long nchunks = (nrows + TN_ROWS - 1) / TN_ROWS;
  const long long wid = (long long)blockIdx.x * 4 + w, nw = (long long)gridDim.x * 4;

  const double *acol[MAXT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    int col = (t0 + tt) * 16 + c;
    col = col < L ? col : L - 1;
    acol[tt] = colp(A, col) + 2 * g;
  }
  const double *bcol = colp(B, c < kb ? c : kb - 1) + 2 * g;

  d4 acc[MAXT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) acc[tt] = d4{0.0, 0.0, 0.0, 0.0};

  // chunk order: grid-stride (wave wid takes wid, wid + nw, ...), or (contig) workgroup b owns
  // the contiguous range [b nchunks / G, (b + 1) nchunks / G) and its 4 waves interleave in it
  long long cb = wid, ce = nchunks, cs = nw;
  if (contig) {
    cb = nchunks * blockIdx.x / gridDim.x + w;
    ce = nchunks * (blockIdx.x + 1) / gridDim.x;
    cs = 4;
  }
  for (long long ch = cb; ch < ce; ch += cs) {
    const long long r0 = ch * TN_ROWS;
    d2 bq[8], cur[8], nxt[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) bq[p] = *(const d2 *)(bcol + r0 + 8 * p);
#pragma unroll
    for (int p = 0; p < 8; ++p) cur[p] = *(const d2 *)(acol[0] + r0 + 8 * p);
#pragma unroll
    for (int tt = 0; tt < MAXT; ++tt) {
      if (tt < nt) {
        if (tt + 1 < nt) {
#pragma unroll
          for (int p = 0; p < 8; ++p) nxt[p] = *(const d2 *)(acol[tt + 1] + r0 + 8 * p);
        }
#pragma unroll
        for (int p = 0; p < 8; ++p) {
          acc[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(cur[p].x, bq[p].x, acc[tt], 0, 0, 0);
          acc[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(cur[p].y, bq[p].y, acc[tt], 0, 0, 0);
        }
        if (tt + 1 < nt) {
#pragma unroll
          for (int p = 0; p < 8; ++p) cur[p] = nxt[p];
        }
      }
    }
  }
  // sum the four waves' accumulators: (2,3) -> (0,1) -> 0
  if (w >= 2) {
#pragma unroll
    for (int tt = 0; tt < MAXT; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w - 2][tt * 4 + r][l] = acc[tt][r];
  }
  __syncthreads();
  if (w < 2) {
#pragma unroll
    for (int tt = 0; tt < MAXT; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[tt][r] += red[w][tt * 4 + r][l];
  }
  __syncthreads();
  if (w == 1) {
#pragma unroll
    for (int tt = 0; tt < MAXT; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[0][tt * 4 + r][l] = acc[tt][r];
  }
  __syncthreads();
  if (w == 0 && c < kb) {
    double *out = partial + (long long)blockIdx.x * L * kb;
#pragma unroll
    for (int tt = 0; tt < MAXT; ++tt) {
      if (tt < nt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = (t0 + tt) * 16 + g + 4 * r;
          if (i < L) out[i + (long long)c * L] = acc[tt][r] + red[0][tt * 4 + r][l];
        }
      }
    }
  }
}

constexpr int TN_MAXT = 8;

static int tn_resident_blocks() {
  static int cached = 0;
  if (!cached) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_gemm_tn<TN_MAXT>, 256, 0) != hipSuccess ||
        per_cu < 1 || cus < 1)
      return 512;
    cached = per_cu * cus;
  }
  return cached;
}

int gemm_tn_blocks(int nrows, int L) {
  const long long waves = (nrows + TN_ROWS - 1) / TN_ROWS;
  long long b = (waves + 3) / 4;
  int cap = tn_resident_blocks();
  // MIGMRES_TN_COR=1: with several groups of column tiles (L > 16 TN_MAXT) every group's
  // workgroups resident at once (one round) instead of group after group
  static const bool cor = [] {
    const char *e = std::getenv("MIGMRES_TN_COR");
    return e && e[0] == '1';
  }();
  const int ny = L > 0 ? ((L + 15) / 16 + TN_MAXT - 1) / TN_MAXT : 1;
  if (cor && ny > 1) cap = cap / ny > 0 ? cap / ny : 1;
  if (b > cap) b = cap;
  return b < 1 ? 1 : (int)b;
}

void launch_gemm_tn_partial(hipStream_t s, MvDesc A, int L, MvDesc B, int kb, int nrows,
                            double *partial, int nblocks) {
  if (L > 512 || kb > 16) throw Error(MIGMRES_EINVAL, "gemm_tn: L <= 512 and kb <= 16 per launch");
  const int ntiles = (L + 15) / 16;
  static const int contig = [] {  // MIGMRES_TN_CONTIG=1: contiguous chunk range per workgroup
    const char *e = std::getenv("MIGMRES_TN_CONTIG");
    return e ? std::atoi(e) : 0;
  }();
  const dim3 grid(nblocks, (ntiles + TN_MAXT - 1) / TN_MAXT);
  k_gemm_tn<TN_MAXT><<<grid, 256, 0, s>>>(A, L, B, kb, nrows, partial, contig);
  LAUNCH_CHECK();
}

__global__ __launch_bounds__(256) void k_reduce(const double *__restrict__ partial, int nblocks,
                                                int nout, double alpha, double *__restrict__ out) {
  // 64 outputs x 4 slices per workgroup; each thread keeps 4 independent running sums
  // over blocks b = s, s+4, ... so loads stay in flight; fixed combine order.
  __shared__ double red[4][64];
  const int l = threadIdx.x & 63, s = threadIdx.x >> 6;
  const int o = blockIdx.x * 64 + l;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (o < nout) {
    int b = s;
    for (; b + 12 < nblocks; b += 16) {
      a0 += partial[(long long)b * nout + o];
      a1 += partial[(long long)(b + 4) * nout + o];
      a2 += partial[(long long)(b + 8) * nout + o];
      a3 += partial[(long long)(b + 12) * nout + o];
    }
    for (; b < nblocks; b += 4) a0 += partial[(long long)b * nout + o];
  }
  red[s][l] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (s == 0 && o < nout) out[o] = alpha * ((red[0][l] + red[1][l]) + (red[2][l] + red[3][l]));
}

// Partials of nblocks workgroups (block-major: partial[b * nout + o]) summed per output in a
// fixed order: 64 outputs per workgroup and 16 slices (b = s mod 16), each slice with 8 loads in
// flight into 4 running sums, then a fixed tree over the slices.  The 16 x 8 loads in flight
// per output column make it 4 dependent rounds at 512 partial rows (the 4-slice form took 32:
// 14.8 us per launch at 128^3, more than the 2 MB it reads).
constexpr int RLD_S = 16;
__global__ __launch_bounds__(64 * RLD_S) void k_reduce_ld(const double *__restrict__ partial, int nblocks,
                                                          int rows, int nout, int ldo, double alpha,
                                                          double *__restrict__ out) {
  __shared__ double red[RLD_S][64];
  const int l = threadIdx.x & 63, s = threadIdx.x >> 6;
  const int o = blockIdx.x * 64 + l;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  if (o < nout) {
    int b = s;
    for (; b + 7 * RLD_S < nblocks; b += 8 * RLD_S) {
      double x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = partial[(long long)(b + j * RLD_S) * nout + o];
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j & 3] += x[j];
    }
    for (int j = 0; b < nblocks; b += RLD_S, ++j) a[j & 3] += partial[(long long)b * nout + o];
  }
  red[s][l] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
#pragma unroll
  for (int h = RLD_S / 2; h > 0; h >>= 1) {
    if (s < h) red[s][l] = red[s][l] + red[s + h][l];
    __syncthreads();
  }
  if (s == 0 && o < nout)
    out[(o % rows) + (long long)(o / rows) * ldo] = alpha * red[0][l];
}

void launch_reduce_partials_ld(hipStream_t s, const double *partial, int nblocks, int rows, int cols,
                               int ldo, double alpha, double *out) {
  const int nout = rows * cols;
  if (nout <= 0) return;
  k_reduce_ld<<<cdiv(nout, 64), 64 * RLD_S, 0, s>>>(partial, nblocks, rows, nout, ldo, alpha, out);
  LAUNCH_CHECK();
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
      // 8 columns' loads in flight before their FMAs; an odd tail row pairs with the zero
      // padding row (every multivector has ld > n_local), read unguarded
      int jj = 0;
      for (; jj + 8 <= jn; jj += 8) {
        d2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *(const d2 *)(colp(A, j0 + jj + u) + r);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const double *mrow = &Ms[(jj + u) * KX];
#pragma unroll
          for (int c = 0; c < KX; ++c) {
            acc0[c] += v[u].x * mrow[c];
            acc1[c] += v[u].y * mrow[c];
          }
        }
      }
      for (; jj < jn; ++jj) {
        const double *ap = colp(A, j0 + jj) + r;
        const d2 v = *(const d2 *)ap;
        const double a0 = v.x, a1 = v.y;
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
      double n0, n1;
      if (beta == 0.0) {
        n0 = alpha * acc0[c];
        n1 = alpha * acc1[c];
      } else {
        const d2 xo = *(const d2 *)xp;  // padding row of an odd tail reads zero
        n0 = beta * xo.x + alpha * acc0[c];
        n1 = beta * xo.y + alpha * acc1[c];
      }
      if (two) {  // one 16-byte store per lane (two 8-byte stores write every line in halves)
        *(d2 *)xp = d2{n0, n1};
      } else {
        xp[0] = n0;
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

// Import pack / unpack in the exchange layout [neighbour][column][count]: one contiguous
// message per neighbour and apply (Epetra packs row-interleaved per export LID,
// Epetra_MultiVector.cpp:778-783; one message per peer either way).  grp[i] = (offset,
// count) of entry i's neighbour group in the export (or remote) list; entry i of column c
// sits at offset*k + c*count + (i - offset).
__global__ __launch_bounds__(256) void k_pack(MvDesc X, const int *__restrict__ lids,
                                              const int2 *__restrict__ grp, int count, int k,
                                              double *__restrict__ send) {
  const int c = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  const int2 g = grp[i];
  send[(long long)g.x * k + (long long)c * g.y + (i - g.x)] = colp(X, c)[lids[i]];
}
__global__ __launch_bounds__(256) void k_unpack(const double *__restrict__ recv,
                                                const int2 *__restrict__ grp, int count, int k,
                                                double *__restrict__ ghost, long long ldg) {
  const int c = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  const int2 g = grp[i];
  ghost[(long long)c * ldg + i] = recv[(long long)g.x * k + (long long)c * g.y + (i - g.x)];
}

// Point-Jacobi (Ifpack2::Relaxation "Jacobi", Ifpack2_Relaxation_def.hpp:1390-1454).
// dinv[i] = 1 / (first entry of local row i whose local column is i; 0 if none): the owned
// rows come first in the column map, so an owned row's diagonal has local column == row.
__global__ __launch_bounds__(256) void k_diag_inv(const int *__restrict__ rowptr,
                                                  const int *__restrict__ cols,
                                                  const double *__restrict__ vals, int n,
                                                  double *__restrict__ dinv) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  double d = 0.0;
  for (int p = rowptr[r]; p < rowptr[r + 1]; ++p)
    if (cols[p] == r) {
      d = vals[p];
      break;
    }
  dinv[r] = 1.0 / d;
}

// Y = (omega * dinv_i) * X (first sweep from zero) or Y = 1*Y + (omega * dinv_i) * X
// (later sweeps, X = the residual): the KokkosBlas mult expression c*C + (ab*A_i)*B,
// each product and the sum rounded separately.
template <bool ACC>
__global__ __launch_bounds__(256) void k_jacobi(MvDesc X, MvDesc Y, const double *__restrict__ dinv,
                                                double omega, int nrows) {
#pragma clang fp contract(off)
  const int c = blockIdx.y;
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  const double t = (omega * dinv[r]) * colp(X, c)[r];
  double *y = colp(Y, c) + r;
  *y = ACC ? 1.0 * (*y) + t : t;
}

// Ifpack2::Relaxation::compute()'s inverse diagonal (Ifpack2_Relaxation_def.hpp:990-1280):
// the diagonal copy; with l1 (more than one process) d += boost = sum of |a / 2| over the
// entries whose local column index exceeds the local row count (the reference's `>`: the
// first ghost column does not count; a ghost's index is n_present + its slot), when |d| <
// eta boost; then 1 / d, or with fix_tiny 1 / min (1 / eps for min = 0) where |d| <= |min|.
__global__ __launch_bounds__(256) void k_relax_diag(const int *__restrict__ rowptr, const int *__restrict__ cols,
                                                    const double *__restrict__ vals, int n, int n_present, int l1,
                                                    double eta, int fix_tiny, double min_val,
                                                    double *__restrict__ dinv) {
#pragma clang fp contract(off)
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  double d = 0.0;
  for (int p = rowptr[r]; p < rowptr[r + 1]; ++p)
    if (cols[p] == r) {
      d = vals[p];
      break;
    }
  if (l1) {
    double boost = 0.0;
    for (int p = rowptr[r]; p < rowptr[r + 1]; ++p) {
      const int c = cols[p];
      if (c >= n && (long long)n_present + (c - n) > n) boost += fabs(vals[p] / 2.0);
    }
    if (fabs(d) < eta * boost) d += boost;
  }
  if (fix_tiny && fabs(d) <= fabs(min_val))
    dinv[r] = min_val == 0.0 ? 1.0 / 2.220446049250313e-16 : 1.0 / min_val;
  else
    dinv[r] = 1.0 / d;
}

// Ifpack2::Chebyshev's inverse diagonal: reciprocal_threshold of the diagonal copy
// (Ifpack2_Details_Chebyshev_def.hpp:104-115): |d| < |min_val| stores min_val itself.
__global__ __launch_bounds__(256) void k_diag_recip_threshold(const int *__restrict__ rowptr,
                                                              const int *__restrict__ cols,
                                                              const double *__restrict__ vals, int n,
                                                              double min_val, double *__restrict__ dinv) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  double d = 0.0;
  for (int p = rowptr[r]; p < rowptr[r + 1]; ++p)
    if (cols[p] == r) {
      d = vals[p];
      break;
    }
  dinv[r] = fabs(d) < fabs(min_val) ? min_val : 1.0 / d;
}

// The ChebyshevKernel step (Ifpack2_Details_ChebyshevKernel_def.hpp:160-169, 472-480) on a
// residual R = B - A X formed by the SpMM: W = beta W + (alpha d_i) R (BETA) or
// W = (alpha d_i) R, then X = X + W (XMODE 1), X = W (XMODE 2, the zero-start first step)
// or X untouched (XMODE 0); each product and sum rounded separately.
// With B given (B.base != null) R holds A X and the residual b - (A X) is formed here: the
// same bits as the SpMM's -1 * sum + 1 * b, without a copy of B.
template <bool BETA, int XMODE>
__global__ __launch_bounds__(256) void k_cheb_update(MvDesc B, MvDesc R, MvDesc W, MvDesc X,
                                                     const double *__restrict__ dinv, double alpha, double beta,
                                                     int nrows) {
#pragma clang fp contract(off)
  const int c = blockIdx.y;
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  const double res = B.base ? colp(B, c)[r] - colp(R, c)[r] : colp(R, c)[r];
  const double t = (alpha * dinv[r]) * res;
  double *wp = colp(W, c) + r;
  const double w = BETA ? beta * (*wp) + t : t;
  *wp = w;
  if (XMODE == 1) {
    double *xp = colp(X, c) + r;
    *xp = *xp + w;
  } else if (XMODE == 2) {
    colp(X, c)[r] = w;
  }
}

__global__ __launch_bounds__(256) void k_abs(MvDesc Y, int nrows) {
  const int c = blockIdx.y;
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  double *y = colp(Y, c) + r;
  if (*y < 0.0) *y = -*y;
}

// Y = a A + b B with each product and the sum rounded separately (KokkosBlas axpby as the
// textbook Chebyshev's P = Z + beta P and X = X + alpha P evaluate it).
__global__ __launch_bounds__(256) void k_lincomb(double a, MvDesc A, double b, MvDesc B, MvDesc Y, int nrows) {
#pragma clang fp contract(off)
  const int c = blockIdx.y;
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  const double pa = a * colp(A, c)[r], pb = b * colp(B, c)[r];
  colp(Y, c)[r] = pa + pb;
}

__global__ __launch_bounds__(256) void k_scaled_copy(const double *__restrict__ a, double omega, double *out, int n) {
#pragma clang fp contract(off)
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r < n) out[r] = omega * a[r];
}
void launch_scaled_copy(hipStream_t s, const double *a, double omega, double *out, int n) {
  if (n <= 0) return;
  k_scaled_copy<<<cdiv(n, 256), 256, 0, s>>>(a, omega, out, n);
  LAUNCH_CHECK();
}

void launch_diag_inv(hipStream_t s, const int *rowptr, const int *cols, const double *vals, int n,
                     double *dinv) {
  if (n <= 0) return;
  k_diag_inv<<<cdiv(n, 256), 256, 0, s>>>(rowptr, cols, vals, n, dinv);
  LAUNCH_CHECK();
}
void launch_relax_diag(hipStream_t s, const int *rowptr, const int *cols, const double *vals, int n, int n_present,
                       bool l1, double eta, bool fix_tiny, double min_val, double *dinv) {
  if (n <= 0) return;
  k_relax_diag<<<cdiv(n, 256), 256, 0, s>>>(rowptr, cols, vals, n, n_present, l1 ? 1 : 0, eta, fix_tiny ? 1 : 0,
                                            min_val, dinv);
  LAUNCH_CHECK();
}
void launch_diag_recip_threshold(hipStream_t s, const int *rowptr, const int *cols, const double *vals, int n,
                                 double min_val, double *dinv) {
  if (n <= 0) return;
  k_diag_recip_threshold<<<cdiv(n, 256), 256, 0, s>>>(rowptr, cols, vals, n, min_val, dinv);
  LAUNCH_CHECK();
}
void launch_cheb_update(hipStream_t s, MvDesc B, MvDesc R, MvDesc W, MvDesc X, const double *dinv, double alpha,
                        double beta, bool use_beta, int xmode, int nrows) {
  if (nrows <= 0 || W.ncols <= 0) return;
  const dim3 g(cdiv(nrows, 256), W.ncols);
  if (use_beta) {
    if (xmode == 1) k_cheb_update<true, 1><<<g, 256, 0, s>>>(B, R, W, X, dinv, alpha, beta, nrows);
    else if (xmode == 2) k_cheb_update<true, 2><<<g, 256, 0, s>>>(B, R, W, X, dinv, alpha, beta, nrows);
    else k_cheb_update<true, 0><<<g, 256, 0, s>>>(B, R, W, X, dinv, alpha, beta, nrows);
  } else {
    if (xmode == 1) k_cheb_update<false, 1><<<g, 256, 0, s>>>(B, R, W, X, dinv, alpha, beta, nrows);
    else if (xmode == 2) k_cheb_update<false, 2><<<g, 256, 0, s>>>(B, R, W, X, dinv, alpha, beta, nrows);
    else k_cheb_update<false, 0><<<g, 256, 0, s>>>(B, R, W, X, dinv, alpha, beta, nrows);
  }
  LAUNCH_CHECK();
}
void launch_abs(hipStream_t s, MvDesc Y, int nrows) {
  if (nrows <= 0 || Y.ncols <= 0) return;
  k_abs<<<dim3(cdiv(nrows, 256), Y.ncols), 256, 0, s>>>(Y, nrows);
  LAUNCH_CHECK();
}
void launch_lincomb(hipStream_t s, double a, MvDesc A, double b, MvDesc B, MvDesc Y, int nrows) {
  if (nrows <= 0 || Y.ncols <= 0) return;
  k_lincomb<<<dim3(cdiv(nrows, 256), Y.ncols), 256, 0, s>>>(a, A, b, B, Y, nrows);
  LAUNCH_CHECK();
}
void launch_jacobi(hipStream_t s, MvDesc X, MvDesc Y, const double *dinv, double omega, int nrows,
                   bool accumulate) {
  if (nrows <= 0 || Y.ncols <= 0) return;
  if (accumulate)
    k_jacobi<true><<<dim3(cdiv(nrows, 256), Y.ncols), 256, 0, s>>>(X, Y, dinv, omega, nrows);
  else
    k_jacobi<false><<<dim3(cdiv(nrows, 256), Y.ncols), 256, 0, s>>>(X, Y, dinv, omega, nrows);
  LAUNCH_CHECK();
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
void launch_pack(hipStream_t s, MvDesc X, const int *lids, const int2 *grp, int count, double *send, int k) {
  if (count <= 0 || k <= 0) return;
  k_pack<<<dim3(cdiv(count, 256), k), 256, 0, s>>>(X, lids, grp, count, k, send);
  LAUNCH_CHECK();
}
void launch_unpack(hipStream_t s, const double *recv, const int2 *grp, int count, int k, double *ghost,
                   long long ldg) {
  if (count <= 0 || k <= 0) return;
  k_unpack<<<dim3(cdiv(count, 256), k), 256, 0, s>>>(recv, grp, count, k, ghost, ldg);
  LAUNCH_CHECK();
}

// Reverse exchange of the transposed apply (Y = alpha A^T X + beta Y): the contributions one
// neighbour computed for rows this rank owns, in the pack layout [column][count], added to
// rows lids[0 .. count) (distinct within one neighbour's list), neighbour after neighbour.
__global__ __launch_bounds__(256) void k_export_add(MvDesc T, const int *__restrict__ lids, int count,
                                                    const double *__restrict__ recv) {
#pragma clang fp contract(off)
  const int c = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  double *p = colp(T, c) + lids[i];
  *p = *p + recv[(long long)c * count + i];
}
void launch_export_add(hipStream_t s, MvDesc T, const int *lids, int count, int k, const double *recv) {
  if (count <= 0 || k <= 0) return;
  k_export_add<<<dim3(cdiv(count, 256), k), 256, 0, s>>>(T, lids, count, recv);
  LAUNCH_CHECK();
}
// Y = alpha T + beta Y with k_spmm's output rule (beta == 0 ignores Y)
__global__ __launch_bounds__(256) void k_combine(MvDesc T, MvDesc Y, int nrows, double alpha, double beta) {
#pragma clang fp contract(off)
  const int c = blockIdx.y;
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  const double t = colp(T, c)[r];
  double *yp = colp(Y, c) + r;
  if (beta == 0.0)
    *yp = (alpha == 1.0) ? t : alpha * t;
  else
    *yp = alpha * t + beta * (*yp);
}
void launch_combine(hipStream_t s, MvDesc T, MvDesc Y, int nrows, double alpha, double beta) {
  if (nrows <= 0 || Y.ncols <= 0) return;
  k_combine<<<dim3(cdiv(nrows, 256), Y.ncols), 256, 0, s>>>(T, Y, nrows, alpha, beta);
  LAUNCH_CHECK();
}

}  // namespace migmres
