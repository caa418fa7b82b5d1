// Device-resident ICGS building blocks (belos/src/BelosICGSOrthoManager.hpp).
//
// The reference drives ICGS from the host: every inner product is a MvTransMv/MvDot whose
// result comes back to the host before the next update.  Here the coefficients stay in a
// device state block (IcgsState) and every step reads what the previous step reduced, so a
// whole projectAndNormalize is one stream of kernels with a single device-to-host copy at
// the end.  Decisions the reference takes between steps (dependency tests, rank) are
// recorded as flags and acted on by the host afterwards (the fallback restarts from the
// saved input block, exactly as the reference restarts from tmpX).
//
//   k_gemm_nn_dot   X = beta X + alpha A M, plus per-column partials of sum(X_new * D)
//                   (blkOrtho's second update fused with MvDot(X, X), newDot)
//   k_fb_a/b/c      findBasis column j (BelosICGSOrthoManager.hpp:1002-1091): oldDot and
//                   the first projection; first update fused with the second projection;
//                   second update fused with newDot = <Xj, oldMXj>
//   k_fb_scalar     the scalar logic between those steps (diag, dependency flags, B column)
#include "icgs.h"

namespace migmres {

typedef double d2 __attribute__((ext_vector_type(2)));
typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double *colp_(const MvDesc &d, int c) {
  return d.base + (long long)(d.cols ? d.cols[c] : c) * d.ld;
}
static inline int cdiv_(long long a, long long b) { return (int)((a + b - 1) / b); }

#define LAUNCH_CHECK_()                                                                     \
  do {                                                                                      \
    hipError_t e_ = hipGetLastError();                                                      \
    if (e_ != hipSuccess) throw Error(MIGMRES_EHIP, std::string("kernel launch: ") + hipGetErrorString(e_)); \
  } while (0)

// Threads per workgroup of the findBasis / closing-update passes (IC_NT = 256 or 1024; the
// grid covers the CUs with the same number of waves either way).
#ifndef IC_NT
#define IC_NT 1024
#endif
constexpr int ICNT = IC_NT, ICNW = IC_NT / 64;

// Row b of per-workgroup partials (nv <= 17 values) added into v: all 17 loads issued
// unconditionally (indices clamped into the row, values past nv dropped by a select), so
// they are in flight together -- a branch per value made each load wait for the previous.
__device__ __forceinline__ void add_partial_row(double (&v)[17], const double *partial, long long b, int nv) {
  double x[17];
#pragma unroll
  for (int i = 0; i < 17; ++i) x[i] = partial[b * nv + (i < nv ? i : nv - 1)];
#pragma unroll
  for (int i = 0; i < 17; ++i) v[i] += i < nv ? x[i] : 0.0;
}

// Fixed-order block reduction of NV values per thread -> partial[blockIdx.x * nv + i]:
// wave shuffles, then a pairwise tree over the ICNW waves.
template <int NV>
__device__ __forceinline__ void block_reduce_store(double (&v)[NV], int nv, double *partial) {
  __shared__ double red[ICNW][NV];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (i < nv) {
      double x = v[i];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
      if (l == 0) red[w][i] = x;
    }
  }
  __syncthreads();
  if (threadIdx.x < nv) {
    const int i = threadIdx.x;
    double t[ICNW];
#pragma unroll
    for (int q = 0; q < ICNW; ++q) t[q] = red[q][i];
#pragma unroll
    for (int h = 1; h < ICNW; h *= 2)
#pragma unroll
      for (int q = 0; q + h < ICNW; q += 2 * h) t[q] = t[q] + t[q + h];
    partial[(long long)blockIdx.x * nv + i] = t[0];
  }
}

__device__ void fb_scalar_body(IcgsState *st, const double *red, int stage, int j, int k, int complete);

// The pass prologue (FbPro, icgs.h): every workgroup copies the state into LDS, reduces the
// previous pass's partials in a fixed order (the same bits in every workgroup: same data,
// same code) and applies the pending scalar step(s) to its copy; workgroup 0 stores the
// result.  The partials are at most 256 rows x 17 values (35 KB, served from L2 to all but
// the first readers).
__device__ void fb_prologue(const FbPro &p, IcgsState *ls) {
  __shared__ double redv[17];
  __shared__ double wred[ICNW][17];
  constexpr int NWORD = sizeof(IcgsState) / 8;
  static_assert(sizeof(IcgsState) % 8 == 0, "IcgsState is copied in 8-byte words");
  for (int e = threadIdx.x; e < NWORD; e += blockDim.x) ((long long *)ls)[e] = ((const long long *)p.in)[e];
  if (p.stage0 >= 0) {
    if (p.partial) {
      double v[17];
#pragma unroll
      for (int i = 0; i < 17; ++i) v[i] = 0.0;
      for (int b = threadIdx.x; b < p.nblocks; b += blockDim.x) {
        add_partial_row(v, p.partial, b, p.nv);
      }
      const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
      for (int i = 0; i < 17; ++i) {
        if (i < p.nv) {
          double x = v[i];
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
          if (l == 0) wred[w][i] = x;
        }
      }
      __syncthreads();
      if (threadIdx.x < p.nv) {
        const int i = threadIdx.x;
        double t[ICNW];
#pragma unroll
        for (int q = 0; q < ICNW; ++q) t[q] = wred[q][i];
#pragma unroll
        for (int h = 1; h < ICNW; h *= 2)
#pragma unroll
          for (int q = 0; q + h < ICNW; q += 2 * h) t[q] = t[q] + t[q + h];
        redv[i] = t[0];
      }
    } else if (threadIdx.x < p.nv) {
      redv[threadIdx.x] = p.red[threadIdx.x];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      fb_scalar_body(ls, redv, p.stage0, p.j, p.k, p.complete);
      if (p.stage1 >= 0) fb_scalar_body(ls, redv, p.stage1, p.j, p.k, p.complete);
    }
  }
  __syncthreads();
  if (p.stage0 >= 0 && p.out && blockIdx.x == 0)
    for (int e = threadIdx.x; e < NWORD; e += blockDim.x) ((long long *)p.out)[e] = ((const long long *)ls)[e];
}

__global__ __launch_bounds__(ICNT) void k_fb_flush(FbPro pro) {
  __shared__ IcgsState ls;
  fb_prologue(pro, &ls);
}

// 1024 workgroups (4 per CU) stream the findBasis columns at 5.3-5.6 TB/s where 512 gave
// 3.8-4.4 TB/s (tools/mb_lib.cpp, 256^3).
int icgs_blocks(int nrows) {
  constexpr int per = 2048 * (ICNT / 256), cap = 1024 / (ICNT / 256);
  const int b = cdiv_(nrows, per);
  return b < 1 ? 1 : (b > cap ? cap : b);
}

// Store rows (r, r + 1) of a column: one 16-byte store, or only row r when r + 1 == nrows
// (an odd tail).  Two 8-byte stores per lane would write every line in two halves.
__device__ __forceinline__ void st_pair(double *p, double a, double b, bool two) {
  if (two) {
    *(d2 *)p = d2{a, b};
  } else {
    p[0] = a;
  }
}

// out[o] = sum_b partial[b * nv + o], o < nv <= 17: one workgroup, every thread sums a
// fixed subset of blocks for all outputs, then a fixed-shape tree (deterministic).
__global__ __launch_bounds__(256) void k_reduce_small(const double *__restrict__ partial, int nblocks,
                                                      int nv, double *__restrict__ out) {
  double v[17];
#pragma unroll
  for (int i = 0; i < 17; ++i) v[i] = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += 256) {
    add_partial_row(v, partial, b, nv);
  }
  __shared__ double red[4][17];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 17; ++i) {
    if (i < nv) {
      double x = v[i];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
      if (l == 0) red[w][i] = x;
    }
  }
  __syncthreads();
  if (threadIdx.x < nv) {
    const int i = threadIdx.x;
    out[i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

void launch_reduce_small(hipStream_t s, const double *partial, int nblocks, int nv, double *out) {
  k_reduce_small<<<1, 256, 0, s>>>(partial, nblocks, nv, out);
  LAUNCH_CHECK_();
}

// -------------------------------------------------------------------------------------
// X = beta X + alpha A M (M device, L x kx, leading dim ldm) and, if dmode != 0, partials
// of sum_r Xnew[r,c] * D[r,c] (dmode 1: D = Xnew, 2: D given).  Grid-stride over row pairs.
// -------------------------------------------------------------------------------------
// The closing updates' basis loads (each basis element is read once per pass): plain, or
// non-temporal with -DNN_NT_LOAD=1 (an A/B knob, tools/mb_k16.cpp).
#ifndef NN_NT_LOAD
#define NN_NT_LOAD 0
#endif
__device__ __forceinline__ d2 nn_load(const d2 *p) {
  if (NN_NT_LOAD) return __builtin_nontemporal_load(p);
  return *p;
}

template <int KX>
__global__ __launch_bounds__(ICNT) void k_gemm_nn_dot(MvDesc A, int L, const double *__restrict__ M,
                                                     int ldm, MvDesc X, int kx, int nrows,
                                                     double alpha, double beta, int dmode,
                                                     MvDesc D, double *__restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) double Ms[];  // L x KX
  for (int e = threadIdx.x; e < L * KX; e += ICNT) {
    const int j = e / KX, c = e % KX;
    Ms[e] = c < kx ? M[j + (long long)c * ldm] : 0.0;
  }
  __syncthreads();
  double dacc[KX + 1];  // dmode 3: [KX] = <Xnew_0, Xnew_1> (findBasis head, see k_fb_scalar stage 7)
#pragma unroll
  for (int c = 0; c <= KX; ++c) dacc[c] = 0.0;
  for (long long r = 2LL * ((long long)blockIdx.x * ICNT + threadIdx.x); r < nrows;
       r += 2LL * gridDim.x * ICNT) {
    const bool two = r + 1 < nrows;
    double acc0[KX], acc1[KX];
#pragma unroll
    for (int c = 0; c < KX; ++c) acc0[c] = acc1[c] = 0.0;
    // NB columns per step, all loads issued before the FMAs (more bytes in flight per wave);
    // rows past nrows are the zero padding of the multivector (ld > nrows), read unguarded.
#ifndef NND_NB
#define NND_NB 8
#endif
    constexpr int NB = NND_NB;
    int j = 0;
    for (; j + NB <= L; j += NB) {
      d2 v[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) v[u] = nn_load((const d2 *)(colp_(A, j + u) + r));
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const double *mrow = &Ms[(j + u) * KX];
#pragma unroll
        for (int c = 0; c < KX; ++c) {
          acc0[c] += v[u].x * mrow[c];
          acc1[c] += v[u].y * mrow[c];
        }
      }
    }
    for (; j < L; ++j) {
      const d2 v = *(const d2 *)(colp_(A, j) + r);
      const double *mrow = &Ms[j * KX];
#pragma unroll
      for (int c = 0; c < KX; ++c) {
        acc0[c] += v.x * mrow[c];
        acc1[c] += v.y * mrow[c];
      }
    }
    double f0 = 0.0, f1 = 0.0;  // new column 0 (dmode 3)
#pragma unroll
    for (int c = 0; c < KX; ++c) {
      if (c < kx) {
        double *xp = colp_(X, c) + r;
        double n0, n1 = 0.0;
        if (beta == 0.0) {
          n0 = alpha * acc0[c];
          if (two) n1 = alpha * acc1[c];
        } else {
          const d2 xo = *(const d2 *)xp;  // padding row of an odd tail reads zero
          n0 = beta * xo.x + alpha * acc0[c];
          if (two) n1 = beta * xo.y + alpha * acc1[c];
        }
        st_pair(xp, n0, n1, two);
        if (dmode == 1 || dmode == 3) {
          dacc[c] += n0 * n0 + n1 * n1;
          if (dmode == 3) {
            if (c == 0) {
              f0 = n0;
              f1 = n1;
            } else if (c == 1) {
              dacc[KX] += f0 * n0 + f1 * n1;
            }
          }
        } else if (dmode == 2) {
          const double *dp = colp_(D, c) + r;
          dacc[c] += n0 * dp[0] + (two ? n1 * dp[1] : 0.0);
        }
      }
    }
  }
  if (dmode == 3) {
    // compact [self dots (kx), cross] for the partial layout
#pragma unroll
    for (int c = 0; c < KX; ++c)
      if (c == kx) dacc[c] = dacc[KX];
    block_reduce_store<KX + 1>(dacc, kx + 1, partial);
  } else if (dmode) {
    block_reduce_store<KX + 1>(dacc, kx, partial);
  }
}

void launch_gemm_nn_dot(hipStream_t s, MvDesc A, int L, const double *M, int ldm, MvDesc X,
                        int nrows, double alpha, double beta, int dmode, MvDesc D, double *partial,
                        int nblocks) {
  const int kx = X.ncols;
  if (kx > 16) throw Error(MIGMRES_EINVAL, "gemm_nn_dot: at most 16 columns");
  if (L > 1024) throw Error(MIGMRES_EINVAL, "gemm_nn_dot: at most 1024 coefficient rows");
  const int KX = kx <= 1 ? 1 : kx <= 2 ? 2 : kx <= 4 ? 4 : kx <= 8 ? 8 : 16;
  const size_t lds = sizeof(double) * (size_t)(L > 0 ? L : 1) * KX;
  switch (KX) {
    case 1: k_gemm_nn_dot<1><<<nblocks, ICNT, lds, s>>>(A, L, M, ldm, X, kx, nrows, alpha, beta, dmode, D, partial); break;
    case 2: k_gemm_nn_dot<2><<<nblocks, ICNT, lds, s>>>(A, L, M, ldm, X, kx, nrows, alpha, beta, dmode, D, partial); break;
    case 4: k_gemm_nn_dot<4><<<nblocks, ICNT, lds, s>>>(A, L, M, ldm, X, kx, nrows, alpha, beta, dmode, D, partial); break;
    case 8: k_gemm_nn_dot<8><<<nblocks, ICNT, lds, s>>>(A, L, M, ldm, X, kx, nrows, alpha, beta, dmode, D, partial); break;
    default: k_gemm_nn_dot<16><<<nblocks, ICNT, lds, s>>>(A, L, M, ldm, X, kx, nrows, alpha, beta, dmode, D, partial); break;
  }
  LAUNCH_CHECK_();
}

// -------------------------------------------------------------------------------------
// blkOrtho's first update fused with its second projection:
//   X1 = X - Q C1 (in place)   and   partial[wg] = Q^T X1  (L x k per workgroup)
// One pass over Q instead of two (the reference does MvTimesMatAddMv, then MvTransMv).
// A workgroup stages a 16-row chunk of Q (all L <= 256 columns) in LDS, then
//   phase 1: D = Qc C1 (16 rows x k, K = Q columns split over the 4 waves, C1 register
//            resident), waves summed in a fixed order -> X1 (written out, kept in LDS),
//   phase 2: acc += Qc^T X1 (L x k over the chunk's 16 rows),
// while the loads of the next two chunks are in flight in registers (counted waits: the
// loads are branch-free and the barriers are raw s_barrier, see lds_barrier()).
// Both products use v_mfma_f64_4x4x4f64 (4 independent 4x4x4 blocks per instruction):
// measured 72 TF/s against 47 TF/s for v_mfma_f64_16x16x4f64 (tools/mb_mfma.hip), and its
// 4-wide N matches k = 4, 8, 12, 16 without padding.  Lane maps (probed on gfx950):
//   A: lane 16k + 4b + m -> block b row m, K index k;  B: lane 16k + 4b + n -> block b
//   column n;  D: lane 16m + 4b + n -> block b (m, n).
// With lane l, c = l & 15, g = l >> 4 the A operand is element (c, g) of a 16 x 4 tile
// (rows 4b + m = c), the same addressing as a 16x16x4 A operand.
// LDS: Qs[Lp][17] (odd stride: both phases' reads are conflict-free), Xs[16][16], red[4][4][64].
// -------------------------------------------------------------------------------------
constexpr int NT_ROWS = 16, NT_MAXL = 256, NT_LDQ = 17;
#ifndef NT_GS
#define NT_GS 0
#endif
#ifndef NT_DIAG_MASK  // bit 0 phase 1, bit 1 phase 2, bit 2 LDS staging, bit 3 X1 traffic (tools/mb_nntn.hip)
#define NT_DIAG_MASK 15
#endif

static size_t nt_lds_bytes(int L) {
  const int Lp = (L + 15) & ~15;
  return sizeof(double) * ((size_t)Lp * NT_LDQ + 256 + 4 * 256);
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads()'s release fence waits for
// vmcnt(0), which on gfx9 also counts stores: one global store before it would drain the
// register prefetches that are meant to stay in flight across the barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// The prologue split in two so that a pass can issue its first row loads in between:
// fb_pro_load issues this thread's global loads (one state word, its rows of partials);
// fb_pro_finish consumes them with LDS traffic and raw barriers only, so the pass's loads
// issued in between stay in flight (a __syncthreads() would wait for them: vmcnt(0)).
struct ProRegs {
  long long w;
  double v[17];
};

__device__ __forceinline__ void fb_pro_load(const FbPro &p, ProRegs &r) {
  constexpr int NWORD = sizeof(IcgsState) / 8;
  static_assert(NWORD <= ICNT, "one state word per thread");
  const int t = threadIdx.x;
  r.w = t < NWORD ? ((const long long *)p.in)[t] : 0;
#pragma unroll
  for (int i = 0; i < 17; ++i) r.v[i] = 0.0;
  if (p.stage0 >= 0) {
    if (p.partial) {
      for (int b = t; b < p.nblocks; b += ICNT) {
        add_partial_row(r.v, p.partial, b, p.nv);
      }
    } else if (t < p.nv) {
      r.v[0] = p.red[t];
    }
  }
}

__device__ __forceinline__ void fb_pro_finish(const FbPro &p, ProRegs &r, IcgsState *ls) {
  __shared__ double redv[17];
  __shared__ double wred[ICNW][17];
  constexpr int NWORD = sizeof(IcgsState) / 8;
  const int t = threadIdx.x;
  if (t < NWORD) ((long long *)ls)[t] = r.w;
  if (p.stage0 >= 0) {
    if (p.partial) {
      const int l = t & 63, w = t >> 6;
#pragma unroll
      for (int i = 0; i < 17; ++i) {
        if (i < p.nv) {
          double x = r.v[i];
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
          if (l == 0) wred[w][i] = x;
        }
      }
      lds_barrier();
      if (t < p.nv) {
        double q[ICNW];
#pragma unroll
        for (int w2 = 0; w2 < ICNW; ++w2) q[w2] = wred[w2][t];
#pragma unroll
        for (int h = 1; h < ICNW; h *= 2)
#pragma unroll
          for (int w2 = 0; w2 + h < ICNW; w2 += 2 * h) q[w2] = q[w2] + q[w2 + h];
        redv[t] = q[0];
      }
    } else if (t < p.nv) {
      redv[t] = r.v[0];
    }
    lds_barrier();
    if (t == 0) {
      fb_scalar_body(ls, redv, p.stage0, p.j, p.k, p.complete);
      if (p.stage1 >= 0) fb_scalar_body(ls, redv, p.stage1, p.j, p.k, p.complete);
    }
  }
  lds_barrier();
  if (p.stage0 >= 0 && p.out && blockIdx.x == 0 && t < NWORD) ((long long *)p.out)[t] = ((const long long *)ls)[t];
}

__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

template <int NM, int NJ, bool ST>
__global__ __launch_bounds__(256, 2) void k_nn_tn(MvDesc Q, int L, const double *__restrict__ C1, int ldc,
                                                  MvDesc X, int k, int nrows, double *__restrict__ partial,
                                                  double *__restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int Lp = (L + 15) & ~15;
  double *Qs = sm;
  double *Xs = sm + (size_t)Lp * NT_LDQ;
  double *red = Xs + 256;
  const int t = threadIdx.x, w = t >> 6, l = t & 63, c = l & 15, g = l >> 4;
  const int n4 = l & 3;                            // B / D column within a 4-wide group
  const int drow = 4 * ((l >> 2) & 3) + (l >> 4);  // D row of this lane (block b, row m)
  for (int e = t; e < (Lp - L) * NT_LDQ; e += 256) Qs[L * NT_LDQ + e] = 0.0;

  // phase-1 B operand: C1[i = 4s + g][j = 4 jg + n4] for the wave's K steps s = w + 4m
  double b1[16][NJ];
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int i = 4 * (w + 4 * m) + g;
#pragma unroll
    for (int jg = 0; jg < NJ; ++jg) {
      const int j = 4 * jg + n4;
      b1[m][jg] = (i < L && j < k) ? C1[i + (long long)j * ldc] : 0.0;
    }
  }
  double acc2[4][NJ];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int jg = 0; jg < NJ; ++jg) acc2[m][jg] = 0.0;

  // loader: Q column lcol + 32 m (clamped to L - 1: duplicates rewrite the same value),
  // rows lrow, lrow + 1 -- 8 lanes = one 128-B line.  Q may be a column table (a view).
  const int lrow = 2 * (t & 7), lcol = t >> 3;
  const double *qcol[NM];
  int scol[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    const int i = lcol + 32 * m;
    scol[m] = i < L ? i : L - 1;
    qcol[m] = colp_(Q, scol[m]) + lrow;
  }
  // X1 rows: wave w updates rows 4w + (l >> 4), column l & 15 of every chunk (one 8-byte
  // load and one store per lane and chunk, the same in every wave so that the wait counts
  // stay static; columns >= k read column k - 1 and store into the sink).
  const int xrow = 4 * w + (l >> 4), xc = l & 15;
  const bool xcol_ok = xc < k;
  const double *xsrc = colp_(X, xcol_ok ? xc : k - 1);
  double *xdst = colp_(X, xcol_ok ? xc : k - 1);
  const long long nchunks = (nrows + NT_ROWS - 1) / NT_ROWS;
  const long long G = gridDim.x;
  auto clampc = [&](long long chunk) { return chunk < nchunks ? chunk : nchunks - 1; };
  auto loadq = [&](d2(&p)[NM], long long chunk) {
    chunk = clampc(chunk);
#pragma unroll
    for (int m = 0; m < NM; ++m) p[m] = *(const d2 *)(qcol[m] + chunk * NT_ROWS);
  };
  auto loadx = [&](double &xv, long long chunk) { xv = xsrc[clampc(chunk) * NT_ROWS + xrow]; };

  // A chunk past the end (second half of the last 2-chunk step) runs the same instruction
  // stream on clamped data with X1 = 0, adding nothing; keeping both halves unconditional
  // keeps the wait counts static.
  auto body = [&](d2(&p)[NM], double &xv, long long chunk) {
    const bool live = chunk < nchunks;
    const long long r0 = chunk * NT_ROWS;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      if (NT_DIAG_MASK & 4) {
        Qs[scol[m] * NT_LDQ + lrow] = p[m].x;
        Qs[scol[m] * NT_LDQ + lrow + 1] = p[m].y;
      } else if (p[m].x == 12345.0) {
        Qs[0] = p[m].y;
      }
    }
    lds_barrier();
    loadq(p, chunk + 2 * G);
    // phase 1: this wave's share of D[r][j] = sum_i Q[r][i] C1[i][j]
    double a1[NJ];
#pragma unroll
    for (int jg = 0; jg < NJ; ++jg) a1[jg] = 0.0;
#pragma unroll
    for (int m = 0; m < ((NT_DIAG_MASK & 1) ? 16 : 0); ++m) {
      const int s = w + 4 * m;
      if (4 * s < L) {
        const double qa = Qs[(4 * s + g) * NT_LDQ + c];
#pragma unroll
        for (int jg = 0; jg < NJ; ++jg) a1[jg] = mfma4(qa, b1[m][jg], a1[jg]);
      }
    }
#pragma unroll
    for (int jg = 0; jg < NJ; ++jg) red[(w * 4 + jg) * 64 + l] = a1[jg];
    lds_barrier();
    {
      // wave w: rows 4w + (l >> 4); D lane of (row, column) = 16 (l >> 4) + 4 w + (column & 3)
      const int jg = (xc >> 2) < NJ ? (xc >> 2) : NJ - 1;
      const int o = 16 * (l >> 4) + 4 * w + (xc & 3);
      const double d = (red[jg * 64 + o] + red[(4 + jg) * 64 + o]) +
                       (red[(8 + jg) * 64 + o] + red[(12 + jg) * 64 + o]);
      const bool ok = xcol_ok && live && r0 + xrow < nrows;
      const double x1 = ok ? xv - d : 0.0;
      double *dst = ok ? xdst + r0 + xrow : sink + (blockIdx.x * 256 + t);
      if ((NT_DIAG_MASK & 8) && ST) *dst = x1;
      Xs[xrow * 16 + xc] = x1;
      if (NT_DIAG_MASK & 8) loadx(xv, chunk + 2 * G);
    }
    lds_barrier();
    // phase 2: acc[tile][jg] += Q[:, tile]^T X1[:, 4 jg .. 4 jg + 3] over the 16 rows
    double xb[4][NJ];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int jg = 0; jg < NJ; ++jg) xb[s][jg] = Xs[(4 * s + g) * 16 + 4 * jg + n4];
#pragma unroll
    for (int m = 0; m < ((NT_DIAG_MASK & 2) ? 4 : 0); ++m) {
      const int tt = w + 4 * m;
      if (16 * tt < L) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const double qa = Qs[(16 * tt + c) * NT_LDQ + 4 * s + g];
#pragma unroll
          for (int jg = 0; jg < NJ; ++jg) acc2[m][jg] = mfma4(qa, xb[s][jg], acc2[m][jg]);
        }
      }
    }
    lds_barrier();
  };

  d2 pa[NM], pb[NM];
  double xa, xb2;
  const long long ch0 = blockIdx.x;
  loadq(pa, ch0);
  loadx(xa, ch0);
  asm volatile("" ::: "memory");  // keep pa's loads older than pb's (static wait counts in the loop)
  loadq(pb, ch0 + G);
  loadx(xb2, ch0 + G);
  for (long long ch = ch0; ch < nchunks; ch += 2 * G) {
    body(pa, xa, ch);
    body(pb, xb2, ch + G);
  }
  double *out = partial + (long long)blockIdx.x * L * k;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int tt = w + 4 * m;
    const int i = 16 * tt + drow;
#pragma unroll
    for (int jg = 0; jg < NJ; ++jg) {
      const int j = 4 * jg + n4;
      if (i < L && j < k) out[i + (long long)j * L] = acc2[m][jg];
    }
  }
}

// Wide variants for k <= 8 stage RW-row chunks (RW = 32: two 512-thread workgroups per CU;
// RW = 64: one 1024-thread workgroup), 256-512 B per column per visit instead of 128 B: with
// 16-row chunks the Q stream alone fell from 6.4 TB/s at L = 64 to 3.7 TB/s at L = 200
// (tools/mb_nntn.hip, tools/mb_stream.hip).
// The loader stages Q AND X (columns L .. L+k-1 of the staged image) with the same 16-byte
// loads, so X needs no load of its own: a separate, conditional X load made the compiler
// copy its register at the loop back-edge behind an s_waitcnt vmcnt(0), which drained the
// next chunk's Q prefetch every iteration (5.1 -> see DESIGN.md section 4).
//   phase 1: wave w = (row block rb = w % RB, K quarter kq = w / RB) forms a 16 x k partial
//            of Qc C1; the 4 K quarters are summed in a fixed order by the X1 owners,
//   X1:      thread t owns row t % RW of column t / RW < k: X1 = X - D goes to HBM and back
//            into the staged X column, which phase 2 reads as its B operand,
//   phase 2: wave w accumulates Q tiles w, w + NWAVE, ... (16 columns each) against X1.
// LDS: Qs[Lp][RW + 1] (Lp = round16(L + 4 NJ); columns past L + k stay zero) |
//      red[NWAVE][NJ][64] | C1s[Lq][4 NJ] (Lq = round16(L), zero past L and k).
// Workgroup b owns the contiguous chunk range [c0, c1): consecutive visits to a column are
// adjacent pieces (tools/mb_stream.hip, 32-row chunks: 6.0-6.3 TB/s in this order against
// 5.8-5.9 TB/s grid-stride).
// RW = 16 with an image of at most 7 x 32 columns (LX = L + k) keeps C1 in registers instead
// (see k_nn_tn_w), so its LDS is the image + red only.
// The 512-thread variant on 16-row chunks (NT = 512) always does: its 8 waves split phase 1's K
// in eighths, so each lane holds half as many C1 entries.
template <int RW, int NT = 16 * RW>
static constexpr bool nw_creg(int NM) { return RW == 16 && (NT == 512 || NM <= 7); }
template <int RW, int NT = 16 * RW>
static size_t nw_lds_bytes(int L, int NJ, int LX = 0) {
  const int Lp = (L + 4 * NJ + 15) & ~15, Lq = nw_creg<RW, NT>((LX + 31) >> 5) ? 0 : (L + 15) & ~15;
  return sizeof(double) * ((size_t)Lp * (RW + 1) + (NT / 64) * NJ * 64 + (size_t)Lq * 4 * NJ);
}

template <int RW, int NM, int NJ, bool ST, int NT = 16 * RW, int VIS = RW>
__global__ __launch_bounds__(NT) void k_nn_tn_w(MvDesc Q, int L, const double *__restrict__ C1, int ldc,
                                                MvDesc X, int kx, int nrows, double *__restrict__ partial,
                                                double *__restrict__ sink) {
  // NT threads: 16 RW (phase 1 in K quarters) or, for RW = 16, 512 (K eighths: KQ = 8)
  // VIS rows per column visit: RW (each chunk loaded on its own), or 2 RW for RW = 16 (a
  // 32-row visit -- 256 B per column -- loaded at once and published to the 16-row image in
  // two halves; the 16-row form's 128-byte visits stream at ~4-4.6 TB/s, 256-byte ones ~5.6)
  static_assert(VIS == RW || (RW == 16 && VIS == 32 && NT == 256 && !ST), "visit = chunk, or 2 x 16 rows read-only");
  constexpr int NTH = NT, NWAVE = NTH / 64, RB = RW / 16, KQ = NWAVE / RB, LDQ = RW + 1, LPC = VIS / 2;
  constexpr int CPR = NTH / LPC, NLD = (32 * NM + CPR - 1) / CPR, MS = (8 * NM + KQ - 1) / KQ;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  // kx > 8: workgroup pairs take the two column halves of X (columns h0 .. h0 + k - 1) over
  // the same chunk range at the same time and on the same XCD (blocks 16 q + x and
  // 16 q + x + 8, x < 8; block b is dispatched to XCD b mod 8), so each chunk of Q comes from
  // HBM once and the pair's second read hits that XCD's L2 or the Infinity Cache.  Partials:
  // half 0 at [rng][L][8], half 1 after all nrng of them at [rng][L][kx - 8].
  int rng = blockIdx.x, nrng = gridDim.x, h0 = 0;
  if (kx > 8 && NJ < 4) {
    const int x = blockIdx.x & 15;
    h0 = (x >> 3) * 8;
    rng = (blockIdx.x >> 4) * 8 + (x & 7);
    nrng = gridDim.x >> 1;
  }
  const int k = (kx > 8 && NJ < 4) ? (h0 ? kx - 8 : 8) : kx;
  C1 += (long long)h0 * ldc;
  double *const pout = partial + (long long)(h0 ? nrng : 0) * L * 8 + (long long)rng * L * k;
  auto xcol = [&](int j) { return colp_(X, h0 + j); };
  const int LX = L + k;
  const int Lp = (L + 4 * NJ + 15) & ~15, Lq = (L + 15) & ~15;
  double *Qs = sm;
  double *red = Qs + (size_t)Lp * LDQ;
  double *C1s = red + NWAVE * NJ * 64;
  const int t = threadIdx.x, w = t >> 6, l = t & 63, c = l & 15, g = l >> 4, n4 = l & 3;
  const int rb = w % RB, kq = w / RB;
  for (int e = t; e < Lp * LDQ; e += NTH) Qs[e] = 0.0;
  // RW = 16, NM <= 7: phase 1's B operands are the same for every chunk (wave kq takes K
  // steps kq, kq + 4, ...), so each lane keeps its C1 entries in registers -- 4 of the 5 LDS
  // reads per phase-1 MFMA step at k = 16.  Wider images would need more than the 256
  // registers per lane that two waves per SIMD leave (2 NM x 4 doubles of C1 alone).
  constexpr bool CREG = nw_creg<RW, NT>(NM) && VIS == RW;
  double c1r[CREG ? MS : 1][NJ];
  if constexpr (CREG) {
#pragma unroll
    for (int m = 0; m < MS; ++m) {
      const int i = 4 * (kq + KQ * m) + g;
#pragma unroll
      for (int jg = 0; jg < NJ; ++jg) {
        const int j = 4 * jg + n4;
        c1r[m][jg] = (i < L && j < k) ? C1[i + (long long)j * ldc] : 0.0;
      }
    }
  } else {
    for (int e = t; e < Lq * 4 * NJ; e += NTH) {
      const int i = e / (4 * NJ), j = e % (4 * NJ);
      C1s[e] = (i < L && j < k) ? C1[i + (long long)j * ldc] : 0.0;
    }
  }
  // 16-column tiles of the staged image: 2 NM (L + k <= 32 NM), shared round-robin by the waves
  constexpr int NTILE = 2 * NM, TPW = (NTILE + NWAVE - 1) / NWAVE;
  double acc2[TPW][NJ];
#pragma unroll
  for (int m = 0; m < TPW; ++m)
#pragma unroll
    for (int jg = 0; jg < NJ; ++jg) acc2[m][jg] = 0.0;

  // loader: staged column lcol + 32 m (clamped to LX - 1: duplicates rewrite the same
  // value), rows lrow, lrow + 1 of the chunk; staged columns >= L come from X.
  const int lrow = 2 * (t % LPC), lcol = t / LPC;
  const int lhalf = lrow / RW;  // VIS = 2 RW: the half of the visit this lane's rows are in
  const double *lsrc[NLD];
  int lsts[NLD];
#pragma unroll
  for (int m = 0; m < NLD; ++m) {
    int i = lcol + CPR * m;
    i = i < LX ? i : LX - 1;
    lsts[m] = i * LDQ + lrow % RW;
    lsrc[m] = (i < L ? colp_(Q, i) : xcol(i - L)) + lrow;
  }
  // X1 element e = t mod (RW k): row xr of column xj.  Threads t >= RW k repeat an element
  // and store the same value again, so the X1 store is unconditional: a conditional store
  // makes the compiler drain the whole prefetch (vmcnt(0)) at the top of the next chunk.
  const int xe = t % (RW * k), xr = xe % RW, xj = xe / RW;
  const bool xprim = t < RW * k;
  double *xdst = xcol(xj);
  const int xjg = xj >> 2;
  const int xr16 = xr & 15, xrb = xr >> 4;
  const int xo = 16 * (xr16 & 3) + 4 * (xr16 >> 2) + (xj & 3);  // D lane of (row, column)
  double *xs = Qs + (size_t)(L + xj) * LDQ + xr;
  const long long nchunks = (nrows + RW - 1) / RW;
  // chunk order: workgroup rng owns [c0, c1) (NT_GS = 0), or takes every nrng-th chunk from
  // rng on (NT_GS = 1: the resident grid sweeps one contiguous band of rows at a time)
  const long long c0 = NT_GS ? rng : nchunks * rng / nrng, c1 = NT_GS ? nchunks : nchunks * (rng + 1) / nrng;
  const long long cstep = NT_GS ? nrng : 1;

  // (A 2-deep prefetch measured no faster: for the 32-row, C1-in-LDS form at one workgroup
  // per CU, where the LDS reads -- about 200 ds_read_b64 per wave per chunk -- bound it, and
  // for the 512-thread 16-row form at k = 16, L = 128 .. 400, chunks in pairs.)
  auto clampc = [&](long long chunk) { return chunk < c1 ? chunk : c1 - 1; };
  // A store behind the prologue loads, like the X1 store behind the in-loop prefetch: the
  // loop header then sees the same pending-event order on both incoming edges and waits
  // vmcnt(1) for the last prefetched column instead of vmcnt(0) (which waits for the X1
  // store's completion).  partial[0] of this workgroup is rewritten at the end.
  // One chunk: publish the prefetched image pp, refill pp with chunk `nxt`, both phases.
  // publish the prefetched visit (VIS = 2 RW: only the lanes holding half h write)
  auto publish = [&](d2(&pp)[NLD], int h) __attribute__((always_inline)) {
    const bool mine = VIS == RW || lhalf == h;
#pragma unroll
    for (int m = 0; m < NLD; ++m) {
      if (NT_DIAG_MASK & 4) {
        if (mine) {
          Qs[lsts[m]] = pp[m].x;
          Qs[lsts[m] + 1] = pp[m].y;
        }
      } else if (pp[m].x == 12345.0) {
        Qs[0] = pp[m].y;
      }
    }
  };
  // both phases on chunk ch of the published image
  auto compute = [&](long long ch) __attribute__((always_inline)) {
    const long long r0 = ch * RW;
    const double xval = *xs;
    // phase 1: rows 16 rb .. 16 rb + 15, K steps s = kq + KQ m (4 s < L <= 32 NM)
    double a1[NJ];
#pragma unroll
    for (int jg = 0; jg < NJ; ++jg) a1[jg] = 0.0;
#pragma unroll
    for (int m = 0; m < ((NT_DIAG_MASK & 1) ? MS : 0); ++m) {
      const int s = kq + KQ * m;
      if (4 * s < L) {
        const double qa = Qs[(4 * s + g) * LDQ + 16 * rb + c];
#pragma unroll
        for (int jg = 0; jg < NJ; ++jg)
          a1[jg] = mfma4(qa, CREG ? c1r[CREG ? m : 0][jg] : C1s[(4 * s + g) * 4 * NJ + 4 * jg + n4], a1[jg]);
      }
    }
#pragma unroll
    for (int jg = 0; jg < NJ; ++jg) red[((kq * RB + rb) * NJ + jg) * 64 + l] = a1[jg];
    lds_barrier();
    {
      auto rd = [&](int q) { return red[((q * RB + xrb) * NJ + xjg) * 64 + xo]; };
      double d = (rd(0) + rd(1)) + (rd(2) + rd(3));
      if constexpr (KQ == 8) d += (rd(4) + rd(5)) + (rd(6) + rd(7));
      const double x1 = xval - d;
      if ((NT_DIAG_MASK & 8) && ST) xdst[r0 + xr] = x1;
      if (xprim) *xs = x1;
    }
    lds_barrier();
    // phase 2: tiles w, w + NWAVE, ... against the RW rows of X1 (staged columns L + j); a
    // K step's X1 operands are read once and reused by all of the wave's tiles (LDS reads
    // per wave and chunk: RW/4 (NJ + TPW) instead of RW/4 TPW (1 + NJ))
    if (NT_DIAG_MASK & 2) {
#pragma unroll
      for (int s = 0; s < RW / 4; ++s) {
        double xb[NJ];
#pragma unroll
        for (int jg = 0; jg < NJ; ++jg) xb[jg] = Qs[(L + 4 * jg + n4) * LDQ + 4 * s + g];
#pragma unroll
        for (int mm = 0; mm < TPW; ++mm) {
          const int tt = w + NWAVE * mm;
          if (16 * tt < L) {
            const double qa = Qs[(16 * tt + c) * LDQ + 4 * s + g];
#pragma unroll
            for (int jg = 0; jg < NJ; ++jg) acc2[mm][jg] = mfma4(qa, xb[jg], acc2[mm][jg]);
          }
        }
      }
    }
  };
  auto body = [&](d2(&pp)[NLD], long long ch, long long nxt) {
    publish(pp, 0);
    lds_barrier();
    {
      const long long cn = clampc(nxt) * RW;
#pragma unroll
      for (int m = 0; m < NLD; ++m) pp[m] = *(const d2 *)(lsrc[m] + cn);
    }
    if (ch < c1) compute(ch);
    lds_barrier();
  };
  if constexpr (VIS != RW) {
    // 32-row visits (RW = 16): visit v = chunks 2v, 2v + 1, loaded by one set of 16-byte loads
    // (16 lanes per column) and published half by half into the 16-row image; the next visit's
    // loads are issued once the second half is published and land during its chunk's phases
    // (a second register set -- 1.5 visits of cover -- pushed the kernel past the two waves
    // per SIMD that its registers allow, or into scratch).
    const long long nvis = (nchunks + 1) / 2;
    const long long v0 = nvis * rng / nrng, v1 = nvis * (rng + 1) / nrng;
    auto load = [&](d2(&pp)[NLD], long long v) __attribute__((always_inline)) {
      const long long rv = (v < nvis ? v : nvis - 1) * VIS;
#pragma unroll
      for (int m = 0; m < NLD; ++m) pp[m] = *(const d2 *)(lsrc[m] + rv);
    };
    auto visit = [&](d2(&pp)[NLD], long long v, long long nxt) __attribute__((always_inline)) {
      publish(pp, 0);
      lds_barrier();
      if (v < v1 && 2 * v < nchunks) compute(2 * v);
      lds_barrier();
      publish(pp, 1);
      lds_barrier();
      load(pp, nxt);
      if (v < v1 && 2 * v + 1 < nchunks) compute(2 * v + 1);
      lds_barrier();
    };
    d2 pa[NLD];
    load(pa, v0);
    for (long long v = v0; v < v1; ++v) visit(pa, v, v + 1);
  } else {
  const long long cf = c0 < c1 ? c0 : nchunks - 1;  // empty range (k > 8, few chunks): any valid chunk
  {
    // 1-deep register prefetch: the next chunk's loads are issued right after the barrier
    // that publishes the current one and stay in flight through both phases.  Rows past nrows
    // are zero padding in Q and X, so their X1 is zero and is stored back unguarded.
    d2 p[NLD];
#pragma unroll
    for (int m = 0; m < NLD; ++m) p[m] = *(const d2 *)(lsrc[m] + cf * RW);
    if ((NT_DIAG_MASK & 8) && ST) pout[0] = 0.0;
    for (long long ch = c0; ch < c1; ch += cstep) body(p, ch, ch + cstep);
  }
  }
  // partial (L x k) of this workgroup: tile tt rows 16 tt + 4 b + m
  double *out = pout;
#pragma unroll
  for (int mm = 0; mm < TPW; ++mm) {
    const int tt = w + NWAVE * mm;
    const int i = 16 * tt + 4 * ((l >> 2) & 3) + (l >> 4);
#pragma unroll
    for (int jg = 0; jg < NJ; ++jg) {
      const int j = 4 * jg + n4;
      if (16 * tt < L && i < L && j < k) out[i + (long long)j * L] = acc2[mm][jg];
    }
  }
}

// -------------------------------------------------------------------------------------
// k > 8 (<= 16), L <= 256: the fused update + projection with each wave owning ROWS instead of
// a share of the K (projection) dimension, so phase 1 needs no cross-wave reduction and a
// chunk costs two barriers instead of four.  The workgroup stages a 16-row chunk of Q and X
// (all L + 16 columns) in LDS with coalesced 16-byte loads (128 B per column) and keeps the
// next chunk's loads in flight in registers; wave w then takes rows 4w .. 4w + 3 alone:
//   phase 1: D1 (4 rows x 16) = Q(rows, :) C1 on v_mfma_f64_4x4x4f64 with the four blocks as
//            the four 4-column groups of X: A = Q(rows, 4s .. 4s + 3) (the same for every
//            block: broadcast LDS reads), B = C1(4s .. 4s + 3, 4b .. 4b + 3) from LDS;
//   X1 = X - D1 in the D layout, which is the B layout phase 2 needs (lane 16 m + 4 b + n
//            holds (row m, column 4 b + n) in both) -- X1 never leaves the registers;
//   phase 2: acc[t] += Q(rows, 4t .. 4t + 3)^T X1, one 4 x 16 accumulator per 4-column group
//            of Q (L / 4 doubles per lane).
// The four waves' accumulators are summed in a fixed order at the end: one L x k partial per
// workgroup, the layout of k_nn_tn_w's single-launch form.  Read-only (k > 8 never stores X1).
// LDS: img[16][LDQ] (LDQ = 4 mod 32 doubles: both phases' A reads are conflict-free) and
// C1s[L / 4][64].
// -------------------------------------------------------------------------------------
static constexpr int pw_ldq(int LT) { return ((LT + 16 - 4 + 31) / 32) * 32 + 4; }
static size_t pw_lds_bytes(int LT) {
  const size_t img = (size_t)16 * pw_ldq(LT), c1 = (size_t)(LT / 4) * 64;
  const size_t red = (size_t)(LT / 4) * 64;  // the final reduction reuses img (img >= red)
  return sizeof(double) * ((img > red ? img : red) + c1);
}

template <int LT>
__global__ __launch_bounds__(256) void k_nn_tn_pw(MvDesc Q, int L, const double *__restrict__ C1, int ldc,
                                                  MvDesc X, int k, int nrows, double *__restrict__ partial,
                                                  double *__restrict__ sink) {
  constexpr int NA = LT / 4, LDQ = pw_ldq(LT), LX = LT + 16, NLD = (LX + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double *img = sm;
  double *C1s = sm + ((size_t)16 * LDQ > (size_t)NA * 64 ? (size_t)16 * LDQ : (size_t)NA * 64);
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  // C1 in the B layout: lane 16 kk + 4 b + n of step s holds C1[4 s + kk][4 b + n] = [.][l & 15]
  for (int e = t; e < NA * 64; e += 256) {
    const int s = e >> 6, ll = e & 63, i = 4 * s + (ll >> 4), j = ll & 15;
    C1s[e] = (i < L && j < k) ? C1[i + (long long)j * ldc] : 0.0;
  }
  // columns L .. LT - 1 of the image (Q padding) and the X columns past k stay zero
  for (int e = t; e < 16 * LDQ; e += 256) img[e] = 0.0;
  __syncthreads();
  // loader: image column lcol + 32 m (Q for < L, X column c - LT for LT <= c < LT + k),
  // rows lrow, lrow + 1 of the chunk: 8 lanes = one 128-B line per column
  const int lrow = 2 * (t & 7), lcol = t >> 3;
  const double *lsrc[NLD];
  int ldst[NLD];
  bool lon[NLD];
#pragma unroll
  for (int m = 0; m < NLD; ++m) {
    const int c = lcol + 32 * m;
    lon[m] = c < L || (c >= LT && c < LT + k);
    const int cc = !lon[m] ? 0 : c;
    lsrc[m] = (cc < LT ? colp_(Q, cc) : colp_(X, cc - LT)) + lrow;
    ldst[m] = lrow * LDQ + c;
  }
  const long long nchunks = (nrows + 15) / 16;
  const long long c0 = nchunks * blockIdx.x / gridDim.x, c1 = nchunks * (blockIdx.x + 1) / gridDim.x;
  double acc[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) acc[a] = 0.0;
  const int r0 = 4 * w;
  const int am = l & 3, ak = l >> 4;  // A operand: row m = l & 3, K index = l >> 4
  d2 p[NLD];
  if (c0 < c1) {
#pragma unroll
    for (int m = 0; m < NLD; ++m) p[m] = *(const d2 *)(lsrc[m] + c0 * 16);
  }
  for (long long ch = c0; ch < c1; ++ch) {
    lds_barrier();  // every wave is done with the previous chunk's image
#pragma unroll
    for (int m = 0; m < NLD; ++m) {
      if (lon[m]) {
        img[ldst[m]] = p[m].x;
        img[ldst[m] + LDQ] = p[m].y;
      }
    }
    {
      const long long nx = ch + 1 < c1 ? ch + 1 : ch;
#pragma unroll
      for (int m = 0; m < NLD; ++m) p[m] = *(const d2 *)(lsrc[m] + nx * 16);
    }
    lds_barrier();  // image published
    // Both phases in batches of BT K steps whose LDS operands are read one batch ahead (the
    // compiler, left to itself, kept 2-4 reads in flight and each MFMA waited out the LDS
    // latency).  The empty asm statements keep each batch's reads above the previous batch's
    // MFMAs.
    constexpr int BT = 6;
    // phase 1: D1 = Q(rows r0 .. r0 + 3, :) C1 in two interleaved accumulator chains
    double d1q[2] = {0.0, 0.0};
    const double *arow = img + (r0 + am) * LDQ + ak;
    {
      double ca[BT], cb[BT], na[BT], nb[BT];
#pragma unroll
      for (int j = 0; j < BT; ++j) {
        ca[j] = j < NA ? arow[4 * j] : 0.0;
        cb[j] = j < NA ? C1s[j * 64 + l] : 0.0;
      }
#pragma unroll
      for (int s0 = 0; s0 < NA; s0 += BT) {
#pragma unroll
        for (int j = 0; j < BT; ++j) {
          const int s = s0 + BT + j;
          na[j] = s < NA ? arow[4 * s] : 0.0;
          nb[j] = s < NA ? C1s[s * 64 + l] : 0.0;
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < BT; ++j)
          if (s0 + j < NA) d1q[j & 1] = mfma4(ca[j], cb[j], d1q[j & 1]);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < BT; ++j) {
          ca[j] = na[j];
          cb[j] = nb[j];
        }
      }
    }
    const double d1 = d1q[0] + d1q[1];
    // X1 (row r0 + (l >> 4), column l & 15), in place in the B layout of phase 2
    const double x1 = img[(r0 + (l >> 4)) * LDQ + LT + (l & 15)] - d1;
    // phase 2: acc[t] += Q(rows, 4t .. 4t + 3)^T X1
    const double *a2 = img + (r0 + ak) * LDQ + am;
    {
      constexpr int B2 = 2 * BT;
      double ca[B2], na[B2];
#pragma unroll
      for (int j = 0; j < B2; ++j) ca[j] = j < NA ? a2[4 * j] : 0.0;
#pragma unroll
      for (int a0 = 0; a0 < NA; a0 += B2) {
#pragma unroll
        for (int j = 0; j < B2; ++j) {
          const int a = a0 + B2 + j;
          na[j] = a < NA ? a2[4 * a] : 0.0;
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < B2; ++j)
          if (a0 + j < NA) acc[a0 + j] = mfma4(ca[j], x1, acc[a0 + j]);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < B2; ++j) ca[j] = na[j];
      }
    }
  }
  // fixed-order sum of the four waves' partials: ((w0 + w1) + w2) + w3
  double *red = img;
  for (int q = 0; q < 4; ++q) {
    lds_barrier();
    if (w == q) {
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        double v = acc[a];
        if (q > 0) v = red[a * 64 + l] + v;
        red[a * 64 + l] = v;
      }
    }
  }
  lds_barrier();
  // partial (L x k, column-major) of this workgroup: red[a][lane 16 m + 4 b + n] = C2[4a + m][4b + n]
  double *out = partial + (long long)blockIdx.x * L * k;
  for (int e = t; e < NA * 64; e += 256) {
    const int a = e >> 6, ll = e & 63, i = 4 * a + (ll >> 4), j = ll & 15;
    if (i < L && j < k) out[i + (long long)j * L] = red[e];
  }
  (void)sink;
}

// -------------------------------------------------------------------------------------
// k > 8 (<= 16): the fused update + projection with both products on v_mfma_f64_16x16x4f64 and
// C1 in registers (round 4).  The 4x4x4 forms above hold C1's B operand 4-fold replicated (the
// same 4 x 4 block for each of the four row blocks of an instruction), so a 32-row image with
// C1 in registers did not fit and C1 went to LDS (L x 16 doubles), which kept the 32-row image
// (256-byte column visits) at one workgroup per CU from L ~ 144 on.  Here phase 1 forms the
// TRANSPOSED update, D1^T = C1^T Qc^T: the A operand C1^T[j][4 s + kk] = C1[4 s + (l >> 4)][l & 15]
// is one register per lane and K step (L / 16 per wave with the K dimension split in quarters),
// the B operand Qc^T[4 s + kk][row] is the staged image's column-major element, and lane l ends
// with D1 for chunk row 16 rb + (l & 15), X columns (l >> 4) + 4 r.  Phase 2 accumulates
// C2 += Qc^T X1 per 16-column tile of Q (A = image, B = X1 from the image's X columns).
// 512 threads = 2 row blocks x 4 K quarters; the quarters are summed in a fixed order,
// ((q0 + q2) + (q1 + q3)), through an 8 KB buffer, so the LDS is the image + 8 KB: two
// workgroups per CU up to L = 256 at k = 16.  Read-only (X1 stays in the LDS image).
// -------------------------------------------------------------------------------------
static size_t m16_lds_bytes(int L) {
  const size_t lp = (size_t)((L + 16 + 15) & ~15);
  return sizeof(double) * (lp * 33 + 4 * 256);
}

template <int LQ, int WPE>
__global__ __launch_bounds__(512, WPE) void k_nn_tn_m16(MvDesc Q, int L, const double *__restrict__ C1, int ldc,
                                                        MvDesc X, int k, int nrows, double *__restrict__ partial,
                                                        double *__restrict__ sink) {
  // LQ = ceil(L / 16): MS = LQ K steps per wave in phase 1 (4 LQ steps of 4 over the quarters),
  // TPW 16-column tiles per wave in phase 2, NM 32-column loads per lane for the L + 16 image
  // columns.  Steps and tiles past L read image columns >= L (X or zero columns, all inside the
  // image) against zero C1 entries / into discarded rows, so they add exact zeros.  Q and X
  // are plain (no column table).
  constexpr int RW = 32, LDQ = RW + 1, LPC = RW / 2, CPR = 512 / LPC;
  constexpr int MS = LQ, TPW = (LQ + 7) / 8, NM = (LQ + 2) / 2;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int Lp = (L + 16 + 15) & ~15, LX = L + k;
  double *Qs = sm;
  double *red = sm + (size_t)Lp * LDQ;
  const int t = threadIdx.x, l = t & 63, c = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int rb = w & 1, kq = w >> 1;
  for (int e = t; e < Lp * LDQ + 4 * 256; e += 512) sm[e] = 0.0;
  // phase 1's A operands for the K steps s = kq + 4 m of this wave
  double c1r[MS];
#pragma unroll
  for (int m = 0; m < MS; ++m) {
    const int i = 4 * (kq + 4 * m) + g;
    c1r[m] = (i < L && c < k) ? C1[i + (long long)c * ldc] : 0.0;
  }
  d4 acc[TPW];
#pragma unroll
  for (int mm = 0; mm < TPW; ++mm) acc[mm] = d4{0.0, 0.0, 0.0, 0.0};
  // loader: image column lcol + 32 m (clamped to LX - 1), rows lrow, lrow + 1 of the chunk
  const int lrow = 2 * (t % LPC), lcol = t / LPC;
  // (image column of load m: one register each; the 64-bit source address and the LDS slot are
  // re-derived per chunk, which keeps the wide images out of scratch)
  int lci[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    const int i = lcol + CPR * m;
    lci[m] = i < LX ? i : LX - 1;
  }
  auto lsrc = [&](int m, long long r0) __attribute__((always_inline)) {
    const int i = lci[m];
    return (const d2 *)((i < L ? Q.base + (long long)i * Q.ld : X.base + (long long)(i - L) * X.ld) + lrow + r0);
  };
  const long long nchunks = (nrows + RW - 1) / RW;
  const long long c0 = nchunks * blockIdx.x / gridDim.x, c1 = nchunks * (blockIdx.x + 1) / gridDim.x;
  d2 p[NM];
  if (c0 < c1) {
#pragma unroll
    for (int m = 0; m < NM; ++m) p[m] = *lsrc(m, c0 * RW);
  }
  lds_barrier();  // the zeroed image
  const double *b1 = Qs + g * LDQ + 16 * rb + c + 4 * kq * LDQ;  // phase 1, step m: + 16 m LDQ
  for (long long ch = c0; ch < c1; ++ch) {
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const int o = lci[m] * LDQ + lrow;
      Qs[o] = p[m].x;
      Qs[o + 1] = p[m].y;
    }
    lds_barrier();
    {
      const long long nx = (ch + 1 < c1 ? ch + 1 : ch) * RW;
#pragma unroll
      for (int m = 0; m < NM; ++m) p[m] = *lsrc(m, nx);
    }
    // phase 1: D1^T (16 X columns x 16 chunk rows of row block rb), K quarter kq, in batches of
    // 4 K steps (a batch's LDS reads, then its MFMAs: the empty asm statements keep the
    // compiler from hoisting every read of the chunk)
    d4 d = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int m0 = 0; m0 < MS; m0 += 4) {
      double b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (m0 + u < MS) b[u] = b1[16 * (m0 + u) * LDQ];
      asm volatile("" ::: "memory");
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (m0 + u < MS) d = __builtin_amdgcn_mfma_f64_16x16x4f64(c1r[m0 + u], b[u], d, 0, 0, 0);
      asm volatile("" : "+v"(d)::"memory");  // the batch's MFMAs stay ahead of the next batch's reads
    }
    // fixed-order sum of the K quarters: (q0 + q2) + (q1 + q3)
    if (kq >= 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((kq - 2) * 2 + rb) * 256 + 64 * r + l] = d[r];
    }
    lds_barrier();
    if (kq < 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) d[r] = d[r] + red[(kq * 2 + rb) * 256 + 64 * r + l];
    }
    if (kq == 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(2 + rb) * 256 + 64 * r + l] = d[r];
    }
    lds_barrier();
    if (kq == 0) {
      // X1 = X - D1 into the image's X columns (columns >= k: zero minus zero)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double *xs = Qs + (size_t)(L + g + 4 * r) * LDQ + 16 * rb + c;
        *xs = *xs - (d[r] + red[(2 + rb) * 256 + 64 * r + l]);
      }
    }
    lds_barrier();
    // phase 2: C2 tile (16 Q columns x 16 X columns) += Qc^T X1, tiles w, w + 8, ... (< L / 16:
    // a wave-uniform bound)
#pragma unroll
    for (int sp = 0; sp < RW / 4; ++sp) {
      const double xb = Qs[(L + c) * LDQ + 4 * sp + g];
      double a[TPW];
#pragma unroll
      for (int mm = 0; mm < TPW; ++mm)
        if (16 * (w + 8 * mm) < L) a[mm] = Qs[(16 * (w + 8 * mm) + c) * LDQ + 4 * sp + g];
      asm volatile("" ::: "memory");
#pragma unroll
      for (int mm = 0; mm < TPW; ++mm) {
        if (16 * (w + 8 * mm) < L) acc[mm] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mm], xb, acc[mm], 0, 0, 0);
        asm volatile("" : "+v"(acc[mm])::"memory");
      }
    }
    lds_barrier();
  }
  // partial (L x k, column-major) of this workgroup: D[Q column 16 tt + g + 4 r][X column c]
  double *out = partial + (long long)blockIdx.x * L * k;
#pragma unroll
  for (int mm = 0; mm < TPW; ++mm) {
    const int tt = w + 8 * mm;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * tt + g + 4 * r;
      if (16 * tt < L && i < L && c < k) out[i + (long long)c * L] = acc[mm][r];
    }
  }
  (void)sink;
}

typedef void (*nt_kernel_t)(MvDesc, int, const double *, int, MvDesc, int, int, double *, double *);

// The 16x16x4 form (k_nn_tn_m16): MIGMRES_NT_M16 = 0 off, 1 (default) from L = M16_MIN_L on,
// 2 every k > 8 shape from L = 16 (read per launch, so a test can switch it).  At k <= 8 (X's
// columns 8 .. 15 zero) it lost to the wide form below L = 64 (profiles/r4u_k8_small_l.txt).
constexpr int M16_MIN_L = 48;
static int m16_mode() {
  const char *e = std::getenv("MIGMRES_NT_M16");
  return e ? std::atoi(e) : 1;
}
static bool m16_ok(int L, int k) {
  const int m = m16_mode();
  return m != 0 && k > 8 && k <= 16 && L >= (m >= 2 ? 16 : M16_MIN_L) && L + 16 <= 512;
}
// One instantiation per 16-column step of L; two workgroups per CU (4 waves per SIMD: 128
// registers) up to L = 240, else one.  Measured (tools/mb_k16.cpp, 256^3, k = 16, same box,
// profiles/r4q_k16_nn_tn_sweep.txt) against the forms above: L = 64 2.42 -> 2.16 ms, 128 4.56 ->
// 3.62, 208 6.63 -> 5.66 (5.3 TB/s), 272 9.86 -> 8.00, 400 13.35 -> 11.56; L = 256 with two
// workgroups per CU spilled (24 registers) and ran at 4.36 TB/s, hence one there.  Below L = 48
// the per-wave-rows form stays ahead (L = 16: 0.86 vs 1.19 ms).
static nt_kernel_t m16_pick(int L) {
  switch ((L + 15) >> 4) {
#define M16_CASE(N) \
  case N:           \
    return k_nn_tn_m16<N, (N <= 15 ? 4 : 2)>;
    M16_CASE(1) M16_CASE(2) M16_CASE(3) M16_CASE(4) M16_CASE(5) M16_CASE(6) M16_CASE(7) M16_CASE(8)
    M16_CASE(9) M16_CASE(10) M16_CASE(11) M16_CASE(12) M16_CASE(13) M16_CASE(14) M16_CASE(15) M16_CASE(16)
    M16_CASE(17) M16_CASE(18) M16_CASE(19) M16_CASE(20) M16_CASE(21) M16_CASE(22) M16_CASE(23) M16_CASE(24)
    M16_CASE(25) M16_CASE(26) M16_CASE(27) M16_CASE(28) M16_CASE(29) M16_CASE(30) M16_CASE(31)
#undef M16_CASE
    default: return nullptr;
  }
}
// resident workgroups per CU (LDS and registers), cached per image width
static int m16_per_cu(int L) {
  static int cache[513] = {};
  int &v = cache[L];
  if (!v) {
    int per_cu = 0;
    const nt_kernel_t f = m16_pick(L);
    if (hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, 512, m16_lds_bytes(L)) != hipSuccess)
      per_cu = 1;
    v = per_cu < 1 ? 1 : per_cu > 2 ? 2 : per_cu;
  }
  return v;
}

static int pw_mode() {
  static int m = -1;
  if (m < 0) {
    const char *e = std::getenv("MIGMRES_NT_PW");
    m = e ? std::atoi(e) : 1;
  }
  return m;
}
// The per-wave-rows form for k > 8, measured against the kernels it replaces at 256^3, k = 16
// (tools/mb_k16.cpp, same box, profiles/r3m_k16_nn_tn_sweep.txt): L = 16 0.85 vs 2.02 ms (the
// narrow k_nn_tn ran below L = 64), 32 1.37 vs 2.13, 48 1.82 vs 2.85, 64 2.36 vs 2.60, 96 3.46 vs
// 3.59; from L = 128 on k_nn_tn_w is ahead (4.51 vs 4.58 ms, L = 192 6.08 vs 6.81).  Every form
// of the phase structure tried (this one without the cross-wave reduction, two accumulator
// chains, LDS operands read a batch ahead) stays near 4.0-4.6 TB/s = 30 TF/s of fp64 MFMA at
// L >= 160 with the clock at 2.0-2.3 GHz under this load (GRBM_GUI_ACTIVE, r3m).  Default
// (MIGMRES_NT_PW=1) L <= 112; 2: up to L = 256; 0: off.
static bool pw_ok(int L, int k) {
  const int m = pw_mode();
  return m != 0 && k > 8 && k <= 16 && L >= 16 && L <= (m >= 2 ? 256 : 112);
}
static nt_kernel_t pw_pick(int L) {
  switch ((L + 15) >> 4) {
#define PW_CASE(N) \
  case N:          \
    return k_nn_tn_pw<16 * N>;
    PW_CASE(1) PW_CASE(2) PW_CASE(3) PW_CASE(4) PW_CASE(5) PW_CASE(6) PW_CASE(7) PW_CASE(8)
    PW_CASE(9) PW_CASE(10) PW_CASE(11) PW_CASE(12) PW_CASE(13) PW_CASE(14) PW_CASE(15) PW_CASE(16)
#undef PW_CASE
    default: return nullptr;
  }
}
static int pw_per_cu(int L) {
  static int cache[17] = {};
  const int n = (L + 15) >> 4;
  int &v = cache[n];
  if (!v) {
    int per_cu = 0;
    const nt_kernel_t f = pw_pick(L);
    if (hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, 256, pw_lds_bytes(16 * n)) != hipSuccess)
      per_cu = 1;
    v = per_cu < 1 ? 1 : per_cu > 4 ? 4 : per_cu;
  }
  return v;
}

template <int NJ, bool ST>
static nt_kernel_t nt_pick_nm(int L) {
  switch ((L + 31) >> 5) {
    case 1: return k_nn_tn<1, NJ, ST>;
    case 2: return k_nn_tn<2, NJ, ST>;
    case 3: return k_nn_tn<3, NJ, ST>;
    case 4: return k_nn_tn<4, NJ, ST>;
    case 5: return k_nn_tn<5, NJ, ST>;
    case 6: return k_nn_tn<6, NJ, ST>;
    case 7: return k_nn_tn<7, NJ, ST>;
    default: return k_nn_tn<8, NJ, ST>;
  }
}

template <bool ST>
static nt_kernel_t nt_pick(int L, int k) {
  switch ((k + 3) >> 2) {
    case 1: return nt_pick_nm<1, ST>(L);
    case 2: return nt_pick_nm<2, ST>(L);
    case 3: return nt_pick_nm<3, ST>(L);
    default: return nt_pick_nm<4, ST>(L);
  }
}

#ifndef NT_WIDE_RW
#define NT_WIDE_RW 32
#endif
#ifndef NT_WIDE_WGCU
#define NT_WIDE_WGCU (NT_WIDE_RW == 32 ? 2 : 1)
#endif
constexpr int NW_RW = NT_WIDE_RW;  // rows per chunk of the wide variant (32: 2 WGs/CU, 64: 1 WG/CU)
constexpr int NW_WG_PER_CU = NT_WIDE_WGCU;

template <int RW, int NJ, bool ST, int NT = 16 * RW, int VIS = RW>
static nt_kernel_t nw_pick_nm(int LX) {
  switch ((LX + 31) >> 5) {
#define NW_CASE(N) \
  case N:          \
    return k_nn_tn_w<RW, N, NJ, ST, NT, VIS>;
    NW_CASE(1) NW_CASE(2) NW_CASE(3) NW_CASE(4) NW_CASE(5) NW_CASE(6) NW_CASE(7) NW_CASE(8)
    NW_CASE(9) NW_CASE(10) NW_CASE(11) NW_CASE(12) NW_CASE(13) NW_CASE(14) NW_CASE(15)
#undef NW_CASE
    default: return k_nn_tn_w<RW, 16, NJ, ST, NT, VIS>;
  }
}


// The wide variant wins from L = 16 on at k = 8 (round 4, see nw_min_l; it used to win only from
// L = 64, where the per-chunk latency was not hidden below).  Up to L + k = 256 NW_WG_PER_CU workgroups' LDS fit in 160 KiB; wider
// images (k = 16 in column halves: L up to 400 at Num Blocks 25) run one workgroup per CU.
// k > 8 with all columns in one workgroup can also run on 16-row chunks (256 threads): the
// image takes half the LDS, so two workgroups share a CU up to L = 256 and one barrier-bound
// workgroup's MFMA phases overlap the other's loads; and it fits one workgroup up to
// L + k = 512, so no column-half pairs are needed.  Measured at 256^3, k = 16
// (tools/mb_k16.cpp, same box): L = 192 7.20 -> 6.58 ms, L = 256 9.16 -> 8.39 ms (two
// workgroups per CU instead of one), L = 400 20.4 (pairs) -> 18.4 ms; but one 16-row
// workgroup per CU where the 32-row one also fits once is slower (L = 272: 13.0 vs 9.6 ms),
// and so is L <= 128 (two 32-row workgroups fit already).  MIGMRES_NW16: 0 off, 1 (default)
// those two cases, 2 every k > 8 shape, 3 every k > 8 shape with 512 threads.
static int nw16_mode() {
  static int m = -1;
  if (m < 0) {
    const char *e = std::getenv("MIGMRES_NW16");
    m = e ? std::atoi(e) : 1;
  }
  return m;
}
// Resident 16-row workgroups of NT threads per CU (LDS and the registers that hold C1), at most 2.
template <int NT>
static int nw16_occ(int L, int k) {
  static int cache[513] = {};
  int &v = cache[L + k];
  if (!v) {
    int per_cu = 0;
    const nt_kernel_t f = nw_pick_nm<16, 4, false, NT>(L + k);
    if (hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, NT, nw_lds_bytes<16, NT>(L, 4, L + k)) != hipSuccess)
      per_cu = 1;
    v = per_cu < 1 ? -1 : per_cu > 2 ? 2 : per_cu;
  }
  return v < 0 ? 0 : v;
}
// 16-row chunks: 256 threads, or 512 where the 32-row image does not fit the LDS (mode 1) or
// always (MIGMRES_NW16=3).  Measured (tools/mb_k16.cpp, k = 16, same box): L = 400 18.4 ms
// (256) -> 13.3 ms (512) against 20.4 ms for the column-half pairs; L = 352 equal; at
// L <= 272 the 256-thread / 32-row choices are 2-20 % faster.
static int nw16_threads(int L, int k) {
  const int m = nw16_mode();
  if (m == 3) return 512;
  if (m == 1 && (160 * 1024) / nw_lds_bytes<NW_RW>(L, 4) == 0) return 512;
  return 256;
}
// 16-row workgroups (256 threads) read 32-row visits (k_nn_tn_w VIS = 32): MIGMRES_NT_VIS32=1.
// Off by default: measured slower at k = 16 (tools/mb_k16.cpp, same box: L = 224 8.45 vs
// 7.99 ms, L = 256 9.49 vs 8.82; profiles/r3_k16_nntn_vis32.txt) -- the wider visits do not
// make up for the loads' shorter cover (issued after the second half is published).
static bool nw16_vis32() {
  static int v = -1;
  if (v < 0) {
    const char *e = std::getenv("MIGMRES_NT_VIS32");
    v = e ? std::atoi(e) : 0;
  }
  return v != 0;
}
static int nw16_per_cu(int L, int k) { return nw16_threads(L, k) == 512 ? nw16_occ<512>(L, k) : nw16_occ<256>(L, k); }
static int nw_rw(int L, int k) {
  if (k > 8 && k <= 16 && L >= 64 && L + k <= 512) {
    const int m = nw16_mode();
    if (m >= 2) return 16;
    if (m == 1) {
      const int fit32 = (int)((160 * 1024) / nw_lds_bytes<NW_RW>(L, 4));
      if ((fit32 == 1 && nw16_per_cu(L, k) >= 2) || fit32 == 0) return 16;
    }
  }
  return NW_RW;
}
static int nw_wg_per_cu(int L, int k) {
  if (nw_rw(L, k) == 16) return nw16_per_cu(L, k);
  const int fit = (int)((160 * 1024) / nw_lds_bytes<NW_RW>(L, (k + 3) >> 2));
  return fit < NW_WG_PER_CU ? fit : NW_WG_PER_CU;
}
// k > 8: one workgroup stages each chunk of Q once and forms all k columns (NJ = 4) when its
// image and C1 fit the LDS (L <= 320 at k = 16); wider images run the two column halves in
// workgroup pairs on one XCD (paired: every chunk of Q enters two CUs, from HBM once and from
// L2 / the Infinity Cache once -- twice the bytes into the CUs, which is what bounds it).
static bool nw_single16(int L, int k) { return k > 8 && k <= 16 && L >= 64 && L + k <= 512 && nw_wg_per_cu(L, k) >= 1; }
// Smallest L of the wide form at k <= 8 (MIGMRES_NW_MIN_L, read per call): 16 for 4 <= k <= 8,
// where it now beats the narrow k_nn_tn at every L (256^3 k = 8, tools/mb_k16.cpp,
// profiles/r4u_k8_small_l.txt: L = 16 1.15 -> 0.94 ms, 48 1.97 -> 1.45, 56 2.10 -> 1.58; same-box
// bench lines, sweep_r4v_*: 256^3 99.1 -> 100.0 it/s, FlanProxy k = 4 1285 -> 1306), 64 below
// k = 4 (not measured).
static int nw_min_l(int k) {
  const char *e = std::getenv("MIGMRES_NW_MIN_L");
  return e ? std::atoi(e) : (k >= 4 ? 16 : 64);
}
static bool nw_ok(int L, int k) {
  if (k > 8) return k <= 16 && (nw_single16(L, k) || (L >= 64 && nw_ok(L, 8)));  // all columns, or halves
  return L >= nw_min_l(k) && L + k <= 512 && nw_wg_per_cu(L, k) >= 1;
}
bool nn_tn_paired(int L, int k) { return k > 8 && !m16_ok(L, k) && !pw_ok(L, k) && !nw_single16(L, k); }

static int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  return cus;
}

int nn_tn_blocks(int nrows, int L, int k) {
  if (m16_ok(L, k)) {
    const long long nchunks = (nrows + 31) / 32;
    long long b = (long long)m16_per_cu(L) * cu_count();
    if (b > nchunks) b = nchunks;
    return b < 1 ? 1 : (int)b;
  }
  if (pw_ok(L, k)) {
    const long long nchunks = (nrows + 15) / 16;
    long long b = (long long)pw_per_cu(L) * cu_count();
    if (b > nchunks) b = nchunks;
    return b < 1 ? 1 : (int)b;
  }
  if (nw_ok(L, k)) {
    const int kh = k > 8 ? 8 : k;
    const int rw = nw_rw(L, k);
    const long long nchunks = (nrows + rw - 1) / rw;
    const long long want = (long long)nw_wg_per_cu(L, k > 8 ? k : kh) * cu_count();
    if (nn_tn_paired(L, k)) {  // pairs of workgroups per chunk range, ranges in groups of 8 (one per XCD)
      const long long want = (long long)nw_wg_per_cu(L, kh) * cu_count();
      long long r = (want / 2) / 8 * 8;
      if (r > nchunks) r = nchunks / 8 * 8;
      if (r < 8) r = 8;
      return (int)(2 * r);
    }
    const long long b = want < nchunks ? want : nchunks;
    return b < 1 ? 1 : (int)b;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nt_pick<true>(L, k), 256, nt_lds_bytes(L)) != hipSuccess ||
      per_cu < 1)
    per_cu = 2;
  const long long nchunks = (nrows + NT_ROWS - 1) / NT_ROWS;
  long long b = (long long)per_cu * cu_count();
  if (b > nchunks) b = nchunks;
  return b < 1 ? 1 : (int)b;
}

bool nn_tn_supported(int L, int k) {
  return L >= 1 && k >= 1 && k <= 16 && (L <= NT_MAXL || m16_ok(L, k) || nw_ok(L, k) || pw_ok(L, k));
}

void launch_nn_tn(hipStream_t s, MvDesc Q, int L, const double *C1, int ldc, MvDesc X, int nrows,
                  double *partial, int nblocks, double *sink, bool store_x1) {
  const int k = X.ncols;
  if (!nn_tn_supported(L, k))
    throw Error(MIGMRES_EINVAL, "nn_tn: 1 <= k <= 16 and L <= 256 (L + k <= 512 for k <= 8, L >= 64)");
  if (m16_ok(L, k) && !Q.cols && !X.cols) {
    if (store_x1) throw Error(MIGMRES_EINVAL, "nn_tn: k > 8 is read-only");
    m16_per_cu(L);  // raises the kernel's dynamic LDS limit
    hipLaunchKernelGGL(m16_pick(L), dim3(nblocks), dim3(512), m16_lds_bytes(L), s, Q, L, C1, ldc, X, k, nrows,
                       partial, sink);
    LAUNCH_CHECK_();
    return;
  }
  if (pw_ok(L, k)) {
    if (store_x1) throw Error(MIGMRES_EINVAL, "nn_tn: k > 8 is read-only");
    const int LT = 16 * ((L + 15) >> 4);
    pw_per_cu(L);  // raises the kernel's dynamic LDS limit
    hipLaunchKernelGGL(pw_pick(L), dim3(nblocks), dim3(256), pw_lds_bytes(LT), s, Q, L, C1, ldc, X, k, nrows,
                       partial, sink);
    LAUNCH_CHECK_();
    return;
  }

  if (nw_ok(L, k)) {
    const bool paired = nn_tn_paired(L, k);
    if (paired && (nblocks % 16 != 0 || (long long)(nblocks / 2) > ((long long)nrows + NW_RW - 1) / NW_RW + 7))
      throw Error(MIGMRES_EINVAL, "nn_tn: k > 8 needs a grid of 16 q workgroups (nn_tn_blocks)");
    if (k > 8 && store_x1) throw Error(MIGMRES_EINVAL, "nn_tn: k > 8 is read-only");
    const int NJ = k > 8 ? (paired ? 2 : 4) : (k + 3) >> 2;
    const int kh = paired ? 8 : k;
    if (nw_rw(L, k) == 16) {
      const bool t512 = nw16_threads(L, k) == 512;
      // 32-row visits where C1 is in LDS anyway (images past 7 x 32 columns): same LDS and
      // occupancy as the 16-row visit form
      // (up to 10 x 32 columns: two waves per SIMD still fit its registers)
      const bool v32 = !t512 && nw16_vis32() && ((L + kh + 31) >> 5) > 7 && ((L + kh + 31) >> 5) <= 10;
      nt_kernel_t f = t512 ? nw_pick_nm<16, 4, false, 512>(L + kh)
                      : v32 ? nw_pick_nm<16, 4, false, 256, 32>(L + kh)
                            : nw_pick_nm<16, 4, false>(L + kh);
      static bool attr16[3][17] = {};
      const int nm = (L + kh + 31) >> 5;
      const int fv = t512 ? 1 : v32 ? 2 : 0;
      if (!attr16[fv][nm]) {
        if (hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
          throw Error(MIGMRES_EHIP, "nn_tn: cannot raise the dynamic LDS limit");
        attr16[fv][nm] = true;
      }
      const size_t lds16 = t512 ? nw_lds_bytes<16, 512>(L, 4, L + kh) : nw_lds_bytes<16>(L, 4, L + kh);
      hipLaunchKernelGGL(f, dim3(nblocks), dim3(t512 ? 512 : 256), lds16, s, Q, L, C1, ldc, X, k, nrows,
                         partial, sink);
      LAUNCH_CHECK_();
      return;
    }
    nt_kernel_t f = store_x1 ? (NJ == 1 ? nw_pick_nm<NW_RW, 1, true>(L + kh) : nw_pick_nm<NW_RW, 2, true>(L + kh))
                  : NJ == 4  ? nw_pick_nm<NW_RW, 4, false>(L + kh)
                             : (NJ == 1 ? nw_pick_nm<NW_RW, 1, false>(L + kh) : nw_pick_nm<NW_RW, 2, false>(L + kh));
    const size_t lds = nw_lds_bytes<NW_RW>(L, NJ);
    static bool attr_set[2][4][17] = {};
    const int nm = (L + kh + 31) >> 5;
    if (!attr_set[store_x1][NJ - 1][nm]) {
      if (hipFuncSetAttribute((const void *)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
        throw Error(MIGMRES_EHIP, "nn_tn: cannot raise the dynamic LDS limit");
      attr_set[store_x1][NJ - 1][nm] = true;
    }
    hipLaunchKernelGGL(f, dim3(nblocks), dim3(16 * NW_RW), lds, s, Q, L, C1, ldc, X, k, nrows, partial, sink);
  } else {
    hipLaunchKernelGGL(store_x1 ? nt_pick<true>(L, k) : nt_pick<false>(L, k), dim3(nblocks), dim3(256),
                       nt_lds_bytes(L), s, Q, L, C1, ldc, X, k, nrows, partial, sink);
  }
  LAUNCH_CHECK_();
}

// -------------------------------------------------------------------------------------
// findBasis column kernels on the block X (nrows x k, k <= 16), column j.
// -------------------------------------------------------------------------------------
// Row pairs: each thread handles rows (r, r+1) with 16-byte loads; the padding row of a
// pair (r+1 == nrows) reads the zero padding and is never written.
// (a) normalise column j-1 in place by inv[j-1]; partials [oldDot_j, <X_i, X_j> i<j]
__global__ __launch_bounds__(ICNT) void k_fb_a(MvDesc X, int j, FbPro pro, int nrows,
                                              double *__restrict__ partial) {
  __shared__ IcgsState ls;
  fb_prologue(pro, &ls);
  double v[17];
#pragma unroll
  for (int i = 0; i < 17; ++i) v[i] = 0.0;
  const double invp = j > 0 ? ls.inv[j - 1] : 1.0;
  double *xj = colp_(X, j);
  double *xp = j > 0 ? colp_(X, j - 1) : xj;
  for (long long r = 2LL * ((long long)blockIdx.x * ICNT + threadIdx.x); r < nrows;
       r += 2LL * gridDim.x * ICNT) {
    const d2 x = *(const d2 *)(xj + r);
    v[0] += x.x * x.x + x.y * x.y;
    if (j > 0) {
      const d2 p = *(const d2 *)(xp + r);
      const double q0 = invp * p.x, q1 = invp * p.y;
      st_pair(xp + r, q0, q1, r + 1 < nrows);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (i < j - 1) {
          const d2 y = *(const d2 *)(colp_(X, i) + r);
          v[1 + i] += y.x * x.x + y.y * x.y;
        } else if (i == j - 1) {
          v[1 + i] += q0 * x.x + q1 * x.y;
        }
      }
    }
  }
  block_reduce_store<17>(v, j + 1, partial);
}

// (b) x1 = X_j - sum_i X_i P_i  -> S ; partials <X_i, x1> (i < j)
__global__ __launch_bounds__(ICNT) void k_fb_b(MvDesc X, int j, const IcgsState *__restrict__ st,
                                              double *__restrict__ S, int nrows,
                                              double *__restrict__ partial) {
  double v[16];
  double P[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    v[i] = 0.0;
    P[i] = i < j ? st->P[i] : 0.0;
  }
  const double *xj = colp_(X, j);
  for (long long r = 2LL * ((long long)blockIdx.x * ICNT + threadIdx.x); r < nrows;
       r += 2LL * gridDim.x * ICNT) {
    d2 q[16];
    double t0 = 0.0, t1 = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < j) {
        q[i] = *(const d2 *)(colp_(X, i) + r);
        t0 += q[i].x * P[i];
        t1 += q[i].y * P[i];
      }
    const d2 x = *(const d2 *)(xj + r);
    const double a0 = x.x - t0, a1 = x.y - t1;
    st_pair(S + r, a0, a1, r + 1 < nrows);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < j) v[i] += q[i].x * a0 + q[i].y * a1;
  }
  block_reduce_store<16>(v, j, partial);
}

// (c) x2 = S - sum_i X_i P2_i -> X_j ; partials <x2, X_j(old)>
__global__ __launch_bounds__(ICNT) void k_fb_c(MvDesc X, int j, const IcgsState *__restrict__ st,
                                              const double *__restrict__ S, int nrows,
                                              double *__restrict__ partial) {
  double v[1] = {0.0};
  double P[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) P[i] = i < j ? st->P2[i] : 0.0;
  double *xj = colp_(X, j);
  for (long long r = 2LL * ((long long)blockIdx.x * ICNT + threadIdx.x); r < nrows;
       r += 2LL * gridDim.x * ICNT) {
    double t0 = 0.0, t1 = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < j) {
        const d2 y = *(const d2 *)(colp_(X, i) + r);
        t0 += y.x * P[i];
        t1 += y.y * P[i];
      }
    const d2 sv = *(const d2 *)(S + r);
    const d2 old = *(const d2 *)(xj + r);
    const double a0 = sv.x - t0, a1 = sv.y - t1;
    v[0] += a0 * old.x + a1 * old.y;
    st_pair(xj + r, a0, a1, r + 1 < nrows);
  }
  block_reduce_store<1>(v, 1, partial);
}

// Two passes per column instead of three.  The first projection of column j+1 onto the
// basis is accumulated in the same pass that finishes column j (k_fb_ca), against column j
// before its normalisation: <x2_j, X_{j+1}> is scaled by 1/diag_j afterwards (k_fb_scalar
// stage 6).  Column j - 1 stays unnormalised in memory until the pass that finishes column
// j (k_fb_ca) writes it back as x2_{j-1} * (1/diag_{j-1}) -- the value the reference stores
// -- and both passes of column j apply that scaling to it on the fly.  The first update
// x1 = X_j - sum_i X_i P_i is not stored between the passes: k_fb_ca recomputes it with the
// same operations in the same order (bit-identical), which saves writing and re-reading a
// column per step; k_fb_b2 is read-only.
//
// (a01) partials [oldDot_0, oldDot_1, <X_0, X_1>] with X_0 not yet normalised.
__global__ __launch_bounds__(ICNT) void k_fb_a01(MvDesc X, int nrows, double *__restrict__ partial) {
  double v[3] = {0.0, 0.0, 0.0};
  const double *x0 = colp_(X, 0), *x1 = colp_(X, 1);
  for (long long r = 2LL * ((long long)blockIdx.x * ICNT + threadIdx.x); r < nrows;
       r += 2LL * gridDim.x * ICNT) {
    const d2 a = *(const d2 *)(x0 + r);
    const d2 b = *(const d2 *)(x1 + r);
    v[0] += a.x * a.x + a.y * a.y;
    v[1] += b.x * b.x + b.y * b.y;
    v[2] += a.x * b.x + a.y * b.y;
  }
  block_reduce_store<3>(v, 3, partial);
}

// The column index j is a template parameter (k <= 16): the per-thread arrays hold exactly
// the j prior columns, and each thread takes U row pairs (one grid stride apart, so every
// wave-instruction still reads 1 KB contiguous per column) with all their loads issued
// before the arithmetic -- (j + 1) U 16-byte loads in flight per thread.  With one pair per
// thread the j = 1 pass had two loads in flight per thread.
template <int J>
struct FbU {
  static constexpr int U = J <= 2 ? 4 : J <= 5 ? 2 : 1;
};

// Row pair u of this thread's group starting at pair p0: the global pair (reversed when
// rev), clamped to a valid pair when past the end (ok = false: loaded, not used).
__device__ __forceinline__ long long fb_pair(long long p0, int u, long long stride, long long np, int rev,
                                             bool &ok) {
  const long long pu = p0 + u * stride;
  ok = pu < np;
  const long long pc = ok ? pu : np - 1;
  return 2 * (rev ? np - 1 - pc : pc);
}

// (b2) x1 = X_j - sum_i X_i P_i with X_{j-1} scaled by inv[j-1]; partials <X_i, x1> (i < j)
// and <x1, x1> (index j, the DGKS re-orthogonalisation test).  Writes nothing.
template <int J>
__global__ __launch_bounds__(ICNT) void k_fb_b2(MvDesc X, FbPro pro, int nrows, double *__restrict__ partial,
                                               int rev) {
  constexpr int U = FbU<J>::U;
  ProRegs pr;
  fb_pro_load(pro, pr);
  const double *xc[J + 1];
#pragma unroll
  for (int i = 0; i <= J; ++i) xc[i] = colp_(X, i);
  const long long np = (nrows + 1) / 2, stride = (long long)gridDim.x * ICNT;
  d2 q[U][J + 1];
  bool ok[U];
  // rows of group p0 (clamped past the end: loaded, not used)
  auto load = [&](long long p0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long r = fb_pair(p0, u, stride, np, rev, ok[u]);
#pragma unroll
      for (int i = 0; i <= J; ++i) q[u][i] = *(const d2 *)(xc[i] + r);
    }
  };
  long long p0 = (long long)blockIdx.x * ICNT + threadIdx.x;
  load(p0);  // in flight during the prologue
  __shared__ IcgsState ls;
  fb_pro_finish(pro, pr, &ls);
  double v[J + 1];
  double P[J];
#pragma unroll
  for (int i = 0; i <= J; ++i) v[i] = 0.0;
#pragma unroll
  for (int i = 0; i < J; ++i) P[i] = ls.P[i];
  const double invp = ls.inv[J - 1];
  for (; p0 < np; p0 += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      q[u][J - 1].x = invp * q[u][J - 1].x;
      q[u][J - 1].y = invp * q[u][J - 1].y;
      double t0 = 0.0, t1 = 0.0;
#pragma unroll
      for (int i = 0; i < J; ++i) {
        t0 += q[u][i].x * P[i];
        t1 += q[u][i].y * P[i];
      }
      const double a0 = q[u][J].x - t0, a1 = q[u][J].y - t1;
#pragma unroll
      for (int i = 0; i < J; ++i) v[i] += q[u][i].x * a0 + q[u][i].y * a1;
      v[J] += a0 * a0 + a1 * a1;
    }
    load(p0 + U * stride);
  }
  block_reduce_store<J + 1>(v, J + 1, partial);
}

// (ca) x1 as in (b2), x2 = x1 - sum_i X_i P2_i -> X_j (not normalised), X_{j-1} * inv[j-1]
// -> X_{j-1}; partials [newDot_j = <x2, X_j old>, and if j + 1 < k: oldDot_{j+1},
// <X_i, X_{j+1}> (i < j), <x2, X_{j+1}>]
template <int J>
__global__ __launch_bounds__(ICNT) void k_fb_ca(MvDesc X, int has_next, FbPro pro, int nrows,
                                               double *__restrict__ partial, int rev) {
  constexpr int U = FbU<J>::U;
  ProRegs pr;
  fb_pro_load(pro, pr);
  const double *xc[J + 1];
#pragma unroll
  for (int i = 0; i <= J; ++i) xc[i] = colp_(X, i);
  double *xj = colp_(X, J);
  double *xprev = colp_(X, J - 1);
  const double *xn = colp_(X, has_next ? J + 1 : J);
  const long long np = (nrows + 1) / 2, stride = (long long)gridDim.x * ICNT;
  d2 q[U][J + 2];  // [J] = X_j old, [J + 1] = X_{j+1}
  bool ok[U];
  long long rr[U];
  auto load = [&](long long p0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      rr[u] = fb_pair(p0, u, stride, np, rev, ok[u]);
#pragma unroll
      for (int i = 0; i <= J; ++i) q[u][i] = *(const d2 *)(xc[i] + rr[u]);
      q[u][J + 1] = has_next ? *(const d2 *)(xn + rr[u]) : d2{0.0, 0.0};
    }
  };
  long long p0 = (long long)blockIdx.x * ICNT + threadIdx.x;
  load(p0);  // in flight during the prologue
  __shared__ IcgsState ls;
  fb_pro_finish(pro, pr, &ls);
  double v[J + 3];
#pragma unroll
  for (int i = 0; i < J + 3; ++i) v[i] = 0.0;
  double P[J], P2[J];
#pragma unroll
  for (int i = 0; i < J; ++i) {
    P[i] = ls.P[i];
    P2[i] = ls.P2[i];
  }
  const double invp = ls.inv[J - 1];
  for (; p0 < np; p0 += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      const long long r = rr[u];
      const bool two = r + 1 < nrows;
      q[u][J - 1].x = invp * q[u][J - 1].x;
      q[u][J - 1].y = invp * q[u][J - 1].y;
      double t0 = 0.0, t1 = 0.0;
#pragma unroll
      for (int i = 0; i < J; ++i) {
        t0 += q[u][i].x * P[i];
        t1 += q[u][i].y * P[i];
      }
      const d2 old = q[u][J];
      const double s0 = old.x - t0, s1 = old.y - t1;
      double u0 = 0.0, u1 = 0.0;
#pragma unroll
      for (int i = 0; i < J; ++i) {
        u0 += q[u][i].x * P2[i];
        u1 += q[u][i].y * P2[i];
      }
      const double a0 = s0 - u0, a1 = s1 - u1;
      v[0] += a0 * old.x + a1 * old.y;
      st_pair(xj + r, a0, a1, two);
      st_pair(xprev + r, q[u][J - 1].x, q[u][J - 1].y, two);
      if (has_next) {
        const d2 nx = q[u][J + 1];
        v[1] += nx.x * nx.x + nx.y * nx.y;
#pragma unroll
        for (int i = 0; i < J; ++i) v[2 + i] += q[u][i].x * nx.x + q[u][i].y * nx.y;
        v[2 + J] += a0 * nx.x + a1 * nx.y;
      }
    }
    load(p0 + U * stride);
  }
  block_reduce_store<J + 3>(v, has_next ? J + 3 : 1, partial);
}

__global__ __launch_bounds__(ICNT) void k_scale_col(MvDesc X, int j, FbPro pro, int nrows) {
  __shared__ IcgsState ls;
  fb_prologue(pro, &ls);
  const double inv = ls.inv[j];
  double *x = colp_(X, j);
  const long long np = (nrows + 1) / 2;
  for (long long pp = (long long)blockIdx.x * ICNT + threadIdx.x; pp < np; pp += (long long)gridDim.x * ICNT) {
    const long long r = 2 * pp;
    const d2 v = *(const d2 *)(x + r);
    st_pair(x + r, inv * v.x, inv * v.y, r + 1 < nrows);
  }
}

// Scalar step after a reduction (red = reduced vector).  stage: 0 after (a), 1 after (b),
// 2 after (c), 3 after blkOrtho's projections (C = C1 + C2, dependency test), 4 for the
// k == 1 normalisation.

__global__ void k_fb_scalar(IcgsState *st, const double *__restrict__ red, int stage, int j, int k,
                            int complete) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  fb_scalar_body(st, red, stage, j, k, complete);
}

// Single-rank form of reduce_small + fb_scalar: one workgroup reduces the partials, then
// its thread 0 takes the scalar step (saves a launch per findBasis step).
__global__ __launch_bounds__(256) void k_reduce_scalar(const double *__restrict__ partial, int nblocks, int nv,
                                                       double *__restrict__ out, IcgsState *st, int stage, int j,
                                                       int k, int complete) {
  double v[17];
#pragma unroll
  for (int i = 0; i < 17; ++i) v[i] = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += 256) {
    add_partial_row(v, partial, b, nv);
  }
  __shared__ double red[4][17];
  __shared__ double sum[17];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 17; ++i) {
    if (i < nv) {
      double x = v[i];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
      if (l == 0) red[w][i] = x;
    }
  }
  __syncthreads();
  if (threadIdx.x < nv) {
    const int i = threadIdx.x;
    sum[i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
    out[i] = sum[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) fb_scalar_body(st, sum, stage, j, k, complete);
}

__device__ void fb_scalar_body(IcgsState *st, const double *red, int stage, int j, int k, int complete) {
  if (stage == 0) {
    st->oldDot[j] = red[0];
    if (st->oldDot[j] < 0.0) st->neg = 1.0;
    for (int i = 0; i < j; ++i) {
      st->P[i] = red[1 + i];
      st->prod[i] = red[1 + i];
    }
    if (j == 0) {  // no projection: newDot = oldDot
      const double nd = st->oldDot[0];
      st->newDot[0] = nd;
      const double tol = complete ? st->sing_tol : st->blk_tol;
      const bool dep = complete ? fabs(nd) < fabs(tol * st->oldDot[0]) : fabs(nd) < fabs(st->oldDot[0] * tol);
      if (dep && st->failed < 0) st->failed = 0;
      const double diag = sqrt(fabs(nd));
      st->diag[0] = diag;
      st->inv[0] = 1.0 / diag;
      st->B[0] = diag;
    }
  } else if (stage == 1) {
    // red[0..j-1] = <X_i, x1>, red[j] = <x1, x1>.  DGKS (BelosDGKSOrthoManager.hpp:1086-1119)
    // projects a second time only if sqrt|<x1,x1>| < dep_tol sqrt|oldDot|; otherwise the
    // second update runs with zero coefficients, which leaves x1 unchanged bit for bit.
    const bool reorth = !st->dgks || sqrt(fabs(red[j])) < st->dep_tol * sqrt(fabs(st->oldDot[j]));
    for (int i = 0; i < j; ++i) {
      st->P2[i] = reorth ? red[i] : 0.0;
      if (reorth) st->prod[i] = st->prod[i] + red[i];
    }
  } else if (stage == 2) {
    const double nd = red[0];
    st->newDot[j] = nd;
    const double tol = complete ? st->sing_tol : st->blk_tol;
    const bool dep = complete ? fabs(nd) < fabs(tol * st->oldDot[j]) : fabs(nd) < fabs(st->oldDot[j] * tol);
    if (dep && st->failed < 0) st->failed = j;
    const double diag = sqrt(fabs(nd));
    st->diag[j] = diag;
    st->inv[j] = 1.0 / diag;
    st->B[j + 16 * j] = diag;
    for (int i = 0; i < j; ++i) st->B[i + 16 * j] = st->prod[i];
  } else if (stage == 3) {
    // red = newDot (k values); oldDot from the Gram block recorded earlier
    for (int c = 0; c < k; ++c)
      if (fabs(red[c]) < fabs(st->blk_old[c] * st->blk_tol)) st->dep = 1.0;
  } else if (stage == 5) {
    // after k_fb_a01: column 0 (no projection) and the first projection of column 1
    st->oldDot[0] = red[0];
    st->oldDot[1] = red[1];
    if (red[0] < 0.0 || red[1] < 0.0) st->neg = 1.0;
    const double nd = red[0];
    st->newDot[0] = nd;
    const double tol = complete ? st->sing_tol : st->blk_tol;
    const bool dep = complete ? fabs(nd) < fabs(tol * nd) : fabs(nd) < fabs(nd * tol);
    if (dep && st->failed < 0) st->failed = 0;
    const double diag = sqrt(fabs(nd));
    st->diag[0] = diag;
    st->inv[0] = 1.0 / diag;
    st->B[0] = diag;
    st->P[0] = red[2] * st->inv[0];
    st->prod[0] = st->P[0];
  } else if (stage == 7) {
    // findBasis head from blkOrtho's closing dots (dmode 3 of k_gemm_nn_dot): red[0], red[1]
    // = <X_0, X_0>, <X_1, X_1>, red[k] = <X_0, X_1>; then as stage 5
    st->oldDot[0] = red[0];
    st->oldDot[1] = red[1];
    if (red[0] < 0.0 || red[1] < 0.0) st->neg = 1.0;
    const double nd = red[0];
    st->newDot[0] = nd;
    const double tol = complete ? st->sing_tol : st->blk_tol;
    const bool dep = complete ? fabs(nd) < fabs(tol * nd) : fabs(nd) < fabs(nd * tol);
    if (dep && st->failed < 0) st->failed = 0;
    const double diag = sqrt(fabs(nd));
    st->diag[0] = diag;
    st->inv[0] = 1.0 / diag;
    st->B[0] = diag;
    st->P[0] = red[k] * st->inv[0];
    st->prod[0] = st->P[0];
  } else if (stage == 6) {
    // after k_fb_ca: finish column j as stage 2, then column j+1's first projection
    const double nd = red[0];
    st->newDot[j] = nd;
    const double tol = complete ? st->sing_tol : st->blk_tol;
    const bool dep = complete ? fabs(nd) < fabs(tol * st->oldDot[j]) : fabs(nd) < fabs(st->oldDot[j] * tol);
    if (dep && st->failed < 0) st->failed = j;
    const double diag = sqrt(fabs(nd));
    st->diag[j] = diag;
    st->inv[j] = 1.0 / diag;
    st->B[j + 16 * j] = diag;
    for (int i = 0; i < j; ++i) st->B[i + 16 * j] = st->prod[i];
    if (j + 1 < k) {
      st->oldDot[j + 1] = red[1];
      if (red[1] < 0.0) st->neg = 1.0;
      for (int i = 0; i < j; ++i) st->P[i] = red[2 + i];
      st->P[j] = red[2 + j] * st->inv[j];
      for (int i = 0; i <= j; ++i) st->prod[i] = st->P[i];
    }
  } else if (stage == 4) {
    const double d = red[0];
    const double b = sqrt(fabs(d));
    st->B[0] = b;
    st->diag[0] = b;
    st->inv[0] = fabs(b) > 0.0 ? 1.0 / b : 1.0;
  }
}

// Record blkOrtho's oldDot = diag(X^T X) from the Gram block (rows L..L+k-1 of the
// (L+k) x k product) and reset the per-call flags.
__global__ void k_blk_old(IcgsState *st, const double *__restrict__ G, int ldg, int L, int k) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int c = 0; c < k; ++c) st->blk_old[c] = G[(L + c) + (long long)c * ldg];
}

__global__ void k_state_reset(IcgsState *st, double blk_tol, double sing_tol, int dgks, double dep_tol) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  st->dgks = dgks;
  st->dep_tol = dep_tol;
  st->failed = -1;
  st->dep = 0.0;
  st->neg = 0.0;
  st->blk_tol = blk_tol;
  st->sing_tol = sing_tol;
  for (int i = 0; i < 256; ++i) st->B[i] = 0.0;
}

// C_out[i + j*ldo] = C1[i + j*ld1] + C2[i + j*ld2] for i < L, j < k
__global__ void k_add_coef(const double *__restrict__ C1, int ld1, const double *__restrict__ C2, int ld2,
                           double *__restrict__ out, int ldo, int L, int k) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= L * k) return;
  const int i = e % L, j = e / L;
  out[i + (long long)j * ldo] = C1[i + (long long)j * ld1] + C2[i + (long long)j * ld2];
}

void launch_fb_a(hipStream_t s, MvDesc X, int j, const FbPro &pro, int nrows, double *partial, int nb) {
  k_fb_a<<<nb, ICNT, 0, s>>>(X, j, pro, nrows, partial);
  LAUNCH_CHECK_();
}
void launch_fb_b(hipStream_t s, MvDesc X, int j, const IcgsState *st, double *S, int nrows, double *partial, int nb) {
  k_fb_b<<<nb, ICNT, 0, s>>>(X, j, st, S, nrows, partial);
  LAUNCH_CHECK_();
}
void launch_fb_c(hipStream_t s, MvDesc X, int j, const IcgsState *st, const double *S, int nrows, double *partial,
                 int nb) {
  k_fb_c<<<nb, ICNT, 0, s>>>(X, j, st, S, nrows, partial);
  LAUNCH_CHECK_();
}
void launch_fb_a01(hipStream_t s, MvDesc X, int nrows, double *partial, int nb) {
  k_fb_a01<<<nb, ICNT, 0, s>>>(X, nrows, partial);
  LAUNCH_CHECK_();
}
#define FB_CASES(M) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)
void launch_fb_b2(hipStream_t s, MvDesc X, int j, const FbPro &pro, int nrows, double *partial, int nb,
                  int rev) {
  switch (j) {
#define B2_CASE(J) \
  case J:          \
    k_fb_b2<J><<<nb, ICNT, 0, s>>>(X, pro, nrows, partial, rev); \
    break;
    FB_CASES(B2_CASE)
#undef B2_CASE
    default:
      throw Error(MIGMRES_EINVAL, "fb_b2: column index must be in 1..15");
  }
  LAUNCH_CHECK_();
}
void launch_fb_ca(hipStream_t s, MvDesc X, int j, int has_next, const FbPro &pro, int nrows, double *partial,
                  int nb, int rev) {
  switch (j) {
#define CA_CASE(J) \
  case J:          \
    k_fb_ca<J><<<nb, ICNT, 0, s>>>(X, has_next, pro, nrows, partial, rev); \
    break;
    FB_CASES(CA_CASE)
#undef CA_CASE
    default:
      throw Error(MIGMRES_EINVAL, "fb_ca: column index must be in 1..15");
  }
  LAUNCH_CHECK_();
}
void launch_scale_col(hipStream_t s, MvDesc X, int j, const FbPro &pro, int nrows, int nb) {
  // launched on a rank that owns no rows too: its prologue applies the pending scalar step,
  // which every rank must take to keep the device state (and the decisions read from it) equal
  k_scale_col<<<nb > 0 ? nb : 1, ICNT, 0, s>>>(X, j, pro, nrows);
  LAUNCH_CHECK_();
}
void launch_fb_flush(hipStream_t s, const FbPro &pro) {
  k_fb_flush<<<1, ICNT, 0, s>>>(pro);
  LAUNCH_CHECK_();
}
void launch_reduce_scalar(hipStream_t s, const double *partial, int nblocks, int nv, double *red, IcgsState *st,
                          int stage, int j, int k, int complete) {
  k_reduce_scalar<<<1, 256, 0, s>>>(partial, nblocks, nv, red, st, stage, j, k, complete);
  LAUNCH_CHECK_();
}
void launch_fb_scalar(hipStream_t s, IcgsState *st, const double *red, int stage, int j, int k, int complete) {
  k_fb_scalar<<<1, 64, 0, s>>>(st, red, stage, j, k, complete);
  LAUNCH_CHECK_();
}
void launch_blk_old(hipStream_t s, IcgsState *st, const double *G, int ldg, int L, int k) {
  k_blk_old<<<1, 64, 0, s>>>(st, G, ldg, L, k);
  LAUNCH_CHECK_();
}
void launch_state_reset(hipStream_t s, IcgsState *st, double blk_tol, double sing_tol, int dgks, double dep_tol) {
  k_state_reset<<<1, 64, 0, s>>>(st, blk_tol, sing_tol, dgks, dep_tol);
  LAUNCH_CHECK_();
}
void launch_add_coef(hipStream_t s, const double *C1, int ld1, const double *C2, int ld2, double *out, int ldo,
                     int L, int k) {
  if (L * k <= 0) return;
  k_add_coef<<<cdiv_((long long)L * k, 256), 256, 0, s>>>(C1, ld1, C2, ld2, out, ldo, L, k);
  LAUNCH_CHECK_();
}

// -------------------------------------------------------------------------------------
// findBasis in Gram form: ICGS with two passes, completeBasis = false, 2 <= k <= 8 -- the
// blkOrtho -> findBasis step of every block iteration (FastIcgs::find_basis_gram).
//
// Column-by-column CGS2 over the block (BelosICGSOrthoManager.hpp:1002-1222) computes, in
// exact arithmetic, B = R with R^T R = X^T X (the Cholesky factor of the block's Gram
// matrix, positive diagonal) and X <- X R^{-1}; its dependency ratio newDot_j / oldDot_j
// (:1190) is R_jj^2 / (X^T X)_jj.  Here the block is streamed twice after the closing
// update instead of in 2k - 1 passes over 2 .. k + 2 columns (24Nk bytes against about 8N x
// 92 at k = 8):
//   k_gemm_nn_gram  blkOrtho's closing update X <- X - Q M with the partials of G1 = X^T X
//                   (k_fbg_gram: G1 in a read pass of its own, for the unfused A/B form)
//   k_fbg_chol 1    blkOrtho's dependency test on diag(G1) (:1433-1442), R1 = chol(G1),
//                   the gate, T1 = R1^{-1}
//   k_fbg_a         partials of G2 = Y^T Y, Y = X T1 formed in registers    (read k columns)
//   k_fbg_chol 2    R2 = chol(G2), T2 = R2^{-1}, B = R2 R1
//   k_fbg_b         X <- (X T1) T2, Y re-formed bit for bit          (read + write k columns)
// -- CholQR2 (the reference's s-step GMRES normalises with CholQR too:
// Belos_Tpetra_GmresSstep.hpp:16, 162-168), as accurate as CGS2 on a well-conditioned block.
// The gate keeps it to such blocks: a pivot ratio R1_jj^2 / G1_jj below `gate` (100 blk_tol
// by default, far above the reference's own threshold) sets gram_skip, k_fbg_a / k_fbg_b
// return at once, and the host runs the column passes on the block, which still holds X - Q M.
// Packed upper triangle: entry (i, j), i <= j, at j (j + 1) / 2 + i.  Partials are stored
// value-major (partial[i * gridDim.x + b]) so that k_fbg_chol reads them coalesced.
// -------------------------------------------------------------------------------------
constexpr int FBG_NT = 256;

template <int NV>
__device__ __forceinline__ void fbg_reduce_store(double (&v)[NV], double *partial) {
  __shared__ double red[FBG_NT / 64][NV];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    double x = v[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
    if (l == 0) red[w][i] = x;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NV; i += FBG_NT)
    partial[(long long)i * gridDim.x + blockIdx.x] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

__device__ __forceinline__ long long fbg_row(long long p, long long np, int rev) {
  return 2 * (rev ? np - 1 - p : p);
}

template <int K>
__device__ __forceinline__ void fbg_gram_acc(const d2 (&x)[K], double (&g)[K * (K + 1) / 2]) {
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int i = 0; i <= j; ++i) g[j * (j + 1) / 2 + i] += x[i].x * x[j].x + x[i].y * x[j].y;
}

// x <- x T, T upper triangular (T[i + 16 c]); in place from the last column down (column c
// of the product reads x_0 .. x_c only).
template <int K>
__device__ __forceinline__ void fbg_apply(d2 (&x)[K], const double (&T)[16 * K]) {
#pragma unroll
  for (int c = K - 1; c >= 0; --c) {
    d2 a = x[0] * T[16 * c];
#pragma unroll
    for (int i = 1; i <= c; ++i) a += x[i] * T[i + 16 * c];
    x[c] = a;
  }
}

// Rows past nrows are the zero padding of the multivectors (ld > nrows): an odd tail's second
// row reads as zero, adds nothing to a Gram matrix and is not stored.
template <int K>
__global__ __launch_bounds__(FBG_NT) void k_gemm_nn_gram(MvDesc A, int L, const double *__restrict__ M, int ldm,
                                                        MvDesc X, int nrows, double *__restrict__ partial,
                                                        NngPro pro) {
  extern __shared__ __attribute__((aligned(16))) double Mg[];  // L x K
  const bool first = blockIdx.x == 0;
  for (int e = threadIdx.x; e < L * K; e += FBG_NT) {
    const int j = e / K, c = e % K;
    double m;
    if (pro.C1) {
      m = pro.C1[j + (long long)c * pro.ld1] + pro.C2[j + (long long)c * pro.ld2];  // k_add_coef's sum
      if (first) pro.cout[j + (long long)c * pro.ldo] = m;
    } else {
      m = M[j + (long long)c * ldm];
    }
    Mg[e] = m;
  }
  if (first && pro.st && threadIdx.x == 0) {  // k_state_reset, then k_blk_old
    IcgsState *st = pro.st;
    st->dgks = pro.dgks;
    st->dep_tol = pro.dep_tol;
    st->failed = -1;
    st->dep = 0.0;
    st->neg = 0.0;
    st->blk_tol = pro.blk_tol;
    st->sing_tol = pro.sing_tol;
    for (int i = 0; i < 256; ++i) st->B[i] = 0.0;
    for (int c = 0; c < K; ++c) st->blk_old[c] = pro.G[(L + c) + (long long)c * pro.ldg];
  }
  __syncthreads();
  constexpr int NV = K * (K + 1) / 2, NB = 8;
  double g[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) g[i] = 0.0;
  // row pairs grid-stride (the resident grid sweeps one band at a time), or (pro.contig)
  // workgroup b streams its own contiguous range of 512-row steps
  long long rb = 2LL * ((long long)blockIdx.x * FBG_NT + threadIdx.x), re = nrows, rs = 2LL * gridDim.x * FBG_NT;
  if (pro.contig) {
    const long long nst = ((long long)nrows + 2 * FBG_NT - 1) / (2 * FBG_NT);
    rb = (nst * blockIdx.x / gridDim.x) * 2 * FBG_NT + 2 * threadIdx.x;
    re = (nst * (blockIdx.x + 1) / gridDim.x) * 2 * FBG_NT;
    re = re < nrows ? re : nrows;
    rs = 2 * FBG_NT;
  }
  for (long long r = rb; r < re; r += rs) {
    d2 acc[K];
#pragma unroll
    for (int c = 0; c < K; ++c) acc[c] = d2{0.0, 0.0};
    int j = 0;
    for (; j + NB <= L; j += NB) {
      d2 v[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) v[u] = nn_load((const d2 *)(colp_(A, j + u) + r));
#pragma unroll
      for (int u = 0; u < NB; ++u)
#pragma unroll
        for (int c = 0; c < K; ++c) acc[c] += v[u] * Mg[(j + u) * K + c];
    }
    for (; j < L; ++j) {
      const d2 v = *(const d2 *)(colp_(A, j) + r);
#pragma unroll
      for (int c = 0; c < K; ++c) acc[c] += v * Mg[j * K + c];
    }
    const bool two = r + 1 < nrows;
#pragma unroll
    for (int c = 0; c < K; ++c) {
      double *xp = colp_(X, c) + r;
      acc[c] = *(const d2 *)xp - acc[c];
      st_pair(xp, acc[c].x, acc[c].y, two);
    }
    fbg_gram_acc<K>(acc, g);
  }
  fbg_reduce_store<NV>(g, partial);
}

template <int K>
__global__ __launch_bounds__(FBG_NT) void k_fbg_gram(MvDesc X, int nrows, double *__restrict__ partial, int rev) {
  constexpr int NV = K * (K + 1) / 2;
  double g[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) g[i] = 0.0;
  const long long np = ((long long)nrows + 1) / 2, stride = (long long)gridDim.x * FBG_NT;
  for (long long p = (long long)blockIdx.x * FBG_NT + threadIdx.x; p < np; p += stride) {
    const long long r = fbg_row(p, np, rev);
    d2 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = *(const d2 *)(colp_(X, c) + r);
    fbg_gram_acc<K>(x, g);
  }
  fbg_reduce_store<NV>(g, partial);
}

template <int K>
__global__ __launch_bounds__(FBG_NT) void k_fbg_a(MvDesc X, int nrows, const IcgsState *__restrict__ st,
                                                 const double *__restrict__ w, double *__restrict__ partial, int rev) {
  if (st->gram_skip || st->gram_single) return;
  __shared__ double T1[16 * K];
  for (int e = threadIdx.x; e < 16 * K; e += FBG_NT) T1[e] = w[e];
  __syncthreads();
  constexpr int NV = K * (K + 1) / 2;
  double g[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) g[i] = 0.0;
  const long long np = ((long long)nrows + 1) / 2, stride = (long long)gridDim.x * FBG_NT;
  for (long long p = (long long)blockIdx.x * FBG_NT + threadIdx.x; p < np; p += stride) {
    const long long r = fbg_row(p, np, rev);
    d2 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = *(const d2 *)(colp_(X, c) + r);
    fbg_apply<K>(x, T1);
    fbg_gram_acc<K>(x, g);
  }
  fbg_reduce_store<NV>(g, partial);
}

template <int K>
__global__ __launch_bounds__(FBG_NT) void k_fbg_b(MvDesc X, int nrows, const IcgsState *__restrict__ st,
                                                 const double *__restrict__ w, int rev) {
  if (st->gram_skip) return;
  const bool single = st->gram_single != 0;  // DGKS CholQR1: X T1 only
  __shared__ double T1[16 * K], T2[16 * K];
  for (int e = threadIdx.x; e < 16 * K; e += FBG_NT) {
    T1[e] = w[e];
    T2[e] = w[256 + e];
  }
  __syncthreads();
  const long long np = ((long long)nrows + 1) / 2, stride = (long long)gridDim.x * FBG_NT;
  for (long long p = (long long)blockIdx.x * FBG_NT + threadIdx.x; p < np; p += stride) {
    const long long r = fbg_row(p, np, rev);
    d2 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = *(const d2 *)(colp_(X, c) + r);
    fbg_apply<K>(x, T1);
    if (!single) fbg_apply<K>(x, T2);
    const bool two = r + 1 < nrows;
#pragma unroll
    for (int c = 0; c < K; ++c) st_pair(colp_(X, c) + r, x[c].x, x[c].y, two);
  }
}

template <int K>
__device__ __forceinline__ void fbg_step(const double (&g)[K * (K + 1) / 2], int stage, IcgsState *st,
                                         double *__restrict__ w, double gate, bool gw, double *Tl, int *fl);

// k_fbg_a / k_fbg_b with the k x k step in their prologue (FBG_PRO): every workgroup's thread 0
// takes the step from the all-reduced sums (the same inputs, so the same decisions on every
// workgroup), workgroup 0 also writing the state, T and R; then the pass.  Two one-workgroup
// launches (four with a distributed reduction) fewer per block iteration.
template <int K>
__global__ __launch_bounds__(FBG_NT) void k_fbg_a_p(MvDesc X, int nrows, IcgsState *st, double *__restrict__ w,
                                                   const double *__restrict__ gsum, double gate,
                                                   double *__restrict__ partial, int rev) {
  constexpr int NV = K * (K + 1) / 2;
  __shared__ double T1[16 * K];
  __shared__ int fl[2];
  if (threadIdx.x == 0) {
    double g[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) g[i] = gsum[i];
    fbg_step<K>(g, 1, st, w, gate, blockIdx.x == 0, T1, fl);
  }
  __syncthreads();
  if (fl[0] || fl[1]) return;  // handed back, or DGKS's single pass (no G2)
  double g[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) g[i] = 0.0;
  const long long np = ((long long)nrows + 1) / 2, stride = (long long)gridDim.x * FBG_NT;
  for (long long p = (long long)blockIdx.x * FBG_NT + threadIdx.x; p < np; p += stride) {
    const long long r = fbg_row(p, np, rev);
    d2 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = *(const d2 *)(colp_(X, c) + r);
    fbg_apply<K>(x, T1);
    fbg_gram_acc<K>(x, g);
  }
  fbg_reduce_store<NV>(g, partial);
}

template <int K>
__global__ __launch_bounds__(FBG_NT) void k_fbg_b_p(MvDesc X, int nrows, IcgsState *st, double *__restrict__ w,
                                                   const double *__restrict__ gsum, double gate, int rev) {
  constexpr int NV = K * (K + 1) / 2;
  if (st->gram_skip) return;
  const bool single = st->gram_single != 0;  // DGKS CholQR1: X T1 only
  __shared__ double T1[16 * K], T2[16 * K];
  __shared__ int fl[2];
  for (int e = threadIdx.x; e < 16 * K; e += FBG_NT) T1[e] = w[e];
  if (threadIdx.x == 0) {
    fl[0] = 0;
    if (!single) {
      double g[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) g[i] = gsum[i];
      fbg_step<K>(g, 2, st, w, gate, blockIdx.x == 0, T2, fl);
    }
  }
  __syncthreads();
  if (fl[0]) return;  // R2's gate: the block goes back to the column passes (X unchanged)
  const long long np = ((long long)nrows + 1) / 2, stride = (long long)gridDim.x * FBG_NT;
  for (long long p = (long long)blockIdx.x * FBG_NT + threadIdx.x; p < np; p += stride) {
    const long long r = fbg_row(p, np, rev);
    d2 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = *(const d2 *)(colp_(X, c) + r);
    fbg_apply<K>(x, T1);
    if (!single) fbg_apply<K>(x, T2);
    const bool two = r + 1 < nrows;
#pragma unroll
    for (int c = 0; c < K; ++c) st_pair(colp_(X, c) + r, x[c].x, x[c].y, two);
  }
}

// findBasis in Gram form for 9 <= k <= 16.  A row pair's k(k+1)/2 register sums and the
// hoisted T matrices no longer fit (k_fbg_b<16> spilled 708 B per lane and ran at 1.9 TB/s),
// so both products run on v_mfma_f64_16x16x4f64:
//  * X T in the transposed form (X T)^T = T^T X^T, 16 rows per MFMA chain: the B operand of
//    step s is X[r0 + (l & 15)][4 s + (l >> 4)] (16 rows of a column: one 128-B segment per
//    16 lanes), the A operand T[4 s + (l >> 4)][l & 15] (4 registers per lane for the whole
//    launch), and D[q] = (X T)[r0 + (l & 15)][4 q + (l >> 4)] -- exactly the B operand of step
//    q of a second product, so (X T1) T2 needs no transpose;
//  * the Gram matrix: each wave writes its 128 rows x 16 columns to LDS column-major (stride
//    FBM_S) and accumulates G = Y^T Y, whose A and B operands are then the same element.
// Y = X T1 is formed by the same MFMA sequence in k_fbg_gram_m<K, true> and k_fbg_b_m, so the
// block k_fbg_b_m writes is (Y T2) of the Y whose Gram matrix gave T2.  Columns >= k are zero.
constexpr int FBM_S = 132;  // 128 rows + 4 (LDS column stride)

template <int K>
__device__ __forceinline__ void fbm_coef(const double *__restrict__ w, double (&a)[4]) {
  const int l = threadIdx.x & 63, c = l & 15;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int i = 4 * s + (l >> 4);
    a[s] = (i <= c && c < K) ? w[i + 16 * c] : 0.0;
  }
}
__device__ __forceinline__ d4 fbm_mul(const double (&a)[4], const double (&b)[4]) {
  d4 d = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4; ++s) d = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], d, 0, 0, 0);
  return d;
}
// per-lane column pointers of the B-operand layout: column 4 s + (l >> 4), nullptr past k
template <int K>
__device__ __forceinline__ void fbm_cols(const MvDesc &X, double *(&xp)[4]) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int c = 4 * s + (l >> 4);
    xp[s] = c < K ? colp_(X, c) : nullptr;
  }
}

// APPLY: partials of G2 = (X T1)^T (X T1) (k_fbg_a); else of G1 = X^T X (k_fbg_gram).
// Partials block-major (partial[b * NV + i]) for launch_reduce_partials.
template <int K, bool APPLY>
__global__ __launch_bounds__(FBG_NT) void k_fbg_gram_m(MvDesc X, int nrows, const IcgsState *__restrict__ st,
                                                      const double *__restrict__ w, double *__restrict__ partial,
                                                      int rev) {
  if (APPLY && (st->gram_skip || st->gram_single)) return;
  constexpr int NV = K * (K + 1) / 2, NW = FBG_NT / 64;
  __shared__ __attribute__((aligned(16))) double tile[NW][16 * FBM_S];
  __shared__ double red[NW][NV];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6, lr = l & 15, lc = l >> 4;
  double *tw = tile[wv];
  double a1[4] = {0.0, 0.0, 0.0, 0.0};
  if (APPLY) fbm_coef<K>(w, a1);
  double *xp[4];
  fbm_cols<K>(X, xp);
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  const long long nq = ((long long)nrows + 127) / 128;
  for (long long q = (long long)blockIdx.x * NW + wv; q < nq; q += (long long)gridDim.x * NW) {
    const long long r0 = 128 * (rev ? nq - 1 - q : q);
    double xv[8][4];
#pragma unroll
    for (int g = 0; g < 8; ++g)
#pragma unroll
      for (int s = 0; s < 4; ++s) xv[g][s] = xp[s] ? xp[s][r0 + 16 * g + lr] : 0.0;  // rows >= nrows: zero padding
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      if (APPLY) {
        const d4 y = fbm_mul(a1, xv[g]);
#pragma unroll
        for (int s = 0; s < 4; ++s) xv[g][s] = y[s];
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) tw[(4 * s + lc) * FBM_S + 16 * g + lr] = xv[g][s];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own stores before its reads
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      const double a = tw[lr * FBM_S + 4 * s + lc];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, acc, 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next stores
  }
  // lane l holds G[(l >> 4) + 4 q][l & 15], q = 0..3
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = lc + 4 * q, j = lr;
    if (i <= j && j < K) red[wv][j * (j + 1) / 2 + i] = acc[q];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NV; i += FBG_NT)
    partial[(long long)blockIdx.x * NV + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

// X <- (X T1) T2 for 9 <= k <= 16 (k_fbg_b's step), both products on MFMA as above
template <int K>
__global__ __launch_bounds__(FBG_NT) void k_fbg_b_m(MvDesc X, int nrows, const IcgsState *__restrict__ st,
                                                   const double *__restrict__ w, int rev) {
  if (st->gram_skip) return;
  const bool single = st->gram_single != 0;  // DGKS CholQR1: X T1 only
  constexpr int NW = FBG_NT / 64;
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6, lr = l & 15;
  double a1[4], a2[4];
  fbm_coef<K>(w, a1);
  fbm_coef<K>(w + 256, a2);
  double *xp[4];
  fbm_cols<K>(X, xp);
  const long long nq = ((long long)nrows + 63) / 64;
  for (long long q = (long long)blockIdx.x * NW + wv; q < nq; q += (long long)gridDim.x * NW) {
    const long long r0 = 64 * (rev ? nq - 1 - q : q);
    double xv[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int s = 0; s < 4; ++s) xv[g][s] = xp[s] ? xp[s][r0 + 16 * g + lr] : 0.0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const d4 y = fbm_mul(a1, xv[g]);
      double yb[4] = {y[0], y[1], y[2], y[3]};
      const d4 z = single ? y : fbm_mul(a2, yb);
      const long long r = r0 + 16 * g + lr;
      if (r < nrows) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if (xp[s]) xp[s][r] = z[s];
      }
    }
  }
}

// The k x k step of k_fbg_chol for 9 <= k <= 16 on the summed Gram matrix (packed upper
// triangle in g): the same operations in the same order per element, with R and T in LDS and
// the independent elements on separate threads (one thread would hold 400+ live doubles).
__global__ __launch_bounds__(256) void k_fbg_chol_l(const double *__restrict__ gsum, int k, int stage,
                                                   IcgsState *st, double *__restrict__ w, double gate) {
  __shared__ double g[136], R[16][17], T[16][17];
  __shared__ int ok, any2, all2;
  const int t = threadIdx.x, nv = k * (k + 1) / 2;
  if (t < nv) g[t] = gsum[t];
  if (t == 0) ok = 1, any2 = 0, all2 = 1;
  __syncthreads();
  if (stage == 2 && (st->gram_skip || st->gram_single)) return;
  if (stage == 1 && t == 0) {
    st->gram_skip = 0;
    st->gram_single = 0;
    st->gram_mixed = 0;
    bool dep = false;
    for (int c = 0; c < k; ++c) dep = dep || fabs(g[c * (c + 1) / 2 + c]) < fabs(st->blk_old[c] * st->blk_tol);
    if (dep) st->dep = 1.0;
  }
  for (int j = 0; j < k; ++j) {
    if (t == 0) {
      const double gjj = g[j * (j + 1) / 2 + j];
      double s = gjj;
      for (int i = 0; i < j; ++i) s -= R[i][j] * R[i][j];
      if (!(gjj > 0.0 && s >= gate * gjj)) ok = 0;
      if (j > 0) {  // DGKS findBasis: a second projection iff sqrt|newDot| < dep_tol sqrt|oldDot|
        const bool two = sqrt(fabs(s)) < st->dep_tol * sqrt(fabs(gjj));
        any2 |= two;
        all2 &= two;
      }
      R[j][j] = sqrt(fabs(s));
    }
    __syncthreads();
    if (t > j && t < k) {
      double v = g[t * (t + 1) / 2 + j];
      for (int i = 0; i < j; ++i) v -= R[i][j] * R[i][t];
      R[j][t] = v / R[j][j];
    }
    __syncthreads();
  }
  if (!ok) {
    if (t == 0) st->gram_skip = 1;
    return;
  }
  const bool dgks = stage == 1 && st->dgks;
  if (dgks && any2 && !all2) {  // DGKS re-projects some columns only: the column passes
    if (t == 0) st->gram_skip = st->gram_mixed = 1;
    return;
  }
  const bool single = dgks && !any2;  // DGKS: one projection per column = CholQR1, B = R1
  if (single && t == 0) st->gram_single = 1;
  if (single && t < nv) {
    int c = 0;
    while ((c + 1) * (c + 2) / 2 <= t) ++c;
    const int i = t - c * (c + 1) / 2;
    st->B[i + 16 * c] = R[i][c];
  }
  if (t < k) {  // column t of T = R^{-1}
    const int c = t;
    T[c][c] = 1.0 / R[c][c];
    for (int i = c - 1; i >= 0; --i) {
      double v = 0.0;
      for (int m = i + 1; m <= c; ++m) v += R[i][m] * T[m][c];
      T[i][c] = -v / R[i][i];
    }
    double *Tout = w + (stage == 1 ? 0 : 256);
    for (int i = 0; i <= c; ++i) Tout[i + 16 * c] = T[i][c];
    if (stage == 1)
      for (int i = 0; i <= c; ++i) w[512 + i + 16 * c] = R[i][c];
  }
  if (stage == 2 && t < nv) {  // B = R2 R1, element (i, c) of the packed upper triangle
    int c = 0;
    while ((c + 1) * (c + 2) / 2 <= t) ++c;
    const int i = t - c * (c + 1) / 2;
    double v = 0.0;
    for (int m = i; m <= c; ++m) v += R[i][m] * w[512 + m + 16 * c];
    st->B[i + 16 * c] = v;
  }
}

// The k x k step of findBasis in Gram form on the summed Gram matrix g (packed upper
// triangle), by one thread: stage 1 = blkOrtho's dependency test on diag(G1), R1 = chol(G1)
// with the pivot-ratio gate and DGKS's per-column decisions, T1 = R1^{-1}; stage 2 = R2, T2,
// B = R2 R1.  gw: write the state, T and R to global memory (one workgroup does); Tl (LDS,
// optional): T for the caller's pass; fl (optional): {hand the block back, DGKS single pass}.
// Register arrays (fully unrolled): the factorisations are chains of dependent operations,
// which through LDS cost tens of us.
template <int K>
__device__ __forceinline__ void fbg_step(const double (&g)[K * (K + 1) / 2], int stage, IcgsState *st,
                                         double *__restrict__ w, double gate, bool gw, double *Tl, int *fl) {
  int skip = 0, single_f = 0;
  if (stage == 1 && gw) {
    st->gram_skip = 0;
    st->gram_single = 0;
    st->gram_mixed = 0;
    bool dep = false;
#pragma unroll
    for (int c = 0; c < K; ++c) dep = dep || fabs(g[c * (c + 1) / 2 + c]) < fabs(st->blk_old[c] * st->blk_tol);
    if (dep) st->dep = 1.0;
  }
  // G = R^T R, R upper triangular with a positive diagonal; pivot ratios against the gate
  double R[K][K], T[K][K];
  bool ok = true, any2 = false, all2 = true;
  const double dep_tol = st->dep_tol;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double gjj = g[j * (j + 1) / 2 + j];
    double s = gjj;
#pragma unroll
    for (int i = 0; i < j; ++i) s -= R[i][j] * R[i][j];
    ok = ok && gjj > 0.0 && s >= gate * gjj;
    if (j > 0) {  // DGKS findBasis: a second projection iff sqrt|newDot| < dep_tol sqrt|oldDot|
      const bool two = sqrt(fabs(s)) < dep_tol * sqrt(fabs(gjj));
      any2 = any2 || two;
      all2 = all2 && two;
    }
    const double d = sqrt(fabs(s));
    R[j][j] = d;
#pragma unroll
    for (int c = j + 1; c < K; ++c) {
      double t = g[c * (c + 1) / 2 + j];
#pragma unroll
      for (int i = 0; i < j; ++i) t -= R[i][j] * R[i][c];
      R[j][c] = t / d;
    }
  }
  const bool dgks = stage == 1 && st->dgks;
  if (!ok) {
    skip = 1;
    if (gw) st->gram_skip = 1;
  } else if (dgks && any2 && !all2) {  // DGKS re-projects some columns only: the column passes
    skip = 1;
    if (gw) {
      st->gram_skip = 1;
      st->gram_mixed = 1;
    }
  } else {
    const bool single = dgks && !any2;  // DGKS: one projection per column = CholQR1, B = R1
    single_f = single ? 1 : 0;
    if (single && gw) {
      st->gram_single = 1;
#pragma unroll
      for (int c = 0; c < K; ++c)
#pragma unroll
        for (int i = 0; i <= c; ++i) st->B[i + 16 * c] = R[i][c];
    }
    // T = R^{-1}
#pragma unroll
    for (int c = 0; c < K; ++c) {
      T[c][c] = 1.0 / R[c][c];
#pragma unroll
      for (int i = c - 1; i >= 0; --i) {
        double t = 0.0;
#pragma unroll
        for (int m = i + 1; m <= c; ++m) t += R[i][m] * T[m][c];
        T[i][c] = -t / R[i][i];
      }
    }
    if (Tl) {
#pragma unroll
      for (int c = 0; c < K; ++c)
#pragma unroll
        for (int i = 0; i <= c; ++i) Tl[i + 16 * c] = T[i][c];
    }
    if (gw) {
      double *Tout = w + (stage == 1 ? 0 : 256);
#pragma unroll
      for (int c = 0; c < K; ++c)
#pragma unroll
        for (int i = 0; i <= c; ++i) Tout[i + 16 * c] = T[i][c];
      if (stage == 1) {
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
          for (int i = 0; i <= c; ++i) w[512 + i + 16 * c] = R[i][c];
      } else {
        // B = R2 R1: the reference's B (projection coefficients above the diagonal, the norms on it)
        double R1[K][K];
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
          for (int i = 0; i <= c; ++i) R1[i][c] = w[512 + i + 16 * c];
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
          for (int i = 0; i <= c; ++i) {
            double t = 0.0;
#pragma unroll
            for (int m = i; m <= c; ++m) t += R[i][m] * R1[m][c];
            st->B[i + 16 * c] = t;
          }
      }
    }
  }
  if (fl) {
    fl[0] = skip;
    fl[1] = single_f;
  }
}

// One workgroup: the fixed-order sum of the partial rows, then thread 0 takes the step.
template <int K>
__global__ __launch_bounds__(256) void k_fbg_chol(const double *__restrict__ partial, int nblocks, int stage,
                                                  IcgsState *st, double *__restrict__ w, double gate,
                                                  double *__restrict__ sums) {
  constexpr int NV = K * (K + 1) / 2;
  double v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = 0.0;
  // the same order as one load round per block row (v += row b for b = t, t + 256, ...), with
  // up to four rows' loads in flight before their sums (1 round at <= 1024 rows instead of 4)
  for (int b0 = threadIdx.x; b0 < nblocks; b0 += 4 * 256) {
    double x[4][NV];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int b = b0 + u * 256 < nblocks ? b0 + u * 256 : b0;
#pragma unroll
      for (int i = 0; i < NV; ++i) x[u][i] = partial[(long long)i * nblocks + b];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b0 + u * 256 < nblocks) {
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] += x[u][i];
      }
  }
  __shared__ double red[4][NV];
  __shared__ double G[NV];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    double x = v[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
    if (l == 0) red[wv][i] = x;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    const int i = threadIdx.x;
    G[i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
    if (sums) sums[i] = G[i];
  }
  __syncthreads();
  if (stage == 0 || threadIdx.x != 0) return;
  if (stage == 2 && (st->gram_skip || st->gram_single)) return;
  double g[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) g[i] = G[i];
  fbg_step<K>(g, stage, st, w, gate, true, nullptr, nullptr);
}

// The fixed-order sum of value-major Gram partials (partial[i * nblocks + b]): one wave per
// value (16 waves), each lane 16 rows' loads in flight, then the wave's tree -- a few us where
// the one-workgroup k_fbg_chol sum took ~13 us before its serial step.
constexpr int GS_NT = 1024;
template <int NV>
__global__ __launch_bounds__(GS_NT) void k_gram_sum(const double *__restrict__ partial, int nblocks,
                                                    double *__restrict__ sums) {
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = wv; i < NV; i += GS_NT / 64) {
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int b0 = l; b0 < nblocks; b0 += 16 * 64) {
      double x[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int b = b0 + 64 * u;
        x[u] = b < nblocks ? partial[(long long)i * nblocks + b] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) a[u & 3] += x[u];
    }
    double x = (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
    if (l == 0) sums[i] = x;
  }
}

// Workgroups of a Gram-form pass: as many as are resident at once (one round, so the
// grid-stride sweeps end together), at most 1024 partial rows, at least 512 row pairs each.
template <class F>
static int fbg_resident(F kern, size_t lds) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, FBG_NT, lds) != hipSuccess || per_cu < 1)
    per_cu = 2;
  const long long b = (long long)per_cu * cu_count();
  return b > 1024 ? 1024 : (int)b;
}
static int fbg_nb(int resident, int nrows) {
  const long long cap = (((long long)nrows + 1) / 2 + 511) / 512;
  const long long b = resident < cap ? resident : cap;
  return b < 1 ? 1 : (int)b;
}

#define FBG_CASES(M) M(2) M(3) M(4) M(5) M(6) M(7) M(8)
#define FBM_CASES(M) M(9) M(10) M(11) M(12) M(13) M(14) M(15) M(16)

int launch_gemm_nn_gram(hipStream_t s, MvDesc A, int L, const double *M, int ldm, MvDesc X, int nrows,
                        double *partial, const NngPro &pro) {
  const int k = X.ncols;
  if (k < 2 || k > 8 || L < 0 || L > 1024) throw Error(MIGMRES_EINVAL, "gemm_nn_gram: 2 <= k <= 8 and L <= 1024");
  const size_t lds = sizeof(double) * (size_t)(L > 0 ? L : 1) * k;
  static const int contig = [] {  // MIGMRES_NNG_CONTIG=1: contiguous row range per workgroup
    const char *e = std::getenv("MIGMRES_NNG_CONTIG");
    return e ? std::atoi(e) : 0;
  }();
  NngPro pr = pro;
  pr.contig = contig;
  static int occ[9][1025];
  int nb = 1;
  switch (k) {
#define NNG_CASE(K)                                                              \
  case K:                                                                        \
    if (!occ[K][L]) occ[K][L] = fbg_resident(k_gemm_nn_gram<K>, lds);           \
    nb = fbg_nb(occ[K][L], nrows);                                               \
    k_gemm_nn_gram<K><<<nb, FBG_NT, lds, s>>>(A, L, M, ldm, X, nrows, partial, pr); \
    break;
    FBG_CASES(NNG_CASE)
#undef NNG_CASE
  }
  LAUNCH_CHECK_();
  return nb;
}

int launch_fbg_gram(hipStream_t s, MvDesc X, int k, int nrows, double *partial, int rev) {
  static int occ[17];
  int nb = 1;
  switch (k) {
#define FG_CASE(K)                                                 \
  case K:                                                          \
    if (!occ[K]) occ[K] = fbg_resident(k_fbg_gram<K>, 0);          \
    nb = fbg_nb(occ[K], nrows);                                    \
    k_fbg_gram<K><<<nb, FBG_NT, 0, s>>>(X, nrows, partial, rev);   \
    break;
    FBG_CASES(FG_CASE)
#undef FG_CASE
#define FGM_CASE(K)                                                                      \
  case K:                                                                                \
    if (!occ[K]) occ[K] = fbg_resident(k_fbg_gram_m<K, false>, 0);                       \
    nb = fbg_nb(occ[K], nrows);                                                          \
    k_fbg_gram_m<K, false><<<nb, FBG_NT, 0, s>>>(X, nrows, nullptr, nullptr, partial, rev); \
    break;
    FBM_CASES(FGM_CASE)
#undef FGM_CASE
    default:
      throw Error(MIGMRES_EINVAL, "fbg_gram: 2 <= k <= 16");
  }
  LAUNCH_CHECK_();
  return nb;
}

int launch_fbg_a(hipStream_t s, MvDesc X, int k, int nrows, const IcgsState *st, const double *w, double *partial,
                 int rev) {
  static int occ[17];
  int nb = 1;
  switch (k) {
#define FA_CASE(K)                                                       \
  case K:                                                                \
    if (!occ[K]) occ[K] = fbg_resident(k_fbg_a<K>, 0);                   \
    nb = fbg_nb(occ[K], nrows);                                          \
    k_fbg_a<K><<<nb, FBG_NT, 0, s>>>(X, nrows, st, w, partial, rev);     \
    break;
    FBG_CASES(FA_CASE)
#undef FA_CASE
#define FAM_CASE(K)                                                                 \
  case K:                                                                           \
    if (!occ[K]) occ[K] = fbg_resident(k_fbg_gram_m<K, true>, 0);                   \
    nb = fbg_nb(occ[K], nrows);                                                     \
    k_fbg_gram_m<K, true><<<nb, FBG_NT, 0, s>>>(X, nrows, st, w, partial, rev);     \
    break;
    FBM_CASES(FAM_CASE)
#undef FAM_CASE
    default:
      throw Error(MIGMRES_EINVAL, "fbg_a: 2 <= k <= 16");
  }
  LAUNCH_CHECK_();
  return nb;
}

void launch_fbg_b(hipStream_t s, MvDesc X, int k, int nrows, const IcgsState *st, const double *w, int rev) {
  static int occ[17];
  switch (k) {
#define FB2_CASE(K)                                                               \
  case K:                                                                         \
    if (!occ[K]) occ[K] = fbg_resident(k_fbg_b<K>, 0);                            \
    k_fbg_b<K><<<fbg_nb(occ[K], nrows), FBG_NT, 0, s>>>(X, nrows, st, w, rev);    \
    break;
    FBG_CASES(FB2_CASE)
#undef FB2_CASE
#define FBM2_CASE(K)                                                                  \
  case K:                                                                             \
    if (!occ[K]) occ[K] = fbg_resident(k_fbg_b_m<K>, 0);                              \
    k_fbg_b_m<K><<<fbg_nb(occ[K], nrows), FBG_NT, 0, s>>>(X, nrows, st, w, rev);      \
    break;
    FBM_CASES(FBM2_CASE)
#undef FBM2_CASE
    default:
      throw Error(MIGMRES_EINVAL, "fbg_b: 2 <= k <= 16");
  }
  LAUNCH_CHECK_();
}

void launch_fbg_chol(hipStream_t s, const double *partial, int nblocks, int k, int stage, IcgsState *st, double *w,
                     double gate, double *sums) {
  switch (k) {
#define FC_CASE(K)                                                                   \
  case K:                                                                            \
    k_fbg_chol<K><<<1, 256, 0, s>>>(partial, nblocks, stage, st, w, gate, sums);     \
    break;
    FBG_CASES(FC_CASE)
#undef FC_CASE
    default:
      throw Error(MIGMRES_EINVAL, "fbg_chol: 2 <= k <= 8");
  }
  LAUNCH_CHECK_();
}

void launch_gram_sum(hipStream_t s, const double *partial, int nblocks, int k, double *sums) {
  switch (k) {
#define GSUM_CASE(K)                                                                          \
  case K:                                                                                     \
    k_gram_sum<K *(K + 1) / 2><<<1, GS_NT, 0, s>>>(partial, nblocks, sums);                   \
    break;
    FBG_CASES(GSUM_CASE)
#undef GSUM_CASE
    default:
      throw Error(MIGMRES_EINVAL, "gram_sum: 2 <= k <= 8");
  }
  LAUNCH_CHECK_();
}

int launch_fbg_a_p(hipStream_t s, MvDesc X, int k, int nrows, IcgsState *st, double *w, const double *gsum,
                   double gate, double *partial, int rev) {
  static int occ[9];
  int nb = 1;
  switch (k) {
#define FAP_CASE(K)                                                                    \
  case K:                                                                              \
    if (!occ[K]) occ[K] = fbg_resident(k_fbg_a_p<K>, 0);                               \
    nb = fbg_nb(occ[K], nrows);                                                        \
    k_fbg_a_p<K><<<nb, FBG_NT, 0, s>>>(X, nrows, st, w, gsum, gate, partial, rev);     \
    break;
    FBG_CASES(FAP_CASE)
#undef FAP_CASE
    default:
      throw Error(MIGMRES_EINVAL, "fbg_a_p: 2 <= k <= 8");
  }
  LAUNCH_CHECK_();
  return nb;
}

void launch_fbg_b_p(hipStream_t s, MvDesc X, int k, int nrows, IcgsState *st, double *w, const double *gsum,
                    double gate, int rev) {
  static int occ[9];
  switch (k) {
#define FBP_CASE(K)                                                                                  \
  case K:                                                                                            \
    if (!occ[K]) occ[K] = fbg_resident(k_fbg_b_p<K>, 0);                                             \
    k_fbg_b_p<K><<<fbg_nb(occ[K], nrows), FBG_NT, 0, s>>>(X, nrows, st, w, gsum, gate, rev);         \
    break;
    FBG_CASES(FBP_CASE)
#undef FBP_CASE
    default:
      throw Error(MIGMRES_EINVAL, "fbg_b_p: 2 <= k <= 8");
  }
  LAUNCH_CHECK_();
}

void launch_fbg_chol_l(hipStream_t s, const double *gsum, int k, int stage, IcgsState *st, double *w, double gate) {
  if (k < 2 || k > 16) throw Error(MIGMRES_EINVAL, "fbg_chol_l: 2 <= k <= 16");
  k_fbg_chol_l<<<1, 256, 0, s>>>(gsum, k, stage, st, w, gate);
  LAUNCH_CHECK_();
}


// -------------------------------------------------------------------------------------
// Batched k = 1 ICGS for pseudo-block GMRES (solver.cpp, PseudoEngine::batched_ortho): the n
// right-hand sides' bases interleaved as QB (column q n + i = basis vector q of right-hand side
// i: a plain contiguous range of the iteration-major basis while every slot is active) and
// their new vectors as X (n columns).  The block kernels form every cross product QB^T X;
// right-hand side j keeps its own entries (rows q n + j of column j), the rest is masked to
// zero, so each column is projected against its own basis only.
// -------------------------------------------------------------------------------------
__global__ void k_blockdiag(const double *__restrict__ C1, const double *__restrict__ C2, int LB, int n, int L,
                            double *__restrict__ M) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= LB * n) return;
  const int r = e % LB, j = e / LB;
  const bool mine = r % n == j;  // QB's column r = q n + i belongs to right-hand side i
  M[e] = mine ? (C2 ? C1[e] + C2[e] : C1[e]) : 0.0;
}
void launch_blockdiag(hipStream_t s, const double *C1, const double *C2, int LB, int n, int L, double *M) {
  k_blockdiag<<<(LB * n + 255) / 256, 256, 0, s>>>(C1, C2, LB, n, L, M);
  LAUNCH_CHECK_();
}

// B[j] = sqrt(|dot_j|) (MvNorm) and x_j *= 1 / B[j] when B[j] > 0 (MvScale), as the k = 1
// branch of projectAndNormalize does it
__global__ __launch_bounds__(256) void k_norm_scale(MvDesc X, int nrows, const double *__restrict__ dots,
                                                    double *__restrict__ B) {
  const int j = blockIdx.y;
  const double b = sqrt(fabs(dots[j]));
  if (blockIdx.x == 0 && threadIdx.x == 0) B[j] = b;
  if (!(fabs(b) > 0.0)) return;
  const double inv = 1.0 / b;
  double *x = colp_(X, j);
  for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < nrows; r += (long long)gridDim.x * 256)
    x[r] = inv * x[r];
}
void launch_norm_scale(hipStream_t s, MvDesc X, int nrows, const double *dots, double *B) {
  const int gx = std::max(1, std::min(1024, (nrows + 255) / 256));
  k_norm_scale<<<dim3(gx, X.ncols), 256, 0, s>>>(X, nrows, dots, B);
  LAUNCH_CHECK_();
}

}  // namespace migmres
