// Device-resident ICGS state and kernel launchers (icgs.hip).
#pragma once

#include "internal.h"

namespace migmres {

// Coefficients and decisions of one projectAndNormalize / normalize call, kept on the
// device between kernels and copied to the host once at the end.
struct IcgsState {
  double oldDot[16], newDot[16], diag[16], inv[16], P[16], P2[16], prod[16];
  double B[256];  // k x k normalisation coefficients, column-major, leading dimension 16
  double blk_old[16];
  double blk_tol, sing_tol, dep, neg;
  int failed;  // first findBasis column found dependent, -1 if none
  int dgks;    // 1: DGKSOrthoManager findBasis (second projection only under dep_tol)
  double dep_tol;
  int gram_skip;  // findBasis in Gram form handed the block back to the column passes
  // DGKS in Gram form: no column of the block took DGKS's second projection (its criterion on
  // the first pass's pivots): CholQR1, B = R1 (gram_single); some but not all did: the column
  // passes decide column by column (gram_mixed, with gram_skip)
  int gram_single, gram_mixed, gram_pad_;
};

// findBasis in Gram form (icgs.hip; ICGS with two passes, 2 <= k <= 16).  The partial-writing
// launchers return their number of workgroups (rows of partials, at most 1024): the packed
// upper triangle of the k x k Gram matrix, value-major (partial[i * nb + b]) for k <= 8 (read
// by launch_fbg_chol), block-major (partial[b * nv + i]) for k > 8 (launch_reduce_partials,
// then launch_fbg_chol_l).  launch_gemm_nn_gram: k <= 8 only.
// w: 768 doubles of device scratch (T1, T2, R1).
// NngPro (optional): the small steps between blkOrtho's passes folded into the closing update's
// prologue -- M = C1 + C2 formed as the coefficients are staged (k_add_coef's sum, same
// rounding), workgroup 0 storing it to `cout` for the host, resetting the state and recording
// oldDot = diag of the Gram block G (k_state_reset + k_blk_old): three launches fewer per block.
struct NngPro {
  const double *C1 = nullptr, *C2 = nullptr;  // null: M as given
  int ld1 = 0, ld2 = 0;
  double *cout = nullptr;
  int ldo = 0;
  IcgsState *st = nullptr;  // null: no state step
  const double *G = nullptr;
  int ldg = 0, dgks = 0;
  double blk_tol = 0.0, sing_tol = 0.0, dep_tol = 0.0;
  int contig = 0;  // (tuning) row order of the pass: 0 grid-stride, 1 contiguous range per workgroup
};
int launch_gemm_nn_gram(hipStream_t s, MvDesc A, int L, const double *M, int ldm, MvDesc X, int nrows,
                        double *partial, const NngPro &pro = NngPro());
int launch_fbg_gram(hipStream_t s, MvDesc X, int k, int nrows, double *partial, int rev);
int launch_fbg_a(hipStream_t s, MvDesc X, int k, int nrows, const IcgsState *st, const double *w, double *partial,
                 int rev);
void launch_fbg_b(hipStream_t s, MvDesc X, int k, int nrows, const IcgsState *st, const double *w, int rev);
// stage 0: sums of the partials only (-> sums); 1: dependency test, R1, gate, T1; 2: R2, T2, B
void launch_fbg_chol(hipStream_t s, const double *partial, int nblocks, int k, int stage, IcgsState *st, double *w,
                     double gate, double *sums);
// k <= 8 with the step in the passes' prologues: sums of value-major partials (k(k+1)/2
// values), then k_fbg_a_p (stage 1 from gsum; returns its partial rows) and k_fbg_b_p (stage 2)
void launch_gram_sum(hipStream_t s, const double *partial, int nblocks, int k, double *sums);
int launch_fbg_a_p(hipStream_t s, MvDesc X, int k, int nrows, IcgsState *st, double *w, const double *gsum,
                   double gate, double *partial, int rev);
void launch_fbg_b_p(hipStream_t s, MvDesc X, int k, int nrows, IcgsState *st, double *w, const double *gsum,
                    double gate, int rev);
// the same step for k > 8 from the summed Gram matrix (nv = k(k+1)/2 values)
void launch_fbg_chol_l(hipStream_t s, const double *gsum, int k, int stage, IcgsState *st, double *w, double gate);

// Pass prologue: the reduction + scalar step still pending from the previous pass, taken by
// every workgroup of the next pass from the previous pass's per-workgroup partials (one
// rank) or from the all-reduced vector (several ranks), instead of a separate launch.
// Every workgroup applies the step to its own LDS copy of `in`; workgroup 0 also stores the
// result to `out` (the state double-buffers: the other workgroups still read `in`).
// stage0 < 0: nothing pending (`in` is used as is, `out` unused).
struct FbPro {
  const double *partial;  // partial[b * nv + i], b < nblocks; nullptr: use red
  const double *red;
  int nblocks, nv;
  int stage0, stage1;  // scalar stages applied in order (stage1 < 0: only stage0)
  int j, k, complete;
  const IcgsState *in;
  IcgsState *out;
};

int icgs_blocks(int nrows);
void launch_reduce_small(hipStream_t s, const double *partial, int nblocks, int nv, double *out);
void launch_gemm_nn_dot(hipStream_t s, MvDesc A, int L, const double *M, int ldm, MvDesc X,
                        int nrows, double alpha, double beta, int dmode, MvDesc D, double *partial,
                        int nblocks);
// X1 = X - Q C1 and per-workgroup partials of Q^T X1 (L x k, column-major).  store_x1:
// X1 is written back over X; otherwise X is left as it was (X1 lives only in the kernel,
// and the closing update subtracts Q (C1 + C2) from the original X instead).
// sink: scratch of nblocks * 256 doubles that absorbs the stores of padding lanes.
bool nn_tn_supported(int L, int k);
int nn_tn_blocks(int nrows, int L, int k);
// k > 8: whether launch_nn_tn runs the column halves in workgroup pairs (partials: half 0
// [nb/2][L][8] then half 1 [nb/2][L][k-8]) rather than all k columns per workgroup ([nb][L][k]).
bool nn_tn_paired(int L, int k);
void launch_nn_tn(hipStream_t s, MvDesc Q, int L, const double *C1, int ldc, MvDesc X, int nrows,
                  double *partial, int nblocks, double *sink, bool store_x1 = true);
void launch_fb_a(hipStream_t s, MvDesc X, int j, const FbPro &pro, int nrows, double *partial, int nb);
void launch_fb_b(hipStream_t s, MvDesc X, int j, const IcgsState *st, double *S, int nrows, double *partial, int nb);
void launch_fb_c(hipStream_t s, MvDesc X, int j, const IcgsState *st, const double *S, int nrows, double *partial,
                 int nb);
// Two-pass-per-column findBasis (see icgs.hip): a01 head, b2 = normalise previous column +
// first update + second projection, ca = second update + next column's first projection.
// rev = 1 sweeps the rows from the top down: consecutive passes alternate direction so each
// pass starts on the rows the previous one touched last (still in the Infinity Cache).
void launch_fb_a01(hipStream_t s, MvDesc X, int nrows, double *partial, int nb);
void launch_fb_b2(hipStream_t s, MvDesc X, int j, const FbPro &pro, int nrows, double *partial, int nb,
                  int rev = 0);
void launch_fb_ca(hipStream_t s, MvDesc X, int j, int has_next, const FbPro &pro, int nrows, double *partial,
                  int nb, int rev = 0);
void launch_scale_col(hipStream_t s, MvDesc X, int j, const FbPro &pro, int nrows, int nb);
// the prologue alone (one workgroup): applies a pending step with nothing after it
void launch_fb_flush(hipStream_t s, const FbPro &pro);
// reduce_small followed by fb_scalar in one single-workgroup launch (single rank only)
void launch_reduce_scalar(hipStream_t s, const double *partial, int nblocks, int nv, double *red, IcgsState *st,
                          int stage, int j, int k, int complete);
void launch_fb_scalar(hipStream_t s, IcgsState *st, const double *red, int stage, int j, int k, int complete);
void launch_blk_old(hipStream_t s, IcgsState *st, const double *G, int ldg, int L, int k);
void launch_state_reset(hipStream_t s, IcgsState *st, double blk_tol, double sing_tol, int dgks = 0,
                        double dep_tol = 0.0);
void launch_add_coef(hipStream_t s, const double *C1, int ld1, const double *C2, int ld2, double *out, int ldo,
                     int L, int k);

// Pseudo-block GMRES, batched k = 1 ICGS: M = blockdiag(C1 [+ C2]) (LB = n L rows, n columns,
// column j keeps rows j L .. j L + L - 1); B[j] = sqrt|dots[j]| and column j of X scaled by 1/B[j].
void launch_blockdiag(hipStream_t s, const double *C1, const double *C2, int LB, int n, int L, double *M);
void launch_norm_scale(hipStream_t s, MvDesc X, int nrows, const double *dots, double *B);

}  // namespace migmres
