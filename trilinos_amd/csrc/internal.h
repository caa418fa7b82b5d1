// Internal declarations shared by the migmres host runtime and the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/migmres.h"

namespace migmres {

// Error carried across the C ABI as (code, message).
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

// Thread-local message behind migmres_last_error().
void set_last_error(const std::string &msg);

// Run f, translating exceptions into the C ABI's (code, message) convention.
template <class F>
int guard(F &&f) {
  try {
    f();
    return MIGMRES_OK;
  } catch (const Error &e) {
    set_last_error(e.what());
    return e.code;
  } catch (const std::bad_alloc &) {
    set_last_error("out of host memory");
    return MIGMRES_ENOMEM;
  } catch (const std::exception &e) {
    set_last_error(e.what());
    return MIGMRES_EINVAL;
  }
}

#define MIG_HIP(call)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (call);                                                                \
    if (e_ != hipSuccess)                                                                  \
      throw ::migmres::Error(MIGMRES_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define MIG_CHECK(cond, msg)                                                               \
  do {                                                                                     \
    if (!(cond)) throw ::migmres::Error(MIGMRES_EINVAL, msg);                              \
  } while (0)

// Column-block descriptor handed to kernels by value.  Column c of the block starts at
// base + (cols ? cols[c] : c) * ld; rows are contiguous (column-major, Epetra layout).
struct MvDesc {
  double *base;
  long long ld;
  const int *cols;  // device column table for non-contiguous views, else nullptr
  int ncols;
};

// ---------------------------------------------------------------------------------
// Kernel launchers (kernels.hip).  All are asynchronous on `s`.
// ---------------------------------------------------------------------------------

// Y[:,c] = alpha * (A X)[:,c] + beta * Y[:,c] for the local CSR rows.  Column ids
// >= n_local index the ghost block (column-major, leading dim ldg).  Row sums are
// accumulated in stored order without contraction (Epetra GeneralMM order).
// Column scale of the fused right Jacobi preconditioner: the operand of every entry is
// (omega d^-1)_col * x_col, formed exactly as k_jacobi forms (omega D^-1) X.  own: n_local
// (+2 zero) entries; ghost: the owners' values of the ghost columns (ldg + 2 entries, zero
// padded), imported once.  Both null: no scaling.
struct ColScale {
  const double *own = nullptr;
  const double *ghost = nullptr;
};
// Row-pair SpMM (plan from make_pair_plan); vals padded by 8 entries, ghost ld even.
// sel/nsel: optional subset of pairs (rows for launch_spmm) to compute -- the interior and
// boundary halves of the halo overlap.
void launch_spmm_pair(hipStream_t s, int n_local, int max_keys, int rmax, const double *sv, const int *sk,
                      const unsigned short *sm, MvDesc X, const double *ghost, long long ldg, MvDesc Y,
                      double alpha, double beta, const int *sel = nullptr, int nsel = 0, ColScale cs = {});
// General rows: thread per row over the SELL-64 copy (make_sell64); sel lists rows.
// xr (optional, n_local x 8 doubles): scratch for a row-interleaved copy of X's owned rows,
// so each entry's k operands are one contiguous segment instead of k column gathers;
// xr_ready: an earlier launch of this apply already filled it (k <= 8).  Returns whether xr
// holds X's columns after this call (pass it as xr_ready to the next launch of the apply).
bool launch_spmm_sell(hipStream_t s, int n_local, const long long *off, const int *len, const int *scol,
                      const double *sval, MvDesc X, const double *ghost, long long ldg, MvDesc Y, double alpha,
                      double beta, const int *sel = nullptr, int nsel = 0, double *xr = nullptr,
                      bool xr_ready = false, ColScale cs = {});
// 3 x 3 block rows (make_bsr3): block rows with len 0 are skipped (left to the row kernel);
// xr as for launch_spmm_sell (n_local x 8 doubles, filled here for k >= 2).
void launch_spmm_bsr3(hipStream_t s, int nbr, int n_local, const long long *off, const int *len, const int *bcol,
                      const double *bval, MvDesc X, MvDesc Y, double alpha, double beta, double *xr,
                      ColScale cs = {});
void launch_spmm(hipStream_t s, int row_begin, int row_end, const int *rowptr, const int *cols,
                 const double *vals, MvDesc X, int n_local, const double *ghost, long long ldg,
                 MvDesc Y, double alpha, double beta, const int *sel = nullptr, int nsel = 0, ColScale cs = {});
// Row-pair templates (make_pair_templates): every pair whose template id is not kTplNone;
// the others are left to one of the kernels above.
// colscale (optional): Y = alpha A diag(colscale) X + beta Y with diag(colscale) X formed per
// operand exactly as k_jacobi forms (omega D^-1) X (the right Jacobi preconditioner fused).
void launch_spmm_tpl(hipStream_t s, int n_local, const unsigned char *tid, const int2 *rec, int ntpl, int maxk,
                     const double *vals, int nvals, MvDesc X, MvDesc Y, double alpha, double beta,
                     const double *colscale = nullptr, int xcd_slabs = 0, int kcmax = 8);
// The lane-shared form for stencil-group templates (make_stencil_groups; G = 3 or 9 groups,
// centers[G] pair offsets, grp ntpl * G packed slot words): same pairs, same bits.  Returns
// false (nothing launched) for a G it is not instantiated for.
bool launch_spmm_tpl3(hipStream_t s, int n_local, const unsigned char *tid, const unsigned long long *grp, int ntpl,
                      int G, const int *centers, const double *vals, int nvals, MvDesc X, MvDesc Y, double alpha,
                      double beta, const double *colscale = nullptr, int xcd_slabs = 0, int kcmax = 8);
// The 2.5-D march over the same stencil-group templates (make_march_geometry, plan.cpp): the
// local pairs read as planes of nyl lines of nxp pairs, group g's centre = ga[g] planes +
// gb[g] lines.  Workgroups own 64-pair x 4-line tiles and march a slab of planes, staging each
// plane tile (with a one-pair / one-line halo) in LDS once, so every X pair is loaded from
// memory about once instead of once per key.  Pairs whose keys would cross a line or plane
// edge of this geometry must not be templated (march_check counts them; the runtime uses the
// march only when there are none).  Same products and stored-order sums: same bits.
struct MarchGeom {
  int nxp = 0, nyl = 0, plane = 0, nz = 0;  // pairs per line, lines per plane, pairs per plane, planes
  int ga[9] = {}, gb[9] = {};
};
bool launch_spmm_march(hipStream_t s, int n_local, const unsigned char *tid, const unsigned long long *grp, int ntpl,
                       int G, const MarchGeom &geom, const double *vals, int nvals, MvDesc X, MvDesc Y, double alpha,
                       double beta, const double *colscale = nullptr, int kcmax = 2, int sz = 0, int pd = 1);
// The march for a UNIFORM 27-point stencil (G = 9 groups over every (plane, line) offset in
// {-1, 0, 1}^2): one coefficient table U (slot i of group g) for every templated pair, the
// slots a template leaves unused reading only neighbours outside the grid (march27_check).
// The two diagonal slots of the 27-point pattern: the centre group (g = 4), row 0's c.lo and
// row 1's c.hi.
constexpr unsigned long long kMarch27Diag = (1ULL << 25) | (1ULL << 28);
struct March27Coef {
  double w[9][6];
  // two_valued (27-point only): every w[g][i] is v2[(sel >> (6 g + i)) & 1] with sel =
  // kMarch27Diag (Brick3D: diagonal and neighbour value), so the kernel keeps 2 values
  // instead of 54 in scalar registers
  int two_valued = 0;
  double v2[2] = {0.0, 0.0};
  unsigned long long sel = 0;
  unsigned long long used = 0;  // slots the full template uses (the others are skipped by every pair)
};
// The march for the 7-point pattern (G = 5: groups (z - 1), (y - 1), x line, (y + 1), (z + 1)
// with neighbour halves only on the x line): coefficients in registers, only plane z staged,
// the (z +- 1) centres from the lane's own loads; pd planes of loads in flight (1..3), nl lines
// per thread (1, 2: tiles of 4 nl lines).
// uni (optional): the stencil is uniform in the sense of march27_check over the five groups --
// one coefficient table for every pair, absent entries reading out-of-grid zeros -- and its
// full template uses exactly kMarch7Used, so the kernel keeps no per-lane coefficients or masks.
constexpr unsigned long long kMarch7Used =
    (1ULL << 1) | (1ULL << 4) | (1ULL << 7) | (1ULL << 10) | (0x3FULL << 12) | (1ULL << 19) | (1ULL << 22) |
    (1ULL << 25) | (1ULL << 28);
bool launch_spmm_march7(hipStream_t s, int n_local, const unsigned char *tid, const unsigned long long *grp, int ntpl,
                        const MarchGeom &geom, const double *vals, int nvals, MvDesc X, MvDesc Y, double alpha,
                        double beta, const double *colscale = nullptr, int sz = 0, int pd = 2, int nl = 1,
                        const struct March27Coef *uni = nullptr, bool all_templated = false);
bool launch_spmm_march27(hipStream_t s, int n_local, const unsigned char *tid, const MarchGeom &geom,
                         const March27Coef &U, MvDesc X, MvDesc Y, double alpha, double beta,
                         const double *colscale = nullptr, int sz = 0, int pd = 2, bool all_templated = false);
// Templated pairs with an unused slot whose neighbour lies inside the grid (umask[t]: used slots
// of template t, bit 6 g + i); the uniform form needs none.
int march27_check(hipStream_t s, int npairs, const unsigned char *tid, const unsigned long long *umask, int ntpl,
                  const MarchGeom &geom, int G = 9, unsigned long long skip = 0);
// Number of templated pairs that the march geometry cannot serve (a used x-neighbour half
// across a line end, a group line outside the plane).  tbounds: per template {needs x-1 half,
// needs x+1 half, lowest group line offset, highest}.
int march_check(hipStream_t s, int npairs, const unsigned char *tid, const int4 *tbounds, int ntpl, int nxp, int nyl);
// out[r] = omega * a[r] (r < n)
void launch_scaled_copy(hipStream_t s, const double *a, double omega, double *out, int n);

// Partial products for C = A^T B over `nrows` rows: writes nblocks x (L*kb) partials.
// workgroups (= rows of partials) of a launch over L columns (L = 0: the single-group count)
int gemm_tn_blocks(int nrows, int L = 0);
void launch_gemm_tn_partial(hipStream_t s, MvDesc A, int L, MvDesc B, int kb, int nrows,
                            double *partial, int nblocks);
// out[o] = alpha * sum_b partial[b*nout + o] (fixed order: deterministic).
void launch_reduce_partials(hipStream_t s, const double *partial, int nblocks, int nout,
                            double alpha, double *out);

// The same with the (rows x cols) result written column-major with leading dimension ldo.
void launch_reduce_partials_ld(hipStream_t s, const double *partial, int nblocks, int rows, int cols,
                               int ldo, double alpha, double *out);

// X = beta*X + alpha * A * M, M (L x kx) device column-major with leading dim ldm.
void launch_gemm_nn(hipStream_t s, MvDesc A, int L, const double *M, int ldm, MvDesc X,
                    int nrows, double alpha, double beta);

// Per-column reductions: op 0 = sum a*b, 1 = sum |a|, 2 = max |a|.  Partials nblocks x k.
int coldot_blocks(int nrows);
void launch_coldot_partial(hipStream_t s, MvDesc A, MvDesc B, int nrows, int op, double *partial,
                           int nblocks);
void launch_reduce_max(hipStream_t s, const double *partial, int nblocks, int nout, double *out);

// Elementwise: Y = alpha*A + beta*B ; Y *= alpha (or alphas[c]) ; Y = v ; Y = A.
void launch_axpby(hipStream_t s, double alpha, MvDesc A, double beta, MvDesc B, MvDesc Y, int nrows);
void launch_scale(hipStream_t s, MvDesc Y, int nrows, double alpha, const double *alphas);
void launch_fill(hipStream_t s, MvDesc Y, int nrows, double v);
void launch_copy(hipStream_t s, MvDesc A, MvDesc Y, int nrows);
// Epetra_MultiVector::Random semantics over global rows [first, first+nrows).
void launch_random(hipStream_t s, MvDesc Y, int nrows, long long first, long long n_global,
                   unsigned int seed);
// Point Jacobi: dinv = 1/diag(local CSR); Y = (omega*dinv)*X or Y = 1*Y + (omega*dinv)*X.
void launch_diag_inv(hipStream_t s, const int *rowptr, const int *cols, const double *vals, int n,
                     double *dinv);
void launch_jacobi(hipStream_t s, MvDesc X, MvDesc Y, const double *dinv, double omega, int nrows,
                   bool accumulate);
// Ifpack2::Relaxation's inverse diagonal with the l1 and fix-tiny options (kernels.hip).
void launch_relax_diag(hipStream_t s, const int *rowptr, const int *cols, const double *vals, int n, int n_present,
                       bool l1, double eta, bool fix_tiny, double min_val, double *dinv);
// Ifpack2::Chebyshev: dinv = reciprocal_threshold(diag, min_val); the ChebyshevKernel step
// W = [beta W +] (alpha dinv) R, X = X + W (xmode 1) / X = W (2) / untouched (0); Y = a A + b B
// without contraction.
void launch_diag_recip_threshold(hipStream_t s, const int *rowptr, const int *cols, const double *vals, int n,
                                 double min_val, double *dinv);
// (B.base != null: R holds A X and the kernel forms b - (A X) itself)
void launch_cheb_update(hipStream_t s, MvDesc B, MvDesc R, MvDesc W, MvDesc X, const double *dinv, double alpha,
                        double beta, bool use_beta, int xmode, int nrows);
void launch_lincomb(hipStream_t s, double a, MvDesc A, double b, MvDesc B, MvDesc Y, int nrows);
void launch_abs(hipStream_t s, MvDesc Y, int nrows);  // Y = |Y| (negative entries negated)
// Import exchange layout [neighbour][column][count] (grp[i] = (offset, count) of entry i's
// neighbour group): send[off*k + c*cnt + i-off] = X[lids[i], c]; ghost[c*ldg + i] = recv[...].
void launch_pack(hipStream_t s, MvDesc X, const int *lids, const int2 *grp, int count, double *send, int k);
// transposed apply: T[lids[i]] += recv[c * count + i] (one neighbour's contributions); Y = alpha T + beta Y
void launch_export_add(hipStream_t s, MvDesc T, const int *lids, int count, int k, const double *recv);
void launch_combine(hipStream_t s, MvDesc T, MvDesc Y, int nrows, double alpha, double beta);
void launch_unpack(hipStream_t s, const double *recv, const int2 *grp, int count, int k, double *ghost,
                   long long ldg);

// MIGMRES_SETUP_TRACE=1: wall-clock checkpoints of operator setup on stderr (tuning aid).
void setup_mark(const char *what);

}  // namespace migmres
