// Point-Jacobi preconditioner on the device: Ifpack2::Relaxation with "relaxation: type" =
// "Jacobi" (ifpack2/src/Ifpack2_Relaxation_def.hpp; compute() :990-1270 keeps the
// reciprocal of the diagonal, ApplyInverseJacobi :1390-1454 applies it), the
// right/left preconditioner of config 5.
#include "runtime.h"

using namespace migmres;

migmres_prec::~migmres_prec() {
  if (d_dinv) hipFree(d_dinv);
  if (d_sdinv) hipFree(d_sdinv);
  if (d_gsdinv) hipFree(d_gsdinv);
  delete work;
  delete xcopy;
}

namespace migmres {

// Y = M X.  Zero starting solution: the first sweep is Y = (omega d^-1) X; every further
// sweep forms R = X - A Y (SpMM with alpha = -1, beta = 1 on a copy of X: y - sum, the
// Tpetra::Details::residual expression) and Y = 1*Y + (omega d^-1) R.
// Do any columns of X and Y share memory?  (Ifpack2 compares the data pointers,
// Ifpack2_Relaxation_def.hpp:543-551; a column-range overlap test also catches views that
// start at different columns of one block.)
static bool mv_overlap(const migmres_mv &X, const migmres_mv &Y) {
  if (X.ncols == 0 || Y.ncols == 0 || X.n_local == 0) return false;
  for (int i = 0; i < X.ncols; ++i) {
    const double *a0 = X.base + X.col_offset(i), *a1 = a0 + X.n_local;
    for (int j = 0; j < Y.ncols; ++j) {
      const double *b0 = Y.base + Y.col_offset(j), *b1 = b0 + Y.n_local;
      if (a0 < b1 && b0 < a1) return true;
    }
  }
  return false;
}

void prec_apply(migmres_prec &M, const migmres_mv &X_in, migmres_mv &Y) {
  MIG_CHECK(X_in.ncols == Y.ncols, "Jacobi apply: X and Y column counts differ");
  MIG_CHECK(X_in.n_local == M.A->n_local && Y.n_local == M.A->n_local, "Jacobi apply: row map mismatch");
  migmres_ctx *c = M.ctx;
  const int n = M.A->n_local;
  // X aliasing Y (apply(x, x)): sweep from a deep copy of X, as the reference does
  const migmres_mv *Xp = &X_in;
  if (mv_overlap(X_in, Y)) {
    if (!M.xcopy || M.xcopy->ncols != X_in.ncols) {
      delete M.xcopy;
      M.xcopy = mv_create(c, X_in.n_global, X_in.n_local, X_in.ncols);
    }
    mv_assign(X_in, *M.xcopy);
    Xp = M.xcopy;
  }
  const migmres_mv &X = *Xp;
  {
    ProfScope ps(c, K_AXPBY, 8.0 * n * (2.0 * X.ncols + 1.0));
    launch_jacobi(c->stream, X.desc(), Y.desc(), M.d_dinv, M.damping, n, false);
  }
  if (M.sweeps > 1) {
    if (!M.work || M.work->ncols != X.ncols) {
      delete M.work;
      M.work = mv_create(c, X.n_global, X.n_local, X.ncols);
    }
    for (int j = 1; j < M.sweeps; ++j) {
      mv_assign(X, *M.work);
      crs_apply(*M.A, Y, *M.work, -1.0, 1.0);
      ProfScope ps(c, K_AXPBY, 8.0 * n * (3.0 * X.ncols + 1.0));
      launch_jacobi(c->stream, M.work->desc(), Y.desc(), M.d_dinv, M.damping, n, true);
    }
  }
  ++M.n_apply;
}

}  // namespace migmres

extern "C" int migmres_jacobi_create(migmres_crs *A, int sweeps, double damping, migmres_prec **out) {
  return guard([&] {
    MIG_CHECK(A && out, "jacobi_create: null argument");
    MIG_CHECK(sweeps >= 1, "\"relaxation: sweeps\" must be >= 1");
    auto *M = new migmres_prec();
    M->ctx = A->ctx;
    M->A = A;
    M->sweeps = sweeps;
    M->damping = damping;
    const int n = A->n_local;
    MIG_HIP(hipMalloc(&M->d_dinv, sizeof(double) * (n > 0 ? n : 1)));
    launch_diag_inv(A->ctx->stream, A->d_rowptr, A->d_cols, A->d_vals, n, M->d_dinv);
    // the fused form's column scale omega * dinv, with two zero entries past n for the row-pair
    // kernels' reads of a last half-filled pair
    MIG_HIP(hipMalloc(&M->d_sdinv, sizeof(double) * ((size_t)n + 2)));
    MIG_HIP(hipMemsetAsync(M->d_sdinv, 0, sizeof(double) * ((size_t)n + 2), A->ctx->stream));
    launch_scaled_copy(A->ctx->stream, M->d_dinv, damping, M->d_sdinv, n);
    MIG_HIP(hipStreamSynchronize(A->ctx->stream));
    if (sweeps == 1) prec_import_ghost_scale(*M);  // the fused form's ghost column scale
    *out = M;
  });
}

extern "C" int migmres_prec_destroy(migmres_prec *M) {
  return guard([&] { delete M; });
}

extern "C" int migmres_prec_apply(migmres_prec *M, const migmres_mv *X, migmres_mv *Y) {
  return guard([&] {
    MIG_CHECK(M && X && Y, "prec_apply: null argument");
    prec_apply(*M, *X, *Y);
  });
}

extern "C" int migmres_prec_diagonal(const migmres_prec *M, double *dinv_out) {
  return guard([&] {
    MIG_CHECK(M && dinv_out, "prec_diagonal: null argument");
    MIG_HIP(hipMemcpy(dinv_out, M->d_dinv, sizeof(double) * M->A->n_local, hipMemcpyDeviceToHost));
  });
}
