// Preconditioners on the device: point Jacobi, Ifpack2::Relaxation with "relaxation: type" =
// "Jacobi" (ifpack2/src/Ifpack2_Relaxation_def.hpp; compute() :990-1270 keeps the
// reciprocal of the diagonal, ApplyInverseJacobi :1390-1454 applies it), the
// right/left preconditioner of config 5; and the
// Chebyshev smoother, Ifpack2::Chebyshev.
#include <cmath>
#include <limits>
#include <memory>

#include "runtime.h"

using namespace migmres;

migmres_prec::~migmres_prec() {
  if (d_dinv) hipFree(d_dinv);
  if (d_sdinv) hipFree(d_sdinv);
  if (d_gsdinv) hipFree(d_gsdinv);
  delete work;
  delete xcopy;
  delete cheb_w;
  delete cheb_p;
}

namespace migmres {

// Y = M X.  Zero starting solution: the first sweep is Y = (omega d^-1) X; every further
// sweep forms R = X - A Y (SpMM with alpha = -1, beta = 1 on a copy of X: y - sum, the
// Tpetra::Details::residual expression) and Y = 1*Y + (omega d^-1) R.
// scratch multivector with X's shape, (re)made when the column count changes
static migmres_mv &scratch(migmres_mv *&w, const migmres_mv &X) {
  if (!w || w->ncols != X.ncols) {
    delete w;
    w = mv_create(X.ctx, X.n_global, X.n_local, X.ncols);
  }
  return *w;
}

// R = B - A X (the Tpetra::Details::residual expression b - sum, by the SpMM with alpha = -1,
// beta = 1 on a copy of B)
static void residual(migmres_prec &M, const migmres_mv &B, const migmres_mv &X, migmres_mv &R) {
  mv_assign(B, R);
  crs_apply(*M.A, X, R, -1.0, 1.0);
}

// Ifpack2::Chebyshev::apply: X = M B (Ifpack2_Details_Chebyshev_def.hpp:909-957).
static void chebyshev_apply(migmres_prec &M, const migmres_mv &B, migmres_mv &X) {
  migmres_ctx *c = M.ctx;
  const int n = M.A->n_local;
  const migmres_chebyshev_params &p = M.cheb;
  const int deg = p.degree;
  if (p.textbook_algorithm) {  // textbookApplyImpl (:1163-1208)
    const double lmax = M.cheb_lmax, lmin = lmax / M.cheb_ratio;
    const double d = (lmax + lmin) / 2.0, cc = (lmax - lmin) / 2.0;
    if (p.zero_starting_solution && deg > 0) mv_init(X, 0.0);
    migmres_mv &R = scratch(M.work, B), &P = scratch(M.cheb_p, B), &Z = scratch(M.cheb_w, B);
    double alpha = 0.0;
    for (int i = 0; i < deg; ++i) {
      residual(M, B, X, R);
      ProfScope ps(c, K_AXPBY, 8.0 * n * (6.0 * B.ncols + 1.0));
      launch_jacobi(c->stream, R.desc(), Z.desc(), M.d_dinv, 1.0, n, false);  // Z = D^-1 R
      if (i == 0) {
        mv_assign(Z, P);
        alpha = 2.0 / d;
      } else {
        const double beta = alpha * (cc / 2.0) * (cc / 2.0);
        alpha = 1.0 / (d - beta);
        launch_lincomb(c->stream, 1.0, Z.desc(), beta, P.desc(), P.desc(), n);  // P = Z + beta P
      }
      launch_lincomb(c->stream, alpha, P.desc(), 1.0, X.desc(), X.desc(), n);  // X = X + alpha P
    }
    return;
  }
  if (deg <= 0) return;  // ifpackApplyImpl (:1221-1339)
  if (M.cheb_lmin == 1.0 && M.cheb_lmax == M.cheb_lmin) {  // A = I: X = D^-1 B (:1250-1253)
    ProfScope ps(c, K_AXPBY, 8.0 * n * (2.0 * B.ncols + 1.0));
    launch_jacobi(c->stream, B.desc(), X.desc(), M.d_dinv, 1.0, n, false);
    return;
  }
  // Chebyshev::apply (Ifpack2_Details_Chebyshev_def.hpp:920-932)
  MIG_CHECK(std::isfinite(M.cheb_lmax), "Ifpack2::Chebyshev::apply: There is no estimate for the max eigenvalue.");
  MIG_CHECK(std::isfinite(M.cheb_lmin), "Ifpack2::Chebyshev::apply: There is no estimate for the min eigenvalue.");
  MIG_CHECK(std::isfinite(M.cheb_ratio),
            "Ifpack2::Chebyshev::apply: There is no estimate for the ratio of the max eigenvalue to the min eigenvalue.");
  const double alpha = M.cheb_lmax / M.cheb_ratio;
  const double beta = p.boost_factor * M.cheb_lmax;
  const double delta = 2.0 / (beta - alpha);
  const double theta = (beta + alpha) / 2.0;
  const double s1 = theta * delta;
  migmres_mv &W = scratch(M.cheb_w, B);
  const MvDesc none{nullptr, 0, nullptr, 0};
  if (p.zero_starting_solution) {  // W = (1/theta) D^-1 B, X = W
    ProfScope ps(c, K_AXPBY, 8.0 * n * (3.0 * B.ncols + 1.0));
    launch_cheb_update(c->stream, none, B.desc(), W.desc(), X.desc(), M.d_dinv, 1.0 / theta, 0.0, false, 2, n);
  } else {  // W = (1/theta) D^-1 (B - A X), X += W
    migmres_mv &R = scratch(M.work, B);
    crs_apply(*M.A, X, R, 1.0, 0.0);  // R = A X; the update forms b - (A X)
    ProfScope ps(c, K_AXPBY, 8.0 * n * (5.0 * B.ncols + 1.0));
    launch_cheb_update(c->stream, B.desc(), R.desc(), W.desc(), X.desc(), M.d_dinv, 1.0 / theta, 0.0, false, 1, n);
  }
  double rhok = 1.0 / s1;
  for (int k = 1; k < deg; ++k) {
    const double rhokp1 = 1.0 / (2.0 * s1 - rhok);
    const double dtemp1 = rhokp1 * rhok;
    const double dtemp2 = 2.0 * rhokp1 * delta;
    rhok = rhokp1;
    migmres_mv &R = scratch(M.work, B);
    crs_apply(*M.A, X, R, 1.0, 0.0);
    ProfScope ps(c, K_AXPBY, 8.0 * n * (7.0 * B.ncols + 1.0));
    launch_cheb_update(c->stream, B.desc(), R.desc(), W.desc(), X.desc(), M.d_dinv, dtemp2, dtemp1, true, 1, n);
  }
}

// powerMethodWithInitGuess (Ifpack2_Details_Chebyshev_def.hpp:1344-1406) on D^-1 A.
static double power_method(migmres_prec &M, migmres_mv &x, migmres_mv &y) {
  migmres_ctx *c = M.ctx;
  const int n = M.A->n_local;
  double nrm = 0.0, top = 0.0, bottom = 0.0, lambda = 0.0;
  mv_norm(x, &nrm, 2);
  MIG_CHECK(nrm != 0.0, "Ifpack2::Chebyshev::powerMethodWithInitGuess: the initial guess has zero norm");
  mv_scale(x, 1.0 / nrm);
  for (int it = 0; it < M.cheb.eigenvalue_max_iterations; ++it) {
    crs_apply(*M.A, x, y, 1.0, 0.0);
    launch_jacobi(c->stream, y.desc(), y.desc(), M.d_dinv, 1.0, n, false);  // y = D^-1 y
    mv_dot(y, x, &top);
    mv_dot(x, x, &bottom);
    lambda = top / bottom;
    mv_norm(y, &nrm, 2);
    if (nrm == 0.0) return 0.0;
    mv_assign(y, x);
    mv_scale(x, 1.0 / nrm);
  }
  return lambda;
}

// compute() (Ifpack2_Details_Chebyshev_def.hpp:739-896) after the inverse diagonal.
static void chebyshev_compute(migmres_prec &M) {
  const migmres_chebyshev_params &p = M.cheb;
  if (!p.assume_matrix_unchanged || (std::isnan(M.cheb_computed_lmax) && std::isnan(p.max_eigenvalue))) {
    std::unique_ptr<migmres_mv> x(mv_create(M.ctx, M.A->n_global, M.A->n_local, 1));
    std::unique_ptr<migmres_mv> y(mv_create(M.ctx, M.A->n_global, M.A->n_local, 1));
    unsigned seed = p.seed;
    mv_random(*x, &seed);
    double lmax = power_method(M, *x, *y);
    if (lmax < 0.0) {  // powerMethod (:1457-1471): once more from |random|, the next draw of the stream
      mv_random(*x, &seed);
      launch_abs(M.ctx->stream, x->desc(), M.A->n_local);  // PositivizeVector (:191-221)
      lmax = power_method(M, *x, *y);
    }
    MIG_CHECK(std::isfinite(lmax),
              "Ifpack2::Chebyshev::compute: Estimation of the max eigenvalue of D^{-1} A failed, by producing Inf "
              "or NaN.  This probably means that the matrix contains Inf or NaN values, or that it is badly scaled.");
    M.cheb_computed_lmax = lmax;
  }
  M.cheb_lmax = std::isnan(p.max_eigenvalue) ? M.cheb_computed_lmax : p.max_eigenvalue;
  M.cheb_lmin = M.cheb_lmax / p.ratio_eigenvalue;
  M.cheb_ratio = p.ratio_eigenvalue;
  if (!p.textbook_algorithm && std::fabs(M.cheb_lmax - 1.0) < 1.0e-6) {  // Ifpack's lambdaMax ~ 1 case
    M.cheb_lmin = 1.0;
    M.cheb_lmax = 1.0;
    M.cheb_ratio = 1.0;
  }
}

void prec_apply(migmres_prec &M, const migmres_mv &X_in, migmres_mv &Y) {
  MIG_CHECK(X_in.ncols == Y.ncols, "preconditioner apply: X and Y column counts differ");
  if (M.kind == 2) {  // a user operator as the preconditioner
    op_apply(*M.uop, X_in, Y);
    ++M.n_apply;
    return;
  }
  MIG_CHECK(X_in.n_local == M.A->n_local && Y.n_local == M.A->n_local, "preconditioner apply: row map mismatch");
  migmres_ctx *c = M.ctx;
  const int n = M.A->n_local;
  // X aliasing Y (apply(x, x)): work from a deep copy of X, as the reference does
  const migmres_mv *Xp = &X_in;
  if (mv_overlap(X_in, Y)) {
    mv_assign(X_in, scratch(M.xcopy, X_in));
    Xp = M.xcopy;
  }
  const migmres_mv &X = *Xp;
  if (M.kind == 1) {
    chebyshev_apply(M, X, Y);
    ++M.n_apply;
    return;
  }
  // ApplyInverseJacobi / ApplyInverseRichardson (Ifpack2_Relaxation_def.hpp:1323-1454)
  const bool jacobi = M.rtype == 0;
  if (M.zero_start) {  // first sweep from Y = 0: Y = (omega d^-1) X, or Y = omega X
    ProfScope ps(c, K_AXPBY, 8.0 * n * (2.0 * X.ncols + 1.0));
    if (jacobi) {
      launch_jacobi(c->stream, X.desc(), Y.desc(), M.d_dinv, M.damping, n, false);
    } else {
      mv_assign(X, Y);
      mv_scale(Y, M.damping);
    }
  }
  const int start = M.zero_start ? 1 : 0;
  if (M.sweeps > start) {
    migmres_mv &R = scratch(M.work, X);
    for (int j = start; j < M.sweeps; ++j) {
      residual(M, X, Y, R);  // R = X - A Y
      ProfScope ps(c, K_AXPBY, 8.0 * n * (3.0 * X.ncols + 1.0));
      if (jacobi)  // Y = 1*Y + (omega d^-1) R
        launch_jacobi(c->stream, R.desc(), Y.desc(), M.d_dinv, M.damping, n, true);
      else  // Y.update(omega, R, 1): omega R + 1 Y
        launch_lincomb(c->stream, M.damping, R.desc(), 1.0, Y.desc(), Y.desc(), n);
    }
  }
  ++M.n_apply;
}

}  // namespace migmres

extern "C" int migmres_relaxation_params_default(migmres_relaxation_params *p) {
  return guard([&] {
    MIG_CHECK(p, "relaxation_params_default: null argument");
    *p = migmres_relaxation_params{};
    p->type = 0;
    p->sweeps = 1;
    p->damping = 1.0;
    p->zero_starting_solution = 1;
    p->use_l1 = 0;
    p->l1_eta = 1.5;
    p->min_diagonal_value = 0.0;
    p->fix_tiny_diagonal_entries = 0;
    p->check_diagonal_entries = 0;
  });
}

extern "C" int migmres_relaxation_create(migmres_crs *A, const migmres_relaxation_params *p, migmres_prec **out) {
  return guard([&] {
    MIG_CHECK(A && p && out, "relaxation_create: null argument");
    MIG_CHECK(p->type == 0 || p->type == 1, "\"relaxation: type\": the device path implements Jacobi and Richardson");
    MIG_CHECK(p->sweeps >= 0, "\"relaxation: sweeps\" must be nonnegative");
    std::unique_ptr<migmres_prec> M(new migmres_prec());
    M->ctx = A->ctx;
    M->A = A;
    M->rtype = p->type;
    M->sweeps = p->sweeps;
    M->damping = p->damping;
    M->zero_start = p->zero_starting_solution != 0;
    const int n = A->n_local;
    const int n_present = A->n_cols - (int)A->plan.remote_lids.size();
    MIG_HIP(hipMalloc(&M->d_dinv, sizeof(double) * (n > 0 ? n : 1)));
    // IsParallel_: the l1 boost only on more than one process (Ifpack2_Relaxation_def.hpp:1052)
    launch_relax_diag(A->ctx->stream, A->d_rowptr, A->d_cols, A->d_vals, n, n_present,
                      p->use_l1 && A->ctx->nranks > 1, p->l1_eta, p->fix_tiny_diagonal_entries != 0,
                      p->min_diagonal_value, M->d_dinv);
    // the fused form's column scale omega * dinv, with two zero entries past n for the row-pair
    // kernels' reads of a last half-filled pair
    MIG_HIP(hipMalloc(&M->d_sdinv, sizeof(double) * ((size_t)n + 2)));
    MIG_HIP(hipMemsetAsync(M->d_sdinv, 0, sizeof(double) * ((size_t)n + 2), A->ctx->stream));
    launch_scaled_copy(A->ctx->stream, M->d_dinv, p->damping, M->d_sdinv, n);
    MIG_HIP(hipStreamSynchronize(A->ctx->stream));
    // the fused right Jacobi (one zero-start Jacobi sweep) and its ghost column scale
    if (M->rtype == 0 && M->sweeps == 1 && M->zero_start) prec_import_ghost_scale(*M);
    *out = M.release();
  });
}

extern "C" int migmres_jacobi_create(migmres_crs *A, int sweeps, double damping, migmres_prec **out) {
  return guard([&] {
    MIG_CHECK(sweeps >= 1, "\"relaxation: sweeps\" must be >= 1");
    migmres_relaxation_params p;
    migmres_relaxation_params_default(&p);
    p.sweeps = sweeps;
    p.damping = damping;
    const int rc = migmres_relaxation_create(A, &p, out);
    if (rc != MIGMRES_OK) throw Error(rc, migmres_last_error());
  });
}

extern "C" int migmres_chebyshev_params_default(migmres_chebyshev_params *p) {
  return guard([&] {
    MIG_CHECK(p, "chebyshev_params_default: null argument");
    *p = migmres_chebyshev_params{};
    p->degree = 1;
    p->max_eigenvalue = std::numeric_limits<double>::quiet_NaN();
    p->ratio_eigenvalue = 30.0;
    p->boost_factor = 1.1;
    p->min_diagonal_value = std::numeric_limits<double>::epsilon();
    p->eigenvalue_max_iterations = 10;
    p->zero_starting_solution = 1;
    p->assume_matrix_unchanged = 0;
    p->textbook_algorithm = 0;
    p->seed = 1;
  });
}

extern "C" int migmres_chebyshev_create(migmres_crs *A, const migmres_chebyshev_params *p, migmres_prec **out) {
  return guard([&] {
    MIG_CHECK(A && p && out, "chebyshev_create: null argument");
    // Details::Chebyshev::setParameters' checks (:465-582)
    MIG_CHECK(p->degree >= 0, "\"chebyshev: degree\" must be a nonnegative integer");
    MIG_CHECK(std::isnan(p->max_eigenvalue) || std::isfinite(p->max_eigenvalue),
              "\"chebyshev: max eigenvalue\" must be finite");
    MIG_CHECK(std::isfinite(p->ratio_eigenvalue) && p->ratio_eigenvalue >= 1.0,
              "\"chebyshev: ratio eigenvalue\" must be finite and >= 1");
    MIG_CHECK(p->boost_factor >= 1.0, "\"chebyshev: boost factor\" must be >= 1");
    MIG_CHECK(std::isfinite(p->min_diagonal_value), "\"chebyshev: min diagonal value\" must be finite");
    MIG_CHECK(p->eigenvalue_max_iterations >= 0, "\"chebyshev: eigenvalue max iterations\" must be nonnegative");
    std::unique_ptr<migmres_prec> M(new migmres_prec());
    M->ctx = A->ctx;
    M->A = A;
    M->kind = 1;
    M->cheb = *p;
    M->cheb_computed_lmax = std::numeric_limits<double>::quiet_NaN();
    const int n = A->n_local;
    MIG_HIP(hipMalloc(&M->d_dinv, sizeof(double) * (n > 0 ? n : 1)));
    launch_diag_recip_threshold(A->ctx->stream, A->d_rowptr, A->d_cols, A->d_vals, n, p->min_diagonal_value,
                                M->d_dinv);
    chebyshev_compute(*M);
    MIG_HIP(hipStreamSynchronize(A->ctx->stream));
    *out = M.release();
  });
}

extern "C" int migmres_chebyshev_lambdas(const migmres_prec *M, double *lmax, double *lmin, double *computed) {
  return guard([&] {
    MIG_CHECK(M && M->kind == 1, "chebyshev_lambdas: not a Chebyshev preconditioner");
    if (lmax) *lmax = M->cheb_lmax;
    if (lmin) *lmin = M->cheb_lmin;
    if (computed) *computed = M->cheb_computed_lmax;
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
    MIG_CHECK(M->kind != 2, "prec_diagonal: a user operator has no diagonal");
    MIG_HIP(hipMemcpy(dinv_out, M->d_dinv, sizeof(double) * M->A->n_local, hipMemcpyDeviceToHost));
  });
}
