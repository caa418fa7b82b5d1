// A C++ driver of the drop-in boundary that does what the reference's
// belos/epetra/example/BlockGmres/BlockGmresEpetraGaleriEx.cpp does -- Galeri "Laplace3D" on a
// uniform map, B = A * Xexact with Epetra_MultiVector::Random, X = 0, BlockGmresSolMgr with the
// command-line parameters, then the true relative residuals -- through include/migmres.h only
// (plain g++, no HIP headers).  Output lines follow the reference driver's summary so that a run
// reads like the recorded reference run.
//
//   block_gmres_galeri_ex [--nx=64] [--num-rhs=8] [--block-size=8] [--ortho=ICGS] [--tol=1e-8]
//                         [--max-subspace=50] [--max-restarts=50] [--max-iters=N]
//
// Xexact's seed: the reference's Xexact is the third Epetra_MultiVector the driver constructs,
// each construction consuming two std::rand() calls (Epetra_Util seeds from rand()), so its
// MINSTD stream starts at the 6th value of glibc's unseeded rand(): 424238335.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "migmres.h"

static void check(int rc, const char *what) {
  if (rc != MIGMRES_OK) {
    std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, migmres_last_error());
    std::exit(2);
  }
}

static bool opt(const char *arg, const char *name, std::string *val) {
  const size_t n = std::strlen(name);
  if (std::strncmp(arg, name, n) != 0 || arg[n] != '=') return false;
  *val = arg + n + 1;
  return true;
}

int main(int argc, char **argv) {
  int nx = 64, numrhs = 8, block = 8, maxsub = 50, maxrestarts = 50;
  long long maxiters = -1;
  double tol = 1.0e-8;
  std::string ortho = "ICGS", v;
  for (int i = 1; i < argc; ++i) {
    if (opt(argv[i], "--nx", &v)) nx = std::atoi(v.c_str());
    else if (opt(argv[i], "--num-rhs", &v)) numrhs = std::atoi(v.c_str());
    else if (opt(argv[i], "--block-size", &v)) block = std::atoi(v.c_str());
    else if (opt(argv[i], "--ortho", &v)) ortho = v;
    else if (opt(argv[i], "--tol", &v)) tol = std::atof(v.c_str());
    else if (opt(argv[i], "--max-subspace", &v)) maxsub = std::atoi(v.c_str());
    else if (opt(argv[i], "--max-restarts", &v)) maxrestarts = std::atoi(v.c_str());
    else if (opt(argv[i], "--max-iters", &v)) maxiters = std::atoll(v.c_str());
    else {
      std::fprintf(stderr, "unknown option %s\n", argv[i]);
      return 2;
    }
  }
  migmres_ctx *ctx = nullptr;
  check(migmres_ctx_create(0, 0, 1, nullptr, &ctx), "ctx_create");
  migmres_crs *A = nullptr;
  check(migmres_crs_create_galeri(ctx, "Laplace3D", nx, nx, nx, &A), "crs_create_galeri");
  const long long n = (long long)nx * nx * nx;
  if (maxiters < 0) maxiters = n / block - 1;  // the example's default: NumGlobalElements / blockSize - 1
  migmres_mv *X = nullptr, *B = nullptr, *Xex = nullptr, *R = nullptr;
  check(migmres_mv_create(ctx, n, (int)n, numrhs, &X), "mv_create");
  check(migmres_mv_create(ctx, n, (int)n, numrhs, &B), "mv_create");
  check(migmres_mv_create(ctx, n, (int)n, numrhs, &Xex), "mv_create");
  check(migmres_mv_create(ctx, n, (int)n, numrhs, &R), "mv_create");
  unsigned int seed = 424238335u;
  check(migmres_mv_random(Xex, &seed), "mv_random");
  check(migmres_crs_apply(A, Xex, B, 1.0, 0.0), "crs_apply");
  check(migmres_mv_init(X, 0.0), "mv_init");

  migmres_solver *S = nullptr;
  check(migmres_solver_create(ctx, &S), "solver_create");
  check(migmres_solver_set_int(S, "Block Size", block), "set Block Size");
  check(migmres_solver_set_int(S, "Num Blocks", maxsub), "set Num Blocks");
  check(migmres_solver_set_int(S, "Maximum Iterations", maxiters), "set Maximum Iterations");
  check(migmres_solver_set_int(S, "Maximum Restarts", maxrestarts), "set Maximum Restarts");
  check(migmres_solver_set_double(S, "Convergence Tolerance", tol), "set Convergence Tolerance");
  check(migmres_solver_set_string(S, "Orthogonalization", ortho.c_str()), "set Orthogonalization");
  int converged = 0, iters = 0;
  check(migmres_solver_solve(S, A, X, B, &converged), "solve");
  check(migmres_solver_num_iters(S, &iters), "num_iters");
  long long cnt[9] = {0};
  check(migmres_solver_counters(S, cnt, 9), "counters");

  // true residuals ||B - A X|| / ||B|| (the example's final check)
  check(migmres_crs_apply(A, X, R, 1.0, 0.0), "crs_apply");
  check(migmres_mv_add_mv(1.0, B, -1.0, R, R), "mv_add_mv");
  std::vector<double> rn((size_t)numrhs), bn((size_t)numrhs);
  check(migmres_mv_norm(R, rn.data(), MIGMRES_TWO_NORM), "mv_norm");
  check(migmres_mv_norm(B, bn.data(), MIGMRES_TWO_NORM), "mv_norm");
  std::printf("Dimension of matrix: %lld\n", n);
  std::printf("Number of right-hand sides: %d\n", numrhs);
  std::printf("Block size used by solver: %d\n", block);
  std::printf("Max number of Gmres iterations: %lld\n", maxiters);
  std::printf("Relative residual tolerance: %g\n", tol);
  std::printf("Number of iterations: %d\n", iters);
  std::printf("Operator applications: %lld (+1 for B = A Xexact)\n", cnt[0]);
  std::printf("Restarts: %lld\nExplicit residual checks: %lld\n", cnt[2], cnt[1]);
  bool bad = false;
  double rmin = 1e300, rmax = 0.0;
  for (int i = 0; i < numrhs; ++i) {
    const double rel = rn[(size_t)i] / bn[(size_t)i];
    rmin = std::fmin(rmin, rel);
    rmax = std::fmax(rmax, rel);
    std::printf("Problem %d : \t%g\n", i, rel);
    if (rel > tol) bad = true;
  }
  std::printf("True relative residuals: min %.1e max %.1e\n", rmin, rmax);
  migmres_solver_destroy(S);
  for (migmres_mv *m : {X, B, Xex, R}) migmres_mv_destroy(m);
  migmres_crs_destroy(A);
  migmres_ctx_destroy(ctx);
  if (!converged || bad) {
    std::printf("End Result: TEST FAILED\n");
    return 1;
  }
  std::printf("End Result: TEST PASSED\n");
  return 0;
}
