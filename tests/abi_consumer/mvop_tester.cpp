// A C++ consumer of the C ABI: include/migmres_belos.hpp (the Belos traits adapter of
// INTEGRATION.md section 2) compiled against include/migmres.h only, linked to
// libmigmres.so, and driven through the Belos MultiVecTraits / OperatorTraits contract
// suite -- TestMultiVecTraits (belos/src/BelosMVOPTester.hpp:84-1430) and TestOperatorTraits
// (:1452-1600) as belos/epetra/test/MVOPTester/cxx_main.cpp:46-103 runs them (a 100-row
// tridiagonal (-1 2 -1) operator, initial block of 5 columns) -- followed by a Block GMRES
// solve through the solver manager entry points.
//
// Each check below restates one invariant of the tester (same sizes, index sets, tolerance
// 100 eps, exact-zero checks where the tester requires them).  Prints "MVOPTESTER PASSED"
// and "SOLVE PASSED" and exits 0, or names the failed check and exits 1.
//
// usage: mvop_tester [n_rows]     (needs a GPU; run by tests/test_abi_consumer.py)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "migmres.h"
#include "migmres_belos.hpp"

using migmres_belos::DenseView;
using migmres_belos::MV;
using migmres_belos::MVT;
using migmres_belos::Op;
using migmres_belos::OPT;

static const double kTol = 100.0 * 2.220446049250313e-16;  // BelosMVOPTester.hpp:104
static int g_fail = 0;

#define EXPECT(cond, what)                                  \
  do {                                                      \
    if (!(cond)) {                                          \
      std::printf("FAILED: %s (line %d)\n", what, __LINE__); \
      g_fail = 1;                                           \
      return false;                                         \
    }                                                       \
  } while (0)

// Teuchos::SerialDenseMatrix stand-in (column-major, stride = rows).
struct Dense {
  int rows, cols;
  std::vector<double> v;
  Dense(int r, int c) : rows(r), cols(c), v((size_t)r * c, 0.0) {}
  double &operator()(int i, int j) { return v[(size_t)i + (size_t)j * rows]; }
  DenseView view() { return DenseView{v.data(), rows, rows, cols}; }
  void scale(double a) {
    for (auto &x : v) x *= a;
  }
  double normOne() const {
    double m = 0.0;
    for (int j = 0; j < cols; ++j) {
      double s = 0.0;
      for (int i = 0; i < rows; ++i) s += std::fabs(v[(size_t)i + (size_t)j * rows]);
      m = s > m ? s : m;
    }
    return m;
  }
  void random(unsigned &state) {  // Teuchos::randomSyncedMatrix: entries in [-1, 1]
    for (auto &x : v) {
      state = state * 1103515245u + 12345u;
      x = 2.0 * ((state >> 8) / 16777216.0) - 1.0;
    }
  }
};

static std::vector<double> norms(const MV &m, int n) {
  std::vector<double> r((size_t)n, -1.0);
  MVT::MvNorm(m, r);
  return r;
}

static bool test_multivec_traits(const MV &A) {
  const int numvecs = 10, numvecs_2 = 5;
  std::vector<int> ind = {0, 5, 2, 2, 9};  // BelosMVOPTester.hpp:188-195 (duplicates on purpose)
  unsigned sdm_state = 7;

  EXPECT(MVT::GetNumberVecs(A) > 0, "GetNumberVecs > 0");
  EXPECT(MVT::GetGlobalLength(A) > 0, "GetGlobalLength > 0");
  {  // Clone and MvNorm
    auto B = MVT::Clone(A, numvecs);
    std::vector<double> nrm((size_t)2 * numvecs, 0.0);
    EXPECT(MVT::GetNumberVecs(*B) == numvecs, "Clone: number of vectors");
    EXPECT(MVT::GetGlobalLength(*B) == MVT::GetGlobalLength(A), "Clone: length");
    MVT::MvInit(*B);  // Clone's contents are undefined; the tester only needs finite norms
    MVT::MvNorm(*B, nrm);
    EXPECT(nrm.size() == (size_t)2 * numvecs, "MvNorm resized its output");
    for (int i = 0; i < numvecs; ++i) EXPECT(nrm[(size_t)i] >= 0.0, "negative norm");
  }
  {  // MvRandom, MvNorm, MvInit
    auto B = MVT::Clone(A, numvecs);
    MVT::MvInit(*B);
    auto n0 = norms(*B, numvecs);
    for (double x : n0) EXPECT(x == 0.0, "MvInit: zero vector has non-zero norm");
    MVT::MvRandom(*B);
    auto n1 = norms(*B, numvecs);
    MVT::MvRandom(*B);
    auto n2 = norms(*B, numvecs);
    for (int i = 0; i < numvecs; ++i) {
      EXPECT(n1[(size_t)i] != 0.0 && n2[(size_t)i] != 0.0, "MvRandom: empty vector");
      EXPECT(n1[(size_t)i] > 0.0 && n2[(size_t)i] > 0.0, "MvRandom: negative norm");
      EXPECT(n1[(size_t)i] != n2[(size_t)i], "MvRandom: vectors not random enough");
    }
  }
  {  // MvRandom, MvScale (scalar and vector)
    auto B = MVT::Clone(A, numvecs);
    MVT::MvRandom(*B);
    MVT::MvScale(*B, 0.0);
    for (double x : norms(*B, numvecs)) EXPECT(x == 0.0, "MvScale(0): non-zero norm");
    MVT::MvRandom(*B);
    MVT::MvScale(*B, std::vector<double>((size_t)numvecs, 0.0));
    for (double x : norms(*B, numvecs)) EXPECT(x == 0.0, "MvScale(zeros): non-zero norm");
  }
  {  // MvInit(1): norm sqrt(n); MvInit(0) after
    auto B = MVT::Clone(A, numvecs);
    MVT::MvInit(*B, 1.0);
    const double want = std::sqrt((double)MVT::GetGlobalLength(A));
    for (double x : norms(*B, numvecs)) EXPECT(std::fabs(x - want) <= kTol * want, "MvInit(1): norm != sqrt(n)");
    MVT::MvInit(*B, 0.0);
    for (double x : norms(*B, numvecs)) EXPECT(x == 0.0, "MvInit(0): non-zero norm");
  }
  {  // CloneCopy(MV, index): sizes, values, independence
    auto B = MVT::Clone(A, numvecs);
    MVT::MvRandom(*B);
    auto nb = norms(*B, numvecs);
    auto C = MVT::CloneCopy(*B, ind);
    auto nc = norms(*C, numvecs);
    EXPECT(MVT::GetNumberVecs(*C) == numvecs_2, "CloneCopy(ind): count");
    EXPECT(MVT::GetGlobalLength(*C) == MVT::GetGlobalLength(*B), "CloneCopy(ind): length");
    for (int i = 0; i < numvecs_2; ++i)
      EXPECT(std::fabs(nc[(size_t)i] - nb[(size_t)ind[(size_t)i]]) <= kTol, "CloneCopy(ind): values");
    MVT::MvInit(*B, 0.0);
    auto nc2 = norms(*C, numvecs);
    for (int i = 0; i < numvecs_2; ++i)
      EXPECT(std::fabs(nc2[(size_t)i] - nc[(size_t)i]) <= kTol, "CloneCopy(ind): not independent");
  }
  {  // CloneCopy(MV)
    auto B = MVT::Clone(A, numvecs);
    MVT::MvRandom(*B);
    auto nb = norms(*B, numvecs);
    auto C = MVT::CloneCopy(*B);
    auto nc = norms(*C, numvecs);
    EXPECT(MVT::GetNumberVecs(*C) == numvecs, "CloneCopy: count");
    for (int i = 0; i < numvecs; ++i) EXPECT(std::fabs(nc[(size_t)i] - nb[(size_t)i]) <= kTol, "CloneCopy: values");
    MVT::MvInit(*B, 0.0);
    auto nc2 = norms(*C, numvecs);
    for (int i = 0; i < numvecs; ++i)
      EXPECT(std::fabs(nc2[(size_t)i] - nc[(size_t)i]) <= kTol, "CloneCopy: not independent");
  }
  {  // CloneViewNonConst(MV, index)
    auto B = MVT::Clone(A, numvecs);
    MVT::MvRandom(*B);
    auto nb = norms(*B, numvecs);
    auto C = MVT::CloneViewNonConst(*B, ind);
    auto nc = norms(*C, numvecs);
    EXPECT(MVT::GetNumberVecs(*C) == numvecs_2, "CloneViewNonConst: count");
    for (int i = 0; i < numvecs_2; ++i)
      EXPECT(std::fabs(nc[(size_t)i] - nb[(size_t)ind[(size_t)i]]) <= kTol, "CloneViewNonConst: values");
  }
  {  // CloneView(const MV, index)
    auto B = MVT::Clone(A, numvecs);
    MVT::MvRandom(*B);
    auto nb = norms(*B, numvecs);
    auto C = MVT::CloneView(*B, ind);
    auto nc = norms(*C, numvecs_2);
    EXPECT(MVT::GetNumberVecs(*C) == numvecs_2, "CloneView: count");
    for (int i = 0; i < numvecs_2; ++i)
      EXPECT(std::fabs(nc[(size_t)i] - nb[(size_t)ind[(size_t)i]]) <= kTol, "CloneView: values");
  }
  for (int variant = 0; variant < 2; ++variant) {  // SetBlock: C (5 or 6 columns) into every other column of B
    const int CSize = variant == 0 ? numvecs_2 : 6, setSize = 5, BSize = 2 * setSize;
    auto B = MVT::Clone(A, BSize);
    auto C = MVT::Clone(A, CSize);
    std::vector<int> sind((size_t)setSize);
    for (int i = 0; i < setSize; ++i) sind[(size_t)i] = 2 * i;
    MVT::MvRandom(*B);
    MVT::MvRandom(*C);
    auto nb1 = norms(*B, BSize), nc1 = norms(*C, CSize);
    MVT::SetBlock(*C, sind, *B);
    auto nb2 = norms(*B, BSize), nc2 = norms(*C, CSize);
    for (int i = 0; i < CSize; ++i) EXPECT(std::fabs(nc1[(size_t)i] - nc2[(size_t)i]) <= kTol, "SetBlock changed C");
    for (int i = 0; i < BSize; ++i) {
      if (i % 2 == 0)
        EXPECT(std::fabs(nb2[(size_t)i] - nc1[(size_t)(i / 2)]) <= kTol, "SetBlock: copied vectors do not agree");
      else
        EXPECT(std::fabs(nb1[(size_t)i] - nb2[(size_t)i]) <= kTol, "SetBlock: wrong vectors modified");
    }
    MVT::MvInit(*C, 0.0);
    auto nb3 = norms(*B, BSize);
    for (int i = 0; i < BSize; ++i) EXPECT(std::fabs(nb3[(size_t)i] - nb2[(size_t)i]) <= kTol, "SetBlock: not a copy");
  }
  {  // MvTransMv: 0 * B^T C == 0; |c_ij| <= |b_i||c_j|; zero B or C gives zeros
    const int p = 7, q = 9;
    auto B = MVT::Clone(A, p);
    auto C = MVT::Clone(A, q);
    Dense SDM(p, q);
    MVT::MvRandom(*B);
    auto nb = norms(*B, p);
    MVT::MvRandom(*C);
    auto nc = norms(*C, q);
    MVT::MvTransMv(0.0, *B, *C, SDM.view());
    EXPECT(SDM.rows == p && SDM.cols == q, "MvTransMv: size");
    EXPECT(SDM.normOne() == 0.0, "MvTransMv: 0 * B^T C != 0");
    MVT::MvTransMv(1.0, *B, *C, SDM.view());
    for (int i = 0; i < p; ++i)
      for (int j = 0; j < q; ++j)
        EXPECT(std::fabs(SDM(i, j)) <= std::fabs(nb[(size_t)i] * nc[(size_t)j]), "MvTransMv: triangle inequality");
    MVT::MvInit(*C);
    MVT::MvRandom(*B);
    MVT::MvTransMv(1.0, *B, *C, SDM.view());
    for (double x : SDM.v) EXPECT(x == 0.0, "MvTransMv: B^T 0 != 0");
    MVT::MvInit(*B);
    MVT::MvRandom(*C);
    MVT::MvTransMv(1.0, *B, *C, SDM.view());
    for (double x : SDM.v) EXPECT(x == 0.0, "MvTransMv: 0^T C != 0");
  }
  {  // MvDot
    const int p = 7, q = 9;
    auto B = MVT::Clone(A, p);
    auto C = MVT::Clone(A, p);
    std::vector<double> iprods((size_t)(p + q), 0.0);
    MVT::MvRandom(*B);
    MVT::MvRandom(*C);
    auto nb = norms(*B, p), nc = norms(*C, p);
    MVT::MvDot(*B, *C, iprods);
    EXPECT(iprods.size() == (size_t)(p + q), "MvDot resized its output");
    for (int i = 0; i < p; ++i)
      EXPECT(std::fabs(iprods[(size_t)i]) <= std::fabs(nb[(size_t)i] * nc[(size_t)i]), "MvDot: inequality");
    MVT::MvInit(*B);
    MVT::MvRandom(*C);
    MVT::MvDot(*B, *C, iprods);
    for (int i = 0; i < p; ++i) EXPECT(iprods[(size_t)i] == 0.0, "MvDot: <0, c> != 0");
    MVT::MvInit(*C);
    MVT::MvRandom(*B);
    MVT::MvDot(*B, *C, iprods);
    for (int i = 0; i < p; ++i) EXPECT(iprods[(size_t)i] == 0.0, "MvDot: <b, 0> != 0");
  }
  {  // MvAddMv: 0B + 1C == C, 1B + 0C == B, invariant under the initial D, inputs unmodified
    const int p = 7;
    auto B = MVT::Clone(A, p), C = MVT::Clone(A, p), D = MVT::Clone(A, p);
    Dense ab(1, 2);
    ab.random(sdm_state);
    const double alpha = ab(0, 0), beta = ab(0, 1);
    MVT::MvRandom(*B);
    MVT::MvRandom(*C);
    auto nb1 = norms(*B, p), nc1 = norms(*C, p);
    MVT::MvAddMv(0.0, *B, 1.0, *C, *D);
    auto nb2 = norms(*B, p), nc2 = norms(*C, p), nd = norms(*D, p);
    for (int i = 0; i < p; ++i) {
      EXPECT(std::fabs(nb1[(size_t)i] - nb2[(size_t)i]) <= kTol, "MvAddMv modified B");
      EXPECT(std::fabs(nc1[(size_t)i] - nc2[(size_t)i]) <= kTol, "MvAddMv modified C");
      EXPECT(std::fabs(nc1[(size_t)i] - nd[(size_t)i]) <= kTol, "MvAddMv: 0B + 1C != C");
    }
    MVT::MvAddMv(1.0, *B, 0.0, *C, *D);
    nd = norms(*D, p);
    for (int i = 0; i < p; ++i) EXPECT(std::fabs(nb1[(size_t)i] - nd[(size_t)i]) <= kTol, "MvAddMv: 1B + 0C != B");
    MVT::MvRandom(*D);
    MVT::MvAddMv(alpha, *B, beta, *C, *D);
    auto nd1 = norms(*D, p);
    MVT::MvInit(*D);
    MVT::MvAddMv(alpha, *B, beta, *C, *D);
    auto nd2 = norms(*D, p);
    nb2 = norms(*B, p);
    nc2 = norms(*C, p);
    for (int i = 0; i < p; ++i) {
      EXPECT(std::fabs(nb1[(size_t)i] - nb2[(size_t)i]) <= kTol, "MvAddMv modified B");
      EXPECT(std::fabs(nc1[(size_t)i] - nc2[(size_t)i]) <= kTol, "MvAddMv modified C");
      EXPECT(std::fabs(nd1[(size_t)i] - nd2[(size_t)i]) <= kTol, "MvAddMv depends on the initial D");
    }
  }
  {  // MvAddMv with aliased arguments (D and C views of B)
    const int p = 7;
    auto B = MVT::Clone(A, p);
    std::vector<int> all((size_t)p);
    for (int i = 0; i < p; ++i) all[(size_t)i] = i;
    auto C = MVT::CloneView(*B, all);
    auto D = MVT::CloneViewNonConst(*B, all);
    MVT::MvRandom(*B);
    auto nb = norms(*B, p);
    MVT::MvAddMv(0.0, *B, 1.0, *C, *D);
    auto nd = norms(*D, p);
    for (int i = 0; i < p; ++i) EXPECT(std::fabs(nb[(size_t)i] - nd[(size_t)i]) <= kTol, "aliased MvAddMv: 0B + 1C");
    MVT::MvAddMv(1.0, *B, 0.0, *C, *D);
    nd = norms(*D, p);
    for (int i = 0; i < p; ++i) EXPECT(std::fabs(nb[(size_t)i] - nd[(size_t)i]) <= kTol, "aliased MvAddMv: 1B + 0C");
  }
  for (int shape = 0; shape < 2; ++shape) {  // MvTimesMatAddMv 7 x 5, then 5 x 7
    const int p = shape == 0 ? 7 : 5, q = shape == 0 ? 5 : 7;
    auto B = MVT::Clone(A, p), C = MVT::Clone(A, q);
    Dense SDM(p, q);
    // alpha 0, beta 1: C unchanged
    MVT::MvRandom(*B);
    MVT::MvRandom(*C);
    auto nb1 = norms(*B, p), nc1 = norms(*C, q);
    SDM.random(sdm_state);
    MVT::MvTimesMatAddMv(0.0, *B, SDM.view(), 1.0, *C);
    auto nb2 = norms(*B, p), nc2 = norms(*C, q);
    for (int i = 0; i < p; ++i) EXPECT(std::fabs(nb1[(size_t)i] - nb2[(size_t)i]) <= kTol, "MvTimesMatAddMv modified B");
    for (int i = 0; i < q; ++i) EXPECT(std::fabs(nc1[(size_t)i] - nc2[(size_t)i]) <= kTol, "test 1/5: C changed");
    // alpha 0, beta 0: C zero
    MVT::MvRandom(*B);
    MVT::MvRandom(*C);
    SDM.random(sdm_state);
    MVT::MvTimesMatAddMv(0.0, *B, SDM.view(), 0.0, *C);
    for (double x : norms(*C, q)) EXPECT(x == 0.0, "test 2/6: C not zero");
    // alpha 1, SDM = I (padded), beta 0: C = B (first min(p, q) columns), the rest zero
    MVT::MvRandom(*B);
    MVT::MvRandom(*C);
    nb1 = norms(*B, p);
    SDM.scale(0.0);
    for (int i = 0; i < (p < q ? p : q); ++i) SDM(i, i) = 1.0;
    MVT::MvTimesMatAddMv(1.0, *B, SDM.view(), 0.0, *C);
    nc2 = norms(*C, q);
    for (int i = 0; i < (p < q ? p : q); ++i)
      EXPECT(std::fabs(nb1[(size_t)i] - nc2[(size_t)i]) <= kTol, "test 3/7: C != B");
    for (int i = p; i < q; ++i) EXPECT(nc2[(size_t)i] == 0.0, "test 7: padding columns not zero");
    // alpha 1, SDM = 0, beta 1: C unchanged
    MVT::MvRandom(*B);
    MVT::MvRandom(*C);
    nc1 = norms(*C, q);
    SDM.scale(0.0);
    MVT::MvTimesMatAddMv(1.0, *B, SDM.view(), 1.0, *C);
    nc2 = norms(*C, q);
    for (int i = 0; i < q; ++i) EXPECT(std::fabs(nc1[(size_t)i] - nc2[(size_t)i]) <= kTol, "test 4/8: C changed");
  }
  return true;
}

static bool test_operator_traits(const MV &A, const Op &M) {
  const int numvecs = 10;
  auto B = MVT::Clone(A, numvecs), C = MVT::Clone(A, numvecs);
  MVT::MvInit(*B);
  MVT::MvRandom(*C);
  auto nb1 = norms(*B, numvecs);
  OPT::Apply(M, *B, *C);
  auto nb2 = norms(*B, numvecs), nc2 = norms(*C, numvecs);
  for (int i = 0; i < numvecs; ++i) {
    EXPECT(std::fabs(nb2[(size_t)i] - nb1[(size_t)i]) <= kTol, "Apply modified its input");
    EXPECT(nc2[(size_t)i] == 0.0, "Apply: OP * 0 != 0");
  }
  MVT::MvRandom(*B);
  nb1 = norms(*B, numvecs);
  OPT::Apply(M, *B, *C);
  nb2 = norms(*B, numvecs);
  nc2 = norms(*C, numvecs);
  for (int i = 0; i < numvecs; ++i) {
    EXPECT(std::fabs(nb2[(size_t)i] - nb1[(size_t)i]) <= kTol, "Apply modified its input");
    EXPECT(nc2[(size_t)i] != 0.0, "Apply: OP * random == 0");
  }
  MVT::MvInit(*C);
  OPT::Apply(M, *B, *C);
  auto nc_zero_start = norms(*C, numvecs);
  MVT::MvRandom(*C);
  OPT::Apply(M, *B, *C);
  auto nc_rand_start = norms(*C, numvecs);
  for (int i = 0; i < numvecs; ++i)
    EXPECT(nc_zero_start[(size_t)i] == nc_rand_start[(size_t)i], "Apply depends on the initial destination");
  // A^T (migmres_crs_apply_mode): the operator is the symmetric (-1, 2, -1) tridiagonal, so A^T B
  // equals A B up to the order of the sums
  EXPECT(OPT::HasApplyTranspose(M), "HasApplyTranspose");
  auto CT = MVT::Clone(*C, numvecs);
  OPT::Apply(M, *B, *C);
  OPT::Apply(M, *B, *CT, migmres_belos::TRANS);
  MVT::MvAddMv(1.0, *CT, -1.0, *C, *CT);
  auto nd = norms(*CT, numvecs), nc = norms(*C, numvecs);
  for (int i = 0; i < numvecs; ++i) EXPECT(nd[(size_t)i] <= 1e-13 * nc[(size_t)i], "Apply(TRANS) != Apply on a symmetric operator");
  return true;
}

// Block GMRES through the solver-manager entry points on the
// Galeri 2-D Laplacian, checked by its own explicit residual.
static bool test_solve(migmres_ctx *ctx) {
  const int nx = 40, ny = 40, k = 4;
  const long long n = (long long)nx * ny;
  migmres_crs *A = nullptr;
  migmres_belos::check(migmres_crs_create_galeri(ctx, "Laplace2D", nx, ny, 1, &A), "crs_create_galeri");
  long long first;
  int nl;
  migmres_belos::check(migmres_map_uniform(n, 1, 0, &first, &nl), "map_uniform");
  migmres_mv *Xe, *B, *X, *R;
  migmres_belos::check(migmres_mv_create(ctx, n, nl, k, &Xe), "mv_create");
  migmres_belos::check(migmres_mv_create(ctx, n, nl, k, &B), "mv_create");
  migmres_belos::check(migmres_mv_create(ctx, n, nl, k, &X), "mv_create");
  migmres_belos::check(migmres_mv_create(ctx, n, nl, k, &R), "mv_create");
  unsigned seed = 1;
  migmres_belos::check(migmres_mv_random(Xe, &seed), "mv_random");
  migmres_belos::check(migmres_crs_apply(A, Xe, B, 1.0, 0.0), "apply");
  migmres_belos::check(migmres_mv_init(X, 0.0), "mv_init");
  migmres_solver *s = nullptr;
  migmres_belos::check(migmres_solver_create_named(ctx, "BLOCK GMRES", &s), "solver_create");
  migmres_belos::check(migmres_solver_set_int(s, "Block Size", k), "set Block Size");
  migmres_belos::check(migmres_solver_set_int(s, "Num Blocks", 30), "set Num Blocks");
  migmres_belos::check(migmres_solver_set_int(s, "Maximum Iterations", 1000), "set Maximum Iterations");
  migmres_belos::check(migmres_solver_set_int(s, "Maximum Restarts", 50), "set Maximum Restarts");
  migmres_belos::check(migmres_solver_set_double(s, "Convergence Tolerance", 1e-9), "set tol");
  // "Orthogonalization" left at the reference default ("DGKS", BelosBlockGmresSolMgr.hpp:323-338)
  EXPECT(migmres_solver_set_string(s, "Orthogonalization", "QR") != MIGMRES_OK, "bad parameter accepted");
  int converged = 0, iters = 0;
  migmres_belos::check(migmres_solver_solve(s, A, X, B, &converged), "solve");
  migmres_belos::check(migmres_solver_num_iters(s, &iters), "num_iters");
  migmres_belos::check(migmres_mv_add_mv(1.0, B, 0.0, B, R), "copy");
  migmres_belos::check(migmres_crs_apply(A, X, R, -1.0, 1.0), "residual");
  std::vector<double> rn((size_t)k), bn((size_t)k);
  migmres_belos::check(migmres_mv_norm(R, rn.data(), MIGMRES_TWO_NORM), "norm");
  migmres_belos::check(migmres_mv_norm(B, bn.data(), MIGMRES_TWO_NORM), "norm");
  double worst = 0.0;
  for (int j = 0; j < k; ++j) worst = rn[(size_t)j] / bn[(size_t)j] > worst ? rn[(size_t)j] / bn[(size_t)j] : worst;
  std::printf("solve: converged %d, %d iterations, max ||B - A X|| / ||B|| = %.3e\n", converged, iters, worst);
  EXPECT(converged == 1 && iters > 0 && worst <= 1e-9, "Block GMRES solve");
  migmres_solver_destroy(s);
  for (migmres_mv *m : {Xe, B, X, R}) migmres_mv_destroy(m);
  migmres_crs_destroy(A);
  return true;
}

int main(int argc, char **argv) {
  const long long dim = argc > 1 ? std::atoll(argv[1]) : 100;  // cxx_main.cpp: dim = 100
  const int block = 5;
  if (migmres_abi_version() != MIGMRES_ABI_VERSION) {
    std::printf("FAILED: ABI version %d, header %d\n", migmres_abi_version(), MIGMRES_ABI_VERSION);
    return 1;
  }
  migmres_ctx *ctx = nullptr;
  try {
    migmres_belos::check(migmres_ctx_create(0, 0, 1, nullptr, &ctx), "ctx_create");
    // the MVOPTester operator: tridiagonal (-1 2 -1), rows in InsertGlobalValues order
    // (off-diagonals first, then the diagonal; cxx_main.cpp:103-150)
    std::vector<long long> rowptr{0}, gcols;
    std::vector<double> vals;
    for (long long g = 0; g < dim; ++g) {
      if (g > 0) gcols.push_back(g - 1), vals.push_back(-1.0);
      if (g < dim - 1) gcols.push_back(g + 1), vals.push_back(-1.0);
      gcols.push_back(g), vals.push_back(2.0);
      rowptr.push_back((long long)gcols.size());
    }
    migmres_crs *Acrs = nullptr;
    migmres_belos::check(migmres_crs_create(ctx, dim, 0, (int)dim, rowptr.data(), gcols.data(), vals.data(), &Acrs),
                         "crs_create");
    migmres_mv *iv = nullptr;
    migmres_belos::check(migmres_mv_create(ctx, dim, (int)dim, block, &iv), "mv_create");
    MV ivec(ctx, iv);
    MVT::MvRandom(ivec);
    const bool mv_ok = test_multivec_traits(ivec);
    const bool op_ok = mv_ok && test_operator_traits(ivec, Op{Acrs});
    if (mv_ok && op_ok) std::printf("MVOPTESTER PASSED\n");
    const bool solve_ok = test_solve(ctx);
    if (solve_ok) std::printf("SOLVE PASSED\n");
    migmres_crs_destroy(Acrs);
  } catch (const std::exception &e) {
    std::printf("FAILED: exception %s\n", e.what());
    g_fail = 1;
  }
  if (ctx) migmres_ctx_destroy(ctx);
  return g_fail;
}
