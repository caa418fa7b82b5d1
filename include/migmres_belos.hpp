/*
 * migmres_belos.hpp -- header-only C++ traits adapter over the C ABI (include/migmres.h):
 * the Belos::MultiVecTraits / Belos::OperatorTraits static interface for a thin handle class,
 * i.e. what belos/epetra/src/BelosEpetraAdapter.hpp:447-1064 (MultiVecTraits<double,
 * Epetra_MultiVector>) and :1074-1114 (OperatorTraits<double, Epetra_MultiVector,
 * Epetra_Operator>) provide for Epetra, written against libmigmres.so.
 *
 * It depends on nothing but migmres.h and the C++ standard library, so it compiles (and is
 * tested: tests/abi_consumer/mvop_tester.cpp) without Belos or Teuchos.  A Belos build
 * specialises the real traits by forwarding to these functions:
 * Teuchos::SerialDenseMatrix maps onto DenseView {values(), stride(), numRows(), numCols()},
 * Teuchos::RCP onto std::shared_ptr, Belos::NormType onto NormType.
 *
 * Errors: every ABI failure throws migmres_belos::Failure carrying migmres_last_error(),
 * the analogue of EpetraMultiVecFailure / EpetraOpFailure (BelosEpetraAdapter.hpp:97-108).
 */
#ifndef MIGMRES_BELOS_HPP
#define MIGMRES_BELOS_HPP

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "migmres.h"

namespace migmres_belos {

struct Failure : std::runtime_error {
  int code;
  Failure(int c, const std::string &what) : std::runtime_error(what), code(c) {}
};

inline void check(int rc, const char *op) {
  if (rc != MIGMRES_OK) throw Failure(rc, std::string(op) + ": " + migmres_last_error());
}

enum NormType { OneNorm, TwoNorm, InfNorm };  // Belos::NormType (BelosTypes.hpp)
enum ETrans { NOTRANS, TRANS, CONJTRANS };    // Belos::ETrans

// Column-major dense block (Teuchos::SerialDenseMatrix<int,double> layout).
struct DenseView {
  double *values;
  int stride, rows, cols;
};

// A multivector handle: owns a block, or views columns of a parent it keeps alive.
class MV {
 public:
  MV(migmres_ctx *ctx, migmres_mv *h, std::shared_ptr<migmres_mv> parent = nullptr)
      : ctx_(ctx), h_(h, [](migmres_mv *p) { migmres_mv_destroy(p); }), parent_(std::move(parent)) {}
  migmres_mv *get() const { return h_.get(); }
  migmres_ctx *ctx() const { return ctx_; }
  // the owning block (this one if it owns, else the parent it views)
  std::shared_ptr<migmres_mv> root() const { return parent_ ? parent_ : h_; }

 private:
  migmres_ctx *ctx_;
  std::shared_ptr<migmres_mv> h_;
  std::shared_ptr<migmres_mv> parent_;
};

// An operator handle (the CRS matrix; Belos::OperatorTraits::Apply = migmres_crs_apply).
struct Op {
  migmres_crs *A;
};

// Belos::MultiVecTraits<double, MV> (belos/src/BelosMultiVecTraits.hpp:138-347).
struct MVT {
  static void shape(const MV &mv, long long *ng, int *nl, int *nc, int *cs) {
    check(migmres_mv_shape(mv.get(), ng, nl, nc, cs), "MvShape");
  }
  static std::shared_ptr<MV> Clone(const MV &mv, int numvecs) {
    long long ng;
    int nl, nc, cs;
    shape(mv, &ng, &nl, &nc, &cs);
    migmres_mv *p = nullptr;
    check(migmres_mv_create(mv.ctx(), ng, nl, numvecs, &p), "Clone");
    return std::make_shared<MV>(mv.ctx(), p);
  }
  static std::shared_ptr<MV> CloneCopy(const MV &mv) {
    auto c = Clone(mv, GetNumberVecs(mv));
    Assign(mv, *c);
    return c;
  }
  static std::shared_ptr<MV> CloneCopy(const MV &mv, const std::vector<int> &index) {
    auto v = CloneView(mv, index);
    auto c = Clone(mv, (int)index.size());
    Assign(*v, *c);
    return c;
  }
  static std::shared_ptr<MV> CloneViewNonConst(MV &mv, const std::vector<int> &index) {
    migmres_mv *p = nullptr;
    check(migmres_mv_view(mv.get(), index.data(), (int)index.size(), &p), "CloneViewNonConst");
    return std::make_shared<MV>(mv.ctx(), p, mv.root());
  }
  static std::shared_ptr<const MV> CloneView(const MV &mv, const std::vector<int> &index) {
    return CloneViewNonConst(const_cast<MV &>(mv), index);
  }
  static std::shared_ptr<MV> CloneViewRange(MV &mv, int first, int n) {  // Teuchos::Range1D form
    migmres_mv *p = nullptr;
    check(migmres_mv_view_range(mv.get(), first, n, &p), "CloneView(Range1D)");
    return std::make_shared<MV>(mv.ctx(), p, mv.root());
  }
  static long long GetGlobalLength(const MV &mv) {
    long long ng;
    int nl, nc, cs;
    shape(mv, &ng, &nl, &nc, &cs);
    return ng;
  }
  static int GetNumberVecs(const MV &mv) {
    long long ng;
    int nl, nc, cs;
    shape(mv, &ng, &nl, &nc, &cs);
    return nc;
  }
  static bool HasConstantStride(const MV &mv) {
    long long ng;
    int nl, nc, cs;
    shape(mv, &ng, &nl, &nc, &cs);
    return cs != 0;
  }
  // mv = beta mv + alpha A B
  static void MvTimesMatAddMv(double alpha, const MV &A, const DenseView &B, double beta, MV &mv) {
    check(migmres_mv_times_mat_add_mv(alpha, A.get(), B.values, B.stride, beta, mv.get()), "MvTimesMatAddMv");
  }
  static void MvAddMv(double alpha, const MV &A, double beta, const MV &B, MV &mv) {
    check(migmres_mv_add_mv(alpha, A.get(), beta, B.get(), mv.get()), "MvAddMv");
  }
  static void MvScale(MV &mv, double alpha) { check(migmres_mv_scale(mv.get(), alpha), "MvScale"); }
  static void MvScale(MV &mv, const std::vector<double> &alphas) {
    check(migmres_mv_scale_vec(mv.get(), alphas.data()), "MvScale(vector)");
  }
  // C = alpha A^T mv, replicated on every rank (the result is the caller's host block)
  static void MvTransMv(double alpha, const MV &A, const MV &mv, DenseView C) {
    check(migmres_mv_trans_mv(alpha, A.get(), mv.get(), C.values, C.stride), "MvTransMv");
  }
  // b[i] = <A_i, mv_i>; b keeps its size (MVOPTester: "should not be resized")
  static void MvDot(const MV &mv, const MV &A, std::vector<double> &b) {
    if ((int)b.size() < GetNumberVecs(mv)) b.resize((size_t)GetNumberVecs(mv));
    check(migmres_mv_dot(mv.get(), A.get(), b.data()), "MvDot");
  }
  static void MvNorm(const MV &mv, std::vector<double> &normvec, NormType type = TwoNorm) {
    if ((int)normvec.size() < GetNumberVecs(mv)) normvec.resize((size_t)GetNumberVecs(mv));
    const int t = type == OneNorm ? MIGMRES_ONE_NORM : type == TwoNorm ? MIGMRES_TWO_NORM : MIGMRES_INF_NORM;
    check(migmres_mv_norm(mv.get(), normvec.data(), t), "MvNorm");
  }
  static void SetBlock(const MV &A, const std::vector<int> &index, MV &mv) {
    check(migmres_mv_set_block(A.get(), index.data(), (int)index.size(), mv.get()), "SetBlock");
  }
  static void Assign(const MV &A, MV &mv) { check(migmres_mv_assign(A.get(), mv.get()), "Assign"); }
  // Epetra_MultiVector::Random draws a new stream per call; the seed advances across calls so
  // two MvRandom calls differ (MVOPTester "Vectors not random enough").
  static void MvRandom(MV &mv) { check(migmres_mv_random(mv.get(), &seed()), "MvRandom"); }
  static void MvInit(MV &mv, double alpha = 0.0) { check(migmres_mv_init(mv.get(), alpha), "MvInit"); }
  static unsigned &seed() {
    static unsigned s = 1;
    return s;
  }
};

// Belos::OperatorTraits<double, MV, Op> (belos/src/BelosOperatorTraits.hpp:108-155).
struct OPT {
  static void Apply(const Op &op, const MV &x, MV &y, ETrans trans = NOTRANS) {
    const int mode = trans == NOTRANS ? MIGMRES_NO_TRANS : trans == TRANS ? MIGMRES_TRANS : MIGMRES_CONJ_TRANS;
    check(migmres_crs_apply_mode(op.A, x.get(), y.get(), mode, 1.0, 0.0), "Apply");  // halo + SpMM (or A^T)
  }
  static bool HasApplyTranspose(const Op &) { return true; }
};

}  // namespace migmres_belos

#endif  // MIGMRES_BELOS_HPP
