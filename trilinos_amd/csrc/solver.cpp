// Block GMRES solver manager, block Arnoldi iteration and ICGS orthogonalisation on
// device multivectors.  Host C++ keeps exactly the reference's control flow and small
// dense algebra; every N-sized operation is a HIP kernel (runtime.cpp / kernels.hip).
//
//   ICGS                 belos/src/BelosICGSOrthoManager.hpp:646-1701
//   BlockGmresIter       belos/src/BelosBlockGmresIter.hpp:405-868
//   StatusTestImpResNorm belos/src/BelosStatusTestImpResNorm.hpp:492-749, 808-845
//   StatusTestMaxIters   belos/src/BelosStatusTestMaxIters.hpp:165-172
//   LinearProblem        belos/src/BelosLinearProblem.hpp:642-1231
//   BlockGmresSolMgr     belos/src/BelosBlockGmresSolMgr.hpp:430-1303
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <string>

#include "icgs.h"
#include "runtime.h"

using namespace migmres;

namespace {


struct MvPtr {
  migmres_mv *p = nullptr;
  MvPtr() = default;
  explicit MvPtr(migmres_mv *q) : p(q) {}
  MvPtr(const MvPtr &) = delete;
  MvPtr &operator=(const MvPtr &) = delete;
  MvPtr(MvPtr &&o) noexcept : p(o.p) { o.p = nullptr; }
  MvPtr &operator=(MvPtr &&o) noexcept {
    reset();
    p = o.p;
    o.p = nullptr;
    return *this;
  }
  ~MvPtr() { reset(); }
  void reset() {
    if (p) {
      if (p->d_cols) hipStreamSynchronize(p->ctx->stream);
      delete p;
    }
    p = nullptr;
  }
  migmres_mv &operator*() const { return *p; }
  migmres_mv *operator->() const { return p; }
};

MvPtr view(migmres_mv &m, int first, int n) { return MvPtr(mv_view_range(&m, first, n)); }

double dot1(const migmres_mv &a, const migmres_mv &b) {
  double r = 0.0;
  mv_dot(a, b, &r);
  return r;
}

const double kEps = std::numeric_limits<double>::epsilon();

// ------------------------------------------------------------------------------------
// ICGS orthogonalisation manager (max_ortho_steps = 2, blk_tol = 10 sqrt(eps),
// sing_tol = 10 eps: BelosICGSOrthoManager.hpp:561-573)
// ------------------------------------------------------------------------------------
// With dgks = true the same object is Belos::DGKSOrthoManager (BelosDGKSOrthoManager.hpp,
// defaults 536-556: 2 passes, blk_tol = 10 sqrt(eps), dep_tol = 1/sqrt(2), sing_tol = 10 eps):
// the same projectAndNormalize / blkOrtho, but blkOrtho1, findBasis and blkOrthoSing
// re-orthogonalise only when the first pass lost too much (the dep_tol criterion).
struct Icgs {
  int steps = 2;
  double blk_tol = 10.0 * std::sqrt(kEps);
  double sing_tol = 10.0 * kEps;
  bool dgks = false;
  double dep_tol = 1.0 / std::sqrt(2.0);
  unsigned int seed = 12345u;  // MvRandom stream for rank-deficiency fallbacks
  long long sing_count = 0;

  // projectAndNormalizeWithMxImpl (BelosICGSOrthoManager.hpp:646-821).
  // C is (Q.ncols x X.ncols, ldc), B is (X.ncols x X.ncols, ldb), both host.
  int project_and_normalize(migmres_mv &X, migmres_mv &Q, double *C, int ldc, double *B, int ldb) {
    const int xc = X.ncols;
    if (xc == 1) {
      blk_ortho1(X, Q, C, ldc);
      const double d = dot1(X, X);
      B[0] = std::sqrt(std::fabs(d));
      if (std::fabs(B[0]) > 0.0) mv_scale(X, 1.0 / B[0]);
      return 1;
    }
    MvPtr tmpX(mv_create(X.ctx, X.n_global, X.n_local, xc));
    mv_assign(X, *tmpX);
    int rank;
    if (blk_ortho(X, Q, C, ldc)) {
      rank = blk_ortho_sing(*tmpX, Q, C, ldc, B, ldb);
      mv_assign(*tmpX, X);
    } else {
      rank = find_basis(X, B, ldb, false);
      if (rank < xc) {
        rank = blk_ortho_sing(*tmpX, Q, C, ldc, B, ldb);
        mv_assign(*tmpX, X);
      }
    }
    MIG_HIP(hipStreamSynchronize(X.ctx->stream));
    return rank;
  }

  int normalize(migmres_mv &X, double *B, int ldb) { return find_basis(X, B, ldb, true); }

  // blkOrtho1 (BelosICGSOrthoManager.hpp:1231-1322; DGKS: BelosDGKSOrthoManager.hpp:1245-1321), and
  // the projection passes of blkOrtho (ICGS :1328-1445, DGKS :1373-1490, the same for both)
  void blk_ortho1(migmres_mv &X, migmres_mv &Q, double *C, int ldc) {
    const int L = Q.ncols, k = X.ncols;
    double old_dot = 0.0;
    if (dgks && k == 1) old_dot = dot1(X, X);
    mv_trans_mv(1.0, Q, X, C, ldc);
    mv_times_mat_add_mv(-1.0, Q, C, ldc, 1.0, X);
    std::vector<double> C2((size_t)L * k);
    if (dgks && k == 1) {  // DGKS blkOrtho on k > 1 columns: the passes below
      const double new_dot = dot1(X, X);
      if (std::sqrt(std::fabs(new_dot)) < dep_tol * std::sqrt(std::fabs(old_dot))) {
        mv_trans_mv(1.0, Q, X, C2.data(), L);
        for (int i = 0; i < L; ++i) C[i] += C2[(size_t)i];
        mv_times_mat_add_mv(-1.0, Q, C2.data(), L, 1.0, X);
      }
      return;
    }
    for (int s = 1; s < steps; ++s) {
      mv_trans_mv(1.0, Q, X, C2.data(), L);
      for (int j = 0; j < k; ++j)
        for (int i = 0; i < L; ++i) C[i + (size_t)j * ldc] += C2[i + (size_t)j * L];
      mv_times_mat_add_mv(-1.0, Q, C2.data(), L, 1.0, X);
    }
  }

  // blkOrtho (BelosICGSOrthoManager.hpp:1328-1445); returns the dependency flag.
  bool blk_ortho(migmres_mv &X, migmres_mv &Q, double *C, int ldc) {
    const int L = Q.ncols, k = X.ncols;
    std::vector<double> old_dot((size_t)k), new_dot((size_t)k);
    mv_dot(X, X, old_dot.data());
    blk_ortho1(X, Q, C, ldc);
    mv_dot(X, X, new_dot.data());
    (void)L;
    for (int i = 0; i < k; ++i)
      if (std::fabs(new_dot[(size_t)i]) < std::fabs(old_dot[(size_t)i] * blk_tol)) return true;
    return false;
  }

  // findBasis (BelosICGSOrthoManager.hpp:936-1225), howMany = all columns.
  int find_basis(migmres_mv &X, double *B, int ldb, bool complete) {
    const int xc = X.ncols;
    MvPtr old_xj(mv_create(X.ctx, X.n_global, X.n_local, 1));
    std::vector<double> P2, product;
    for (int j = 0; j < xc; ++j) {
      MvPtr Xj = view(X, j, 1);
      MvPtr prevX = view(X, 0, j);
      bool add_vec = false;
      if (j > 0) mv_assign(*Xj, *old_xj);
      double old_dot = dot1(*Xj, *Xj);
      if (old_dot < 0.0) throw Error(MIGMRES_ESTATE, "ICGS: negative definiteness in inner product");
      product.assign((size_t)j, 0.0);
      double new_dot;
      if (j > 0) {
        P2.assign((size_t)j, 0.0);
        for (int s = 0; s < steps; ++s) {
          if (dgks && s > 0) {  // BelosDGKSOrthoManager.hpp:1086-1119
            const double nd = dot1(*Xj, *Xj);
            if (!(std::sqrt(std::fabs(nd)) < dep_tol * std::sqrt(std::fabs(old_dot)))) break;
          }
          mv_trans_mv(1.0, *prevX, *Xj, P2.data(), j);
          mv_times_mat_add_mv(-1.0, *prevX, P2.data(), j, 1.0, *Xj);
          for (int i = 0; i < j; ++i) product[(size_t)i] = (s == 0) ? P2[(size_t)i] : product[(size_t)i] + P2[(size_t)i];
        }
        new_dot = dot1(*Xj, *old_xj);
      } else {
        new_dot = old_dot;
      }
      if (complete) {
        if (std::fabs(new_dot) < std::fabs(sing_tol * old_dot)) {
          add_vec = true;
          MvPtr t(mv_create(X.ctx, X.n_global, X.n_local, 1));
          mv_random(*t, &seed);
          old_dot = dot1(*t, *t);
          std::vector<double> pr((size_t)(j > 0 ? j : 1));
          for (int s = 0; s < steps && j > 0; ++s) {
            mv_trans_mv(1.0, *prevX, *t, pr.data(), j);
            mv_times_mat_add_mv(-1.0, *prevX, pr.data(), j, 1.0, *t);
          }
          new_dot = dot1(*t, *t);
          if (std::fabs(new_dot) >= std::fabs(old_dot * sing_tol))
            mv_assign(*t, *Xj);
          else
            return j;
        }
      } else if (std::fabs(new_dot) < std::fabs(old_dot * blk_tol)) {
        return j;
      }
      const double diag = std::sqrt(std::fabs(new_dot));
      if (!dgks || std::fabs(diag) > 0.0) mv_scale(*Xj, 1.0 / diag);
      B[j + (size_t)j * ldb] = add_vec ? 0.0 : diag;
      if (!add_vec)
        for (int i = 0; i < j; ++i) B[i + (size_t)j * ldb] = product[(size_t)i];
    }
    return xc;
  }

  // blkOrthoSing (BelosICGSOrthoManager.hpp:1449-1701), including the reference's use of a
  // newDot that is only refreshed on the random-vector path.
  int blk_ortho_sing(migmres_mv &X, migmres_mv &Q, double *C, int ldc, double *B, int ldb) {
    ++sing_count;
    const int xc = X.ncols, L = Q.ncols;
    double new_dot = 0.0;
    std::vector<double> tc((size_t)L + xc), c2((size_t)L + xc);
    for (int j = 0; j < xc; ++j) {
      MvPtr Xj = view(X, j, 1);
      MvPtr lastQ = view(X, 0, j);
      migmres_mv *Qs[2] = {&Q, lastQ.p};
      double *Cs[2] = {C, B};
      const int lds[2] = {ldc, ldb};
      const int nq = j > 0 ? 2 : 1;
      double old_dot = dot1(*Xj, *Xj);
      for (int i = 0; i < nq; ++i) {
        const int q = Qs[i]->ncols;
        double *col = Cs[i] + (size_t)j * lds[i];
        mv_trans_mv(1.0, *Qs[i], *Xj, col, q);
        mv_times_mat_add_mv(-1.0, *Qs[i], col, q, 1.0, *Xj);
      }
      bool second = true;
      if (dgks) {  // BelosDGKSOrthoManager.hpp:1590-1625: re-orthogonalise on |new| < |old dep_tol|
        new_dot = dot1(*Xj, *Xj);
        second = std::fabs(new_dot) < std::fabs(old_dot * dep_tol);
      }
      for (int s = 1; s < steps && second; ++s) {
        for (int i = 0; i < nq; ++i) {
          const int q = Qs[i]->ncols;
          double *col = Cs[i] + (size_t)j * lds[i];
          mv_trans_mv(1.0, *Qs[i], *Xj, c2.data(), q);
          for (int r = 0; r < q; ++r) col[r] += c2[(size_t)r];
          mv_times_mat_add_mv(-1.0, *Qs[i], c2.data(), q, 1.0, *Xj);
        }
        if (dgks) new_dot = dot1(*Xj, *Xj);
      }
      const bool dep = std::fabs(new_dot) < std::fabs(old_dot * sing_tol);
      if (!dep) {
        const double diag = std::sqrt(std::fabs(new_dot));
        mv_scale(*Xj, 1.0 / diag);
        B[j + (size_t)j * ldb] = diag;
      } else {
        MvPtr t(mv_create(X.ctx, X.n_global, X.n_local, 1));
        mv_random(*t, &seed);
        old_dot = dot1(*t, *t);
        for (int s = 0; s < steps; ++s)
          for (int i = 0; i < nq; ++i) {
            const int q = Qs[i]->ncols;
            mv_trans_mv(1.0, *Qs[i], *t, tc.data(), q);
            mv_times_mat_add_mv(-1.0, *Qs[i], tc.data(), q, 1.0, *t);
          }
        new_dot = dot1(*t, *t);
        if (std::fabs(new_dot) >= std::fabs(old_dot * sing_tol)) {
          const double diag = std::sqrt(std::fabs(new_dot));
          B[j + (size_t)j * ldb] = 0.0;
          mv_add_mv(1.0 / diag, *t, 0.0, *t, *Xj);
        } else {
          return j;
        }
      }
    }
    return xc;
  }
};

// ------------------------------------------------------------------------------------
// Device-resident ICGS (same operation sequence as Icgs above; coefficients and
// decisions stay on the device, one host synchronisation per call).  Falls back to the
// host-driven Icgs -- from the saved input block -- whenever the reference would leave
// the fast path (blkOrtho dependency, findBasis rank deficiency).
// ------------------------------------------------------------------------------------
struct FastIcgs {
  migmres_ctx *ctx = nullptr;
  Icgs *slow = nullptr;
  int n_local = 0, kmax = 0, Lmax = 0;
  long long n_global = 0;
  int nblk_tn = 1, nblk_ic = 1;
  double *partial = nullptr, *R1 = nullptr, *R2 = nullptr, *Cout = nullptr, *red = nullptr, *S = nullptr;
  double *cout_own = nullptr;  // Cout's own buffer (Cout may point behind the state instead)
  double *sink = nullptr;  // absorbs the padding-lane stores of the fused update kernel
  IcgsState *st = nullptr;   // current state (one of stb)
  IcgsState *stb[2] = {nullptr, nullptr};
  double *pbuf[2] = {nullptr, nullptr};  // per-workgroup partials, alternating between passes
  // The reduction + scalar step a pass leaves pending; the next pass takes it in its
  // prologue (FbPro) -- no separate reduce / scalar launches between the findBasis passes.
  struct Pending {
    bool on = false;
    const double *partial = nullptr;  // nullptr: the all-reduced vector in `red`
    int nv = 0, s0 = -1, s1 = -1, j = 0, k = 0, complete = 0;
  } pend;
  double *h = nullptr;  // pinned: state + C
  // Work the caller enqueues behind the state copy before the host waits for it (the next
  // block's SpMM): the GPU keeps running while the host takes the least-squares update.
  std::function<void()> before_wait;
  hipEvent_t ev_fetch = nullptr;
  MvPtr tmpX;
  long long calls = 0, fallbacks = 0;
  bool use_fused = true;  // MIGMRES_NO_FUSED_NN_TN=1 selects the two-kernel form (A/B timing)
  int fb_rev = 1;         // findBasis b2 passes sweep rows top-down (MIGMRES_FB_REV=0: all bottom-up)
  bool x1_store = false;  // fused pass writes X1 back (MIGMRES_NN_TN_STORE=1, A/B timing)
  int nt_cache[1025][4] = {};
  // findBasis in Gram form (icgs.hip k_fbg_*; ICGS with two passes, 2 <= k <= 8).
  // MIGMRES_FB_GRAM=0 keeps the column passes; MIGMRES_FB_GRAM_FUSE=0 takes G1 in a pass of
  // its own instead of in the closing update; MIGMRES_FB_GRAM_GATE overrides the pivot-ratio
  // gate (default 100 blk_tol; a value above 1 hands every block to the column passes).
  struct GramBufs {
    double *part = nullptr, *sum = nullptr, *w = nullptr;
    ~GramBufs() {
      for (double *p : {part, sum, w})
        if (p) hipFree(p);
    }
  } gb;
  bool gram_on = [] {
    const char *e = std::getenv("MIGMRES_FB_GRAM");
    return !(e && e[0] == '0');
  }();
  bool gram_fuse = [] {
    const char *e = std::getenv("MIGMRES_FB_GRAM_FUSE");
    return !(e && e[0] == '0');
  }();
  double gram_gate = [] {
    const char *e = std::getenv("MIGMRES_FB_GRAM_GATE");
    return e ? std::atof(e) : 0.0;
  }();
  long long gram_calls = 0, gram_skips = 0, gram_singles = 0, gram_mixed = 0;

  ~FastIcgs() { release(); }
  void release() {
    if (ctx) hipStreamSynchronize(ctx->stream);
    for (void *p : {(void *)partial, (void *)R1, (void *)R2, (void *)cout_own, (void *)red, (void *)S, (void *)stb[0],
                    (void *)stb[1], (void *)sink, (void *)pbuf[1]})
      if (p) hipFree(p);
    if (ev_fetch) hipEventDestroy(ev_fetch);
    ev_fetch = nullptr;
    stb[0] = stb[1] = nullptr;
    pbuf[0] = pbuf[1] = nullptr;
    pend = Pending{};
    if (h) hipHostFree(h);
    partial = R1 = R2 = Cout = cout_own = red = S = sink = nullptr;
    st = nullptr;
    h = nullptr;
    tmpX.reset();
  }

  bool supports(int k) const { return k >= 1 && k <= 16; }

  void setup(migmres_ctx *c, long long ng, int nl, int k, int lmax) {
    if (ctx == c && n_local == nl && n_global == ng && k <= kmax && lmax <= Lmax) return;
    release();
    ctx = c;
    n_global = ng;
    n_local = nl;
    kmax = k;
    Lmax = lmax;
    nblk_tn = gemm_tn_blocks(nl);
    nblk_ic = icgs_blocks(nl);
    for (auto &row : nt_cache)
      for (int &v : row) v = 0;
    const char *nf = std::getenv("MIGMRES_NO_FUSED_NN_TN");
    use_fused = !(nf && nf[0] == '1');
    const char *fr = std::getenv("MIGMRES_FB_REV");
    fb_rev = !(fr && fr[0] == '0');
    const char *xs = std::getenv("MIGMRES_NN_TN_STORE");
    x1_store = xs && xs[0] == '1';
    size_t np = std::max({(size_t)nblk_tn * 512 * 16, (size_t)nblk_ic * 17,
                          (size_t)nn_tn_blocks(nl, 16, 1) * 256 * 16,
                          (size_t)1024 * (size_t)std::min(lmax, 1024) * 8});  // wide nn_tn halves
    for (int L = 64; L <= std::min(lmax, 512); L += 16)  // k = 16 in one workgroup (16- or 32-row chunks)
      if (nn_tn_supported(L, 16)) np = std::max(np, (size_t)nn_tn_blocks(nl, L, 16) * L * 16);
    MIG_HIP(hipMalloc(&partial, sizeof(double) * np));
    MIG_HIP(hipMalloc(&R1, sizeof(double) * (size_t)(lmax + k) * k));
    MIG_HIP(hipMalloc(&R2, sizeof(double) * (size_t)(lmax + k) * k));
    MIG_HIP(hipMalloc(&Cout, sizeof(double) * (size_t)(lmax + k) * k));
    cout_own = Cout;
    MIG_HIP(hipMalloc(&red, sizeof(double) * 64));
    // any nn_tn grid: at most 2048 workgroup-slots of 1024 threads' worth of lanes
    MIG_HIP(hipMalloc(&sink, sizeof(double) * 1024 * 2048));
    const size_t sbytes = sizeof(double) * ((size_t)(nl > 0 ? nl : 1) + 64);
    MIG_HIP(hipMalloc(&S, sbytes));
    MIG_HIP(hipMemset(S, 0, sbytes));  // zero padding row read by the row-pair kernels
    MIG_HIP(hipEventCreateWithFlags(&ev_fetch, hipEventDisableTiming));
    // each state buffer carries a coefficient block behind it, so the block iteration's one D2H
    // copy takes the state and the coefficients C together (fetch) when Cout sits behind st
    for (int i = 0; i < 2; ++i)
      MIG_HIP(hipMalloc(&stb[i], sizeof(IcgsState) + sizeof(double) * (size_t)(lmax + k) * k));
    st = stb[0];
    pbuf[0] = partial;
    MIG_HIP(hipMalloc(&pbuf[1], sizeof(double) * (size_t)nblk_ic * 17));
    MIG_HIP(hipHostMalloc(&h, sizeof(IcgsState) + sizeof(double) * (size_t)(lmax + k) * k, hipHostMallocDefault));
  }

  void allreduce(double *d, size_t n) {
    if (!ctx->dist || n == 0) return;
    ctx->allreduce_async(d, n);
  }

  // Prologue for the next pass: the pending step (if any), reading the current state and
  // writing the other buffer, which becomes current.
  FbPro take_pending() {
    FbPro p{};
    p.in = st;
    p.stage0 = p.stage1 = -1;
    if (!pend.on) return p;
    IcgsState *other = st == stb[0] ? stb[1] : stb[0];
    p.partial = pend.partial;
    p.red = red;
    p.nblocks = nblk_ic;
    p.nv = pend.nv;
    p.stage0 = pend.s0;
    p.stage1 = pend.s1;
    p.j = pend.j;
    p.k = pend.k;
    p.complete = pend.complete;
    p.out = other;
    st = other;
    pend.on = false;
    return p;
  }
  // Partials buffer for a pass that may itself read the pending partials in its prologue.
  double *next_partial() const { return pend.on && pend.partial == pbuf[0] ? pbuf[1] : pbuf[0]; }
  // After a pass that wrote nv partials per workgroup to `pp`: its reduction and scalar
  // stage(s) become pending.  On several ranks the partials are reduced and all-reduced now
  // (the next prologue reads `red`).
  void set_pending(double *pp, int nv, int s0, int s1, int j, int k, int complete) {
    pend.on = true;
    pend.partial = pp;
    pend.nv = nv;
    pend.s0 = s0;
    pend.s1 = s1;
    pend.j = j;
    pend.k = k;
    pend.complete = complete;
    if (ctx->dist) {
      ProfScope ps(ctx, K_REDUCE, 8.0 * nblk_ic * nv);
      launch_reduce_small(ctx->stream, pp, nblk_ic, nv, red);
      allreduce(red, (size_t)nv);
      pend.partial = nullptr;
    }
  }
  // Apply a pending step with no pass after it.
  void flush_pending() {
    if (!pend.on) return;
    const FbPro p = take_pending();
    launch_fb_flush(ctx->stream, p);
  }

  // out (L x kb, leading dim ldo) = A^T B, summed over ranks.
  void tn(const MvDesc &A, int L, const MvDesc &B, int kb, double *out, int ldo) {
    for (int a0 = 0; a0 < L; a0 += 512) {
      const int lc = std::min(512, L - a0);
      MvDesc Ac = A;
      Ac.ncols = lc;
      if (A.cols)
        Ac.cols = A.cols + a0;
      else
        Ac.base = A.base + (long long)a0 * A.ld;
      const int nb = gemm_tn_blocks(n_local, lc);  // <= nblk_tn (the partials buffer's rows)
      {
        ProfScope ps(ctx, K_GEMM_TN, 8.0 * n_local * (lc + kb) + 8.0 * nb * lc * kb);
        launch_gemm_tn_partial(ctx->stream, Ac, lc, B, kb, n_local, partial, nb);
      }
      ProfScope ps(ctx, K_REDUCE, 8.0 * nb * lc * kb);
      launch_reduce_partials_ld(ctx->stream, partial, nb, lc, kb, ldo, 1.0, out + a0);
    }
    if (ldo == L) allreduce(out, (size_t)L * kb);
  }

  // dot: 0 none, 1 column self dots, 3 self dots + <X_0, X_1>
  void nn(const MvDesc &Q, int L, const double *M, int ldm, const MvDesc &X, int k, int dot) {
    if (!dot) {
      ProfScope ps(ctx, K_GEMM_NN, 8.0 * n_local * (L + 2.0 * k));
      launch_gemm_nn(ctx->stream, Q, L, M, ldm, X, n_local, -1.0, 1.0);
      return;
    }
    flush_pending();
    ProfScope ps(ctx, K_GEMM_NN_DOT, 8.0 * n_local * (L + 2.0 * k));
    launch_gemm_nn_dot(ctx->stream, Q, L, M, ldm, X, n_local, -1.0, 1.0, dot, X, pbuf[0], nblk_ic);
  }

  // X1 = X - Q C1 (C1 leading dim ldc1) then out = Q^T X1, summed over ranks: one fused pass
  // over Q when the shape allows it, else MvTimesMatAddMv followed by MvTransMv.  Returns
  // whether X now holds X1.  The fused pass leaves X unchanged unless x1_store is set: the
  // caller's closing update then forms X - Q (C1 + C2) from the original X, so the pass is
  // read-only (a k-column write in a read stream costs far more than its bytes:
  // tools/mb_rw.hip, 6.2 TB/s read-only against 5.0 TB/s with the write at L = 104).
  bool nn_then_tn(const MvDesc &Q, int L, const double *C1, int ldc1, const MvDesc &X, int k, double *out) {
    // Measured at 256^3, k = 8 (tools/mb_lib.cpp): the fused kernel beats the two streaming
    // kernels from L = 16 on (1.3 vs 1.4 ms at L = 16, 9.0 vs 10.5 ms at L = 200).
    const bool fused_wins = L >= 16;
    // k > 8 (L >= 64): both 8-column halves of X in one launch of the wide fused kernel, the
    // two workgroups of a chunk range on one XCD (Q from HBM once; each column of X1 and of
    // C2 depends on its own column of X and C1 only, so the halves are the same arithmetic);
    // the narrow kernel ran at 1.65 TB/s at k = 16
    if (use_fused && !Q.cols && k > 8 && !x1_store && L >= 64 && nn_tn_supported(L, k)) {
      const int nb = nt_blocks(L, k);
      {
        ProfScope ps(ctx, K_NN_TN, 8.0 * n_local * (L + k) + 8.0 * nb / 2 * L * k);
        launch_nn_tn(ctx->stream, Q, L, C1, ldc1, X, n_local, partial, nb, sink, false);
      }
      ProfScope ps(ctx, K_REDUCE, 8.0 * nb / 2 * L * k);
      if (nn_tn_paired(L, k)) {
        launch_reduce_partials_ld(ctx->stream, partial, nb / 2, L, 8, L, 1.0, out);
        launch_reduce_partials_ld(ctx->stream, partial + (size_t)(nb / 2) * L * 8, nb / 2, L, k - 8, L, 1.0,
                                  out + (size_t)8 * L);
      } else {
        launch_reduce_partials_ld(ctx->stream, partial, nb, L, k, L, 1.0, out);
      }
      allreduce(out, (size_t)L * k);
      return false;
    }
    if (use_fused && fused_wins && !Q.cols && nn_tn_supported(L, k)) {
      const int nb = nt_blocks(L, k);
      {
        ProfScope ps(ctx, K_NN_TN, 8.0 * n_local * (L + (x1_store ? 2.0 : 1.0) * k) + 8.0 * nb * L * k);
        launch_nn_tn(ctx->stream, Q, L, C1, ldc1, X, n_local, partial, nb, sink, x1_store);
      }
      {
        ProfScope ps(ctx, K_REDUCE, 8.0 * nb * L * k);
        launch_reduce_partials_ld(ctx->stream, partial, nb, L, k, L, 1.0, out);
      }
      allreduce(out, (size_t)L * k);
      return x1_store;
    }
    nn(Q, L, C1, ldc1, X, k, 0);
    tn(Q, L, X, k, out, L);
    return true;
  }

  int nt_blocks(int L, int k) {
    int &v = nt_cache[L][(k + 3) / 4 - 1];
    if (v == 0) v = nn_tn_blocks(n_local, L, k);
    return v;
  }

  // head_ready: the closing update of blkOrtho (k_gemm_nn_dot dmode 3) left its partials
  // [<X_0,X_0>, <X_1,X_1>, ..., <X_0,X_1> at k] pending with the dependency test (stage 3);
  // the first pass applies that and the findBasis head (stage 7) in its prologue, so the
  // a01 pass is skipped.
  void find_basis(const MvDesc &X, int k, int complete, bool head_ready = false) {
    const double n = (double)n_local;
    if (k == 1) {
      {
        ProfScope ps(ctx, K_FB, 8.0 * n);
        double *pp = next_partial();
        const FbPro pro = take_pending();
        launch_fb_a(ctx->stream, X, 0, pro, n_local, pp, nblk_ic);
        set_pending(pp, 1, 0, -1, 0, k, complete);
      }
    } else {
      if (head_ready) {
        pend.s1 = 7;  // after stage 3 (set by the closing update)
        pend.complete = complete;
      } else {
        flush_pending();
        ProfScope ps(ctx, K_FB, 16.0 * n);
        launch_fb_a01(ctx->stream, X, n_local, pbuf[0], nblk_ic);
        set_pending(pbuf[0], 3, 5, -1, 0, k, complete);
      }
      for (int j = 1; j < k; ++j) {
        {
          ProfScope ps(ctx, K_FB, 8.0 * n * (j + 1));
          double *pp = next_partial();
          const FbPro pro = take_pending();
          launch_fb_b2(ctx->stream, X, j, pro, n_local, pp, nblk_ic, fb_rev);
          set_pending(pp, j + 1, 1, -1, j, k, complete);
        }
        const int has_next = j + 1 < k;
        {
          ProfScope ps(ctx, K_FB, 8.0 * n * (j + 3 + has_next));
          double *pp = next_partial();
          const FbPro pro = take_pending();
          launch_fb_ca(ctx->stream, X, j, has_next, pro, n_local, pp, nblk_ic, 0);
          set_pending(pp, has_next ? j + 3 : 1, 6, -1, j, k, complete);
        }
      }
    }
    ProfScope ps(ctx, K_SCALE, 16.0 * n);
    const FbPro pro = take_pending();
    launch_scale_col(ctx->stream, X, k - 1, pro, n_local, nblk_ic);
  }

  bool gram_ok(int L, int k) const {
    // k <= 8: the closing update carries G1's partials (its LDS holds L x k coefficients);
    // 9 <= k <= 16: plain closing update, then G1 in a pass of its own (MFMA Gram kernels).
    // DGKS (the Belos default) takes it with its own decisions: for k > 1 its blkOrtho is
    // ICGS's (both passes, BelosDGKSOrthoManager.hpp:1373-1492), and its findBasis projects each
    // column once and a second time only if sqrt|newDot| < dep_tol sqrt|oldDot| after the first
    // (:1094-1119).  The first pass's newDot / oldDot of column j are the Cholesky pivot ratio
    // R1_jj^2 / G1_jj, so k_fbg_chol takes DGKS's decision per column on it: no column asks a
    // second projection -> CholQR1 (X T1, B = R1: one Gram-Schmidt pass per column, as DGKS);
    // every column j >= 1 asks it -> CholQR2 (two passes, as DGKS); some do -> the column passes
    // on the block, which decide column by column.  The dependency test newDot < blk_tol
    // oldDot (:1204-1210) is taken on the pivots as for ICGS.  MIGMRES_FB_GRAM_DGKS=0 keeps
    // DGKS on the column passes.
    return gram_on && (!slow->dgks || gram_dgks) && slow->steps == 2 && k >= 2 && L >= 1 && L <= 1024 &&
           ((k <= 8 && L * k <= 7680) || (k > 8 && k <= 16));
  }
  // MIGMRES_FBG_PRO=0: k <= 8 takes the k x k steps in one-workgroup launches (k_fbg_chol)
  bool fbg_pro = [] {
    const char *e = std::getenv("MIGMRES_FBG_PRO");
    return !(e && e[0] == '0');
  }();
  // MIGMRES_FOLD_SMALL=0: the state reset, blk_old and C1 + C2 as separate launches
  bool fold_small = [] {
    const char *e = std::getenv("MIGMRES_FOLD_SMALL");
    return !(e && e[0] == '0');
  }();
  bool gram_dgks = [] {
    const char *e = std::getenv("MIGMRES_FB_GRAM_DGKS");
    return !(e && e[0] == '0');
  }();
  void gram_alloc() {
    if (gb.part) return;
    MIG_HIP(hipMalloc(&gb.part, sizeof(double) * 1024 * 136));
    MIG_HIP(hipMalloc(&gb.sum, sizeof(double) * 272));
    MIG_HIP(hipMalloc(&gb.w, sizeof(double) * 768));
  }
  // findBasis in Gram form (icgs.hip): CholQR2 of the block with the reference's dependency
  // tests on its pivots.  nb1: rows of G1 partials the closing update (k_gemm_nn_gram) left
  // in gb.part, 0 to take G1 in a pass of its own.
  void find_basis_gram(const MvDesc &X, int k, int nb1) {
    ++gram_calls;
    const int nv = k * (k + 1) / 2;
    const double n = (double)n_local;
    const double gate = gram_gate > 0.0 ? gram_gate : 100.0 * slow->blk_tol;
    auto chol = [&](int stage, int nb) {
      ProfScope ps(ctx, K_REDUCE, 8.0 * nb * nv);
      if (k > 8) {  // block-major partials: fixed-order sum, all-reduce, the k x k step
        launch_reduce_partials(ctx->stream, gb.part, nb, nv, 1.0, gb.sum);
        allreduce(gb.sum, (size_t)nv);
        launch_fbg_chol_l(ctx->stream, gb.sum, k, stage, st, gb.w, gate);
      } else if (ctx->dist) {
        launch_fbg_chol(ctx->stream, gb.part, nb, k, 0, st, gb.w, gate, gb.sum);
        allreduce(gb.sum, (size_t)nv);
        launch_fbg_chol(ctx->stream, gb.sum, 1, k, stage, st, gb.w, gate, nullptr);
      } else {
        launch_fbg_chol(ctx->stream, gb.part, nb, k, stage, st, gb.w, gate, nullptr);
      }
    };
    const int rev = nb1 ? 1 : 0;  // sweep directions alternate from pass to pass
    if (k <= 8 && fbg_pro) {
      // the k x k steps in the passes' prologues: sum (+ all-reduce) -> pass -> sum -> pass
      if (!nb1) {
        ProfScope ps(ctx, K_FB, 8.0 * n * k);
        nb1 = launch_fbg_gram(ctx->stream, X, k, n_local, gb.part, 1);
      }
      double *s1 = gb.sum, *s2 = gb.sum + 136;
      {
        ProfScope ps(ctx, K_REDUCE, 8.0 * nb1 * nv);
        launch_gram_sum(ctx->stream, gb.part, nb1, k, s1);
        allreduce(s1, (size_t)nv);
      }
      int nb2;
      {
        ProfScope ps(ctx, K_FB, 8.0 * n * k);
        nb2 = launch_fbg_a_p(ctx->stream, X, k, n_local, st, gb.w, s1, gate, gb.part, rev);
      }
      {
        ProfScope ps(ctx, K_REDUCE, 8.0 * nb2 * nv);
        launch_gram_sum(ctx->stream, gb.part, nb2, k, s2);
        allreduce(s2, (size_t)nv);
      }
      ProfScope ps(ctx, K_FB, 16.0 * n * k);
      launch_fbg_b_p(ctx->stream, X, k, n_local, st, gb.w, s2, gate, 1 - rev);
      return;
    }
    if (!nb1) {
      ProfScope ps(ctx, K_FB, 8.0 * n * k);
      nb1 = launch_fbg_gram(ctx->stream, X, k, n_local, gb.part, 1);
    }
    chol(1, nb1);
    int nb2;
    {
      ProfScope ps(ctx, K_FB, 8.0 * n * k);
      nb2 = launch_fbg_a(ctx->stream, X, k, n_local, st, gb.w, gb.part, rev);
    }
    chol(2, nb2);
    ProfScope ps(ctx, K_FB, 16.0 * n * k);
    launch_fbg_b(ctx->stream, X, k, n_local, st, gb.w, 1 - rev);
  }

  void fetch(int L, int k) {
    flush_pending();
    if (L > 0 && Cout == (double *)(st + 1)) {  // one copy: the state and C behind it
      MIG_HIP(hipMemcpyAsync(h, st, sizeof(IcgsState) + sizeof(double) * (size_t)L * k, hipMemcpyDeviceToHost,
                             ctx->stream));
    } else {
      MIG_HIP(hipMemcpyAsync(h, st, sizeof(IcgsState), hipMemcpyDeviceToHost, ctx->stream));
      if (L > 0)
        MIG_HIP(hipMemcpyAsync(h + sizeof(IcgsState) / sizeof(double), Cout, sizeof(double) * (size_t)L * k,
                               hipMemcpyDeviceToHost, ctx->stream));
    }
    if (before_wait) {
      MIG_HIP(hipEventRecord(ev_fetch, ctx->stream));
      before_wait();
      MIG_HIP(hipEventSynchronize(ev_fetch));
    } else {
      MIG_HIP(hipStreamSynchronize(ctx->stream));
    }
  }
  const IcgsState &hst() const { return *reinterpret_cast<const IcgsState *>(h); }
  const double *hC() const { return h + sizeof(IcgsState) / sizeof(double); }

  void save_input(migmres_mv &X) {
    if (!tmpX.p) tmpX = MvPtr(mv_create(ctx, n_global, n_local, kmax));  // first use
    ProfScope ps(ctx, K_COPY, 16.0 * n_local * X.ncols);
    MvPtr t = view(*tmpX, 0, X.ncols);
    launch_copy(ctx->stream, X.desc(), t->desc(), n_local);
  }
  void restore_input(migmres_mv &X) {
    MvPtr t = view(*tmpX, 0, X.ncols);
    launch_copy(ctx->stream, t->desc(), X.desc(), n_local);
  }

  // projectAndNormalize(X, [C], B, [Q]).  The reference keeps a copy of X (tmpX) to restart
  // from when a dependency is found; when the caller can recompute X exactly (regen: the
  // same deterministic SpMM that produced it, not counted as an operator application) no
  // copy is made.
  int project_and_normalize(migmres_mv &X, migmres_mv &Q, double *C, int ldc, double *B, int ldb,
                            const std::function<void()> *regen = nullptr) {
    const int k = X.ncols, L = Q.ncols;
    // DGKS blkOrtho1 decides its second pass on a dot product between the passes: host path
    if (k == 1 && slow->dgks) return slow->project_and_normalize(X, Q, C, ldc, B, ldb);
    ++calls;
    pend = Pending{};
    Cout = cout_own;
    const MvDesc xd = X.desc(), qd = Q.desc();
    if (k == 1) {  // blkOrtho1, then MvDot and MvScale
      launch_state_reset(ctx->stream, st, slow->blk_tol, slow->sing_tol, slow->dgks ? 1 : 0, slow->dep_tol);
      enqueue_k1(X, Q);
      fetch(L, 1);
      return result_k1(L, C, B);
    }
    if (!regen) save_input(X);
    // blkOrtho: oldDot comes from the Gram block of [Q X]^T X when Q and X are adjacent
    const bool adjacent = Q.contiguous() && X.contiguous() && Q.ld == X.ld && X.base == Q.base + (long long)L * Q.ld;
    if (adjacent) {
      MvDesc qx = qd;
      qx.ncols = L + k;
      tn(qx, L + k, xd, k, R1, L + k);
    } else {
      tn(qd, L, xd, k, R1, L + k);
      tn(xd, k, xd, k, R1 + L, L + k);
      allreduce(R1, (size_t)(L + k) * k);
    }
    // The state is first read by blk_old (or by the closing update's prologue, which then takes
    // the reset, blk_old and the coefficient sum C1 + C2 in its workgroup 0: no kernel between
    // the passes reads it).
    const bool x1 = nn_then_tn(qd, L, R1, L + k, xd, k, R2);
    const bool gram = gram_ok(L, k);
    // the Gram path takes no pending steps (st stays put): C goes behind st, one D2H copy
    Cout = gram ? (double *)(st + 1) : cout_own;
    const bool fold = gram && gram_fuse && k <= 8 && !x1 && fold_small;
    if (!fold) {
      launch_state_reset(ctx->stream, st, slow->blk_tol, slow->sing_tol, slow->dgks ? 1 : 0, slow->dep_tol);
      launch_blk_old(ctx->stream, st, R1, L + k, L, k);
      launch_add_coef(ctx->stream, R1, L + k, R2, L, Cout, L, L, k);
    }
    // X2 = X1 - Q C2 (reference order) when X holds X1, else X - Q (C1 + C2)
    const double *M2 = x1 ? R2 : Cout;
    if (gram) {
      gram_alloc();
      flush_pending();
      int nb1 = 0;
      {
        ProfScope ps(ctx, K_GEMM_NN_DOT, 8.0 * n_local * (L + 2.0 * k));
        if (fold) {
          NngPro pro;
          pro.C1 = R1;
          pro.ld1 = L + k;
          pro.C2 = R2;
          pro.ld2 = L;
          pro.cout = Cout;
          pro.ldo = L;
          pro.st = st;
          pro.G = R1;
          pro.ldg = L + k;
          pro.dgks = slow->dgks ? 1 : 0;
          pro.blk_tol = slow->blk_tol;
          pro.sing_tol = slow->sing_tol;
          pro.dep_tol = slow->dep_tol;
          nb1 = launch_gemm_nn_gram(ctx->stream, qd, L, nullptr, L, xd, n_local, gb.part, pro);
        } else if (gram_fuse && k <= 8)
          nb1 = launch_gemm_nn_gram(ctx->stream, qd, L, M2, L, xd, n_local, gb.part);
        else
          launch_gemm_nn(ctx->stream, qd, L, M2, L, xd, n_local, -1.0, 1.0);
      }
      find_basis_gram(xd, k, nb1);
    } else {
      nn(qd, L, M2, L, xd, k, 3);
      set_pending(pbuf[0], k + 1, 3, -1, 0, k, 0);
      find_basis(xd, k, 0, true);
    }
    fetch(L, k);
    if (hst().neg != 0.0) throw Error(MIGMRES_ESTATE, "ICGS: negative definiteness in inner product");
    if (gram && hst().gram_single) ++gram_singles;
    if (gram && hst().gram_mixed) ++gram_mixed;
    if (gram && hst().dep == 0.0 && hst().gram_skip) {
      // a column too close to the span of the others for the Gram form: the column passes on
      // the block, which the skipped passes left holding X2
      ++gram_skips;
      ++fallbacks;  // not the final block when the speculative SpMM (if any) read it
      before_wait = nullptr;
      find_basis(xd, k, 0, false);
      fetch(L, k);
      if (hst().neg != 0.0) throw Error(MIGMRES_ESTATE, "ICGS: negative definiteness in inner product");
    }
    const IcgsState &s = hst();
    if (s.dep != 0.0 || s.failed >= 0) {
      ++fallbacks;
      if (regen)
        (*regen)();
      else
        restore_input(X);
      const int rank = slow->blk_ortho_sing(X, Q, C, ldc, B, ldb);
      MIG_HIP(hipStreamSynchronize(ctx->stream));
      return rank;
    }
    for (int j = 0; j < k; ++j) {
      for (int i = 0; i < L; ++i) C[i + (size_t)j * ldc] = hC()[i + (size_t)j * L];
      for (int i = 0; i < k; ++i) B[i + (size_t)j * ldb] = s.B[i + 16 * j];
    }
    return k;
  }

  // The k == 1 projectAndNormalize as a kernel chain ending in the D2H copy of the state
  // and coefficients, without the wait: PseudoBlockGmres enqueues every right-hand side's
  // chain (one FastIcgs each) and waits once (fetch_async / result_k1).
  void enqueue_k1(migmres_mv &X, migmres_mv &Q) {
    const int L = Q.ncols;
    Cout = cout_own;
    ++calls;
    pend = Pending{};
    launch_state_reset(ctx->stream, st, slow->blk_tol, slow->sing_tol, slow->dgks ? 1 : 0, slow->dep_tol);
    const MvDesc xd = X.desc(), qd = Q.desc();
    tn(qd, L, xd, 1, R1, L);
    const bool x1 = nn_then_tn(qd, L, R1, L, xd, 1, R2);
    launch_add_coef(ctx->stream, R1, L, R2, L, Cout, L, L, 1);
    nn(qd, L, x1 ? R2 : Cout, L, xd, 1, 1);
    set_pending(pbuf[0], 1, 4, -1, 0, 1, 0);
    ProfScope ps(ctx, K_SCALE, 16.0 * n_local);
    const FbPro pro = take_pending();
    launch_scale_col(ctx->stream, xd, 0, pro, n_local, nblk_ic);
  }
  void fetch_async(int L, int k) {
    flush_pending();
    MIG_HIP(hipMemcpyAsync(h, st, sizeof(IcgsState), hipMemcpyDeviceToHost, ctx->stream));
    if (L > 0)
      MIG_HIP(hipMemcpyAsync(h + sizeof(IcgsState) / sizeof(double), Cout, sizeof(double) * (size_t)L * k,
                             hipMemcpyDeviceToHost, ctx->stream));
  }
  int result_k1(int L, double *C, double *B) const {
    for (int i = 0; i < L; ++i) C[i] = hC()[i];
    B[0] = hst().B[0];
    return 1;
  }

  // normalize = findBasis(completeBasis = true)
  int normalize(migmres_mv &X, double *B, int ldb) {
    ++calls;
    const int k = X.ncols;
    pend = Pending{};
    launch_state_reset(ctx->stream, st, slow->blk_tol, slow->sing_tol, slow->dgks ? 1 : 0, slow->dep_tol);
    save_input(X);
    find_basis(X.desc(), k, 1);
    fetch(0, k);
    const IcgsState &s = hst();
    if (s.neg != 0.0) throw Error(MIGMRES_ESTATE, "ICGS: negative definiteness in inner product");
    if (s.failed >= 0) {
      ++fallbacks;
      restore_input(X);
      const int rank = slow->normalize(X, B, ldb);
      MIG_HIP(hipStreamSynchronize(ctx->stream));
      return rank;
    }
    for (int j = 0; j < k; ++j)
      for (int i = 0; i < k; ++i) B[i + (size_t)j * ldb] = s.B[i + 16 * j];
    return k;
  }
};

// ------------------------------------------------------------------------------------
// Small dense helpers (Teuchos::BLAS semantics, column-major)
// ------------------------------------------------------------------------------------
void rotg(double &a, double &b, double &c, double &s) {
  const double roe = std::fabs(a) > std::fabs(b) ? a : b;
  const double scale = std::fabs(a) + std::fabs(b);
  if (scale == 0.0) {
    c = 1.0;
    s = 0.0;
    a = 0.0;
    b = 0.0;
    return;
  }
  double r = scale * std::sqrt((a / scale) * (a / scale) + (b / scale) * (b / scale));
  r = std::copysign(1.0, roe) * r;
  c = a / r;
  s = b / r;
  double z = 1.0;
  if (std::fabs(a) > std::fabs(b)) z = s;
  if (std::fabs(b) >= std::fabs(a) && c != 0.0) z = 1.0 / c;
  a = r;
  b = z;
}

struct Params {
  double tol = 1e-8;
  int max_restarts = 20;
  int max_iters = 1000;
  int num_blocks = 300;
  int block_size = 1;
  bool adaptive = true;
  bool flexible = false;
  bool exp_res_test = false;
  bool pseudo = false;  // PseudoBlockGmresSolMgr instead of BlockGmresSolMgr
  int def_quorum = 1;   // "Deflation Quorum" (pseudo-block only)
  std::string ortho = "DGKS";
  std::string imp_scale = "Norm of Preconditioned Initial Residual";
  std::string exp_scale = "Norm of Initial Residual";
  int verbosity = 0;
  int output_freq = -1;
  // recorded and reported, no effect on the device path (BelosBlockGmresSolMgr.hpp:459-486)
  std::string timer_label = "Belos";
  int output_style = 0;  // Belos::General
  bool show_max_res_norm_only = false;
  // "Orthogonalization Constant": DGKS's dep_tol when > 0 (BelosBlockGmresSolMgr.hpp:607-625)
  double ortho_kappa = -1.0;
  double dgks_dep_tol() const { return ortho_kappa > 0 ? ortho_kappa : 1.0 / std::sqrt(2.0); }
};

}  // namespace

// ------------------------------------------------------------------------------------
// Solver state
// ------------------------------------------------------------------------------------
struct migmres_solver {
  migmres_ctx *ctx = nullptr;
  Params p;
  migmres_prec *left = nullptr, *right = nullptr;  // borrowed (setLeftPrec / setRightPrec)
  std::unique_ptr<migmres_prec> uprec[2];  // wrappers of user-operator preconditioners (set_prec_op)
  Icgs ortho;
  FastIcgs fast;
  bool use_fast = true;
  // results
  int num_iters = 0;
  double achieved_tol = 0.0;
  bool loa = false;
  std::vector<double> history;
  int hist_cols = 0;
  // setUserConvStatusTest (pseudo-block only)
  migmres_status_fn user_test = nullptr;
  void *user_data = nullptr;
  int user_combo = MIGMRES_COMBO_SEQ;
  long long n_apply = 0, n_explicit = 0, n_restarts = 0, n_block_iters = 0, n_prec = 0, n_deflations = 0;
  double t_total = 0, t_spmm = 0, t_ortho = 0, t_lsq = 0, t_comm = 0;
  double t_check = 0, t_restart = 0, t_setup = 0;
  bool sync_timers() const { return (p.verbosity & 1) != 0; }
};

namespace {

using Clock = std::chrono::steady_clock;
double since(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }

// LinearProblem (BelosLinearProblem.hpp) with optional left/right preconditioners.
struct Problem {
  migmres_solver *S;
  migmres_crs *A;              // the operator as a CRS, or null when it is a user operator:
  migmres_op *Aop = nullptr;   // y = op(x) through its callback
  migmres_mv *X, *B;
  migmres_prec *LP = nullptr, *RP = nullptr;
  MvPtr R0, PR0;  // PR0 empty: PR0 == R0 (no left preconditioner)
  MvPtr tmp;      // scratch of apply()
  std::vector<int> ls_idx, cur;
  int ls_num = 0;
  MvPtr curX, curB;

  migmres_mv &pr0() { return PR0.p ? *PR0 : *R0; }
  MvPtr clone(int k) { return MvPtr(mv_create(X->ctx, X->n_global, X->n_local, k)); }
  migmres_mv &scratch(int k) {
    if (!tmp.p || tmp->ncols != k) tmp = clone(k);
    return *tmp;
  }
  void op_raw(const migmres_mv &x, migmres_mv &y) {  // uncounted
    if (A)
      crs_apply(*A, x, y, 1.0, 0.0);
    else
      op_apply(*Aop, x, y);
  }
  void op(const migmres_mv &x, migmres_mv &y) {  // OPT::Apply(A)
    auto t0 = Clock::now();
    op_raw(x, y);
    ++S->n_apply;
    if (S->p.verbosity & 1) {
      MIG_HIP(hipStreamSynchronize(X->ctx->stream));
      S->t_spmm += since(t0);
    }
  }
  // every operator is the library's own (CRS, Jacobi, Chebyshev): it may be re-applied to
  // regenerate a block, or applied ahead of need
  bool own_ops() const { return A && !(LP && LP->kind == 2) && !(RP && RP->kind == 2); }
  void prec(migmres_prec &M, const migmres_mv &x, migmres_mv &y) {
    prec_apply(M, x, y);
    ++S->n_prec;
  }
  // apply (BelosLinearProblem.hpp:989-1072): y = M_L A M_R x
  void apply(const migmres_mv &x, migmres_mv &y) {
    if (!LP && !RP) {
      op(x, y);
    } else if (LP && RP) {
      migmres_mv &t = scratch(y.ncols);
      prec(*RP, x, y);
      op(y, t);
      prec(*LP, t, y);
    } else if (LP) {
      migmres_mv &t = scratch(y.ncols);
      op(x, t);
      prec(*LP, t, y);
    } else {
      // right Jacobi fused into the template SpMM where the operator allows it (one launch,
      // no M x round trip through HBM; same bits); MIGMRES_NO_FUSED_JACOBI=1 disables
      const auto t0 = Clock::now();
      if (fuse_jacobi && A && crs_apply_jacobi_fused(*A, *RP, x, y)) {
        ++RP->n_apply;
        ++S->n_prec;
        ++S->n_apply;
        if (S->p.verbosity & 1) {  // same phase accounting as op()
          MIG_HIP(hipStreamSynchronize(A->ctx->stream));
          S->t_spmm += since(t0);
        }
        return;
      }
      migmres_mv &t = scratch(y.ncols);
      prec(*RP, x, t);
      op(t, y);
    }
  }
  const bool fuse_jacobi = [] {
    const char *e = std::getenv("MIGMRES_NO_FUSED_JACOBI");
    return !(e && e[0] == '1');
  }();
  // applyRightPrec (BelosLinearProblem.hpp:1103-1114)
  void apply_right_prec(const migmres_mv &x, migmres_mv &y) {
    if (RP)
      prec(*RP, x, y);
    else
      mv_add_mv(1.0, x, 0.0, x, y);
  }
  void set_problem() {  // setProblem (BelosLinearProblem.hpp:836-946)
    R0 = clone(X->ncols);
    op(*X, *R0);
    mv_add_mv(-1.0, *R0, 1.0, *B, *R0);
    PR0.reset();
    if (LP) {
      PR0 = clone(X->ncols);
      prec(*LP, *R0, *PR0);
    }
  }
  unsigned int aug_seed = 20250219u;  // MvRandom stream for augmented right-hand sides
  std::vector<int> vld, newi;
  bool augmented = false;

  // setLSIndex (BelosLinearProblem.hpp:642-705): a block with -1 entries is augmented --
  // curX = zeros and curB = random with the valid columns copied in (SetBlock).
  void set_ls_index(const std::vector<int> &idx) {
    ls_idx = idx;
    ++ls_num;
    cur.clear();
    vld.clear();
    newi.clear();
    for (size_t j = 0; j < idx.size(); ++j)
      if (idx[j] >= 0) {
        cur.push_back(idx[j]);
        vld.push_back(idx[j]);
        newi.push_back((int)j);
      }
    const int bs = (int)idx.size();
    augmented = (int)vld.size() != bs;
    if (augmented) {
      curX = MvPtr(mv_create(X->ctx, X->n_global, X->n_local, bs));
      mv_init(*curX, 0.0);
      curB = MvPtr(mv_create(B->ctx, B->n_global, B->n_local, bs));
      mv_random(*curB, &aug_seed);
      MvPtr bsrc(mv_view(B, vld.data(), (int)vld.size()));
      MvPtr bdst(mv_view(curB.p, newi.data(), (int)newi.size()));
      mv_assign(*bsrc, *bdst);
      MvPtr xsrc(mv_view(X, vld.data(), (int)vld.size()));
      MvPtr xdst(mv_view(curX.p, newi.data(), (int)newi.size()));
      mv_assign(*xsrc, *xdst);
      MIG_HIP(hipStreamSynchronize(X->ctx->stream));
    } else {
      curX = MvPtr(mv_view(X, cur.data(), (int)cur.size()));
      curB = MvPtr(mv_view(B, cur.data(), (int)cur.size()));
    }
  }
  // setCurrLS (BelosLinearProblem.hpp:709-739)
  void set_curr_ls() {
    if (!augmented) return;
    MvPtr src(mv_view(curX.p, newi.data(), (int)newi.size()));
    MvPtr dst(mv_view(X, vld.data(), (int)vld.size()));
    mv_assign(*src, *dst);
    MIG_HIP(hipStreamSynchronize(X->ctx->stream));
  }
  // updateSolution(update, updateLP = true) (BelosLinearProblem.hpp:743-812): X += M_R update
  void update_solution(const MvPtr &upd) {
    if (!upd.p) return;
    if (RP) {
      MvPtr ru = clone(upd->ncols);
      prec(*RP, *upd, *ru);
      mv_add_mv(1.0, *curX, 1.0, *ru, *curX);
    } else {
      mv_add_mv(1.0, *curX, 1.0, *upd, *curX);
    }
  }
  // updateSolution(update, updateLP = false): out = X + M_R update (X itself when no update)
  void updated_solution(const MvPtr &upd, migmres_mv &out) {
    if (!upd.p) {
      mv_assign(*curX, out);
    } else if (RP) {
      MvPtr ru = clone(upd->ncols);
      prec(*RP, *upd, *ru);
      mv_add_mv(1.0, *curX, 1.0, *ru, out);
    } else {
      mv_add_mv(1.0, *curX, 1.0, *upd, out);
    }
  }
  // computeCurrResVec: R = B - A*Xs (BelosLinearProblem.hpp:1196-1231)
  void curr_res_vec(migmres_mv &R, const migmres_mv *Xs = nullptr) {
    op(Xs ? *Xs : *curX, R);
    mv_add_mv(-1.0, R, 1.0, *curB, R);
  }
  // computeCurrPrecResVec: R = M_L (B - A*X) (BelosLinearProblem.hpp:1117-1195)
  void curr_prec_res_vec(migmres_mv &R) {
    if (!LP) {
      curr_res_vec(R);
      return;
    }
    MvPtr t = clone(R.ncols);
    curr_res_vec(*t);
    prec(*LP, *t, R);
  }
};

// Residual status tests: StatusTestImpResNorm (implicit with the explicit confirmation and
// loss-of-accuracy logic, BelosStatusTestImpResNorm.hpp:492-749) and StatusTestGenResNorm
// (implicit or explicit form, BelosStatusTestGenResNorm.hpp:455-600).
struct ResTest {
  enum Kind { IMP_RES_NORM, GEN_IMPLICIT, GEN_EXPLICIT } kind;
  std::string scale_type;
  double tol, curr_tol;
  bool first = true, loss = false, passed = false;
  int cur_ls_num = 0, numrhs = 0, cur_num_rhs = 0;
  long long n_explicit = 0;
  std::vector<int> cur_idx;
  std::vector<double> scale, resvector, testvector;
  MvPtr cur_soln;
  bool have_soln = false;
  int quorum = -1;       // setQuorum: passes when >= quorum columns pass (-1: all)
  std::vector<int> ind;  // convIndices(): the right-hand sides that passed
  ResTest(Kind k, double t, const std::string &st) : kind(k), scale_type(st), tol(t), curr_tol(t) {}
};

struct Iter {  // BlockGmresIter / BlockFGmresIter state (H and R share storage)
  int k, nb, sd, cur_dim = 0, num_iters = 0;
  MvPtr V;
  MvPtr Z;  // flexible: Z_j = M_R V_j (BelosBlockFGmresIter.hpp:316)
  std::vector<double> R, z, beta, cs, sn;
  int ldr() const { return sd; }
  double &Rat(int i, int j) { return R[(size_t)i + (size_t)j * sd]; }
  double &zat(int i, int j) { return z[(size_t)i + (size_t)j * sd]; }
};

struct Engine {
  migmres_solver *S;
  Problem lp;
  // checkStatusTest (BelosBlockGmresSolMgr.hpp:807-903): conv = imp, or SEQ(imp, exp)
  ResTest imp, exp;
  bool seq = false, flexible = false;
  bool conv_passed = false;
  int max_iters;
  int mi_n_iters = 0;
  bool mi_passed = false;

  Engine(migmres_solver *s, double tol, int mi)
      : S(s), imp(ResTest::IMP_RES_NORM, tol, s->p.imp_scale), exp(ResTest::GEN_EXPLICIT, tol, s->p.exp_scale),
        max_iters(mi) {}
  ResTest &exp_conv() { return seq ? exp : imp; }

  void setup_status_tests(bool has_left, bool has_right) {
    flexible = S->p.flexible;
    bool exp_test = S->p.exp_res_test;
    if (flexible && !has_right) {
      flexible = false;
      MIG_CHECK(!has_left, "BlockGmresSolMgr: flexible GMRES needs a right, not a left, preconditioner");
    }
    if (has_left && !flexible) exp_test = true;
    seq = exp_test;
    if (seq)
      imp.kind = ResTest::GEN_IMPLICIT;
    else
      imp.kind = flexible ? ResTest::GEN_IMPLICIT : ResTest::IMP_RES_NORM;
  }

  std::vector<double> native_residuals(Iter &it) {  // getNativeResiduals
    std::vector<double> r((size_t)it.k);
    for (int j = 0; j < it.k; ++j) {
      double s = 0.0, scl = 0.0, ssq = 1.0;
      for (int i = 0; i < it.k; ++i) {  // dnrm2 scaled sum of squares
        const double v = it.zat(it.cur_dim + i, j);
        if (v != 0.0) {
          const double a = std::fabs(v);
          if (scl < a) {
            ssq = 1.0 + ssq * (scl / a) * (scl / a);
            scl = a;
          } else {
            ssq += (a / scl) * (a / scl);
          }
        }
      }
      s = scl * std::sqrt(ssq);
      r[(size_t)j] = s;
    }
    return r;
  }

  // getCurrentUpdate (BelosBlockGmresIter.hpp:500-535): TRSM on host, V*y on device.
  MvPtr current_update(Iter &it) {
    const int c = it.cur_dim, k = it.k;
    if (c == 0) return MvPtr();
    std::vector<double> y((size_t)c * k);
    for (int j = 0; j < k; ++j)
      for (int i = 0; i < c; ++i) y[(size_t)i + (size_t)j * c] = it.zat(i, j);
    for (int j = 0; j < k; ++j)
      for (int i = c - 1; i >= 0; --i) {
        double t = y[(size_t)i + (size_t)j * c];
        for (int q = i + 1; q < c; ++q) t -= it.Rat(i, q) * y[(size_t)q + (size_t)j * c];
        y[(size_t)i + (size_t)j * c] = t / it.Rat(i, i);
      }
    MvPtr upd(mv_create(lp.X->ctx, lp.X->n_global, lp.X->n_local, k));
    MvPtr Vc = view(it.Z.p ? *it.Z : *it.V, 0, c);  // BlockFGmresIter: Z y (:488-523)
    mv_times_mat_add_mv(1.0, *Vc, y.data(), c, 0.0, *upd);
    return upd;
  }

  bool max_iters_check(Iter &it) {
    mi_n_iters = it.num_iters;
    mi_passed = mi_n_iters >= max_iters;
    return mi_passed;
  }

  // firstCallCheckStatusSetup scaling (GenResNorm :643-700, ImpResNorm :815-845)
  void scale_setup(ResTest &t) {
    t.numrhs = lp.B->ncols;
    t.scale.clear();
    if (t.scale_type == "None") return;
    t.scale.assign((size_t)t.numrhs, 0.0);
    if (t.scale_type == "Norm of RHS")
      mv_norm(*lp.B, t.scale.data(), MIGMRES_TWO_NORM);
    else if (t.scale_type == "Norm of Initial Residual")
      mv_norm(*lp.R0, t.scale.data(), MIGMRES_TWO_NORM);
    else
      mv_norm(lp.pr0(), t.scale.data(), MIGMRES_TWO_NORM);
  }
  double scaled(const ResTest &t, int p, double r) const {
    const double s = t.scale.empty() ? 0.0 : t.scale[(size_t)p];
    return s != 0.0 ? r / s / 1.0 : r / 1.0;
  }

  bool res_check(ResTest &t, Iter &it) {
    return res_check(t, [&] { return native_residuals(it); }, [&] { return current_update(it); });
  }
  // checkStatus of either test over any iteration: native residual norms and the current
  // solution update come from the callbacks (BlockGmresIter or PseudoBlockGmresIter).
  bool res_check(ResTest &t, const std::function<std::vector<double>()> &native,
                 const std::function<MvPtr()> &update) {
    if (t.first) {
      t.first = false;
      scale_setup(t);
      t.resvector.assign((size_t)t.numrhs, 0.0);
      t.testvector.assign((size_t)t.numrhs, 1.0);
      t.cur_ls_num = lp.ls_num;
      t.cur_idx = lp.ls_idx;
      t.cur_num_rhs = 0;
      for (int i : t.cur_idx)
        if (i > -1 && i < t.numrhs) ++t.cur_num_rhs;
    }
    if (t.cur_ls_num != lp.ls_num) {
      t.cur_ls_num = lp.ls_num;
      t.cur_idx = lp.ls_idx;
      t.cur_num_rhs = 0;
      for (int i : t.cur_idx)
        if (i > -1 && i < t.numrhs) ++t.cur_num_rhs;
      t.have_soln = false;
    } else if (t.passed) {
      return true;
    }
    const int k = lp.curX->ncols;
    auto explicit_norms = [&](std::vector<double> &out) {
      ++t.n_explicit;
      ++S->n_explicit;
      MvPtr upd = update();
      if (!t.cur_soln.p || t.cur_soln->ncols != k) t.cur_soln = lp.clone(k);
      lp.updated_solution(upd, *t.cur_soln);
      t.have_soln = true;
      MvPtr cur_res = lp.clone(k);
      lp.curr_res_vec(*cur_res, t.cur_soln.p);
      out.assign((size_t)k, 0.0);
      mv_norm(*cur_res, out.data(), MIGMRES_TWO_NORM);
    };
    std::vector<double> res;
    if (t.kind == ResTest::GEN_EXPLICIT)
      explicit_norms(res);
    else
      res = native();
    for (size_t i = 0; i < t.cur_idx.size(); ++i)
      if (t.cur_idx[i] != -1) t.resvector[(size_t)t.cur_idx[i]] = res[i];
    for (int p : t.cur_idx)
      if (p != -1) t.testvector[(size_t)p] = scaled(t, p, t.resvector[(size_t)p]);
    const double tol_now = t.kind == ResTest::IMP_RES_NORM ? t.curr_tol : t.tol;
    std::vector<int> ind, lcl;
    for (size_t i = 0; i < t.cur_idx.size(); ++i) {
      const int p = t.cur_idx[i];
      if (p == -1) continue;
      const double tv = t.testvector[(size_t)p];
      if (tv > tol_now) {
      } else if (tv <= tol_now) {
        ind.push_back(p);
        lcl.push_back((int)i);
      } else {
        throw Error(MIGMRES_ESTATE, "residual status test: residual norm is NaN");
      }
    }
    int have = (int)ind.size();
    if (have && t.kind == ResTest::IMP_RES_NORM) {
      std::vector<double> tmp_res;
      explicit_norms(tmp_res);
      std::vector<double> tmp_test((size_t)have);
      for (int i = 0; i < have; ++i) tmp_test[(size_t)i] = scaled(t, ind[(size_t)i], tmp_res[(size_t)lcl[(size_t)i]]);
      int have2 = 0;
      for (int i = 0; i < have; ++i) {
        if (tmp_test[(size_t)i] <= t.tol) {
          ind[(size_t)have2++] = ind[(size_t)i];
        } else {
          const double diff = std::fabs(t.testvector[(size_t)ind[(size_t)i]] - tmp_test[(size_t)i]);
          if (diff > t.curr_tol) {
            t.loss = true;
            ind[(size_t)have2++] = ind[(size_t)i];
          } else {
            t.curr_tol = t.curr_tol - (3.0 / 2.0) * diff;
            while (t.curr_tol < 0.0) t.curr_tol += (1.0 / 10.0) * diff;
          }
        }
      }
      have = have2;
    }
    t.ind.assign(ind.begin(), ind.begin() + have);
    t.passed = have >= (t.quorum == -1 ? t.cur_num_rhs : t.quorum);
    return t.passed;
  }

  bool conv_check(Iter &it) {  // StatusTestCombo SEQ (BelosStatusTestCombo.hpp:360-380)
    if (!seq) return conv_passed = res_check(imp, it);
    if (!res_check(imp, it)) return conv_passed = false;
    return conv_passed = res_check(exp, it);
  }

  bool check(Iter &it) {  // StatusTestCombo OR: both members evaluated
    auto t0 = Clock::now();
    struct T {
      migmres_solver *S;
      Clock::time_point t0;
      ~T() { S->t_check += since(t0); }
    } tm{S, t0};
    const bool a = max_iters_check(it);
    const bool b = conv_check(it);
    S->history.insert(S->history.end(), imp.testvector.begin(), imp.testvector.end());
    S->hist_cols = (int)imp.testvector.size();
    return a || b;
  }

  void initialize(Iter &it, migmres_mv &V0, const std::vector<double> &z0) {  // initializeGmres
    const int k = it.k;
    it.cur_dim = 0;
    MvPtr v = view(*it.V, 0, k);
    mv_add_mv(1.0, V0, 0.0, V0, *v);
    std::fill(it.z.begin(), it.z.end(), 0.0);
    for (int j = 0; j < k; ++j)
      for (int i = 0; i < k; ++i) it.zat(i, j) = z0[(size_t)i + (size_t)j * k];
  }

  void update_lsqr(Iter &it, int dim = -1) {  // updateLSQR (BelosBlockGmresIter.hpp:770-868)
    auto t0 = Clock::now();
    const int k = it.k;
    int cur = it.cur_dim;
    if (dim >= it.cur_dim && dim < k * it.nb) cur = dim;
    if (k == 1) {
      for (int i = 0; i < cur; ++i) {
        const double x = it.Rat(i, cur), y = it.Rat(i + 1, cur);
        it.Rat(i, cur) = it.cs[(size_t)i] * x + it.sn[(size_t)i] * y;
        it.Rat(i + 1, cur) = it.cs[(size_t)i] * y - it.sn[(size_t)i] * x;
      }
      rotg(it.Rat(cur, cur), it.Rat(cur + 1, cur), it.cs[(size_t)cur], it.sn[(size_t)cur]);
      it.Rat(cur + 1, cur) = 0.0;
      const double x = it.zat(cur, 0), y = it.zat(cur + 1, 0);
      it.zat(cur, 0) = it.cs[(size_t)cur] * x + it.sn[(size_t)cur] * y;
      it.zat(cur + 1, 0) = it.cs[(size_t)cur] * y - it.sn[(size_t)cur] * x;
    } else {
      for (int j = 0; j < k; ++j) {
        const int cj = cur + j;
        for (int i = 0; i < cj; ++i) {
          double sigma = 0.0;
          for (int q = 0; q < k; ++q) sigma += it.Rat(i + 1 + q, i) * it.Rat(i + 1 + q, cj);
          sigma += it.Rat(i, cj);
          sigma *= it.beta[(size_t)i];
          for (int q = 0; q < k; ++q) it.Rat(i + 1 + q, cj) += (-sigma) * it.Rat(i + 1 + q, i);
          it.Rat(i, cj) -= sigma;
        }
        int maxidx = 0;
        double maxabs = -1.0;
        for (int q = 0; q < k + 1; ++q) {
          const double a = std::fabs(it.Rat(cj + q, cj));
          if (a > maxabs) {
            maxabs = a;
            maxidx = q;
          }
        }
        const double maxelem = it.Rat(cj + maxidx, cj);
        for (int q = 0; q < k + 1; ++q) it.Rat(cj + q, cj) /= maxelem;
        double sigma = 0.0;
        for (int q = 0; q < k; ++q) sigma += it.Rat(cj + 1 + q, cj) * it.Rat(cj + 1 + q, cj);
        if (sigma == 0.0) {
          it.beta[(size_t)cj] = 0.0;
        } else {
          const double d = it.Rat(cj, cj);
          const double mu = std::sqrt(d * d + sigma);
          const double vscale = d < 0.0 ? d - mu : -sigma / (d + mu);
          it.beta[(size_t)cj] = 2.0 * 1.0 * vscale * vscale / (sigma + vscale * vscale);
          it.Rat(cj, cj) = maxelem * mu;
          for (int q = 0; q < k; ++q) it.Rat(cj + 1 + q, cj) /= vscale;
        }
        for (int col = 0; col < k; ++col) {
          double s2 = 0.0;
          for (int q = 0; q < k; ++q) s2 += it.Rat(cj + 1 + q, cj) * it.zat(cj + 1 + q, col);
          s2 += it.zat(cj, col);
          s2 *= it.beta[(size_t)cj];
          for (int q = 0; q < k; ++q) it.zat(cj + 1 + q, col) += (-s2) * it.Rat(cj + 1 + q, cj);
          it.zat(cj, col) -= s2;
        }
      }
    }
    if (dim >= it.cur_dim && dim < k * it.nb) it.cur_dim = dim + k;
    S->t_lsq += since(t0);
  }

  struct OrthoFailure {};

  int normalize(migmres_mv &V0, double *B, int ldb) {
    auto t0 = Clock::now();
    const int r = (S->use_fast && S->fast.supports(V0.ncols)) ? S->fast.normalize(V0, B, ldb)
                                                             : S->ortho.normalize(V0, B, ldb);
    S->t_ortho += since(t0);
    return r;
  }

  void iterate(Iter &it) {  // BlockGmresIter::iterate (BelosBlockGmresIter.hpp:659-766)
    const int k = it.k, search = k * it.nb;
    std::vector<double> subH, subH2;
    // Op V_prev for the next block may already have been computed behind the previous
    // iteration's state copy (speculatively: unused when the iteration loop ends there or
    // the orthogonalisation fell back and changed the block; it is counted when used).
    bool spec_ready = false;
    const char *se = std::getenv("MIGMRES_SPEC_SPMM");
    const bool spec_on = !(se && se[0] == '0') && !it.Z.p && !lp.LP && !lp.RP && lp.A && !(S->p.verbosity & 1);
    while (!check(it) && it.cur_dim + k <= search) {
      ++it.num_iters;
      ++S->n_block_iters;
      const int lcl = it.cur_dim + k, c = it.cur_dim;
      MvPtr Vnext = view(*it.V, lcl, k);
      MvPtr Vprev = view(*it.V, c, k);
      MvPtr Znext;
      if (it.Z.p) {  // BlockFGmresIter::iterate (BelosBlockFGmresIter.hpp:680-691)
        Znext = view(*it.Z, c, k);
        lp.apply_right_prec(*Vprev, *Znext);
        lp.op(*Znext, *Vnext);
      } else if (spec_ready) {
        ++S->n_apply;  // OPT::Apply(A) done ahead
      } else {
        lp.apply(*Vprev, *Vnext);
      }
      spec_ready = false;
      MvPtr Vnn;
      bool spec_issued = false;
      const bool spec = spec_on && S->use_fast && S->fast.supports(k) && lcl + k <= search;
      if (spec) {
        Vnn = view(*it.V, lcl + k, k);
        S->fast.before_wait = [&] {
          crs_apply(*lp.A, *Vnext, *Vnn, 1.0, 0.0);
          spec_issued = true;
        };
      }
      struct HookReset {
        std::function<void()> &f;
        ~HookReset() { f = nullptr; }
      } hook_reset{S->fast.before_wait};
      const long long fb0 = S->fast.fallbacks;
      MvPtr Q = view(*it.V, 0, lcl);
      subH.assign((size_t)lcl * k, 0.0);
      subH2.assign((size_t)k * k, 0.0);
      auto t0 = Clock::now();
      // X = Op V_prev again, bit for bit, if the device ICGS has to restart from its input
      const std::function<void()> regen = [&] {
        if (Znext.p)
          lp.op_raw(*Znext, *Vnext);
        else if (!lp.LP && !lp.RP)
          lp.op_raw(*Vprev, *Vnext);
        else {  // not counted: the reference copies its input instead
          const long long na = S->n_apply, np = S->n_prec;
          lp.apply(*Vprev, *Vnext);
          S->n_apply = na;
          S->n_prec = np;
        }
      };
      const int rank = S->use_fast && S->fast.supports(k)
                           ? S->fast.project_and_normalize(*Vnext, *Q, subH.data(), lcl, subH2.data(), k,
                                                           lp.own_ops() ? &regen : nullptr)
                           : S->ortho.project_and_normalize(*Vnext, *Q, subH.data(), lcl, subH2.data(), k);
      S->t_ortho += since(t0);
      S->fast.before_wait = nullptr;
      spec_ready = spec_issued && S->fast.fallbacks == fb0 && rank == k;
      for (int j = 0; j < k; ++j) {
        for (int i = 0; i < lcl; ++i) it.Rat(i, c + j) = subH[(size_t)i + (size_t)j * lcl];
        for (int i = 0; i < k; ++i) it.Rat(lcl + i, c + j) = subH2[(size_t)i + (size_t)j * k];
      }
      if (rank != k) throw OrthoFailure{};
      update_lsqr(it);
      it.cur_dim += k;
    }
  }

  // BlockGmresSolMgr::solve (BelosBlockGmresSolMgr.hpp:916-1303), plain and flexible.
  bool solve() {
    const Params &p = S->p;
    int block = p.block_size;
    const int numrhs = lp.B->ncols;
    int start = 0, to_solve = numrhs;
    int cur_rhs = std::min(to_solve, block);
    std::vector<int> idx;
    auto make_idx = [&]() {
      idx.clear();
      if (p.adaptive) {
        block = cur_rhs;
        for (int i = 0; i < cur_rhs; ++i) idx.push_back(start + i);
      } else {
        for (int i = 0; i < cur_rhs; ++i) idx.push_back(start + i);
        for (int i = cur_rhs; i < block; ++i) idx.push_back(-1);
      }
    };
    make_idx();
    lp.set_ls_index(idx);
    const long long dim = lp.B->n_global;
    bool converged = true;
    S->loa = false;
    while (to_solve > 0) {
      int nb = p.num_blocks;
      if ((long long)block * p.num_blocks > dim) nb = (int)(block == 1 ? dim / block : (dim - block) / block);
      auto ts0 = Clock::now();
      Iter it;
      it.k = block;
      it.nb = nb;
      it.sd = block * (nb + 1);
      it.V = MvPtr(mv_create(lp.X->ctx, lp.X->n_global, lp.X->n_local, it.sd));
      if (flexible) it.Z = MvPtr(mv_create(lp.X->ctx, lp.X->n_global, lp.X->n_local, it.sd));
      it.R.assign((size_t)it.sd * (it.sd - block), 0.0);
      it.z.assign((size_t)it.sd * block, 0.0);
      it.beta.assign((size_t)it.sd, 0.0);
      it.cs.assign((size_t)it.sd, 0.0);
      it.sn.assign((size_t)it.sd, 0.0);
      MvPtr V0(mv_create(lp.X->ctx, lp.X->n_global, lp.X->n_local, block));
      // the first block: (preconditioned) residual, R0 for flexible GMRES (:1025-1047)
      auto residual = [&](migmres_mv &R) {
        if (flexible)
          lp.curr_res_vec(R);
        else
          lp.curr_prec_res_vec(R);
      };
      if (idx.back() == -1) {
        residual(*V0);
      } else {
        MvPtr r0v(mv_view(flexible ? lp.R0.p : &lp.pr0(), idx.data(), (int)idx.size()));
        mv_assign(*r0v, *V0);
      }
      std::vector<double> z0((size_t)block * block, 0.0);
      S->ortho.dgks = S->p.ortho == "DGKS";
      S->ortho.dep_tol = S->p.dgks_dep_tol();
      if (S->use_fast && S->fast.supports(block)) {
        S->fast.slow = &S->ortho;
        S->fast.setup(lp.X->ctx, lp.X->n_global, lp.X->n_local, block, it.sd);
      }
      if (normalize(*V0, z0.data(), block) != block)
        throw Error(MIGMRES_ESTATE, "BlockGmresSolMgr: failed to compute initial block of orthonormal vectors");
      initialize(it, *V0, z0);
      if (S->sync_timers()) MIG_HIP(hipStreamSynchronize(lp.X->ctx->stream));
      S->t_setup += since(ts0);
      int restarts = 0;
      while (true) {
        try {
          iterate(it);
          if (conv_passed) {
            if (exp_conv().loss) {
              S->loa = true;
              converged = false;
            }
            break;
          } else if (mi_passed) {
            converged = false;
            break;
          } else if (it.cur_dim == it.k * it.nb) {
            if (restarts >= p.max_restarts) {
              converged = false;
              break;
            }
            ++restarts;
            auto tr0 = Clock::now();
            MvPtr upd = current_update(it);
            if (flexible) {  // the update is already preconditioned (:1114-1118)
              if (upd.p) mv_add_mv(1.0, *lp.curX, 1.0, *upd, *lp.curX);
            } else {
              lp.update_solution(upd);
            }
            residual(*V0);
            std::fill(z0.begin(), z0.end(), 0.0);
            if (normalize(*V0, z0.data(), block) != block)
              throw Error(MIGMRES_ESTATE, "BlockGmresSolMgr: failed to compute initial block after restart");
            initialize(it, *V0, z0);
            S->t_restart += since(tr0);
          } else {
            throw Error(MIGMRES_ESTATE, "BlockGmresSolMgr: invalid return from iterate()");
          }
        } catch (const OrthoFailure &) {
          if (block != 1) {
            if (!conv_passed) converged = false;
            break;
          }
          update_lsqr(it, it.cur_dim);
          check(it);
          if (!conv_passed) converged = false;
          break;
        }
      }
      // the solution of this block (:1190-1212)
      if (flexible) {
        MvPtr upd = current_update(it);
        if (upd.p) mv_add_mv(1.0, *lp.curX, 1.0, *upd, *lp.curX);
      } else if (exp_conv().have_soln) {
        ResTest &e = exp_conv();
        mv_add_mv(0.0, *e.cur_soln, 1.0, *e.cur_soln, *lp.curX);
      } else {
        MvPtr upd = current_update(it);
        lp.update_solution(upd);
      }
      lp.set_curr_ls();
      S->n_restarts += restarts;
      start += cur_rhs;
      to_solve -= cur_rhs;
      if (to_solve > 0) {
        cur_rhs = std::min(to_solve, block);
        make_idx();
        lp.set_ls_index(idx);
      }
    }
    MIG_HIP(hipStreamSynchronize(lp.X->ctx->stream));
    S->num_iters = mi_n_iters;
    // achievedTol (:1268-1290): the explicit test's values when it ran, else the implicit ones
    const std::vector<double> *tv = &imp.testvector;
    if (seq && !exp.testvector.empty()) tv = &exp.testvector;
    S->achieved_tol = tv->empty() ? 0.0 : *std::max_element(tv->begin(), tv->end());
    return converged && !S->loa;
  }
};

// ------------------------------------------------------------------------------------
// Pseudo-block GMRES: k single-vector GMRES iterations sharing one operator application per
// step (BelosPseudoBlockGmresIter.hpp, BelosPseudoBlockGmresSolMgr.hpp).  Right-hand side i
// owns the basis columns V[:, j*nslots + slot], j = 0 .. nb, of one device multivector
// (iteration-major, so while every slot is active the bases of step c are the contiguous
// columns 0 .. (c+1) nslots - 1, and the new vectors the next nslots: the batched ICGS reads
// them without a column table); its Hessenberg column, Givens rotations and least-squares
// right-hand side stay on the host.  Deflation of converged right-hand sides drops their
// state; slots are never moved.
// ------------------------------------------------------------------------------------
struct PseudoRhs {
  int slot;
  std::vector<double> H, z, cs, sn;  // H is (nb+1) x nb column-major
};

struct PseudoIter {
  int nb = 0, cur_dim = 0, num_iters = 0, nslots = 0;
  MvPtr V;  // N x nslots*(nb+1)
  std::vector<PseudoRhs> st;
  int col(const PseudoRhs &r, int j) const { return j * nslots + r.slot; }
  // basis columns first .. first + cnt - 1 of one right-hand side (a column-table view)
  MvPtr basis(const PseudoRhs &r, int first, int cnt) const {
    std::vector<int> idx((size_t)cnt);
    for (int q = 0; q < cnt; ++q) idx[(size_t)q] = col(r, first + q);
    return MvPtr(mv_view(V.p, idx.data(), cnt));
  }
  double &Hat(PseudoRhs &r, int i, int j) const { return r.H[(size_t)i + (size_t)j * (nb + 1)]; }
};

struct PseudoEngine : Engine {
  PseudoEngine(migmres_solver *s, double tol, int mi) : Engine(s, tol, mi) {}

  // One device ICGS state per right-hand side slot (ICGS; DGKS's k = 1 blkOrtho1 decides its
  // second pass on the host between the passes and keeps the host path).
  std::vector<std::unique_ptr<FastIcgs>> rhs_fast;
  int rhs_nb = 0;
  bool device_ortho() const { return S->use_fast && !S->ortho.dgks && S->ortho.steps == 2; }
  FastIcgs &rhs_ortho(int slot) {
    auto &f = rhs_fast[(size_t)slot];
    if (!f) {
      f.reset(new FastIcgs());
      f->slow = &S->ortho;
      f->setup(lp.X->ctx, lp.X->n_global, lp.X->n_local, 1, rhs_nb + 1);
    }
    return *f;
  }

  // Batched k = 1 ICGS (blkOrtho1 with two passes, then MvNorm / MvScale) for every right-hand
  // side in one launch per pass: the bases side by side as one column table, the block
  // kernels with block-diagonal coefficients (icgs.hip, launch_blockdiag).  Three passes over
  // the bases (QB^T X; the fused X1 = X - QB M1 with QB^T X1; the closing X - QB (M1 + M2)
  // with the column dots) instead of three k = 1 chains per right-hand side.
  // MIGMRES_PSEUDO_BATCHED=0 keeps the per-right-hand-side chains.
  const bool batched_on = [] {
    const char *e = std::getenv("MIGMRES_PSEUDO_BATCHED");
    return !(e && e[0] == '0');
  }();
  double *bt_buf = nullptr, *bt_part = nullptr, *bt_sink = nullptr, *bt_host = nullptr;
  size_t bt_cap = 0, bt_pcap = 0;
  ~PseudoEngine() {
    for (double *p : {bt_buf, bt_part, bt_sink})
      if (p) (void)hipFree(p);
    if (bt_host) (void)hipHostFree(bt_host);
  }
  bool batched_ok(int n, int L) const {
    return batched_on && device_ortho() && n >= 2 && n <= 8 && n * L <= 512 && nn_tn_supported(n * L, n);
  }
  void batched_ortho(PseudoIter &it, int c, const std::vector<int> &vcols) {
    migmres_ctx *ctx = lp.X->ctx;
    hipStream_t s = ctx->stream;
    const int n = (int)it.st.size(), L = c + 1, LB = n * L, nl = lp.X->n_local;
    std::vector<int> qcols((size_t)LB);
    for (int q = 0; q < L; ++q)  // iteration-major: contiguous while every slot is active
      for (int i = 0; i < n; ++i) qcols[(size_t)(q * n + i)] = it.col(it.st[(size_t)i], q);
    MvPtr QB(mv_view(it.V.p, qcols.data(), LB));
    MvPtr X(mv_view(it.V.p, vcols.data(), n));
    const int nblk_tn = gemm_tn_blocks(nl), nblk_tl = gemm_tn_blocks(nl, LB), nblk_nt = nn_tn_blocks(nl, LB, n),
              nblk_ic = icgs_blocks(nl);
    const size_t need = (size_t)4 * LB * n + 2 * (size_t)n;
    if (need > bt_cap) {
      if (bt_buf) (void)hipFree(bt_buf);
      if (bt_host) (void)hipHostFree(bt_host);
      MIG_HIP(hipMalloc(&bt_buf, sizeof(double) * need));
      MIG_HIP(hipHostMalloc(&bt_host, sizeof(double) * need, hipHostMallocDefault));
      bt_cap = need;
    }
    const size_t pneed = std::max({(size_t)nblk_tn * LB * n, (size_t)nblk_nt * LB * n, (size_t)nblk_ic * (n + 1)});
    if (pneed > bt_pcap) {
      if (bt_part) (void)hipFree(bt_part);
      MIG_HIP(hipMalloc(&bt_part, sizeof(double) * pneed));
      bt_pcap = pneed;
    }
    if (!bt_sink) MIG_HIP(hipMalloc(&bt_sink, sizeof(double) * 1024 * 2048));
    double *C1 = bt_buf, *C2 = C1 + (size_t)LB * n, *M1 = C2 + (size_t)LB * n, *M = M1 + (size_t)LB * n;
    double *dots = M + (size_t)LB * n, *Bn = dots + n;
    {
      ProfScope ps(ctx, K_GEMM_TN, 8.0 * nl * (LB + n));
      launch_gemm_tn_partial(s, QB->desc(), LB, X->desc(), n, nl, bt_part, nblk_tl);
    }
    {
      ProfScope ps(ctx, K_REDUCE, 8.0 * nblk_tl * LB * n);
      launch_reduce_partials_ld(s, bt_part, nblk_tl, LB, n, LB, 1.0, C1);
    }
    ctx->allreduce_async(C1, (size_t)LB * n);
    launch_blockdiag(s, C1, nullptr, LB, n, L, M1);
    {
      ProfScope ps(ctx, K_NN_TN, 8.0 * nl * (LB + n));
      launch_nn_tn(s, QB->desc(), LB, M1, LB, X->desc(), nl, bt_part, nblk_nt, bt_sink, false);
    }
    {
      ProfScope ps(ctx, K_REDUCE, 8.0 * nblk_nt * LB * n);
      launch_reduce_partials_ld(s, bt_part, nblk_nt, LB, n, LB, 1.0, C2);
    }
    ctx->allreduce_async(C2, (size_t)LB * n);
    launch_blockdiag(s, C1, C2, LB, n, L, M);
    {
      ProfScope ps(ctx, K_GEMM_NN_DOT, 8.0 * nl * (LB + 2.0 * n));
      launch_gemm_nn_dot(s, QB->desc(), LB, M, LB, X->desc(), nl, -1.0, 1.0, 1, X->desc(), bt_part, nblk_ic);
    }
    launch_reduce_partials(s, bt_part, nblk_ic, n, 1.0, dots);
    ctx->allreduce_async(dots, (size_t)n);
    {
      ProfScope ps(ctx, K_SCALE, 16.0 * nl * n);
      launch_norm_scale(s, X->desc(), nl, dots, Bn);
    }
    MIG_HIP(hipMemcpyAsync(bt_host, M, sizeof(double) * ((size_t)LB * n + 2 * n), hipMemcpyDeviceToHost, s));
    MIG_HIP(hipStreamSynchronize(s));
    const double *Mh = bt_host, *Bh = bt_host + (size_t)LB * n + n;
    for (int i = 0; i < n; ++i) {
      PseudoRhs &rs = it.st[(size_t)i];
      for (int q = 0; q <= c; ++q) it.Hat(rs, q, c) = Mh[(size_t)(q * n + i) + (size_t)i * LB];
      it.Hat(rs, c + 1, c) = Bh[i];
    }
  }

  void setup_pseudo_tests(bool has_left) {  // checkStatusTest (:1156-1265)
    seq = S->p.exp_res_test || has_left;
    imp.kind = seq ? ResTest::GEN_IMPLICIT : ResTest::IMP_RES_NORM;
    imp.quorum = exp.quorum = S->p.def_quorum;
  }

  std::vector<double> native(PseudoIter &it) {  // getNativeResiduals (:487-510)
    std::vector<double> r(it.st.size());
    for (size_t i = 0; i < it.st.size(); ++i) r[i] = std::fabs(it.st[i].z[(size_t)it.cur_dim]);
    return r;
  }

  MvPtr update(PseudoIter &it) {  // getCurrentUpdate (:447-484)
    const int c = it.cur_dim;
    if (c == 0) return MvPtr();
    const int n = (int)it.st.size();
    MvPtr upd = lp.clone(n);
    std::vector<double> y((size_t)c);
    for (int i = 0; i < n; ++i) {
      PseudoRhs &r = it.st[(size_t)i];
      for (int q = 0; q < c; ++q) y[(size_t)q] = r.z[(size_t)q];
      for (int q = c - 1; q >= 0; --q) {
        double t = y[(size_t)q];
        for (int u = q + 1; u < c; ++u) t -= it.Hat(r, q, u) * y[(size_t)u];
        y[(size_t)q] = t / it.Hat(r, q, q);
      }
      MvPtr Vi = it.basis(r, 0, c);
      MvPtr ui = view(*upd, i, 1);
      mv_times_mat_add_mv(1.0, *Vi, y.data(), c, 0.0, *ui);
    }
    return upd;
  }

  bool check(PseudoIter &it) {
    auto t0 = Clock::now();
    mi_n_iters = it.num_iters;
    mi_passed = mi_n_iters >= max_iters;
    auto nat = [&] { return native(it); };
    auto upd = [&] { return update(it); };
    if (!seq)
      conv_passed = res_check(imp, nat, upd);
    else
      conv_passed = res_check(imp, nat, upd) && res_check(exp, nat, upd);
    if (S->user_test) {  // StatusTestCombo(combo, residual test, user test) (:1216-1240)
      auto user = [&] {
        return S->user_test(S->user_data, it.num_iters, (int)imp.testvector.size(), imp.testvector.data()) != 0;
      };
      if (S->user_combo == MIGMRES_COMBO_SEQ)
        conv_passed = conv_passed && user();
      else if (S->user_combo == MIGMRES_COMBO_AND)
        conv_passed = user() && conv_passed;
      else
        conv_passed = user() || conv_passed;
    }
    S->history.insert(S->history.end(), imp.testvector.begin(), imp.testvector.end());
    S->hist_cols = (int)imp.testvector.size();
    S->t_check += since(t0);
    return mi_passed || conv_passed;
  }

  // iterate (BelosPseudoBlockGmresIter.hpp:743-871): AU = Op U, then each right-hand side
  // projects and normalises its own new vector against its own basis.
  void iterate(PseudoIter &it) {
    const int n = (int)it.st.size();
    std::vector<int> ucols((size_t)n), vcols((size_t)n);
    std::vector<double> h, r(1);
    while (!check(it) && it.cur_dim < it.nb) {
      ++it.num_iters;
      ++S->n_block_iters;
      const int c = it.cur_dim;
      for (int i = 0; i < n; ++i) {
        ucols[(size_t)i] = it.col(it.st[(size_t)i], c);
        vcols[(size_t)i] = it.col(it.st[(size_t)i], c + 1);
      }
      MvPtr U(mv_view(it.V.p, ucols.data(), n));
      MvPtr AU(mv_view(it.V.p, vcols.data(), n));
      lp.apply(*U, *AU);
      auto t0 = Clock::now();
      h.assign((size_t)c + 1, 0.0);
      if (batched_ok(n, c + 1)) {
        batched_ortho(it, c, vcols);
      } else if (device_ortho()) {
        // every right-hand side's ICGS chain on the stream (its own FastIcgs state), one wait
        std::vector<MvPtr> ws, qs;
        for (int i = 0; i < n; ++i) {
          PseudoRhs &rs = it.st[(size_t)i];
          ws.push_back(view(*it.V, vcols[(size_t)i], 1));
          qs.push_back(it.basis(rs, 0, c + 1));
          FastIcgs &f = rhs_ortho(rs.slot);
          f.enqueue_k1(*ws.back(), *qs.back());
          f.fetch_async(c + 1, 1);
        }
        MIG_HIP(hipStreamSynchronize(lp.X->ctx->stream));
        for (int i = 0; i < n; ++i) {
          PseudoRhs &rs = it.st[(size_t)i];
          const FastIcgs &f = rhs_ortho(rs.slot);
          if (f.hst().neg != 0.0) throw Error(MIGMRES_ESTATE, "ICGS: negative definiteness in inner product");
          f.result_k1(c + 1, h.data(), r.data());
          for (int q = 0; q <= c; ++q) it.Hat(rs, q, c) = h[(size_t)q];
          it.Hat(rs, c + 1, c) = r[0];
        }
      } else {
        for (int i = 0; i < n; ++i) {
          PseudoRhs &rs = it.st[(size_t)i];
          MvPtr w = view(*it.V, vcols[(size_t)i], 1);
          MvPtr Q = it.basis(rs, 0, c + 1);
          S->ortho.project_and_normalize(*w, *Q, h.data(), c + 1, r.data(), 1);
          for (int q = 0; q <= c; ++q) it.Hat(rs, q, c) = h[(size_t)q];
          it.Hat(rs, c + 1, c) = r[0];
        }
      }
      S->t_ortho += since(t0);
      update_lsqr(it);
      it.cur_dim += 1;
    }
  }

  void update_lsqr(PseudoIter &it) {  // updateLSQR (:876-915), Givens per right-hand side
    const int c = it.cur_dim;
    for (PseudoRhs &r : it.st) {
      for (int j = 0; j < c; ++j) {
        const double x = it.Hat(r, j, c), y = it.Hat(r, j + 1, c);
        it.Hat(r, j, c) = r.cs[(size_t)j] * x + r.sn[(size_t)j] * y;
        it.Hat(r, j + 1, c) = r.cs[(size_t)j] * y - r.sn[(size_t)j] * x;
      }
      rotg(it.Hat(r, c, c), it.Hat(r, c + 1, c), r.cs[(size_t)c], r.sn[(size_t)c]);
      it.Hat(r, c + 1, c) = 0.0;
      const double x = r.z[(size_t)c], y = r.z[(size_t)c + 1];
      r.z[(size_t)c] = r.cs[(size_t)c] * x + r.sn[(size_t)c] * y;
      r.z[(size_t)c + 1] = r.cs[(size_t)c] * y - r.sn[(size_t)c] * x;
    }
  }

  // Fresh states: R's columns normalised one by one into slot column 0 (:1340-1360).
  void start_states(PseudoIter &it, migmres_mv &R) {
    const int n = R.ncols;
    it.st.assign((size_t)n, PseudoRhs());
    for (int i = 0; i < n; ++i) {
      PseudoRhs &r = it.st[(size_t)i];
      r.slot = i;
      r.H.assign((size_t)(it.nb + 1) * it.nb, 0.0);
      r.z.assign((size_t)it.nb + 1, 0.0);
      r.cs.assign((size_t)it.nb + 1, 0.0);
      r.sn.assign((size_t)it.nb + 1, 0.0);
      MvPtr src = view(R, i, 1);
      MvPtr v0 = view(*it.V, it.col(r, 0), 1);
      mv_assign(*src, *v0);
      double b = 0.0;
      if (S->ortho.normalize(*v0, &b, 1) != 1)
        throw Error(MIGMRES_ESTATE, "PseudoBlockGmresSolMgr: failed to compute initial block of orthonormal vectors");
      r.z[0] = b;
    }
    it.cur_dim = 0;
  }

  // PseudoBlockGmresSolMgr::solve (BelosPseudoBlockGmresSolMgr.hpp:1268-1668)
  bool solve() {
    const Params &p = S->p;
    int block = p.block_size;
    const int numrhs = lp.B->ncols;
    int start = 0, to_solve = numrhs;
    int cur = std::min(to_solve, block);
    block = cur;
    std::vector<int> idx;
    for (int i = 0; i < cur; ++i) idx.push_back(start + i);
    lp.set_ls_index(idx);
    bool converged = true;
    S->loa = false;
    S->ortho.dgks = p.ortho == "DGKS";
    S->ortho.dep_tol = p.dgks_dep_tol();
    PseudoIter it;
    it.nb = p.num_blocks;
    it.nslots = block;
    it.V = MvPtr(mv_create(lp.X->ctx, lp.X->n_global, lp.X->n_local, block * (p.num_blocks + 1)));
    rhs_nb = p.num_blocks;
    rhs_fast.clear();
    rhs_fast.resize((size_t)block);
    while (to_solve > 0) {
      auto ts0 = Clock::now();
      std::vector<int> cur_idx(idx.begin(), idx.begin() + cur);
      it.num_iters = 0;
      {
        MvPtr R0(mv_view(&lp.pr0(), idx.data(), (int)idx.size()));
        start_states(it, *R0);
      }
      S->t_setup += since(ts0);
      int restarts = 0;
      while (true) {
        iterate(it);
        if (conv_passed) {
          if (exp_conv().loss) {
            S->loa = true;
            converged = false;
          }
          const std::vector<int> conv_idx = exp_conv().ind;
          if (conv_idx.size() == cur_idx.size()) break;
          // deflate the converged right-hand sides (:1397-1466)
          lp.set_curr_ls();
          std::vector<int> keep, def;
          for (size_t i = 0; i < cur_idx.size(); ++i) {
            const bool found = std::find(conv_idx.begin(), conv_idx.end(), cur_idx[i]) != conv_idx.end();
            (found ? def : keep).push_back((int)i);
          }
          if (it.cur_dim) {
            MvPtr upd = update(it);
            MvPtr dupd(mv_view(upd.p, def.data(), (int)def.size()));
            lp.set_ls_index(conv_idx);
            if (lp.RP) {
              MvPtr ru = lp.clone(dupd->ncols);
              lp.prec(*lp.RP, *dupd, *ru);
              mv_add_mv(1.0, *lp.curX, 1.0, *ru, *lp.curX);
            } else {
              mv_add_mv(1.0, *lp.curX, 1.0, *dupd, *lp.curX);
            }
          }
          std::vector<int> kept_idx;
          std::vector<PseudoRhs> kept;
          for (int i : keep) {
            kept_idx.push_back(cur_idx[(size_t)i]);
            kept.push_back(std::move(it.st[(size_t)i]));
          }
          cur_idx = kept_idx;
          lp.set_ls_index(cur_idx);
          it.st = std::move(kept);
          ++S->n_deflations;
        } else if (mi_passed) {
          converged = false;
          break;
        } else if (it.cur_dim == it.nb) {
          if (restarts >= p.max_restarts) {
            converged = false;
            break;
          }
          ++restarts;
          auto tr0 = Clock::now();
          lp.update_solution(update(it));
          MvPtr R0 = lp.clone((int)cur_idx.size());
          lp.curr_prec_res_vec(*R0);
          start_states(it, *R0);
          S->t_restart += since(tr0);
        } else {
          throw Error(MIGMRES_ESTATE, "PseudoBlockGmresSolMgr: invalid return from iterate()");
        }
      }
      if (exp_conv().have_soln) {
        ResTest &e = exp_conv();
        mv_add_mv(0.0, *e.cur_soln, 1.0, *e.cur_soln, *lp.curX);
      } else {
        lp.update_solution(update(it));
      }
      lp.set_curr_ls();
      S->n_restarts += restarts;
      start += cur;
      to_solve -= cur;
      if (to_solve > 0) {
        cur = std::min(to_solve, block);
        block = cur;
        idx.clear();
        for (int i = 0; i < cur; ++i) idx.push_back(start + i);
        if (p.def_quorum > block) imp.quorum = exp.quorum = block;
        lp.set_ls_index(idx);
      }
    }
    MIG_HIP(hipStreamSynchronize(lp.X->ctx->stream));
    S->num_iters = mi_n_iters;
    const std::vector<double> *tv = &imp.testvector;
    if (seq && !exp.testvector.empty()) tv = &exp.testvector;
    S->achieved_tol = tv->empty() ? 0.0 : *std::max_element(tv->begin(), tv->end());
    return converged && !S->loa;
  }
};

}  // namespace


extern "C" int migmres_solver_create(migmres_ctx *ctx, migmres_solver **out) {
  return guard([&] {
    MIG_CHECK(ctx && out, "bad solver arguments");
    auto *s = new migmres_solver();
    s->ctx = ctx;
    *out = s;
  });
}

// SolverFactory names (Belos_Details_EBelosSolverType.cpp:55-100, reviseParameterListForAlias
// :213-222): "GMRES" / "PSEUDOBLOCK GMRES" -> PseudoBlockGmresSolMgr, "BLOCK GMRES" ->
// BlockGmresSolMgr, "FLEXIBLE GMRES" -> BlockGmresSolMgr with "Flexible Gmres" = true.
extern "C" int migmres_solver_create_named(migmres_ctx *ctx, const char *name, migmres_solver **out) {
  return guard([&] {
    MIG_CHECK(ctx && out && name, "bad solver arguments");
    std::string n(name);
    for (char &ch : n) ch = (char)std::toupper((unsigned char)ch);
    bool pseudo = false, flexible = false;
    if (n == "GMRES" || n == "PSEUDOBLOCK GMRES" || n == "PSEUDO BLOCK GMRES" || n == "PSEUDOBLOCKGMRES")
      pseudo = true;
    else if (n == "FLEXIBLE GMRES")
      flexible = true;
    else if (n != "BLOCK GMRES")
      throw Error(MIGMRES_EINVAL, "solver \"" + std::string(name) + "\" is not implemented on the device path");
    auto *s = new migmres_solver();
    s->ctx = ctx;
    s->p.pseudo = pseudo;
    s->p.flexible = flexible;
    if (pseudo) s->p.ortho = "ICGS";  // BelosPseudoBlockGmresSolMgr.hpp:506
    *out = s;
  });
}

extern "C" int migmres_solver_destroy(migmres_solver *s) {
  return guard([&] { delete s; });
}

extern "C" int migmres_solver_set_int(migmres_solver *s, const char *name, long long v) {
  return guard([&] {
    const std::string n(name);
    if (n == "Block Size") {
      MIG_CHECK(v > 0, "\"Block Size\" must be strictly positive");
      s->p.block_size = (int)v;
    } else if (n == "Num Blocks") {
      MIG_CHECK(v > 0, "\"Num Blocks\" must be strictly positive");
      s->p.num_blocks = (int)v;
    } else if (n == "Maximum Iterations") {
      s->p.max_iters = (int)v;
    } else if (n == "Maximum Restarts") {
      s->p.max_restarts = (int)v;
    } else if (n == "Adaptive Block Size") {
      s->p.adaptive = v != 0;
    } else if (n == "Flexible Gmres") {
      MIG_CHECK(!s->p.pseudo, "\"Flexible Gmres\" is not a PseudoBlockGmresSolMgr parameter");
      s->p.flexible = v != 0;
    } else if (n == "Deflation Quorum") {
      MIG_CHECK(s->p.pseudo, "\"Deflation Quorum\" is a PseudoBlockGmresSolMgr parameter");
      MIG_CHECK(v >= 1, "\"Deflation Quorum\" must be positive");
      s->p.def_quorum = (int)v;
    } else if (n == "Explicit Residual Test") {
      s->p.exp_res_test = v != 0;
    } else if (n == "Verbosity") {
      s->p.verbosity = (int)v;
    } else if (n == "Output Frequency") {
      s->p.output_freq = (int)v;
    } else if (n == "Output Style") {
      s->p.output_style = (int)v;
    } else if (n == "Show Maximum Residual Norm Only") {
      s->p.show_max_res_norm_only = v != 0;
    } else {
      throw Error(MIGMRES_EINVAL, "unknown integer parameter \"" + n + "\"");
    }
  });
}

extern "C" int migmres_solver_set_double(migmres_solver *s, const char *name, double v) {
  return guard([&] {
    const std::string n(name);
    if (n == "Convergence Tolerance")
      s->p.tol = v;
    else if (n == "Orthogonalization Constant")
      s->p.ortho_kappa = v;
    else
      throw Error(MIGMRES_EINVAL, "unknown double parameter \"" + n + "\"");
  });
}

extern "C" int migmres_solver_set_string(migmres_solver *s, const char *name, const char *v) {
  return guard([&] {
    const std::string n(name), val(v);
    if (n == "Orthogonalization") {
      MIG_CHECK(val == "DGKS" || val == "ICGS" || val == "IMGS",
                "\"Orthogonalization\" must be either \"DGKS\", \"ICGS\", or \"IMGS\"");
      MIG_CHECK(val == "ICGS" || val == "DGKS", "\"IMGS\" is not implemented on the device path");
      s->p.ortho = val;
    } else if (n == "Implicit Residual Scaling" || n == "Explicit Residual Scaling") {
      // convertStringToScaleType (BelosTypes.cpp:106-123); "User Provided" needs a user norm
      MIG_CHECK(val == "Norm of Initial Residual" || val == "Norm of Preconditioned Initial Residual" ||
                    val == "Norm of RHS" || val == "None",
                "invalid residual scaling type \"" + val + "\"");
      (n[0] == 'I' ? s->p.imp_scale : s->p.exp_scale) = val;
    } else if (n == "Timer Label") {
      s->p.timer_label = val;
    } else {
      throw Error(MIGMRES_EINVAL, "unknown string parameter \"" + n + "\"");
    }
  });
}

namespace {
// the parameter list of a solver (names/types of BelosBlockGmresSolMgr.hpp:438-486 and
// BelosPseudoBlockGmresSolMgr.hpp:494-507) as "name\ttype\tvalue" lines
std::string param_text(const Params &p) {
  std::string out;
  char num[64];
  auto line = [&](const char *name, const char *type, const std::string &v) {
    out += name;
    out += '\t';
    out += type;
    out += '\t';
    out += v;
    out += '\n';
  };
  auto i = [&](const char *name, long long v) {
    std::snprintf(num, sizeof num, "%lld", v);
    line(name, "int", num);
  };
  auto b = [&](const char *name, bool v) { line(name, "bool", v ? "true" : "false"); };
  std::snprintf(num, sizeof num, "%.17g", p.tol);
  line("Convergence Tolerance", "double", num);
  i("Maximum Restarts", p.max_restarts);
  i("Maximum Iterations", p.max_iters);
  i("Num Blocks", p.num_blocks);
  i("Block Size", p.block_size);
  if (!p.pseudo) b("Adaptive Block Size", p.adaptive);
  i("Verbosity", p.verbosity);
  i("Output Frequency", p.output_freq);
  if (p.pseudo) i("Deflation Quorum", p.def_quorum);
  line("Orthogonalization", "string", p.ortho);
  if (!p.pseudo) b("Flexible Gmres", p.flexible);
  b("Explicit Residual Test", p.exp_res_test);
  line("Implicit Residual Scaling", "string", p.imp_scale);
  line("Explicit Residual Scaling", "string", p.exp_scale);
  i("Output Style", p.output_style);
  b("Show Maximum Residual Norm Only", p.show_max_res_norm_only);
  line("Timer Label", "string", p.timer_label);
  std::snprintf(num, sizeof num, "%.17g", p.ortho_kappa);
  line("Orthogonalization Constant", "double", num);
  return out;
}
void put_text(const std::string &t, char *buf, int len, int *needed) {
  if (needed) *needed = (int)t.size() + 1;
  if (buf && len > 0) {
    const size_t n = std::min(t.size(), (size_t)len - 1);
    std::memcpy(buf, t.data(), n);
    buf[n] = '\0';
  }
}
}  // namespace

extern "C" int migmres_solver_valid_parameters(const migmres_solver *s, char *buf, int len, int *needed) {
  return guard([&] {
    MIG_CHECK(s, "bad arguments");
    Params d;
    d.pseudo = s->p.pseudo;
    if (d.pseudo) d.ortho = "ICGS";  // BelosPseudoBlockGmresSolMgr.hpp:506
    put_text(param_text(d), buf, len, needed);
  });
}
extern "C" int migmres_solver_current_parameters(const migmres_solver *s, char *buf, int len, int *needed) {
  return guard([&] {
    MIG_CHECK(s, "bad arguments");
    put_text(param_text(s->p), buf, len, needed);
  });
}
extern "C" int migmres_solver_get_int(const migmres_solver *s, const char *name, long long *v) {
  return guard([&] {
    MIG_CHECK(s && name && v, "bad arguments");
    const std::string n(name);
    const Params &p = s->p;
    if (n == "Block Size") *v = p.block_size;
    else if (n == "Num Blocks") *v = p.num_blocks;
    else if (n == "Maximum Iterations") *v = p.max_iters;
    else if (n == "Maximum Restarts") *v = p.max_restarts;
    else if (n == "Adaptive Block Size" && !p.pseudo) *v = p.adaptive;
    else if (n == "Flexible Gmres" && !p.pseudo) *v = p.flexible;
    else if (n == "Deflation Quorum" && p.pseudo) *v = p.def_quorum;
    else if (n == "Explicit Residual Test") *v = p.exp_res_test;
    else if (n == "Verbosity") *v = p.verbosity;
    else if (n == "Output Frequency") *v = p.output_freq;
    else if (n == "Output Style") *v = p.output_style;
    else if (n == "Show Maximum Residual Norm Only") *v = p.show_max_res_norm_only;
    else throw Error(MIGMRES_EINVAL, "unknown integer parameter \"" + n + "\"");
  });
}
extern "C" int migmres_solver_get_double(const migmres_solver *s, const char *name, double *v) {
  return guard([&] {
    MIG_CHECK(s && name && v, "bad arguments");
    const std::string n(name);
    if (n == "Convergence Tolerance") *v = s->p.tol;
    else if (n == "Orthogonalization Constant") *v = s->p.ortho_kappa;
    else throw Error(MIGMRES_EINVAL, "unknown double parameter \"" + n + "\"");
  });
}
extern "C" int migmres_solver_get_string(const migmres_solver *s, const char *name, char *v, int len) {
  return guard([&] {
    MIG_CHECK(s && name && v && len > 0, "bad arguments");
    const std::string n(name);
    const std::string &val = n == "Orthogonalization" ? s->p.ortho
                             : n == "Implicit Residual Scaling" ? s->p.imp_scale
                             : n == "Explicit Residual Scaling" ? s->p.exp_scale
                             : n == "Timer Label" ? s->p.timer_label
                             : throw Error(MIGMRES_EINVAL, "unknown string parameter \"" + n + "\"");
    put_text(val, v, len, nullptr);
  });
}
extern "C" int migmres_solver_reset(migmres_solver *s, int type) {
  return guard([&] {
    MIG_CHECK(s, "bad arguments");
    MIG_CHECK((type & ~(MIGMRES_RESET_PROBLEM | MIGMRES_RESET_RECYCLE)) == 0, "reset: unknown ResetType bits");
    if (type & MIGMRES_RESET_PROBLEM) {
      s->num_iters = 0;
      s->achieved_tol = 0.0;
      s->loa = false;
      s->history.clear();
      s->hist_cols = 0;
      s->n_apply = s->n_explicit = s->n_restarts = s->n_block_iters = s->n_prec = s->n_deflations = 0;
      s->fast.gram_calls = s->fast.gram_skips = s->fast.gram_singles = s->fast.gram_mixed = 0;
    }
  });
}
extern "C" int migmres_solver_set_user_conv_test(migmres_solver *s, migmres_status_fn fn, void *user, int combo) {
  return guard([&] {
    MIG_CHECK(s, "bad arguments");
    MIG_CHECK(s->p.pseudo, "setUserConvStatusTest() has not been overridden for BlockGmresSolMgr "
                           "(BelosSolverManager.hpp:147-155); use the pseudo-block solver");
    MIG_CHECK(combo == MIGMRES_COMBO_AND || combo == MIGMRES_COMBO_OR || combo == MIGMRES_COMBO_SEQ,
              "combo must be MIGMRES_COMBO_AND, _OR or _SEQ");
    s->user_test = fn;
    s->user_data = user;
    s->user_combo = combo;
  });
}

static int solve_impl(migmres_solver *s, migmres_crs *A, migmres_op *Aop, migmres_mv *X, const migmres_mv *B,
                      int *converged) {
  return guard([&] {
    MIG_CHECK(s && (A || Aop) && X && B, "bad solve arguments");
    if (!A && Aop->crs) A = Aop->crs;
    const int a_local = A ? A->n_local : Aop->n_local;
    MIG_CHECK(s->p.ortho == "ICGS" || s->p.ortho == "DGKS", "\"Orthogonalization\" must be \"ICGS\" or \"DGKS\"");
    MIG_CHECK(X->ncols == B->ncols && X->n_local == a_local && B->n_local == a_local,
              "LinearProblem: inconsistent X/B/A shapes");
    s->history.clear();
    s->n_apply = s->n_explicit = s->n_restarts = s->n_block_iters = s->n_prec = s->n_deflations = 0;
    s->fast.gram_calls = s->fast.gram_skips = s->fast.gram_singles = s->fast.gram_mixed = 0;
    s->t_spmm = s->t_ortho = s->t_lsq = s->t_check = s->t_restart = s->t_setup = 0.0;
    const double comm0 = s->ctx->comm_seconds;
    auto t0 = Clock::now();
    for (migmres_prec *M : {s->left, s->right})
      MIG_CHECK(!M || M->n_local() == a_local, "preconditioner and operator row maps differ");
    bool ok;
    if (s->p.pseudo) {
      MIG_CHECK(s->p.def_quorum <= s->p.block_size,
                "\"Deflation Quorum\" must not be larger than \"Block Size\" (BelosPseudoBlockGmresSolMgr.hpp:994-999)");
      PseudoEngine E(s, s->p.tol, s->p.max_iters);
      E.lp.S = s;
      E.lp.A = A;
      E.lp.Aop = A ? nullptr : Aop;
      E.lp.X = X;
      E.lp.B = const_cast<migmres_mv *>(B);
      E.lp.LP = s->left;
      E.lp.RP = s->right;
      E.setup_pseudo_tests(s->left != nullptr);
      E.lp.set_problem();
      ok = E.solve();
    } else {
      Engine E(s, s->p.tol, s->p.max_iters);
      E.lp.S = s;
      E.lp.A = A;
      E.lp.Aop = A ? nullptr : Aop;
      E.lp.X = X;
      E.lp.B = const_cast<migmres_mv *>(B);
      E.lp.LP = s->left;
      E.lp.RP = s->right;
      E.setup_status_tests(s->left != nullptr, s->right != nullptr);
      E.lp.set_problem();
      ok = E.solve();
    }
    s->t_total = since(t0);
    s->t_comm = s->ctx->comm_seconds - comm0;
    if (converged) *converged = ok ? 1 : 0;
  });
}

extern "C" int migmres_solver_solve(migmres_solver *s, migmres_crs *A, migmres_mv *X,
                                    const migmres_mv *B, int *converged) {
  if (!A) return guard([] { throw Error(MIGMRES_EINVAL, "bad solve arguments"); });
  return solve_impl(s, A, nullptr, X, B, converged);
}
extern "C" int migmres_solver_solve_op(migmres_solver *s, migmres_op *A, migmres_mv *X, const migmres_mv *B,
                                       int *converged) {
  if (!A) return guard([] { throw Error(MIGMRES_EINVAL, "bad solve arguments"); });
  return solve_impl(s, nullptr, A, X, B, converged);
}
extern "C" int migmres_solver_set_prec_op(migmres_solver *s, int side, migmres_op *M) {
  return guard([&] {
    MIG_CHECK(s, "set_prec_op: null solver");
    MIG_CHECK(side == MIGMRES_LEFT_PREC || side == MIGMRES_RIGHT_PREC, "set_prec_op: side must be left (0) or right (1)");
    std::unique_ptr<migmres_prec> &w = s->uprec[side == MIGMRES_LEFT_PREC ? 0 : 1];
    migmres_prec *&slot = side == MIGMRES_LEFT_PREC ? s->left : s->right;
    if (!M) {
      if (slot == w.get()) slot = nullptr;
      w.reset();
      return;
    }
    w.reset(new migmres_prec());
    w->ctx = M->ctx;
    w->kind = 2;
    w->uop = M;
    slot = w.get();
  });
}

extern "C" int migmres_solver_set_prec(migmres_solver *s, int side, migmres_prec *M) {
  return guard([&] {
    MIG_CHECK(s, "set_prec: null solver");
    MIG_CHECK(side == MIGMRES_LEFT_PREC || side == MIGMRES_RIGHT_PREC, "set_prec: side must be left (0) or right (1)");
    (side == MIGMRES_LEFT_PREC ? s->left : s->right) = M;
  });
}

extern "C" int migmres_solver_num_iters(const migmres_solver *s, int *it) {
  return guard([&] { *it = s->num_iters; });
}
extern "C" int migmres_solver_achieved_tol(const migmres_solver *s, double *tol) {
  return guard([&] { *tol = s->achieved_tol; });
}
extern "C" int migmres_solver_loa_detected(const migmres_solver *s, int *loa) {
  return guard([&] { *loa = s->loa ? 1 : 0; });
}
extern "C" int migmres_solver_history(const migmres_solver *s, double *out, int *nrows, int *ncols) {
  return guard([&] {
    const int nc = s->hist_cols > 0 ? s->hist_cols : 1;
    *ncols = s->hist_cols;
    *nrows = s->hist_cols > 0 ? (int)(s->history.size() / nc) : 0;
    if (out) std::memcpy(out, s->history.data(), sizeof(double) * s->history.size());
  });
}
extern "C" int migmres_solver_counters(const migmres_solver *s, long long *out, int n) {
  return guard([&] {
    const long long v[11] = {s->n_apply,       s->n_explicit, s->n_restarts,        s->ortho.sing_count,
                             s->n_block_iters, s->n_prec,     s->n_deflations,      s->fast.gram_calls,
                             s->fast.gram_skips, s->fast.gram_singles, s->fast.gram_mixed};
    for (int i = 0; i < n && i < 11; ++i) out[i] = v[i];
  });
}
extern "C" int migmres_solver_timers(const migmres_solver *s, double *out, int n) {
  return guard([&] {
    const double v[8] = {s->t_total, s->t_spmm, s->t_ortho, s->t_lsq, s->t_comm, s->t_check, s->t_restart, s->t_setup};
    for (int i = 0; i < n && i < 8; ++i) out[i] = v[i];
  });
}

// ICGS entry points on caller-provided multivectors (the OrthoManager drop-in).
static Icgs g_icgs_default;
static Icgs make_dgks() {
  Icgs m;
  m.dgks = true;
  return m;
}
static Icgs g_dgks_default = make_dgks();
extern "C" int migmres_dgks_project_normalize(migmres_mv *X, const migmres_mv *Q, double *C, int ldc,
                                              double *B, int ldb, int *rank) {
  return guard([&] {
    MIG_CHECK(X && Q && C && B && rank, "dgks_project_normalize: null argument");
    *rank = g_dgks_default.project_and_normalize(*X, *const_cast<migmres_mv *>(Q), C, ldc, B, ldb);
  });
}
extern "C" int migmres_dgks_normalize(migmres_mv *X, double *B, int ldb, int *rank) {
  return guard([&] {
    MIG_CHECK(X && B && rank, "dgks_normalize: null argument");
    *rank = g_dgks_default.normalize(*X, B, ldb);
  });
}
extern "C" int migmres_icgs_project_normalize(migmres_mv *X, const migmres_mv *Q, double *C, int ldc,
                                              double *B, int ldb, int *rank) {
  return guard([&] {
    MIG_CHECK(X && Q && rank, "bad ICGS arguments");
    *rank = g_icgs_default.project_and_normalize(*X, *const_cast<migmres_mv *>(Q), C, ldc, B, ldb);
  });
}
extern "C" int migmres_icgs_normalize(migmres_mv *X, double *B, int ldb, int *rank) {
  return guard([&] {
    MIG_CHECK(X && rank, "bad ICGS arguments");
    *rank = g_icgs_default.normalize(*X, B, ldb);
    MIG_HIP(hipStreamSynchronize(X->ctx->stream));
  });
}
