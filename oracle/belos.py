"""Belos Block GMRES restatement (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Mirrors, operation by operation, the reference solver stack for double/Epetra:
  ICGSOrthoManager   belos/src/BelosICGSOrthoManager.hpp
  BlockGmresIter     belos/src/BelosBlockGmresIter.hpp
  StatusTestImpResNorm / MaxIters / Combo(OR)
                     belos/src/BelosStatusTestImpResNorm.hpp, BelosStatusTestMaxIters.hpp,
                     BelosStatusTestCombo.hpp
  LinearProblem      belos/src/BelosLinearProblem.hpp
  BlockGmresSolMgr   belos/src/BelosBlockGmresSolMgr.hpp
Multivectors are numpy arrays (rows x columns); the dense coefficient matrices are the
column-major Teuchos::SerialDenseMatrix blocks of the reference, held as 2-D arrays.
"""

import math

import numpy as np

from . import epetra

EPS = np.finfo(np.float64).eps
ICGS_BLK_TOL = 10.0 * math.sqrt(EPS)   # BelosICGSOrthoManager.hpp:565-568
ICGS_SING_TOL = 10.0 * EPS             # BelosICGSOrthoManager.hpp:570-573
ICGS_MAX_STEPS = 2                     # BelosICGSOrthoManager.hpp:561-562


class OrthoFailure(Exception):
    """GmresIterationOrthoFailure (BelosGmresIteration.hpp)."""


class RandomSource:
    """MvRandom stand-in: a deterministic Epetra MINSTD stream.  The reference seeds each
    new multivector from std::rand(), so this path is reproducible only up to the seed."""

    def __init__(self, seed=12345):
        self.seed = seed

    def vec(self, n):
        v, self.seed = epetra.epetra_random_mv(self.seed, n, 1)
        return v[:, 0].copy()


# Summation order of the inner products (test infrastructure): "blas" is the restatement's
# default; "reversed" sums the same products over the rows in reverse order.  Running the
# oracle both ways measures how far rounding alone moves a solve's residual history -- the
# yardstick for the GPU's differently ordered (blocked, MFMA) sums (tests/test_gpu_solver.py).
SUM_ORDER = "blas"


class summation_order:
    """with summation_order("reversed"): ... -- the oracle's inner products in another order."""

    def __init__(self, order):
        self.order = order

    def __enter__(self):
        global SUM_ORDER
        self.prev, SUM_ORDER = SUM_ORDER, self.order
        return self

    def __exit__(self, *exc):
        global SUM_ORDER
        SUM_ORDER = self.prev


def _tn(Q, X):
    """Q^T X (MvTransMv)."""
    if SUM_ORDER == "reversed":
        return Q[::-1].T @ X[::-1]
    return Q.T @ X


def _dot(a, b):
    if SUM_ORDER == "reversed":
        return float(np.dot(a[::-1], b[::-1]))
    return float(np.dot(a, b))


def _coldots(X, Y):
    if SUM_ORDER == "reversed":
        return np.einsum("ij,ij->j", X[::-1], Y[::-1])
    return np.einsum("ij,ij->j", X, Y)


# MultiVecTraits operations on host arrays (rows x columns), as the Epetra adapter maps them
# (belos/epetra/src/BelosEpetraAdapter.hpp: MvTimesMatAddMv -> Epetra_MultiVector::Multiply('N',
# 'N'), MvTransMv -> Multiply('T','N'), MvDot -> Dot, MvNorm -> Norm1/Norm2/NormInf;
# epetra/src/Epetra_MultiVector.cpp:1936-2083, 1123-1156, 1547-1577).  The ICGS restatement
# below uses the same products (_tn, Q @ C, _coldots); these are what
# tests/test_oracle_pins.py pins to Epetra's own MultiVector known answers.
def mv_times_mat_add_mv(alpha, A, B, beta, C):
    """C <- alpha A B + beta C  (Multiply('N','N', alpha, A, B, beta))."""
    return alpha * (A @ B) + beta * C


def mv_trans_mv(alpha, A, B, beta=0.0, C=None):
    """alpha A^T B + beta C  (Multiply('T','N', alpha, A, B, beta))."""
    out = alpha * _tn(A, B)
    return out if C is None else out + beta * C


def mv_dot(A, B):
    return _coldots(A, B)


def mv_norm(A, kind="2"):
    if kind == "1":
        return np.abs(A).sum(axis=0)
    if kind == "inf":
        return np.abs(A).max(axis=0)
    return np.sqrt(_coldots(A, A))


# ---------------------------------------------------------------------------
# ICGS
# ---------------------------------------------------------------------------


class ICGS:
    """ICGSOrthoManager with the default 2 passes and tolerances."""

    def __init__(self, rng=None, steps=ICGS_MAX_STEPS, blk_tol=ICGS_BLK_TOL, sing_tol=ICGS_SING_TOL):
        self.steps = steps
        self.blk_tol = blk_tol
        self.sing_tol = sing_tol
        self.rng = rng or RandomSource()
        self.counters = {"blkOrthoSing": 0}

    # projectAndNormalizeWithMxImpl  (BelosICGSOrthoManager.hpp:646-821)
    def project_and_normalize(self, X, Q, C, B):
        """X (N x k) is overwritten; C (L x k) and B (k x k) receive the coefficients.
        Returns the rank."""
        xc = X.shape[1]
        if xc == 1:
            self._blk_ortho1(X, Q, C)
            d = _dot(X[:, 0], X[:, 0])
            B[0, 0] = math.sqrt(abs(d))
            if abs(B[0, 0]) > 0.0:
                X *= 1.0 / B[0, 0]
            return 1
        tmpX = X.copy()
        dep = self._blk_ortho(X, Q, C)
        if dep:
            rank = self._blk_ortho_sing(tmpX, Q, C, B)
            X[:] = tmpX
        else:
            rank = self.find_basis(X, B, complete_basis=False)
            if rank < xc:
                rank = self._blk_ortho_sing(tmpX, Q, C, B)
                X[:] = tmpX
        return rank

    def normalize(self, X, B):
        """normalize (BelosICGSOrthoManager.hpp:828-839) = findBasis(completeBasis=true)."""
        return self.find_basis(X, B, complete_basis=True)

    def _blk_ortho1(self, X, Q, C):
        """blkOrtho1 (BelosICGSOrthoManager.hpp:1231-1322), no mass operator."""
        C[:] = _tn(Q, X)
        X -= Q @ C
        for _ in range(1, self.steps):
            C2 = _tn(Q, X)
            C += C2
            X -= Q @ C2
        return False

    def _blk_ortho(self, X, Q, C):
        """blkOrtho (BelosICGSOrthoManager.hpp:1328-1445)."""
        old = _coldots(X, X)
        C[:] = _tn(Q, X)
        X -= Q @ C
        for _ in range(1, self.steps):
            C2 = _tn(Q, X)
            C += C2
            X -= Q @ C2
        new = _coldots(X, X)
        return bool(np.any(np.abs(new) < np.abs(old * self.blk_tol)))

    def find_basis(self, X, B, complete_basis):
        """findBasis (BelosICGSOrthoManager.hpp:936-1225), howMany = all columns."""
        xc = X.shape[1]
        for j in range(xc):
            Xj = X[:, j]
            prevX = X[:, :j]
            add_vec = False
            old_xj = Xj.copy() if j > 0 else None
            old_dot = _dot(Xj, Xj)
            if old_dot < 0.0:
                raise ValueError("negative definiteness in inner product")
            product = np.zeros(j)
            if j > 0:
                for i in range(self.steps):
                    P2 = _tn(prevX, Xj)
                    Xj -= prevX @ P2
                    product = P2.copy() if i == 0 else product + P2
                new_dot = _dot(Xj, old_xj)
            else:
                new_dot = old_dot
            if complete_basis:
                if abs(new_dot) < abs(self.sing_tol * old_dot):
                    add_vec = True
                    t = self.rng.vec(X.shape[0])
                    old_dot = _dot(t, t)
                    for _ in range(self.steps):
                        if j > 0:
                            pr = _tn(prevX, t)
                            t -= prevX @ pr
                    new_dot = _dot(t, t)
                    if abs(new_dot) >= abs(old_dot * self.sing_tol):
                        Xj[:] = t
                    else:
                        return j
            else:
                if abs(new_dot) < abs(old_dot * self.blk_tol):
                    return j
            diag = math.sqrt(abs(new_dot))
            Xj *= 1.0 / diag
            B[j, j] = 0.0 if add_vec else diag
            if not add_vec:
                B[:j, j] = product
        return xc

    def _blk_ortho_sing(self, X, Q, C, B):
        """blkOrthoSing (BelosICGSOrthoManager.hpp:1449-1701), kept faithful including its
        use of `newDot` before assignment in the dependency test (it is initialised to zero
        once and only refreshed on the random-vector path)."""
        self.counters["blkOrthoSing"] += 1
        xc = X.shape[1]
        new_dot = 0.0
        for j in range(xc):
            Qs = [Q] + ([X[:, :j]] if j > 0 else [])
            Cs = [C] + ([B] if j > 0 else [])
            Xj = X[:, j]
            old_dot = _dot(Xj, Xj)
            for Qi, Ci in zip(Qs, Cs):
                nq = Qi.shape[1]
                Ci[:nq, j] = _tn(Qi, Xj)
                Xj -= Qi @ Ci[:nq, j]
            for _ in range(1, self.steps):
                for Qi, Ci in zip(Qs, Cs):
                    nq = Qi.shape[1]
                    C2 = _tn(Qi, Xj)
                    Ci[:nq, j] += C2
                    Xj -= Qi @ C2
            dep = abs(new_dot) < abs(old_dot * self.sing_tol)
            if not dep:
                diag = math.sqrt(abs(new_dot))
                Xj *= 1.0 / diag
                B[j, j] = diag
            else:
                t = self.rng.vec(X.shape[0])
                old_dot = _dot(t, t)
                for _ in range(self.steps):
                    for Qi in Qs:
                        pr = _tn(Qi, t)
                        t -= Qi @ pr
                new_dot = _dot(t, t)
                if abs(new_dot) >= abs(old_dot * self.sing_tol):
                    diag = math.sqrt(abs(new_dot))
                    B[j, j] = 0.0
                    Xj[:] = (1.0 / diag) * t
                else:
                    return j
        return xc


# ---------------------------------------------------------------------------
# Linear problem and status tests
# ---------------------------------------------------------------------------


LP_AUGMENT_SEED = 20250219  # MvRandom stream for augmented right-hand sides


class LinearProblem:
    """BelosLinearProblem (BelosLinearProblem.hpp) with optional left/right preconditioners
    (callables Y = M(X), e.g. oracle.ifpack2.Jacobi)."""

    def __init__(self, A, X, B, left=None, right=None):
        self.A = A          # callable: Y = A(X)
        self.LP, self.RP = left, right
        self.X = np.array(X, dtype=np.float64, copy=True)
        self.B = np.array(B, dtype=np.float64, copy=True)
        self.n_apply = 0
        self.n_prec = 0
        self.ls_num = 0
        self.ls_idx = []
        self.aug_seed = LP_AUGMENT_SEED

    def _op(self, x):
        self.n_apply += 1
        return self.A(x)

    def _prec(self, M, x):
        self.n_prec += 1
        return M(x)

    def apply(self, x):
        """apply (BelosLinearProblem.hpp:989-1072): y = M_L A M_R x."""
        if self.RP is not None:
            x = self._prec(self.RP, x)
        y = self._op(x)
        if self.LP is not None:
            y = self._prec(self.LP, y)
        return y

    def apply_op(self, x):
        """applyOp (BelosLinearProblem.hpp:1075-1086)."""
        return self._op(x)

    def apply_right_prec(self, x):
        """applyRightPrec (BelosLinearProblem.hpp:1103-1114)."""
        if self.RP is not None:
            return self._prec(self.RP, x)
        return 1.0 * x + 0.0 * x

    def set_problem(self):
        """setProblem (BelosLinearProblem.hpp:836-946): R0 = B - A X; PR0 = M_L R0."""
        R = self._op(self.X)
        self.R0 = (-1.0 * R) + (1.0 * self.B)
        self.PR0 = self._prec(self.LP, self.R0) if self.LP is not None else self.R0
        return True

    def set_ls_index(self, idx):
        """setLSIndex (BelosLinearProblem.hpp:642-705).  With -1 entries the block is
        augmented: curX = zeros, curB = random, valid columns copied in (SetBlock)."""
        self.ls_idx = list(idx)
        self.ls_num += 1
        self.vld = [i for i in idx if i >= 0]
        self.new = [j for j, i in enumerate(idx) if i >= 0]
        bs = len(idx)
        if len(self.vld) != bs:
            self.curX = np.zeros((self.X.shape[0], bs))
            self.curB, self.aug_seed = epetra.epetra_random_mv(self.aug_seed, self.B.shape[0], bs)
            self.curB[:, self.new] = self.B[:, self.vld]
            self.curX[:, self.new] = self.X[:, self.vld]
        else:
            self.curX = self.X[:, idx].copy()
            self.curB = self.B[:, idx].copy()

    def set_curr_ls(self):
        """setCurrLS (BelosLinearProblem.hpp:709-739): copy the solved columns back."""
        self.X[:, self.vld] = self.curX[:, self.new]

    def cur_x(self):
        return self.curX

    def cur_b(self):
        return self.curB

    def update_solution(self, update, update_lp):
        """updateSolution (BelosLinearProblem.hpp:743-812): X + M_R update."""
        if update is None:
            return self.curX
        if self.RP is not None:
            update = self._prec(self.RP, update)
        if update_lp:
            self.curX = self.curX + update
            return self.curX
        return self.curX + update

    def curr_res_vec(self, Xs=None):
        """computeCurrResVec (BelosLinearProblem.hpp:1196-1231): R = B - A X."""
        Xs = self.curX if Xs is None else Xs
        R = self._op(Xs)
        return (-1.0 * R) + (1.0 * self.curB)

    def curr_prec_res_vec(self, Xs=None):
        """computeCurrPrecResVec (BelosLinearProblem.hpp:1117-1195): M_L (B - A X)."""
        R = self.curr_res_vec(Xs)
        return self._prec(self.LP, R) if self.LP is not None else R


def _scale_vector(lp, scale_type):
    """firstCallCheckStatusSetup scaling (BelosStatusTestGenResNorm.hpp:643-700,
    BelosStatusTestImpResNorm.hpp:815-845); None for "None" (divide by scalevalue 1)."""
    if scale_type == "Norm of RHS":
        return np.linalg.norm(lp.B, axis=0)
    if scale_type == "Norm of Initial Residual":
        return np.linalg.norm(lp.R0, axis=0)
    if scale_type == "Norm of Preconditioned Initial Residual":
        return np.linalg.norm(lp.PR0, axis=0)
    if scale_type == "None":
        return None
    raise ValueError("invalid residual scaling type %r" % (scale_type,))


SCALE_TYPES = ("Norm of Initial Residual", "Norm of Preconditioned Initial Residual", "Norm of RHS", "None")


class StatusTestMaxIters:
    def __init__(self, max_iters):
        self.max_iters = max_iters
        self.reset()

    def reset(self):
        self.n_iters = 0
        self.status = None

    def check(self, it):
        self.n_iters = it.num_iters
        self.status = self.n_iters >= self.max_iters
        return self.status


class StatusTestImpResNorm:
    """StatusTestImpResNorm with scaling 'Norm of Preconditioned Initial Residual'
    (BelosStatusTestImpResNorm.hpp:492-749, 808-845)."""

    def __init__(self, tol, scale_type="Norm of Preconditioned Initial Residual", quorum=-1):
        self.tol = tol
        self.scale_type = scale_type
        self.quorum = quorum
        self.reset()

    def reset(self):
        self.status = None
        self.ind = []
        self.curr_tol = self.tol
        self.first = True
        self.loss = False
        self.cur_soln = None
        self.cur_ls_num = 0
        self.n_explicit = 0
        self.testvector = None

    def check(self, it):
        lp = it.lp
        if self.first:
            self.first = False
            self.scale = _scale_vector(lp, self.scale_type)
            self.numrhs = lp.B.shape[1]
            self.resvector = np.zeros(self.numrhs)
            self.testvector = np.ones(self.numrhs)
            self.cur_ls_num = lp.ls_num
            self.cur_idx = list(lp.ls_idx)
            self.cur_num_rhs = sum(1 for i in self.cur_idx if 0 <= i < self.numrhs)
        if self.cur_ls_num != lp.ls_num:
            self.cur_ls_num = lp.ls_num
            self.cur_idx = list(lp.ls_idx)
            self.cur_num_rhs = sum(1 for i in self.cur_idx if 0 <= i < self.numrhs)
            self.cur_soln = None
        elif self.status:
            return self.status
        res = it.native_residuals()
        for i, p in enumerate(self.cur_idx):
            if p != -1:
                self.resvector[p] = res[i]
        for p in self.cur_idx:
            if p != -1:
                s = 0.0 if self.scale is None else self.scale[p]
                self.testvector[p] = self.resvector[p] / s / 1.0 if s != 0.0 else self.resvector[p] / 1.0
        ind, lcl = [], []
        for i, p in enumerate(self.cur_idx):
            if p == -1:
                continue
            tv = self.testvector[p]
            if tv > self.curr_tol:
                pass
            elif tv <= self.curr_tol:
                ind.append(p)
                lcl.append(i)
            else:
                self.status = False
                raise FloatingPointError("implicit residual norm is NaN")
        have = len(ind)
        if have:
            self.n_explicit += 1
            upd = it.current_update()
            self.cur_soln = lp.update_solution(upd, False)
            cur_res = lp.curr_res_vec(self.cur_soln)
            tmp_res = np.linalg.norm(cur_res, axis=0)
            tmp_test = []
            for i in range(have):
                s = 0.0 if self.scale is None else self.scale[ind[i]]
                tmp_test.append(tmp_res[lcl[i]] / s / 1.0 if s != 0.0 else tmp_res[lcl[i]] / 1.0)
            have2 = 0
            for i in range(have):
                if tmp_test[i] <= self.tol:
                    ind[have2] = ind[i]
                    have2 += 1
                else:
                    diff = abs(self.testvector[ind[i]] - tmp_test[i])
                    if diff > self.curr_tol:
                        self.loss = True
                        ind[have2] = ind[i]
                        have2 += 1
                    else:
                        self.curr_tol = self.curr_tol - (3.0 / 2.0) * diff
                        while self.curr_tol < 0.0:
                            self.curr_tol += (1.0 / 10.0) * diff
            have = have2
        self.ind = ind[:have]
        need = self.cur_num_rhs if self.quorum == -1 else self.quorum
        self.status = have >= need
        return self.status


class StatusTestGenResNorm:
    """StatusTestGenResNorm, implicit (native residuals) or explicit (||B - A X||) form
    (BelosStatusTestGenResNorm.hpp:455-600, 643-700).  No loss-of-accuracy check."""

    loss = False

    def __init__(self, tol, explicit=False, scale_type="Norm of Preconditioned Initial Residual", quorum=-1):
        self.tol = tol
        self.explicit = explicit
        self.scale_type = scale_type
        self.quorum = quorum
        self.reset()

    def reset(self):
        self.status = None
        self.ind = []
        self.first = True
        self.cur_soln = None
        self.cur_ls_num = 0
        self.n_explicit = 0
        self.testvector = None

    def check(self, it):
        lp = it.lp
        if self.first:
            self.first = False
            self.scale = _scale_vector(lp, self.scale_type)
            self.numrhs = lp.B.shape[1]
            self.resvector = np.zeros(self.numrhs)
            self.testvector = np.ones(self.numrhs)
            self.cur_ls_num = lp.ls_num
            self.cur_idx = list(lp.ls_idx)
            self.cur_num_rhs = sum(1 for i in self.cur_idx if 0 <= i < self.numrhs)
        if self.cur_ls_num != lp.ls_num:
            self.cur_ls_num = lp.ls_num
            self.cur_idx = list(lp.ls_idx)
            self.cur_num_rhs = sum(1 for i in self.cur_idx if 0 <= i < self.numrhs)
            self.cur_soln = None
        elif self.status:
            return self.status
        if self.explicit:
            self.n_explicit += 1
            upd = it.current_update()
            self.cur_soln = lp.update_solution(upd, False)
            res = np.linalg.norm(lp.curr_res_vec(self.cur_soln), axis=0)
        else:
            res = it.native_residuals()
        for i, p in enumerate(self.cur_idx):
            if p != -1:
                self.resvector[p] = res[i]
        for p in self.cur_idx:
            if p != -1:
                s = 0.0 if self.scale is None else self.scale[p]
                self.testvector[p] = self.resvector[p] / s / 1.0 if s != 0.0 else self.resvector[p] / 1.0
        self.ind = []
        for p in self.cur_idx:
            if p == -1:
                continue
            tv = self.testvector[p]
            if tv > self.tol:
                pass
            elif tv <= self.tol:
                self.ind.append(p)
            else:
                self.status = False
                raise FloatingPointError("StatusTestGenResNorm: NaN detected")
        need = self.cur_num_rhs if self.quorum == -1 else self.quorum
        self.status = len(self.ind) >= need
        return self.status


class StatusTestSeq:
    """StatusTestCombo SEQ: later members are checked only when the earlier ones pass
    (BelosStatusTestCombo.hpp:360-380)."""

    loss = False

    def __init__(self, *tests):
        self.tests = tests
        self.status = None

    @property
    def testvector(self):
        return self.tests[0].testvector

    @property
    def n_explicit(self):
        return sum(t.n_explicit for t in self.tests)

    @property
    def ind(self):
        return self.tests[-1].ind

    @property
    def cur_soln(self):
        return self.tests[-1].cur_soln

    def reset(self):
        for t in self.tests:
            t.reset()
        self.status = None

    def check(self, it):
        for t in self.tests:
            if not t.check(it):
                self.status = False
                return False
        self.status = True
        return True


class StatusTestOr:
    """StatusTestCombo OR: every member is evaluated (BelosStatusTestCombo.hpp:314-327)."""

    def __init__(self, *tests):
        self.tests = tests
        self.history = []

    def reset(self):
        for t in self.tests:
            t.reset()

    def check(self, it):
        passed = False
        for t in self.tests:
            if t.check(it):
                passed = True
        imp = self.tests[-1]
        if imp.testvector is not None:
            self.history.append(imp.testvector.copy())
        return passed


# ---------------------------------------------------------------------------
# Block GMRES iteration and solver manager
# ---------------------------------------------------------------------------


class BlockGmresIter:
    """BelosBlockGmresIter.hpp (keepHessenberg=false, so H and R share storage)."""

    def __init__(self, lp, stest, ortho, k, nb):
        self.lp, self.stest, self.ortho = lp, stest, ortho
        self.k, self.nb = k, nb
        n = lp.B.shape[0]
        sd = k * (nb + 1)
        self.V = np.zeros((n, sd))
        self.R = np.zeros((sd, sd - k))
        self.z = np.zeros((sd, k))
        self.beta = np.zeros(sd)
        self.cs = np.zeros(sd)
        self.sn = np.zeros(sd)
        self.cur_dim = 0
        self.num_iters = 0

    def max_subspace_dim(self):
        return self.k * self.nb

    def initialize(self, V0, z0):
        """initializeGmres (BelosBlockGmresIter.hpp:564-653) with curDim = 0."""
        k = self.k
        self.cur_dim = 0
        self.V[:, :k] = 1.0 * V0 + 0.0 * V0
        self.z[:] = 0.0
        self.z[:k, :k] = z0

    def native_residuals(self):
        """getNativeResiduals (BelosBlockGmresIter.hpp:542-557)."""
        c, k = self.cur_dim, self.k
        return np.linalg.norm(self.z[c:c + k, :], axis=0)

    def current_update(self):
        """getCurrentUpdate (BelosBlockGmresIter.hpp:500-535): TRSM then V*y."""
        c, k = self.cur_dim, self.k
        if c == 0:
            return None
        y = self.z[:c, :k].copy()
        Rc = self.R[:c, :c]
        # upper triangular back substitution (BLAS TRSM, left/upper/no-trans/non-unit)
        for i in range(c - 1, -1, -1):
            if i + 1 < c:
                y[i, :] -= Rc[i, i + 1:c] @ y[i + 1:c, :]
            y[i, :] /= Rc[i, i]
        return self.V[:, :c] @ y

    def iterate(self):
        """iterate (BelosBlockGmresIter.hpp:659-766)."""
        k = self.k
        search = k * self.nb
        while (not self.stest.check(self)) and self.cur_dim + k <= search:
            self.num_iters += 1
            lcl = self.cur_dim + k
            c = self.cur_dim
            self.V[:, lcl:lcl + k] = self.lp.apply(self.V[:, c:c + k])
            Vnext = self.V[:, lcl:lcl + k].copy()
            Q = self.V[:, :lcl]
            subH = np.zeros((lcl, k))
            subH2 = np.zeros((k, k))
            rank = self.ortho.project_and_normalize(Vnext, Q, subH, subH2)
            self.V[:, lcl:lcl + k] = Vnext
            self.R[:lcl, c:c + k] = subH
            self.R[lcl:lcl + k, c:c + k] = subH2
            if rank != k:
                raise OrthoFailure("couldn't generate basis of full rank")
            self.update_lsqr()
            self.cur_dim += k

    def update_lsqr(self, dim=-1):
        """updateLSQR (BelosBlockGmresIter.hpp:770-868)."""
        R, z, k = self.R, self.z, self.k
        cur = self.cur_dim
        if self.cur_dim <= dim < self.max_subspace_dim():
            cur = dim
        if k == 1:
            for i in range(cur):
                x, y = R[i, cur], R[i + 1, cur]
                R[i, cur] = self.cs[i] * x + self.sn[i] * y
                R[i + 1, cur] = self.cs[i] * y - self.sn[i] * x
            a, b = R[cur, cur], R[cur + 1, cur]
            r, c, s = _rotg(a, b)
            R[cur, cur] = r
            self.cs[cur], self.sn[cur] = c, s
            R[cur + 1, cur] = 0.0
            x, y = z[cur, 0], z[cur + 1, 0]
            z[cur, 0] = c * x + s * y
            z[cur + 1, 0] = c * y - s * x
        else:
            beta = self.beta
            for j in range(k):
                cj = cur + j
                for i in range(cj):
                    sigma = float(np.dot(R[i + 1:i + 1 + k, i], R[i + 1:i + 1 + k, cj]))
                    sigma += R[i, cj]
                    sigma *= beta[i]
                    R[i + 1:i + 1 + k, cj] += (-sigma) * R[i + 1:i + 1 + k, i]
                    R[i, cj] -= sigma
                col = R[cj:cj + k + 1, cj]
                maxidx = int(np.argmax(np.abs(col)))
                maxelem = col[maxidx]
                R[cj:cj + k + 1, cj] /= maxelem
                sigma = float(np.dot(R[cj + 1:cj + 1 + k, cj], R[cj + 1:cj + 1 + k, cj]))
                if sigma == 0.0:
                    beta[cj] = 0.0
                else:
                    mu = math.sqrt(R[cj, cj] * R[cj, cj] + sigma)
                    if R[cj, cj] < 0.0:
                        vscale = R[cj, cj] - mu
                    else:
                        vscale = -sigma / (R[cj, cj] + mu)
                    beta[cj] = 2.0 * 1.0 * vscale * vscale / (sigma + vscale * vscale)
                    R[cj, cj] = maxelem * mu
                    R[cj + 1:cj + 1 + k, cj] /= vscale
                for i in range(k):
                    sigma = float(np.dot(R[cj + 1:cj + 1 + k, cj], z[cj + 1:cj + 1 + k, i]))
                    sigma += z[cj, i]
                    sigma *= beta[cj]
                    z[cj + 1:cj + 1 + k, i] += (-sigma) * R[cj + 1:cj + 1 + k, cj]
                    z[cj, i] -= sigma
        if self.cur_dim <= dim < self.max_subspace_dim():
            self.cur_dim = dim + k


class BlockFGmresIter(BlockGmresIter):
    """BelosBlockFGmresIter.hpp: flexible Block GMRES.  Z keeps the preconditioned basis
    (Z_j = M_R V_j, :645-740); the update is Z y (:488-523).  updateLSQR is the same
    Householder/Givens update as BlockGmresIter (:750-825)."""

    def __init__(self, lp, stest, ortho, k, nb):
        super().__init__(lp, stest, ortho, k, nb)
        self.Z = np.zeros_like(self.V)

    def current_update(self):
        c, k = self.cur_dim, self.k
        if c == 0:
            return None
        y = self.z[:c, :k].copy()
        Rc = self.R[:c, :c]
        for i in range(c - 1, -1, -1):
            if i + 1 < c:
                y[i, :] -= Rc[i, i + 1:c] @ y[i + 1:c, :]
            y[i, :] /= Rc[i, i]
        return self.Z[:, :c] @ y

    def iterate(self):
        k = self.k
        search = k * self.nb
        while (not self.stest.check(self)) and self.cur_dim + k <= search:
            self.num_iters += 1
            lcl = self.cur_dim + k
            c = self.cur_dim
            self.Z[:, c:c + k] = self.lp.apply_right_prec(self.V[:, c:c + k])
            self.V[:, lcl:lcl + k] = self.lp.apply_op(self.Z[:, c:c + k])
            Vnext = self.V[:, lcl:lcl + k].copy()
            Q = self.V[:, :lcl]
            subH = np.zeros((lcl, k))
            subH2 = np.zeros((k, k))
            rank = self.ortho.project_and_normalize(Vnext, Q, subH, subH2)
            self.V[:, lcl:lcl + k] = Vnext
            self.R[:lcl, c:c + k] = subH
            self.R[lcl:lcl + k, c:c + k] = subH2
            if rank != k:
                raise OrthoFailure("couldn't generate basis of full rank")
            self.update_lsqr()
            self.cur_dim += k


def _rotg(a, b):
    """BLAS drotg (reference algorithm): returns (r, c, s)."""
    roe = a if abs(a) > abs(b) else b
    scale = abs(a) + abs(b)
    if scale == 0.0:
        return 0.0, 1.0, 0.0
    r = scale * math.sqrt((a / scale) ** 2 + (b / scale) ** 2)
    r = math.copysign(1.0, roe) * r
    return r, a / r, b / r


DEFAULTS = {   # BelosBlockGmresSolMgr.hpp:317-335
    "Convergence Tolerance": 1e-8, "Maximum Restarts": 20, "Maximum Iterations": 1000,
    "Num Blocks": 300, "Block Size": 1, "Adaptive Block Size": True,
    "Orthogonalization": "DGKS", "Flexible Gmres": False, "Explicit Residual Test": False,
    "Implicit Residual Scaling": "Norm of Preconditioned Initial Residual",
    "Explicit Residual Scaling": "Norm of Initial Residual",
    "Orthogonalization Constant": -1.0,
}


class BlockGmresSolMgr:
    """BlockGmresSolMgr::solve (BelosBlockGmresSolMgr.hpp:916-1303), plain and flexible
    ("Flexible Gmres", BlockFGmresIter); status tests as checkStatusTest (:807-903):
    MaxIters OR (ImpResNorm | GenResNorm implicit | SEQ(implicit, explicit))."""

    def __init__(self, lp, params):
        p = dict(DEFAULTS)
        p.update(params)
        self.p = p
        self.lp = lp
        if p["Orthogonalization"] == "ICGS":
            self.ortho = ICGS()
        elif p["Orthogonalization"] == "DGKS":
            from .dgks import DGKS
            self.ortho = DGKS()
            if p["Orthogonalization Constant"] > 0:   # setDepTol(orthoKappa) (BelosBlockGmresSolMgr.hpp:607-625)
                self.ortho.dep_tol = float(p["Orthogonalization Constant"])
        else:
            raise ValueError("oracle supports ICGS and DGKS")

    def _status_tests(self, tol):
        """checkStatusTest (BelosBlockGmresSolMgr.hpp:807-903)."""
        p, lp = self.p, self.lp
        self.flexible = bool(p["Flexible Gmres"])
        exp_test = bool(p["Explicit Residual Test"])
        if self.flexible and lp.RP is None:
            self.flexible = False
            if lp.LP is not None:
                raise ValueError("flexible GMRES needs a right, not a left, preconditioner")
        if lp.LP is not None and not self.flexible:
            exp_test = True
        self.exp_test = exp_test
        imp_scale, exp_scale = p["Implicit Residual Scaling"], p["Explicit Residual Scaling"]
        if exp_test:
            self.imp = StatusTestGenResNorm(tol, False, imp_scale)
            self.exp = StatusTestGenResNorm(tol, True, exp_scale)
            self.conv = StatusTestSeq(self.imp, self.exp)
        else:
            self.imp = (StatusTestGenResNorm(tol, False, imp_scale) if self.flexible
                        else StatusTestImpResNorm(tol, imp_scale))
            self.exp = self.conv = self.imp

    def solve(self):
        p, lp = self.p, self.lp
        tol = float(p["Convergence Tolerance"])
        self.max_iter_test = StatusTestMaxIters(int(p["Maximum Iterations"]))
        self._status_tests(tol)
        self.stest = StatusTestOr(self.max_iter_test, self.conv)
        block = int(p["Block Size"])
        nb_param = int(p["Num Blocks"])
        max_restarts = int(p["Maximum Restarts"])
        numrhs = lp.B.shape[1]
        start = 0
        to_solve = numrhs
        cur_rhs = min(to_solve, block)
        if p["Adaptive Block Size"]:
            block = cur_rhs
            idx = list(range(start, start + cur_rhs))
        else:
            idx = list(range(start, start + cur_rhs)) + [-1] * (block - cur_rhs)
        lp.set_ls_index(idx)
        dim = lp.B.shape[0]
        self.stest.reset()
        self.loa = False
        converged = True
        self.n_restarts_total = 0
        self.iters_total = 0
        while to_solve > 0:
            if block * nb_param > dim:
                nb = dim // block if block == 1 else (dim - block) // block
            else:
                nb = nb_param
            it = (BlockFGmresIter if self.flexible else BlockGmresIter)(lp, self.stest, self.ortho, block, nb)
            if self.flexible:
                V0 = lp.curr_res_vec() if idx[-1] == -1 else lp.R0[:, idx].copy()
            else:
                V0 = lp.curr_prec_res_vec() if idx[-1] == -1 else lp.PR0[:, idx].copy()
            z0 = np.zeros((block, block))
            rank = self.ortho.normalize(V0, z0)
            if rank != block:
                raise OrthoFailure("failed to compute initial block")
            it.initialize(V0, z0)
            restarts = 0
            while True:
                try:
                    it.iterate()
                    if self.conv.status:
                        if self.exp.loss:
                            self.loa = True
                            converged = False
                        break
                    elif self.max_iter_test.status:
                        converged = False
                        break
                    elif it.cur_dim == it.max_subspace_dim():
                        if restarts >= max_restarts:
                            converged = False
                            break
                        restarts += 1
                        upd = it.current_update()
                        if self.flexible:
                            if upd is not None:
                                lp.curX = 1.0 * lp.curX + 1.0 * upd
                            V0 = lp.curr_res_vec()
                        else:
                            lp.update_solution(upd, True)
                            V0 = lp.curr_prec_res_vec()
                        z0 = np.zeros((block, block))
                        rank = self.ortho.normalize(V0, z0)
                        if rank != block:
                            raise OrthoFailure("failed to compute initial block after restart")
                        it.initialize(V0, z0)
                    else:
                        raise RuntimeError("invalid return from iterate()")
                except OrthoFailure:
                    if block != 1:
                        if not self.conv.status:
                            converged = False
                        break
                    it.update_lsqr(it.cur_dim)
                    self.stest.check(it)
                    if not self.conv.status:
                        converged = False
                    break
            if self.flexible:
                upd = it.current_update()
                if upd is not None:
                    lp.curX = 1.0 * lp.curX + 1.0 * upd
            elif self.exp.cur_soln is not None:
                lp.curX = 0.0 * self.exp.cur_soln + 1.0 * self.exp.cur_soln
            else:
                upd = it.current_update()
                lp.update_solution(upd, True)
            lp.set_curr_ls()
            self.n_restarts_total += restarts
            start += cur_rhs
            to_solve -= cur_rhs
            if to_solve > 0:
                cur_rhs = min(to_solve, block)
                if p["Adaptive Block Size"]:
                    block = cur_rhs
                    idx = list(range(start, start + cur_rhs))
                else:
                    idx = list(range(start, start + cur_rhs)) + [-1] * (block - cur_rhs)
                lp.set_ls_index(idx)
        self.num_iters = self.max_iter_test.n_iters
        tv = self.exp.testvector if self.exp_test else self.imp.testvector
        if tv is None or len(tv) < 1:
            tv = self.imp.testvector
        self.achieved_tol = float(np.max(tv))
        self.converged = converged and not self.loa
        return self.converged


def solve(A, B, params, X0=None, left=None, right=None):
    """Convenience driver: returns dict with X, iterations, history, counters."""
    X0 = np.zeros_like(B) if X0 is None else X0
    lp = LinearProblem(A, X0, B, left=left, right=right)
    lp.set_problem()
    sm = BlockGmresSolMgr(lp, params)
    ok = sm.solve()
    return dict(X=lp.X, converged=ok, iterations=sm.num_iters, achieved_tol=sm.achieved_tol,
                loa=sm.loa, n_apply=lp.n_apply, n_prec=lp.n_prec, n_explicit=sm.conv.n_explicit,
                restarts=sm.n_restarts_total, history=np.array(sm.stest.history),
                blk_ortho_sing=sm.ortho.counters.get("blkOrthoSing", 0),
                fb_decisions={key: sm.ortho.counters.get(key, 0) for key in ("fb_single", "fb_double", "fb_mixed")})
