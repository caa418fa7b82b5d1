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


def _dot(a, b):
    return float(np.dot(a, b))


def _coldots(X, Y):
    return np.einsum("ij,ij->j", X, Y)


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
        C[:] = Q.T @ X
        X -= Q @ C
        for _ in range(1, self.steps):
            C2 = Q.T @ X
            C += C2
            X -= Q @ C2
        return False

    def _blk_ortho(self, X, Q, C):
        """blkOrtho (BelosICGSOrthoManager.hpp:1328-1445)."""
        old = _coldots(X, X)
        C[:] = Q.T @ X
        X -= Q @ C
        for _ in range(1, self.steps):
            C2 = Q.T @ X
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
                    P2 = prevX.T @ Xj
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
                            pr = prevX.T @ t
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
                Ci[:nq, j] = Qi.T @ Xj
                Xj -= Qi @ Ci[:nq, j]
            for _ in range(1, self.steps):
                for Qi, Ci in zip(Qs, Cs):
                    nq = Qi.shape[1]
                    C2 = Qi.T @ Xj
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
                        pr = Qi.T @ t
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
    """BelosLinearProblem for an unpreconditioned operator (BelosLinearProblem.hpp)."""

    def __init__(self, A, X, B):
        self.A = A          # callable: Y = A(X)
        self.X = np.array(X, dtype=np.float64, copy=True)
        self.B = np.array(B, dtype=np.float64, copy=True)
        self.n_apply = 0
        self.ls_num = 0
        self.ls_idx = []
        self.aug_seed = LP_AUGMENT_SEED

    def apply(self, x):
        self.n_apply += 1
        return self.A(x)

    def set_problem(self):
        """setProblem (BelosLinearProblem.hpp:836-946): R0 = B - A X; PR0 = R0."""
        R = self.apply(self.X)
        self.R0 = self.B - R
        self.PR0 = self.R0
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
        """updateSolution (BelosLinearProblem.hpp:743-812), no right preconditioner."""
        if update is None:
            return self.curX
        if update_lp:
            self.curX = self.curX + update
            return self.curX
        return self.curX + update

    def curr_res_vec(self, Xs=None):
        """computeCurrResVec (BelosLinearProblem.hpp:1196-1231): R = B - A X."""
        Xs = self.curX if Xs is None else Xs
        R = self.apply(Xs)
        return (-1.0 * R) + (1.0 * self.curB)


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

    def __init__(self, tol):
        self.tol = tol
        self.reset()

    def reset(self):
        self.status = None
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
            self.scale = np.linalg.norm(lp.PR0, axis=0)
            self.numrhs = lp.PR0.shape[1]
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
                s = self.scale[p]
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
                s = self.scale[ind[i]]
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
        need = self.cur_num_rhs
        self.status = have >= need
        return self.status


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


def _rotg(a, b):
    """BLAS drotg (reference algorithm): returns (r, c, s)."""
    roe = a if abs(a) > abs(b) else b
    scale = abs(a) + abs(b)
    if scale == 0.0:
        return 0.0, 1.0, 0.0
    r = scale * math.sqrt((a / scale) ** 2 + (b / scale) ** 2)
    r = math.copysign(1.0, roe) * r
    return r, a / r, b / r


DEFAULTS = {
    "Convergence Tolerance": 1e-8, "Maximum Restarts": 20, "Maximum Iterations": 1000,
    "Num Blocks": 300, "Block Size": 1, "Adaptive Block Size": True,
    "Orthogonalization": "DGKS",
}


class BlockGmresSolMgr:
    """BlockGmresSolMgr::solve (BelosBlockGmresSolMgr.hpp:916-1303), non-flexible,
    implicit residual test with loss-of-accuracy check (ImpResNorm OR MaxIters)."""

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
        else:
            raise ValueError("oracle supports ICGS and DGKS")

    def solve(self):
        p, lp = self.p, self.lp
        tol = float(p["Convergence Tolerance"])
        self.max_iter_test = StatusTestMaxIters(int(p["Maximum Iterations"]))
        self.imp = StatusTestImpResNorm(tol)
        self.stest = StatusTestOr(self.max_iter_test, self.imp)
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
            it = BlockGmresIter(lp, self.stest, self.ortho, block, nb)
            if idx[-1] == -1:
                V0 = lp.curr_res_vec()
            else:
                V0 = lp.PR0[:, idx].copy()
            z0 = np.zeros((block, block))
            rank = self.ortho.normalize(V0, z0)
            if rank != block:
                raise OrthoFailure("failed to compute initial block")
            it.initialize(V0, z0)
            restarts = 0
            while True:
                try:
                    it.iterate()
                    if self.imp.status:
                        if self.imp.loss:
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
                        lp.update_solution(upd, True)
                        V0 = lp.curr_res_vec()
                        z0 = np.zeros((block, block))
                        rank = self.ortho.normalize(V0, z0)
                        if rank != block:
                            raise OrthoFailure("failed to compute initial block after restart")
                        it.initialize(V0, z0)
                    else:
                        raise RuntimeError("invalid return from iterate()")
                except OrthoFailure:
                    if block != 1:
                        if not self.imp.status:
                            converged = False
                        break
                    it.update_lsqr(it.cur_dim)
                    self.stest.check(it)
                    if not self.imp.status:
                        converged = False
                    break
            if self.imp.cur_soln is not None:
                lp.curX = 0.0 * self.imp.cur_soln + 1.0 * self.imp.cur_soln
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
        self.achieved_tol = float(np.max(self.imp.testvector))
        self.converged = converged and not self.loa
        return self.converged


def solve(A, B, params, X0=None):
    """Convenience driver: returns dict with X, iterations, history, counters."""
    X0 = np.zeros_like(B) if X0 is None else X0
    lp = LinearProblem(A, X0, B)
    lp.set_problem()
    sm = BlockGmresSolMgr(lp, params)
    ok = sm.solve()
    return dict(X=lp.X, converged=ok, iterations=sm.num_iters, achieved_tol=sm.achieved_tol,
                loa=sm.loa, n_apply=lp.n_apply, n_explicit=sm.imp.n_explicit,
                restarts=sm.n_restarts_total, history=np.array(sm.stest.history),
                blk_ortho_sing=sm.ortho.counters.get("blkOrthoSing", 0))
