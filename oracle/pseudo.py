"""Pseudo-block GMRES restatement (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

k independent single-vector GMRES iterations that share one operator application per step:
  PseudoBlockGmresIter    belos/src/BelosPseudoBlockGmresIter.hpp (iterate :743-871,
                          getCurrentUpdate :447-484, getNativeResiduals :487-510,
                          initialize :514-690, updateLSQR :876-915)
  PseudoBlockGmresSolMgr  belos/src/BelosPseudoBlockGmresSolMgr.hpp (defaults :494-507,
                          checkStatusTest :1156-1265, solve :1268-1668 with deflation of
                          converged right-hand sides, "Deflation Quorum")
Each right-hand side i owns a basis V_i (N x (nb+1)), Hessenberg H_i, rotations cs_i/sn_i and
least-squares right-hand side z_i; every step orthogonalises A u_i against V_i alone with
the single-vector projectAndNormalize of the orthogonalization manager.
"""

import numpy as np

from .belos import (ICGS, LinearProblem, StatusTestGenResNorm, StatusTestImpResNorm, StatusTestMaxIters,
                    StatusTestOr, StatusTestSeq, _rotg)

DEFAULTS = {   # BelosPseudoBlockGmresSolMgr.hpp:494-507
    "Convergence Tolerance": 1e-8, "Maximum Restarts": 20, "Maximum Iterations": 1000,
    "Num Blocks": 300, "Block Size": 1, "Deflation Quorum": 1, "Orthogonalization": "ICGS",
    "Explicit Residual Test": False,
    "Implicit Residual Scaling": "Norm of Preconditioned Initial Residual",
    "Explicit Residual Scaling": "Norm of Initial Residual",
    "Orthogonalization Constant": -1.0,
}


class RhsState:
    """The per-right-hand-side part of PseudoBlockGmresIterState."""

    def __init__(self, n, nb):
        self.V = np.zeros((n, nb + 1))
        self.H = np.zeros((nb + 1, nb))
        self.z = np.zeros(nb + 1)
        self.cs = np.zeros(nb + 1)
        self.sn = np.zeros(nb + 1)


class PseudoBlockGmresIter:
    def __init__(self, lp, stest, ortho, nb):
        self.lp, self.stest, self.ortho, self.nb = lp, stest, ortho, nb
        self.num_iters = 0
        self.cur_dim = 0
        self.st = []

    def max_subspace_dim(self):
        return self.nb

    def initialize(self, states, cur_dim):
        self.st = states
        self.cur_dim = cur_dim

    def native_residuals(self):
        return np.array([abs(s.z[self.cur_dim]) for s in self.st])

    def current_update(self):
        c = self.cur_dim
        if c == 0:
            return None
        out = np.zeros((self.lp.B.shape[0], len(self.st)))
        for i, s in enumerate(self.st):
            y = s.z[:c].copy()
            for r in range(c - 1, -1, -1):       # TRSM, upper, non-unit
                if r + 1 < c:
                    y[r] -= float(s.H[r, r + 1:c] @ y[r + 1:c])
                y[r] /= s.H[r, r]
            out[:, i] = s.V[:, :c] @ y
        return out

    def iterate(self):
        nrhs = len(self.st)
        U = np.column_stack([s.V[:, self.cur_dim] for s in self.st]) if nrhs else None
        while (not self.stest.check(self)) and self.cur_dim < self.nb:
            self.num_iters += 1
            AU = self.lp.apply(U)
            c = self.cur_dim
            for i, s in enumerate(self.st):
                w = AU[:, i:i + 1].copy()
                h = np.zeros((c + 1, 1))
                r = np.zeros((1, 1))
                self.ortho.project_and_normalize(w, s.V[:, :c + 1], h, r)
                s.H[:c + 1, c] = h[:, 0]
                s.H[c + 1, c] = r[0, 0]
                s.V[:, c + 1] = w[:, 0]
                AU[:, i] = w[:, 0]
            U = AU
            self.update_lsqr()
            self.cur_dim += 1

    def update_lsqr(self, dim=-1):
        c = self.cur_dim
        if self.cur_dim <= dim < self.nb:
            c = dim
        for s in self.st:
            H = s.H
            for j in range(c):
                x, y = H[j, c], H[j + 1, c]
                H[j, c] = s.cs[j] * x + s.sn[j] * y
                H[j + 1, c] = s.cs[j] * y - s.sn[j] * x
            rr, cc, ss = _rotg(H[c, c], H[c + 1, c])
            H[c, c] = rr
            s.cs[c], s.sn[c] = cc, ss
            H[c + 1, c] = 0.0
            x, y = s.z[c], s.z[c + 1]
            s.z[c] = cc * x + ss * y
            s.z[c + 1] = cc * y - ss * x


class PseudoBlockGmresSolMgr:
    def __init__(self, lp, params):
        p = dict(DEFAULTS)
        p.update(params)
        self.p, self.lp = p, lp
        if p["Orthogonalization"] == "ICGS":
            self.ortho = ICGS()
        elif p["Orthogonalization"] == "DGKS":
            from .dgks import DGKS
            self.ortho = DGKS()
            if p["Orthogonalization Constant"] > 0:   # setDepTol(orthoKappa) (BelosPseudoBlockGmresSolMgr.hpp:736-754)
                self.ortho.dep_tol = float(p["Orthogonalization Constant"])
        else:
            raise ValueError("oracle supports ICGS and DGKS")

    def _normalize_columns(self, R0, nb):
        states = []
        for i in range(R0.shape[1]):
            s = RhsState(R0.shape[0], nb)
            v = R0[:, i:i + 1].copy()
            b = np.zeros((1, 1))
            if self.ortho.normalize(v, b) != 1:
                raise RuntimeError("failed to compute initial block of orthonormal vectors")
            s.V[:, 0] = v[:, 0]
            s.z[0] = b[0, 0]
            states.append(s)
        return states

    def solve(self):
        p, lp = self.p, self.lp
        tol = float(p["Convergence Tolerance"])
        quorum = int(p["Deflation Quorum"])
        self.max_iter_test = StatusTestMaxIters(int(p["Maximum Iterations"]))
        exp_test = bool(p["Explicit Residual Test"]) or lp.LP is not None
        self.exp_test = exp_test
        if exp_test:
            self.imp = StatusTestGenResNorm(tol, False, p["Implicit Residual Scaling"], quorum)
            self.exp = StatusTestGenResNorm(tol, True, p["Explicit Residual Scaling"], quorum)
            self.conv = StatusTestSeq(self.imp, self.exp)
        else:
            self.imp = StatusTestImpResNorm(tol, p["Implicit Residual Scaling"], quorum)
            self.exp = self.conv = self.imp
        self.stest = StatusTestOr(self.max_iter_test, self.conv)
        block = int(p["Block Size"])
        nb = int(p["Num Blocks"])
        max_restarts = int(p["Maximum Restarts"])
        numrhs = lp.B.shape[1]
        start, to_solve = 0, numrhs
        cur = min(to_solve, block)
        block = cur
        idx = list(range(start, start + cur))
        lp.set_ls_index(idx)
        self.stest.reset()
        self.loa = False
        converged = True
        self.n_restarts_total = 0
        self.n_deflations = 0
        it = PseudoBlockGmresIter(lp, self.stest, self.ortho, nb)
        while to_solve > 0:
            cur_rhs_idx = list(idx[:cur])
            it.num_iters = 0
            it.nb = nb
            it.initialize(self._normalize_columns(lp.PR0[:, idx].copy(), nb), 0)
            restarts = 0
            while True:
                it.iterate()
                if self.conv.status:
                    if self.exp.loss:
                        self.loa = True
                        converged = False
                    conv_idx = list(self.exp.ind)
                    if len(conv_idx) == len(cur_rhs_idx):
                        break
                    # deflate the converged right-hand sides (:1397-1466)
                    self.n_deflations += 1
                    lp.set_curr_ls()
                    keep, def_lcl = [], []
                    for i, g in enumerate(cur_rhs_idx):
                        (def_lcl if g in conv_idx else keep).append(i)
                    if it.cur_dim:
                        upd = it.current_update()
                        lp.set_ls_index(conv_idx)
                        lp.update_solution(upd[:, def_lcl], True)
                        lp.set_curr_ls()
                    cur_rhs_idx = [cur_rhs_idx[i] for i in keep]
                    lp.set_ls_index(cur_rhs_idx)
                    it.initialize([it.st[i] for i in keep], it.cur_dim)
                elif self.max_iter_test.status:
                    converged = False
                    break
                elif it.cur_dim == it.max_subspace_dim():
                    if restarts >= max_restarts:
                        converged = False
                        break
                    restarts += 1
                    lp.update_solution(it.current_update(), True)
                    R0 = lp.curr_prec_res_vec()
                    it.initialize(self._normalize_columns(R0, nb), 0)
                else:
                    raise RuntimeError("invalid return from iterate()")
            if self.exp.cur_soln is not None:
                lp.curX = 0.0 * self.exp.cur_soln + 1.0 * self.exp.cur_soln
            else:
                lp.update_solution(it.current_update(), True)
            lp.set_curr_ls()
            self.n_restarts_total += restarts
            start += cur
            to_solve -= cur
            if to_solve > 0:
                cur = min(to_solve, block)
                block = cur
                idx = list(range(start, start + cur))
                if quorum > block:
                    self.imp.quorum = block
                    if self.exp is not self.imp:
                        self.exp.quorum = block
                lp.set_ls_index(idx)
        self.num_iters = self.max_iter_test.n_iters
        tv = self.exp.testvector if exp_test else self.imp.testvector
        if tv is None or len(tv) < 1:
            tv = self.imp.testvector
        self.achieved_tol = float(np.max(tv))
        self.converged = converged and not self.loa
        return self.converged


def solve(A, B, params, X0=None, left=None, right=None):
    X0 = np.zeros_like(B) if X0 is None else X0
    lp = LinearProblem(A, X0, B, left=left, right=right)
    lp.set_problem()
    sm = PseudoBlockGmresSolMgr(lp, params)
    ok = sm.solve()
    return dict(X=lp.X, converged=ok, iterations=sm.num_iters, achieved_tol=sm.achieved_tol, loa=sm.loa,
                n_apply=lp.n_apply, n_prec=lp.n_prec, n_explicit=sm.conv.n_explicit,
                restarts=sm.n_restarts_total, deflations=sm.n_deflations, history=np.array(sm.stest.history))
