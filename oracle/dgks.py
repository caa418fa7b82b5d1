"""DGKSOrthoManager restatement (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

belos/src/BelosDGKSOrthoManager.hpp, double precision, no mass operator (Op == I), default
parameters (lines 536-556): max_blk_ortho = 2, blk_tol = 10 sqrt(eps),
dep_tol = 1/sqrt(2), sing_tol = 10 eps.

Differences from ICGS (oracle/belos.py), which it otherwise shares (projectAndNormalize
control flow BelosDGKSOrthoManager.hpp:644-815 and blkOrtho 1328-1490 are the same
operation sequence):
  * blkOrtho1 (1245-1321) re-orthogonalises only if sqrt|newDot| < dep_tol sqrt|oldDot|;
  * findBasis (1000-1243) makes one projection and a second one only under the same
    DGKS criterion on <X_j, X_j> after the first;
  * blkOrthoSing (1495-1752) re-orthogonalises column j only if |newDot| < |oldDot dep_tol|
    (no square roots there) and, unlike ICGS, uses the freshly computed newDot.
"""

import math

import numpy as np

from .belos import ICGS, ICGS_BLK_TOL, ICGS_SING_TOL, _dot, _tn

DGKS_DEP_TOL = 1.0 / math.sqrt(2.0)   # BelosDGKSOrthoManager.hpp:546-550


class DGKS(ICGS):
    def __init__(self, rng=None, steps=2, blk_tol=ICGS_BLK_TOL, dep_tol=DGKS_DEP_TOL, sing_tol=ICGS_SING_TOL):
        super().__init__(rng=rng, steps=steps, blk_tol=blk_tol, sing_tol=sing_tol)
        self.dep_tol = dep_tol

    def _blk_ortho1(self, X, Q, C):
        """blkOrtho1 (BelosDGKSOrthoManager.hpp:1245-1321)."""
        old = _dot(X[:, 0], X[:, 0])
        C[:] = _tn(Q, X)
        X -= Q @ C
        new = _dot(X[:, 0], X[:, 0])
        if math.sqrt(abs(new)) < self.dep_tol * math.sqrt(abs(old)):
            C2 = _tn(Q, X)
            C += C2
            X -= Q @ C2
        return False

    def find_basis(self, X, B, complete_basis):
        """findBasis (BelosDGKSOrthoManager.hpp:1000-1243), howMany = all columns."""
        xc = X.shape[1]
        twos = []  # per column j >= 1: did DGKS's criterion ask the second projection?
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
                product = _tn(prevX, Xj)
                Xj -= prevX @ product
                new_dot = _dot(Xj, Xj)
                twos.append(math.sqrt(abs(new_dot)) < self.dep_tol * math.sqrt(abs(old_dot)))
                if twos[-1]:
                    P2 = _tn(prevX, Xj)
                    product = product + P2
                    Xj -= prevX @ P2
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
            if abs(diag) > 0.0:
                Xj *= 1.0 / diag
            B[j, j] = 0.0 if add_vec else diag
            if not add_vec:
                B[:j, j] = product
        if not complete_basis and xc > 1:
            # the block's decision pattern (the device's Gram form takes one per block:
            # tests/test_gpu_solver.py::test_dgks_gram_decisions_match_oracle)
            key = "fb_single" if not any(twos) else "fb_double" if all(twos) else "fb_mixed"
            self.counters[key] = self.counters.get(key, 0) + 1
        return xc

    def _blk_ortho_sing(self, X, Q, C, B):
        """blkOrthoSing (BelosDGKSOrthoManager.hpp:1495-1752)."""
        self.counters["blkOrthoSing"] += 1
        xc = X.shape[1]
        for j in range(xc):
            Qs = [Q] + ([X[:, :j]] if j > 0 else [])
            Cs = [C] + ([B] if j > 0 else [])
            Xj = X[:, j]
            old_dot = _dot(Xj, Xj)
            for Qi, Ci in zip(Qs, Cs):
                nq = Qi.shape[1]
                Ci[:nq, j] = _tn(Qi, Xj)
                Xj -= Qi @ Ci[:nq, j]
            new_dot = _dot(Xj, Xj)
            if abs(new_dot) < abs(old_dot * self.dep_tol):
                for Qi, Ci in zip(Qs, Cs):
                    nq = Qi.shape[1]
                    C2 = _tn(Qi, Xj)
                    Ci[:nq, j] += C2
                    Xj -= Qi @ C2
                new_dot = _dot(Xj, Xj)
            if not abs(new_dot) < abs(old_dot * self.sing_tol):
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
