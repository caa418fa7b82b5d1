"""Ifpack2 mirror for the device preconditioner: Ifpack2::Relaxation with
"relaxation: type" = "Jacobi" (ifpack2/src/Ifpack2_Relaxation_def.hpp; parameter names and
defaults :264-300, apply :1390-1454).  The operator runs on the device through the C ABI
(migmres_jacobi_create / migmres_prec_apply); there is no host fallback.
"""

import ctypes as C

import numpy as np

from ._lib import call, dptr

# Ifpack2_Relaxation_def.hpp:264-300 (the subset the device path implements)
DEFAULT_PARAMETERS = {
    "relaxation: type": "Jacobi",
    "relaxation: sweeps": 1,
    "relaxation: damping factor": 1.0,
    "relaxation: zero starting solution": True,
    "relaxation: use l1": False,
    "relaxation: fix tiny diagonal entries": False,
    "relaxation: check diagonal entries": False,
}


class Relaxation:
    """Ifpack2::Relaxation<CrsMatrix>: setParameters -> initialize -> compute -> apply."""

    def __init__(self, A):
        self.A = A
        self.params = dict(DEFAULT_PARAMETERS)
        self.h = None
        self._initialized = False

    def setParameters(self, params):
        for k, v in params.items():
            if k not in DEFAULT_PARAMETERS:
                raise KeyError(f'"{k}" is not a valid Ifpack2::Relaxation parameter for the device path')
            self.params[k] = v
        p = self.params
        if p["relaxation: type"] != "Jacobi":
            raise NotImplementedError('the device path implements "relaxation: type" = "Jacobi"')
        if int(p["relaxation: sweeps"]) < 0:
            raise ValueError('"relaxation: sweeps" must be nonnegative')
        if not p["relaxation: zero starting solution"]:
            raise NotImplementedError('"relaxation: zero starting solution" = false is not implemented')
        for k in ("relaxation: use l1", "relaxation: fix tiny diagonal entries",
                  "relaxation: check diagonal entries"):
            if p[k]:
                raise NotImplementedError(f'"{k}" = true is not implemented')

    def initialize(self):
        self._initialized = True

    def isInitialized(self):
        return self._initialized

    def compute(self):
        """Extract and invert the diagonal on the device."""
        if not self._initialized:
            self.initialize()
        self._free()
        h = C.c_void_p()
        call("migmres_jacobi_create", self.A.h, int(self.params["relaxation: sweeps"]),
             float(self.params["relaxation: damping factor"]), C.byref(h))
        self.h = h

    def isComputed(self):
        return self.h is not None

    def apply(self, X, Y, alpha=1.0, beta=0.0):
        """Y = alpha M X (Ifpack2_Relaxation_def.hpp:494-592): beta != 0 is rejected as in the
        reference, alpha == 0 zeroes Y, X may be Y (the sweeps then read a copy of X)."""
        if self.h is None:
            raise RuntimeError("Ifpack2::Relaxation::apply: compute() has not been called")
        if X.ncols != Y.ncols:
            raise RuntimeError("Ifpack2::Relaxation::apply: X and Y have different numbers of columns")
        if beta != 0.0:
            raise NotImplementedError(f"Ifpack2::Relaxation::apply: beta = {beta} != 0 case not implemented")
        if alpha == 0.0:
            Y.put_scalar(0.0)
            return
        call("migmres_prec_apply", self.h, X.h, Y.h)
        if alpha != 1.0:
            call("migmres_mv_scale", Y.h, float(alpha))

    def applyMat(self, X, Y):
        """Y = A X with the preconditioner's matrix (Ifpack2_Relaxation_def.hpp:596-615)."""
        if self.h is None:
            raise RuntimeError("Ifpack2::Relaxation::applyMat: compute() has not been called")
        if X.ncols != Y.ncols:
            raise ValueError("Ifpack2::Relaxation::applyMat: X and Y have different numbers of columns")
        self.A.apply(X, Y)

    def inverseDiagonal(self):
        out = np.zeros(self.A.n_local)
        call("migmres_prec_diagonal", self.h, dptr(out))
        return out

    def _free(self):
        if self.h is not None:
            call("migmres_prec_destroy", self.h)
            self.h = None

    def __del__(self):
        try:
            self._free()
        except Exception:
            pass
