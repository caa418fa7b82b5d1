"""Ifpack2 mirror for the device preconditioners: Ifpack2::Relaxation with
"relaxation: type" = "Jacobi" (ifpack2/src/Ifpack2_Relaxation_def.hpp; parameter names and
defaults :264-300, apply :1390-1454) and Ifpack2::Chebyshev (Ifpack2_Chebyshev_def.hpp over
Ifpack2_Details_Chebyshev_def.hpp).  The operators run on the device through the C ABI
(migmres_jacobi_create / migmres_chebyshev_create / migmres_prec_apply); there is no host
fallback.
"""

import ctypes as C

import numpy as np

from ._lib import call, dptr

# Ifpack2_Relaxation_def.hpp:243-307 (the parameters of the types the device path implements)
DEFAULT_PARAMETERS = {
    "relaxation: type": "Jacobi",
    "relaxation: sweeps": 1,
    "relaxation: damping factor": 1.0,
    "relaxation: zero starting solution": True,
    "relaxation: use l1": False,
    "relaxation: l1 eta": 1.5,
    "relaxation: min diagonal value": 0.0,
    "relaxation: fix tiny diagonal entries": False,
    "relaxation: check diagonal entries": False,
}
RELAXATION_TYPES = {"Jacobi": 0, "Richardson": 1}


class _RelaxParams(C.Structure):
    """migmres_relaxation_params (include/migmres.h)."""
    _fields_ = [("type", C.c_int), ("sweeps", C.c_int), ("damping", C.c_double),
                ("zero_starting_solution", C.c_int), ("use_l1", C.c_int), ("l1_eta", C.c_double),
                ("min_diagonal_value", C.c_double), ("fix_tiny_diagonal_entries", C.c_int),
                ("check_diagonal_entries", C.c_int)]


class Relaxation:
    """Ifpack2::Relaxation<CrsMatrix>: setParameters -> initialize -> compute -> apply.
    "relaxation: type" "Jacobi" or "Richardson" (the Gauss-Seidel family is sequential and not
    on the device path)."""

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
        if p["relaxation: type"] not in RELAXATION_TYPES:
            raise NotImplementedError('the device path implements "relaxation: type" = "Jacobi" and "Richardson"')
        if int(p["relaxation: sweeps"]) < 0:
            raise ValueError('"relaxation: sweeps" must be nonnegative')

    def initialize(self):
        self._initialized = True

    def isInitialized(self):
        return self._initialized

    def compute(self):
        """Extract and invert the diagonal on the device (l1 / fix-tiny options applied)."""
        if not self._initialized:
            self.initialize()
        self._free()
        p = self.params
        cp = _RelaxParams()
        call("migmres_relaxation_params_default", C.byref(cp))
        cp.type = RELAXATION_TYPES[p["relaxation: type"]]
        cp.sweeps = int(p["relaxation: sweeps"])
        cp.damping = float(p["relaxation: damping factor"])
        cp.zero_starting_solution = 1 if p["relaxation: zero starting solution"] else 0
        cp.use_l1 = 1 if p["relaxation: use l1"] else 0
        cp.l1_eta = float(p["relaxation: l1 eta"])
        cp.min_diagonal_value = float(p["relaxation: min diagonal value"])
        cp.fix_tiny_diagonal_entries = 1 if p["relaxation: fix tiny diagonal entries"] else 0
        cp.check_diagonal_entries = 1 if p["relaxation: check diagonal entries"] else 0
        h = C.c_void_p()
        call("migmres_relaxation_create", self.A.h, C.byref(cp), C.byref(h))
        self.h = h

    def isComputed(self):
        return self.h is not None

    def apply(self, X, Y, alpha=1.0, beta=0.0):
        """Y = alpha M X (Ifpack2_Relaxation_def.hpp:494-592): beta != 0 is rejected as in the
        reference, alpha == 0 zeroes Y, X may be Y (the sweeps then read a copy of X); with
        "zero starting solution" false the sweeps start from Y's contents."""
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
        if self.h is not None and self.A.comm.h:
            call("migmres_prec_destroy", self.h)
        self.h = None

    def __del__(self):
        try:
            self._free()
        except Exception:
            pass


class _ChebParams(C.Structure):
    """migmres_chebyshev_params (include/migmres.h)."""
    _fields_ = [("degree", C.c_int), ("max_eigenvalue", C.c_double), ("ratio_eigenvalue", C.c_double),
                ("boost_factor", C.c_double), ("min_diagonal_value", C.c_double),
                ("eigenvalue_max_iterations", C.c_int), ("zero_starting_solution", C.c_int),
                ("assume_matrix_unchanged", C.c_int), ("textbook_algorithm", C.c_int), ("seed", C.c_uint)]


# Ifpack2_Details_Chebyshev_def.hpp:280-300, 333-677 (the device path's subset; "chebyshev: max
# eigenvalue" unset = estimate by the power method).  "chebyshev: min eigenvalue" is accepted
# and, as in the reference (:870-881), not used: lambdaMin = lambdaMax / ratio.
CHEBYSHEV_PARAMETERS = {
    "chebyshev: degree": 1,
    "chebyshev: ratio eigenvalue": 30.0,
    "chebyshev: boost factor": 1.1,
    "chebyshev: min diagonal value": float(np.finfo(np.float64).eps),
    "chebyshev: eigenvalue max iterations": 10,
    "chebyshev: zero starting solution": True,
    "chebyshev: assume matrix does not change": False,
    "chebyshev: textbook algorithm": False,
}
_CHEB_OPTIONAL = ("chebyshev: max eigenvalue", "chebyshev: min eigenvalue")
# ML / Ifpack aliases the reference reads (:489-494, 559-566, 573-577); the Ifpack2 name wins
_CHEB_ALIASES = {"smoother: Chebyshev alpha": "chebyshev: ratio eigenvalue",
                 "smoother: sweeps": "chebyshev: degree", "relaxation: sweeps": "chebyshev: degree",
                 "eigen-analysis: iterations": "chebyshev: eigenvalue max iterations"}


class Chebyshev:
    """Ifpack2::Chebyshev<CrsMatrix>: setParameters -> initialize -> compute -> apply.
    `seed` picks the power method's start vector (Epetra MINSTD stream; the reference's
    Tpetra randomize() stream is not reproduced)."""

    def __init__(self, A, seed=1):
        self.A = A
        self.seed = int(seed)
        self.params = dict(CHEBYSHEV_PARAMETERS)
        self.h = None
        self._initialized = False

    def setParameters(self, params):
        given = dict(params)
        for alias, name in _CHEB_ALIASES.items():
            if alias in given:
                v = given.pop(alias)
                given.setdefault(name, v)
        for k, v in given.items():
            if k not in CHEBYSHEV_PARAMETERS and k not in _CHEB_OPTIONAL:
                raise KeyError(f'"{k}" is not a valid Ifpack2::Chebyshev parameter for the device path')
            self.params[k] = v
        p = self.params
        if int(p["chebyshev: degree"]) < 0:
            raise ValueError('"chebyshev: degree" must be a nonnegative integer')
        if not float(p["chebyshev: ratio eigenvalue"]) >= 1.0:
            raise ValueError('"chebyshev: ratio eigenvalue" must be >= 1')
        if not float(p["chebyshev: boost factor"]) >= 1.0:
            raise ValueError('"chebyshev: boost factor" must be >= 1')
        for k in _CHEB_OPTIONAL:
            if k in p and not np.isfinite(float(p[k])):
                raise ValueError(f'"{k}" must be finite')
        if self.h is not None:   # the parameters of apply() change with them
            self.compute()

    def initialize(self):
        self._initialized = True

    def isInitialized(self):
        return self._initialized

    def _cparams(self):
        p = self.params
        out = _ChebParams()
        call("migmres_chebyshev_params_default", C.byref(out))
        out.degree = int(p["chebyshev: degree"])
        out.max_eigenvalue = float(p.get("chebyshev: max eigenvalue", float("nan")))
        out.ratio_eigenvalue = float(p["chebyshev: ratio eigenvalue"])
        out.boost_factor = float(p["chebyshev: boost factor"])
        out.min_diagonal_value = float(p["chebyshev: min diagonal value"])
        out.eigenvalue_max_iterations = int(p["chebyshev: eigenvalue max iterations"])
        out.zero_starting_solution = 1 if p["chebyshev: zero starting solution"] else 0
        out.assume_matrix_unchanged = 1 if p["chebyshev: assume matrix does not change"] else 0
        out.textbook_algorithm = 1 if p["chebyshev: textbook algorithm"] else 0
        out.seed = self.seed
        return out

    def compute(self):
        """Inverse diagonal and (unless given) the power-method estimate, on the device."""
        if not self._initialized:
            self.initialize()
        self._free()
        h = C.c_void_p()
        cp = self._cparams()
        call("migmres_chebyshev_create", self.A.h, C.byref(cp), C.byref(h))
        self.h = h

    def isComputed(self):
        return self.h is not None

    def _lambdas(self):
        a, b, c = C.c_double(), C.c_double(), C.c_double()
        call("migmres_chebyshev_lambdas", self.h, C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value

    def getLambdaMaxForApply(self):
        return self._lambdas()[0]

    def getComputedLambdaMax(self):
        return self._lambdas()[2]

    def apply(self, X, Y, alpha=1.0, beta=0.0):
        """Y = beta Y + alpha M X (Ifpack2_Chebyshev_def.hpp:418-495): alpha == 0 scales Y by
        beta (zeroes it for beta == 0), alpha != 1 folds into a copy of X, beta != 0 keeps a
        copy of Y to add at the end; X may be Y."""
        if self.h is None:
            raise RuntimeError("Ifpack2::Chebyshev::apply(): You must call the compute() method before "
                               "you may call apply().")
        if X.ncols != Y.ncols:
            raise RuntimeError("Ifpack2::Chebyshev::apply(): X and Y must have the same number of columns.")
        if alpha == 0.0:
            if beta == 0.0:
                Y.put_scalar(0.0)
            else:
                call("migmres_mv_scale", Y.h, float(beta))
            return
        from .linalg import MultiVector
        Yorig = None
        if beta != 0.0:
            Yorig = MultiVector(Y.comm, Y.n_global, Y.ncols)
            call("migmres_mv_assign", Y.h, Yorig.h)
        Xin = X
        if alpha != 1.0:
            Xin = MultiVector(X.comm, X.n_global, X.ncols)
            call("migmres_mv_assign", X.h, Xin.h)
            call("migmres_mv_scale", Xin.h, float(alpha))
        call("migmres_prec_apply", self.h, Xin.h, Y.h)
        if beta != 0.0:
            call("migmres_mv_add_mv", float(beta), Yorig.h, 1.0, Y.h, Y.h)

    def applyMat(self, X, Y):
        if X.ncols != Y.ncols:
            raise ValueError("Ifpack2::Chebyshev::applyMat: X.getNumVectors() != Y.getNumVectors().")
        self.A.apply(X, Y)

    def inverseDiagonal(self):
        out = np.zeros(self.A.n_local)
        call("migmres_prec_diagonal", self.h, dptr(out))
        return out

    def _free(self):
        if self.h is not None and self.A.comm.h:
            call("migmres_prec_destroy", self.h)
        self.h = None

    def __del__(self):
        try:
            self._free()
        except Exception:
            pass
