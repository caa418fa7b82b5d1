"""Belos solver-layer mirror over the C ABI.

  MultiVecTraits     Belos::MultiVecTraits<double,MV> (belos/src/BelosMultiVecTraits.hpp:138-347,
                     Epetra specialisation belos/epetra/src/BelosEpetraAdapter.hpp:447-1064)
  OperatorTraits     Belos::OperatorTraits<double,MV,OP> (belos/src/BelosOperatorTraits.hpp:108-155)
  ICGSOrthoManager   Belos::ICGSOrthoManager (belos/src/BelosICGSOrthoManager.hpp:646-839)
  DGKSOrthoManager   Belos::DGKSOrthoManager (belos/src/BelosDGKSOrthoManager.hpp:644-840)
  LinearProblem      Belos::LinearProblem (belos/src/BelosLinearProblem.hpp)
  BlockGmresSolMgr   Belos::BlockGmresSolMgr (belos/src/BelosBlockGmresSolMgr.hpp)

Same names, argument meaning and error behaviour as the reference; the N-sized work runs
in HIP kernels, the control flow in the C++ solver behind include/migmres.h.
"""

import ctypes as C

import numpy as np

from ._lib import STATUS_FN, call, dptr, iptr
from .linalg import MultiVector, TWO_NORM, ONE_NORM, INF_NORM  # noqa: F401

Converged, Unconverged = "Converged", "Unconverged"  # Belos::ReturnType (BelosTypes.hpp:155-157)
TwoNorm, OneNorm, InfNorm = TWO_NORM, ONE_NORM, INF_NORM


class MultiVecTraits:
    """Static MVT interface.  Dense coefficient matrices are numpy arrays (column-major
    Teuchos::SerialDenseMatrix semantics); results that the reference returns in a
    SerialDenseMatrix / std::vector are returned as numpy arrays."""

    @staticmethod
    def Clone(mv, numvecs):
        return MultiVector(mv.comm, mv.n_global, numvecs)

    @staticmethod
    def CloneCopy(mv, index=None):
        src = mv if index is None else mv.view(index)
        out = MultiVector(mv.comm, mv.n_global, src.ncols)
        call("migmres_mv_assign", src.h, out.h)
        return out

    @staticmethod
    def CloneView(mv, index):
        return mv.view(index)

    CloneViewNonConst = CloneView

    @staticmethod
    def GetGlobalLength(mv):
        return mv.n_global

    @staticmethod
    def GetNumberVecs(mv):
        return mv.ncols

    @staticmethod
    def HasConstantStride(mv):
        return mv.constant_stride

    @staticmethod
    def MvTimesMatAddMv(alpha, A, B, beta, mv):
        B = np.asfortranarray(B, dtype=np.float64)
        if B.shape != (A.ncols, mv.ncols):
            raise ValueError("MvTimesMatAddMv: B must be A.ncols x mv.ncols")
        call("migmres_mv_times_mat_add_mv", float(alpha), A.h, dptr(B), max(B.shape[0], 1),
             float(beta), mv.h)

    @staticmethod
    def MvAddMv(alpha, A, beta, B, mv):
        call("migmres_mv_add_mv", float(alpha), A.h, float(beta), B.h, mv.h)

    @staticmethod
    def MvScale(mv, alpha):
        if np.ndim(alpha) == 0:
            call("migmres_mv_scale", mv.h, float(alpha))
        else:
            a = np.ascontiguousarray(alpha, dtype=np.float64)
            if a.size != mv.ncols:
                raise ValueError("MvScale: one scaling coefficient per column")
            call("migmres_mv_scale_vec", mv.h, dptr(a))

    @staticmethod
    def MvTransMv(alpha, A, mv):
        """C = alpha * A^T mv, replicated on every rank."""
        Cm = np.zeros((A.ncols, mv.ncols), dtype=np.float64, order="F")
        call("migmres_mv_trans_mv", float(alpha), A.h, mv.h, dptr(Cm), max(A.ncols, 1))
        return Cm

    @staticmethod
    def MvDot(mv, A):
        out = np.zeros(mv.ncols)
        call("migmres_mv_dot", mv.h, A.h, dptr(out))
        return out

    @staticmethod
    def MvNorm(mv, type=TwoNorm):
        out = np.zeros(mv.ncols)
        call("migmres_mv_norm", mv.h, dptr(out), int(type))
        return out

    @staticmethod
    def SetBlock(A, index, mv):
        idx = np.ascontiguousarray(index, dtype=np.int32)
        call("migmres_mv_set_block", A.h, iptr(idx), idx.size, mv.h)

    @staticmethod
    def Assign(A, mv):
        call("migmres_mv_assign", A.h, mv.h)

    @staticmethod
    def MvRandom(mv, seed=1):
        return mv.random(seed)

    @staticmethod
    def MvInit(mv, alpha=0.0):
        mv.put_scalar(alpha)

    @staticmethod
    def MvPrint(mv):
        return str(mv.download())


class OperatorTraits:
    @staticmethod
    def Apply(Op, x, y, trans=False):
        """BelosOperatorTraits.hpp:108-155 (trans: NOTRANS / TRANS as a bool or 0/1/2)."""
        if trans:
            Op.apply(x, y, 1.0, 0.0, int(trans))
        else:
            Op.apply(x, y)

    @staticmethod
    def HasApplyTranspose(Op):
        return hasattr(Op, "multiply")


class ICGSOrthoManager:
    """projectAndNormalize / normalize with the reference defaults (2 passes,
    blk_tol = 10 sqrt(eps), sing_tol = 10 eps)."""

    _pn, _n = "migmres_icgs_project_normalize", "migmres_icgs_normalize"

    def projectAndNormalize(self, X, Q):
        """Returns (rank, C, B) with C = (Q.ncols x X.ncols), B = (X.ncols x X.ncols)."""
        Cm = np.zeros((Q.ncols, X.ncols), order="F")
        Bm = np.zeros((X.ncols, X.ncols), order="F")
        r = C.c_int()
        call(self._pn, X.h, Q.h, dptr(Cm), max(Q.ncols, 1), dptr(Bm), max(X.ncols, 1), C.byref(r))
        return r.value, Cm, Bm

    def normalize(self, X):
        Bm = np.zeros((X.ncols, X.ncols), order="F")
        r = C.c_int()
        call(self._n, X.h, dptr(Bm), max(X.ncols, 1), C.byref(r))
        return r.value, Bm


class DGKSOrthoManager(ICGSOrthoManager):
    """Belos::DGKSOrthoManager (belos/src/BelosDGKSOrthoManager.hpp) with its defaults
    (2 passes, blk_tol = 10 sqrt(eps), dep_tol = 1/sqrt(2), sing_tol = 10 eps)."""

    _pn, _n = "migmres_dgks_project_normalize", "migmres_dgks_normalize"


class LinearProblem:
    """Belos::LinearProblem(A, X, B) (belos/src/BelosLinearProblem.hpp) with optional
    left/right preconditioners (setLeftPrec / setRightPrec, :170-175), e.g.
    trilinos_amd.ifpack2.Relaxation."""

    def __init__(self, A, X, B):
        self.A, self.X, self.B = A, X, B
        self.LP = self.RP = None
        self._set = False

    def setLeftPrec(self, LP):
        self.LP = LP

    def setRightPrec(self, RP):
        self.RP = RP

    def getLeftPrec(self):
        return self.LP

    def getRightPrec(self):
        return self.RP

    def isLeftPrec(self):
        return self.LP is not None

    def isRightPrec(self):
        return self.RP is not None

    def setProblem(self):
        if self.X is None or self.B is None or self.A is None:
            return False
        if self.X.ncols != self.B.ncols:
            return False
        self._set = True
        return True

    def isProblemSet(self):
        return self._set


_INT_PARAMS = {"Block Size", "Num Blocks", "Maximum Iterations", "Maximum Restarts", "Verbosity",
               "Output Frequency", "Deflation Quorum", "Output Style"}
_BOOL_PARAMS = {"Adaptive Block Size", "Flexible Gmres", "Explicit Residual Test",
                "Show Maximum Residual Norm Only"}
_DOUBLE_PARAMS = {"Convergence Tolerance", "Orthogonalization Constant"}
_STRING_PARAMS = {"Orthogonalization", "Implicit Residual Scaling", "Explicit Residual Scaling", "Timer Label"}

# Belos::OutputType (BelosTypes.hpp): "Output Style" takes either the enum or its int
General, Brief = 0, 1

# BelosBlockGmresSolMgr.hpp:317-338, 438-486 and DefaultSolverParameters::convTol
DEFAULT_PARAMETERS = {
    "Convergence Tolerance": 1e-8, "Maximum Restarts": 20, "Maximum Iterations": 1000,
    "Num Blocks": 300, "Block Size": 1, "Adaptive Block Size": True, "Verbosity": 0,
    "Output Frequency": -1, "Orthogonalization": "DGKS", "Flexible Gmres": False,
    "Explicit Residual Test": False,
    "Implicit Residual Scaling": "Norm of Preconditioned Initial Residual",
    "Explicit Residual Scaling": "Norm of Initial Residual",
    # recorded and reported; the device path writes no status output (BelosBlockGmresSolMgr.hpp:459-486)
    "Output Style": General, "Show Maximum Residual Norm Only": False, "Timer Label": "Belos",
    # > 0 with "DGKS": the ortho manager's dep_tol (BelosBlockGmresSolMgr.hpp:607-625)
    "Orthogonalization Constant": -1.0,
}
SCALE_TYPES = ("Norm of Initial Residual", "Norm of Preconditioned Initial Residual", "Norm of RHS", "None")


class BlockGmresSolMgr:
    """Belos::BlockGmresSolMgr over the device solver.

    Parameters use the reference ParameterList names.  "ICGS" and "DGKS" (the reference
    default) orthogonalization run on the device path; "IMGS" raises at solve().
    """

    _solver_name = "BLOCK GMRES"
    _defaults = DEFAULT_PARAMETERS

    def __init__(self, problem=None, params=None):
        self.problem = problem
        self.params = dict(self._defaults)
        h = C.c_void_p()
        self.comm = None
        self.h = None
        self._pending = {}
        if params:
            self.setParameters(params)

    def _ensure(self):
        if self.h is None:
            if self.problem is None:
                raise RuntimeError("BlockGmresSolMgr: no LinearProblem set")
            self.comm = self.problem.A.comm
            h = C.c_void_p()
            call("migmres_solver_create_named", self.comm.h, self._solver_name.encode(), C.byref(h))
            self.h = h
            for k, v in self.params.items():
                self._push(k, v)

    def _push(self, name, v):
        n = name.encode()
        if name in _INT_PARAMS:
            call("migmres_solver_set_int", self.h, n, int(v))
        elif name in _BOOL_PARAMS:
            call("migmres_solver_set_int", self.h, n, 1 if v else 0)
        elif name in _DOUBLE_PARAMS:
            call("migmres_solver_set_double", self.h, n, float(v))
        elif name in _STRING_PARAMS:
            if name == "Orthogonalization" and v not in ("DGKS", "ICGS", "IMGS"):
                raise ValueError('"Orthogonalization" must be either "DGKS", "ICGS", or "IMGS".')
            if name == "Orthogonalization" and v not in ("ICGS", "DGKS"):
                return  # validated at solve()
            call("migmres_solver_set_string", self.h, n, str(v).encode())

    def setProblem(self, problem):
        self.problem = problem

    def getValidParameters(self):
        if self.h is not None:
            return self._abi_params("migmres_solver_valid_parameters")
        return dict(self._defaults)

    def _abi_params(self, fn):
        """The library's parameter list text ("name\ttype\tvalue" lines) as a dict."""
        need = C.c_int()
        call(fn, self.h, None, 0, C.byref(need))
        buf = C.create_string_buffer(need.value)
        call(fn, self.h, buf, need.value, C.byref(need))
        out = {}
        for line in buf.value.decode().splitlines():
            name, typ, val = line.split("\t")
            out[name] = (int(val) if typ == "int" else val == "true" if typ == "bool"
                         else float(val) if typ == "double" else val)
        return out

    def reset(self, type=1):
        """SolverManager::reset(ResetType): 1 = Belos::Problem, 2 = Belos::RecycleSubspace."""
        self._ensure()
        call("migmres_solver_reset", self.h, int(type))

    def setUserConvStatusTest(self, test, comboType="SEQ"):
        """StatusTestCombo(comboType, residual test, test) -- pseudo-block GMRES only, as in the
        reference.  test(iters, res) -> bool, res = the scaled implicit residual norms."""
        self._ensure()
        combo = {"AND": 0, "OR": 1, "SEQ": 2}[comboType]
        if test is None:
            self._user_cb = None
            call("migmres_solver_set_user_conv_test", self.h, None, None, combo)
            return
        self._user_cb = STATUS_FN(lambda _u, it, n, r: 1 if test(it, np.ctypeslib.as_array(r, (n,)).copy()) else 0)
        call("migmres_solver_set_user_conv_test", self.h, self._user_cb, None, combo)

    def setParameters(self, params):
        for k, v in params.items():
            if k not in self._defaults:
                raise KeyError(f'"{k}" is not a valid {type(self).__name__} parameter')
            if k == "Block Size" and int(v) <= 0:
                raise ValueError('"Block Size" must be strictly positive.')
            if k == "Num Blocks" and int(v) <= 0:
                raise ValueError('"Num Blocks" must be strictly positive.')
            if k == "Orthogonalization" and v not in ("DGKS", "ICGS", "IMGS"):
                raise ValueError('"Orthogonalization" must be either "DGKS", "ICGS", or "IMGS".')
            if k in ("Implicit Residual Scaling", "Explicit Residual Scaling") and v not in SCALE_TYPES:
                raise ValueError(f'invalid residual scaling type "{v}"')
            self.params[k] = v
            if self.h is not None:
                self._push(k, v)

    def getCurrentParameters(self):
        if self.h is not None:
            return self._abi_params("migmres_solver_current_parameters")
        return dict(self.params)

    def solve(self):
        if self.problem is None or not self.problem.isProblemSet():
            raise RuntimeError("BlockGmresSolMgr::solve(): Linear problem is not ready, "
                               "setProblem() has not been called.")
        if self.params["Orthogonalization"] not in ("ICGS", "DGKS"):
            raise NotImplementedError('device Block GMRES implements "Orthogonalization" = "ICGS" and "DGKS"')
        self._ensure()
        from .linalg import Operator
        for side, M in ((0, self.problem.LP), (1, self.problem.RP)):
            if isinstance(M, Operator):   # a user operator as the preconditioner
                call("migmres_solver_set_prec_op", self.h, side, M.h)
            else:
                call("migmres_solver_set_prec_op", self.h, side, None)
                call("migmres_solver_set_prec", self.h, side, M.h if M is not None else None)
        conv = C.c_int()
        fn = "migmres_solver_solve_op" if isinstance(self.problem.A, Operator) else "migmres_solver_solve"
        call(fn, self.h, self.problem.A.h, self.problem.X.h, self.problem.B.h, C.byref(conv))
        return Converged if conv.value else Unconverged

    def getNumIters(self):
        v = C.c_int()
        call("migmres_solver_num_iters", self.h, C.byref(v))
        return v.value

    def achievedTol(self):
        v = C.c_double()
        call("migmres_solver_achieved_tol", self.h, C.byref(v))
        return v.value

    def isLOADetected(self):
        v = C.c_int()
        call("migmres_solver_loa_detected", self.h, C.byref(v))
        return bool(v.value)

    def residualHistory(self):
        nr, nc = C.c_int(), C.c_int()
        call("migmres_solver_history", self.h, None, C.byref(nr), C.byref(nc))
        out = np.zeros(max(nr.value * nc.value, 1))
        call("migmres_solver_history", self.h, dptr(out), C.byref(nr), C.byref(nc))
        return out[:nr.value * nc.value].reshape(nr.value, nc.value)

    def counters(self):
        out = (C.c_longlong * 11)()
        call("migmres_solver_counters", self.h, out, 11)
        keys = ("applies", "explicit_checks", "restarts", "blk_ortho_sing", "block_iterations",
                "prec_applies", "deflations", "gram_calls", "gram_skips", "gram_dgks_single", "gram_dgks_mixed")
        return dict(zip(keys, list(out)))

    def timers(self):
        out = (C.c_double * 8)()
        call("migmres_solver_timers", self.h, out, 8)
        keys = ("total", "spmm", "ortho", "lsqr", "comm", "status", "restart", "setup")
        return dict(zip(keys, list(out)))

    def __del__(self):
        try:
            if self.h is not None and (self.comm is None or self.comm.h):
                call("migmres_solver_destroy", self.h)
        except Exception:
            pass


# BelosPseudoBlockGmresSolMgr.hpp:494-507
PSEUDO_DEFAULT_PARAMETERS = {
    "Convergence Tolerance": 1e-8, "Maximum Restarts": 20, "Maximum Iterations": 1000,
    "Num Blocks": 300, "Block Size": 1, "Verbosity": 0, "Output Frequency": -1,
    "Deflation Quorum": 1, "Orthogonalization": "ICGS", "Explicit Residual Test": False,
    "Implicit Residual Scaling": "Norm of Preconditioned Initial Residual",
    "Explicit Residual Scaling": "Norm of Initial Residual",
    "Output Style": General, "Show Maximum Residual Norm Only": False, "Timer Label": "Belos",
    "Orthogonalization Constant": -1.0,
}


class PseudoBlockGmresSolMgr(BlockGmresSolMgr):
    """Belos::PseudoBlockGmresSolMgr over the device solver: "Block Size" single-vector
    GMRES iterations sharing each operator application, with deflation of converged
    right-hand sides ("Deflation Quorum")."""

    _solver_name = "PSEUDOBLOCK GMRES"
    _defaults = PSEUDO_DEFAULT_PARAMETERS


def SolverFactory(name, problem=None, params=None):
    """Belos::SolverFactory::create for the GMRES family (Belos_Details_EBelosSolverType.cpp)."""
    n = name.upper()
    if n in ("GMRES", "PSEUDOBLOCK GMRES", "PSEUDO BLOCK GMRES", "PSEUDOBLOCKGMRES"):
        return PseudoBlockGmresSolMgr(problem, params)
    if n == "BLOCK GMRES":
        return BlockGmresSolMgr(problem, params)
    if n == "FLEXIBLE GMRES":
        p = dict(params or {})
        p["Flexible Gmres"] = True
        return BlockGmresSolMgr(problem, p)
    raise ValueError(f'solver "{name}" is not implemented on the device path')
