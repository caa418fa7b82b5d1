"""Problems of the reference's own unit tests that hold known answers, shared by the oracle
pins (CPU, test_oracle_pins.py) and the same checks through the C ABI on the GPU
(test_gpu_known_answers.py).  Test infrastructure only.

* Ifpack2 Relaxation Test0 / Test1 / Test3
  (ifpack2/test/unit_tests/Ifpack2_UnitTestRelaxation.cpp:70-241): 5 rows per process of
  tif_utest::create_test_matrix (Ifpack2_UnitTestHelpers.hpp:279-330) -- a tridiagonal
  pattern with 2 on the diagonal and explicitly stored zeros beside it; x = 1 (2 columns):
  applyMat -> all 2, Jacobi apply -> all 0.5, apply(x, x) -> all 0.5, and apply on a
  process that owns no rows does not fail.
* Epetra CrsMatrix power method (epetra/test/CrsMatrix/cxx_main.cpp:124-317, 957-986): the
  (-1, 2, -1) tridiagonal on 10000 P + min(P, 3) rows (off-diagonals inserted before the
  diagonal), 3 n - 2 entries; the power method (200 iterations, residual ||A q - lambda q||
  checked at iterations 0, 100 and 199, tolerance 0.1) must succeed for A and A^T, and again
  after A[0,0] is multiplied by 10.
* Belos test_bl_gmres_diag.cpp (belos/epetra/test/BlockGmres/test_bl_gmres_diag.cpp:165-420):
  Block GMRES (Block Size 1, Num Blocks n, 100 iterations, 10 restarts, tol 1e-10, default
  orthogonalization) on n = 10 diagonal operators, x = 1: inv(diag(1..10)) x = [1, 1/2, ...,
  1/10]; inv(4 I) x = 1/4; and the nested inv(inv(4 I) 4 I) x = 1 with ||y - 1|| < 1e-10.
"""

import numpy as np


def ifpack2_test_matrix_rows(n_global, val=0.0):
    """create_test_matrix: row 0 (2, val), middle rows (val, 2, val), last row (val, 2),
    in that insertion order."""
    def gen(first, m):
        rp, gc, vv = [0], [], []
        for g in range(first, first + m):
            if g == 0:
                cols, vals = [0, 1], [2.0, val]
            elif g == n_global - 1:
                cols, vals = [g - 1, g], [val, 2.0]
            else:
                cols, vals = [g - 1, g, g + 1], [val, 2.0, val]
            if n_global == 1:
                cols, vals = [0], [2.0]
            gc += cols
            vv += vals
            rp.append(len(gc))
        return np.array(rp, np.int64), np.array(gc, np.int64), np.array(vv)
    return gen


def epetra_tridiag_rows(n_global, diag0=2.0):
    """cxx_main.cpp:145-186: per row the off-diagonal -1 entries (left, right) are inserted,
    then the diagonal 2 (`diag0` for row 0: the 10x test at :283-294)."""
    def gen(first, m):
        rp, gc, vv = [0], [], []
        for g in range(first, first + m):
            if g == 0:
                off = [1]
            elif g == n_global - 1:
                off = [n_global - 2]
            else:
                off = [g - 1, g + 1]
            gc += off + [g]
            vv += [-1.0] * len(off) + [diag0 if g == 0 else 2.0]
            rp.append(len(gc))
        return np.array(rp, np.int64), np.array(gc, np.int64), np.array(vv)
    return gen


def epetra_crs_test_size(P):
    """NumGlobalEquations = 10000 P + min(P, 3) (cxx_main.cpp:124-127)."""
    return 10000 * P + min(P, 3)


class NumpyOps:
    """power_method's operations on (n, 1) numpy arrays (the oracle side)."""

    def __init__(self, apply):
        self._apply = apply

    def norm2(self, v):
        from oracle import belos as ob
        return float(ob.mv_norm(v)[0])

    def dot(self, a, b):
        from oracle import belos as ob
        return float(ob.mv_dot(a, b)[0])

    def scale(self, out, alpha, v):      # out.Scale(alpha, v): out = alpha v
        out[:] = alpha * v

    def apply(self, x, y):               # y = A x
        y[:] = self._apply(x)

    def update(self, out, a, A, b, B):   # out.Update(a, A, b, B, 0.0)
        out[:] = a * A + b * B


def power_method(ops, z, q, resid, niters=200, tolerance=1.0e-1):
    """cxx_main.cpp:957-986 over `ops` (NumpyOps, or the device MultiVecTraits in
    test_gpu_known_answers.py) on vectors z (holding z.Random()), q and resid.  Returns
    (ierr, lambda, lambdas, residuals); residuals only where the reference computes them
    (iter % 100 == 0 or the last iteration)."""
    lam = 0.0
    lambdas, residuals = [], []
    residual = None
    ierr = 1
    for it in range(niters):
        normz = ops.norm2(z)
        ops.scale(q, 1.0 / normz, z)          # q.Scale(1.0/normz, z)
        ops.apply(q, z)                       # A.Multiply(TransA, q, z)
        lam = ops.dot(q, z)                   # q.Dot(z, lambda)
        lambdas.append(lam)
        if it % 100 == 0 or it + 1 == niters:
            ops.update(resid, 1.0, z, -lam, q)  # resid.Update(1.0, z, -lambda, q, 0.0)
            residual = ops.norm2(resid)
            residuals.append((it, residual))
        if residual < tolerance:
            ierr = 0
            break
    return ierr, lam, lambdas, residuals


def transpose_apply(rowptr, lcols, vals, X, ncols):
    """Epetra_CrsMatrix::GeneralMTM's C loop (Epetra_CrsMatrix.cpp:3587-3650, P = 1): Y = 0,
    then for each row i in order, y[col] += value * x[i]."""
    rows = np.repeat(np.arange(len(rowptr) - 1), np.diff(rowptr))
    Y = np.zeros((ncols, X.shape[1]))
    for k in range(X.shape[1]):
        # np.add.at accumulates unbuffered in index order: the loop's order per y entry
        np.add.at(Y[:, k], lcols, vals * X[rows, k])
    return Y


DIAG_TEST_PARAMS = {"Block Size": 1, "Num Blocks": 10, "Maximum Iterations": 100, "Maximum Restarts": 10,
                    "Convergence Tolerance": 1.0e-10}


def laplace1d_rows(n_global):
    """Ifpack2_UnitTestChebyshev2.cpp:384-416: row 0 (2, -1), middle rows (-1, 2, -1), last
    row (-1, 2), in that insertion order."""
    def gen(first, m):
        rp, gc, vv = [0], [], []
        for g in range(first, first + m):
            if g == 0:
                cols, vals = [0, 1], [2.0, -1.0]
            elif g == n_global - 1:
                cols, vals = [g - 1, g], [-1.0, 2.0]
            else:
                cols, vals = [g - 1, g, g + 1], [-1.0, 2.0, -1.0]
            gc += cols
            vv += vals
            rp.append(len(gc))
        return np.asarray(rp, dtype=np.int64), np.asarray(gc, dtype=np.int64), np.asarray(vv)
    return gen


def laplace1d_lambda_max(n):
    """Demmel's bound the reference test sets as "chebyshev: max eigenvalue" (:424-426)."""
    return 2.0 * (1.0 - np.cos((np.pi * n) / (n + 1.0)))


# Ifpack2_UnitTestChebyshev2.cpp:312-314: degree 50, 15 (then 30) power iterations, 10000 rows
CHEB2_ROWS, CHEB2_DEGREE, CHEB2_EIG_ITERS = 10000, 50, 15
