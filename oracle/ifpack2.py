"""Ifpack2 point-Jacobi restatement (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Ifpack2::Relaxation with "relaxation: type" = "Jacobi" (ifpack2/src/Ifpack2_Relaxation_def.hpp):
  compute():  D^{-1} = reciprocal of the diagonal copy (:1240-1270, no tiny-entry fix, the
              default); the diagonal entry of a row is its (first) entry in column == row.
  apply():    ApplyInverseJacobi (:1390-1454).  With "zero starting solution" (default
              true) the first sweep is Y = (omega * d_i^{-1}) * X (KokkosBlas mult with
              c = 0, KokkosBlas1_mult_impl.hpp:93-104); every further sweep is
              R = X - A Y (Tpetra::Details::residual: b - sum, sum in stored order) and
              Y = 1*Y + (omega * d_i^{-1}) * R.
The Epetra/Ifpack twin (Ifpack_PointRelaxation.cpp:457-480) gives the same bits for
omega = 1 (x*d vs d*x).
"""

import numpy as np


def crs_diagonal(rowptr, gcols, vals, first, nloc):
    """Diagonal copy of a row block (global columns): first entry with column == row, 0 if
    the row has none (Tpetra getLocalDiagCopy via getLocalDiagOffsets)."""
    d = np.zeros(nloc)
    for i in range(nloc):
        g = first + i
        for p in range(int(rowptr[i]), int(rowptr[i + 1])):
            if int(gcols[p]) == g:
                d[i] = vals[p]
                break
    return d


def crs_diagonal_fast(rowptr, gcols, vals, first, nloc):
    """Vectorised crs_diagonal (the last diagonal hit wins only if a row repeats its
    diagonal column, which no generator here does)."""
    rows = np.repeat(np.arange(nloc), np.diff(rowptr))
    hit = gcols == rows + first
    d = np.zeros(nloc)
    d[rows[hit]] = vals[hit]
    return d


class Jacobi:
    """Y = M X for point Jacobi with `sweeps` sweeps and damping `damping`."""

    def __init__(self, A, diag, sweeps=1, damping=1.0, zero_start=True):
        if not zero_start:
            raise ValueError("only 'relaxation: zero starting solution' = true is restated")
        if sweeps < 1:
            raise ValueError("sweeps must be >= 1")
        self.A = A
        self.dinv = 1.0 / np.asarray(diag, dtype=np.float64)
        self.sweeps = sweeps
        self.damping = float(damping)
        self.n_apply = 0

    def __call__(self, X):
        self.n_apply += 1
        X = np.asarray(X, dtype=np.float64)
        ab = (self.damping * self.dinv)[:, None]
        Y = ab * X
        for _ in range(1, self.sweeps):
            R = X - self.A(Y)
            Y = 1.0 * Y + ab * R
        return Y
