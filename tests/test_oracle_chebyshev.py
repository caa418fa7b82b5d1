"""The Chebyshev restatement (oracle/ifpack2.py Chebyshev) against the reference's own unit
tests, on the CPU.

* Ifpack2_UnitTestChebyshev.cpp Test0: the diag(2) test matrix with lambdaMax = 1, eigRatio =
  1/0.9 makes degree 1 an exact solve (apply = 0.5 within 1e-13) and degree 4 stays within 1e-4.
* Ifpack2_UnitTestChebyshev2.cpp Convergence: the 1-D Poisson matrix (10000 rows, Demmel's
  lambdaMax), degree 50.  With lambdaMax given, and with the power method's estimate after 30
  iterations (Test 6), Ifpack's variant is no worse than the textbook variant (4 digits of
  slack, :754-771); both reduce the residual.
"""

import numpy as np

from oracle import epetra as oe
from oracle.ifpack2 import Chebyshev, crs_diagonal_fast, reciprocal_threshold
from tests.known_answers import (CHEB2_DEGREE, CHEB2_EIG_ITERS, CHEB2_ROWS, ifpack2_test_matrix_rows,
                                 laplace1d_lambda_max, laplace1d_rows)


def _op(gen, n):
    A = oe.DistCrs(gen, n, 1)
    rp, gc, vv = gen(0, n)
    return A, crs_diagonal_fast(rp, gc, vv, 0, n)


def test_chebyshev_test0_known_answers():
    n = 5
    A, d = _op(ifpack2_test_matrix_rows(n), n)
    params = {"chebyshev: degree": 1, "chebyshev: min eigenvalue": 0.0, "chebyshev: max eigenvalue": 1.0,
              "chebyshev: ratio eigenvalue": 1.0 / 0.9}
    x = np.ones((n, 2))
    assert np.array_equal(A.apply(x), np.full((n, 2), 2.0))
    M = Chebyshev(A.apply, d, params)
    np.testing.assert_allclose(M(x), 0.5, rtol=0, atol=1e-13)
    M = Chebyshev(A.apply, d, dict(params, **{"chebyshev: degree": 4}))
    np.testing.assert_allclose(M(x), 0.5, rtol=0, atol=1e-4)


def test_reciprocal_threshold_stores_min_value():
    """|d| < minVal stores minVal itself (not its reciprocal): Ifpack2_Details_Chebyshev_def.hpp:109-114."""
    out = reciprocal_threshold(np.array([2.0, 1e-20, -4.0, 0.0]), 1e-8)
    assert np.array_equal(out, [0.5, 1e-8, -0.25, 1e-8])


def _max_res(A, B, X):
    return np.linalg.norm(B - A.apply(X), axis=0).max()


def test_chebyshev2_convergence_ifpack_no_worse_than_textbook():
    n = CHEB2_ROWS
    A, d = _op(laplace1d_rows(n), n)
    xe, _ = oe.epetra_random_mv(3, n, 1)
    B = A.apply(xe)
    r0 = np.linalg.norm(B)
    base = {"chebyshev: degree": CHEB2_DEGREE, "chebyshev: eigenvalue max iterations": CHEB2_EIG_ITERS}
    # Test 1 (lambdaMax given): both variants reduce the residual
    p = dict(base, **{"chebyshev: max eigenvalue": laplace1d_lambda_max(n)})
    assert _max_res(A, B, Chebyshev(A.apply, d, p)(B)) < 1e-2 * r0
    assert _max_res(A, B, Chebyshev(A.apply, d, dict(p, **{"chebyshev: textbook algorithm": True}))(B)) < 1e-2 * r0
    # Test 6 (estimate after 2 x 15 power iterations): the reference's check (:754-771) -- the
    # textbook variant diverges on the under-estimate, Ifpack's boost factor keeps it stable
    p = dict(base, **{"chebyshev: eigenvalue max iterations": 2 * CHEB2_EIG_ITERS})
    ifp = _max_res(A, B, Chebyshev(A.apply, d, p)(B))
    txt = _max_res(A, B, Chebyshev(A.apply, d, dict(p, **{"chebyshev: textbook algorithm": True}))(B))
    assert ifp < 1e-2 * r0
    assert not (ifp > txt and abs(ifp - txt) / txt > 1e-4), (ifp, txt)


def test_power_method_estimate_bounds_the_spectrum():
    """D^-1 A of the 1-D Poisson matrix has eigenvalues 1 - cos(j pi / (n + 1)) in (0, 2): the
    Rayleigh quotients rise towards 2 with the iteration count and never exceed it."""
    n = 400
    A, d = _op(laplace1d_rows(n), n)
    est = [Chebyshev(A.apply, d, {"chebyshev: eigenvalue max iterations": it}).computed_lmax for it in (5, 20, 80)]
    assert 0.0 < est[0] <= est[1] <= est[2] <= 2.0
