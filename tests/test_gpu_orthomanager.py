"""Belos OrthoManager tester invariants on the device ICGS / DGKS managers.

Follows belos/src/BelosOrthoManagerTest.hpp::runTests as driven by
belos/epetra/test/OrthoManager/belos_orthomanager_epetra.cpp:369-378 (sizeS = 5, sizeX1 = 11,
sizeX2 = 13, numRows = 100 per process) for managers that do not claim to be rank revealing
(BelosOrthoManagerFactory.hpp:102-109: only TSQR does, so the rank-deficient cases are not
run), plus a 2^20-row case whose reductions span many workgroups:

* X1 random, normalize(X1) has full rank and ||X1^T X1 - I||_F <= 1e-12 (:400-419);
* X2 random, projectAndNormalize(X2, [X1]) has full rank, ||X2^T X2 - I||_F <= 1e-12 and
  ||X2^T X1||_F <= 1e-12 (:426-463);
* testNormalize (:1171-1279) on a random S: ||Q^T Q - I||_F <= TOL and
  ||S - Q B||_F <= ||S||_F TOL, TOL = eps sqrt(m n^2) sqrt(n);
* testProjectAndNormalizeNew (:1319-1460) of a random S against X1 and X2 (passed as one
  block [X1 X2]; C is their stacked coefficient blocks): the same orthonormality bound,
  ||S - Q B - X1 C1 - X2 C2||_F <= ||S||_F TOL and ||X_i^T Q||_F <= ||S||_F TOL.

The random fills are Epetra_MultiVector::Random streams (MultiVector.random).
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EPS = np.finfo(np.float64).eps
SIZE_S, SIZE_X1, SIZE_X2 = 5, 11, 13


@pytest.fixture(scope="module")
def comm():
    import torch
    assert torch.cuda.is_available()
    import trilinos_amd as ta
    return ta.Comm(device=0)


def _random(ta, comm, n, k, seed):
    mv = ta.MultiVector(comm, n, k)
    mv.random(seed)
    return mv


def _fro(a):
    return float(np.linalg.norm(a))


@pytest.mark.parametrize("n", [100, 1 << 20])
@pytest.mark.parametrize("manager", ["ICGS", "DGKS"])
def test_orthomanager_tester(comm, manager, n):
    import trilinos_amd as ta
    om = ta.ICGSOrthoManager() if manager == "ICGS" else ta.DGKSOrthoManager()

    X1 = _random(ta, comm, n, SIZE_X1, 1)
    rank, _ = om.normalize(X1)
    assert rank == SIZE_X1
    x1 = X1.download()
    assert _fro(x1.T @ x1 - np.eye(SIZE_X1)) <= 1e-12

    X2 = _random(ta, comm, n, SIZE_X2, 2)
    rank, _, _ = om.projectAndNormalize(X2, X1)
    assert rank == SIZE_X2
    x2 = X2.download()
    assert _fro(x2.T @ x2 - np.eye(SIZE_X2)) <= 1e-12
    assert _fro(x2.T @ x1) <= 1e-12

    tol = EPS * np.sqrt(n * SIZE_S * SIZE_S) * np.sqrt(SIZE_S)

    # testNormalize
    S = _random(ta, comm, n, SIZE_S, 3)
    s = S.download()
    rank, B = om.normalize(S)
    assert rank == SIZE_S
    q = S.download()
    assert _fro(q.T @ q - np.eye(SIZE_S)) <= tol
    assert _fro(s - q @ B) <= _fro(s) * tol

    # testProjectAndNormalizeNew against [X1 X2]
    x = np.hstack([x1, x2])
    X = ta.MultiVector(comm, n, SIZE_X1 + SIZE_X2)
    X.upload(x)
    S = _random(ta, comm, n, SIZE_S, 4)
    s = S.download()
    rank, C, B = om.projectAndNormalize(S, X)
    assert rank == SIZE_S
    q = S.download()
    atol = _fro(s)
    assert _fro(q.T @ q - np.eye(SIZE_S)) <= tol
    assert _fro(s - q @ B - x1 @ C[:SIZE_X1] - x2 @ C[SIZE_X1:]) <= atol * tol
    assert _fro(x1.T @ q) <= atol * tol
    assert _fro(x2.T @ q) <= atol * tol
