"""Known answers held by the reference's own unit tests, through the C ABI on the GPU (the
same problems pin the oracle in test_oracle_pins.py; definitions in known_answers.py).

* Ifpack2_UnitTestRelaxation.cpp Test0 / Test1 / Test3: applyMat = 2, Jacobi apply = 0.5,
  apply(x, x) = 0.5 (the aliased input is copied first), and apply on a process that owns no
  rows -- one GPU and the loopback communicator at P = 2, 3.
* epetra/test/CrsMatrix/cxx_main.cpp power method on the (-1, 2, -1) tridiagonal (10001 rows)
  and on the 10x first diagonal: the device MultiVecTraits + SpMM reproduce the reference's
  success (residual < 0.1 within 200 iterations) at the oracle's iteration, and every lambda
  within 1e-12 relative of the oracle's.
* belos test_bl_gmres_diag.cpp: device Block GMRES on diag(1..10) and 4 I returns
  [1, 1/2, ..., 1/10] and 1/4 with the oracle's iteration counts and history.
"""

import numpy as np
import pytest

from tests.known_answers import (DIAG_TEST_PARAMS, NumpyOps, epetra_tridiag_rows, ifpack2_test_matrix_rows,
                                 power_method)
from tests.parity import hist_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    import torch
    assert torch.cuda.is_available()
    import trilinos_amd as ta
    return ta.Comm(device=0)


def _relaxation_checks(comm, n):
    import trilinos_amd as ta
    gen = ifpack2_test_matrix_rows(n)
    first, nloc = ta.uniform_map(n, comm.nranks, comm.rank)
    rp, gc, vv = gen(first, nloc)
    A = ta.CrsMatrix(comm, n, rp, gc, vv)
    prec = ta.Relaxation(A)
    prec.setParameters({"relaxation: type": "Jacobi"})
    prec.initialize()
    prec.compute()
    x = ta.MultiVector(comm, n, 2)
    y = ta.MultiVector(comm, n, 2)
    x.put_scalar(1.0)
    prec.applyMat(x, y)
    two = y.download()
    prec.apply(x, y)
    half = y.download()
    prec.apply(x, x)  # Test1: x == y
    alias = x.download()
    return nloc, two, half, alias


def test_ifpack2_relaxation_known_answers_one_gpu(comm):
    nloc, two, half, alias = _relaxation_checks(comm, 5)
    assert nloc == 5
    assert np.array_equal(two, np.full((5, 2), 2.0))
    assert np.array_equal(half, np.full((5, 2), 0.5))
    assert np.array_equal(alias, np.full((5, 2), 0.5))


@pytest.mark.parametrize("n,P", [(10, 2), (15, 3), (2, 3)])
def test_ifpack2_relaxation_known_answers_ranks(n, P):
    """5 rows per process (Test0/Test1) and, for n = 2 over 3 ranks, a process with no rows
    (Test3: apply must not fail there)."""
    from tests.test_gpu_loopback import run_ranks
    res = run_ranks(P, lambda c: _relaxation_checks(c, n))
    assert sum(r[0] for r in res) == n
    if n == 2:
        assert res[2][0] == 0
    for nloc, two, half, alias in res:
        assert np.array_equal(two, np.full((nloc, 2), 2.0))
        assert np.array_equal(half, np.full((nloc, 2), 0.5))
        assert np.array_equal(alias, np.full((nloc, 2), 0.5))


class DeviceOps:
    """power_method's operations through the C ABI (MultiVecTraits / OperatorTraits)."""

    def __init__(self, A):
        import trilinos_amd as ta
        self.ta, self.A = ta, A
        self.MVT = ta.MultiVecTraits

    def norm2(self, v):
        return float(self.MVT.MvNorm(v)[0])

    def dot(self, a, b):
        return float(self.MVT.MvDot(a, b)[0])

    def scale(self, out, alpha, v):
        self.MVT.Assign(v, out)
        self.MVT.MvScale(out, alpha)

    def apply(self, x, y):
        self.ta.OperatorTraits.Apply(self.A, x, y)

    def update(self, out, a, A, b, B):
        self.MVT.MvAddMv(a, A, b, B, out)


@pytest.mark.parametrize("diag0", [2.0, 20.0])
def test_epetra_power_method_known_answers(comm, diag0):
    import trilinos_amd as ta
    from oracle import epetra as oe
    n = 10001
    gen = epetra_tridiag_rows(n, diag0)
    rp, gc, vv = gen(0, n)
    A = ta.CrsMatrix(comm, n, rp, gc, vv)
    assert A.nnz_local == 3 * n - 2
    z0, _ = oe.epetra_random_mv(7, n, 1)
    z = ta.MultiVector(comm, n, 1)
    z.upload(z0)
    q, r = ta.MultiVector(comm, n, 1), ta.MultiVector(comm, n, 1)
    ierr, lam, lambdas, res = power_method(DeviceOps(A), z, q, r)
    Aor = oe.DistCrs(gen, n, 1)
    ierr_o, lam_o, lambdas_o, res_o = power_method(NumpyOps(Aor.apply), z0.copy(), np.zeros((n, 1)),
                                                   np.zeros((n, 1)))
    assert ierr == ierr_o == 0
    assert len(lambdas) == len(lambdas_o)
    np.testing.assert_allclose(lambdas, lambdas_o, rtol=1e-12, atol=0)
    np.testing.assert_allclose([v for _, v in res], [v for _, v in res_o], rtol=1e-9, atol=1e-13)
    if diag0 == 20.0:
        assert abs(lam - 20.0) < 0.2


def _diag_solve(comm, d):
    import trilinos_amd as ta
    n = len(d)
    A = ta.CrsMatrix(comm, n, np.arange(n + 1), np.arange(n), np.asarray(d, dtype=np.float64))
    b = ta.MultiVector(comm, n, 1)
    b.put_scalar(1.0)
    X = ta.MultiVector(comm, n, 1)
    X.put_scalar(0.0)
    lp = ta.LinearProblem(A, X, b)
    assert lp.setProblem()
    sm = ta.BlockGmresSolMgr(lp, DIAG_TEST_PARAMS)
    ret = sm.solve()
    return ret, sm, X.download()


@pytest.mark.parametrize("d,want", [(np.arange(1.0, 11.0), 1.0 / np.arange(1.0, 11.0)),
                                    (np.full(10, 4.0), np.full(10, 0.25))])
def test_belos_gmres_diag_known_answers(comm, d, want):
    import trilinos_amd as ta
    from oracle import belos as ob, epetra as oe
    ret, sm, X = _diag_solve(comm, d)
    assert ret == ta.Converged
    np.testing.assert_allclose(X[:, 0], want, rtol=0, atol=1e-10)
    n = len(d)
    Aor = oe.DistCrs(lambda f, m: (np.arange(m + 1), np.arange(f, f + m), d[f:f + m].copy()), n, 1)
    ref = ob.solve(Aor.apply, np.ones((n, 1)), DIAG_TEST_PARAMS)
    assert sm.getNumIters() == ref["iterations"]
    hist_close(sm.residualHistory(), ref["history"])
