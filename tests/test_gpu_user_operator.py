"""User operators on the whole-solver path (migmres_op_create / migmres_solver_solve_op /
migmres_solver_set_prec_op; the reference's LinearProblem applies any OP through
OperatorTraits::Apply, BelosOperatorTraits.hpp:108-155, BelosLinearProblem.hpp:989-1072).

* belos/epetra/test/BlockGmres/test_bl_gmres_diag.cpp with its own operator classes as
  callbacks: Diagonal_Operator (y.Scale(v, x)), Diagonal_Operator_2 (y_i = (i+1) v x_i),
  Iterative_Inverse_Operator (a Block GMRES solve per apply), Composed_Operator -- inv(D2) 1 =
  [1, 1/2, ..., 1/10], inv(4 I) 1 = 1/4 and the nested inv(inv(4 I) 4 I) 1 = 1 to 1e-10
  (:364-395), the outer solve applying an operator that runs a whole inner device solve; the
  iteration counts and histories equal the oracle's (tests/test_oracle_pins.py restates the
  same nesting);
* a CRS operator through a callback gives the same solve, bit for bit, as the CRS itself;
* a user operator as the right preconditioner equals the library's Jacobi bit for bit;
* a callback that fails ends the solve with MIGMRES_EOP.
"""

import numpy as np
import pytest

from tests.known_answers import DIAG_TEST_PARAMS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    import torch
    assert torch.cuda.is_available()
    import trilinos_amd as ta
    return ta.Comm(device=0)


def _diag_crs(comm, d):
    import trilinos_amd as ta
    n = len(d)
    return ta.CrsMatrix(comm, n, np.arange(n + 1), np.arange(n), np.asarray(d, dtype=np.float64))


def diagonal_operator(comm, n, v):
    """Diagonal_Operator (:100-115): y.Scale(v, x), i.e. y_i = v * x_i."""
    import trilinos_amd as ta
    MVT = ta.MultiVecTraits

    def apply(X, Y):
        MVT.Assign(X, Y)
        MVT.MvScale(Y, v)
    return ta.Operator(comm, n, apply)


def diagonal_operator_2(comm, n, v):
    """Diagonal_Operator_2 (:119-138): y_i = (i+1) v x_i -- a diagonal CRS holding (i+1) v
    computes the same product."""
    import trilinos_amd as ta
    D = _diag_crs(comm, np.arange(1, n + 1) * v)
    return ta.Operator(comm, n, lambda X, Y: D.apply(X, Y)), D


class IterativeInverse:
    """Iterative_Inverse_Operator (:233-305): each apply is x.PutScalar(0), setProblem(x, b)
    and a Block GMRES solve (Num Blocks n / bs, Block Size bs, 100 iterations, 10 restarts,
    tol 1e-10, default orthogonalization) with operator `op`."""

    def __init__(self, comm, n, bs, op):
        import trilinos_amd as ta
        self.ta, self.op, self.n = ta, op, n
        self.params = {"Num Blocks": n // bs, "Block Size": bs, "Maximum Iterations": 100,
                       "Maximum Restarts": 10, "Convergence Tolerance": 1.0e-10}
        self.solver = ta.BlockGmresSolMgr(None, self.params)
        self.iters = []

    def __call__(self, B, X):
        X.put_scalar(0.0)
        lp = self.ta.LinearProblem(self.op, X, B)
        assert lp.setProblem()
        self.solver.setProblem(lp)
        ret = self.solver.solve()
        self.iters.append((self.solver.getNumIters(), ret == self.ta.Converged))

    def operator(self, comm):
        return self.ta.Operator(comm, self.n, lambda X, Y: self(X, Y))


def test_bl_gmres_diag_inverse_of_d2(comm):
    import trilinos_amd as ta
    n = 10
    D2, _keep = diagonal_operator_2(comm, n, 1.0)
    A2 = IterativeInverse(comm, n, 1, D2)
    X, Y = ta.MultiVector(comm, n, 1), ta.MultiVector(comm, n, 1)
    X.put_scalar(1.0)
    A2(X, Y)
    np.testing.assert_allclose(Y.download()[:, 0], 1.0 / np.arange(1, n + 1), rtol=0, atol=1e-10)
    assert A2.iters[-1][1]


def test_bl_gmres_diag_nested_inverse(comm):
    """The outer Block GMRES applies C = inv(D) B, whose every apply is an inner device solve:
    ||inv(C) 1 - 1|| < 1e-10 (:364-395)."""
    import trilinos_amd as ta
    from oracle import belos as ob
    from oracle import epetra as oe
    n = 10
    inner = IterativeInverse(comm, n, 1, diagonal_operator(comm, n, 4.0))
    Bop = diagonal_operator(comm, n, 4.0)
    MVT = ta.MultiVecTraits

    def composed_apply(X, Y):  # Composed_Operator (:142-175): ytemp = B x, y = Inner(ytemp)
        ytemp = ta.MultiVector(comm, n, X.ncols)
        Bop.apply(X, ytemp)
        inner(ytemp, Y)
    C = ta.Operator(comm, n, composed_apply)
    outer = IterativeInverse(comm, n, 1, C)
    X, Y = ta.MultiVector(comm, n, 1), ta.MultiVector(comm, n, 1)
    X.put_scalar(1.0)
    inner(X, Y)
    np.testing.assert_allclose(Y.download(), 0.25, rtol=0, atol=1e-10)
    n_inner_before = len(inner.iters)
    outer(X, Y)
    y = Y.download()
    MVT.MvAddMv(-1.0, X, 1.0, Y, Y)
    assert float(MVT.MvNorm(Y)[0]) < 1e-10
    assert outer.iters[-1][1]
    assert len(inner.iters) > n_inner_before  # the outer solve ran inner solves
    # the oracle's nesting (test_oracle_pins.py::test_belos_gmres_diag_known_answers)
    D = oe.DistCrs(lambda f, m: (np.arange(m + 1), np.arange(f, f + m), np.full(m, 4.0)), n, 1)

    def o_inner(b):
        return ob.solve(D.apply, b, DIAG_TEST_PARAMS)["X"]
    r = ob.solve(lambda v: o_inner(4.0 * v), np.ones((n, 1)), DIAG_TEST_PARAMS)
    assert r["iterations"] == outer.iters[-1][0]
    np.testing.assert_allclose(y, r["X"], rtol=0, atol=1e-12)


def _laplace(comm, nx):
    import trilinos_amd as ta
    from oracle import epetra as oe
    n = nx ** 3
    first, nloc = ta.uniform_map(n, comm.nranks, comm.rank)
    return n, ta.CrsMatrix(comm, n, *oe.laplace3d_rows(nx, nx, nx, first, nloc))


def _solve(comm, n, A, prec=None, k=4):
    import trilinos_amd as ta
    from oracle import epetra as oe
    B0, _ = oe.epetra_random_mv(3, n, k)
    X, B = ta.MultiVector(comm, n, k), ta.MultiVector(comm, n, k)
    X.put_scalar(0.0)
    B.upload(B0)
    lp = ta.LinearProblem(A, X, B)
    if prec is not None:
        lp.setRightPrec(prec)
    assert lp.setProblem()
    sm = ta.BlockGmresSolMgr(lp, {"Block Size": k, "Num Blocks": 20, "Maximum Iterations": 300,
                                  "Convergence Tolerance": 1e-9, "Orthogonalization": "ICGS"})
    ret = sm.solve()
    return ret, sm.getNumIters(), X.download()


def test_crs_through_callback_equals_crs(comm):
    import trilinos_amd as ta
    n, A = _laplace(comm, 12)
    want = _solve(comm, n, A)
    got = _solve(comm, n, ta.Operator(comm, n, lambda X, Y: A.apply(X, Y)))
    assert want[0] == got[0] and want[1] == got[1]
    assert np.array_equal(want[2], got[2])


def test_user_right_preconditioner_equals_jacobi(comm):
    import trilinos_amd as ta
    n, A = _laplace(comm, 10)
    J = ta.Relaxation(A)
    J.setParameters({"relaxation: type": "Jacobi", "relaxation: damping factor": 0.8})
    J.initialize()
    J.compute()
    want = _solve(comm, n, A, J)
    got = _solve(comm, n, A, ta.Operator(comm, n, lambda X, Y: J.apply(X, Y)))
    assert want[0] == got[0] and want[1] == got[1]
    assert np.array_equal(want[2], got[2])


def test_failing_callback_fails_the_solve(comm):
    import trilinos_amd as ta
    n = 10

    def bad(X, Y):
        raise ValueError("operator broke")
    op = ta.Operator(comm, n, bad)
    with pytest.raises(ta.linalg.MigmresError):
        IterativeInverse(comm, n, 1, op)(*(ta.MultiVector(comm, n, 1) for _ in range(2)))
    assert isinstance(op.error, ValueError)
