"""The reference's re-solve and augmented-solve drivers on orsirr1.hb, through the device
solver managers, plus the "Orthogonalization Constant" parameter against the oracle.

* belos/epetra/test/BlockGmres/test_resolve_gmres_hb.cpp (block and --pseudo): solve; X = 0,
  reset(Belos::Problem), solve; X = 0, LinearProblem::setProblem + SolverManager::setProblem,
  solve; new "Timer Label" + reset, solve; a solver built without problem or parameters, then
  setProblem + getValidParameters + setParameters, solve.  Every re-solve must converge and
  its residual vector differ from the first solve's by at most SCT::prec() (= 2 eps) in norm.
* test_pseudo_gmres_hb.cpp: pseudo-block GMRES, 5 random right-hand sides, block size 5,
  Deflation Quorum 5, Num Blocks 100; then 15 (the 5 solved + 10 new), block size 3, quorum 3,
  "Norm of RHS" scaling; every actual relative residual <= tol.  The right-hand sides are
  seeded synthetic columns of the reference's shape (Epetra's Random stream is not restated);
  both solves match the oracle's iteration counts and implicit history.
* "Orthogonalization Constant" > 0 with DGKS sets the ortho manager's dep_tol
  (BelosBlockGmresSolMgr.hpp:607-625, BelosPseudoBlockGmresSolMgr.hpp:736-754).
"""

import numpy as np
import pytest

from tests.parity import hist_close, oracle_rerun

pytestmark = pytest.mark.gpu

SCT_PREC = 2.0 * np.finfo(np.float64).eps   # Teuchos::ScalarTraits<double>::prec() = eps * base


@pytest.fixture(scope="module")
def comm():
    import torch
    assert torch.cuda.is_available()
    import trilinos_amd as ta
    return ta.Comm(device=0)


def _orsirr1(comm):
    import trilinos_amd as ta
    from tests.test_oracle_pins import orsirr1_problem
    n, gen, b, _ = orsirr1_problem()
    rp, gc, vv = gen(0, n)
    return n, gen, b, ta.CrsMatrix(comm, n, rp, gc, vv)


def _resid(ta, A, X, B):
    """resid = B - A X on the device (MVT::MvAddMv(-1, AX, 1, B, resid))."""
    R = ta.MultiVector(A.comm, X.n_global, X.ncols)
    A.apply(X, R)
    ta.MultiVecTraits.MvAddMv(-1.0, R, 1.0, B, R)
    return R


@pytest.mark.parametrize("pseudo", [False, True])
def test_resolve_gmres_hb(comm, pseudo):
    import trilinos_amd as ta
    from oracle import belos as ob, epetra as oe, pseudo as op
    n, gen, b, A = _orsirr1(comm)
    B = ta.MultiVector(comm, n, 1)
    B.upload(b[:, None])
    X = ta.MultiVector(comm, n, 1)
    X.put_scalar(0.0)
    maxiters = n - 1
    params = {"Num Blocks": maxiters, "Block Size": 1, "Maximum Iterations": maxiters, "Maximum Restarts": 15,
              "Convergence Tolerance": 1e-5, "Orthogonalization": "DGKS", "Verbosity": 1 + 2}
    cls = ta.PseudoBlockGmresSolMgr if pseudo else ta.BlockGmresSolMgr
    lp = ta.LinearProblem(A, X, B)
    assert lp.setProblem()
    sm = cls(lp, params)
    assert sm.solve() == ta.Converged
    iters = sm.getNumIters()
    hist = sm.residualHistory()
    resid = _resid(ta, A, X, B).download()

    Aor = oe.DistCrs(gen, n, 1)
    solve = op.solve if pseudo else ob.solve
    ref = solve(Aor.apply, b[:, None], params)
    assert iters == ref["iterations"]
    if not pseudo:
        assert iters == 209   # the recorded reference run
    hist_close(hist, ref["history"], oracle_rerun(solve, Aor.apply, b[:, None], params))

    def resolved(label, X_out):
        assert sm.solve() == ta.Converged, label
        assert sm.getNumIters() == iters, label
        d = np.linalg.norm(_resid(ta, A, X_out, B).download() - resid, axis=0)
        assert d.max() <= SCT_PREC, (label, d)

    X.put_scalar(0.0)                       # reset(Belos::Problem)
    sm.reset(1)
    resolved("manager reset", X)
    X.put_scalar(0.0)                       # LinearProblem::setProblem + SolverManager::setProblem
    assert lp.setProblem()
    sm.setProblem(lp)
    resolved("manager setProblem()", X)
    sm.setParameters({"Timer Label": "Belos Resolve w/ New Label"})
    assert sm.getCurrentParameters()["Timer Label"] == "Belos Resolve w/ New Label"
    X.put_scalar(0.0)
    sm.reset(1)
    resolved("label reset", X)

    X2 = ta.MultiVector(comm, n, 1)         # a solver made without problem or parameter list
    X2.put_scalar(0.0)
    lp2 = ta.LinearProblem(A, X2, B)
    assert lp2.setProblem()
    sm = cls()
    sm.setProblem(lp2)
    valid = sm.getValidParameters()
    assert valid["Timer Label"] == "Belos" and valid["Orthogonalization Constant"] == -1.0
    sm.setParameters(dict(params, **{"Timer Label": "Belos Resolve"}))
    resolved("new solver", X2)


def test_pseudo_gmres_hb(comm):
    import trilinos_amd as ta
    from oracle import epetra as oe, pseudo as op
    n, gen, _, A = _orsirr1(comm)
    Aor = oe.DistCrs(gen, n, 1)
    init_numrhs, aug_numrhs, tol = 5, 10, 1e-5
    base = {"Num Blocks": 100, "Maximum Iterations": n - 1, "Maximum Restarts": 15,
            "Convergence Tolerance": tol, "Verbosity": 1 + 2}
    init_params = dict(base, **{"Block Size": 5, "Deflation Quorum": 5, "Timer Label": "Belos Init"})
    aug_params = dict(base, **{"Block Size": 3, "Deflation Quorum": 3, "Timer Label": "Belos Aug",
                               "Implicit Residual Scaling": "Norm of RHS",
                               "Explicit Residual Scaling": "Norm of RHS"})

    def run(Xtrue, X0, params):
        k = Xtrue.shape[1]
        Bh = Aor.apply(Xtrue)
        B, X = ta.MultiVector(comm, n, k), ta.MultiVector(comm, n, k)
        B.upload(Bh)
        X.upload(X0)
        lp = ta.LinearProblem(A, X, B)
        assert lp.setProblem()
        sm = ta.PseudoBlockGmresSolMgr(lp, params)
        ret = sm.solve()
        Xd = X.download()
        act = np.linalg.norm(Bh - Aor.apply(Xd), axis=0) / np.linalg.norm(Bh, axis=0)
        ref = op.solve(Aor.apply, Bh, params, X0=X0.copy())
        assert ret == ta.Converged and ref["converged"]
        assert sm.getNumIters() == ref["iterations"]
        hist_close(sm.residualHistory(), ref["history"],
                   oracle_rerun(op.solve, Aor.apply, Bh, params, X0=X0.copy()))
        assert (act <= tol).all(), act
        return Xd

    init_true, _ = oe.epetra_random_mv(11, n, init_numrhs)
    init_X = run(init_true, np.zeros((n, init_numrhs)), init_params)
    aug_true, _ = oe.epetra_random_mv(12, n, init_numrhs + aug_numrhs)
    aug_true[:, :init_numrhs] = init_true     # augB's first columns are initB
    X0 = np.zeros((n, init_numrhs + aug_numrhs))
    X0[:, :init_numrhs] = init_X              # augX's first columns are the initial solution
    run(aug_true, X0, aug_params)


@pytest.mark.parametrize("pseudo", [False, True])
@pytest.mark.parametrize("kappa", [0.3, 0.99])
def test_orthogonalization_constant(comm, pseudo, kappa):
    """DGKS with dep_tol = kappa: kappa = 0.99 re-orthogonalises nearly every column, 0.3
    almost none; the device solve follows the oracle's iteration count and history."""
    import trilinos_amd as ta
    from oracle import belos as ob, epetra as oe, pseudo as op
    nx, ny, k = 24, 23, 3
    n = nx * ny
    gen = lambda f, m: oe.laplace2d_rows(nx, ny, f, m)  # noqa: E731
    Aor = oe.DistCrs(gen, n, 1)
    Xe, _ = oe.epetra_random_mv(5, n, k)
    Bh = Aor.apply(Xe)
    params = {"Block Size": k, "Num Blocks": 25, "Maximum Iterations": 600, "Maximum Restarts": 40,
              "Convergence Tolerance": 1e-9, "Orthogonalization": "DGKS", "Orthogonalization Constant": kappa}
    A = ta.CrsMatrix.galeri(comm, "Laplace2D", nx, ny)
    B, X = ta.MultiVector(comm, n, k), ta.MultiVector(comm, n, k)
    B.upload(Bh)
    X.put_scalar(0.0)
    lp = ta.LinearProblem(A, X, B)
    assert lp.setProblem()
    sm = (ta.PseudoBlockGmresSolMgr if pseudo else ta.BlockGmresSolMgr)(lp, params)
    assert sm.getCurrentParameters()["Orthogonalization Constant"] == kappa
    assert sm.solve() == ta.Converged
    solve = op.solve if pseudo else ob.solve
    ref = solve(Aor.apply, Bh, params)
    assert sm.getNumIters() == ref["iterations"]
    hist_close(sm.residualHistory(), ref["history"], oracle_rerun(solve, Aor.apply, Bh, params))
