"""PseudoBlockGmresSolMgr on the device against the oracle
(oracle/pseudo.py): iteration counts, restarts, deflations, operator applies, explicit
checks and the implicit residual history with the tolerance of test_gpu_solver.py.
Pinning: PseudoBlockGmres(1 RHS) is checked equal to the pinned BlockGmres(k = 1)
restatement in tests/test_oracle_prec.py."""

import numpy as np
import pytest

from tests.test_gpu_loopback import run_ranks
from tests.parity import hist_close as _hist_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    import torch
    assert torch.cuda.is_available()
    import trilinos_amd as ta
    return ta.Comm(device=0)


def _problem(kind, dims, nrhs, seed=3):
    from oracle import epetra as oe
    nx, ny, nz = dims
    if kind == "Laplace2D":
        n, gen = nx * ny, (lambda f, m: oe.laplace2d_rows(nx, ny, f, m))
    elif kind == "Brick3D":
        n, gen = nx * ny * nz, (lambda f, m: oe.brick3d_rows(nx, ny, nz, f, m))
    else:
        n, gen = nx * ny * nz, (lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m))
    Xe, _ = oe.epetra_random_mv(seed, n, nrhs)
    Xe[:, 0] = np.sin(np.arange(n) * 0.01)   # a smooth column converges first: deflation
    return n, gen, Xe


CASES = [
    ("Laplace2D", (30, 30, 1), 4, {"Block Size": 4, "Num Blocks": 20}, None),
    ("Laplace2D", (30, 30, 1), 4, {"Block Size": 4, "Num Blocks": 20, "Deflation Quorum": 4}, None),
    ("Laplace2D", (28, 31, 1), 5, {"Block Size": 3, "Num Blocks": 15, "Orthogonalization": "DGKS"}, None),
    ("Laplace3D", (12, 12, 12), 8, {"Block Size": 8, "Num Blocks": 12, "Explicit Residual Test": True}, None),
    ("Brick3D", (10, 10, 10), 4, {"Block Size": 4, "Num Blocks": 10}, ("right", 2, 0.8)),
    ("Laplace3D", (10, 10, 10), 3, {"Block Size": 3, "Num Blocks": 10}, ("left", 2, 1.0)),
]


def _params(extra):
    p = {"Maximum Iterations": 800, "Maximum Restarts": 80, "Convergence Tolerance": 1e-9}
    p.update(extra)
    return p


def _oracle(gen, n, P, Xe, params, prec):
    from oracle import epetra as oe, pseudo
    from oracle.ifpack2 import Jacobi, crs_diagonal_fast
    A = oe.DistCrs(gen, n, P)
    B = A.apply(Xe)
    kw = {}
    if prec:
        side, sweeps, om = prec
        rp, gc, vv = gen(0, n)
        kw[side] = Jacobi(A.apply, crs_diagonal_fast(rp, gc, vv, 0, n), sweeps, om)
    return A, B, pseudo.solve(A.apply, B, params, **kw)


def _device(comm, kind, dims, n, B, params, prec):
    import trilinos_amd as ta
    first, nloc = ta.uniform_map(n, comm.nranks, comm.rank)
    A = ta.CrsMatrix.galeri(comm, kind, *dims)
    k = B.shape[1]
    Bd = ta.MultiVector(comm, n, k)
    Bd.upload(B[first:first + nloc])
    X = ta.MultiVector(comm, n, k)
    X.put_scalar(0.0)
    lp = ta.LinearProblem(A, X, Bd)
    M = None
    if prec:
        side, sweeps, om = prec
        M = ta.Relaxation(A)
        M.setParameters({"relaxation: sweeps": sweeps, "relaxation: damping factor": om})
        M.compute()
        (lp.setLeftPrec if side == "left" else lp.setRightPrec)(M)
    assert lp.setProblem()
    sm = ta.SolverFactory("GMRES", lp, params)
    assert isinstance(sm, ta.PseudoBlockGmresSolMgr)
    ret = sm.solve()
    return first, ret, sm.getNumIters(), sm.counters(), sm.residualHistory(), X.download(), sm.achievedTol()


def _rerun(gen, n, P, Xe, params, prec):
    def run():
        from oracle import belos as ob
        with ob.summation_order("reversed"):
            return _oracle(gen, n, P, Xe, params, prec)[2]["history"]
    return run


def _check(res, ref, A, B, X, rerun=None):
    import trilinos_amd as ta
    _, ret, iters, c, h, _, tol = res
    assert (ret == ta.Converged) == ref["converged"]
    assert iters == ref["iterations"]
    assert c["restarts"] == ref["restarts"] and c["deflations"] == ref["deflations"]
    assert c["applies"] == ref["n_apply"] and c["prec_applies"] == ref["n_prec"]
    assert c["explicit_checks"] == ref["n_explicit"]
    _hist_close(h, ref["history"], rerun)
    assert abs(tol - ref["achieved_tol"]) <= max(1e-12, np.abs(h - ref["history"]).max())
    rel = np.linalg.norm(B - A.apply(X), axis=0) / np.linalg.norm(B, axis=0)
    rel_ref = np.linalg.norm(B - A.apply(ref["X"]), axis=0) / np.linalg.norm(B, axis=0)
    np.testing.assert_allclose(rel, rel_ref, rtol=1e-3, atol=1e-12)


@pytest.mark.parametrize("batched", ["1", "0"])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_pseudo_block_solves_match_oracle(comm, case, batched, monkeypatch):
    """Both device orthogonalisations: all right-hand sides batched through the block kernels
    (default) and one k = 1 chain per right-hand side (MIGMRES_PSEUDO_BATCHED=0)."""
    monkeypatch.setenv("MIGMRES_PSEUDO_BATCHED", batched)
    kind, dims, nrhs, extra, prec = CASES[case]
    n, gen, Xe = _problem(kind, dims, nrhs)
    params = _params(extra)
    A, B, ref = _oracle(gen, n, 1, Xe, params, prec)
    assert ref["converged"]
    res = _device(comm, kind, dims, n, B, params, prec)
    _check(res, ref, A, B, res[5], _rerun(gen, n, 1, Xe, params, prec))


@pytest.mark.parametrize("case,P", [(0, 2), (4, 3)])
def test_distributed_pseudo_block(case, P):
    kind, dims, nrhs, extra, prec = CASES[case]
    n, gen, Xe = _problem(kind, dims, nrhs)
    params = _params(extra)
    A, B, ref = _oracle(gen, n, P, Xe, params, prec)
    out = run_ranks(P, lambda comm: _device(comm, kind, dims, n, B, params, prec))
    X = np.zeros_like(B)
    for r in out:
        X[r[0]:r[0] + r[5].shape[0]] = r[5]
    rerun = _rerun(gen, n, P, Xe, params, prec)
    for r in out:
        _check(r, ref, A, B, X, rerun)


def test_pseudo_parameter_validation(comm):
    import trilinos_amd as ta
    from trilinos_amd._lib import MigmresError
    n, gen, Xe = _problem("Laplace2D", (10, 10, 1), 2)
    A = ta.CrsMatrix.galeri(comm, "Laplace2D", 10, 10)
    X = ta.MultiVector(comm, n, 2)
    B = ta.MultiVector(comm, n, 2)
    lp = ta.LinearProblem(A, X, B)
    lp.setProblem()
    with pytest.raises(KeyError):
        ta.PseudoBlockGmresSolMgr(lp, {"Flexible Gmres": True})
    sm = ta.PseudoBlockGmresSolMgr(lp, {"Block Size": 2, "Deflation Quorum": 3})
    with pytest.raises(MigmresError):
        sm.solve()


def test_solver_manager_parameter_lists_and_reset(comm):
    """getValidParameters / getCurrentParameters / reset through the C ABI
    (BelosSolverManager.hpp:98-101, 177): the valid list is the reference's defaults, the
    current list follows setParameters, reset(Problem) clears the previous solve's results."""
    import trilinos_amd as ta
    from trilinos_amd._lib import MigmresError
    from trilinos_amd.belos import DEFAULT_PARAMETERS, PSEUDO_DEFAULT_PARAMETERS
    n, gen, Xe = _problem("Laplace2D", (12, 11, 1), 2)
    A = ta.CrsMatrix.galeri(comm, "Laplace2D", 12, 11)
    for cls, defaults in ((ta.BlockGmresSolMgr, DEFAULT_PARAMETERS),
                          (ta.PseudoBlockGmresSolMgr, PSEUDO_DEFAULT_PARAMETERS)):
        Xd, B = ta.MultiVector(comm, n, 2), ta.MultiVector(comm, n, 2)
        Xv = ta.MultiVector(comm, n, 2)
        Xv.upload(Xe)
        A.apply(Xv, B)
        Xd.put_scalar(0.0)
        lp = ta.LinearProblem(A, Xd, B)
        lp.setProblem()
        sm = cls(lp, {"Block Size": 2, "Num Blocks": 7, "Convergence Tolerance": 1e-7,
                      "Orthogonalization": "ICGS"})
        sm._ensure()
        assert sm.getValidParameters() == defaults
        cur = sm.getCurrentParameters()
        assert cur == dict(defaults, **{"Block Size": 2, "Num Blocks": 7, "Convergence Tolerance": 1e-7,
                                        "Orthogonalization": "ICGS"})
        assert sm.solve() == ta.Converged and sm.getNumIters() > 0
        sm.reset(1)
        assert sm.getNumIters() == 0 and sm.residualHistory().size == 0
        assert sm.counters()["applies"] == 0
        with pytest.raises(MigmresError):
            sm.reset(4)


def test_user_conv_status_test(comm):
    """setUserConvStatusTest (pseudo-block only, BelosPseudoBlockGmresSolMgr.hpp:1070-1078,
    combined with the residual test at :1216-1240): SEQ with an always-passing test = no user
    test; SEQ that passes only from a later iteration on delays convergence to it; AND with a
    never-passing test runs to Maximum Iterations; BlockGmresSolMgr refuses, as the reference's
    base class throws."""
    import trilinos_amd as ta
    from trilinos_amd._lib import MigmresError
    n, gen, Xe = _problem("Laplace2D", (14, 13, 1), 2)
    params = {"Block Size": 2, "Num Blocks": 200, "Maximum Iterations": 200, "Convergence Tolerance": 1e-6}

    def run(test, combo):
        A = ta.CrsMatrix.galeri(comm, "Laplace2D", 14, 13)
        Xv, B, X = ta.MultiVector(comm, n, 2), ta.MultiVector(comm, n, 2), ta.MultiVector(comm, n, 2)
        Xv.upload(Xe)
        A.apply(Xv, B)
        X.put_scalar(0.0)
        lp = ta.LinearProblem(A, X, B)
        lp.setProblem()
        sm = ta.PseudoBlockGmresSolMgr(lp, params)
        seen = []
        if test is not None:
            sm.setUserConvStatusTest(lambda it, res: (seen.append((it, res.copy())), test(it, res))[1], combo)
        ret = sm.solve()
        return ret, sm.getNumIters(), sm.residualHistory(), seen

    ret0, it0, h0, _ = run(None, "SEQ")
    assert ret0 == ta.Converged and it0 + 30 < params["Maximum Iterations"]
    ret1, it1, h1, seen1 = run(lambda it, res: True, "SEQ")
    assert (ret1, it1) == (ret0, it0) and np.array_equal(h1, h0)
    # SEQ: the user test is asked only once the residual test passed (some column converged)
    assert seen1 and all(np.any(r <= 1e-6) for _, r in seen1)
    late = it0 + 10
    ret2, it2, _, _ = run(lambda it, res: it >= late, "SEQ")
    assert ret2 == ta.Converged and it2 == late
    params["Maximum Iterations"] = it0 + 20
    ret3, it3, _, seen3 = run(lambda it, res: False, "AND")
    assert ret3 == ta.Unconverged and it3 == params["Maximum Iterations"] and len(seen3) >= it3
    A = ta.CrsMatrix.galeri(comm, "Laplace2D", 14, 13)
    lp = ta.LinearProblem(A, ta.MultiVector(comm, n, 2), ta.MultiVector(comm, n, 2))
    lp.setProblem()
    sm = ta.BlockGmresSolMgr(lp, params)
    with pytest.raises(MigmresError):
        sm.setUserConvStatusTest(lambda it, res: True)
