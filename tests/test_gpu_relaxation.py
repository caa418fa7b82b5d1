"""Ifpack2::Relaxation's full option set on the device against oracle/ifpack2.py Relaxation:
"relaxation: type" Jacobi and Richardson, several sweeps and damping factors, zero and
nonzero starting solution, "use l1" (with its off-process boost, so on P > 1 ranks) and
"fix tiny diagonal entries" / "min diagonal value".  Elementwise work plus the bit-exact SpMM:
the device result equals the oracle's bit for bit, P = 1 and 3.  Known answers:
Ifpack2_UnitTestRelaxation.cpp Test4 (l1) and Richardson apply on the diag(2) test matrix.
"""

import numpy as np
import pytest

from tests.known_answers import ifpack2_test_matrix_rows
from tests.parity import hist_close, oracle_rerun
from tests.test_gpu_loopback import run_ranks

pytestmark = pytest.mark.gpu


def _gen(kind):
    from oracle import epetra as oe
    if kind == "tiny":   # a 2-D Laplacian whose diagonal entry of every 7th row is 1e-20
        def g(f, m):
            rp, gc, vv = oe.laplace2d_rows(23, 21, f, m)
            vv = np.array(vv, dtype=np.float64)
            for i in range(m):
                if (f + i) % 7 == 0:
                    for e in range(rp[i], rp[i + 1]):
                        if gc[e] == f + i:
                            vv[e] = 1e-20
            return rp, gc, vv
        return 23 * 21, g
    return 29 * 31, (lambda f, m: oe.laplace2d_rows(29, 31, f, m))


def _device(comm, n, gen, params, X, Y0):
    import trilinos_amd as ta
    first, nloc = ta.uniform_map(n, comm.nranks, comm.rank)
    rp, gc, vv = gen(first, nloc)
    A = ta.CrsMatrix(comm, n, rp, gc, vv)
    M = ta.Relaxation(A)
    M.setParameters(params)
    M.initialize()
    M.compute()
    k = X.shape[1]
    Xd, Yd = ta.MultiVector(comm, n, k), ta.MultiVector(comm, n, k)
    Xd.upload(X[first:first + nloc])
    if Y0 is None:
        Yd.put_scalar(0.0)
    else:
        Yd.upload(Y0[first:first + nloc])
    M.apply(Xd, Yd)
    return first, Yd.download(), M.inverseDiagonal()


CASES = [
    ("lap", {"relaxation: sweeps": 3, "relaxation: damping factor": 0.8}, False),
    ("lap", {"relaxation: sweeps": 2, "relaxation: zero starting solution": False}, True),
    ("lap", {"relaxation: type": "Richardson", "relaxation: damping factor": 0.2}, False),
    ("lap", {"relaxation: type": "Richardson", "relaxation: sweeps": 4, "relaxation: damping factor": 0.2,
             "relaxation: zero starting solution": False}, True),
    ("lap", {"relaxation: use l1": True, "relaxation: l1 eta": 10.0, "relaxation: sweeps": 2}, False),
    ("tiny", {"relaxation: fix tiny diagonal entries": True, "relaxation: min diagonal value": 1e-8}, False),
    ("tiny", {"relaxation: fix tiny diagonal entries": True, "relaxation: check diagonal entries": True}, False),
]


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_relaxation_options_bit_exact(case, P):
    import trilinos_amd as ta
    from oracle import epetra as oe
    from oracle.ifpack2 import Relaxation
    kind, params, nonzero = CASES[case]
    n, gen = _gen(kind)
    X, _ = oe.epetra_random_mv(5, n, 3)
    Y0 = oe.epetra_random_mv(8, n, 3)[0] if nonzero else None
    Mo = Relaxation(oe.DistCrs(gen, n, P), params)
    want = Mo(X, Y0)
    if P == 1:
        res = [_device(ta.Comm(device=0), n, gen, params, X, Y0)]
    else:
        res = run_ranks(P, lambda c: _device(c, n, gen, params, X, Y0))
    for first, got, dinv in res:
        m = got.shape[0]
        assert np.array_equal(dinv, Mo.dinv[first:first + m])
        assert np.array_equal(got, want[first:first + m])
    if params.get("relaxation: use l1") and P > 1:
        from oracle.ifpack2 import relaxation_inverse_diagonal
        plain = relaxation_inverse_diagonal(oe.DistCrs(gen, n, P), {})
        assert np.any(plain != Mo.dinv)  # the l1 boost changed some rows


@pytest.mark.parametrize("rtype", ["Jacobi", "Richardson"])
def test_relaxation_test4_and_richardson_known_answers(rtype):
    """Ifpack2_UnitTestRelaxation.cpp Test4 ("use l1", Jacobi) and Richardson: apply on the
    diag(2) test matrix with 5 rows per process succeeds -- here also equal to the oracle
    (1/2 for Jacobi, omega = 1 for Richardson: y = x)."""
    n, P = 10, 2
    gen = ifpack2_test_matrix_rows(n)
    params = {"relaxation: type": rtype}
    if rtype == "Jacobi":
        params["relaxation: use l1"] = True
    X = np.ones((n, 2))
    for first, got, _ in run_ranks(P, lambda c: _device(c, n, gen, params, X, None)):
        assert got.shape[0] == 5
        np.testing.assert_array_equal(got, np.full((5, 2), 0.5 if rtype == "Jacobi" else 1.0))


def test_block_gmres_with_richardson_right_prec():
    import trilinos_amd as ta
    from oracle import belos as ob, epetra as oe
    from oracle.ifpack2 import Relaxation
    comm = ta.Comm(device=0)
    nx, ny, nz = 12, 11, 10
    n = nx * ny * nz
    gen = lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m)  # noqa: E731
    prm = {"relaxation: type": "Richardson", "relaxation: sweeps": 2, "relaxation: damping factor": 0.1}
    Aor = oe.DistCrs(gen, n, 1)
    Mo = Relaxation(Aor, prm)
    Xe, _ = oe.epetra_random_mv(3, n, 4)
    Bh = Aor.apply(Xe)
    params = {"Block Size": 4, "Num Blocks": 15, "Maximum Iterations": 300, "Maximum Restarts": 20,
              "Convergence Tolerance": 1e-9, "Orthogonalization": "ICGS"}
    ref = ob.solve(Aor.apply, Bh, params, right=Mo)
    A = ta.CrsMatrix.galeri(comm, "Laplace3D", nx, ny, nz)
    M = ta.Relaxation(A)
    M.setParameters(prm)
    M.compute()
    B, X = ta.MultiVector(comm, n, 4), ta.MultiVector(comm, n, 4)
    B.upload(Bh)
    X.put_scalar(0.0)
    lp = ta.LinearProblem(A, X, B)
    lp.setRightPrec(M)
    assert lp.setProblem()
    sm = ta.BlockGmresSolMgr(lp, params)
    assert (sm.solve() == ta.Converged) == ref["converged"]
    assert sm.getNumIters() == ref["iterations"]
    hist_close(sm.residualHistory(), ref["history"], oracle_rerun(ob.solve, Aor.apply, Bh, params, right=Mo))
