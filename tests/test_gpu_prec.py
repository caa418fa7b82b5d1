"""Preconditioned and flexible Block GMRES on the device:
point Jacobi (Ifpack2::Relaxation) as the right or left preconditioner, BlockFGmresIter,
and the GenResNorm implicit / explicit status tests, against the oracle.

Parity bar: Jacobi apply and the 27-point Brick3D SpMM bit for bit; solves with the same
iteration counts, operator/preconditioner applies, explicit checks and implicit residual
history as test_gpu_solver.py.  Pinning: see tests/test_oracle_prec.py (no reference run
of these paths is recorded, so they are pinned through the pinned unpreconditioned
restatement and closed forms)."""

import numpy as np
import pytest

from tests.test_gpu_loopback import run_ranks
from tests.parity import hist_close as _hist_close, true_residuals_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    import torch
    assert torch.cuda.is_available()
    import trilinos_amd as ta
    return ta.Comm(device=0)


def _gen(kind, dims):
    from oracle import epetra as oe
    nx, ny, nz = dims
    if kind == "Brick3D":
        return nx * ny * nz, (lambda f, m: oe.brick3d_rows(nx, ny, nz, f, m))
    return nx * ny * nz, (lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m))


def _oracle_jacobi(gen, n, P, sweeps, damping):
    from oracle import epetra as oe
    from oracle.ifpack2 import Jacobi, crs_diagonal_fast
    A = oe.DistCrs(gen, n, P)
    rp, gc, vv = gen(0, n)
    return A, Jacobi(A.apply, crs_diagonal_fast(rp, gc, vv, 0, n), sweeps, damping)


@pytest.mark.parametrize("kind,dims,k", [("Brick3D", (11, 9, 10), 8), ("Laplace3D", (16, 16, 16), 5),
                                         ("Brick3D", (7, 8, 9), 3)])
def test_brick_spmm_and_jacobi_bit_exact(comm, kind, dims, k):
    import trilinos_amd as ta
    from oracle import epetra as oe
    n, gen = _gen(kind, dims)
    A = ta.CrsMatrix.galeri(comm, kind, *dims)
    X, _ = oe.epetra_random_mv(7, n, k)
    Xd = ta.MultiVector(comm, n, k)
    Xd.upload(X)
    Yd = ta.MultiVector(comm, n, k)
    A.apply(Xd, Yd)
    Aor = oe.DistCrs(gen, n, 1)
    assert np.array_equal(Yd.download(), Aor.apply(X))
    for sweeps, om in [(1, 1.0), (1, 0.7), (2, 1.0), (3, 0.8)]:
        M = ta.Relaxation(A)
        M.setParameters({"relaxation: sweeps": sweeps, "relaxation: damping factor": om})
        M.compute()
        _, Mor = _oracle_jacobi(gen, n, 1, sweeps, om)
        assert np.array_equal(M.inverseDiagonal(), Mor.dinv)
        M.apply(Xd, Yd)
        assert np.array_equal(Yd.download(), Mor(X)), (sweeps, om)


CASES = [
    # (kind, dims, k, nb, side, sweeps, damping, extra params)
    ("Brick3D", (10, 10, 10), 4, 8, "right", 1, 1.0, {}),
    ("Brick3D", (10, 10, 10), 4, 8, "right", 2, 0.8, {"Flexible Gmres": True}),
    ("Laplace3D", (14, 14, 14), 8, 5, "right", 2, 0.8, {}),
    ("Laplace3D", (12, 12, 12), 3, 10, "left", 2, 1.0, {}),
    ("Brick3D", (9, 9, 9), 2, 10, None, 0, 0.0, {"Explicit Residual Test": True,
                                                 "Explicit Residual Scaling": "Norm of RHS"}),
    ("Laplace3D", (12, 12, 12), 4, 6, "right", 3, 0.9, {"Orthogonalization": "DGKS", "Flexible Gmres": True}),
    ("Laplace3D", (10, 11, 12), 3, 7, "both", 2, 0.9, {"Implicit Residual Scaling": "Norm of RHS"}),
]


def _run_case(comm, n, kind, dims, k, params, side, sweeps, damping, B_host, first=0):
    import trilinos_amd as ta
    nloc = ta.uniform_map(n, comm.nranks, comm.rank)[1]
    A = ta.CrsMatrix.galeri(comm, kind, *dims)
    B = ta.MultiVector(comm, n, k)
    B.upload(B_host[first:first + nloc])
    X = ta.MultiVector(comm, n, k)
    X.put_scalar(0.0)
    lp = ta.LinearProblem(A, X, B)
    Ms = []
    if side is not None:
        for s in (("left", "right") if side == "both" else (side,)):
            M = ta.Relaxation(A)
            M.setParameters({"relaxation: sweeps": sweeps, "relaxation: damping factor": damping})
            M.compute()
            Ms.append(M)
            (lp.setLeftPrec if s == "left" else lp.setRightPrec)(M)
    assert lp.setProblem()
    sm = ta.BlockGmresSolMgr(lp, params)
    ret = sm.solve()
    return ret, sm.getNumIters(), sm.counters(), sm.residualHistory(), X.download(), sm.achievedTol()


def oracle_case_rerun(gen, n, P, k, params, side, sweeps, damping):
    """_hist_close's rerun: the oracle case with reversed-order inner products."""
    def run():
        from oracle import belos as ob
        with ob.summation_order("reversed"):
            return _oracle_case(gen, n, P, k, params, side, sweeps, damping)[2]["history"]
    return run


def _oracle_case(gen, n, P, k, params, side, sweeps, damping):
    from oracle import belos as ob, epetra as oe
    Aor, Mor = _oracle_jacobi(gen, n, P, max(sweeps, 1), damping or 1.0)
    Xe, _ = oe.epetra_random_mv(5, n, k)
    B = Aor.apply(Xe)
    kw = {}
    if side in ("left", "both"):
        kw["left"] = Mor
    if side in ("right", "both"):
        kw["right"] = Mor
    return Aor, B, ob.solve(Aor.apply, B, params, **kw)


def _check(res, ref, Aor, B, X, rerun=None, drift_ok=False):
    import trilinos_amd as ta
    ret, iters, c, h, _, tol = res
    assert (ret == ta.Converged) == ref["converged"]
    assert iters == ref["iterations"]
    assert c["applies"] == ref["n_apply"] and c["prec_applies"] == ref["n_prec"]
    assert c["explicit_checks"] == ref["n_explicit"] and c["restarts"] == ref["restarts"]
    _hist_close(h, ref["history"], rerun, drift_ok=drift_ok)
    dh = float(np.abs(h - ref["history"]).max())
    assert abs(tol - ref["achieved_tol"]) <= max(1e-12, dh)
    # the true residuals of the returned X move with the implicit ones (twice their distance)
    rel = np.linalg.norm(B - Aor.apply(X), axis=0) / np.linalg.norm(B, axis=0)
    rel_ref = np.linalg.norm(B - Aor.apply(ref["X"]), axis=0) / np.linalg.norm(B, axis=0)
    true_residuals_close(rel, rel_ref, dh)


@pytest.mark.parametrize("case", range(len(CASES)))
def test_preconditioned_solves_match_oracle(comm, case):
    kind, dims, k, nb, side, sweeps, damping, extra = CASES[case]
    n, gen = _gen(kind, dims)
    params = {"Block Size": k, "Num Blocks": nb, "Maximum Iterations": 600, "Maximum Restarts": 60,
              "Convergence Tolerance": 1e-9, "Orthogonalization": "ICGS"}
    params.update(extra)
    Aor, B, ref = _oracle_case(gen, n, 1, k, params, side, sweeps, damping)
    assert ref["converged"]
    res = _run_case(comm, n, kind, dims, k, params, side, sweeps, damping, B)
    _check(res, ref, Aor, B, res[4], oracle_case_rerun(gen, n, 1, k, params, side, sweeps, damping))


@pytest.mark.parametrize("case,P", [(1, 2), (3, 3), (6, 2)])
def test_distributed_preconditioned_solves(case, P):
    import trilinos_amd as ta
    kind, dims, k, nb, side, sweeps, damping, extra = CASES[case]
    n, gen = _gen(kind, dims)
    params = {"Block Size": k, "Num Blocks": nb, "Maximum Iterations": 600, "Maximum Restarts": 60,
              "Convergence Tolerance": 1e-9, "Orthogonalization": "ICGS"}
    params.update(extra)
    Aor, B, ref = _oracle_case(gen, n, P, k, params, side, sweeps, damping)

    def rank_fn(comm):
        first = ta.uniform_map(n, comm.nranks, comm.rank)[0]
        return first, _run_case(comm, n, kind, dims, k, params, side, sweeps, damping, B, first)

    out = run_ranks(P, rank_fn)
    X = np.zeros((n, k))
    for first, r in out:
        X[first:first + r[4].shape[0]] = r[4]
    rerun = oracle_case_rerun(gen, n, P, k, params, side, sweeps, damping)
    for first, r in out:
        _check(r, ref, Aor, B, X, rerun)


@pytest.mark.parametrize("kind,dims,k,damping", [("Brick3D", (12, 11, 10), 8, 1.0), ("Laplace3D", (13, 12, 11), 4, 0.7),
                                                 ("Laplace2D", (41, 37, 1), 3, 1.0)])
def test_fused_right_jacobi_bit_identical(comm, kind, dims, k, damping, monkeypatch):
    """Right Jacobi (one sweep) fused into the template SpMM forms each operand as
    (omega D^-1) x exactly like the separate Jacobi kernel: the same solve with
    MIGMRES_NO_FUSED_JACOBI=1 returns bit-identical solutions, histories and counters."""
    n, _ = _gen(kind, dims)
    params = {"Block Size": k, "Num Blocks": 12, "Maximum Iterations": 300, "Maximum Restarts": 30,
              "Convergence Tolerance": 1e-9, "Orthogonalization": "ICGS"}
    rng = np.random.default_rng(3)
    B = rng.standard_normal((n, k))
    fused = _run_case(comm, n, kind, dims, k, params, "right", 1, damping, B)
    monkeypatch.setenv("MIGMRES_NO_FUSED_JACOBI", "1")
    plain = _run_case(comm, n, kind, dims, k, params, "right", 1, damping, B)
    assert fused[0] == plain[0] and fused[1] == plain[1] and fused[2] == plain[2]
    assert np.array_equal(fused[3], plain[3])
    assert np.array_equal(fused[4], plain[4])


@pytest.mark.parametrize("kind,dims,k,P", [("Brick3D", (10, 9, 12), 8, 2), ("Brick3D", (9, 10, 11), 8, 3),
                                           ("Laplace3D", (12, 11, 10), 4, 3), ("FlanProxy", (9, 8, 7), 4, 2)])
def test_fused_right_jacobi_under_halo_bit_identical(kind, dims, k, P, monkeypatch):
    """The fused right Jacobi on P ranks (loopback): the halo carries X itself, the interior
    pairs run fused while it is in flight, and the pairs / rows that read ghost columns take
    the owners' omega d^-1 (imported once) in the pair / SELL kernels -- bit-identical to the
    unfused Jacobi pass + SpMM (MIGMRES_NO_FUSED_JACOBI=1): solutions, histories, counters."""
    import trilinos_amd as ta
    n = 3 * dims[0] * dims[1] * dims[2] if kind == "FlanProxy" else dims[0] * dims[1] * dims[2]
    params = {"Block Size": k, "Num Blocks": 8, "Maximum Iterations": 300, "Maximum Restarts": 30,
              "Convergence Tolerance": 1e-9, "Orthogonalization": "ICGS"}
    rng = np.random.default_rng(11)
    B = rng.standard_normal((n, k))

    def run():
        def rank_fn(c):
            first = ta.uniform_map(n, c.nranks, c.rank)[0]
            return first, _run_case(c, n, kind, dims, k, params, "right", 1, 0.9, B, first)
        return run_ranks(P, rank_fn)

    fused = run()
    monkeypatch.setenv("MIGMRES_NO_FUSED_JACOBI", "1")
    plain = run()
    for (f0, a), (f1, b) in zip(fused, plain):
        assert f0 == f1
        assert a[0] == b[0] and a[1] == b[1] and a[2] == b[2]
        assert np.array_equal(a[3], b[3])
        assert np.array_equal(a[4], b[4])


@pytest.mark.parametrize("kind,dims,k,generic", [("Brick3D", (12, 10, 9), 8, True), ("Brick3D", (12, 10, 9), 8, False),
                                                 ("Brick3D", (14, 7, 6), 3, False), ("Laplace3D", (14, 9, 8), 5, False),
                                                 ("Laplace3D", (12, 10, 9), 8, False)])
def test_fused_right_jacobi_march_matches_template_kernels(comm, kind, dims, k, generic, monkeypatch):
    """The fused right Jacobi through the plane march (the staged operand is (omega d^-1) x,
    formed once per X pair; the 7-point specialisation for Laplace3D, the uniform 27-point one
    or the general march for Brick3D) against the same solve through the template kernels (MIGMRES_NO_MARCH=1):
    bit-identical solutions, histories and counters."""
    if generic:
        monkeypatch.setenv("MIGMRES_MARCH_GENERIC", "1")
    n, _ = _gen(kind, dims)
    params = {"Block Size": k, "Num Blocks": 10, "Maximum Iterations": 300, "Maximum Restarts": 30,
              "Convergence Tolerance": 1e-9, "Orthogonalization": "ICGS"}
    B = np.random.default_rng(5).standard_normal((n, k))
    march = _run_case(comm, n, kind, dims, k, params, "right", 1, 0.8, B)
    monkeypatch.setenv("MIGMRES_NO_MARCH", "1")
    tpl = _run_case(comm, n, kind, dims, k, params, "right", 1, 0.8, B)
    assert march[0] == tpl[0] and march[1] == tpl[1] and march[2] == tpl[2]
    assert np.array_equal(march[3], tpl[3])
    assert np.array_equal(march[4], tpl[4])
