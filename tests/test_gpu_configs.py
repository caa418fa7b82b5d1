"""BASELINE.json's configurations 3-5 on the HIP path ("untested configs").

* Config 3 (7-point Laplacian, k = 16 right-hand sides, 1-D row partition): Block GMRES
  solves with Block Size 16 against the oracle on one GPU and through the loopback
  communicator at P = 2 and 4 (the distributed path above RCCL), and at full per-GPU size
  (256^3, the slice one of 8 GPUs holds at 512^3) the size-independent properties of
  test_gpu_fullsize.py: monotone implicit residuals, implicit = explicit after a cycle, bit
  for bit reproducible.
* Config 5 (27-point Brick3D, Ifpack2 Jacobi, k = 8): right-preconditioned solves against the
  oracle (one GPU, P = 2), and the full 384^3 problem on one GPU (basis 94 GB + CSR 18 GB
  fit in 288 GB): sampled SpMM / Jacobi rows bit for bit, then the properties above.
* Config 4 (SuiteSparse Flan_1565, k = 4): the file is not in this image, so a synthetic
  stand-in of its shape ("FlanProxy", include/migmres.h: 3 dofs per node of a hexahedral
  node grid, 73 nnz per row, scrambled numbering; 1,574,640 rows / 115.2 M nnz at 81x81x80
  nodes vs Flan_1565's 1,564,794 / 114.2 M) through the general SELL-64 SpMM: small solves
  against the oracle (P = 1, 3) and, at full size, sampled rows bit for bit plus a cycle's
  properties.  Parity is against the oracle on the same generated rows; no reference run of
  Flan_1565 exists here ("parity unpinned" for this matrix).

Tolerances are test_gpu_solver.py's (1e-12 of ||r0|| per restart cycle).
"""

import numpy as np
import pytest

from tests.test_gpu_loopback import run_ranks
from tests.test_gpu_prec import _check, _oracle_case, _run_case, oracle_case_rerun

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
    if kind == "Laplace3D":
        return nx * ny * nz, (lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m))
    if kind == "Brick3D":
        return nx * ny * nz, (lambda f, m: oe.brick3d_rows(nx, ny, nz, f, m))
    assert kind == "FlanProxy"
    # the oracle's own restatement of the stand-in's specification (not the product generator)
    return 3 * nx * ny * nz, (lambda f, m: oe.flan_proxy_rows(nx, ny, nz, f, m))


def _params(k, nb, **kw):
    p = {"Block Size": k, "Num Blocks": nb, "Maximum Iterations": 600, "Maximum Restarts": 60,
         "Convergence Tolerance": 1e-9, "Orthogonalization": "ICGS"}
    p.update(kw)
    return p


# ----------------------------------------------------------------------------------------
# small problems against the oracle
# ----------------------------------------------------------------------------------------

SOLVES = [
    # kind, dims, k, params, prec side, sweeps, damping
    # config 3 (k = 16): converged after 10 restarts (ICGS) / 12 restarts (DGKS).  (Num Blocks 5
    # on the same problem ends in a loss-of-accuracy detection whose iteration count the
    # oracle itself changes, 89 -> 88, when only its summation order changes: not a parity case.)
    ("Laplace3D", (12, 12, 12), 16, _params(16, 6, **{"Convergence Tolerance": 1e-8}), None, 0, 0.0),
    ("Laplace3D", (11, 10, 9), 16, _params(16, 5, **{"Convergence Tolerance": 1e-8}, Orthogonalization="DGKS"),
     None, 0, 0.0),
    ("Brick3D", (10, 10, 10), 8, _params(8, 6), "right", 1, 1.0),              # config 5
    ("Brick3D", (12, 11, 10), 8, _params(8, 5), "right", 2, 0.8),
    ("Brick3D", (9, 10, 11), 8, _params(8, 4, **{"Flexible Gmres": True}), "right", 1, 1.0),
    ("FlanProxy", (9, 8, 7), 4, _params(4, 10), None, 0, 0.0),                 # config 4 shape
    ("FlanProxy", (11, 9, 8), 4, _params(4, 8), "right", 1, 1.0),
]
# Cases whose restarted histories move past 1e-12 under any change of summation order -- the
# oracle's own reversed-order rerun moves them too (tests/parity.py).  Measured on MI355X
# (profiles/r3_parity_margins.jsonl): case 1 (k = 16 DGKS, 12 restarts) 1.8e-12 vs oracle drift
# 1.9e-12; case 4 (flexible GMRES, Brick3D + Jacobi) 5.9e-11 vs drift 2.4e-11.  Every other
# case meets the strict 1e-12 bar.
RESTART_SENSITIVE = {1, 4}


@pytest.mark.parametrize("case", range(len(SOLVES)))
def test_config_solves_match_oracle(comm, case):
    kind, dims, k, params, side, sweeps, damping = SOLVES[case]
    n, gen = _gen(kind, dims)
    Aor, B, ref = _oracle_case(gen, n, 1, k, params, side, sweeps, damping)
    assert ref["converged"]
    res = _run_case(comm, n, kind, dims, k, params, side, sweeps, damping, B)
    _check(res, ref, Aor, B, res[4], oracle_case_rerun(gen, n, 1, k, params, side, sweeps, damping),
           drift_ok=case in RESTART_SENSITIVE)


@pytest.mark.parametrize("dims,nb,P,m16", [((20, 20, 20), 24, 1, "1"), ((18, 17, 16), 23, 2, "1"),
                                            ((20, 20, 20), 24, 1, "0")])
def test_k16_full_cycle_matches_oracle(comm, monkeypatch, dims, nb, P, m16):
    """Config 3's block size through a whole long cycle (tol 1e-15: never converges, so every
    block step runs): L = 16 .. 16 (nb - 1), which takes the fused update + projection through
    each of its k = 16 forms -- by default (MIGMRES_NT_M16=1) the 16x16x4 form k_nn_tn_m16 from
    L = 48 on (two workgroups per CU up to L = 256, one beyond) and the per-wave-rows form
    below; with MIGMRES_NT_M16=0 the earlier selection (MIGMRES_NW16=1): 32-row chunks (L = 64
    .. 128 and 272 .. 336), 16-row chunks in two 256-thread workgroups per CU (L = 160 .. 256;
    C1 in registers up to L = 208) and 512-thread 16-row workgroups (L = 352, 368) -- and the
    Gram-form findBasis at k = 16; counts and residual history against the oracle."""
    import trilinos_amd as ta
    monkeypatch.setenv("MIGMRES_NT_M16", m16)
    k = 16
    params = _params(k, nb, **{"Convergence Tolerance": 1e-15, "Maximum Iterations": nb, "Maximum Restarts": 0})
    n, gen = _gen("Laplace3D", dims)
    Aor, B, ref = _oracle_case(gen, n, P, k, params, None, 0, 0.0)
    assert not ref["converged"] and ref["iterations"] == nb
    rerun = oracle_case_rerun(gen, n, P, k, params, None, 0, 0.0)
    if P == 1:
        res = _run_case(comm, n, "Laplace3D", dims, k, params, None, 0, 0.0, B)
        _check(res, ref, Aor, B, res[4], rerun)
        return

    def rank_fn(c):
        first = ta.uniform_map(n, c.nranks, c.rank)[0]
        return first, _run_case(c, n, "Laplace3D", dims, k, params, None, 0, 0.0, B, first)

    out = run_ranks(P, rank_fn)
    X = np.zeros((n, k))
    for first, r in out:
        X[first:first + r[4].shape[0]] = r[4]
    for first, r in out:
        _check(r, ref, Aor, B, X, rerun)


@pytest.mark.parametrize("case,P", [(0, 2), (0, 4), (2, 2), (5, 3)])
def test_config_solves_distributed(case, P):
    import trilinos_amd as ta
    kind, dims, k, params, side, sweeps, damping = SOLVES[case]
    n, gen = _gen(kind, dims)
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


@pytest.mark.parametrize("dims,k,P", [((9, 8, 7), 4, 1), ((9, 8, 7), 4, 3), ((13, 7, 5), 7, 2),
                                      ((9, 8, 7), 2, 1), ((9, 8, 7), 3, 2), ((13, 11, 10), 12, 1)])
def test_flan_proxy_spmm_bit_exact(dims, k, P):
    """The general (SELL-64) kernel on the unstructured rows, P = 1 and with ghost columns,
    through the row-interleaved X copy (k <= 4: 2- and 4-wide rows, k = 3 padded; k = 12: an
    8-column chunk -- interleaved where the rows average >= 48 entries -- then a 4-column one)."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    n, gen = _gen("FlanProxy", dims)
    X, _ = oe.epetra_random_mv(3, n, k)
    Yref = oe.DistCrs(gen, n, P).apply(X)

    def rank_fn(c):
        first, nloc = ta.uniform_map(n, c.nranks, c.rank)
        A = ta.CrsMatrix.galeri(c, "FlanProxy", *dims)
        Xd = ta.MultiVector(c, n, k)
        Xd.upload(X[first:first + nloc])
        Yd = ta.MultiVector(c, n, k)
        A.apply(Xd, Yd)
        return first, Yd.download()

    if P == 1:
        import torch
        assert torch.cuda.is_available()
        res = [rank_fn(ta.Comm(device=0))]
    else:
        res = run_ranks(P, rank_fn)
    Y = np.zeros((n, k))
    for first, y in res:
        Y[first:first + y.shape[0]] = y
    assert np.array_equal(Y, Yref)


# ----------------------------------------------------------------------------------------
# full sizes: exact samples and size-independent properties
# ----------------------------------------------------------------------------------------


def _sampled_rows_exact(y, Xh, gen, starts, nloc):
    """Rows [first, first + nloc) of A X against the oracle's stored-order row sums (P = 1:
    columns sorted ascending within each row)."""
    from oracle import epetra as oe
    for first in starts:
        rp, gc, vv = gen(first, nloc)
        rid = np.repeat(np.arange(nloc), np.diff(rp))
        order = np.lexsort((gc, rid))
        gc, vv = gc[order], vv[order]
        cols, lc = np.unique(gc, return_inverse=True)
        ref = oe.csr_rowsum(rp, lc, vv, Xh[cols])
        assert np.array_equal(y[first:first + nloc], ref), first


def _cycle_properties(ta, comm, A, B, n, k, nb, M=None, flexible=False):
    """One restart cycle (tol 0): residuals never increase, the last implicit residual equals
    the explicit ||B - A X|| / ||B|| of the returned X, and a second solve is bit-identical."""
    params = {"Block Size": k, "Num Blocks": nb, "Maximum Iterations": nb, "Maximum Restarts": 0,
              "Convergence Tolerance": 0.0, "Orthogonalization": "ICGS"}
    if flexible:
        params["Flexible Gmres"] = True

    def solve():
        X = ta.MultiVector(comm, n, k)
        X.put_scalar(0.0)
        lp = ta.LinearProblem(A, X, B)
        if M is not None:
            lp.setRightPrec(M)
        assert lp.setProblem()
        sm = ta.BlockGmresSolMgr(lp, params)
        sm.solve()
        assert sm.getNumIters() == nb
        return sm, X

    sm, X = solve()
    hist = sm.residualHistory()
    assert hist.shape[1] == k
    assert np.all(np.diff(hist, axis=0) <= 1e-14)
    R = ta.MultiVector(comm, n, k)
    A.apply(X, R)
    Bh = B.download()
    r = Bh - R.download()
    del R
    expl = np.linalg.norm(r, axis=0) / np.linalg.norm(Bh, axis=0)
    del r, Bh
    assert np.all(expl < 0.95)
    np.testing.assert_allclose(hist[-1], expl, rtol=0, atol=1e-10)
    x1 = X.download()
    del X
    _, X2 = solve()
    assert np.array_equal(x1, X2.download())


def test_fullsize_k16_cycle(comm):
    """Config 3's per-GPU slice: 256^3 rows, k = 16 (basis 16.8 M x 416 doubles = 55.8 GB)."""
    import trilinos_amd as ta
    m, k = 256, 16
    n = m ** 3
    A = ta.CrsMatrix.galeri(comm, "Laplace3D", m, m, m)
    Xe = ta.MultiVector(comm, n, k)
    Xe.random(1)
    B = ta.MultiVector(comm, n, k)
    A.apply(Xe, B)
    del Xe
    _cycle_properties(ta, comm, A, B, n, k, 25)


def test_fullsize_brick384_jacobi_k8(comm):
    """Config 5 on one GPU: Brick3D 384^3 (1.52 G nnz), Jacobi right preconditioner, k = 8."""
    import trilinos_amd as ta
    m, k = 384, 8
    n = m ** 3
    A = ta.CrsMatrix.galeri(comm, "Brick3D", m, m, m)
    assert A.nnz_local == (3 * m - 2) ** 3  # 1,520,875,000
    rng = np.random.default_rng(5)
    Xh = rng.standard_normal((n, k))
    X = ta.MultiVector(comm, n, k)
    X.upload(Xh)
    Y = ta.MultiVector(comm, n, k)
    A.apply(X, Y)
    y = Y.download()
    _, gen = _gen("Brick3D", (m, m, m))
    _sampled_rows_exact(y, Xh, gen, (0, n // 2 - m * m // 2, n - 2 * m * m), 2 * m * m)
    del y
    M = ta.Relaxation(A)
    M.setParameters({"relaxation: sweeps": 1, "relaxation: damping factor": 1.0})
    M.compute()
    dinv = M.inverseDiagonal()
    assert np.all(dinv == 1.0 / 26.0)  # Brick3D keeps 26 on every diagonal
    M.apply(X, Y)
    y = Y.download()
    sl = slice(n // 3, n // 3 + 100000)
    assert np.array_equal(y[sl], (1.0 * dinv[sl, None]) * Xh[sl])
    del y, Xh, X, Y
    Xe = ta.MultiVector(comm, n, k)
    Xe.random(1)
    B = ta.MultiVector(comm, n, k)
    A.apply(Xe, B)
    del Xe
    _cycle_properties(ta, comm, A, B, n, k, 25, M=M)


def test_fullsize_flan_proxy_k4(comm):
    """Config 4's shape: FlanProxy 81 x 81 x 80 nodes (1,574,640 rows, 115.2 M nnz), k = 4."""
    import trilinos_amd as ta
    dims, k = (81, 81, 80), 4
    n, gen = _gen("FlanProxy", dims)
    A = ta.CrsMatrix.galeri(comm, "FlanProxy", *dims)
    assert n == 1574640 and 73.0 < A.nnz_local / n < 73.3
    rng = np.random.default_rng(9)
    Xh = rng.standard_normal((n, k))
    X = ta.MultiVector(comm, n, k)
    X.upload(Xh)
    Y = ta.MultiVector(comm, n, k)
    A.apply(X, Y)
    _sampled_rows_exact(Y.download(), Xh, gen, (0, n // 2, n - 60000), 60000)
    Xe = ta.MultiVector(comm, n, k)
    Xe.random(1)
    B = ta.MultiVector(comm, n, k)
    A.apply(Xe, B)
    _cycle_properties(ta, comm, A, B, n, k, 25)
