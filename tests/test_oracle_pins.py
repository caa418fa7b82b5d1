"""Pin the oracle (oracle/) to the reference before trusting it.

The reference cannot be built here under this task's rules (its build needs CMake-generated
config headers and an external BLAS), so the oracle is pinned by:
  * outputs of the real reference recorded in SURVEY.md section 6 (the example driver
    belos/epetra/example/BlockGmres/BlockGmresEpetraGaleriEx.cpp, --nx=64 --num-rhs=8
    --block-size=8 --ortho=ICGS --tol=1e-8 --max-subspace=50 --max-restarts=50):
    201 iterations, 268 Epetra_CrsMatrix::Multiply calls, 4 restarts, 61 explicit-residual
    checks (268 = 201 + 1 RHS product + 1 initial residual + 4 restarts + 61), true
    relative residuals 3.5e-10 .. 9.9e-9;
  * known-answer values that the reference's own unit tests hold (glibc rand(), MINSTD,
    Epetra_MultiVector closed-form Norm1/Dot/Norm2 from
    epetra/test/MultiVector/ExecuteTestProblems.cpp:227-272).
"""

import math

import numpy as np
import pytest

from oracle import belos as ob, epetra as oe


def test_glibc_rand_stream():
    # glibc rand() without srand(): the stream the reference's std::rand() calls draw from
    assert oe.glibc_rand(6) == [1804289383, 846930886, 1681692777, 1714636915, 1957747793, 424238335]


def test_minstd_stream():
    # Park-Miller minimal standard, seed 1 (Epetra_Util::RandomInt)
    v, s = oe.minstd_stream(1, 3)
    assert v.tolist() == [16807, 282475249, 1622650073] and s == 1622650073
    assert oe.minstd_next(1) == 16807
    # 10000th value of MINSTD from seed 1 is 1043618065 (Park & Miller 1988)
    v, _ = oe.minstd_stream(1, 10000)
    assert int(v[-1]) == 1043618065


def test_epetra_multivector_closed_forms():
    """ExecuteTestProblems.cpp:227-272: A[j][i] = i+1 (i < 9), A[j][9] = 10 + j."""
    L, nv = 10, 4
    A = np.zeros((L, nv))
    for j in range(nv):
        A[:L - 1, j] = np.arange(1, L)
        A[L - 1, j] = L + j
    dl = float(L)
    norm1 = (dl - 1) * dl / 2 + A[L - 1]
    dot = (dl - 1) * dl * (2 * (dl - 1) + 1) / 6 + A[L - 1] ** 2
    np.testing.assert_allclose(np.abs(A).sum(0), norm1, rtol=0, atol=1e-12)
    np.testing.assert_allclose(np.einsum("ij,ij->j", A, A), dot, rtol=0, atol=1e-12)
    np.testing.assert_allclose(np.linalg.norm(A, axis=0), np.sqrt(dot), rtol=1e-15)


def epetra_gemm_kat(case, n, nv, alpha, beta, transb="N", seed=3):
    """Epetra's GEMM known answers (epetra/test/MultiVector/BuildTestProblems.cpp:45-268, driven
    by ExecuteTestProblems.cpp:155-215): returns A, B, C0 and the closed-form result C_GEMM.
    case 2: A, B distributed (n x nv), C local (nv x nv): C = alpha A^T B + beta C0,
            A(i,j) = ((i+1)/n)(j+1), B(i,j) = 1/(((i+1)/n)(j+1)), C_GEMM(i,j) = alpha (i+1) n/(j+1) + beta C0
    case 3: A distributed (n x nv), B local (nv x nv, transposed when transb = "T"), C distributed:
            C = alpha A op(B) + beta C0, A(i,j) = ((i+1)/nv)(j+1), B(i,j) = 1/(((i+1)/nv)(j+1)),
            C_GEMM(i,j) = alpha (i+1) nv/(j+1) + beta C0."""
    rng = np.random.default_rng(seed)
    sf = float(n if case == 2 else nv)
    fi = np.arange(1, n + 1, dtype=float)[:, None]
    fj = np.arange(1, nv + 1, dtype=float)[None, :]
    A = (fi * (1.0 / sf)) * fj
    if case == 2:
        B = 1.0 / ((fi * (1.0 / sf)) * fj)
        C0 = rng.uniform(-1, 1, (nv, nv))
        gi = np.arange(1, nv + 1, dtype=float)[:, None] * sf
    else:
        bi = np.arange(1, nv + 1, dtype=float)[:, None]
        B = 1.0 / ((bi * (1.0 / sf)) * fj)
        if transb == "T":
            B = B.T.copy()  # op(B) = B^T must equal the case-3 B above
        C0 = rng.uniform(-1, 1, (n, nv))
        gi = fi * sf
    return A, B, C0, alpha * (gi / fj) + beta * C0


BAD_RESIDUAL = 5.0e-6  # ExecuteTestProblems.cpp:880-892 (per column 2-norm of C - C_GEMM)


@pytest.mark.parametrize("n", [10, 1000, 4099])
def test_epetra_gemm_known_answers_on_oracle(n):
    """The oracle's MvTransMv / MvTimesMatAddMv against Epetra's own GEMM known answers:
    case 2 (2-D dot product via GEMM, alpha 2, beta 1) and cases 6-7 (vector update via GEMM,
    alpha 2, beta 1.1, B and B^T), under the reference's BadResidual threshold and a 1e-13
    relative bar."""
    nv = 4
    A, B, C0, want = epetra_gemm_kat(2, n, nv, 2.0, 1.0)
    got = ob.mv_trans_mv(2.0, A, B, 1.0, C0)
    assert np.linalg.norm(got - want, axis=0).max() <= BAD_RESIDUAL
    np.testing.assert_allclose(got, want, rtol=1e-13)
    for tb in ("N", "T"):
        A, B, C0, want = epetra_gemm_kat(3, n, nv, 2.0, 1.1, tb)
        got = ob.mv_times_mat_add_mv(2.0, A, B if tb == "N" else B.T, 1.1, C0)
        assert np.linalg.norm(got - want, axis=0).max() <= BAD_RESIDUAL
        np.testing.assert_allclose(got, want, rtol=1e-13)


def test_epetra_localmap_closed_forms_on_oracle():
    """ExecuteTestProblems.cpp:227-272 on the oracle's own MvNorm / MvDot: A[j][i] = i+1
    (i < 9), A[j][9] = 10 + j; Norm1, Dot and Norm2 closed forms (exact in fp64 here)."""
    L, nv = 10, 4
    A = np.zeros((L, nv))
    for j in range(nv):
        A[:L - 1, j] = np.arange(1, L)
        A[L - 1, j] = L + j
    dl = float(L)
    norm1 = (dl - 1.0) * dl / 2.0 + A[L - 1]
    dot = (dl - 1.0) * dl * (2.0 * (dl - 1.0) + 1.0) / 6.0 + A[L - 1] * A[L - 1]
    assert np.array_equal(ob.mv_norm(A, "1"), norm1)
    assert np.array_equal(ob.mv_dot(A, A), dot)
    np.testing.assert_allclose(ob.mv_norm(A, "2"), np.sqrt(dot), rtol=1e-15)
    assert np.abs(ob.mv_norm(A, "2") - np.sqrt(dot)).max() <= BAD_RESIDUAL
    assert np.array_equal(ob.mv_norm(A, "inf"), A[L - 1])


def test_galeri_laplace3d_structure():
    """nnz = 7 m^3 - 6 m^2 (SURVEY.md 8 sizes table); rows sorted by local column."""
    m = 6
    rp, gc, vv = oe.laplace3d_rows(m, m, m, 0, m ** 3)
    assert rp[-1] == 7 * m ** 3 - 6 * m ** 2
    D = oe.DistCrs(lambda f, c: oe.laplace3d_rows(m, m, m, f, c), m ** 3, 1)
    rp, lc, lv = D.crs[0]
    r = 2 * m * m + m + 2  # an interior row: below, lower, left, diag, right, upper, above
    assert lc[rp[r]:rp[r + 1]].tolist() == [r - m * m, r - m, r - 1, r, r + 1, r + m, r + m * m]
    assert lv[rp[r]:rp[r + 1]].tolist() == [-1.0, -1.0, -1.0, 6.0, -1.0, -1.0, -1.0]


def test_reference_run_64cube_icgs():
    """The recorded reference run reproduced by the oracle."""
    m, k = 64, 8
    n = m ** 3
    # Xexact is the 3rd Epetra_MultiVector of the driver (B, X, Xexact), each consuming two
    # rand() calls (Epetra_Util ctor + AllocateForCopy, Epetra_MultiVector.cpp:263-265)
    seed = oe.glibc_rand(6)[5]
    A = oe.DistCrs(lambda f, c: oe.laplace3d_rows(m, m, m, f, c), n, 1)
    Xex, _ = oe.epetra_random_mv(seed, n, k)
    B = A.apply(Xex)
    res = ob.solve(A.apply, B, {"Num Blocks": 50, "Block Size": 8, "Maximum Iterations": n // 8 - 1,
                                "Maximum Restarts": 50, "Convergence Tolerance": 1e-8,
                                "Orthogonalization": "ICGS"})
    assert res["converged"]
    assert res["iterations"] == 201
    assert res["n_apply"] + 1 == 268
    assert res["restarts"] == 4
    assert res["n_explicit"] == 61
    rel = np.linalg.norm(B - A.apply(res["X"]), axis=0) / np.linalg.norm(B, axis=0)
    assert f"{rel.min():.1e}" == "3.5e-10" and f"{rel.max():.1e}" == "9.9e-09"


def orsirr1_problem():
    """test_bl_gmres_hb.cpp's problem: orsirr1.hb, xexact = rand()/RAND_MAX, b = A xexact by
    the CSC product (Trilinos_Util_read_hb.cpp:141-158).  From the committed fixture."""
    import os
    f = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "orsirr1.npz"))
    n = int(f["n"])
    gen, b, xexact = oe.hb_problem(f["colptr"], f["rowind"], f["vals"], bool(f["symmetric"]))
    return n, gen, b, xexact


def test_reference_run_orsirr1_dgks():
    """`test_bl_gmres_hb` (BlockGmres, k = 1, default DGKS, tol 1e-5,
    Num Blocks = Max Iters = n - 1, 15 restarts) on orsirr1.hb: 209 iterations, actual
    relative residual printed as 9.94786e-06."""
    n, gen, b, _ = orsirr1_problem()
    A = oe.DistCrs(gen, n, 1)
    res = ob.solve(A.apply, b[:, None], {"Num Blocks": n - 1, "Block Size": 1, "Maximum Iterations": n - 1,
                                          "Maximum Restarts": 15, "Convergence Tolerance": 1e-5,
                                          "Orthogonalization": "DGKS"})
    assert res["converged"] and res["iterations"] == 209
    rel = np.linalg.norm(b - A.apply(res["X"])[:, 0]) / np.linalg.norm(b)
    assert f"{rel:g}" == "9.94786e-06"


# ---------------------------------------------------------------------------------------
# reference unit-test known answers (tests/known_answers.py)
# ---------------------------------------------------------------------------------------


@pytest.mark.parametrize("P", [1, 2, 3])
def test_ifpack2_relaxation_jacobi_known_answers(P):
    """Ifpack2_UnitTestRelaxation.cpp Test0 / Test1 on the oracle's Jacobi: applyMat(x = 1)
    = 2, apply(x = 1) = 0.5, apply(x, x) = 0.5 (5 rows per process, 2 columns)."""
    from oracle import ifpack2 as oi
    from tests.known_answers import ifpack2_test_matrix_rows
    n = 5 * P
    gen = ifpack2_test_matrix_rows(n)
    A = oe.DistCrs(gen, n, P)
    rp, gc, vv = gen(0, n)
    M = oi.Jacobi(A.apply, oi.crs_diagonal(rp, gc, vv, 0, n))
    x = np.ones((n, 2))
    assert np.array_equal(A.apply(x), np.full((n, 2), 2.0))
    assert np.array_equal(M(x), np.full((n, 2), 0.5))
    x = M(x)  # apply(x, x): the result replaces x
    assert np.array_equal(x, np.full((n, 2), 0.5))


def _power(gen, n, trans, seed=7):
    from tests.known_answers import NumpyOps, power_method, transpose_apply
    A = oe.DistCrs(gen, n, 1)
    rp, lc, lv = A.crs[0]
    apply = (lambda q: transpose_apply(rp, lc, lv, q, n)) if trans else A.apply
    z, _ = oe.epetra_random_mv(seed, n, 1)
    return power_method(NumpyOps(apply), z, np.zeros((n, 1)), np.zeros((n, 1)))


def test_epetra_crsmatrix_power_method_known_answers():
    """epetra/test/CrsMatrix/cxx_main.cpp:124-317: the (-1, 2, -1) tridiagonal on 10001 rows
    has 3 n - 2 entries and 2 per end row / 3 per inner row after FillComplete; the power
    method succeeds (residual < 0.1 within 200 iterations) for A and A^T, with lambda near
    the largest eigenvalue 2 - 2 cos(pi n / (n + 1)); and again after A[0,0] x 10, where the
    dominant eigenvalue separates (~20)."""
    from tests.known_answers import epetra_crs_test_size, epetra_tridiag_rows
    n = epetra_crs_test_size(1)
    assert n == 10001
    gen = epetra_tridiag_rows(n)
    rp, gc, vv = gen(0, n)
    assert rp[-1] == 3 * n - 2
    counts = np.diff(rp)
    assert counts[0] == counts[-1] == 2 and np.all(counts[1:-1] == 3)
    lam_max = 2.0 - 2.0 * math.cos(math.pi * n / (n + 1))
    for trans in (False, True):
        ierr, lam, lambdas, res = _power(gen, n, trans)
        assert ierr == 0, res
        assert 0.99 * lam_max < lam <= lam_max + 1e-12
    # symmetric A: the transposed product differs only in summation order
    _, _, l_n, _ = _power(gen, n, False)
    _, _, l_t, _ = _power(gen, n, True)
    np.testing.assert_allclose(l_n, l_t, rtol=1e-13)
    gen10 = epetra_tridiag_rows(n, diag0=20.0)
    for trans in (False, True):
        ierr, lam, lambdas, res = _power(gen10, n, trans)
        assert ierr == 0 and abs(lam - 20.0) < 0.2, (ierr, lam, res)
    # P > 1 row counts: 10000 P + min(P, 3) global rows, the first three processes one more
    for P in (2, 3, 4, 5):
        n = epetra_crs_test_size(P)
        sizes = [oe.uniform_map(n, P, p)[1] for p in range(P)]
        assert sizes == [10001 if p < 3 else 10000 for p in range(P)]


def _diag_gen(d):
    d = np.asarray(d, dtype=np.float64)

    def gen(first, m):
        return np.arange(m + 1, dtype=np.int64), np.arange(first, first + m, dtype=np.int64), d[first:first + m].copy()
    return gen


def test_belos_gmres_diag_known_answers():
    """belos/epetra/test/BlockGmres/test_bl_gmres_diag.cpp on the oracle's BlockGmresSolMgr
    (default orthogonalization DGKS): inv(diag(1..10)) 1 = [1, 1/2, ..., 1/10];
    inv(4 I) 1 = 1/4; the nested inv(inv(4 I) (4 I)) 1 = 1 with ||y - 1|| < 1e-10 -- the
    inner solve as the outer solve's operator."""
    from tests.known_answers import DIAG_TEST_PARAMS
    n = 10
    x = np.ones((n, 1))
    D2 = oe.DistCrs(_diag_gen(np.arange(1, n + 1)), n, 1)
    r = ob.solve(D2.apply, x, DIAG_TEST_PARAMS)
    assert r["converged"]
    np.testing.assert_allclose(r["X"][:, 0], 1.0 / np.arange(1, n + 1), rtol=0, atol=1e-10)
    D = oe.DistCrs(_diag_gen(np.full(n, 4.0)), n, 1)

    def inner(b):
        return ob.solve(D.apply, b, DIAG_TEST_PARAMS)["X"]
    y = inner(x)
    np.testing.assert_allclose(y, 0.25, rtol=0, atol=1e-10)

    def composed(v):  # Composed_Operator(Inner, B): Inner(B v), B = 4 I
        return inner(4.0 * v)
    r = ob.solve(composed, x, DIAG_TEST_PARAMS)
    assert np.linalg.norm(r["X"] - 1.0) < 1e-10
