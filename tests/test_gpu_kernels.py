"""GPU parity of the individual hot-path kernels against the oracle / fp64 numpy.

SpMM is compared bit for bit (integer index work + stored-order sums).  The MVT
reductions (MFMA inner products, dots, norms) change only the summation order, so they
are compared against fp64 numpy with a relative tolerance of 1e-13 on well-scaled data.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-13


@pytest.fixture(scope="module")
def comm():
    import torch
    assert torch.cuda.is_available()
    import trilinos_amd as ta
    return ta.Comm(device=0)


def _upload(ta, comm, arr):
    n, k = arr.shape
    mv = ta.MultiVector(comm, n, k)
    mv.upload(arr)
    return mv


@pytest.mark.parametrize("kind,dims,k", [("Laplace2D", (100, 100, 1), 1), ("Laplace2D", (37, 23, 1), 3),
                                         ("Laplace3D", (16, 16, 16), 8), ("Laplace3D", (9, 7, 5), 16),
                                         ("Laplace3D", (12, 12, 12), 17)])
def test_spmm_bit_exact(comm, kind, dims, k):
    import trilinos_amd as ta
    from oracle import epetra as oe
    nx, ny, nz = dims
    n = nx * ny * (nz if kind == "Laplace3D" else 1)
    gen = (lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m)) if kind == "Laplace3D" else \
        (lambda f, m: oe.laplace2d_rows(nx, ny, f, m))
    Aor = oe.DistCrs(gen, n, 1)
    X, _ = oe.epetra_random_mv(7, n, k)
    A = ta.CrsMatrix.galeri(comm, kind, nx, ny, nz)
    Xd = _upload(ta, comm, X)
    Yd = ta.MultiVector(comm, n, k)
    A.apply(Xd, Yd)
    assert np.array_equal(Yd.download(), Aor.apply(X))
    # alpha/beta form (Tpetra apply): Y = 2 A X - 0.5 Y
    Y0 = np.random.default_rng(1).standard_normal((n, k))
    Yd.upload(Y0)
    A.apply(Xd, Yd, 2.0, -0.5)
    np.testing.assert_allclose(Yd.download(), 2.0 * Aor.apply(X) - 0.5 * Y0, rtol=1e-15, atol=1e-14)


@pytest.mark.parametrize("per_row,k,pairs", [(4, 8, "default"), (5, 3, "default"), (12, 8, "default"),
                                              (7, 8, "off"), (30, 5, "default"), (75, 4, "default"),
                                              (9, 8, "csr"), (0, 2, "default")])
def test_spmm_unstructured_bit_exact(comm, per_row, k, pairs, monkeypatch):
    """Unstructured rows through all three SpMM kernels: the row-pair kernel (rows of <= 8
    entries whose pairs need <= 12 keys), the SELL-64 row kernel (longer rows, or the pair
    plan switched off with MIGMRES_NO_PAIR_SPMM=1) and the plain CSR row kernel
    (MIGMRES_NO_SELL_SPMM=1).  per_row 0: random row lengths 0..40 (empty rows included)."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    from tests.test_plans import random_rows
    if pairs in ("off", "csr"):
        monkeypatch.setenv("MIGMRES_NO_PAIR_SPMM", "1")
    if pairs == "csr":
        monkeypatch.setenv("MIGMRES_NO_SELL_SPMM", "1")
    n = 3001
    rp, gc, vv = random_rows(n, 0, n, 29, per_row=per_row)
    A = ta.CrsMatrix(comm, n, rp, gc, vv)
    Aor = oe.DistCrs(lambda f, m: random_rows(n, f, m, 29, per_row=per_row), n, 1)
    X, _ = oe.epetra_random_mv(11, n, k)
    Xd = _upload(ta, comm, X)
    Yd = ta.MultiVector(comm, n, k)
    A.apply(Xd, Yd)
    assert np.array_equal(Yd.download(), Aor.apply(X))


def banded_rows(n_global, first, nloc, seed, per_row=20, band=150):
    """Long rows with locality: per_row random columns within +-band of the row, insertion
    order random, plus the diagonal."""
    rng = np.random.default_rng(seed + first)
    rows, cols, vals = [0], [], []
    for r in range(nloc):
        g = first + r
        lo, hi = max(0, g - band), min(n_global, g + band + 1)
        c = rng.choice(np.arange(lo, hi), size=min(per_row, hi - lo), replace=False)
        c = np.concatenate([c[c != g], [g]])
        cols.extend(c.tolist())
        vals.extend(rng.standard_normal(len(c)).tolist())
        rows.append(len(cols))
    return np.array(rows), np.array(cols), np.array(vals)


@pytest.mark.parametrize("kind,k,tpl", [("banded", 8, True), ("banded", 5, True), ("banded", 1, True),
                                        ("banded", 16, True), ("Brick3D", 8, True), ("Brick3D", 3, True),
                                        ("Brick3D", 16, True), ("Laplace3D", 8, True), ("Laplace3D", 5, True),
                                        ("Brick3D", 8, False), ("Laplace3D", 8, False)])
def test_spmm_kernel_choice_bit_exact(comm, kind, k, tpl, monkeypatch):
    """Which SpMM kernel an operator gets (migmres_crs_spmm_kernel): the row-pair template
    kernel for stencils (7-point and 27-point: one byte per row pair), otherwise -- or with
    MIGMRES_NO_TPL_SPMM=1 -- the row-pair kernel for 7-point rows, the SELL-64 row kernel for
    27-point Brick3D rows (config 5) and long banded random rows; bit for bit against the
    oracle either way."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    if not tpl:
        monkeypatch.setenv("MIGMRES_NO_TPL_SPMM", "1")
    if kind == "banded":
        n = 4099
        gen = lambda f, m: banded_rows(n, f, m, 31)
        rp, gc, vv = gen(0, n)
        A = ta.CrsMatrix(comm, n, rp, gc, vv)
    else:
        nx, ny, nz = 13, 12, 11
        n = nx * ny * nz
        gen = (lambda f, m: oe.brick3d_rows(nx, ny, nz, f, m)) if kind == "Brick3D" else \
            (lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m))
        A = ta.CrsMatrix.galeri(comm, kind, nx, ny, nz)
    if tpl and kind != "banded":
        assert A.spmm_kernel() == "tpl"
    else:
        assert A.spmm_kernel() == ("pair" if kind == "Laplace3D" else "sell")
    Aor = oe.DistCrs(gen, n, 1)
    X, _ = oe.epetra_random_mv(13, n, k)
    Xd = _upload(ta, comm, X)
    Yd = ta.MultiVector(comm, n, k)
    A.apply(Xd, Yd)
    assert np.array_equal(Yd.download(), Aor.apply(X))


@pytest.mark.parametrize("n,L,kb", [(1, 1, 1), (63, 5, 3), (64, 16, 16), (1000, 37, 8), (5000, 104, 8),
                                    (4097, 208, 8), (3001, 300, 16), (2049, 600, 20)])
def test_trans_mv_mfma(comm, n, L, kb):
    import trilinos_amd as ta
    rng = np.random.default_rng(n + L)
    A = rng.standard_normal((n, L))
    B = rng.standard_normal((n, kb))
    Ad, Bd = _upload(ta, comm, A), _upload(ta, comm, B)
    C = ta.MultiVecTraits.MvTransMv(-0.5, Ad, Bd)
    ref = -0.5 * (A.T @ B)
    np.testing.assert_allclose(C, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())


def test_trans_mv_views(comm):
    """Non-contiguous column views (CloneView with an index vector)."""
    import trilinos_amd as ta
    rng = np.random.default_rng(3)
    n = 777
    A = rng.standard_normal((n, 12))
    Ad = _upload(ta, comm, A)
    idx = [11, 0, 5, 3, 7]
    V = Ad.view(idx)
    W = Ad.view([2, 9])
    C = ta.MultiVecTraits.MvTransMv(1.0, V, W)
    np.testing.assert_allclose(C, A[:, idx].T @ A[:, [2, 9]], rtol=1e-12, atol=1e-12)
    assert not V.constant_stride and Ad.view_range(2, 3).constant_stride


@pytest.mark.parametrize("n,L,k", [(1, 1, 1), (100, 9, 3), (5000, 104, 8), (4099, 208, 16), (700, 70, 33)])
def test_times_mat_add_mv(comm, n, L, k):
    import trilinos_amd as ta
    rng = np.random.default_rng(n * 7 + L)
    A = rng.standard_normal((n, L))
    M = rng.standard_normal((L, k))
    X = rng.standard_normal((n, k))
    Ad, Xd = _upload(ta, comm, A), _upload(ta, comm, X)
    ta.MultiVecTraits.MvTimesMatAddMv(-1.0, Ad, M, 1.0, Xd)
    np.testing.assert_allclose(Xd.download(), X - A @ M, rtol=1e-12, atol=1e-12 * np.abs(A @ M).max())
    ta.MultiVecTraits.MvTimesMatAddMv(2.0, Ad, M, 0.0, Xd)
    np.testing.assert_allclose(Xd.download(), 2.0 * (A @ M), rtol=1e-12, atol=1e-11)


def test_blas1(comm):
    import trilinos_amd as ta
    MVT = ta.MultiVecTraits
    rng = np.random.default_rng(5)
    n, k = 12345, 6
    A = rng.standard_normal((n, k))
    B = rng.standard_normal((n, k))
    Ad, Bd = _upload(ta, comm, A), _upload(ta, comm, B)
    np.testing.assert_allclose(MVT.MvDot(Ad, Bd), np.einsum("ij,ij->j", A, B), rtol=RTOL * 100)
    np.testing.assert_allclose(MVT.MvNorm(Ad), np.linalg.norm(A, axis=0), rtol=RTOL)
    np.testing.assert_allclose(MVT.MvNorm(Ad, ta.OneNorm), np.abs(A).sum(0), rtol=RTOL)
    np.testing.assert_array_equal(MVT.MvNorm(Ad, ta.InfNorm), np.abs(A).max(0))
    Y = MVT.Clone(Ad, k)
    MVT.MvAddMv(0.5, Ad, -2.0, Bd, Y)
    np.testing.assert_array_equal(Y.download(), 0.5 * A + -2.0 * B)
    MVT.MvScale(Y, 3.0)
    np.testing.assert_array_equal(Y.download(), 3.0 * (0.5 * A + -2.0 * B))
    s = np.arange(1, k + 1, dtype=float)
    MVT.MvScale(Ad, s)
    np.testing.assert_array_equal(Ad.download(), A * s)
    MVT.MvInit(Y, 1.25)
    assert np.all(Y.download() == 1.25)
    C = MVT.CloneCopy(Bd, [4, 1])
    np.testing.assert_array_equal(C.download(), B[:, [4, 1]])
    MVT.SetBlock(C, [0, 5], Y)
    got = Y.download()
    np.testing.assert_array_equal(got[:, [0, 5]], B[:, [4, 1]])
    assert np.all(got[:, 1:5] == 1.25)
    # Epetra_MultiVector::Random semantics (column-major MINSTD stream, Epetra_Util.cpp:71-99)
    from oracle import epetra as oe
    R = MVT.Clone(Ad, 3)
    seed = R.random(1)
    ref, s_ref = oe.epetra_random_mv(1, n, 3)
    np.testing.assert_array_equal(R.download(), ref)
    assert seed == s_ref


def test_icgs_project_normalize(comm):
    """ICGSOrthoManager::projectAndNormalize against the oracle on a Krylov-like block."""
    import trilinos_amd as ta
    from oracle import belos as ob
    rng = np.random.default_rng(11)
    n, L, k = 3000, 24, 8
    Q, _ = np.linalg.qr(rng.standard_normal((n, L)))
    X = rng.standard_normal((n, k)) + Q @ rng.standard_normal((L, k))
    Qd, Xd = _upload(ta, comm, Q), _upload(ta, comm, X)
    rank, C, B = ta.ICGSOrthoManager().projectAndNormalize(Xd, Qd)
    Xo = X.copy()
    Co, Bo = np.zeros((L, k)), np.zeros((k, k))
    r_or = ob.ICGS().project_and_normalize(Xo, Q, Co, Bo)
    assert rank == r_or == k
    np.testing.assert_allclose(C, Co, rtol=1e-11, atol=1e-12)
    np.testing.assert_allclose(B, Bo, rtol=1e-11, atol=1e-12)
    np.testing.assert_allclose(Xd.download(), Xo, rtol=1e-10, atol=1e-12)
    Xn = Xd.download()
    np.testing.assert_allclose(Xn.T @ Xn, np.eye(k), atol=1e-13)
    np.testing.assert_allclose(Q.T @ Xn, 0, atol=1e-13)


@pytest.mark.parametrize("k,near_dep", [(8, False), (1, False), (1, True), (4, True)])
def test_dgks_project_normalize(comm, k, near_dep):
    """DGKSOrthoManager::projectAndNormalize against the oracle.  near_dep makes X lie mostly
    in span(Q), so the DGKS re-orthogonalisation criterion fires (and for k = 1 the second
    blkOrtho1 pass runs)."""
    import trilinos_amd as ta
    from oracle.dgks import DGKS
    rng = np.random.default_rng(17 + k)
    n, L = 3000, 24
    Q, _ = np.linalg.qr(rng.standard_normal((n, L)))
    X = Q @ rng.standard_normal((L, k)) + (1e-3 if near_dep else 1.0) * rng.standard_normal((n, k))
    Qd, Xd = _upload(ta, comm, Q), _upload(ta, comm, X)
    rank, C, B = ta.DGKSOrthoManager().projectAndNormalize(Xd, Qd)
    Xo = X.copy()
    Co, Bo = np.zeros((L, k)), np.zeros((k, k))
    r_or = DGKS().project_and_normalize(Xo, Q, Co, Bo)
    assert rank == r_or == k
    np.testing.assert_allclose(C, Co, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(B, Bo, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(Xd.download(), Xo, rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("n", [10, 4099, 100003])
def test_epetra_gemm_known_answers(comm, n):
    """Epetra's own MultiVector GEMM known answers (BuildTestProblems.cpp:45-268 via
    ExecuteTestProblems.cpp:155-215) through the C ABI: MvTransMv (case 2, alpha 2, beta 1 on
    the host side as Belos applies it) and MvTimesMatAddMv (cases 6-7, alpha 2, beta 1.1),
    under the reference's BadResidual threshold and a 1e-13 relative bar; plus the LocalMap
    Norm1 / Dot / Norm2 closed forms (ExecuteTestProblems.cpp:227-272)."""
    import trilinos_amd as ta
    from tests.test_oracle_pins import epetra_gemm_kat, BAD_RESIDUAL
    MVT = ta.MultiVecTraits
    nv = 4
    A, B, C0, want = epetra_gemm_kat(2, n, nv, 2.0, 1.0)
    got = MVT.MvTransMv(2.0, _upload(ta, comm, A), _upload(ta, comm, B)) + 1.0 * C0
    assert np.linalg.norm(got - want, axis=0).max() <= BAD_RESIDUAL
    np.testing.assert_allclose(got, want, rtol=1e-13)
    A, B, C0, want = epetra_gemm_kat(3, n, nv, 2.0, 1.1)
    Cd = _upload(ta, comm, C0)
    MVT.MvTimesMatAddMv(2.0, _upload(ta, comm, A), B, 1.1, Cd)
    got = Cd.download()
    assert np.linalg.norm(got - want, axis=0).max() <= BAD_RESIDUAL
    np.testing.assert_allclose(got, want, rtol=1e-13)
    L = 10
    A = np.zeros((L, nv))
    for j in range(nv):
        A[:L - 1, j] = np.arange(1, L)
        A[L - 1, j] = L + j
    dl = float(L)
    norm1 = (dl - 1.0) * dl / 2.0 + A[L - 1]
    dot = (dl - 1.0) * dl * (2.0 * (dl - 1.0) + 1.0) / 6.0 + A[L - 1] * A[L - 1]
    Ad = _upload(ta, comm, A)
    assert np.array_equal(MVT.MvNorm(Ad, ta.OneNorm), norm1)
    assert np.array_equal(MVT.MvDot(Ad, Ad), dot)
    np.testing.assert_allclose(MVT.MvNorm(Ad), np.sqrt(dot), rtol=1e-15)


@pytest.mark.parametrize("dims,k", [((12, 11, 10), 8), ((16, 9, 7), 1), ((10, 10, 10), 3), ((14, 8, 6), 5),
                                    ((20, 6, 5), 16), ((8, 7, 9), 9), ((6, 5, 4), 2)])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (-1.0, 1.0), (0.5, -2.0)])
def test_spmm_tpl3_lane_shared_bit_exact(comm, dims, k, alpha, beta, monkeypatch):
    """27-point Brick3D on even-nx grids takes the lane-shared stencil-group kernel when the
    plane march is off (one X load per x-neighbour triple, the neighbours' halves by DPP wave
    shifts; waves of 62 outputs, so several waves and boundary pairs sit in every case): bit
    for bit against the oracle for every column count (chunks of 8, odd remainders), and
    Y = alpha A X + beta Y."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    monkeypatch.setenv("MIGMRES_NO_MARCH", "1")
    nx, ny, nz = dims
    n = nx * ny * nz
    A = ta.CrsMatrix.galeri(comm, "Brick3D", nx, ny, nz)
    assert A.spmm_kernel() == "tpl3"
    Aor = oe.DistCrs(lambda f, m: oe.brick3d_rows(nx, ny, nz, f, m), n, 1)
    X, _ = oe.epetra_random_mv(17, n, k)
    Y0, _ = oe.epetra_random_mv(19, n, k)
    Xd = _upload(ta, comm, X)
    Yd = _upload(ta, comm, Y0)
    A.apply(Xd, Yd, alpha, beta)
    want = alpha * Aor.apply(X) if beta == 0.0 else alpha * Aor.apply(X) + beta * Y0
    assert np.array_equal(Yd.download(), want)


def test_spmm_tpl3_odd_nx_falls_back(comm, monkeypatch):
    """An odd nx puts row pairs across grid lines: no x-neighbour triples, so the operator
    keeps the plain template kernel (still bit-exact, test_spmm_kernel_choice_bit_exact); so
    does the 7-point operator on an even grid when the plane march is off."""
    import trilinos_amd as ta
    assert ta.CrsMatrix.galeri(comm, "Brick3D", 13, 12, 11).spmm_kernel() == "tpl"
    assert ta.CrsMatrix.galeri(comm, "Laplace3D", 13, 12, 12).spmm_kernel() == "tpl"
    monkeypatch.setenv("MIGMRES_NO_MARCH", "1")
    assert ta.CrsMatrix.galeri(comm, "Laplace3D", 12, 12, 12).spmm_kernel() == "tpl"


@pytest.mark.parametrize("dims,k", [((12, 11, 10), 8), ((16, 9, 7), 3), ((8, 7, 9), 9)])
def test_spmm_tpl3_seven_point_bit_exact(comm, dims, k, monkeypatch):
    """The 7-point operator in stencil-group form (MIGMRES_TPL3_SHORT=1: five groups, the x
    triple plus four single y/z keys): bit for bit against the oracle."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    monkeypatch.setenv("MIGMRES_TPL3_SHORT", "1")
    monkeypatch.setenv("MIGMRES_NO_MARCH", "1")
    nx, ny, nz = dims
    n = nx * ny * nz
    A = ta.CrsMatrix.galeri(comm, "Laplace3D", nx, ny, nz)
    assert A.spmm_kernel() == "tpl3"
    Aor = oe.DistCrs(lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m), n, 1)
    X, _ = oe.epetra_random_mv(23, n, k)
    Yd = ta.MultiVector(comm, n, k)
    A.apply(_upload(ta, comm, X), Yd)
    assert np.array_equal(Yd.download(), Aor.apply(X))


@pytest.mark.parametrize("dims,k", [((9, 8, 7), 4), ((11, 9, 8), 1), ((9, 7, 10), 3), ((7, 8, 6), 8), ((9, 6, 5), 9),
                                    ((5, 4, 3), 2)])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (-1.0, 1.0)])
def test_spmm_bsr3_bit_exact(comm, dims, k, alpha, beta):
    """FlanProxy (3 dofs per node, configs[3]'s shape) is detected as 3 x 3 block rows
    (migmres_crs_spmm_kernel "bsr3"): bit for bit against the oracle's rows for every column
    count, and Y = alpha A X + beta Y."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    nx, ny, nz = dims
    n = 3 * nx * ny * nz
    A = ta.CrsMatrix.galeri(comm, "FlanProxy", nx, ny, nz)
    assert A.spmm_kernel() == "bsr3"
    Aor = oe.DistCrs(lambda f, m: oe.flan_proxy_rows(nx, ny, nz, f, m), n, 1)
    X, _ = oe.epetra_random_mv(29, n, k)
    Y0, _ = oe.epetra_random_mv(31, n, k)
    Yd = _upload(ta, comm, Y0)
    A.apply(_upload(ta, comm, X), Yd, alpha, beta)
    want = alpha * Aor.apply(X) if beta == 0.0 else alpha * Aor.apply(X) + beta * Y0
    assert np.array_equal(Yd.download(), want)


def test_spmm_bsr3_detects_not_assumes(comm):
    """Block rows are detected from the CRS: rows whose triple breaks the structure (an entry
    dropped from one row, a row count not divisible by 3) go to the row kernel, the rest stay
    blocked -- bit for bit either way; too few qualifying rows and the format is not used."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    nx, ny, nz, k = 9, 8, 7, 4
    n = 3 * nx * ny * nz - 2                     # last node's triple incomplete
    rp, gc, vv = oe.flan_proxy_rows(nx, ny, nz, 0, n)
    keep = np.ones(len(gc), bool)
    for r in (5, 301, 302, 700):                 # drop each row's 4th entry
        keep[rp[r] + 3] = False
    cnt = np.diff(rp) - np.isin(np.arange(n), [5, 301, 302, 700])
    rp2 = np.concatenate([[0], np.cumsum(cnt)])
    gc2, vv2 = gc[keep], vv[keep]
    gc2 = np.where(gc2 < n, gc2, gc2 % n)        # columns of the cut node fold back in range
    # rows must not repeat a column: rebuild each row unique in insertion order
    rows = [(gc2[rp2[i]:rp2[i + 1]], vv2[rp2[i]:rp2[i + 1]]) for i in range(n)]
    rp3, gc3, vv3 = [0], [], []
    for c, v in rows:
        _, first = np.unique(c, return_index=True)
        first = np.sort(first)
        gc3.extend(c[first].tolist())
        vv3.extend(v[first].tolist())
        rp3.append(len(gc3))
    rp3, gc3, vv3 = np.array(rp3), np.array(gc3), np.array(vv3)
    A = ta.CrsMatrix(comm, n, rp3, gc3, vv3)
    assert A.spmm_kernel() == "bsr3"
    Aor = oe.DistCrs(lambda f, m: (rp3[f:f + m + 1] - rp3[f], gc3[rp3[f]:rp3[f + m]], vv3[rp3[f]:rp3[f + m]]), n, 1)
    X, _ = oe.epetra_random_mv(37, n, k)
    Yd = ta.MultiVector(comm, n, k)
    A.apply(_upload(ta, comm, X), Yd)
    assert np.array_equal(Yd.download(), Aor.apply(X))


@pytest.mark.parametrize("kind,dims,k", [("Laplace3D", (12, 11, 10), 8), ("Laplace3D", (16, 9, 7), 1),
                                         ("Laplace3D", (130, 6, 5), 3), ("Laplace3D", (8, 7, 9), 9),
                                         ("Laplace3D", (6, 3, 3), 2), ("Brick3D", (12, 11, 10), 8),
                                         ("Brick3D", (20, 6, 5), 16), ("Brick3D", (134, 5, 4), 5),
                                         ("Brick3D", (6, 5, 4), 2), ("Brick3D", (10, 10, 10), 3)])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (-1.0, 1.0), (0.5, -2.0)])
@pytest.mark.parametrize("generic", [False, True])
def test_spmm_march_bit_exact(comm, kind, dims, k, alpha, beta, generic, monkeypatch):
    """The 2.5-D plane march (plane tiles of 64 pairs x 4 lines staged in LDS; partial x tiles
    at nx = 130 / 134, partial line tiles, a few planes, odd column counts): by default the
    7-point specialisation for Laplace3D and the uniform 27-point one for Brick3D, with
    MIGMRES_MARCH_GENERIC=1 the general form for both -- bit for bit against the oracle, and
    Y = alpha A X + beta Y."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    if generic:
        monkeypatch.setenv("MIGMRES_MARCH_GENERIC", "1")
    nx, ny, nz = dims
    n = nx * ny * nz
    A = ta.CrsMatrix.galeri(comm, kind, nx, ny, nz)
    assert A.spmm_kernel() == "march"
    gen = (lambda f, m: oe.brick3d_rows(nx, ny, nz, f, m)) if kind == "Brick3D" else \
        (lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m))
    Aor = oe.DistCrs(gen, n, 1)
    X, _ = oe.epetra_random_mv(29, n, k)
    Y0, _ = oe.epetra_random_mv(31, n, k)
    Yd = _upload(ta, comm, Y0)
    A.apply(_upload(ta, comm, X), Yd, alpha, beta)
    want = alpha * Aor.apply(X) if beta == 0.0 else alpha * Aor.apply(X) + beta * Y0
    assert np.array_equal(Yd.download(), want)


@pytest.mark.parametrize("kind,generic,kc,sz,pd,nl", [("Laplace3D", False, "1", "1", "1", "1"),
                                                      ("Laplace3D", False, "1", "3", "2", "1"),
                                                      ("Laplace3D", False, "1", "5", "3", "1"),
                                                      ("Laplace3D", False, "1", "64", "3", "2"),
                                                      ("Laplace3D", False, "1", "2", "2", "2"),
                                                      ("Laplace3D", False, "1", "1", "1", "2"),
                                                      ("Laplace3D", False, "1", "4", "3", "2"),
                                                      ("Laplace3D", True, "1", "1", "1", "1"),
                                                      ("Laplace3D", True, "2", "5", "2", "1"),
                                                      ("Brick3D", True, "1", "3", "2", "1"),
                                                      ("Brick3D", True, "2", "2", "1", "1"),
                                                      ("Brick3D", True, "2", "64", "2", "1")])
@pytest.mark.parametrize("dims", [(14, 9, 11), (140, 13, 6)])
def test_spmm_march_slabs_bit_exact(comm, kind, generic, kc, sz, pd, nl, dims, monkeypatch):
    """The march's walk knobs -- MIGMRES_MARCH_SZ planes per workgroup (one plane, ragged last
    slabs, one slab for all), MIGMRES_MARCH_PD planes of loads in flight, MIGMRES_MARCH_NL lines
    per thread (tiles of 4 or 8 lines), MIGMRES_MARCH_KC columns per staged plane (general
    form) -- change only the walk: same bits as the oracle."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    if generic:
        monkeypatch.setenv("MIGMRES_MARCH_GENERIC", "1")
    monkeypatch.setenv("MIGMRES_MARCH_KC", kc)
    monkeypatch.setenv("MIGMRES_MARCH_SZ", sz)
    monkeypatch.setenv("MIGMRES_MARCH_PD", pd)
    monkeypatch.setenv("MIGMRES_MARCH_NL", nl)
    (nx, ny, nz), k = dims, 5
    n = nx * ny * nz
    A = ta.CrsMatrix.galeri(comm, kind, nx, ny, nz)
    assert A.spmm_kernel() == "march"
    gen = (lambda f, m: oe.brick3d_rows(nx, ny, nz, f, m)) if kind == "Brick3D" else \
        (lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m))
    X, _ = oe.epetra_random_mv(37, n, k)
    Yd = ta.MultiVector(comm, n, k)
    A.apply(_upload(ta, comm, X), Yd)
    assert np.array_equal(Yd.download(), oe.DistCrs(gen, n, 1).apply(X))


@pytest.mark.parametrize("perturb", ["interior", "boundary"])
def test_spmm_march27_needs_uniform_stencil(comm, perturb):
    """The uniform 27-point march needs one coefficient table for every pair: a Brick3D
    operator with one coefficient changed (an interior row, or a boundary row) has templates
    that disagree, so it keeps the lane-shared template kernel -- bit for bit either way."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    nx, ny, nz, k = 12, 10, 9, 4
    n = nx * ny * nz
    rp, gc, vv = oe.brick3d_rows(nx, ny, nz, 0, n)
    vv = np.array(vv, dtype=np.float64)
    row = (nz // 2 * ny + ny // 2) * nx + nx // 2 if perturb == "interior" else 1
    vv[rp[row] + 1] = -1.25
    A = ta.CrsMatrix(comm, n, rp, gc, vv)
    assert A.spmm_kernel() == "tpl3"
    Aor = oe.DistCrs(lambda f, m: (rp, gc, vv) if (f, m) == (0, n) else None, n, 1)
    X, _ = oe.epetra_random_mv(47, n, k)
    Yd = ta.MultiVector(comm, n, k)
    A.apply(_upload(ta, comm, X), Yd)
    assert np.array_equal(Yd.download(), Aor.apply(X))


@pytest.mark.parametrize("mode", ["uniform", "lane", "perturbed"])
def test_spmm_march7_coefficient_forms(comm, mode, monkeypatch):
    """The 7-point march keeps no per-lane coefficients when the stencil is uniform (one table,
    absent entries reading out-of-grid zeros); with per-lane coefficients forced
    (MIGMRES_MARCH7_LANE_COEF=1) or a coefficient perturbed in one interior row (the templates
    then disagree), it reads each lane's template coefficients: bit for bit either way."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    nx, ny, nz, k = 14, 9, 8, 3
    n = nx * ny * nz
    rp, gc, vv = oe.laplace3d_rows(nx, ny, nz, 0, n)
    vv = np.array(vv, dtype=np.float64)
    if mode == "lane":
        monkeypatch.setenv("MIGMRES_MARCH7_LANE_COEF", "1")
    if mode == "perturbed":
        row = (nz // 2 * ny + ny // 2) * nx + nx // 2
        vv[rp[row] + 2] = -0.75
    A = ta.CrsMatrix(comm, n, rp, gc, vv)
    assert A.spmm_kernel() == "march"
    Aor = oe.DistCrs(lambda f, m: (rp, gc, vv), n, 1)
    X, _ = oe.epetra_random_mv(53, n, k)
    Yd = ta.MultiVector(comm, n, k)
    A.apply(_upload(ta, comm, X), Yd)
    assert np.array_equal(Yd.download(), Aor.apply(X))
