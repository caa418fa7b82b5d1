"""Transposed apply Y = alpha A^T X + beta Y (migmres_crs_apply_mode; Tpetra apply mode TRANS,
Tpetra_CrsMatrix_def.hpp:4965-5100; Epetra_CrsMatrix::Multiply(TransA = true) -> GeneralMTM,
Epetra_CrsMatrix.cpp:3587-3650) against the oracle's restatement of GeneralMTM's scatter loop
(tests/known_answers.py::transpose_apply):

* one GPU: bit for bit on unstructured non-symmetric rows, Laplace3D and the (-1, 2, -1)
  tridiagonal, k = 1..9 columns, alpha / beta forms;
* loopback ranks P = 2, 3: every rank's partial A_p^T x_p in row order, the ghost columns'
  contributions added by their owners in ascending PID order (Epetra_Export, combine Add) --
  bit for bit with that order restated in numpy;
* the Epetra CrsMatrix power-method known answer for A^T (epetra/test/CrsMatrix/cxx_main.cpp:
  234-317) through OperatorTraits::Apply(trans) -- VERDICT r3 "what's missing" 2.
"""

import numpy as np
import pytest

from tests.known_answers import NumpyOps, epetra_tridiag_rows, power_method, transpose_apply
from tests.test_gpu_loopback import run_ranks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    import torch
    assert torch.cuda.is_available()
    import trilinos_amd as ta
    return ta.Comm(device=0)


def _gen(kind, n):
    from oracle import epetra as oe
    from tests.test_plans import random_rows
    if kind == "random":
        return n, lambda f, m: random_rows(n, f, m, 11, per_row=0)
    if kind == "laplace3d":
        return n ** 3, lambda f, m: oe.laplace3d_rows(n, n, n, f, m)
    return n, epetra_tridiag_rows(n, 3.0)


def _oracle_trans(gen, n, X, P=1):
    """A^T X in Epetra's order for a P-rank uniform row partition: each rank's rows scatter
    into a zero column-map vector in row order; an owned column's value is then its owner's
    partial plus the other ranks' partials in ascending rank order."""
    import trilinos_amd as ta
    parts = []
    for p in range(P):
        first, nloc = ta.uniform_map(n, P, p)
        rp, gc, vv = gen(first, nloc)
        rp = np.asarray(rp) - rp[0]
        parts.append(transpose_apply(rp, np.asarray(gc), np.asarray(vv), X[first:first + nloc], n))
    out = np.zeros_like(X)
    for q in range(P):
        first, nloc = ta.uniform_map(n, P, q)
        acc = parts[q][first:first + nloc].copy()
        for p in range(P):
            if p != q:
                acc = acc + parts[p][first:first + nloc]
        out[first:first + nloc] = acc
    return out


def _device_trans(comm, gen, n, X, Y0, alpha, beta):
    import trilinos_amd as ta
    first, nloc = ta.uniform_map(n, comm.nranks, comm.rank)
    A = ta.CrsMatrix(comm, n, *gen(first, nloc))
    k = X.shape[1]
    Xd, Yd = ta.MultiVector(comm, n, k), ta.MultiVector(comm, n, k)
    Xd.upload(X[first:first + nloc])
    Yd.upload(Y0[first:first + nloc])
    A.apply(Xd, Yd, alpha, beta, A.TRANS)
    return first, Yd.download()


@pytest.mark.parametrize("kind,n", [("random", 3001), ("laplace3d", 11), ("tridiag", 5000)])
@pytest.mark.parametrize("k", [1, 3, 9])
def test_transpose_apply_bit_exact(comm, kind, n, k):
    n, gen = _gen(kind, n)
    rng = np.random.default_rng(k)
    X = rng.standard_normal((n, k))
    Y0 = np.full((n, k), np.nan)
    want = _oracle_trans(gen, n, X)
    _, got = _device_trans(comm, gen, n, X, Y0, 1.0, 0.0)   # Epetra Multiply(true): beta 0 ignores NaN in Y
    assert np.array_equal(got, want)
    Y0 = rng.standard_normal((n, k))
    _, got = _device_trans(comm, gen, n, X, Y0, -0.5, 2.0)
    assert np.array_equal(got, -0.5 * want + 2.0 * Y0)


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("kind,n", [("random", 1201), ("laplace3d", 9)])
def test_transpose_apply_ranks_bit_exact(P, kind, n):
    n, gen = _gen(kind, n)
    rng = np.random.default_rng(P)
    X = rng.standard_normal((n, 4))
    Y0 = rng.standard_normal((n, 4))
    want = _oracle_trans(gen, n, X, P)
    for first, got in run_ranks(P, lambda c: _device_trans(c, gen, n, X, Y0, 1.0, 0.0)):
        assert np.array_equal(got, want[first:first + got.shape[0]])
    for first, got in run_ranks(P, lambda c: _device_trans(c, gen, n, X, Y0, 3.0, -1.0)):
        assert np.array_equal(got, 3.0 * want[first:first + got.shape[0]] - Y0[first:first + got.shape[0]])


def test_transpose_apply_alias_rejected(comm):
    import trilinos_amd as ta
    n, gen = _gen("tridiag", 100)
    A = ta.CrsMatrix(comm, n, *gen(0, n))
    X = ta.MultiVector(comm, n, 2)
    X.put_scalar(1.0)
    with pytest.raises(Exception, match="alias"):
        A.apply(X, X, 1.0, 0.0, A.TRANS)


@pytest.mark.parametrize("diag0", [2.0, 20.0])
def test_epetra_power_method_transpose_known_answer(comm, diag0):
    """cxx_main.cpp:234-317 runs the power method on A and on A^T (TransA = true); the 10x
    first diagonal makes A non-symmetric in value order only, so A^T's products run in the
    scatter order of GeneralMTM: every lambda within 1e-12 of the oracle's, success at the same
    iteration."""
    import trilinos_amd as ta
    from oracle import epetra as oe
    from tests.test_gpu_known_answers import DeviceOps
    n = 10001
    gen = epetra_tridiag_rows(n, diag0)
    rp, gc, vv = gen(0, n)
    A = ta.CrsMatrix(comm, n, rp, gc, vv)
    assert ta.OperatorTraits.HasApplyTranspose(A)

    class TransOps(DeviceOps):
        def apply(self, x, y):
            self.ta.OperatorTraits.Apply(self.A, x, y, True)
    z0, _ = oe.epetra_random_mv(7, n, 1)
    z = ta.MultiVector(comm, n, 1)
    z.upload(z0)
    q, r = ta.MultiVector(comm, n, 1), ta.MultiVector(comm, n, 1)
    ierr, lam, lambdas, res = power_method(TransOps(A), z, q, r)
    ierr_o, lam_o, lambdas_o, res_o = power_method(NumpyOps(lambda x: transpose_apply(rp, gc, vv, x, n)),
                                                   z0.copy(), np.zeros((n, 1)), np.zeros((n, 1)))
    assert ierr == ierr_o == 0
    assert len(lambdas) == len(lambdas_o)
    np.testing.assert_allclose(lambdas, lambdas_o, rtol=1e-12, atol=0)
    if diag0 == 20.0:
        assert abs(lam - 20.0) < 0.2
