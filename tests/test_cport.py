"""The C/OpenMP CPU baseline (oracle/cport/bgmres.c) against the numpy oracle.

bench.py's cpu_baseline times the C restatement on the benchmark workload; this pins it to
oracle/belos.py (itself pinned to the reference's recorded runs): the
same status-check history (implicit residual norms at every check, restarts included) and
the same final X, within rounding (the C loops and numpy's BLAS sum in different orders).
"""

import ctypes as C
import os

import numpy as np
import pytest

from oracle import belos as ob, epetra as oe

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "oracle", "cport", "libcport.so")


def _lib():
    if not os.path.exists(SO):
        pytest.skip("oracle/cport/libcport.so not built (make -C oracle/cport)")
    return C.CDLL(SO)


def cport_solve(m, k, nb, iters):
    n = m ** 3
    rows = iters + iters // nb + 2
    h = np.zeros((rows, k))
    x = np.zeros((k, n))
    secs = np.zeros(2)
    nh = C.c_int()
    rc = _lib().cport_block_gmres_laplace3d(m, k, nb, iters, 1, h.ctypes.data_as(C.c_void_p), C.byref(nh),
                                            x.ctypes.data_as(C.c_void_p), secs.ctypes.data_as(C.c_void_p))
    assert rc == 0, rc
    return h[:nh.value], x.T


@pytest.mark.parametrize("m,k,nb,iters", [(10, 4, 5, 23), (12, 8, 4, 13), (9, 1, 6, 20), (8, 3, 3, 10),
                                          (8, 16, 2, 5)])
def test_cport_matches_oracle(m, k, nb, iters):
    h, x = cport_solve(m, k, nb, iters)
    n = m ** 3
    A = oe.DistCrs(lambda f, c: oe.laplace3d_rows(m, m, m, f, c), n, 1)
    Xex, _ = oe.epetra_random_mv(1, n, k)
    B = A.apply(Xex)
    ref = ob.solve(A.apply, B, {"Block Size": k, "Num Blocks": nb, "Maximum Iterations": iters,
                                "Maximum Restarts": 1000, "Convergence Tolerance": 0.0,
                                "Orthogonalization": "ICGS"})
    assert ref["iterations"] == iters
    assert h.shape == ref["history"].shape
    np.testing.assert_allclose(h, ref["history"], rtol=0, atol=1e-13)
    np.testing.assert_allclose(x, ref["X"], rtol=0, atol=1e-13 * np.abs(ref["X"]).max())
