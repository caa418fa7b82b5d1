"""findBasis in Gram form -- the device's default for ICGS block iterations with 2 <= k <= 8
(trilinos_amd/csrc/icgs.hip: k_gemm_nn_gram, k_fbg_chol, k_fbg_a, k_fbg_b) -- restated in numpy
against the reference's column-by-column CGS2 findBasis (oracle/belos.py ICGS.find_basis,
BelosICGSOrthoManager.hpp:936-1225): the same B and Q within rounding on well-conditioned
blocks, and a pivot-ratio gate that hands a nearly dependent block to the column passes
before the reference's own dependency threshold is reached.  CPU only."""

import numpy as np
import pytest

from oracle import belos as ob


def gram_find_basis(X, blk_tol=ob.ICGS_BLK_TOL, gate_factor=100.0):
    """CholQR2 as the device runs it; None when the gate hands the block back."""
    G1 = X.T @ X
    R1 = np.linalg.cholesky(G1).T
    if np.any(np.diag(R1) ** 2 < gate_factor * blk_tol * np.diag(G1)):
        return None
    Y = X @ np.linalg.inv(R1)
    R2 = np.linalg.cholesky(Y.T @ Y).T
    return Y @ np.linalg.inv(R2), R2 @ R1


@pytest.mark.parametrize("k", [2, 5, 8])
def test_gram_form_matches_cgs2(k):
    rng = np.random.default_rng(k)
    n = 2000
    X = rng.standard_normal((n, k)) * np.logspace(0, 3, k)[None, :]  # columns of very different size
    Xc, B = X.copy(), np.zeros((k, k))
    assert ob.ICGS().find_basis(Xc, B, complete_basis=False) == k
    Q, Bg = gram_find_basis(X)
    np.testing.assert_allclose(Bg, B, rtol=1e-12, atol=1e-13 * np.abs(B).max())
    np.testing.assert_allclose(Q, Xc, rtol=0, atol=1e-13)
    assert np.abs(Q.T @ Q - np.eye(k)).max() < 1e-14


def test_gram_gate_precedes_reference_threshold():
    rng = np.random.default_rng(3)
    n, k = 2000, 4
    X = rng.standard_normal((n, k))
    X[:, 3] = X[:, 1] + 1e-3 * rng.standard_normal(n)  # pivot ratio ~1e-6: 7 blk_tol
    B = np.zeros((k, k))
    assert ob.ICGS().find_basis(X.copy(), B, complete_basis=False) == k  # the reference: independent
    assert gram_find_basis(X) is None  # the Gram form defers to the column passes
