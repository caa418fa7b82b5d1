"""FillComplete on the device (migmres_crs_create_device, fillcomplete.hip).

The CSR is handed over in HBM (global column ids in insertion order); the column map, the
local ids, the sorted rows and the import's remote lists are built on the GPU.  Parity: the
operator must be the one the host path builds from the same rows (crs_create, itself bit-exact
against the oracle's Epetra restatement, tests/test_plans.py) -- same column map, same import
plan (remote / export lists), same SpMM format -- and its SpMM bit for bit the oracle's, on one
rank and on P ranks through the loopback communicator.  Cases: 7- and 27-point stencils,
unstructured random rows (remote ids in scrambled first-appearance order with PID ties, so
Epetra_Util::Sort's tie order matters; some owned columns never occur, so the column map
keeps only the ones that do), banded long rows and empty rows.
"""

import numpy as np
import pytest

from tests.test_gpu_loopback import run_ranks

pytestmark = pytest.mark.gpu


def _rows(kind, dims):
    from oracle import epetra as oe
    from tests.test_plans import random_rows
    from tests.test_gpu_kernels import banded_rows
    nx, ny, nz = dims
    if kind == "Laplace3D":
        return nx * ny * nz, lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m)
    if kind == "Brick3D":
        return nx * ny * nz, lambda f, m: oe.brick3d_rows(nx, ny, nz, f, m)
    if kind == "banded":
        return nx, lambda f, m: banded_rows(nx, f, m, 7, per_row=ny, band=nz)
    return nx, lambda f, m: random_rows(nx, f, m, 23, per_row=ny)


def _both(comm, n, gen, k):
    import torch
    import trilinos_amd as ta
    first, nloc = ta.uniform_map(n, comm.nranks, comm.rank)
    rp, gc, vv = gen(first, nloc)
    rp = np.asarray(rp, dtype=np.int64)
    gc = np.asarray(gc, dtype=np.int64)
    vv = np.asarray(vv, dtype=np.float64)
    Ah = ta.CrsMatrix(comm, n, rp, gc, vv)
    dev = torch.device("cuda:0")
    Ad = ta.CrsMatrix.from_device(comm, n, torch.from_numpy(rp).to(dev), torch.from_numpy(gc).to(dev),
                                  torch.from_numpy(vv).to(dev))
    same = (np.array_equal(Ah.colmap(), Ad.colmap()) and Ah.n_remote == Ad.n_remote and
            Ah.n_export == Ad.n_export and Ah.nnz_local == Ad.nnz_local and Ah.spmm_kernel() == Ad.spmm_kernel())
    ph, pd = Ah.import_plan(), Ad.import_plan()
    same = same and all(np.array_equal(ph[key], pd[key]) for key in ph)
    from oracle import epetra as oe
    X, _ = oe.epetra_random_mv(17, n, k)
    Xd = ta.MultiVector(comm, n, k)
    Xd.upload(X[first:first + nloc])
    Yh, Yd = ta.MultiVector(comm, n, k), ta.MultiVector(comm, n, k)
    Ah.apply(Xd, Yh)
    Ad.apply(Xd, Yd)
    yh, yd = Yh.download(), Yd.download()
    return first, same, np.array_equal(yh, yd), yd, Ad.n_cols - nloc


CASES = [("Laplace3D", (12, 11, 10), 8, 1), ("Laplace3D", (12, 11, 10), 8, 3), ("Brick3D", (9, 8, 7), 4, 2),
         ("random", (3001, 6, 1), 5, 1), ("random", (3001, 6, 1), 5, 3), ("random", (2000, 0, 1), 3, 4),
         ("banded", (4099, 20, 150), 8, 2), ("Laplace3D", (9, 7, 5), 2, 4)]


@pytest.mark.parametrize("kind,dims,k,P", CASES)
def test_device_fillcomplete_matches_host(kind, dims, k, P):
    import torch
    import trilinos_amd as ta
    from oracle import epetra as oe
    assert torch.cuda.is_available()
    n, gen = _rows(kind, dims)
    Yref = oe.DistCrs(gen, n, P).apply(oe.epetra_random_mv(17, n, k)[0])
    if P == 1:
        res = [_both(ta.Comm(device=0), n, gen, k)]
    else:
        res = run_ranks(P, lambda c: _both(c, n, gen, k))
    Y = np.zeros((n, k))
    for first, same, eq, yd, _ in res:
        assert same, "column map / import plan / format differ from the host FillComplete"
        assert eq, "SpMM differs from the host-built operator"
        Y[first:first + yd.shape[0]] = yd
    assert np.array_equal(Y, Yref)
    if P > 1 and kind == "random":
        assert any(r[4] > 0 for r in res)  # remote columns were exercised


def test_device_fillcomplete_rejects_bad_input():
    """Column ids outside the domain on one rank are refused, as on the host path."""
    import torch
    import trilinos_amd as ta
    comm = ta.Comm(device=0)
    dev = torch.device("cuda:0")
    rp = torch.tensor([0, 1, 2], dtype=torch.int64, device=dev)
    gc = torch.tensor([0, 5], dtype=torch.int64, device=dev)
    vv = torch.ones(2, dtype=torch.float64, device=dev)
    from trilinos_amd._lib import MigmresError
    with pytest.raises(MigmresError):
        ta.CrsMatrix.from_device(comm, 2, rp, gc, vv)
