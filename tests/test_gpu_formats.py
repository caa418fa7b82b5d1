"""SpMM format plans built on the device (formats.hip) against plan.cpp's host builders
(MIGMRES_HOST_FORMATS=1): the pair plan in its SELL layout, the SELL-64 copy, the detected
3 x 3 blocks, the row-pair templates (value dictionary and template ids in first-appearance
order), the stencil groups, the template-rest and interior / boundary unit lists -- compared
through migmres_crs_format_digest (flags, fixed bytes, a hash of every array), on one rank and
on P ranks (ghost columns), for operators built from host rows and from device rows
(migmres_crs_create_device, whose FillComplete then never returns the CSR to the host).
Cases cover each format and each "not applicable" exit: > 255 distinct values (no
templates), rows longer than the pair plan takes, empty rows, an odd row count.
"""

import numpy as np
import pytest

from tests.test_gpu_loopback import run_ranks

pytestmark = pytest.mark.gpu


def _gen(kind, dims):
    from oracle import epetra as oe
    from tests.test_gpu_kernels import banded_rows
    from tests.test_plans import random_rows
    nx, ny, nz = dims
    if kind == "Laplace3D":
        return nx * ny * nz, lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m)
    if kind == "Laplace2D":
        return nx * ny, lambda f, m: oe.laplace2d_rows(nx, ny, f, m)
    if kind == "Brick3D":
        return nx * ny * nz, lambda f, m: oe.brick3d_rows(nx, ny, nz, f, m)
    if kind == "FlanProxy":
        return 3 * nx * ny * nz, lambda f, m: oe.flan_proxy_rows(nx, ny, nz, f, m)
    if kind == "noisy3D":   # a 7-point pattern with distinct values: no template dictionary
        def g(f, m):
            rp, gc, vv = oe.laplace3d_rows(nx, ny, nz, f, m)
            return rp, gc, np.asarray(vv) + 1e-3 * np.arange(len(vv))
        return nx * ny * nz, g
    if kind == "banded":
        return nx, lambda f, m: banded_rows(nx, f, m, 7, per_row=ny, band=nz)
    if kind == "orsirr1":
        from tests.test_oracle_pins import orsirr1_problem
        n, gen, _, _ = orsirr1_problem()
        return n, gen
    return nx, lambda f, m: random_rows(nx, f, m, 23, per_row=ny)


CASES = [("Laplace3D", (12, 11, 10)), ("Laplace2D", (31, 27, 1)), ("Brick3D", (10, 9, 8)),
         ("FlanProxy", (9, 8, 7)), ("noisy3D", (9, 8, 7)), ("banded", (4099, 20, 150)),
         ("random", (3001, 6, 1)), ("random", (2001, 0, 1)), ("orsirr1", (0, 0, 0))]


def _build(comm, n, gen, from_device):
    import trilinos_amd as ta
    first, nloc = ta.uniform_map(n, comm.nranks, comm.rank)
    rp, gc, vv = gen(first, nloc)
    rp, gc, vv = (np.asarray(rp, dtype=np.int64), np.asarray(gc, dtype=np.int64), np.asarray(vv, dtype=np.float64))
    if from_device:
        import torch
        dev = torch.device("cuda:0")
        A = ta.CrsMatrix.from_device(comm, n, torch.from_numpy(rp).to(dev), torch.from_numpy(gc).to(dev),
                                     torch.from_numpy(vv).to(dev))
    else:
        A = ta.CrsMatrix(comm, n, rp, gc, vv)
    return A.spmm_kernel(), A.format_digest()


def _stage(P, n, gen, from_device, monkeypatch, host):
    import trilinos_amd as ta
    monkeypatch.setenv("MIGMRES_HOST_FORMATS", "1" if host else "0")
    if P == 1:
        return [_build(ta.Comm(device=0), n, gen, from_device)]
    return run_ranks(P, lambda c: _build(c, n, gen, from_device))


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("kind,dims", CASES)
def test_device_formats_equal_host_formats(kind, dims, P, monkeypatch):
    n, gen = _gen(kind, dims)
    host = _stage(P, n, gen, False, monkeypatch, True)
    dev = _stage(P, n, gen, False, monkeypatch, False)
    devfc = _stage(P, n, gen, True, monkeypatch, False)
    for h, d, f in zip(host, dev, devfc):
        assert h[0] == d[0] == f[0]
        assert h[1] == d[1], "device-built format plans differ from the host builders'"
        assert h[1] == f[1], "device FillComplete + device formats differ from the host path"
    if P == 1:
        expect = {"Laplace3D": "march", "Laplace2D": "tpl", "Brick3D": "march", "FlanProxy": "bsr3",
                  "noisy3D": "pair", "banded": "sell"}.get(kind)
        if expect:
            assert host[0][0] == expect


@pytest.mark.parametrize("kind,dims", [("Laplace3D", (12, 11, 10)), ("Brick3D", (10, 9, 8))])
def test_template_hash_collision_falls_back_to_host_builder(kind, dims, monkeypatch):
    """A shape-hash collision in the device template builder (forced: MIGMRES_TPL_HASH_BITS=1
    folds the 27 shapes onto two hashes) must not fail the CrsMatrix creation: the plan is
    rebuilt by the host builder (exact shape comparison), so kernel and digest equal the host
    path's (formats.hip threw on a collision and leaked the id buffer)."""
    n, gen = _gen(kind, dims)
    host = _stage(1, n, gen, False, monkeypatch, True)
    monkeypatch.setenv("MIGMRES_TPL_HASH_BITS", "1")
    dev = _stage(1, n, gen, False, monkeypatch, False)
    devfc = _stage(1, n, gen, True, monkeypatch, False)
    assert host[0][0] == dev[0][0] == devfc[0][0] == "march"
    assert host[0][1] == dev[0][1] == devfc[0][1]
