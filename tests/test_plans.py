"""Bit-exact index maps: the library's host plan code (C ABI, no GPU needed) against the
oracle's restatement of Epetra (uniform map, MakeColMap_int + Epetra_Util::Sort,
Epetra_Import remote lists, MakeIndicesLocal + SortEntries)."""

import ctypes as C

import numpy as np
import pytest

from oracle import epetra as oe


def _lib():
    import trilinos_amd._lib as L
    return L


def lib_plan(n_global, P, p, rowptr, gcols, vals):
    L = _lib()
    first, nloc = oe.uniform_map(n_global, P, p)
    f, nl = C.c_longlong(), C.c_int()
    L.call("migmres_map_uniform", n_global, P, p, C.byref(f), C.byref(nl))
    assert (f.value, nl.value) == (first, nloc)
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    gcols = np.ascontiguousarray(gcols, dtype=np.int64)
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    ncol = C.c_int()
    L.call("migmres_plan_colmap", n_global, P, first, nloc, L.lptr(rowptr), L.lptr(gcols), None, C.byref(ncol))
    cm = np.empty(ncol.value, dtype=np.int64)
    L.call("migmres_plan_colmap", n_global, P, first, nloc, L.lptr(rowptr), L.lptr(gcols), L.lptr(cm),
           C.byref(ncol))
    nc = ncol.value
    same, nrem = C.c_int(), C.c_int()
    rl = np.empty(max(nc, 1), dtype=np.int32)
    rg = np.empty(max(nc, 1), dtype=np.int64)
    rp = np.empty(max(nc, 1), dtype=np.int32)
    L.call("migmres_plan_remotes", n_global, P, first, nloc, L.lptr(cm), nc, C.byref(same), L.iptr(rl),
           L.lptr(rg), L.iptr(rp), C.byref(nrem))
    nnz = int(rowptr[-1])
    lc = np.empty(max(nnz, 1), dtype=np.int32)
    lv = np.empty(max(nnz, 1), dtype=np.float64)
    L.call("migmres_plan_local_crs", first, nloc, L.lptr(rowptr), L.lptr(gcols), L.dptr(vals), L.lptr(cm), nc,
           L.iptr(lc), L.dptr(lv))
    r = nrem.value
    return dict(colmap=cm, num_same=same.value, remote_lids=rl[:r], remote_gids=rg[:r], remote_pids=rp[:r],
                lcols=lc[:nnz], lvals=lv[:nnz])


def random_rows(n_global, first, nloc, seed, per_row=6):
    """Unstructured rows: random global columns in arbitrary insertion order, so remote
    first-encounter order is NOT sorted by owner (exercises the non-stable shell sort)."""
    rng = np.random.default_rng(seed + first)
    rows, cols, vals = [0], [], []
    for r in range(nloc):
        c = rng.choice(n_global, size=per_row, replace=False)
        c = np.concatenate([c[c != first + r], [first + r]])
        cols.extend(c.tolist())
        vals.extend(rng.standard_normal(len(c)).tolist())
        rows.append(len(cols))
    return np.array(rows), np.array(cols), np.array(vals)


CASES = [("Laplace2D", (100, 100, 1), P) for P in (1, 2, 3, 4, 7)] + \
        [("Laplace3D", (9, 7, 5), P) for P in (1, 3, 8)] + \
        [("Laplace3D", (16, 16, 16), P) for P in (2, 8)] + \
        [("random", (500, 1, 1), P) for P in (1, 4, 5)]


@pytest.mark.parametrize("kind,dims,P", CASES)
def test_plans_match_oracle(kind, dims, P):
    nx, ny, nz = dims
    n_global = nx * ny * nz
    if kind == "Laplace2D":
        gen = lambda f, m: oe.laplace2d_rows(nx, ny, f, m)  # noqa: E731
    elif kind == "Laplace3D":
        gen = lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m)  # noqa: E731
    else:
        gen = lambda f, m: random_rows(n_global, f, m, 17)  # noqa: E731
    D = oe.DistCrs(gen, n_global, P)
    for p in range(P):
        rp, gc, vv = gen(D.firsts[p], D.nlocs[p])
        got = lib_plan(n_global, P, p, rp, gc, vv)
        np.testing.assert_array_equal(got["colmap"], D.colmaps[p])
        pl = D.plans[p]
        assert got["num_same"] == pl["num_same"]
        np.testing.assert_array_equal(got["remote_lids"], pl["remote_lids"])
        np.testing.assert_array_equal(got["remote_gids"], pl["remote_gids"])
        np.testing.assert_array_equal(got["remote_pids"], pl["remote_pids"])
        orp, olc, olv = D.crs[p]
        np.testing.assert_array_equal(got["lcols"], olc)
        np.testing.assert_array_equal(got["lvals"], olv)


def test_laplace2d_two_ranks_hand_checked():
    """2-D 100^2 over 2 ranks: rank 0 owns GIDs 0..4999 and needs the 100 'upper'
    neighbours 5000..5099 of its last grid row, met in ascending order; rank 1 needs
    4900..4999.  Both column maps are [owned..., ghosts...]."""
    D = oe.DistCrs(lambda f, m: oe.laplace2d_rows(100, 100, f, m), 10000, 2)
    np.testing.assert_array_equal(D.colmaps[0][5000:], np.arange(5000, 5100))
    np.testing.assert_array_equal(D.colmaps[1][5000:], np.arange(4900, 5000))
    np.testing.assert_array_equal(D.plans[0]["export_lids"], np.arange(4900, 5000))
    np.testing.assert_array_equal(D.plans[1]["export_lids"], np.arange(0, 100))
    # Epetra sorts each row by LOCAL id, so the ghost column ends row 4999's entries
    rp, lc, _ = D.crs[1]
    assert lc[rp[0]:rp[1]].tolist() == [0, 1, 100, 5000]


def test_epetra_shell_sort_not_stable():
    """Epetra_Util::Sort is a gap-halving shell sort: equal keys can swap order."""
    keys, (comp,) = oe.epetra_util_sort([1, 1, 0, 1, 0], [[10, 11, 12, 13, 14]])
    assert keys == [0, 0, 1, 1, 1]
    assert comp == [12, 14, 11, 13, 10]  # hand-traced; a stable sort gives [12, 14, 10, 11, 13]


def test_uniform_map_remainder_rule():
    """Epetra_BlockMap.cpp:83-90: the first N%P ranks get one extra row."""
    assert [oe.uniform_map(10, 3, p) for p in range(3)] == [(0, 4), (4, 3), (7, 3)]
    assert [oe.uniform_map(7, 4, p) for p in range(4)] == [(0, 2), (2, 2), (4, 2), (6, 1)]
    ids = np.arange(10)
    np.testing.assert_array_equal(oe.owner_of(ids, 10, 3), [0, 0, 0, 0, 1, 1, 1, 2, 2, 2])
