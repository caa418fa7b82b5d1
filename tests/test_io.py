"""Matrix ingestion: the native MatrixMarket / Harwell-Boeing readers
(trilinos_amd/csrc/io.cpp) against the oracle's restatement of Trilinos_Util_read_hb and a
numpy statement of the MatrixMarket rules (Tpetra::MatrixMarket::Reader::readSparseFile).
The CPU tests call the host-only entry point; the GPU tests build the distributed operator
from the file and solve on it."""

import os

import numpy as np
import pytest

from oracle import belos as ob, epetra as oe

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ORSIRR1 = os.path.join(GOLDEN, "orsirr1.hb")  # belos/epetra/example/BlockGmres/orsirr1.hb (data file)


def _rows(rp, gc, vv):
    """Rows as column-sorted (col, value) lists: the order crs_create stores them in."""
    out = []
    for i in range(rp.size - 1):
        row = sorted(zip(gc[rp[i]:rp[i + 1]].tolist(), vv[rp[i]:rp[i + 1]].tolist()))
        out.append(row)
    return out


def test_hb_orsirr1_matches_oracle_and_fixture():
    import trilinos_amd as ta
    n, rp, gc, vv = ta.matrix_file_rows(ORSIRR1)
    assert n == 1030
    n2, colptr, rowind, vals, sym = oe.read_hb(ORSIRR1)
    assert n2 == n and not sym
    f = np.load(os.path.join(GOLDEN, "orsirr1.npz"))
    assert np.array_equal(f["colptr"], colptr) and np.array_equal(f["rowind"], rowind)
    assert np.array_equal(f["vals"], vals)
    gen, _, _ = oe.hb_problem(colptr, rowind, vals, sym)
    orp, ogc, ovv = gen(0, n)
    got, want = _rows(rp, gc, vv), _rows(orp, ogc, ovv)
    # MSR storage gives every row an explicit diagonal; rows without one in the file gain a 0.0
    for r in range(n):
        w = want[r]
        if r not in [c for c, _ in w]:
            w = sorted(w + [(r, 0.0)])
        assert got[r] == w, r
    # a middle block of rows, as one rank of a uniform map would read it
    n3, rp3, gc3, vv3 = ta.matrix_file_rows(ORSIRR1, 300, 257)
    assert _rows(rp3, gc3, vv3) == got[300:557]


def _write_mm(path, header, size, entries, comments=("% a comment",)):
    with open(path, "w") as fh:
        fh.write(header + "\n")
        for c in comments:
            fh.write(c + "\n")
        fh.write(size + "\n")
        for e in entries:
            fh.write(e + "\n")


def test_matrix_market_general_symmetric_skew_pattern(tmp_path):
    import trilinos_amd as ta
    rng = np.random.default_rng(7)
    n = 23
    dense = np.zeros((n, n))
    ent = []
    for _ in range(70):
        i, j = rng.integers(0, n, 2)
        v = float(rng.standard_normal())
        ent.append((i, j, v))
        dense[i, j] += v  # duplicates are summed
    p = tmp_path / "g.mtx"
    _write_mm(p, "%%MatrixMarket matrix coordinate real general", f"{n} {n} {len(ent)}",
              [f"{i + 1} {j + 1} {v!r}" for i, j, v in ent])
    ng, rp, gc, vv = ta.matrix_file_rows(str(p))
    assert ng == n
    A = np.zeros((n, n))
    for r in range(n):
        for q in range(rp[r], rp[r + 1]):
            assert A[r, gc[q]] == 0.0  # no duplicate survives
            A[r, gc[q]] = vv[q]
    # summation order: file order
    want = np.zeros((n, n))
    for i, j, v in ent:
        want[i, j] = want[i, j] + v
    assert np.array_equal(A, want)

    # symmetric (lower triangle stored) and skew-symmetric, 1-based, mixed whitespace
    low = [(i, j, float(rng.standard_normal())) for i in range(n) for j in range(i + 1) if rng.random() < 0.2]
    for kind, sgn in (("symmetric", 1.0), ("skew-symmetric", -1.0)):
        entries = [(i, j, v) for i, j, v in low if kind == "symmetric" or i != j]
        p = tmp_path / f"{kind}.mtx"
        _write_mm(p, f"%%MatrixMarket matrix coordinate real {kind}", f"  {n}\t{n}  {len(entries)}",
                  [f"{i + 1}\t{j + 1}   {v:.17e}" for i, j, v in entries], comments=("%", "%% two"))
        ng, rp, gc, vv = ta.matrix_file_rows(str(p))
        A = np.zeros((n, n))
        for r in range(n):
            A[r, gc[rp[r]:rp[r + 1]]] = vv[rp[r]:rp[r + 1]]
        want = np.zeros((n, n))
        for i, j, v in entries:
            want[i, j] = v
            if i != j:
                want[j, i] = sgn * v
        assert np.array_equal(A, want), kind

    p = tmp_path / "pat.mtx"
    _write_mm(p, "%%MatrixMarket matrix coordinate pattern general", "3 3 4", ["1 1", "2 3", "3 2", "3 3"])
    ng, rp, gc, vv = ta.matrix_file_rows(str(p))
    assert rp.tolist() == [0, 1, 2, 4] and gc.tolist() == [0, 2, 1, 2] and vv.tolist() == [1.0] * 4


def test_reader_errors(tmp_path):
    import trilinos_amd as ta
    from trilinos_amd._lib import MigmresError
    with pytest.raises(MigmresError, match="cannot open"):
        ta.matrix_file_rows(str(tmp_path / "missing.mtx"))
    p = tmp_path / "dense.mtx"
    _write_mm(p, "%%MatrixMarket matrix array real general", "2 2", ["1", "2", "3", "4"])
    with pytest.raises(MigmresError, match="coordinate"):
        ta.matrix_file_rows(str(p))
    p = tmp_path / "short.mtx"
    _write_mm(p, "%%MatrixMarket matrix coordinate real general", "3 3 3", ["1 1 1.0", "2 2 2.0"])
    with pytest.raises(MigmresError, match="fewer entries"):
        ta.matrix_file_rows(str(p))
    p = tmp_path / "rect.mtx"
    _write_mm(p, "%%MatrixMarket matrix coordinate real general", "3 2 1", ["1 1 1.0"])
    with pytest.raises(MigmresError, match="square"):
        ta.matrix_file_rows(str(p))


@pytest.mark.gpu
def test_gpu_read_file_spmm_bit_exact(tmp_path):
    """Operator read from a MatrixMarket file: SpMM bit-exact against the oracle's CSR rows."""
    import trilinos_amd as ta
    rng = np.random.default_rng(3)
    n, k = 400, 3
    ent = [(i, i, 4.0 + rng.random()) for i in range(n)]
    ent += [(int(rng.integers(0, n)), int(rng.integers(0, n)), float(rng.standard_normal())) for _ in range(3 * n)]
    p = tmp_path / "a.mtx"
    _write_mm(p, "%%MatrixMarket matrix coordinate real general", f"{n} {n} {len(ent)}",
              [f"{i + 1} {j + 1} {v!r}" for i, j, v in ent])
    comm = ta.Comm(device=0)
    A = ta.CrsMatrix.read_file(comm, str(p))
    assert A.n_global == n
    _, rp, gc, vv = ta.matrix_file_rows(str(p))
    Aor = oe.DistCrs(lambda f, m: (rp[f:f + m + 1] - rp[f], gc[rp[f]:rp[f + m]], vv[rp[f]:rp[f + m]]), n, 1)
    Xh = rng.standard_normal((n, k))
    X = ta.MultiVector(comm, n, k)
    X.upload(Xh)
    Y = ta.MultiVector(comm, n, k)
    A.apply(X, Y)
    assert np.array_equal(Y.download(), Aor.apply(Xh))


@pytest.mark.gpu
def test_gpu_orsirr1_from_file_reference_run():
    """test_bl_gmres_hb.cpp's run with the operator ingested from orsirr1.hb by the library
    itself: 209 iterations, actual relative residual 9.94786e-06."""
    import trilinos_amd as ta
    comm = ta.Comm(device=0)
    A = ta.CrsMatrix.read_file(comm, ORSIRR1)
    n = A.n_global
    _, colptr, rowind, vals, sym = oe.read_hb(ORSIRR1)
    gen, b, _ = oe.hb_problem(colptr, rowind, vals, sym)
    B = ta.MultiVector(comm, n, 1)
    B.upload(b[:, None])
    X = ta.MultiVector(comm, n, 1)
    X.put_scalar(0.0)
    lp = ta.LinearProblem(A, X, B)
    assert lp.setProblem()
    sm = ta.BlockGmresSolMgr(lp, {"Num Blocks": n - 1, "Block Size": 1, "Maximum Iterations": n - 1,
                                  "Maximum Restarts": 15, "Convergence Tolerance": 1e-5})
    assert sm.solve() == ta.Converged
    assert sm.getNumIters() == 209
    Aor = oe.DistCrs(gen, n, 1)
    rel = np.linalg.norm(b - Aor.apply(X.download())[:, 0]) / np.linalg.norm(b)
    assert f"{rel:.5e}" == "9.94786e-06"
