"""Epetra-layer restatement (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Each function names the reference code it restates (paths relative to
/root/reference/packages).  Integer/index work is bit-exact by construction;
floating-point kernels keep the reference's operation order where the reference
itself fixes it (CSR row sums, RNG, scaling) and use numpy/BLAS where the
reference calls an external BLAS (dot, gemm), whose summation order is not
pinned by the reference.
"""

import numpy as np

# ---------------------------------------------------------------------------
# Random numbers
# ---------------------------------------------------------------------------

MINSTD_A = 16807
MINSTD_M = 2147483647


def minstd_next(seed):
    """Epetra_Util::RandomInt (epetra/src/Epetra_Util.cpp:71-87): Schrage form
    of seed <- 16807*seed mod (2^31-1)."""
    q, r = 127773, 2836
    hi, lo = divmod(seed, q)
    test = MINSTD_A * lo - r * hi
    return test if test > 0 else test + MINSTD_M


def minstd_stream(seed, n):
    """The next n values of Epetra_Util::RandomInt after `seed` (jump-ahead
    vectorised; exact integer arithmetic).  Returns (values uint64, new_seed)."""
    out = np.empty(n, dtype=np.uint64)
    if n == 0:
        return out, seed
    B = min(n, 1 << 16)
    pw = np.empty(B, dtype=np.uint64)
    acc = 1
    for j in range(B):
        acc = (acc * MINSTD_A) % MINSTD_M
        pw[j] = acc
    s = int(seed)
    pos = 0
    while pos < n:
        b = min(B, n - pos)
        blk = (np.uint64(s) * pw[:b]) % np.uint64(MINSTD_M)
        out[pos:pos + b] = blk
        s = int(blk[-1])
        pos += b
    return out, s


def minstd_doubles(ints):
    """Epetra_Util::RandomDouble (Epetra_Util.cpp:90-99): 2*(i/m)-1, same op order."""
    x = ints.astype(np.float64)
    return 2.0 * (x / 2147483647.0) - 1.0


def epetra_random_mv(seed, nrows, ncols):
    """Epetra_MultiVector::Random (Epetra_MultiVector.cpp:490-515) at P=1: column
    by column, row by row from one Epetra_Util stream seeded with `seed`.
    Returns (column-major ndarray shape (nrows, ncols), new_seed)."""
    ints, s = minstd_stream(seed, nrows * ncols)
    vals = minstd_doubles(ints)
    return vals.reshape(ncols, nrows).T.copy(order="F"), s


def glibc_rand(n, seed=1):
    """glibc rand()/random() TYPE_3 additive-feedback generator (the C library
    the reference links); used for Trilinos_Util_read_hb's random xexact
    (triutils/src/Trilinos_Util_read_hb.cpp:147-150) and for the std::rand()
    seeds of Epetra_Util (epetra/src/Epetra_Util.h:270)."""
    r = [0] * 34
    r[0] = seed
    for i in range(1, 31):
        hi, lo = divmod(r[i - 1], 127773)
        w = 16807 * lo - 2836 * hi
        if w < 0:
            w += 2147483647
        r[i] = w
    for i in range(31, 34):
        r[i] = r[i - 31]
    out = []
    k = 34
    total = 344 + n
    buf = r
    while k < total:
        v = (buf[k - 31] + buf[k - 3]) & 0xFFFFFFFF
        buf.append(v)
        if k >= 344:
            out.append(v >> 1)
        k += 1
    return out


GLIBC_RAND_MAX = 2147483647

# ---------------------------------------------------------------------------
# Maps
# ---------------------------------------------------------------------------


def uniform_map(n_global, nprocs, pid):
    """Epetra_BlockMap::ConstructAutoUniform (epetra/src/Epetra_BlockMap.cpp:60-107).
    Returns (first_gid, n_local)."""
    base = n_global // nprocs
    rem = n_global % nprocs
    start = pid * (base + 1)
    n_local = base
    if pid < rem:
        n_local += 1
    else:
        start -= pid - rem
    return start, n_local


def owner_of(gids, n_global, nprocs):
    """Owning PID of each GID in the uniform map (what Epetra_BlockMap::RemoteIDList
    answers for a linear map)."""
    gids = np.asarray(gids, dtype=np.int64)
    base = n_global // nprocs
    rem = n_global % nprocs
    cut = rem * (base + 1)
    pid = np.where(gids < cut, gids // (base + 1), rem + (gids - cut) // max(base, 1))
    return pid.astype(np.int64)


# ---------------------------------------------------------------------------
# Galeri problem generators (row contents in InsertGlobalValues order)
# ---------------------------------------------------------------------------


def _pad_rows(cols, vals):
    """cols/vals: (nrows, w) with -1 for absent entries -> CSR in insertion order."""
    mask = cols >= 0
    counts = mask.sum(axis=1)
    rowptr = np.zeros(cols.shape[0] + 1, dtype=np.int64)
    np.cumsum(counts, out=rowptr[1:])
    return rowptr, cols[mask].astype(np.int64), vals[mask].astype(np.float64)


def laplace2d_rows(nx, ny, first, nloc):
    """Galeri Laplace2D = Cross2D(4,-1,-1,-1,-1) (galeri/src-epetra/Galeri_CrsMatrices.cpp:273-288,
    CrsMatrices/Galeri_Cross2D.h): per row off-diagonals left,right,lower,upper then the diagonal;
    neighbours from GetNeighboursCartesian2d (Galeri_Utils.cpp:331-346)."""
    g = np.arange(first, first + nloc, dtype=np.int64)
    ix = g % nx
    iy = g // nx
    cols = np.full((nloc, 5), -1, dtype=np.int64)
    cols[:, 0] = np.where(ix == 0, -1, g - 1)
    cols[:, 1] = np.where(ix == nx - 1, -1, g + 1)
    cols[:, 2] = np.where(iy == 0, -1, g - nx)
    cols[:, 3] = np.where(iy == ny - 1, -1, g + nx)
    cols[:, 4] = g
    vals = np.array([-1.0, -1.0, -1.0, -1.0, 4.0])[None, :].repeat(nloc, 0)
    return _pad_rows(cols, vals)


def laplace3d_rows(nx, ny, nz, first, nloc):
    """Galeri Laplace3D = Cross3D(6,-1x6) (Galeri_CrsMatrices.cpp:398-416, Galeri_Cross3D.h:78-128):
    off-diagonals left,right,lower,upper,below,above then the diagonal;
    GetNeighboursCartesian3d (Galeri_Utils.cpp:377-398)."""
    g = np.arange(first, first + nloc, dtype=np.int64)
    nxy = nx * ny
    ixy = g % nxy
    iz = g // nxy
    ix = ixy % nx
    iy = ixy // nx
    cols = np.full((nloc, 7), -1, dtype=np.int64)
    cols[:, 0] = np.where(ix == 0, -1, g - 1)
    cols[:, 1] = np.where(ix == nx - 1, -1, g + 1)
    cols[:, 2] = np.where(iy == 0, -1, g - nx)
    cols[:, 3] = np.where(iy == ny - 1, -1, g + nx)
    cols[:, 4] = np.where(iz == 0, -1, g - nxy)
    cols[:, 5] = np.where(iz == nz - 1, -1, g + nxy)
    cols[:, 6] = g
    vals = np.array([-1.0] * 6 + [6.0])[None, :].repeat(nloc, 0)
    return _pad_rows(cols, vals)


def brick3d_rows(nx, ny, nz, first, nloc, a=26.0, off=-1.0):
    """Galeri/Xpetra Brick3D 27-point stencil with Dirichlet truncation on every face
    (galeri/src-xpetra/Galeri_XpetraMatrixTypes.hpp:533-630, Fill9PointStencil :738-760):
    every in-range neighbour of the 3x3x3 cube gets `off`, the centre `a` (boundary rows
    keep `a`).  Column order is irrelevant (FillComplete sorts each row)."""
    g = np.arange(first, first + nloc, dtype=np.int64)
    nxy = nx * ny
    iz = g // nxy
    iy = (g % nxy) // nx
    ix = g % nx
    cols = np.full((nloc, 27), -1, dtype=np.int64)
    vals = np.full((nloc, 27), off)
    c = 0
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                ok = ((ix + dx >= 0) & (ix + dx < nx) & (iy + dy >= 0) & (iy + dy < ny)
                      & (iz + dz >= 0) & (iz + dz < nz))
                cols[:, c] = np.where(ok, g + dx + dy * nx + dz * nxy, -1)
                if dx == 0 and dy == 0 and dz == 0:
                    vals[:, c] = a
                c += 1
    return _pad_rows(cols, vals)


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(x):
    """64-bit finaliser (MurmurHash3 fmix64) on uint64 arrays, wrapping arithmetic."""
    x = np.asarray(x, dtype=np.uint64).copy()
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xFF51AFD7ED558CCD)
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xC4CEB9FE1A85EC53)
        x ^= x >> np.uint64(33)
    return x


def flan_proxy_rows(nx, ny, nz, first, nloc):
    """The synthetic stand-in for BASELINE configs[3] (SuiteSparse Flan_1565, not in this
    image), restated from its SPECIFICATION (include/migmres.h), not from
    the product's generator: 3 dofs per node of an nx x ny x nz hexahedral node grid (nx odd);
    node v = (ix, iy, iz) couples to every in-range node u of its 3x3x3 neighbourhood, in
    dz, dy, dx order from -1 to 1, unless u != v and
    fmix64(min(u,v) * 0x9e3779b97f4a7c15 + max(u,v)) % 13 == 0 (a symmetric 1/13 of the edges
    dropped); each coupled node contributes its 3 dofs in order.  Rows and columns are numbered
    through the scrambled node order p(ix) = (32 ix + 7) mod nx along each grid line (global id
    3 (p(ix) + nx (iy + ny iz)) + dof).  Off-diagonal value -(h + 1) / 997 with
    h = fmix64(row * 0x100000001b3 XOR col) % 997; the diagonal (stored in its neighbourhood
    position) is 1 + the off-diagonal magnitudes summed in insertion order."""
    assert nx % 2 == 1 and nx > 1 and ny > 0 and nz > 0
    ainv = pow(32, -1, nx)
    g = np.arange(first, first + nloc, dtype=np.int64)
    pv = g // 3
    nxy = nx * ny
    iz, iy = pv // nxy, (pv % nxy) // nx
    ix = ((pv % nx - 7) % nx) * ainv % nx           # undo the scramble
    v = ix + nx * (iy + ny * iz)
    cols = np.full((nloc, 81), -1, dtype=np.int64)
    c = 0
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                jx, jy, jz = ix + dx, iy + dy, iz + dz
                ok = (jx >= 0) & (jx < nx) & (jy >= 0) & (jy < ny) & (jz >= 0) & (jz < nz)
                u = jx + nx * (jy + ny * jz)
                lo = np.minimum(u, v).astype(np.uint64)
                hi = np.maximum(u, v).astype(np.uint64)
                with np.errstate(over="ignore"):
                    key = lo * np.uint64(0x9E3779B97F4A7C15) + hi
                dropped = (u != v) & (_mix64(key) % np.uint64(13) == 0)
                ok &= ~dropped
                pu = ((32 * jx + 7) % nx) + nx * (jy + ny * jz)
                for e in range(3):
                    cols[:, c] = np.where(ok, 3 * pu + e, -1)
                    c += 1
    with np.errstate(over="ignore"):
        h = _mix64((g.astype(np.uint64)[:, None] * np.uint64(0x100000001B3)) ^ cols.astype(np.uint64))
    vals = -((h % np.uint64(997)).astype(np.float64) + 1.0) / 997.0
    is_diag = cols == g[:, None]
    vals[is_diag] = 0.0
    vals[cols < 0] = 0.0
    off = np.zeros(nloc)
    for j in range(cols.shape[1]):            # sequential per row, in insertion order
        off += np.where((cols[:, j] >= 0) & ~is_diag[:, j], -vals[:, j], 0.0)
    vals = np.where(is_diag, 1.0 + off[:, None], vals)
    return _pad_rows(cols, vals)


# ---------------------------------------------------------------------------
# Column map and import plan (bit-exact index maps)
# ---------------------------------------------------------------------------


def epetra_util_sort(keys, companions):
    """Epetra_Util::Sort ascending (epetra/src/Epetra_Util.cpp:113-156): gap-halving
    shell sort, NOT stable; companions are permuted alongside.  Operates on copies."""
    keys = list(keys)
    comps = [list(c) for c in companions]
    n = len(keys)
    # Already non-decreasing input makes no swaps (every inner loop breaks at once).
    if all(keys[i] <= keys[i + 1] for i in range(n - 1)):
        return keys, comps
    m = n // 2
    while m > 0:
        for j in range(n - m):
            k = j
            while k >= 0:
                if keys[k + m] >= keys[k]:
                    break
                keys[k], keys[k + m] = keys[k + m], keys[k]
                for c in comps:
                    c[k], c[k + m] = c[k + m], c[k]
                k -= m
        m //= 2
    return keys, comps


def make_colmap(rowptr, gcols, first, nloc, n_global, nprocs):
    """Epetra_CrsGraph::MakeColMap_int (epetra/src/Epetra_CrsGraph.cpp:1348-1524) with the
    default SortGhostsAssociatedWithEachProcessor_=false: domain-local GIDs first in domain
    order, then remote GIDs in first-encounter order, shell-sorted by owner PID.
    `gcols` are the global column indices in insertion (scan) order.
    Returns int64 array of column GIDs."""
    gcols = np.asarray(gcols, dtype=np.int64)
    local = (gcols >= first) & (gcols < first + nloc)
    present = np.zeros(nloc, dtype=bool)
    present[gcols[local] - first] = True
    remote = gcols[~local]
    if nprocs == 1:
        if remote.size:
            raise ValueError("column ids outside the domain map on one process")
        if present.all():
            return np.arange(first, first + nloc, dtype=np.int64)
    if remote.size:
        uniq, idx = np.unique(remote, return_index=True)
        remote_first = uniq[np.argsort(idx, kind="stable")]
    else:
        remote_first = remote
    pids = owner_of(remote_first, n_global, nprocs)
    _, (rg,) = epetra_util_sort(pids.tolist(), [remote_first.tolist()])
    if present.all():
        front = np.arange(first, first + nloc, dtype=np.int64)
    else:
        front = np.nonzero(present)[0].astype(np.int64) + first
    return np.concatenate([front, np.asarray(rg, dtype=np.int64)])


def local_crs(rowptr, gcols, vals, colmap):
    """Epetra_CrsGraph::MakeIndicesLocal + Epetra_CrsMatrix::SortEntries
    (Epetra_CrsMatrix.cpp:1147-1199): global -> local column ids via the column map,
    then each row sorted ascending by LOCAL id (entries are unique per row)."""
    lut = {int(g): i for i, g in enumerate(colmap)} if colmap.size < 200000 else None
    if lut is not None:
        lcols = np.fromiter((lut[int(g)] for g in gcols), dtype=np.int64, count=len(gcols))
    else:
        order = np.argsort(colmap, kind="stable")
        pos = np.searchsorted(colmap[order], gcols)
        lcols = order[pos]
    nrows = len(rowptr) - 1
    rows = np.repeat(np.arange(nrows), np.diff(rowptr))
    perm = np.lexsort((lcols, rows))
    return rowptr.astype(np.int64), lcols[perm].astype(np.int64), np.asarray(vals)[perm]


def import_plans(colmaps, firsts, nlocs, n_global):
    """Epetra_Import::Construct (epetra/src/Epetra_Import.cpp:292-460) from the uniform
    domain map to each rank's column map, for all ranks at once (emulated communicator).
    Export lists follow Distributor::CreateFromRecvs with Deterministic=true: grouped by
    requesting PID ascending, each group in the requester's order.
    Returns list of dicts per rank."""
    nprocs = len(colmaps)
    plans = []
    for p in range(nprocs):
        cm = colmaps[p]
        first, nloc = firsts[p], nlocs[p]
        src = np.arange(first, first + nloc, dtype=np.int64)
        mn = min(len(src), len(cm))
        same = 0
        while same < mn and cm[same] == src[same]:
            same += 1
        rest = cm[same:]
        mine = (rest >= first) & (rest < first + nloc)
        perm_to = (np.nonzero(mine)[0] + same).astype(np.int64)
        perm_from = (rest[mine] - first).astype(np.int64)
        rem_lids = (np.nonzero(~mine)[0] + same).astype(np.int64)
        rem_gids = rest[~mine]
        rem_pids = owner_of(rem_gids, n_global, nprocs)
        k, (rl, rg) = epetra_util_sort(rem_pids.tolist(), [rem_lids.tolist(), rem_gids.tolist()])
        plans.append(dict(num_same=same, permute_to=perm_to, permute_from=perm_from,
                          remote_lids=np.asarray(rl, dtype=np.int64),
                          remote_gids=np.asarray(rg, dtype=np.int64),
                          remote_pids=np.asarray(k, dtype=np.int64)))
    for p in range(nprocs):
        exp_lids, exp_pids = [], []
        for q in range(nprocs):
            if q == p:
                continue
            pq = plans[q]
            sel = pq["remote_pids"] == p
            g = pq["remote_gids"][sel]
            exp_lids.append(g - firsts[p])
            exp_pids.append(np.full(g.size, q, dtype=np.int64))
        plans[p]["export_lids"] = (np.concatenate(exp_lids) if exp_lids else np.zeros(0, np.int64))
        plans[p]["export_pids"] = (np.concatenate(exp_pids) if exp_pids else np.zeros(0, np.int64))
    return plans


class DistCrs:
    """A 1-D row-partitioned CSR operator over an emulated communicator of `nprocs`
    ranks (Epetra_CrsMatrix after FillComplete + OptimizeStorage)."""

    def __init__(self, row_gen, n_global, nprocs):
        self.n_global = n_global
        self.nprocs = nprocs
        self.firsts, self.nlocs, self.colmaps, self.crs = [], [], [], []
        for p in range(nprocs):
            first, nloc = uniform_map(n_global, nprocs, p)
            rp, gc, vv = row_gen(first, nloc)
            cm = make_colmap(rp, gc, first, nloc, n_global, nprocs)
            self.firsts.append(first)
            self.nlocs.append(nloc)
            self.colmaps.append(cm)
            self.crs.append(local_crs(rp, gc, vv, cm))
        self.plans = import_plans(self.colmaps, self.firsts, self.nlocs, n_global)

    def apply(self, X):
        """Y = A*X for a global column-major X (n_global x k): per rank Import into the
        column map (Epetra_DistObject::DoTransfer), then the CSR row loop of
        Epetra_CrsMatrix::GeneralMM (Epetra_CrsMatrix.cpp:3564-3583): sum=0; sum += v*x
        in stored (local-column) order, no fused multiply-add."""
        X = np.asarray(X, dtype=np.float64)
        if X.ndim == 1:
            X = X[:, None]
        Y = np.empty_like(X)
        for p in range(self.nprocs):
            cm = self.colmaps[p]
            Xc = X[cm, :]
            rp, lc, vv = self.crs[p]
            f, n = self.firsts[p], self.nlocs[p]
            Y[f:f + n, :] = csr_rowsum(rp, lc, vv, Xc)
        return Y


def csr_rowsum(rowptr, lcols, vals, Xc):
    """sum_j v_j * x[col_j] per row, accumulated left to right from 0.0, each product and
    sum rounded separately (the C loop at Epetra_CrsMatrix.cpp:3578-3581)."""
    nrows = len(rowptr) - 1
    counts = np.diff(rowptr)
    k = Xc.shape[1]
    Y = np.zeros((nrows, k))
    if nrows == 0:
        return Y
    maxc = int(counts.max()) if counts.size else 0
    for j in range(maxc):
        has = counts > j
        idx = rowptr[:-1][has] + j
        prod = vals[idx][:, None] * Xc[lcols[idx], :]
        Y[has] = Y[has] + prod
    return Y


def read_hb(path):
    """Harwell-Boeing reader for the RUA/RSA fixtures used by the reference tests
    (triutils/src/Trilinos_Util_read_hb.cpp). Returns (n, colptr, rowind, vals, symmetric)
    with 0-based CSC arrays."""
    with open(path) as f:
        lines = f.read().splitlines()
    ptrcrd, indcrd, valcrd, rhscrd = (int(lines[1][i:i + 14]) for i in (14, 28, 42, 56))
    mxtype = lines[2][:3].upper()
    nrow, ncol, nnz = int(lines[2][14:28]), int(lines[2][28:42]), int(lines[2][42:56])
    start = 4 + (1 if rhscrd > 0 else 0)

    def ints(a, b):
        return np.array(" ".join(lines[a:b]).split(), dtype=np.int64)

    def floats(a, b):
        toks = []
        fmt_w = 16
        fld = lines[3][40:60].strip()
        # (1P5E16.8) / (4E20.12) style: fixed width fields
        import re
        m = re.search(r"(\d+)[EDF](\d+)\.", fld.upper())
        if m:
            fmt_w = int(m.group(2))
        for ln in lines[a:b]:
            for i in range(0, len(ln), fmt_w):
                t = ln[i:i + fmt_w].strip()
                if t:
                    toks.append(t.replace("D", "E").replace("d", "e"))
        return np.array(toks, dtype=np.float64)

    colptr = ints(start, start + ptrcrd) - 1
    rowind = ints(start + ptrcrd, start + ptrcrd + indcrd) - 1
    vals = floats(start + ptrcrd + indcrd, start + ptrcrd + indcrd + valcrd)
    assert colptr.size == ncol + 1 and rowind.size == nnz and vals.size == nnz
    return nrow, colptr, rowind, vals, mxtype[1] == "S"


def scscmv(colptr, rowind, vals, x, symmetric=False):
    """y = A x for a CSC matrix, column by column (triutils/src/Trilinos_Util_scscmv.cpp:40-80):
    y[rowind[i]] += val[i] * x[j] in stored order, plus the mirrored entry for symmetric
    storage.  Returns y."""
    n = colptr.size - 1
    y = np.zeros(n)
    for j in range(n):
        for i in range(colptr[j], colptr[j + 1]):
            r = rowind[i]
            y[r] = y[r] + vals[i] * x[j]
            if symmetric and r != j:
                y[j] = y[j] + vals[i] * x[r]
    return y


def hb_problem(colptr, rowind, vals, symmetric=False):
    """Belos::Util::createEpetraProblem on a Harwell-Boeing file without a right-hand side
    (belos/epetra/src/BelosEpetraUtils.cpp:81-200 -> Trilinos_Util_read_hb.cpp:141-158):
    xexact[i] = rand() / RAND_MAX from glibc's stream, b = scscmv(A, xexact).  Returns
    (row generator for DistCrs, b, xexact); the rows' insertion order does not matter
    (FillComplete sorts them)."""
    n = colptr.size - 1
    xexact = np.array(glibc_rand(n), dtype=np.float64) / 2147483647.0
    b = scscmv(colptr, rowind, vals, xexact, symmetric)
    rows = [[] for _ in range(n)]
    for j in range(n):
        for i in range(colptr[j], colptr[j + 1]):
            rows[rowind[i]].append((j, vals[i]))
            if symmetric and rowind[i] != j:
                rows[j].append((rowind[i], vals[i]))

    def gen(first, nloc):
        rp, gc, vv = [0], [], []
        for r in range(first, first + nloc):
            for c, v in rows[r]:
                gc.append(c)
                vv.append(v)
            rp.append(len(gc))
        return np.array(rp, dtype=np.int64), np.array(gc, dtype=np.int64), np.array(vv)

    return gen, b, xexact
