"""Ifpack2 point-Jacobi restatement (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Ifpack2::Relaxation with "relaxation: type" = "Jacobi" (ifpack2/src/Ifpack2_Relaxation_def.hpp):
  compute():  D^{-1} = reciprocal of the diagonal copy (:1240-1270, no tiny-entry fix, the
              default); the diagonal entry of a row is its (first) entry in column == row.
  apply():    ApplyInverseJacobi (:1390-1454).  With "zero starting solution" (default
              true) the first sweep is Y = (omega * d_i^{-1}) * X (KokkosBlas mult with
              c = 0, KokkosBlas1_mult_impl.hpp:93-104); every further sweep is
              R = X - A Y (Tpetra::Details::residual: b - sum, sum in stored order) and
              Y = 1*Y + (omega * d_i^{-1}) * R.
The Epetra/Ifpack twin (Ifpack_PointRelaxation.cpp:457-480) gives the same bits for
omega = 1 (x*d vs d*x).
"""

import numpy as np


def crs_diagonal(rowptr, gcols, vals, first, nloc):
    """Diagonal copy of a row block (global columns): first entry with column == row, 0 if
    the row has none (Tpetra getLocalDiagCopy via getLocalDiagOffsets)."""
    d = np.zeros(nloc)
    for i in range(nloc):
        g = first + i
        for p in range(int(rowptr[i]), int(rowptr[i + 1])):
            if int(gcols[p]) == g:
                d[i] = vals[p]
                break
    return d


def crs_diagonal_fast(rowptr, gcols, vals, first, nloc):
    """Vectorised crs_diagonal (the last diagonal hit wins only if a row repeats its
    diagonal column, which no generator here does)."""
    rows = np.repeat(np.arange(nloc), np.diff(rowptr))
    hit = gcols == rows + first
    d = np.zeros(nloc)
    d[rows[hit]] = vals[hit]
    return d


class Jacobi:
    """Y = M X for point Jacobi with `sweeps` sweeps and damping `damping`."""

    def __init__(self, A, diag, sweeps=1, damping=1.0, zero_start=True):
        if not zero_start:
            raise ValueError("only 'relaxation: zero starting solution' = true is restated")
        if sweeps < 1:
            raise ValueError("sweeps must be >= 1")
        self.A = A
        self.dinv = 1.0 / np.asarray(diag, dtype=np.float64)
        self.sweeps = sweeps
        self.damping = float(damping)
        self.n_apply = 0

    def __call__(self, X):
        self.n_apply += 1
        X = np.asarray(X, dtype=np.float64)
        ab = (self.damping * self.dinv)[:, None]
        Y = ab * X
        for _ in range(1, self.sweeps):
            R = X - self.A(Y)
            Y = 1.0 * Y + ab * R
        return Y


# ---------------------------------------------------------------------------------------
# Ifpack2::Relaxation's full option set for the types on the device path
# (Ifpack2_Relaxation_def.hpp: defaults :243-307, compute() :990-1280, apply :1323-1454).
# ---------------------------------------------------------------------------------------

RELAXATION_DEFAULTS = {
    "relaxation: type": "Jacobi", "relaxation: sweeps": 1, "relaxation: damping factor": 1.0,
    "relaxation: zero starting solution": True, "relaxation: use l1": False, "relaxation: l1 eta": 1.5,
    "relaxation: min diagonal value": 0.0, "relaxation: fix tiny diagonal entries": False,
    "relaxation: check diagonal entries": False,
}


def relaxation_inverse_diagonal(A, params):
    """compute()'s inverse diagonal over a DistCrs `A` (global vector).  Per rank, from its
    local CRS (local column ids, owned columns first): the first entry with local column ==
    row; with "use l1" on more than one rank, boost = sum of |v / 2| over the entries whose
    local column index exceeds the local row count (:1070-1081, the reference's `>`), added
    when |d| < eta * boost; then 1 / d, or with "fix tiny diagonal entries" 1 / min (1 / eps
    for min = 0) where |d| <= |min| (:1247-1274)."""
    p = dict(RELAXATION_DEFAULTS)
    p.update(params)
    out = np.zeros(A.n_global)
    eps = float(np.finfo(np.float64).eps)
    for q in range(A.nprocs):
        rp, lc, vv = A.crs[q]
        f, nl = A.firsts[q], A.nlocs[q]
        cm = A.colmaps[q]
        for i in range(nl):
            d = 0.0
            for e in range(int(rp[i]), int(rp[i + 1])):
                if cm[lc[e]] == f + i:
                    d = vv[e]
                    break
            if p["relaxation: use l1"] and A.nprocs > 1:
                boost = 0.0
                for e in range(int(rp[i]), int(rp[i + 1])):
                    if lc[e] > nl:
                        boost += abs(vv[e] / 2.0)
                if abs(d) < p["relaxation: l1 eta"] * boost:
                    d += boost
            mn = float(p["relaxation: min diagonal value"])
            if p["relaxation: fix tiny diagonal entries"] and abs(d) <= abs(mn):
                out[f + i] = 1.0 / eps if mn == 0.0 else 1.0 / mn
            else:
                with np.errstate(divide="ignore"):
                    out[f + i] = 1.0 / d
    return out


class Relaxation:
    """Y = M X for Ifpack2::Relaxation "Jacobi" or "Richardson" with any sweeps, damping and
    start (Y0 = the initial Y when "zero starting solution" is false)."""

    def __init__(self, A, params):
        p = dict(RELAXATION_DEFAULTS)
        p.update(params)
        self.p, self.A = p, A
        self.dinv = relaxation_inverse_diagonal(A, p)
        self.n_apply = 0

    def __call__(self, X, Y0=None):
        self.n_apply += 1
        p = self.p
        X = np.asarray(X, dtype=np.float64)
        om = float(p["relaxation: damping factor"])
        jac = p["relaxation: type"] == "Jacobi"
        ab = (om * self.dinv)[:, None]
        zero = p["relaxation: zero starting solution"]
        Y = np.zeros_like(X) if Y0 is None else np.array(Y0, dtype=np.float64)
        if zero:
            Y = ab * X if jac else om * X
        for _ in range(1 if zero else 0, int(p["relaxation: sweeps"])):
            R = X - self.A.apply(Y)
            Y = 1.0 * Y + ab * R if jac else om * R + 1.0 * Y
        return Y

# ---------------------------------------------------------------------------------------
# Ifpack2::Chebyshev (ifpack2/src/Ifpack2_Chebyshev_def.hpp over
# Ifpack2_Details_Chebyshev_def.hpp), the smoother of SURVEY 8(f) rank 2.
#   parameters (Details::Chebyshev :280-300 defaults, setParameters :333-677): "chebyshev:
#     degree" 1, "chebyshev: max eigenvalue" / "min eigenvalue" (unset = estimate), "ratio
#     eigenvalue" 30, "boost factor" 1.1, "min diagonal value" eps, "eigenvalue max
#     iterations" 10, "zero starting solution" true, "textbook algorithm" false;
#   compute() (:739-896): D^-1 by reciprocal_threshold (:95-187: |d| < minVal -> minVal, else
#     1/d -- the reference stores minVal itself, not its reciprocal), the power method on
#     D^-1 A (:1341-1473) unless "assume matrix does not change" with estimates in hand, then
#     lambdaMin = lambdaMax / eigRatio and Ifpack's lambdaMax ~ 1 special case (:884-895);
#   apply() (:909-957): ifpackApplyImpl (:1221-1339) or textbookApplyImpl (:1163-1208), the
#     ChebyshevKernel expression W = beta W + (alpha d_i)(b - A x), X += W
#     (Ifpack2_Details_ChebyshevKernel_def.hpp:160-169, 472-480).
# The power method's initial vector: Tpetra's randomize() stream is not restated; both sides
# use Epetra's MINSTD stream from a seed (oracle.epetra.epetra_random_mv), so the estimate is
# pinned only to this restatement ("parity unpinned" against Tpetra's generator).
# ---------------------------------------------------------------------------------------

CHEBYSHEV_DEFAULTS = {
    "chebyshev: degree": 1,
    "chebyshev: ratio eigenvalue": 30.0,
    "chebyshev: boost factor": 1.1,
    "chebyshev: min diagonal value": float(np.finfo(np.float64).eps),
    "chebyshev: eigenvalue max iterations": 10,
    "chebyshev: zero starting solution": True,
    "chebyshev: assume matrix does not change": False,
    "chebyshev: textbook algorithm": False,
}


def reciprocal_threshold(d, min_val):
    """LocalReciprocalThreshold (Ifpack2_Details_Chebyshev_def.hpp:104-115)."""
    d = np.asarray(d, dtype=np.float64)
    with np.errstate(divide="ignore"):
        inv = 1.0 / d
    return np.where(np.abs(d) < abs(min_val), min_val, inv)


class Chebyshev:
    """Y = M X for Ifpack2::Chebyshev; `A` applies the operator to an (n, k) array, `diag` is
    the diagonal copy, `dot(a, b)` / `norm(a)` are the global inner product and 2-norm."""

    def __init__(self, A, diag, params=None, seed=1, dot=None, norm=None):
        p = dict(CHEBYSHEV_DEFAULTS)
        p.update(params or {})
        self.p = p
        self.A = A
        self.seed = seed
        self.dot = dot or (lambda a, b: float(np.dot(a, b)))
        self.norm = norm or (lambda a: float(np.sqrt(np.dot(a, a))))
        self.user_lmax = p.get("chebyshev: max eigenvalue", np.nan)
        self.eig_ratio = float(p["chebyshev: ratio eigenvalue"])
        self.boost = float(p["chebyshev: boost factor"])
        self.degree = int(p["chebyshev: degree"])
        self.dinv = reciprocal_threshold(diag, float(p["chebyshev: min diagonal value"]))
        self.computed_lmax = np.nan
        self.n_apply = 0
        self.compute()

    def power_method(self, x):
        """powerMethodWithInitGuess (:1344-1406)."""
        lam = 0.0
        nrm = self.norm(x)
        if nrm == 0.0:
            raise RuntimeError("power method initial guess has zero norm")
        x = (1.0 / nrm) * x
        for _ in range(int(self.p["chebyshev: eigenvalue max iterations"])):
            y = self.A(x[:, None])[:, 0]
            y = (1.0 * self.dinv) * y
            lam = self.dot(y, x) / self.dot(x, x)
            nrm = self.norm(y)
            if nrm == 0.0:
                return 0.0
            x = (1.0 / nrm) * y
        return lam

    def compute(self):
        from oracle.epetra import epetra_random_mv
        n = self.dinv.shape[0]
        if not self.p["chebyshev: assume matrix does not change"] or \
                (np.isnan(self.computed_lmax) and np.isnan(self.user_lmax)):
            x, s2 = epetra_random_mv(self.seed, n, 1)
            lam = self.power_method(x[:, 0].copy())
            if lam < 0.0:   # powerMethod (:1457-1471): retry once from |x|, a new draw
                x, _ = epetra_random_mv(s2, n, 1)
                lam = self.power_method(np.abs(x[:, 0]))
            self.computed_lmax = lam
        lmax = self.computed_lmax if np.isnan(self.user_lmax) else float(self.user_lmax)
        lmin = lmax / self.eig_ratio
        ratio = self.eig_ratio
        if not self.p["chebyshev: textbook algorithm"] and abs(lmax - 1.0) < 1.0e-6:
            lmin = lmax = ratio = 1.0
        self.lmax, self.lmin, self.ratio = lmax, lmin, ratio

    def __call__(self, B, X0=None):
        """Ifpack2::Chebyshev::apply(B, X): X = M B (zero start) or the polynomial step from X0."""
        self.n_apply += 1
        B = np.asarray(B, dtype=np.float64)
        X = np.zeros_like(B) if X0 is None else np.array(X0, dtype=np.float64)
        d = self.dinv[:, None]
        if self.p["chebyshev: textbook algorithm"]:
            return self._textbook(B, X, d)
        if self.degree <= 0:
            return X
        lmax, lmin, ratio = self.lmax, self.lmin, self.ratio
        if lmin == 1.0 and lmax == lmin:          # :1250-1253
            return (1.0 * d) * B
        alpha = lmax / ratio
        beta = self.boost * lmax
        delta = 2.0 / (beta - alpha)
        theta = (beta + alpha) / 2.0
        s1 = theta * delta
        zero = self.p["chebyshev: zero starting solution"]
        if zero:
            W = ((1.0 / theta) * d) * B
            X = W.copy()
        else:
            W = ((1.0 / theta) * d) * (B - self.A(X))
            X = X + W
        rhok = 1.0 / s1
        for _ in range(1, self.degree):
            rhokp1 = 1.0 / (2.0 * s1 - rhok)
            dtemp1 = rhokp1 * rhok
            dtemp2 = 2.0 * rhokp1 * delta
            rhok = rhokp1
            W = dtemp1 * W + (dtemp2 * d) * (B - self.A(X))
            X = X + W
        return X

    def _textbook(self, B, X, d):
        """textbookApplyImpl (:1163-1208)."""
        lmax = self.lmax
        lmin = lmax / self.ratio
        dd = (lmax + lmin) / 2.0
        c = (lmax - lmin) / 2.0
        if self.p["chebyshev: zero starting solution"] and self.degree > 0:
            X = np.zeros_like(B)
        P = None
        alpha = 0.0
        for i in range(self.degree):
            R = B - self.A(X)
            Z = (1.0 * d) * R
            if i == 0:
                P = Z.copy()
                alpha = 2.0 / dd
            else:
                beta = alpha * (c / 2.0) * (c / 2.0)
                alpha = 1.0 / (dd - beta)
                P = Z + beta * P
            X = X + alpha * P
        return X
