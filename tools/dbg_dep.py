"""Debug: device vs oracle on dependent-block problems (prints counters and history drift)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import trilinos_amd as ta
from oracle import belos as ob, epetra as oe

comm = ta.Comm(device=0)
for case in ("eig4", "eigvec"):
    n, k = 400, 4
    if case == "eig4":
        vals = np.array([1.0, 2.0, 3.0, 5.0])[np.arange(n) % 4]
    else:
        vals = 1.0 + np.arange(n) * 0.05

    def gen(f, m):
        return np.arange(m + 1), np.arange(f, f + m), vals[f:f + m].copy()

    Aor = oe.DistCrs(gen, n, 1)
    Xe, _ = oe.epetra_random_mv(3, n, k)
    if case == "eigvec":
        Xe[:, 0] = 0
        Xe[5, 0] = 1.0
    Bh = Aor.apply(Xe)
    params = {"Num Blocks": 10 if case == "eig4" else 20, "Block Size": k,
              "Maximum Iterations": 50 if case == "eig4" else 200, "Maximum Restarts": 5,
              "Convergence Tolerance": 1e-10 if case == "eig4" else 1e-8, "Orthogonalization": "ICGS"}
    ref = ob.solve(Aor.apply, Bh, params)
    rp, gc, vv = gen(0, n)
    A = ta.CrsMatrix(comm, n, rp, gc, vv)
    B = ta.MultiVector(comm, n, k)
    B.upload(Bh)
    X = ta.MultiVector(comm, n, k)
    X.put_scalar(0.0)
    lp = ta.LinearProblem(A, X, B)
    lp.setProblem()
    sm = ta.BlockGmresSolMgr(lp, params)
    ret = sm.solve()
    h = sm.residualHistory()
    print(case, "device", sm.getNumIters(), sm.counters(), ret)
    print(case, "oracle", ref["iterations"], ref["restarts"], ref["n_apply"], ref["n_explicit"], ref["blk_ortho_sing"],
          ref["converged"])
    if h.shape == ref["history"].shape:
        d = np.abs(h - ref["history"]).max(axis=1)
        print(case, "hist maxdiff per row (first 12):", " ".join(f"{x:.1e}" for x in d[:12]), "max", d.max())
