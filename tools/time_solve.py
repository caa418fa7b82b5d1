"""Phase breakdown of one fixed-work solve at the bench shape (sync timers)."""
import sys, time
sys.path.insert(0, '.')
import torch
import trilinos_amd as ta
comm = ta.Comm(0)
nx = int(sys.argv[1]) if len(sys.argv) > 1 else 256
k, nb, its = 8, 25, 50
n = nx ** 3
A = ta.CrsMatrix.galeri(comm, "Laplace3D", nx, nx, nx)
Xe = ta.MultiVector(comm, n, k); Xe.random(1)
B = ta.MultiVector(comm, n, k); A.apply(Xe, B)
X = ta.MultiVector(comm, n, k)
for verb in (0, 1, 0):
    X.put_scalar(0.0)
    lp = ta.LinearProblem(A, X, B); lp.setProblem()
    sm = ta.BlockGmresSolMgr(lp, {"Block Size": k, "Num Blocks": nb, "Maximum Iterations": its, "Maximum Restarts": 10**6,
                                  "Convergence Tolerance": 0.0, "Orthogonalization": "ICGS", "Verbosity": verb})
    t0 = time.perf_counter(); sm.solve(); comm.sync(); t1 = time.perf_counter()
    print(f"verbosity={verb} wall {t1-t0:.3f}s", {kk: round(v, 4) for kk, v in sm.timers().items()}, sm.counters())
