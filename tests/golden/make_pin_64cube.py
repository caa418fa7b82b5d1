import sys, time, numpy as np
sys.path.insert(0, '/root/repo')
from oracle import epetra as E, belos as Bl
nx = int(sys.argv[1]) if len(sys.argv) > 1 else 64
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1681692777
N = nx**3; k = 8
A = E.DistCrs(lambda f, n: E.laplace3d_rows(nx, nx, nx, f, n), N, 1)
Xex, _ = E.epetra_random_mv(seed, N, k)
B = A.apply(Xex)
t = time.time()
res = Bl.solve(A.apply, B, {"Num Blocks": 50, "Block Size": 8, "Maximum Iterations": N // 8 - 1,
                            "Maximum Restarts": 50, "Convergence Tolerance": 1e-8, "Orthogonalization": "ICGS"})
R = B - A.apply(res['X'])
rel = np.linalg.norm(R, axis=0) / np.linalg.norm(B, axis=0)
print("seed", seed, "iters", res['iterations'], "conv", res['converged'], "n_apply(solve+setup)", res['n_apply'],
      "explicit", res['n_explicit'], "restarts", res['restarts'], "sing", res['blk_ortho_sing'], "time", time.time() - t)
print("true rel res min/max", rel.min(), rel.max())
print(rel)
