"""Device time of one SpMM x k (HIP events on the library stream, migmres_ctx_profile) for a
Galeri operator, optionally with the fused right Jacobi.  One configuration per process
(environment switches are read when the operator is built).
  python tools/time_spmm.py KIND NX K [jacobi] [reps]"""
import ctypes as C
import sys

sys.path.insert(0, '.')
import torch  # noqa: F401  (initialise HIP through torch first, as the tests do)
import trilinos_amd as ta
from trilinos_amd._lib import call, lib

kind, nx, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
jac = len(sys.argv) > 4 and sys.argv[4] == "jacobi"
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 30
comm = ta.Comm(0)
A = (ta.CrsMatrix.galeri(comm, kind, 81, 81, 80) if kind == "FlanProxy" else  # configs[3]'s shape
     ta.CrsMatrix.galeri(comm, kind, nx, nx, nx))
n = A.n_global
X = ta.MultiVector(comm, n, k)
X.random(1)
Y = ta.MultiVector(comm, n, k)
M = None
if jac:
    M = ta.Relaxation(A)
    M.compute()
    W = ta.MultiVector(comm, n, k)


def once():
    if M is None:
        A.apply(X, Y)
    else:
        # the solver's fused path through a one-iteration right-preconditioned solve would mix in
        # ortho work; time Jacobi + SpMM (unfused) here unless MIGMRES fuses inside apply
        M.apply(X, W)
        A.apply(W, Y)


for _ in range(3):
    once()
comm.sync()
call("migmres_ctx_profile", comm.h, 1)
for _ in range(reps):
    once()
nk = 32
ms, by, cnt = (C.c_double * nk)(), (C.c_double * nk)(), (C.c_longlong * nk)()
call("migmres_ctx_profile_read", comm.h, ms, by, cnt, nk)
out = {lib.migmres_kernel_class_name(i).decode(): round(ms[i] / cnt[i], 4) for i in range(nk) if cnt[i]}
print(kind, nx, k, "jacobi" if jac else "", A.spmm_kernel(), out, flush=True)
