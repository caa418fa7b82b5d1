"""Time MultiVector creation (hipMalloc + zero fill) at the bench shapes."""
import sys, time
sys.path.insert(0, '.')
import torch
import trilinos_amd as ta
comm = ta.Comm(0)
n = 256 ** 3
for ncols in (8, 208, 208, 8):
    t0 = time.perf_counter(); mv = ta.MultiVector(comm, n, ncols); comm.sync(); t1 = time.perf_counter()
    mv.put_scalar(1.0); comm.sync(); t2 = time.perf_counter()
    mv.close(); comm.sync(); t3 = time.perf_counter()
    print(f"ncols={ncols}: create {1e3*(t1-t0):.1f} ms, fill {1e3*(t2-t1):.1f} ms, free {1e3*(t3-t2):.1f} ms")
