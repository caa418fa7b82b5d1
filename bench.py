#!/usr/bin/env python3
"""Block GMRES throughput on MI355X: iterations/s + achieved HBM GB/s.

Workload (BASELINE.json configs[1]): Galeri 3-D 7-point Laplacian n = 256^3 (fp64),
k = 8 right-hand sides, Belos BlockGmresSolMgr with "Block Size" 8, "Num Blocks" 25,
"Orthogonalization" "ICGS", fixed-work mode ("Convergence Tolerance" 0, so every run does
exactly --steps block iterations, restarting every 25).  X0 = 0, B = A * Xexact with
Xexact from Epetra's MINSTD stream seeded with 1 (synthetic data, generated on device).

A "step" is one block-Arnoldi iteration (SpMM x k + ICGS + least-squares update).
With N GPUs (torchrun, one process per GPU) the SAME matrix is 1-D row-partitioned over
the ranks (strong scaling): halo exchange and inner-product reductions run over RCCL.

Output: ONE JSON line on rank 0 with the contract fields plus
  roofline      dominant kernel's algorithmic bytes per launch / mean launch time (HIP
                events inside the library, same stream) against the 8 TB/s HBM peak
  cpu_baseline  the numpy oracle (oracle/) timed on this host on a bounded sample
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "BlockGMRES iterations/sec + achieved HBM GB/s, 3-D 7-pt Laplacian k=8 RHS"


def iteration_bytes_model(n, nnz, k, nb, iters):
    """B_it(L) = 12 nnz + 4(N+1) + 16 N k + 8 N (4L + 2k^2 + 19k - 8),
    L = (j+1) k at block step j of a restart cycle.  Summed over `iters` iterations."""
    tot = 0.0
    for i in range(iters):
        j = i % nb
        L = (j + 1) * k
        tot += 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n * k + 8.0 * n * (4 * L + 2 * k * k + 19 * k - 8)
    return tot


def cpu_baseline(k, nb, seconds):
    """Time the numpy oracle (oracle/, kind "port") on a bounded sample: the same solver
    (ICGS, Block Size k, Num Blocks nb, tol 0) on a 64^3 Laplacian for one restart cycle,
    then scale per-iteration time by the row count (the per-row work is the same) to the
    256^3 workload's iterations/s."""
    from oracle import belos as ob, epetra as oe
    m = 64
    n = m ** 3
    A = oe.DistCrs(lambda f, c: oe.laplace3d_rows(m, m, m, f, c), n, 1)
    Xex, _ = oe.epetra_random_mv(1, n, k)
    B = A.apply(Xex)
    iters = nb
    t0 = time.perf_counter()
    ob.solve(A.apply, B, {"Block Size": k, "Num Blocks": nb, "Maximum Iterations": iters,
                          "Maximum Restarts": 1000, "Convergence Tolerance": 0.0,
                          "Orthogonalization": "ICGS"})
    t = time.perf_counter() - t0
    threads = int(os.environ.get("OPENBLAS_NUM_THREADS", os.environ.get("OMP_NUM_THREADS", os.cpu_count())))
    scale = (256 ** 3) / n
    return {"value": iters / (t * scale), "unit": "iterations/s", "cores": threads, "kind": "port",
            "sample": f"oracle/belos.py on 64^3 (k={k}, Num Blocks {nb}, ICGS, tol 0): {iters} iterations "
                      f"in {t:.2f} s, scaled by 256^3/64^3 rows to the 256^3 workload"}


def pmc_traffic(kernel_class, world):
    """Per-launch HBM traffic of `kernel_class` from the committed rocprofv3 PMC summary
    (profiles/pmc_summary.json, made by tools/pmc_summary.py from separate FETCH_SIZE and
    WRITE_SIZE passes of this bench command, gfx950 corrections per MI355X_MICROARCH.md).
    None when no summary for this configuration exists."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if world != 1 or not os.path.exists(path):
        return None
    try:
        summ = json.load(open(path))
        ent = summ["kernels"].get(kernel_class)
        return None if ent is None else ent["traffic_bytes_per_launch"]
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=25)
    ap.add_argument("--nx", type=int, default=256)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--nb", type=int, default=25)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    # secondary workloads; the defaults are the headline configuration
    ap.add_argument("--solver", default="BLOCK GMRES", choices=["BLOCK GMRES", "FLEXIBLE GMRES", "GMRES"])
    ap.add_argument("--matrix", default="Laplace3D", choices=["Laplace3D", "Brick3D"])
    ap.add_argument("--matrix-file", default=None,
                    help="MatrixMarket / Harwell-Boeing file (configs[3]: SuiteSparse Flan_1565 .mtx, not in this "
                         "image) read natively by every rank; overrides --matrix/--nx")
    ap.add_argument("--prec", default="none", choices=["none", "right", "left"])
    ap.add_argument("--sweeps", type=int, default=1)
    ap.add_argument("--ortho", default="ICGS", choices=["ICGS", "DGKS"])
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)

    import trilinos_amd as ta
    from trilinos_amd._lib import call, lib
    comm = ta.Comm.from_torch_distributed(local) if world > 1 else ta.Comm(local)

    nx, k, nb = args.nx, args.k, args.nb
    if args.matrix_file:
        A = ta.CrsMatrix.read_file(comm, args.matrix_file)
        n = A.n_global
    else:
        n = nx ** 3
        A = ta.CrsMatrix.galeri(comm, args.matrix, nx, nx, nx)
    M = None
    if args.prec != "none":
        M = ta.Relaxation(A)
        M.setParameters({"relaxation: sweeps": args.sweeps})
        M.compute()
    Xex = ta.MultiVector(comm, n, k)
    Xex.random(1)
    B = ta.MultiVector(comm, n, k)
    A.apply(Xex, B)
    X = ta.MultiVector(comm, n, k)
    nnz_local = A.nnz_local
    nnz_total = int(comm.sum_all(np.array([float(nnz_local)]))[0])

    def run(iters):
        X.put_scalar(0.0)
        lp = ta.LinearProblem(A, X, B)
        if M is not None:
            (lp.setLeftPrec if args.prec == "left" else lp.setRightPrec)(M)
        lp.setProblem()
        sm = ta.SolverFactory(args.solver, lp, {"Block Size": k, "Num Blocks": nb, "Maximum Iterations": iters,
                                                "Maximum Restarts": 10 ** 6, "Convergence Tolerance": 0.0,
                                                "Orthogonalization": args.ortho})
        sm.solve()
        assert sm.getNumIters() == iters
        return sm

    def barrier():
        if world > 1:
            dist.barrier()

    run(args.warmup)
    barrier()
    comm.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sm = run(args.steps)
    comm.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    timers = sm.timers()

    # per-kernel device times (HIP events on the library's stream) in a second, identical run
    kstats = {}
    if not args.no_profile:
        import ctypes as C
        call("migmres_ctx_profile", comm.h, 1)
        run(args.steps)
        nk = 32  # more than the library's kernel classes; unused slots read back as 0
        ms, by, cnt = (C.c_double * nk)(), (C.c_double * nk)(), (C.c_longlong * nk)()
        call("migmres_ctx_profile_read", comm.h, ms, by, cnt, nk)
        call("migmres_ctx_profile", comm.h, 0)
        for i in range(nk):
            if cnt[i]:
                kstats[lib.migmres_kernel_class_name(i).decode()] = dict(ms=ms[i], bytes=by[i], launches=cnt[i])

    value = args.steps / elapsed
    model_bytes = iteration_bytes_model(n, nnz_total, k, nb, args.steps)
    headline = (args.solver == "BLOCK GMRES" and args.matrix == "Laplace3D" and args.prec == "none"
                and args.ortho == "ICGS" and not args.matrix_file and nx == 256 and k == 8 and nb == 25)
    mname = os.path.basename(args.matrix_file) if args.matrix_file else f"{args.matrix} n={nx}^3"
    wl = (f"3-D 7-pt Laplacian n={nx}^3 fp64, k={k} RHS, Block GMRES Num Blocks {nb}, ICGS, fixed work (tol 0)"
          if headline else
          f"{mname} fp64, k={k} RHS, {args.solver} Num Blocks {nb}, {args.ortho}, "
          f"Jacobi({args.sweeps} sweeps) {args.prec} preconditioner, fixed work (tol 0)"
          if args.prec != "none" else
          f"{mname} fp64, k={k} RHS, {args.solver} Num Blocks {nb}, {args.ortho}, fixed work (tol 0)")
    out = {
        "metric": METRIC, "value": value, "unit": "iterations/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": (f"{mname} from file, " if args.matrix_file else "synthetic (Galeri " + args.matrix + ", ")
                + "Xexact = Epetra MINSTD stream seed 1, B = A*Xexact)",
        "config": {"workload": wl, "n_global": n, "nnz": nnz_total, "k": k,
                   "num_blocks": nb, "parallelism": f"row1d{world}"},
        "hbm_model": None if not headline else {"bytes_per_iteration": model_bytes / args.steps,
                      "achieved_GBps": model_bytes / elapsed / 1e9 / world,
                      "frac_of_peak_per_gpu": model_bytes / elapsed / 1e9 / world / HBM_PEAK_GBPS},
        "solver_timers_s": timers,
    }
    if kstats:
        dom = max(kstats, key=lambda s: kstats[s]["ms"])
        st = kstats[dom]
        per_launch_bytes = st["bytes"] / st["launches"]
        per_launch_s = st["ms"] / 1e3 / st["launches"]
        ach = per_launch_bytes / per_launch_s / 1e9
        traffic = pmc_traffic(dom, world) if headline else None
        out["roofline"] = {"kernel": dom, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                           "frac": ach / HBM_PEAK_GBPS, "traffic": traffic,
                           "bytes_per_launch": per_launch_bytes, "mean_launch_us": per_launch_s * 1e6}
        out["kernels"] = {kname: dict(ms=v["ms"], launches=v["launches"],
                                      GBps=v["bytes"] / (v["ms"] / 1e3) / 1e9 if v["ms"] > 0 else None)
                          for kname, v in kstats.items()}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and headline:
        out["cpu_baseline"] = cpu_baseline(k, nb, 20)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
