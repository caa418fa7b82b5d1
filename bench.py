#!/usr/bin/env python3
"""Block GMRES throughput on MI355X: iterations/s + achieved HBM GB/s.

Workload (BASELINE.json configs[1]): Galeri 3-D 7-point Laplacian n = 256^3 (fp64),
k = 8 right-hand sides, Belos BlockGmresSolMgr with "Block Size" 8, "Num Blocks" 25,
"Orthogonalization" "ICGS", fixed-work mode ("Convergence Tolerance" 0, so every run does
exactly `steps` block iterations, restarting every 25).  X0 = 0, B = A * Xexact with
Xexact from Epetra's MINSTD stream seeded with 1 (synthetic data, generated on device).

A "step" is one block-Arnoldi iteration (SpMM x k + ICGS + least-squares update).  --steps
is rounded up to whole restart cycles (the line's "steps" is the count timed).
`--gpus N` starts N rank processes (one per GPU) unless torchrun already did; the SAME
matrix is 1-D row-partitioned over the ranks (strong scaling): halo exchange and
inner-product reductions run over RCCL.

Output: ONE JSON line on rank 0 with the contract fields plus
  hbm           the metric's achieved HBM GB/s: algorithmic bytes of the kernels that ran
                (library tally) / timed wall time, per GPU
  roofline      dominant kernel's algorithmic bytes per launch / mean launch time (HIP
                events inside the library, same stream) against the 8 TB/s HBM peak;
                traffic = PMC traffic/algorithmic ratio (profiles/pmc_summary.json) x bytes
  reference_equivalent  SURVEY 8(d)'s reference-algorithm byte model / wall time (labelled,
                not achieved traffic)
  cpu_baseline  the CPU restatement timed on this host on a bounded sample
  ranks         (N > 1) per-rank halo / all-reduce device milliseconds
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


def cpu_baseline(k, nb, m, iters):
    """The reference algorithm on this host's CPU cores (cpu_baseline.kind "port"): the C/OpenMP
    restatement oracle/cport/bgmres.c (validated against the numpy oracle, tests/test_cport.py)
    runs the benchmark's own workload -- Laplace3D m^3, k RHS, Block GMRES ICGS, Num Blocks nb,
    tol 0 -- for `iters` block iterations (one whole restart cycle by default) with
    OMP_NUM_THREADS threads.  With m < 256 the rate is scaled by rows (m^3 / 256^3) and says so."""
    import ctypes as C
    so = os.path.join(ROOT, "oracle", "cport", "libcport.so")
    lib = C.CDLL(so)
    secs = (C.c_double * 2)()
    nh = C.c_int()
    rc = lib.cport_block_gmres_laplace3d(m, k, nb, iters, 1, None, C.byref(nh), None, secs)
    if rc != 0:
        return {"value": None, "error": f"cport returned {rc}"}
    scale = (m ** 3) / (256 ** 3)
    val = iters / secs[0] * scale
    sample = (f"oracle/cport/bgmres.c (C/OpenMP restatement of the reference Block GMRES + ICGS) on Laplace3D "
              f"{m}^3, k={k}, Num Blocks {nb}, tol 0: {iters} block iterations in {secs[0]:.2f} s")
    if m != 256:
        sample += f", scaled by {m}^3/256^3 rows to the 256^3 workload"
    return {"value": val, "unit": "iterations/s", "cores": int(secs[1]), "kind": "port", "sample": sample}


def cpu_baseline_subprocess(threads, k, nb, m, iters, timeout=300):
    """cpu_baseline with OMP_NUM_THREADS=`threads` in a child process (the OpenMP runtime
    reads it once, at start-up).  The child loads only the C restatement, never the GPU."""
    import subprocess
    code = ("import sys, json; sys.path.insert(0, %r); import bench; "
            "print(json.dumps(bench.cpu_baseline(%d, %d, %d, %d)))" % (ROOT, k, nb, m, iters))
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    try:
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=timeout)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:  # the baseline is reported, not required
        return {"value": None, "error": f"{type(e).__name__}: {e}"}


def pmc_ratio(kernel_class, world):
    """HBM traffic / algorithmic bytes of `kernel_class`, from the committed rocprofv3 PMC
    summary (profiles/pmc_summary.json, made by tools/pmc_summary.py from separate FETCH_SIZE
    and WRITE_SIZE passes of this bench command with the gfx950 corrections of
    MI355X_MICROARCH.md, divided by the algorithmic bytes per launch of the same run).  The
    ratio does not depend on --steps; the bench multiplies it by this run's bytes per launch.
    None when no summary exists."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if world != 1 or not os.path.exists(path):
        return None
    try:
        ent = json.load(open(path))["kernels"].get(kernel_class)
        return None if ent is None else ent.get("ratio")
    except Exception:
        return None


def csr_spmm_forms(ta, comm, args, n, k, nnz, call, reps=20):
    """The same operator built again with the stencil formats switched off (the environment
    switches are read at creation), and `reps` applies of X (k columns) timed through the
    library's HIP-event profile: the row-pair CSR kernel (MIGMRES_NO_TPL_SPMM) and the plain
    thread-per-row CSR kernel (also MIGMRES_NO_PAIR_SPMM, MIGMRES_NO_SELL_SPMM).  Fractions on
    the CSR's bytes 12 nnz + 4 (N + 1) + 16 N k."""
    import ctypes as C
    forms = {"csr_pair": {"MIGMRES_NO_TPL_SPMM": "1"},
             "csr_row": {"MIGMRES_NO_TPL_SPMM": "1", "MIGMRES_NO_PAIR_SPMM": "1", "MIGMRES_NO_SELL_SPMM": "1"}}
    csr_bytes = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n * k
    res = {}
    for name, env in forms.items():
        old = {key: os.environ.get(key) for key in env}
        os.environ.update(env)
        try:
            if args.matrix == "FlanProxy":
                A2 = ta.CrsMatrix.galeri(comm, "FlanProxy", 81, 81, 80)
            else:
                A2 = ta.CrsMatrix.galeri(comm, args.matrix, args.nx, args.nx, args.nz if args.nz > 0 else args.nx)
        finally:
            for key, v in old.items():
                if v is None:
                    os.environ.pop(key, None)
                else:
                    os.environ[key] = v
        X2, Y2 = ta.MultiVector(comm, n, k), ta.MultiVector(comm, n, k)
        X2.random(5)
        A2.apply(X2, Y2)  # warm
        call("migmres_ctx_profile", comm.h, 1)
        for _ in range(reps):
            A2.apply(X2, Y2)
        nk = 32
        ms, by, cnt = (C.c_double * nk)(), (C.c_double * nk)(), (C.c_longlong * nk)()
        call("migmres_ctx_profile_read", comm.h, ms, by, cnt, nk)
        call("migmres_ctx_profile", comm.h, 0)
        i = [j for j in range(nk) if cnt[j]]
        t = sum(ms[j] for j in i) / 1e3 / reps
        res[name] = {"kernel": A2.spmm_kernel(), "mean_launch_us": t * 1e6, "csr_bytes": csr_bytes,
                     "achieved": csr_bytes / t / 1e9, "frac": csr_bytes / t / 1e9 / HBM_PEAK_GBPS}
        del A2, X2, Y2
    return res


def spawn_ranks(n, argv, port=None, timeout=None, poll_s=0.1):
    """`bench.py --gpus N` without a torchrun environment: start N rank processes of this
    script (one per GPU, RANK = LOCAL_RANK = i, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1) as
    children, before anything in this process touches the GPU.  Every child is polled: on
    the first non-zero exit the others are terminated (then killed after 10 s) and that exit
    code is returned, so a rank that dies (RCCL init, out of memory, bad device) cannot leave
    its peers blocked in a collective.  Past `timeout` seconds every rank is killed and 124
    is returned.  0 when every rank succeeded.  Rank 0 prints the JSON line."""
    import signal
    import socket
    import subprocess
    if port is None:
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(argv, env=env))

    def stop_all():
        live = [p for p in procs if p.poll() is None]
        for p in live:
            p.send_signal(signal.SIGTERM)
        t_end = time.monotonic() + 10.0
        for p in live:
            try:
                p.wait(timeout=max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    t0 = time.monotonic()
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                print(f"bench.py: rank {r} exited with status {c}; stopping the other ranks", file=sys.stderr,
                      flush=True)
                stop_all()
                return c
            if all(c == 0 for c in codes):
                return 0
            if timeout is not None and time.monotonic() - t0 > timeout:
                print(f"bench.py: ranks still running after {timeout} s; stopping them", file=sys.stderr, flush=True)
                stop_all()
                return 124
            time.sleep(poll_s)
    except BaseException:
        stop_all()
        raise


def start_watchdog(seconds, rank):
    """A hang anywhere in a rank (a collective whose peer died after joining, a stuck device
    call) ends the rank with status 124 after `seconds`, so the launcher (spawn_ranks or
    torchrun's agent) stops the job and reports instead of waiting for its own time limit."""
    import threading

    def fire():
        print(f"bench.py: rank {rank} still running after {seconds} s; exiting (124)", file=sys.stderr, flush=True)
        os._exit(124)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=25)
    ap.add_argument("--nx", type=int, default=256)
    ap.add_argument("--nz", type=int, default=0,
                    help="planes of the Laplace3D / Brick3D grid (0: nx); e.g. --nz 32 gives one GPU the rows one "
                         "rank of the 8-GPU 256^3 run holds")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--nb", type=int, default=25)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-cpu-one-core", action="store_true", help="skip the 1-core cpu_baseline sample")
    ap.add_argument("--cpu-nx", type=int, default=256, help="cpu_baseline sample size (m^3 rows)")
    ap.add_argument("--cpu-iters", type=int, default=0, help="cpu_baseline block iterations (0: one cycle)")
    # secondary workloads; the defaults are the headline configuration
    ap.add_argument("--solver", default="BLOCK GMRES", choices=["BLOCK GMRES", "FLEXIBLE GMRES", "GMRES"])
    ap.add_argument("--matrix", default="Laplace3D", choices=["Laplace3D", "Brick3D", "FlanProxy"],
                    help="FlanProxy: configs[3]'s shape (Flan_1565 is not in this image) -- 81 x 81 x 80 "
                         "hexahedral nodes x 3 dofs = 1,574,640 rows, ~73 nnz per row, unstructured SELL path; "
                         "--nx is ignored")
    ap.add_argument("--matrix-file", default=None,
                    help="MatrixMarket / Harwell-Boeing file (configs[3]: SuiteSparse Flan_1565 .mtx, not in this "
                         "image) read natively by every rank; overrides --matrix/--nx")
    ap.add_argument("--prec", default="none", choices=["none", "right", "left"])
    ap.add_argument("--sweeps", type=int, default=1)
    ap.add_argument("--prec-type", default="jacobi", choices=["jacobi", "chebyshev"],
                    help="the --prec preconditioner: Ifpack2::Relaxation Jacobi (--sweeps) or Ifpack2::Chebyshev "
                         "(--cheb-degree, power-method lambda max)")
    ap.add_argument("--cheb-degree", type=int, default=3)
    ap.add_argument("--ortho", default="ICGS", choices=["ICGS", "DGKS"])
    ap.add_argument("--no-csr-spmm", dest="csr_spmm", action="store_false",
                    help="skip timing the CSR SpMM forms beside the default SpMM (roofline_spmm.csr_forms)")
    ap.add_argument("--comm-timeout", type=float, default=300.0,
                    help="seconds: torch.distributed (gloo) set-up / barrier timeout and the RCCL init watchdog")
    ap.add_argument("--deadline", type=float, default=1500.0,
                    help="seconds: a rank still running after this exits with status 124 (N > 1; 0 = off)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                             timeout=args.deadline + 60 if args.deadline > 0 else None))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        if args.deadline > 0:
            start_watchdog(args.deadline, rank)
        # one GPU per rank: check before set_device (device_count does not initialise HIP)
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        ndev = torch.cuda.device_count()
        if ndev < local_world or local >= ndev:
            sys.exit(f"bench.py: rank {rank}: {ndev} visible GPU(s) for {local_world} local ranks "
                     f"(LOCAL_RANK={local})")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MIGMRES_RCCL_INIT_TIMEOUT", str(int(args.comm_timeout)))
        import datetime
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=args.comm_timeout))
        # every rank alive and through its imports before RCCL's blocking communicator set-up;
        # monitored_barrier names the rank that did not arrive
        dist.monitored_barrier(timeout=datetime.timedelta(seconds=args.comm_timeout))
    torch.cuda.set_device(local)

    import trilinos_amd as ta
    from trilinos_amd._lib import call, lib, rccl_info
    comm = ta.Comm.from_torch_distributed(local) if world > 1 else ta.Comm(local)

    nx, k, nb = args.nx, args.k, args.nb
    if args.matrix_file:
        A = ta.CrsMatrix.read_file(comm, args.matrix_file)
        n = A.n_global
    elif args.matrix == "FlanProxy":
        dims = (81, 81, 80)
        n = 3 * dims[0] * dims[1] * dims[2]
        A = ta.CrsMatrix.galeri(comm, "FlanProxy", *dims)
    else:
        nz = args.nz if args.nz > 0 else nx
        n = nx * nx * nz
        A = ta.CrsMatrix.galeri(comm, args.matrix, nx, nx, nz)
    M = None
    if args.prec != "none":
        if args.prec_type == "chebyshev":
            M = ta.Chebyshev(A)
            M.setParameters({"chebyshev: degree": args.cheb_degree})
        else:
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

    # Time whole restart cycles: the cost of a block iteration grows with its position in the
    # cycle (L = (j+1) k basis vectors to project against), so a partial cycle would flatter
    # the rate.  --steps is rounded up to a multiple of Num Blocks; "steps" reports the count run.
    steps = -(-args.steps // nb) * nb

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
    sm = run(steps)
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
        run(steps)
        nk = 32  # more than the library's kernel classes; unused slots read back as 0
        ms, by, cnt = (C.c_double * nk)(), (C.c_double * nk)(), (C.c_longlong * nk)()
        call("migmres_ctx_profile_read", comm.h, ms, by, cnt, nk)
        call("migmres_ctx_profile", comm.h, 0)
        for i in range(nk):
            if cnt[i]:
                kstats[lib.migmres_kernel_class_name(i).decode()] = dict(ms=ms[i], bytes=by[i], launches=cnt[i])

    value = steps / elapsed
    model_bytes = iteration_bytes_model(n, nnz_total, k, nb, steps)
    headline = (args.solver == "BLOCK GMRES" and args.matrix == "Laplace3D" and args.prec == "none"
                and args.ortho == "ICGS" and not args.matrix_file and nx == 256 and args.nz in (0, 256) and k == 8
                and nb == 25)
    mname = (os.path.basename(args.matrix_file) if args.matrix_file else
             f"FlanProxy n={n} (synthetic stand-in for SuiteSparse Flan_1565)" if args.matrix == "FlanProxy" else
             f"{args.matrix} n={nx}^3" if args.nz in (0, nx) else f"{args.matrix} n={nx}x{nx}x{args.nz}")
    wl = (f"3-D 7-pt Laplacian n={nx}^3 fp64, k={k} RHS, Block GMRES Num Blocks {nb}, ICGS, fixed work (tol 0)"
          if headline else
          f"{mname} fp64, k={k} RHS, {args.solver} Num Blocks {nb}, {args.ortho}, " +
          (f"Chebyshev(degree {args.cheb_degree}) " if args.prec_type == "chebyshev" else
           f"Jacobi({args.sweeps} sweeps) ") + f"{args.prec} preconditioner, fixed work (tol 0)"
          if args.prec != "none" else
          f"{mname} fp64, k={k} RHS, {args.solver} Num Blocks {nb}, {args.ortho}, fixed work (tol 0)")
    # secondary workloads name their own operator / k in the metric (the headline keeps BASELINE's)
    metric = METRIC if headline else (
        f"{args.solver} iterations/sec + achieved HBM GB/s, {mname}"
        + (f" + {args.prec} {args.prec_type}" if args.prec != "none" else "") + f", k={k} RHS")
    out = {
        "metric": metric, "value": value, "unit": "iterations/s", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / steps, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": (f"{mname} from file, " if args.matrix_file else "synthetic (Galeri " + args.matrix + ", ")
                + "Xexact = Epetra MINSTD stream seed 1, B = A*Xexact)",
        "config": {"workload": wl, "n_global": n, "nnz": nnz_total, "k": k,
                   "num_blocks": nb, "parallelism": f"row1d{world}"},
    }
    if steps != args.steps:
        out["steps_requested"] = args.steps
    # host-side phases only: the SpMM / ortho / comm phases are asynchronous device work whose
    # host timers read ~0 unless "Verbosity" synchronises them; their device times are in
    # "kernels" (HIP events on the library's stream)
    out["solver_timers_s"] = {key: timers[key] for key in ("total", "lsqr", "setup")}
    out["rccl"] = rccl_info()
    comm_cls = ("halo", "allreduce")
    if kstats:
        # The metric's "achieved HBM GB/s": the algorithmic bytes the kernels that ran move
        # (per-class byte counts tallied by the library), summed over the
        # profiled solve (same iterations as the timed one) / the timed solve's wall time.
        alg = sum(v["bytes"] for kn, v in kstats.items() if kn not in comm_cls)
        if world > 1:
            t = torch.tensor([alg], dtype=torch.float64)
            dist.all_reduce(t)
            alg = float(t.item())
        gbps = alg / elapsed / 1e9 / world
        out["hbm"] = {"achieved_GBps_per_gpu": gbps, "frac_of_peak": gbps / HBM_PEAK_GBPS,
                      "algorithmic_bytes_per_iteration": alg / steps,
                      "source": "per-kernel algorithmic bytes of the kernels that ran / timed wall time"}
        dom = max((kn for kn in kstats if kn not in comm_cls), key=lambda s: kstats[s]["ms"])
        st = kstats[dom]
        per_launch_bytes = st["bytes"] / st["launches"]
        per_launch_s = st["ms"] / 1e3 / st["launches"]
        ach = per_launch_bytes / per_launch_s / 1e9
        ratio = pmc_ratio(dom, world) if headline else None
        out["roofline"] = {"kernel": dom, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                           "frac": ach / HBM_PEAK_GBPS,
                           "traffic": None if ratio is None else ratio * per_launch_bytes,
                           "traffic_ratio_pmc": ratio,
                           "bytes_per_launch": per_launch_bytes, "mean_launch_us": per_launch_s * 1e6}
        out["kernels"] = {kname: dict(ms=v["ms"], launches=v["launches"],
                                      GBps=v["bytes"] / (v["ms"] / 1e3) / 1e9 if v["ms"] > 0 else None)
                          for kname, v in kstats.items()}
    if kstats and "spmm" in kstats and world == 1:
        # SURVEY 8(d) / north star "fp64 CSR SpMV x 8": the default SpMM kernel on the bytes it
        # moves (its format's fixed bytes + X + Y, tallied per launch by the library), with the
        # PMC traffic ratio of the committed profile, and the CSR kernels of the same operator
        # timed beside it on the CSR's own bytes (12 nnz + 4 (N + 1) + 16 N k)
        st = kstats["spmm"]
        b, t = st["bytes"] / st["launches"], st["ms"] / 1e3 / st["launches"]
        ratio = pmc_ratio("spmm", world) if headline else None
        out["roofline_spmm"] = {"kernel": A.spmm_kernel(), "bound": "hbm", "achieved": b / t / 1e9,
                                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": b / t / 1e9 / HBM_PEAK_GBPS,
                                "bytes_per_launch": b, "mean_launch_us": t * 1e6,
                                "traffic": None if ratio is None else ratio * b, "traffic_ratio_pmc": ratio}
        if args.csr_spmm and not args.matrix_file:
            out["roofline_spmm"]["csr_forms"] = csr_spmm_forms(ta, comm, args, n, k, nnz_total, call)
    if headline:
        # SURVEY.md 8(d)'s model of the REFERENCE algorithm's traffic (column-by-column
        # findBasis, unfused updates) over the same wall time: a reference-equivalent rate,
        # not bytes this implementation moved (it can exceed the HBM peak).
        out["reference_equivalent"] = {"bytes_per_iteration": model_bytes / steps,
                                       "GBps_per_gpu": model_bytes / elapsed / 1e9 / world}
    if world > 1:
        mine = {"rank": rank, "device": local, "rows": A.n_local, "first_row": A.first, "nnz": A.nnz_local,
                "n_remote": A.n_remote, "n_export": A.n_export,
                "halo_bytes_per_apply": 8 * k * (A.n_remote + A.n_export),
                "halo_ms": kstats.get("halo", {}).get("ms"), "halo_launches": kstats.get("halo", {}).get("launches"),
                "allreduce_ms": kstats.get("allreduce", {}).get("ms"),
                "allreduce_launches": kstats.get("allreduce", {}).get("launches")}
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        out["ranks"] = allr
    if rank == 0 and world == 1 and not args.no_cpu_baseline and headline:
        out["cpu_baseline"] = cpu_baseline(k, nb, args.cpu_nx, args.cpu_iters if args.cpu_iters else nb)
        if not args.no_cpu_one_core:
            # the baseline also at 1 core -- one whole restart cycle of the
            # same solver at 128^3 (1/8 of the rows, about 20 s on one core), scaled by rows
            out["cpu_baseline"]["one_core"] = cpu_baseline_subprocess(1, k, nb, 128, nb)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
