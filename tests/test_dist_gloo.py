"""N > 1 logic on CPU with torch.distributed (gloo, world size 2 and 3).

Each rank builds its plan with the library's host plan code (the C ABI used by
crs_create: uniform map, Epetra column map, remote list, local CRS), runs the same
request protocol crs_create runs over RCCL (every rank sends each owner the GIDs it
needs, in its own order; owners answer in requester order) to get the export lists, then
performs the halo exchange the way crs_apply does (pack in the [neighbour][column][count]
layout, one message per neighbour, unpack to the ghost block) and the local CSR row sums.  The result must be bit-identical to the
oracle's emulation of Epetra_CrsMatrix::Multiply on the same partition, and the
distributed dot products (all-reduce of rank partials) must match.
"""

import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import epetra as oe


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from tests.test_plans import lib_plan, random_rows
        kind, dims, k = case
        nx, ny, nz = dims
        n = nx * ny * nz
        if kind == "Laplace3D":
            gen = lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m)  # noqa: E731
        elif kind == "Laplace2D":
            gen = lambda f, m: oe.laplace2d_rows(nx, ny, f, m)  # noqa: E731
        else:
            gen = lambda f, m: random_rows(n, f, m, 23)  # noqa: E731
        first, nloc = oe.uniform_map(n, world, rank)
        rp, gc, vv = gen(first, nloc)
        plan = lib_plan(n, world, rank, rp, gc, vv)

        # request protocol of crs_create: remote GIDs grouped by owner (already PID-sorted)
        rg, rpid = plan["remote_gids"], plan["remote_pids"]
        requests = [rg[rpid == p].tolist() for p in range(world)]
        allreq = [None] * world
        dist.all_gather_object(allreq, requests)
        export_lids, export_pids, send_nbrs = [], [], []
        for qq in range(world):
            if qq == rank:
                continue
            want = allreq[qq][rank]
            if want:
                send_nbrs.append((qq, len(export_lids), len(want)))
                export_lids += [g - first for g in want]
                export_pids += [qq] * len(want)
        # recv groups
        recv_nbrs, i = [], 0
        while i < len(rpid):
            j = i
            while j < len(rpid) and rpid[j] == rpid[i]:
                j += 1
            recv_nbrs.append((int(rpid[i]), i, j - i))
            i = j

        # global X (same on all ranks), local rows
        Xg, _ = oe.epetra_random_mv(5, n, k)
        Xloc = Xg[first:first + nloc]
        n_export, n_remote = len(export_lids), len(rg)
        # exchange layout of crs_apply: [neighbour][column][count], one message per neighbour
        send = np.zeros(max(n_export * k, 1))
        for (p, off, cnt) in send_nbrs:
            for c in range(k):
                send[off * k + c * cnt: off * k + (c + 1) * cnt] = Xloc[export_lids[off:off + cnt], c]
        recv = np.zeros(max(n_remote * k, 1))
        reqs = []
        for (p, off, cnt) in send_nbrs:
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(send[off * k:(off + cnt) * k])), p))
        bufs = []
        for (p, off, cnt) in recv_nbrs:
            b = torch.zeros(cnt * k, dtype=torch.float64)
            reqs.append(dist.irecv(b, p))
            bufs.append((off, cnt, b))
        for r in reqs:
            r.wait()
        for (off, cnt, b) in bufs:
            recv[off * k:(off + cnt) * k] = b.numpy()
        # unpack to the ghost block [k][n_remote]
        ghost = np.zeros((k, max(n_remote, 1)))
        for (p, off, cnt) in recv_nbrs:
            for c in range(k):
                ghost[c, off:off + cnt] = recv[off * k + c * cnt: off * k + (c + 1) * cnt]

        # X-space indices as crs_create builds them: owned -> row id, remote -> n_local + slot
        cm = plan["colmap"]
        xspace = np.full(cm.size, -1, dtype=np.int64)
        own = (cm >= first) & (cm < first + nloc)
        xspace[own] = cm[own] - first
        xspace[plan["remote_lids"]] = nloc + np.arange(n_remote)
        lc = xspace[plan["lcols"]]
        Xc = np.concatenate([Xloc, ghost[:, :n_remote].T], axis=0)
        Y = oe.csr_rowsum(np.asarray(rp, dtype=np.int64), lc, plan["lvals"], Xc)

        # distributed dot (MvDot): rank partial + all-reduce
        part = torch.from_numpy(np.einsum("ij,ij->j", Y, Y).copy())
        dist.all_reduce(part)
        q.put((rank, first, Y, part.numpy(), export_lids, export_pids))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put(("error", rank, traceback.format_exc() + repr(e)))


@pytest.mark.parametrize("world,case", [(2, ("Laplace3D", (10, 9, 8), 8)), (3, ("Laplace2D", (17, 13, 1), 3)),
                                        (2, ("random", (300, 1, 1), 2)), (3, ("Laplace3D", (6, 5, 7), 16))])
def test_distributed_spmv_and_dot(world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [r for r in res if r[0] == "error"]
    assert not errs, errs
    kind, dims, k = case
    nx, ny, nz = dims
    n = nx * ny * nz
    if kind == "Laplace3D":
        gen = lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m)  # noqa: E731
    elif kind == "Laplace2D":
        gen = lambda f, m: oe.laplace2d_rows(nx, ny, f, m)  # noqa: E731
    else:
        from tests.test_plans import random_rows
        gen = lambda f, m: random_rows(n, f, m, 23)  # noqa: E731
    D = oe.DistCrs(gen, n, world)
    Xg, _ = oe.epetra_random_mv(5, n, k)
    Yref = D.apply(Xg)
    res.sort(key=lambda r: r[0])
    Yall = np.zeros((n, k))
    for (rank, first, Y, dots, el, ep) in res:
        Yall[first:first + Y.shape[0]] = Y
        # export lists identical to the oracle's Epetra_Import restatement
        np.testing.assert_array_equal(np.asarray(el, dtype=np.int64), D.plans[rank]["export_lids"])
        np.testing.assert_array_equal(np.asarray(ep, dtype=np.int64), D.plans[rank]["export_pids"])
    assert np.array_equal(Yall, Yref)  # bit-exact distributed SpMV
    ref_dots = np.einsum("ij,ij->j", Yref, Yref)
    for r in res:
        np.testing.assert_allclose(r[3], ref_dots, rtol=1e-13)
