"""Distributed linear algebra objects over the C ABI (the Epetra/Tpetra shape).

  Comm          Epetra_Comm / Teuchos::Comm: one process per GPU, RCCL underneath
  uniform_map   Epetra_BlockMap::ConstructAutoUniform (epetra/src/Epetra_BlockMap.cpp:60-107)
  CrsMatrix     Epetra_CrsMatrix after FillComplete (column map, import plan, SortEntries)
                + Epetra_Operator::Apply / Tpetra::Operator::apply
  MultiVector   Epetra_MultiVector: column-major device block, with views

All data lives on the GPU; host arrays only cross at construction/upload/download.
"""

import ctypes as C
import os

import numpy as np

from ._lib import APPLY_FN, call, dptr, iptr, lptr, lib, MigmresError  # noqa: F401

TWO_NORM, ONE_NORM, INF_NORM = 1, 0, 2


def uniform_map(n_global, nranks, rank):
    """(first_gid, n_local) of `rank` in Epetra's uniform linear map."""
    first, n = C.c_longlong(), C.c_int()
    call("migmres_map_uniform", n_global, nranks, rank, C.byref(first), C.byref(n))
    return first.value, n.value


class Comm:
    """Device context: one GPU, one HIP stream and (for nranks > 1) an RCCL communicator.

    For multi-GPU runs create it on every rank with the same 128-byte unique id, e.g.
    ``Comm.from_torch_distributed(device)`` which broadcasts the id over torch.distributed.
    """

    def __init__(self, device=0, rank=0, nranks=1, unique_id=None):
        h = C.c_void_p()
        uid = None if unique_id is None else C.c_char_p(bytes(unique_id))
        call("migmres_ctx_create", device, rank, nranks, uid, C.byref(h))
        self.h = h
        self.rank, self.nranks, self.device = rank, nranks, device

    @staticmethod
    def unique_id():
        buf = C.create_string_buffer(128)
        call("migmres_comm_unique_id", buf)
        return buf.raw

    @classmethod
    def from_torch_distributed(cls, device):
        import torch
        import torch.distributed as dist
        rank, world = dist.get_rank(), dist.get_world_size()
        if world == 1:
            return cls(device, 0, 1)
        t = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            t[:] = torch.frombuffer(bytearray(cls.unique_id()), dtype=torch.uint8)
        dist.broadcast(t, 0)
        return cls(device, rank, world, bytes(t.numpy().tobytes()))

    def sync(self):
        call("migmres_ctx_sync", self.h)

    def sum_all(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = np.empty_like(x)
        call("migmres_ctx_sum_all", self.h, dptr(x), dptr(out), x.size)
        return out

    def close(self):
        if self.h:
            call("migmres_ctx_destroy", self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def matrix_file_rows(path, first=0, n_local=None):
    """Host-only read of rows [first, first + n_local) of a MatrixMarket / Harwell-Boeing file
    (migmres_matrix_file_rows): (n_global, rowptr, global columns, values), each row's entries
    in insertion order, duplicates summed."""
    ng, nnz_f, sym = C.c_longlong(), C.c_longlong(), C.c_int()
    call("migmres_matrix_file_info", os.fsencode(path), C.byref(ng), C.byref(nnz_f), C.byref(sym))
    n_local = ng.value - first if n_local is None else n_local
    nnz = C.c_longlong()
    call("migmres_matrix_file_rows", os.fsencode(path), first, n_local, None, None, None, C.byref(nnz))
    rp = np.empty(n_local + 1, dtype=np.int64)
    gc = np.empty(max(nnz.value, 1), dtype=np.int64)
    vv = np.empty(max(nnz.value, 1), dtype=np.float64)
    call("migmres_matrix_file_rows", os.fsencode(path), first, n_local, lptr(rp), lptr(gc), dptr(vv), C.byref(nnz))
    return ng.value, rp, gc[:nnz.value], vv[:nnz.value]


def galeri_rows(kind, nx, ny, nz, first, n_local):
    """Host-only generator rows [first, first + n_local) (migmres_plan_galeri): rowptr, GLOBAL
    columns in insertion order, values -- the rows CrsMatrix.galeri builds on each rank."""
    nnz = C.c_longlong()
    call("migmres_plan_galeri", kind.encode(), nx, ny, nz, first, n_local, None, None, None, C.byref(nnz))
    rp = np.empty(n_local + 1, dtype=np.int64)
    gc = np.empty(max(nnz.value, 1), dtype=np.int64)
    vv = np.empty(max(nnz.value, 1), dtype=np.float64)
    call("migmres_plan_galeri", kind.encode(), nx, ny, nz, first, n_local, lptr(rp), lptr(gc), dptr(vv),
         C.byref(nnz))
    return rp, gc[:nnz.value], vv[:nnz.value]


class CrsMatrix:
    """Row-distributed CSR operator.  `rowptr`/`gcols`/`vals` are this rank's rows
    (uniform map) with GLOBAL column ids in insertion order; the library builds the
    column map, local ids and import plan exactly as Epetra's FillComplete does."""

    def __init__(self, comm, n_global, rowptr=None, gcols=None, vals=None, _handle=None):
        self.comm = comm
        if _handle is None:
            first, n_local = uniform_map(n_global, comm.nranks, comm.rank)
            rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
            gcols = np.ascontiguousarray(gcols, dtype=np.int64)
            vals = np.ascontiguousarray(vals, dtype=np.float64)
            if rowptr.size != n_local + 1:
                raise ValueError(f"rowptr must have n_local+1 = {n_local + 1} entries")
            h = C.c_void_p()
            call("migmres_crs_create", comm.h, n_global, first, n_local, lptr(rowptr), lptr(gcols),
                 dptr(vals), C.byref(h))
            _handle = h
        self.h = _handle
        ng, first, nl, nc, nnz, nr, ne = (C.c_longlong(), C.c_longlong(), C.c_int(), C.c_int(),
                                          C.c_longlong(), C.c_int(), C.c_int())
        call("migmres_crs_info", self.h, C.byref(ng), C.byref(first), C.byref(nl), C.byref(nc),
             C.byref(nnz), C.byref(nr), C.byref(ne))
        self.n_global, self.first, self.n_local = ng.value, first.value, nl.value
        self.n_cols, self.nnz_local = nc.value, nnz.value
        self.n_remote, self.n_export = nr.value, ne.value

    @classmethod
    def from_device(cls, comm, n_global, rowptr, gcols, vals):
        """The operator from a CSR already on the GPU (migmres_crs_create_device): FillComplete's
        column map, local ids and sorted rows are built there.  rowptr / gcols: int64 and vals:
        float64 torch tensors on the context's device (this rank's rows, global column ids)."""
        import torch
        first, n_local = uniform_map(n_global, comm.nranks, comm.rank)
        for t, dt in ((rowptr, torch.int64), (gcols, torch.int64), (vals, torch.float64)):
            if t.dtype != dt or not t.is_cuda or not t.is_contiguous():
                raise ValueError("rowptr/gcols int64 and vals float64 contiguous GPU tensors expected")
        if rowptr.numel() != n_local + 1:
            raise ValueError(f"rowptr must have n_local+1 = {n_local + 1} entries")
        torch.cuda.synchronize(rowptr.device)
        h = C.c_void_p()
        call("migmres_crs_create_device", comm.h, n_global, first, n_local, C.c_void_p(rowptr.data_ptr()),
             C.c_void_p(gcols.data_ptr()), C.c_void_p(vals.data_ptr()), C.byref(h))
        return cls(comm, n_global, _handle=h)

    @classmethod
    def galeri(cls, comm, kind, nx, ny, nz=1):
        """Galeri::CreateCrsMatrix("Laplace2D"/"Laplace3D"/"Brick3D") on the uniform "Linear"
        map, generated natively on each rank; "FlanProxy" is the synthetic stand-in of config
        4's Flan_1565 (3 nx ny nz rows, include/migmres.h)."""
        h = C.c_void_p()
        call("migmres_crs_create_galeri", comm.h, kind.encode(), nx, ny, nz, C.byref(h))
        n = nx * ny * (nz if kind in ("Laplace3D", "Brick3D") else 3 * nz if kind == "FlanProxy" else 1)
        return cls(comm, n, _handle=h)

    @classmethod
    def read_file(cls, comm, path):
        """MatrixMarket / Harwell-Boeing file -> distributed operator on the uniform row map
        (Tpetra::MatrixMarket::Reader::readSparseFile; Trilinos_Util_read_hb as used by
        Belos::Util::createEpetraProblem).  Parsed natively on every rank."""
        h = C.c_void_p()
        call("migmres_crs_read_file", comm.h, os.fsencode(path), C.byref(h))
        ng = C.c_longlong()
        call("migmres_matrix_file_info", os.fsencode(path), C.byref(ng), None, None)
        return cls(comm, ng.value, _handle=h)

    def spmm_kernel(self):
        """The SpMM kernel apply() runs: "csr", "pair", "sell", "tpl", "tpl3", "bsr3" or "march"
        (migmres_crs_spmm_kernel)."""
        v = C.c_int()
        call("migmres_crs_spmm_kernel", self.h, C.byref(v))
        return ("csr", "pair", "sell", "tpl", "tpl3", "bsr3", "march")[v.value]

    def format_digest(self):
        """64-bit digests of the SpMM format plans this operator holds
        (migmres_crs_format_digest): equal lists = identical plans."""
        need = C.c_int()
        call("migmres_crs_format_digest", self.h, None, 0, C.byref(need))
        out = (C.c_ulonglong * max(need.value, 1))()
        call("migmres_crs_format_digest", self.h, out, need.value, C.byref(need))
        return list(out)[:need.value]

    def colmap(self):
        out = np.empty(self.n_cols, dtype=np.int64)
        call("migmres_crs_colmap", self.h, lptr(out))
        return out

    def import_plan(self):
        el = np.empty(max(self.n_export, 1), dtype=np.int32)
        ep = np.empty_like(el)
        rl = np.empty(max(self.n_remote, 1), dtype=np.int32)
        rp = np.empty_like(rl)
        call("migmres_crs_import_plan", self.h, iptr(el), iptr(ep), iptr(rl), iptr(rp))
        return dict(export_lids=el[:self.n_export], export_pids=ep[:self.n_export],
                    remote_lids=rl[:self.n_remote], remote_pids=rp[:self.n_remote])

    NO_TRANS, TRANS, CONJ_TRANS = 0, 1, 2  # Teuchos::ETransp

    def apply(self, X, Y, alpha=1.0, beta=0.0, mode=0):
        """Y = alpha*op(A)*X + beta*Y, op(A) = A or A^T by `mode` (Tpetra::CrsMatrix::apply,
        Tpetra_CrsMatrix_def.hpp:5176-5208; with alpha=1, beta=0 this is
        Epetra_CrsMatrix::Multiply(TransA, X, Y), Epetra_CrsMatrix.cpp:3107-3285)."""
        if mode == self.NO_TRANS:
            call("migmres_crs_apply", self.h, X.h, Y.h, alpha, beta)
        else:
            call("migmres_crs_apply_mode", self.h, X.h, Y.h, int(mode), alpha, beta)

    def multiply(self, trans, X, Y):
        """Epetra_CrsMatrix::Multiply(TransA, X, Y)."""
        self.apply(X, Y, 1.0, 0.0, self.TRANS if trans else self.NO_TRANS)

    Apply = apply

    def row_map(self):
        return self.first, self.n_local

    def close(self):
        # a context already destroyed (garbage cycles finalise in any order) took the operator's
        # device memory with it: nothing left to free
        if self.h and self.comm.h:
            call("migmres_crs_destroy", self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Operator:
    """A user operator: the analogue of an Epetra_Operator / Tpetra::Operator subclass handed to
    Belos (BelosOperatorTraits.hpp:108-155), e.g. the Vector_Operator family of
    belos/epetra/test/BlockGmres/test_bl_gmres_diag.cpp.  `apply(X, Y)` is a Python function of
    two device MultiVectors (borrowed handles, valid during the call) that leaves Y = op(X) in the
    context's stream order -- any trilinos_amd call on the same Comm does, nested solves included.
    Usable as the solver's operator (LinearProblem(A=Operator, ...)) and as a preconditioner."""

    def __init__(self, comm, n_global, apply):
        self.comm, self.n_global = comm, n_global
        _, self.n_local = uniform_map(n_global, comm.nranks, comm.rank)
        self._apply = apply
        self.error = None
        self._cb = APPLY_FN(self._trampoline)
        h = C.c_void_p()
        call("migmres_op_create", comm.h, n_global, self.n_local, self._cb, None, C.byref(h))
        self.h = h

    def _trampoline(self, _user, xh, yh):
        try:
            X = MultiVector(self.comm, self.n_global, 0, _handle=C.c_void_p(xh), _borrowed=True)
            Y = MultiVector(self.comm, self.n_global, 0, _handle=C.c_void_p(yh), _borrowed=True)
            self._apply(X, Y)
            return 0
        except BaseException as e:  # reported by the failing library call (MIGMRES_EOP)
            self.error = e.with_traceback(None)  # no frame -> self reference cycle
            return 1

    def apply(self, X, Y):
        call("migmres_op_apply", self.h, X.h, Y.h)

    Apply = apply

    def close(self):
        if self.h and self.comm.h:
            call("migmres_op_destroy", self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiVector:
    """Epetra_MultiVector-like block of `ncols` columns over the uniform row map."""

    def __init__(self, comm, n_global, ncols, _handle=None, _parent=None, _borrowed=False):
        self.comm = comm
        self._parent = _parent  # keeps the parent alive for views
        self._borrowed = _borrowed  # a handle the library owns (user-operator callbacks)
        if _handle is None:
            _, n_local = uniform_map(n_global, comm.nranks, comm.rank)
            h = C.c_void_p()
            call("migmres_mv_create", comm.h, n_global, n_local, ncols, C.byref(h))
            _handle = h
        self.h = _handle
        ng, nl, nc, cs = C.c_longlong(), C.c_int(), C.c_int(), C.c_int()
        call("migmres_mv_shape", self.h, C.byref(ng), C.byref(nl), C.byref(nc), C.byref(cs))
        self.n_global, self.n_local, self.ncols = ng.value, nl.value, nc.value
        self.constant_stride = bool(cs.value)

    # -- views (CloneView / CloneViewNonConst) --------------------------------------
    def view(self, idx):
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        h = C.c_void_p()
        call("migmres_mv_view", self.h, iptr(idx), idx.size, C.byref(h))
        return MultiVector(self.comm, self.n_global, idx.size, _handle=h, _parent=self)

    def view_range(self, first, n):
        h = C.c_void_p()
        call("migmres_mv_view_range", self.h, first, n, C.byref(h))
        return MultiVector(self.comm, self.n_global, n, _handle=h, _parent=self)

    # -- host transfer ---------------------------------------------------------------
    def upload(self, host):
        host = np.asfortranarray(np.asarray(host, dtype=np.float64).reshape(self.n_local, self.ncols))
        call("migmres_mv_upload", self.h, dptr(host), max(self.n_local, 1))

    def download(self):
        out = np.empty((self.n_local, self.ncols), dtype=np.float64, order="F")
        call("migmres_mv_download", self.h, dptr(out), max(self.n_local, 1))
        return out

    def put_scalar(self, v):
        call("migmres_mv_init", self.h, float(v))

    def random(self, seed):
        s = C.c_uint(seed)
        call("migmres_mv_random", self.h, C.byref(s))
        return s.value

    def close(self):
        if self.h and not self._borrowed and self.comm.h:
            call("migmres_mv_destroy", self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
