"""Regenerate the golden fixtures under tests/golden/ from the oracle.

The oracle itself is pinned to the reference (tests/test_oracle_pins.py); these files let
the GPU tests compare against full-size solves without re-running the slow CPU oracle on
the GPU box.  Run:  python tests/golden/make_fixtures.py
"""

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import belos as ob, epetra as oe  # noqa: E402

# Xexact seed of the reference example run: the third Epetra_MultiVector constructed in
# BlockGmresEpetraGaleriEx.cpp (B, X, Xexact), each consuming two glibc rand() calls
# (Epetra_Util() ctor, epetra/src/Epetra_Util.h:270; AllocateForCopy,
# epetra/src/Epetra_MultiVector.cpp:263-265) -> the 6th value of glibc's rand().
SEED_GALERI_EX = oe.glibc_rand(6)[5]

CASES = {
    # name: (kind, dims, k, seed, params)
    "laplace3d_64_k8_icgs_nb50": ("Laplace3D", (64, 64, 64), 8, SEED_GALERI_EX,
                                  {"Num Blocks": 50, "Block Size": 8, "Maximum Iterations": 64 ** 3 // 8 - 1,
                                   "Maximum Restarts": 50, "Convergence Tolerance": 1e-8,
                                   "Orthogonalization": "ICGS"}),
    "laplace2d_100_k1_icgs_nb50": ("Laplace2D", (100, 100, 1), 1, 1,
                                   {"Num Blocks": 50, "Block Size": 1, "Maximum Iterations": 9999,
                                    "Maximum Restarts": 50, "Convergence Tolerance": 1e-8,
                                    "Orthogonalization": "ICGS"}),
}


def problem(kind, dims, k, seed):
    nx, ny, nz = dims
    if kind == "Laplace3D":
        n = nx * ny * nz
        A = oe.DistCrs(lambda f, m: oe.laplace3d_rows(nx, ny, nz, f, m), n, 1)
    else:
        n = nx * ny
        A = oe.DistCrs(lambda f, m: oe.laplace2d_rows(nx, ny, f, m), n, 1)
    Xex, _ = oe.epetra_random_mv(seed, n, k)
    return A, A.apply(Xex)


ORSIRR1_SRC = "/root/reference/packages/belos/epetra/example/BlockGmres/orsirr1.hb"


def orsirr1_fixture():
    """orsirr1.hb (1030 x 1030, 6858 nnz; the matrix of belos/epetra/test/BlockGmres/
    test_bl_gmres_hb.cpp) as CSC arrays, so tests do not read /root/reference.  Data only:
    the Harwell-Boeing file's column pointers, row indices and values."""
    n, colptr, rowind, vals, sym = oe.read_hb(ORSIRR1_SRC)
    np.savez_compressed(os.path.join(HERE, "orsirr1.npz"), n=n, colptr=colptr, rowind=rowind, vals=vals,
                        symmetric=sym)
    print("orsirr1", n, rowind.size)


def main(names=None):
    if not names or "orsirr1" in names:
        orsirr1_fixture()
    for name, (kind, dims, k, seed, params) in CASES.items():
        if names and name not in names:
            continue
        A, B = problem(kind, dims, k, seed)
        res = ob.solve(A.apply, B, params)
        R = B - A.apply(res["X"])
        rel = np.linalg.norm(R, axis=0) / np.linalg.norm(B, axis=0)
        # the same solve with the oracle's inner products summed in reverse row order: how far
        # rounding alone moves the history (the GPU tests' bar beyond 1e-12, test_gpu_solver.py)
        with ob.summation_order("reversed"):
            rev = ob.solve(A.apply, B, params)
        assert rev["iterations"] == res["iterations"] and rev["history"].shape == res["history"].shape
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), history=res["history"], true_rel=rel,
                            history_reversed=rev["history"])
        meta = dict(kind=kind, dims=dims, k=k, seed=seed, params=params, iterations=res["iterations"],
                    converged=bool(res["converged"]), n_apply=res["n_apply"],
                    n_explicit=res["n_explicit"], restarts=res["restarts"],
                    blk_ortho_sing=res["blk_ortho_sing"], true_rel_min=float(rel.min()),
                    true_rel_max=float(rel.max()))
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(meta, f, indent=1)
        print(name, meta)


if __name__ == "__main__":
    main(sys.argv[1:])
