"""CPU oracle for the Block GMRES hot path -- TEST INFRASTRUCTURE ONLY.

This package is a plain-numpy restatement of the reference algorithm (Trilinos
Epetra + Belos, snapshot under /root/reference) used exclusively as the checker:

* ``tests/`` compare the HIP path against it,
* ``__graft_entry__.smoke()`` checks one small solve against it,
* ``bench.py`` times it as the ``cpu_baseline`` leg (kind "port").

Nothing in ``trilinos_amd/`` imports it; the product path never routes through
here and has no CPU fallback.

Pinning status (see DESIGN.md "Oracle"): the reference cannot be built here
under the task rules (its build needs CMake-generated config headers and an
external BLAS), so the oracle is pinned by (a) the reference's own fixture
files (orsirr1.hb) and closed-form known answers from its unit tests, and
(b) outputs of the real reference recorded in SURVEY.md section 6 / BASELINE.md
(64^3 7-pt Laplacian, k=8, ICGS: 201 iterations, 268 Epetra_CrsMatrix::Multiply
calls, true residuals 3.5e-10 .. 9.9e-9; orsirr1.hb, k=1, DGKS, tol 1e-5:
209 iterations, residual 9.94786e-06).
"""

from . import epetra, belos  # noqa: F401
