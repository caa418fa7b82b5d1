"""A compiled C/C++ consumer of the drop-in boundary.

tests/abi_consumer/mvop_tester.cpp includes only include/migmres.h and the traits adapter
include/migmres_belos.hpp, is built with plain g++ (no HIP
headers: the ABI is plain C) and linked to the in-tree libmigmres.so.  On the GPU it runs the
Belos contract suite -- TestMultiVecTraits / TestOperatorTraits
(belos/src/BelosMVOPTester.hpp:84-1430, 1452-1600), driven as
belos/epetra/test/MVOPTester/cxx_main.cpp:46-103 drives it -- and one Block GMRES solve.
"""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIR = os.path.join(ROOT, "tests", "abi_consumer")
BIN = os.path.join(DIR, "mvop_tester")


def test_header_is_plain_c():
    """migmres.h compiles as C (C89 declarations, no C++ or HIP types)."""
    subprocess.check_call(["gcc", "-fsyntax-only", "-std=c99", "-Wall", "-Werror", "-x", "c",
                           os.path.join(ROOT, "include", "migmres.h")])


def test_consumer_builds_against_the_library():
    subprocess.check_call(["make", "-s", "-C", DIR])
    assert os.path.exists(BIN)
    out = subprocess.check_output(["ldd", BIN]).decode()
    assert os.path.join("trilinos_amd", "libmigmres.so") in out.replace("/../..", "").replace("//", "/") or \
        "libmigmres.so =>" in out


@pytest.mark.gpu
def test_mvop_tester_and_solve_on_gpu():
    assert os.path.exists(BIN), "build first: make -C tests/abi_consumer (done by __graft_entry__.build())"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "MVOPTESTER PASSED" in r.stdout and "SOLVE PASSED" in r.stdout


EX = os.path.join(DIR, "block_gmres_galeri_ex")


@pytest.mark.gpu
def test_galeri_example_driver_reproduces_reference_run():
    """tests/abi_consumer/block_gmres_galeri_ex.cpp -- the reference's
    BlockGmresEpetraGaleriEx.cpp flow written against include/migmres.h in C++ -- run with the
    recorded reference run's options (--nx=64 --num-rhs=8 --block-size=8
    --ortho=ICGS --tol=1e-8 --max-subspace=50 --max-restarts=50): the same 201 iterations,
    268 operator applications (267 in the solve + B = A Xexact), 4 restarts, 61 explicit
    residual checks and true residuals 3.5e-10 .. 9.9e-9 as the reference printed."""
    assert os.path.exists(EX), "build first: make -C tests/abi_consumer (done by __graft_entry__.build())"
    r = subprocess.run([EX, "--nx=64", "--num-rhs=8", "--block-size=8", "--ortho=ICGS", "--tol=1e-8",
                        "--max-subspace=50", "--max-restarts=50"], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "End Result: TEST PASSED" in r.stdout
    assert "Number of iterations: 201" in r.stdout
    assert "Operator applications: 267" in r.stdout
    assert "Restarts: 4" in r.stdout and "Explicit residual checks: 61" in r.stdout
    assert "True relative residuals: min 3.5e-10 max 9.9e-09" in r.stdout
