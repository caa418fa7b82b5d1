"""The C-ABI library loads on a CPU-only host and exports every entry point that
include/migmres.h declares (no compute calls are made here)."""

import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "migmres.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(migmres_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    import trilinos_amd._lib as L
    declared = _declared()
    assert len(declared) > 40
    missing = [s for s in declared if not hasattr(L.lib, s)]
    assert not missing, missing
    # the Python binding covers every declared entry point
    assert sorted(set(L.EXPORTED)) == declared


def test_abi_version_and_errors():
    import trilinos_amd._lib as L
    assert L.lib.migmres_abi_version() == 1
    # a host-only call with bad arguments returns an error code and a message
    first, n = ctypes.c_longlong(), ctypes.c_int()
    rc = L.lib.migmres_map_uniform(10, 0, 0, ctypes.byref(first), ctypes.byref(n))
    assert rc != 0 and b"map" in L.lib.migmres_last_error()


def test_library_fails_loudly_without_so(tmp_path, monkeypatch):
    """The product path has no fallback: importing the binding without the .so raises."""
    import importlib.util
    import shutil
    pkg = tmp_path / "trilinos_amd"
    pkg.mkdir()
    shutil.copy(os.path.join(ROOT, "trilinos_amd", "_lib.py"), pkg / "_lib.py")
    spec = importlib.util.spec_from_file_location("ta_lib_nolib", pkg / "_lib.py")
    mod = importlib.util.module_from_spec(spec)
    try:
        spec.loader.exec_module(mod)
    except ImportError as e:
        assert "libmigmres.so is missing" in str(e)
    else:
        raise AssertionError("import succeeded without the library")
