"""ctypes binding of libmigmres.so (the C ABI declared in include/migmres.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C trilinos_amd/csrc``).  There is no fallback: if the library is missing
or fails to load, importing this module raises.
"""

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmigmres.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build the HIP extension first "
        "(python -c 'import __graft_entry__ as g; g.build()' or make -C trilinos_amd/csrc)")

lib = C.CDLL(LIB_PATH, mode=C.RTLD_LOCAL)

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_longlong
f64 = C.c_double
P = C.POINTER

# setUserConvStatusTest callback: (user, iters, nrhs, scaled residual norms) -> passed
STATUS_FN = C.CFUNCTYPE(i32, vp, i32, i32, P(f64))
APPLY_FN = C.CFUNCTYPE(i32, vp, vp, vp)

# name: (argtypes)
_SIGS = {
    "migmres_abi_version": [],
    "migmres_comm_unique_id": [C.c_char_p],
    "migmres_rccl_version": [P(i32)],
    "migmres_ctx_create": [i32, i32, i32, C.c_char_p, P(vp)],
    "migmres_ctx_destroy": [vp],
    "migmres_ctx_sync": [vp],
    "migmres_ctx_rank": [vp, P(i32), P(i32)],
    "migmres_ctx_sum_all": [vp, P(f64), P(f64), i32],
    "migmres_ctx_profile": [vp, i32],
    "migmres_ctx_profile_read": [vp, P(f64), P(f64), P(i64), i32],
    "migmres_map_uniform": [i64, i32, i32, P(i64), P(i32)],
    "migmres_plan_colmap": [i64, i32, i64, i32, P(i64), P(i64), P(i64), P(i32)],
    "migmres_plan_remotes": [i64, i32, i64, i32, P(i64), i32, P(i32), P(i32), P(i64), P(i32), P(i32)],
    "migmres_plan_local_crs": [i64, i32, P(i64), P(i64), P(f64), P(i64), i32, P(i32), P(f64)],
    "migmres_plan_pairs": [i32, P(i64), P(i32), P(i32), P(i32), P(C.c_uint16), P(i64), P(i32)],
    "migmres_plan_pair_templates": [i32, P(i64), P(i32), P(f64), P(C.c_uint8), P(i32), P(f64), P(i32), P(i32),
                                    P(i32), P(i32)],
    "migmres_crs_create": [vp, i64, i64, i32, P(i64), P(i64), P(f64), P(vp)],
    "migmres_crs_create_device": [vp, i64, i64, i32, vp, vp, vp, P(vp)],
    "migmres_crs_create_galeri": [vp, C.c_char_p, i32, i32, i32, P(vp)],
    "migmres_crs_destroy": [vp],
    "migmres_matrix_file_info": [C.c_char_p, P(i64), P(i64), P(i32)],
    "migmres_matrix_file_rows": [C.c_char_p, i64, i32, P(i64), P(i64), P(f64), P(i64)],
    "migmres_crs_read_file": [vp, C.c_char_p, P(vp)],
    "migmres_crs_info": [vp, P(i64), P(i64), P(i32), P(i32), P(i64), P(i32), P(i32)],
    "migmres_crs_colmap": [vp, P(i64)],
    "migmres_crs_import_plan": [vp, P(i32), P(i32), P(i32), P(i32)],
    "migmres_crs_apply": [vp, vp, vp, f64, f64],
    "migmres_crs_apply_mode": [vp, vp, vp, i32, f64, f64],
    "migmres_crs_spmm_kernel": [vp, P(i32)],
    "migmres_mv_create": [vp, i64, i32, i32, P(vp)],
    "migmres_mv_view": [vp, P(i32), i32, P(vp)],
    "migmres_mv_view_range": [vp, i32, i32, P(vp)],
    "migmres_mv_destroy": [vp],
    "migmres_mv_shape": [vp, P(i64), P(i32), P(i32), P(i32)],
    "migmres_mv_upload": [vp, P(f64), i64],
    "migmres_mv_download": [vp, P(f64), i64],
    "migmres_mv_times_mat_add_mv": [f64, vp, P(f64), i32, f64, vp],
    "migmres_mv_add_mv": [f64, vp, f64, vp, vp],
    "migmres_mv_scale": [vp, f64],
    "migmres_mv_scale_vec": [vp, P(f64)],
    "migmres_mv_trans_mv": [f64, vp, vp, P(f64), i32],
    "migmres_mv_dot": [vp, vp, P(f64)],
    "migmres_mv_norm": [vp, P(f64), i32],
    "migmres_mv_init": [vp, f64],
    "migmres_mv_random": [vp, P(C.c_uint)],
    "migmres_mv_assign": [vp, vp],
    "migmres_mv_set_block": [vp, P(i32), i32, vp],
    "migmres_icgs_project_normalize": [vp, vp, P(f64), i32, P(f64), i32, P(i32)],
    "migmres_icgs_normalize": [vp, P(f64), i32, P(i32)],
    "migmres_dgks_project_normalize": [vp, vp, P(f64), i32, P(f64), i32, P(i32)],
    "migmres_dgks_normalize": [vp, P(f64), i32, P(i32)],
    "migmres_plan_galeri": [C.c_char_p, i32, i32, i32, i64, i32, P(i64), P(i64), P(f64), P(i64)],
    "migmres_jacobi_create": [vp, i32, f64, P(vp)],
    "migmres_prec_destroy": [vp],
    "migmres_prec_apply": [vp, vp, vp],
    "migmres_prec_diagonal": [vp, P(f64)],
    "migmres_chebyshev_params_default": [vp],
    "migmres_relaxation_params_default": [vp],
    "migmres_relaxation_create": [vp, vp, P(vp)],
    "migmres_crs_format_digest": [vp, P(C.c_ulonglong), i32, P(i32)],
    "migmres_chebyshev_create": [vp, vp, P(vp)],
    "migmres_chebyshev_lambdas": [vp, P(f64), P(f64), P(f64)],
    "migmres_solver_create": [vp, P(vp)],
    "migmres_solver_create_named": [vp, C.c_char_p, P(vp)],
    "migmres_solver_set_prec": [vp, i32, vp],
    "migmres_solver_destroy": [vp],
    "migmres_solver_set_int": [vp, C.c_char_p, i64],
    "migmres_solver_set_double": [vp, C.c_char_p, f64],
    "migmres_solver_set_string": [vp, C.c_char_p, C.c_char_p],
    "migmres_solver_get_int": [vp, C.c_char_p, P(i64)],
    "migmres_solver_get_double": [vp, C.c_char_p, P(f64)],
    "migmres_solver_get_string": [vp, C.c_char_p, C.c_char_p, i32],
    "migmres_solver_valid_parameters": [vp, C.c_char_p, i32, P(i32)],
    "migmres_solver_current_parameters": [vp, C.c_char_p, i32, P(i32)],
    "migmres_solver_reset": [vp, i32],
    "migmres_solver_set_user_conv_test": [vp, STATUS_FN, vp, i32],
    "migmres_solver_solve": [vp, vp, vp, vp, P(i32)],
    "migmres_solver_solve_op": [vp, vp, vp, vp, P(i32)],
    "migmres_solver_set_prec_op": [vp, i32, vp],
    "migmres_op_create": [vp, C.c_longlong, i32, APPLY_FN, vp, P(vp)],
    "migmres_op_from_crs": [vp, P(vp)],
    "migmres_op_apply": [vp, vp, vp],
    "migmres_op_destroy": [vp],
    "migmres_solver_num_iters": [vp, P(i32)],
    "migmres_solver_achieved_tol": [vp, P(f64)],
    "migmres_solver_loa_detected": [vp, P(i32)],
    "migmres_solver_history": [vp, P(f64), P(i32), P(i32)],
    "migmres_solver_counters": [vp, P(i64), i32],
    "migmres_solver_timers": [vp, P(f64), i32],
}

for _name, _args in _SIGS.items():
    _fn = getattr(lib, _name)
    _fn.argtypes = _args
    _fn.restype = i32
lib.migmres_last_error.argtypes = []
lib.migmres_last_error.restype = C.c_char_p
lib.migmres_kernel_class_name.argtypes = [i32]
lib.migmres_kernel_class_name.restype = C.c_char_p

EXPORTED = sorted(list(_SIGS) + ["migmres_last_error", "migmres_kernel_class_name"])


class MigmresError(RuntimeError):
    """Raised for a nonzero return code (EpetraMultiVecFailure / EpetraOpFailure analogue,
    belos/epetra/src/BelosEpetraAdapter.hpp:97-108)."""

    def __init__(self, fn, code):
        msg = lib.migmres_last_error().decode(errors="replace")
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


def call(name, *args):
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise MigmresError(name, rc)
    return rc


def rccl_info():
    """The RCCL this library is bound to: {"version": "2.27.7", "code": 22707, "library": path}.
    Which librccl.so the process maps depends on import order (torch bundles its own), so
    the path is read from /proc/self/maps."""
    v = i32()
    call("migmres_rccl_version", C.byref(v))
    path = None
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "librccl" in line:
                    path = line.split()[-1]
                    break
    except OSError:
        pass
    c = v.value
    return {"version": f"{c // 10000}.{c // 100 % 100}.{c % 100}", "code": c, "library": path}


def dptr(a):
    return a.ctypes.data_as(P(f64))


def lptr(a):
    return a.ctypes.data_as(P(i64))


def iptr(a):
    return a.ctypes.data_as(P(i32))
