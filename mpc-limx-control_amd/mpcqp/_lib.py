"""ctypes binding of libmpcqp.so (include/mpcqp.h).

The library is the product: HIP kernels for gfx950 behind a C ABI.  There is no Python or
CPU fallback -- if the library is missing, importing the engine raises.
"""
from __future__ import annotations

import ctypes as C
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPCQP_LIB") or os.path.join(os.path.dirname(_PKG), "lib",
                                                       "libmpcqp.so")

MPCQP_OK = 0
STATUS = {0: "OK", 1: "BAD_DIMS", 2: "INFEASIBLE", 3: "ITER_LIMIT", 4: "NOT_PD", 5: "DEVICE",
          6: "BAD_ARG", 7: "NO_DEVICE"}
MPCQP_INFTY = 1e20
MODEL_SRBM, MODEL_LITERAL, MODEL_DENSE = 0, 1, 2
CONS_BOX, CONS_FRICTION = 0, 1
A_ROWMAJOR, A_COLMAJOR = 0, 1

EXPORTS = [
    "mpcqp_discretize", "mpcqp_discretize_quadrature", "mpcqp_build_qp", "mpcqp_solve_dense", "mpcqp_plant_step",
    "mpcqp_ctx_create", "mpcqp_ctx_destroy", "mpcqp_set_stream", "mpcqp_sync",
    "mpcqp_batch_condense", "mpcqp_batch_solve_qp", "mpcqp_batch_solve",
    "mpcqp_ctx_fast_path", "mpcqp_ctx_one_wave_nf", "mpcqp_ctx_overflow_kernel", "mpcqp_ctx_crash_params", "mpcqp_batch_discretize", "mpcqp_batch_condense_solve",
    "mpcqp_debug_phase_cycles", "mpcqp_batch_solve_host",
    "mpcqp_count_solver_flops", "mpcqp_solver_flops",
    "mpcqp_batch_select_min", "mpcqp_batch_select_record", "mpcqp_reduce_records",
    "mpcqp_batch_solve_select",
    "mpcqp_enable_timing", "mpcqp_last_kernel_ms", "mpcqp_kernel_ms_sum",
    "mpcqp_batch_solve_gait", "mpcqp_batch_select_state", "mpcqp_batch_plant_srbm",
    "mpcqp_rollout", "mpcqp_fk_feet", "mpcqp_kf_update", "mpcqp_ctx_reserve",
    "mpcqp_ctx_fk_feet_host", "mpcqp_set_warm_start",
    "mpcqp_shard", "mpcqp_group_create", "mpcqp_group_unique_id", "mpcqp_group_create_rank",
    "mpcqp_group_destroy", "mpcqp_group_info", "mpcqp_group_ctx", "mpcqp_group_solve_select",
    "mpcqp_group_wait", "mpcqp_group_sync", "mpcqp_group_solve_select_host",
    "mpcqp_group_wait_stream", "mpcqp_group_failed",
    "mpcqp_host_register", "mpcqp_host_unregister", "mpcqp_host_alloc", "mpcqp_host_free",
    "mpcqp_status_string", "mpcqp_device_count", "mpcqp_build_id",
]


class MpcqpError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__(f"{fn} failed: {STATUS.get(code, code)} ({code})")
        self.code = code


class Model(C.Structure):
    """mirror of struct mpcqp_model"""
    _fields_ = [("nx", C.c_int), ("nu", C.c_int), ("N", C.c_int), ("model", C.c_int),
                ("constraints", C.c_int), ("Ts", C.c_double), ("mass", C.c_double),
                ("mu", C.c_double), ("Ib", C.c_double * 9), ("fz_min", C.c_double),
                ("fz_max", C.c_double), ("fxy_max", C.c_double), ("u_min", C.c_double),
                ("u_max", C.c_double), ("Q", C.c_void_p), ("R", C.c_void_p),
                ("P", C.c_void_p), ("max_iter", C.c_int), ("max_free", C.c_int)]


_lib = None


def lib():
    """Load libmpcqp.so; raise loudly if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libmpcqp.so not built ({LIB_PATH}); run `make -C mpc-limx-control_amd` "
                          "or __graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
    vp, dp, ip, i = C.c_void_p, C.c_void_p, C.c_void_p, C.c_int
    d = C.c_double
    L.mpcqp_discretize.argtypes = [i, i, d, vp, vp, vp, vp]
    L.mpcqp_discretize_quadrature.argtypes = [i, i, d, vp, vp, vp, vp]
    L.mpcqp_build_qp.argtypes = [i, i, i] + [vp] * 7 + [d, d] + [vp] * 11
    L.mpcqp_solve_dense.argtypes = [i, i, vp, vp, vp, i, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mpcqp_plant_step.argtypes = [i, i, vp, vp, vp, vp]
    L.mpcqp_ctx_create.argtypes = [C.POINTER(Model), i, C.POINTER(vp)]
    L.mpcqp_ctx_destroy.argtypes = [vp]
    L.mpcqp_set_stream.argtypes = [vp, vp]
    L.mpcqp_sync.argtypes = [vp]
    L.mpcqp_batch_condense.argtypes = [vp, i, vp, vp, vp, vp, vp]
    L.mpcqp_batch_solve_qp.argtypes = [vp, i, vp, vp, vp, vp, vp, vp, vp]
    L.mpcqp_batch_solve.argtypes = [vp, i, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mpcqp_ctx_fast_path.argtypes = [vp]
    for name, at in (("mpcqp_ctx_one_wave_nf", [vp]), ("mpcqp_ctx_crash_params", [vp] + [vp] * 4),
                     ("mpcqp_ctx_overflow_kernel", [vp])):
        if hasattr(L, name):  # absent from A/B builds of older sources
            getattr(L, name).argtypes = at
    L.mpcqp_debug_phase_cycles.argtypes = [vp, vp, i]
    if hasattr(L, "mpcqp_count_solver_flops"):  # absent from A/B builds of older sources
        L.mpcqp_count_solver_flops.argtypes = [vp, i]
        L.mpcqp_solver_flops.argtypes = [vp, C.POINTER(C.c_int)]
        L.mpcqp_solver_flops.restype = C.c_double
    L.mpcqp_batch_solve_host.argtypes = [vp, i] + [vp] * 8
    L.mpcqp_batch_discretize.argtypes = [vp, i, vp, vp]
    L.mpcqp_batch_condense_solve.argtypes = [vp, i] + [vp] * 8
    L.mpcqp_batch_select_min.argtypes = [vp, i, vp, vp, C.c_int64, vp]
    L.mpcqp_batch_select_record.argtypes = [vp, i, vp, vp, vp, C.c_int64, vp]
    L.mpcqp_reduce_records.argtypes = [vp, i, vp, vp]
    if hasattr(L, "mpcqp_batch_solve_select"):  # absent from A/B builds of older sources
        L.mpcqp_batch_solve_select.argtypes = [vp, i] + [vp] * 8 + [C.c_int64, vp]
    L.mpcqp_batch_solve_gait.argtypes = [vp, i, i] + [vp] * 4 + [C.c_float, C.c_float] + [vp] * 4
    L.mpcqp_batch_select_state.argtypes = [vp, i, i] + [vp] * 6
    L.mpcqp_batch_plant_srbm.argtypes = [vp, i, i] + [vp] * 5
    L.mpcqp_rollout.argtypes = [vp, i, i, i] + [vp] * 4 + [C.c_float, C.c_float, vp, vp]
    L.mpcqp_fk_feet.argtypes = [vp, i, vp, vp, i, vp]
    L.mpcqp_ctx_fk_feet_host.argtypes = [vp, i, vp, vp, i, vp]
    L.mpcqp_ctx_reserve.argtypes = [vp, i]
    L.mpcqp_set_warm_start.argtypes = [vp, i]
    L.mpcqp_kf_update.argtypes = [vp, i, d] + [vp] * 7
    L.mpcqp_enable_timing.argtypes = [vp, i]
    L.mpcqp_last_kernel_ms.argtypes = [vp, i]
    L.mpcqp_last_kernel_ms.restype = C.c_double
    L.mpcqp_kernel_ms_sum.argtypes = [vp, i, C.POINTER(C.c_int)]
    L.mpcqp_kernel_ms_sum.restype = C.c_double
    if hasattr(L, "mpcqp_group_create"):  # absent from A/B builds of older sources
        L.mpcqp_shard.argtypes = [i, i, i, vp, vp]
        L.mpcqp_group_create.argtypes = [C.POINTER(Model), i, vp, C.POINTER(vp)]
        L.mpcqp_group_unique_id.argtypes = [vp]
        L.mpcqp_group_create_rank.argtypes = [C.POINTER(Model), i, i, i, vp, C.POINTER(vp)]
        L.mpcqp_group_destroy.argtypes = [vp]
        L.mpcqp_group_info.argtypes = [vp, vp, vp, vp]
        L.mpcqp_group_ctx.argtypes = [vp, i]
        L.mpcqp_group_ctx.restype = vp
        L.mpcqp_group_solve_select.argtypes = [vp] * 12
        L.mpcqp_group_wait.argtypes = [vp]
        L.mpcqp_group_sync.argtypes = [vp]
        L.mpcqp_group_solve_select_host.argtypes = [vp, i, i] + [vp] * 9
        L.mpcqp_group_wait_stream.argtypes = [vp, vp]
        L.mpcqp_group_failed.argtypes = [vp]
    if hasattr(L, "mpcqp_host_register"):  # absent from A/B builds of older sources
        L.mpcqp_host_register.argtypes = [vp, C.c_size_t]
        L.mpcqp_host_unregister.argtypes = [vp]
        L.mpcqp_host_alloc.argtypes = [C.c_size_t, vp]
        L.mpcqp_host_free.argtypes = [vp]
    L.mpcqp_status_string.argtypes = [i]
    L.mpcqp_status_string.restype = C.c_char_p
    L.mpcqp_build_id.argtypes = []
    L.mpcqp_build_id.restype = C.c_char_p
    L.mpcqp_device_count.argtypes = []
    _lib = L
    return L


def check(fn, code):
    if code != MPCQP_OK:
        raise MpcqpError(fn, code)
    return code
