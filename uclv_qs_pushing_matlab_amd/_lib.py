"""ctypes binding of libqsp_nmpc.so (the C ABI declared in include/qsp_nmpc.h).

The product path has no CPU fallback: if the HIP library is missing or cannot be
loaded, importing a solver raises.
"""
import ctypes as C
import os

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
# QSP_LIB_PATH: developer override (A/B runs of differently compiled libraries)
LIB_PATH = os.environ.get("QSP_LIB_PATH") or os.path.join(_PKG, "libqsp_nmpc.so")
MAX_CTRL = 64
ABI_VERSION = 4   # include/qsp_nmpc.h QSP_ABI_VERSION

_lib = None


class QspError(RuntimeError):
    pass


class Options(C.Structure):
    _fields_ = [
        ("struct_size", C.c_int32), ("N", C.c_int32), ("batch", C.c_int32), ("nlp_mode", C.c_int32), ("sqp_iters", C.c_int32),
        ("qp_iters", C.c_int32), ("stages_per_lane", C.c_int32), ("device", C.c_int32), ("cost_scale_Ts", C.c_int32),
        ("Ts", C.c_double), ("mu0", C.c_double), ("t_min", C.c_double), ("frac", C.c_double),
        ("sigma_min", C.c_double), ("mu_stop", C.c_double),
        ("tol_stat", C.c_double), ("tol_eq", C.c_double), ("tol_ineq", C.c_double), ("tol_comp", C.c_double),
        ("ls_alpha_min", C.c_double), ("ls_alpha_red", C.c_double), ("ls_eps", C.c_double),
        ("res_stop", C.c_double),
        ("qp_tol_stat", C.c_double), ("qp_tol_eq", C.c_double),
        ("stage0_s_bound", C.c_int32), ("qp_stall_iters", C.c_int32), ("qp_stall_alpha", C.c_double),
        ("qp_mu_max", C.c_double), ("factor_scan", C.c_int32),
    ]


class Shape(C.Structure):
    _fields_ = [
        ("n_ctrl", C.c_int32), ("struct_size", C.c_int32),
        ("ctrl", (C.c_double * 2) * MAX_CTRL),
        ("knots", C.c_double * (MAX_CTRL + 4)),
        ("b", C.c_double), ("c_ellipse", C.c_double), ("mu_sp", C.c_double), ("xwidth", C.c_double),
    ]

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        self.struct_size = C.sizeof(Shape)   # qsp_set_shapes checks the layout (ABI v2)


class ClosedLoopOpts(C.Structure):
    _fields_ = [("plant_delay", C.c_double), ("disturbance", C.c_int32), ("t_dist", C.c_int32),
                ("amplitude", C.c_void_p)]


class DeviceIO(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ("x0", "yref", "yref_e", "X_in", "U_in", "shape_id", "u0", "X_out", "U_out", "PI_out", "status",
                 "cost")] + [("controller", C.c_int32), ("pad_", C.c_int32), ("warm_valid", C.c_void_p),
                             ("PI_in", C.c_void_p)]


_P = C.c_void_p
_I = C.c_int32
_D = C.c_double

# name -> argtypes (all return int status unless listed in _VOID)
_SIGS = {
    "qsp_default_options": [C.POINTER(Options)],
    "qsp_create": [C.POINTER(Options), C.POINTER(_P)],
    "qsp_destroy": [_P],
    "qsp_version": [],
    "qsp_get_layout": [_P, C.POINTER(_I), C.POINTER(_I)],
    "qsp_get_factor_walk": [_P, C.POINTER(_I)],
    "qsp_shape_from_ply": [C.c_char_p, _I, _D, _D, _D, _D, C.POINTER(Shape)],
    "qsp_set_shapes": [_P, C.POINTER(Shape), _I],
    "qsp_set_shape_ids": [_P, _P],
    "qsp_set_cost_W": [_P, _P, _P],
    "qsp_set_constr_h": [_P, _P, _P],
    "qsp_set_ctrl_params": [_P, _D, _D, _D, _D, _D],
    "qsp_set_x0": [_P, _P],
    "qsp_set_yref": [_P, _P, _P],
    "qsp_set_init": [_P, _P, _P, _P],
    "qsp_solve": [_P],
    "qsp_get_u0": [_P, _P],
    "qsp_get_x": [_P, _P],
    "qsp_get_u": [_P, _P],
    "qsp_get_pi": [_P, _P],
    "qsp_get_cost": [_P, _P],
    "qsp_get_status": [_P, _P],
    "qsp_get_sqp_iter": [_P, _P],
    "qsp_get_qp_iter": [_P, _P],
    "qsp_get_qp_capped": [_P, _P],
    "qsp_get_qp_stalled": [_P, _P],
    "qsp_get_residuals": [_P, _P],
    "qsp_get_time_tot": [_P, C.POINTER(_D)],
    "qsp_get_dims": [_P, C.POINTER(_I), C.POINTER(_I)],
    "qsp_set_yref_stage": [_P, _I, _P],
    "qsp_set_yref_e": [_P, _P],
    "qsp_set_init_x": [_P, _P],
    "qsp_set_init_u": [_P, _P],
    "qsp_set_init_pi": [_P, _P],
    "qsp_set_timing": [_P, _I],
    "qsp_get_timings": [_P, C.POINTER(_D), C.POINTER(_D), C.POINTER(_D)],
    "qsp_set_reference_trajectory": [_P, _P, _I],
    "qsp_set_reference_trajectories": [_P, _P, _I],
    "qsp_gen_straight_lines": [_P, _P, _P, _D, _D, _I, C.POINTER(_I)],
    "qsp_get_reference_trajectories": [_P, _P],
    "qsp_controller_solve": [_P, _P, _P],
    "qsp_controller_reset": [_P],
    "qsp_closed_loop": [_P, _P, _P, _I, _P, _P, _P, _P],
    "qsp_closed_loop_ex": [_P, C.POINTER(ClosedLoopOpts), _P, _P, _I, _P, _P, _P, _P, _P],
    "qsp_set_delay_comp": [_P, _D],
    "qsp_get_delay_comp": [_P, C.POINTER(_I)],
    "qsp_delay_buffer_sim": [_P, _P, _P],
    "qsp_delay_buffer_push": [_P, _P],
    "qsp_reproject_contact": [_P, _I, _P, _P, _P, _P, _P],
    "qsp_solve_device": [_P, C.POINTER(DeviceIO), _P],
    "qsp_synchronize": [_P],
    "qsp_set_stream_parts": [_P, _I],
    "qsp_get_stream_parts": [_P, C.POINTER(_I)],
    "qsp_set_kernel_timing": [_P, _I],
    "qsp_get_kernel_times": [_P, C.POINTER(_D), C.POINTER(_I)],
    "qsp_eval_spline": [_P, _I, _P, _P, _P, _P, _P, _P],
    "qsp_eval_dynamics": [_P, _I, _P, _P, _P, _P, _P],
    "qsp_eval_rk4": [_P, _I, _P, _D, _P, _P, _P, _P, _P],
    "qsp_eval_vbound": [_P, _I, _P, _P, _P],
    "qsp_qp_solve": [_P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "qsp_last_error": [],
}
_VOID = {"qsp_default_options"}
EXPORTED = tuple(_SIGS)


def lib():
    """Load the HIP library (raises QspError if it is missing: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise QspError(f"HIP extension not built: {LIB_PATH} missing (run __graft_entry__.build())")
    # One HIP runtime per process: the PyTorch wheel bundles its own libamdhip64 (soname
    # libamdhip64.so.7, linked by its libs under the plain name).  Loading torch first lets
    # our NEEDED libamdhip64.so.7 bind to that copy; loading ours first would leave torch
    # initialising a second runtime, which then finds no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    L.qsp_version.restype = C.c_int
    if L.qsp_version() != ABI_VERSION:
        raise QspError(f"{LIB_PATH}: ABI version {L.qsp_version()}, this binding needs {ABI_VERSION} (rebuild)")
    for name, args in _SIGS.items():
        fn = getattr(L, name)
        fn.argtypes = args
        if name in _VOID:
            fn.restype = None
        elif name == "qsp_last_error":
            fn.restype = C.c_char_p
        else:
            fn.restype = C.c_int
    _lib = L
    return L


def check(rc, what=""):
    if rc != 0:
        msg = lib().qsp_last_error()
        raise QspError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(C.c_void_p)


def f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a


def i32(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.int32)
    if shape is not None:
        a = a.reshape(shape)
    return a
