"""ctypes mirror of include/fddp_hip.h (structs, constants, prototypes).

Shared by the product binding (crocoddyl_amd._lib, libfddp_hip.so) and the
test harness binding of the CPU oracle (tests/oracle_lib.py, liboracle.so),
which exports the same functions with an ``oracle_`` prefix.
"""
import ctypes as C

ABI_VERSION = 3  # FDDP_ABI_VERSION of include/fddp_hip.h this binding was written against

FDDP_OK = 0
FDDP_ERR_INVALID_ARG = -1
FDDP_ERR_RUNTIME = -2
FDDP_ERR_UNSUPPORTED = -3
FDDP_ERR_NO_DEVICE = -4
FDDP_ERR_CALLBACK_ABORT = -5

STATUS_RUNNING, STATUS_CONVERGED, STATUS_REGMAX = 0, 1, 2

KNOT_LQR, KNOT_UNICYCLE, KNOT_EULER_DIFFLQR, KNOT_EULER_FREEFWD, KNOT_EULER_CONTACTFWD, KNOT_IMPULSEFWD = 1, 2, 3, 4, 5, 6
PARAM_HEADER = 4

Q_FX, Q_FU, Q_LXX, Q_LXU, Q_LUU, Q_LX, Q_LU, Q_XNEXT, Q_FS, Q_K, Q_KV = range(11)
Q_COST = 19
Q_VXX, Q_VX, Q_QXX, Q_QXU, Q_QUU, Q_QX, Q_QU = range(11, 18)
Q_QUU_INV = 18

SOLVER_FDDP, SOLVER_BOXFDDP = 0, 1


class Dims(C.Structure):
    _fields_ = [("nx", C.c_int32), ("ndx", C.c_int32), ("nu_max", C.c_int32), ("T", C.c_int32), ("B", C.c_int32)]


class KnotDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("nu", C.c_int32), ("param_offset", C.c_int64), ("param_stride", C.c_int64)]


class Params(C.Structure):
    _fields_ = [("th_acceptstep", C.c_double), ("th_stop", C.c_double), ("th_grad", C.c_double),
                ("th_stepdec", C.c_double), ("th_stepinc", C.c_double), ("th_acceptnegstep", C.c_double),
                ("regfactor", C.c_double), ("regmin", C.c_double), ("regmax", C.c_double),
                ("n_alphas", C.c_int32), ("pad_", C.c_int32), ("alphas", C.c_double * 16)]


class BoxQPParams(C.Structure):
    _fields_ = [("maxiter", C.c_int32), ("n_alphas", C.c_int32), ("th_acceptstep", C.c_double),
                ("th_grad", C.c_double), ("reg", C.c_double), ("alphas", C.c_double * 16)]


class Result(C.Structure):
    _fields_ = [("status", C.c_int32), ("iter", C.c_int32), ("is_feasible", C.c_int32), ("n_iter_run", C.c_int32),
                ("cost", C.c_double), ("stop", C.c_double), ("xreg", C.c_double), ("ureg", C.c_double),
                ("steplength", C.c_double), ("dV", C.c_double), ("dVexp", C.c_double), ("d0", C.c_double),
                ("d1", C.c_double)]


# numpy view of a (Result * B) array: the per-element fields as arrays without a Python loop
RESULT_DTYPE = None


def result_array(r):
    """Structured numpy view of a ctypes (Result * B) array (no copy)."""
    global RESULT_DTYPE
    if RESULT_DTYPE is None:
        import numpy as np
        RESULT_DTYPE = np.dtype({"names": [f for f, _ in Result._fields_],
                                 "formats": ["<i4" if t is C.c_int32 else "<f8" for _, t in Result._fields_],
                                 "offsets": [getattr(Result, f).offset for f, _ in Result._fields_],
                                 "itemsize": C.sizeof(Result)})
    import numpy as np
    return np.frombuffer(r, dtype=RESULT_DTYPE)


P = C.c_void_p
D = C.POINTER(C.c_double)
I32 = C.POINTER(C.c_int32)
U64 = C.POINTER(C.c_uint64)

# fddp_iteration_callback(void* user, int iter, const fddp_result* results, const int32_t* reported, int B)
IterationCallback = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(Result), I32, C.c_int)

# name -> (restype, argtypes); `h` is an opaque handle pointer
PROTOS = {
    "default_params": (None, [C.POINTER(Params)]),
    "destroy": (None, [P]),
    "last_error": (C.c_char_p, []),
    "set_x0": (C.c_int, [P, D]),
    "set_params": (C.c_int, [P, C.POINTER(Params)]),
    "set_candidate": (C.c_int, [P, D, D, C.c_int]),
    "solve": (C.c_int, [P, C.c_int, C.c_int, C.c_double, C.POINTER(Result)]),
    "get_results": (C.c_int, [P, C.POINTER(Result)]),
    "problem_calc": (C.c_int, [P, D]),
    "problem_calc_diff": (C.c_int, [P, D]),
    "compute_direction": (C.c_int, [P, C.c_int, I32]),
    "calc_diff": (C.c_int, [P, D]),
    "backward_pass": (C.c_int, [P, I32]),
    "forward_pass": (C.c_int, [P, C.c_double, D, I32]),
    "update_expected_improvement": (C.c_int, [P]),
    "try_step": (C.c_int, [P, C.c_double, D, I32]),
    "expected_improvement": (C.c_int, [P, D]),
    "stopping_criteria": (C.c_int, [P, D]),
    "set_solver_state": (C.c_int, [P, C.c_int, C.c_double, C.c_double, C.c_int]),
    "get_quantity": (C.c_int, [P, C.c_int, D]),
    "mpc_shift": (C.c_int, [P]),
    "set_solver_kind": (C.c_int, [P, C.c_int]),
    "set_control_limits": (C.c_int, [P, D, D]),
    "set_knots": (C.c_int, [P, C.POINTER(KnotDesc), D, C.c_int64]),
}

# product-only entry points (libfddp_hip)
PROTOS_GPU = {
    "abi_version": (C.c_int, []),
    "create": (C.c_int, [C.POINTER(Dims), C.POINTER(KnotDesc), D, C.c_int64, C.c_int, C.POINTER(P)]),
    "set_model_params": (C.c_int, [P, D, C.c_int64]),
    "set_candidate_device": (C.c_int, [P, D, D, C.c_int]),
    "get_x0": (C.c_int, [P, D]),
    "get_params": (C.c_int, [P, C.POINTER(Params)]),
    "get_xs": (C.c_int, [P, D, C.c_int]),
    "get_us": (C.c_int, [P, D, C.c_int]),
    "get_xs_try": (C.c_int, [P, D]),
    "get_us_try": (C.c_int, [P, D]),
    "set_debug": (C.c_int, [P, C.c_int]),
    "synchronize": (C.c_int, [P]),
    "get_stream": (C.c_int, [P, C.POINTER(P)]),
    "get_timing": (C.c_int, [P, D, C.POINTER(C.c_int64)]),
    "set_timing": (C.c_int, [P, C.c_int]),
    "device_bytes": (C.c_int64, [P]),
    "get_solver_kind": (C.c_int, [P, I32]),
    "set_callback": (C.c_int, [P, IterationCallback, C.c_void_p]),
    "get_line_search_info": (C.c_int, [P, I32, I32]),
    "boxqp_default_params": (None, [C.POINTER(BoxQPParams)]),
    "boxqp_solve": (C.c_int, [C.c_int, C.c_int, C.c_int, D, D, D, D, D, C.POINTER(BoxQPParams), D, U64, U64, D, I32]),
}


def bind(lib, prefix, protos):
    for name, (res, args) in protos.items():
        fn = getattr(lib, prefix + name)
        fn.restype = res
        fn.argtypes = args


def dptr(a):
    """double* of a C-contiguous float64 numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data_as(D)
