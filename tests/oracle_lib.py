"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so) — tests only.

The oracle is test infrastructure (see oracle/fddp_oracle.cpp header). This
module builds it on demand with oracle/Makefile (g++ -fopenmp) and exposes
the same call shapes as libfddp_hip so parity tests read symmetric.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from crocoddyl_amd import _abi  # noqa: E402

ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "liboracle.so")

_lib = None


def build(out_dir=None, arch=None, cxx=None, ldflags=None):
    env = dict(os.environ)
    args = ["make", "-s", "-C", ORACLE_DIR]
    if out_dir:
        args.append(f"OUT={out_dir}")
    if arch:
        args.append(f"ARCH={arch}")
    if cxx:
        args.append(f"CXX={cxx}")
    if ldflags:
        args.append(f"LDFLAGS={ldflags}")
    subprocess.run(args, check=True, env=env)


def lib(path=None):
    global _lib
    if path is not None:
        L = C.CDLL(path)
        _bind(L)
        return L
    if _lib is None:
        srcs = [os.path.join(ORACLE_DIR, f) for f in ("fddp_oracle.cpp", "multibody_oracle.hpp", "floating_oracle.hpp", "Makefile")]
        if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < max(os.path.getmtime(f) for f in srcs):
            build()
        _lib = C.CDLL(ORACLE_SO)
        _bind(_lib)
    return _lib


def _bind(L):
    _abi.bind(L, "oracle_", {k: v for k, v in _abi.PROTOS.items() if k not in ("default_params",)})
    L.oracle_default_params.restype = None
    L.oracle_default_params.argtypes = [C.POINTER(_abi.Params)]
    L.oracle_create.restype = C.c_int
    L.oracle_create.argtypes = [C.POINTER(_abi.Dims), C.POINTER(_abi.KnotDesc), _abi.D, C.c_int64,
                                C.POINTER(C.c_void_p)]
    L.oracle_set_threading.restype = C.c_int
    L.oracle_set_threading.argtypes = [C.c_void_p, C.c_int, C.c_int]
    for n in ("get_xs", "get_us", "get_xs_try", "get_us_try"):
        f = getattr(L, "oracle_" + n)
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, _abi.D]
    L.oracle_get_trace.restype = C.c_int
    L.oracle_get_trace.argtypes = [C.c_void_p, C.c_int, _abi.D, C.c_int]
    L.oracle_get_phase_times.restype = C.c_int
    L.oracle_get_phase_times.argtypes = [C.c_void_p, _abi.D, C.c_int]
    L.oracle_get_quu_inv.restype = C.c_int
    L.oracle_get_quu_inv.argtypes = [C.c_void_p, _abi.D]
    L.oracle_boxqp_solve.restype = C.c_int
    L.oracle_boxqp_solve.argtypes = [C.c_int, C.c_int, _abi.D, _abi.D, _abi.D, _abi.D, _abi.D,
                                     C.POINTER(_abi.BoxQPParams), _abi.D, _abi.U64, _abi.U64, _abi.D, _abi.I32,
                                     _abi.I32]


def boxqp_solve(H, q, lb, ub, xinit, prm):
    """Batched BoxQP on the oracle (same contract as fddp_boxqp_solve).
    H: (B, n, n) row-major numpy; returns dict of x, free_mask, inv_mask,
    Hinv (B, n, n) embedded, status, iters."""
    L = lib()
    H = np.asarray(H, float)
    B, n = H.shape[0], H.shape[1]
    Hc = np.ascontiguousarray(H.transpose(0, 2, 1))
    vs = [np.ascontiguousarray(np.broadcast_to(np.asarray(v, float), (B, n))) for v in (q, lb, ub, xinit)]
    out = dict(x=np.zeros((B, n)), free_mask=np.zeros(B, np.uint64), inv_mask=np.zeros(B, np.uint64),
               Hinv=np.zeros((B, n, n)), status=np.zeros(B, np.int32), iters=np.zeros(B, np.int32))
    rc = L.oracle_boxqp_solve(B, n, _abi.dptr(Hc), *[_abi.dptr(v) for v in vs], C.byref(prm),
                              _abi.dptr(out["x"]), out["free_mask"].ctypes.data_as(_abi.U64),
                              out["inv_mask"].ctypes.data_as(_abi.U64), _abi.dptr(out["Hinv"]),
                              out["status"].ctypes.data_as(_abi.I32), out["iters"].ctypes.data_as(_abi.I32))
    assert rc == 0
    out["Hinv"] = np.ascontiguousarray(out["Hinv"].transpose(0, 2, 1))
    return out


class Oracle:
    """One oracle handle (B problems on the CPU)."""

    def __init__(self, dims, knots, pool, x0s, threads=1, mode=2):
        self.L = lib()
        self.dims = dims
        self.h = C.c_void_p()
        kd = (_abi.KnotDesc * len(knots))(*[_abi.KnotDesc(*k) for k in knots])
        self.pool = np.ascontiguousarray(pool, dtype=np.float64)
        rc = self.L.oracle_create(C.byref(dims), kd, _abi.dptr(self.pool), self.pool.size, C.byref(self.h))
        assert rc == 0, self.L.oracle_last_error()
        self.L.oracle_set_threading(self.h, mode, threads)
        self.set_x0(x0s)

    def __del__(self):
        try:
            self.L.oracle_destroy(self.h)
        except Exception:
            pass

    def set_x0(self, x0s):
        a = np.ascontiguousarray(x0s, dtype=np.float64)
        self.L.oracle_set_x0(self.h, _abi.dptr(a))

    def set_params(self, prm):
        self.L.oracle_set_params(self.h, C.byref(prm))

    def set_candidate(self, xs=None, us=None, is_feasible=False):
        xa = None if xs is None else np.ascontiguousarray(xs, dtype=np.float64)
        ua = None if us is None else np.ascontiguousarray(us, dtype=np.float64)
        self.L.oracle_set_candidate(self.h, _abi.dptr(xa), _abi.dptr(ua), int(is_feasible))

    def solve(self, maxiter=100, is_feasible=False, reg_init=1e-9):
        r = (_abi.Result * self.dims.B)()
        self.L.oracle_solve(self.h, maxiter, int(is_feasible), reg_init, r)
        return r

    def results(self):
        r = (_abi.Result * self.dims.B)()
        self.L.oracle_get_results(self.h, r)
        return r

    def xs(self, trial=False):
        d = self.dims
        a = np.zeros((d.B, d.T + 1, d.nx))
        (self.L.oracle_get_xs_try if trial else self.L.oracle_get_xs)(self.h, _abi.dptr(a))
        return a

    def us(self, trial=False):
        d = self.dims
        a = np.zeros((d.B, d.T, d.nu_max))
        (self.L.oracle_get_us_try if trial else self.L.oracle_get_us)(self.h, _abi.dptr(a))
        return a

    def quantity(self, which, nk, per):
        a = np.zeros((self.dims.B, nk, per))
        self.L.oracle_get_quantity(self.h, which, _abi.dptr(a))
        return a

    def phase_times(self, reset=True):
        """Seconds of thread time per phase, summed over the elements: calc (iteration
        0), calcDiff + gaps, backward, forward."""
        a = np.zeros(4)
        self.L.oracle_get_phase_times(self.h, _abi.dptr(a), int(reset))
        return dict(zip(("calc", "calcDiff", "backward", "forward"), a.tolist()))

    def trace(self, b, maxn=1000):
        a = np.zeros((maxn, 8))
        n = self.L.oracle_get_trace(self.h, b, _abi.dptr(a), maxn)
        return a[:n]

    # step API
    def calc(self):
        c = np.zeros(self.dims.B)
        self.L.oracle_problem_calc(self.h, _abi.dptr(c))
        return c

    def calc_diff(self):
        c = np.zeros(self.dims.B)
        self.L.oracle_problem_calc_diff(self.h, _abi.dptr(c))
        return c

    def set_solver_state(self, it=0, xreg=float("nan"), ureg=float("nan"), was_feasible=0):
        self.L.oracle_set_solver_state(self.h, it, xreg, ureg, was_feasible)

    def compute_direction(self, recalc=True):
        st = np.zeros(self.dims.B, dtype=np.int32)
        self.L.oracle_compute_direction(self.h, int(recalc), st.ctypes.data_as(_abi.I32))
        return st

    def update_expected_improvement(self):
        self.L.oracle_update_expected_improvement(self.h)

    # SolverDDP's phases one at a time (ddp.cpp:157-253, fddp.cpp:149-225)
    def ddp_calc_diff(self):
        c = np.zeros(self.dims.B)
        self.L.oracle_calc_diff(self.h, _abi.dptr(c))
        return c

    def backward_pass(self):
        st = np.zeros(self.dims.B, dtype=np.int32)
        self.L.oracle_backward_pass(self.h, st.ctypes.data_as(_abi.I32))
        return st

    def forward_pass(self, alpha):
        ct = np.zeros(self.dims.B)
        st = np.zeros(self.dims.B, dtype=np.int32)
        rc = self.L.oracle_forward_pass(self.h, alpha, _abi.dptr(ct), st.ctypes.data_as(_abi.I32))
        return rc, ct, st

    def try_step(self, alpha):
        dV = np.zeros(self.dims.B)
        st = np.zeros(self.dims.B, dtype=np.int32)
        self.L.oracle_try_step(self.h, alpha, _abi.dptr(dV), st.ctypes.data_as(_abi.I32))
        return dV, st

    def expected_improvement(self):
        d = np.zeros((self.dims.B, 2))
        self.L.oracle_expected_improvement(self.h, _abi.dptr(d))
        return d

    def stopping_criteria(self):
        s = np.zeros(self.dims.B)
        self.L.oracle_stopping_criteria(self.h, _abi.dptr(s))
        return s

    def mpc_shift(self):
        self.L.oracle_mpc_shift(self.h)

    # SolverBoxFDDP
    def set_solver_kind(self, kind):
        self.L.oracle_set_solver_kind(self.h, int(kind))

    def set_control_limits(self, lb, ub):
        la = None if lb is None else np.ascontiguousarray(lb, dtype=np.float64)
        ua = None if ub is None else np.ascontiguousarray(ub, dtype=np.float64)
        self.L.oracle_set_control_limits(self.h, _abi.dptr(la), _abi.dptr(ua))

    def quu_inv(self):
        d = self.dims
        a = np.zeros((d.B, d.T, d.nu_max * d.nu_max))
        self.L.oracle_get_quu_inv(self.h, _abi.dptr(a))
        return a


def default_params():
    p = _abi.Params()
    lib().oracle_default_params(C.byref(p))
    return p
