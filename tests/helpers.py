"""Shared test plumbing: seeded problems, and a direct C-ABI wrapper of
libfddp_hip with the same call shapes as tests/oracle_lib.Oracle."""
import ctypes as C

import numpy as np

from crocoddyl_amd import _abi, synthetic
from crocoddyl_amd._lib import lib as gpu_lib
from crocoddyl_amd.problem import pack_problem


def setup(name, T=None, B=None, seed=None, drift_free=True):
    x0s, running, terminal = synthetic.build(name, T=T, B=B, seed=seed, drift_free=drift_free)
    B = x0s.shape[0]
    knots, pool = pack_problem(running, terminal, B)
    nx = running[0].state.nx
    ndx = getattr(running[0].state, "ndx", nx)
    nu_max = max(m.nu for m in running)
    dims = _abi.Dims(nx, ndx, nu_max, len(running), B)
    return dict(dims=dims, knots=knots, pool=pool, x0s=x0s, running=running, terminal=terminal)


class Gpu:
    """libfddp_hip handle driven through the C ABI (no facade)."""

    def __init__(self, dims, knots, pool, x0s, device=0):
        self.L = gpu_lib()
        self.dims = dims
        self.h = C.c_void_p()
        kd = (_abi.KnotDesc * len(knots))(*[_abi.KnotDesc(*k) for k in knots])
        self.pool = np.ascontiguousarray(pool, dtype=np.float64)
        self._ok(self.L.fddp_create(C.byref(dims), kd, _abi.dptr(self.pool), self.pool.size, device, C.byref(self.h)))
        self.set_x0(x0s)

    def _ok(self, rc):
        if rc != 0:
            raise RuntimeError(f"libfddp_hip error {rc}: {self.L.fddp_last_error().decode()}")

    def __del__(self):
        try:
            self.L.fddp_destroy(self.h)
        except Exception:
            pass

    def set_x0(self, x0s):
        self._ok(self.L.fddp_set_x0(self.h, _abi.dptr(np.ascontiguousarray(x0s, dtype=np.float64))))

    def set_params(self, prm):
        return self.L.fddp_set_params(self.h, C.byref(prm))

    def set_candidate(self, xs=None, us=None, is_feasible=False):
        xa = None if xs is None else np.ascontiguousarray(xs, dtype=np.float64)
        ua = None if us is None else np.ascontiguousarray(us, dtype=np.float64)
        self._ok(self.L.fddp_set_candidate(self.h, _abi.dptr(xa), _abi.dptr(ua), int(is_feasible)))

    def solve(self, maxiter=100, is_feasible=False, reg_init=1e-9):
        r = (_abi.Result * self.dims.B)()
        self._ok(self.L.fddp_solve(self.h, maxiter, int(is_feasible), reg_init, r))
        return r

    def results(self):
        r = (_abi.Result * self.dims.B)()
        self._ok(self.L.fddp_get_results(self.h, r))
        return r

    def xs(self, trial=False):
        d = self.dims
        a = np.zeros((d.B, d.T + 1, d.nx))
        if trial:
            self._ok(self.L.fddp_get_xs_try(self.h, _abi.dptr(a)))
        else:
            self._ok(self.L.fddp_get_xs(self.h, _abi.dptr(a), 0))
        return a

    def us(self, trial=False):
        d = self.dims
        a = np.zeros((d.B, d.T, d.nu_max))
        if trial:
            self._ok(self.L.fddp_get_us_try(self.h, _abi.dptr(a)))
        else:
            self._ok(self.L.fddp_get_us(self.h, _abi.dptr(a), 0))
        return a

    def quantity(self, which, nk, per):
        a = np.zeros((self.dims.B, nk, per))
        self._ok(self.L.fddp_get_quantity(self.h, which, _abi.dptr(a)))
        return a

    def set_debug(self, on=True):
        self._ok(self.L.fddp_set_debug(self.h, int(on)))

    def calc(self):
        c = np.zeros(self.dims.B)
        self._ok(self.L.fddp_problem_calc(self.h, _abi.dptr(c)))
        return c

    def calc_diff(self):
        c = np.zeros(self.dims.B)
        self._ok(self.L.fddp_problem_calc_diff(self.h, _abi.dptr(c)))
        return c

    def set_solver_state(self, it=0, xreg=float("nan"), ureg=float("nan"), was_feasible=0):
        self._ok(self.L.fddp_set_solver_state(self.h, it, xreg, ureg, was_feasible))

    def compute_direction(self, recalc=True):
        st = np.zeros(self.dims.B, dtype=np.int32)
        self._ok(self.L.fddp_compute_direction(self.h, int(recalc), st.ctypes.data_as(_abi.I32)))
        return st

    def update_expected_improvement(self):
        self._ok(self.L.fddp_update_expected_improvement(self.h))

    def try_step(self, alpha):
        dV = np.zeros(self.dims.B)
        st = np.zeros(self.dims.B, dtype=np.int32)
        self._ok(self.L.fddp_try_step(self.h, alpha, _abi.dptr(dV), st.ctypes.data_as(_abi.I32)))
        return dV, st

    def expected_improvement(self):
        d = np.zeros((self.dims.B, 2))
        self._ok(self.L.fddp_expected_improvement(self.h, _abi.dptr(d)))
        return d

    def stopping_criteria(self):
        s = np.zeros(self.dims.B)
        self._ok(self.L.fddp_stopping_criteria(self.h, _abi.dptr(s)))
        return s

    def mpc_shift(self):
        self._ok(self.L.fddp_mpc_shift(self.h))

    def set_solver_kind(self, kind):
        self._ok(self.L.fddp_set_solver_kind(self.h, int(kind)))

    def set_control_limits(self, lb, ub):
        la = None if lb is None else np.ascontiguousarray(lb, dtype=np.float64)
        ua = None if ub is None else np.ascontiguousarray(ub, dtype=np.float64)
        self._ok(self.L.fddp_set_control_limits(self.h, _abi.dptr(la), _abi.dptr(ua)))

    def quu_inv(self):
        return self.quantity(_abi.Q_QUU_INV, self.dims.T, self.dims.nu_max * self.dims.nu_max)


def rel_err(a, b):
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def results_dict(r):
    return {f: np.array([getattr(x, f) for x in r]) for f, _ in _abi.Result._fields_}
