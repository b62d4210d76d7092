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

    # SolverDDP's phases one at a time (fddp_calc_diff / fddp_backward_pass / fddp_forward_pass)
    def ddp_calc_diff(self):
        c = np.zeros(self.dims.B)
        self._ok(self.L.fddp_calc_diff(self.h, _abi.dptr(c)))
        return c

    def backward_pass(self):
        st = np.zeros(self.dims.B, dtype=np.int32)
        self._ok(self.L.fddp_backward_pass(self.h, st.ctypes.data_as(_abi.I32)))
        return st

    def forward_pass(self, alpha):
        """(rc, cost_try, status); rc != 0 on an argument error (no exception)."""
        ct = np.zeros(self.dims.B)
        st = np.zeros(self.dims.B, dtype=np.int32)
        rc = self.L.fddp_forward_pass(self.h, alpha, _abi.dptr(ct), st.ctypes.data_as(_abi.I32))
        return rc, ct, st

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
    """One max-abs error over the whole array / max(1, max|b|). Coarse: small components
    hide behind large ones. Solve-level parity uses elem_err."""
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def elem_err(a, b, floor=1e-3):
    """Element-wise parity error: max_i |a_i − b_i| / max(|b_i|, s_c(i)).

    s_c is the scale of element i's component c (the last axis: the state / control
    coordinate): max |b[..., c]| over every other axis (the knots of a trajectory, the
    elements of a batch), so each coordinate is compared at its own magnitude and a small
    joint velocity is not hidden behind the base height. Coordinates that are (nearly)
    zero everywhere fall back to `floor` × the array's max |b|. For a 1-D array (costs of
    a batch) every entry is its own component: plain relative error. NaN anywhere → NaN
    (which fails every `<=` bar)."""
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    if b.size == 0:
        return 0.0
    if b.ndim == 1:
        s = np.zeros_like(b)
    else:
        s = np.max(np.abs(b).reshape(-1, b.shape[-1]), axis=0)
    big = float(np.max(np.abs(b))) if np.all(np.isfinite(b)) else np.nan
    s = np.maximum(s, floor * big)
    d = np.abs(a - b) / np.maximum(np.maximum(np.abs(b), s), 1e-300)
    return float(np.nan if np.any(np.isnan(d)) else np.max(d))


def ulp_perturbed(pool, rng):
    """The parameter pool with every non-integer entry (masses, inertias, placements,
    cost weights, references, dt ...; not the structure: counts, kinds, parents) moved by
    one ulp, relative ±2^-52 with random signs."""
    p = np.array(pool, dtype=np.float64, copy=True)
    m = p != np.round(p)
    p[m] *= 1.0 + np.finfo(np.float64).eps * rng.choice([-1.0, 1.0], size=int(m.sum()))
    return p


def ulp_floor(run, pool, reps=3, seed=0):
    """Conditioning floor of a solve protocol: run(pool) -> tuple of output arrays
    (xs, us, costs ...) of the CPU oracle. Returns (run(pool), floors) where floors[i] is
    the largest elem_err of output i over `reps` runs on ulp_perturbed pools: how far the
    reference algorithm itself moves when its inputs carry one rounding error. Two
    correct fp64 implementations (different operation orders) cannot be expected to
    agree closer than this; on the ill-conditioned gait solves (cond(Quu) up to 5e10,
    cost ~1e7) it grows with every FDDP iteration (C5 smoke, T = 8: 2.2e-9 after one
    iteration, 2.4e-8 after three)."""
    base = run(pool)
    rng = np.random.default_rng(seed)
    floors = [0.0] * len(base)
    for _ in range(reps):
        out = run(ulp_perturbed(pool, rng))
        floors = [max(f, elem_err(o, b)) for f, o, b in zip(floors, out, base)]
    return base, floors


FLOOR_FACTOR = 3.0  # parity bar = max(tol, FLOOR_FACTOR x the conditioning floor) (round 6: 4 -> 3)

_LOGGED = []


def parity(name, a, b, tol, floor=None, scale_floor=1e-3):
    """elem_err(a, b) <= bar, recorded: printed and appended as a JSON line to
    $CROCODDYL_AMD_PARITY_LOG when set (so a GPU run leaves every achieved error behind,
    not only the failures). bar = tol, or max(tol, FLOOR_FACTOR * floor) when the
    oracle's conditioning floor (ulp_floor) of the same protocol is given."""
    import json
    import os
    e = elem_err(a, b, scale_floor)
    bar = tol if floor is None else max(tol, FLOOR_FACTOR * floor)
    test = os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0]
    rec = {"test": test, "check": name, "elem_err": e, "tol": tol, "floor": floor, "bar": bar, "ok": bool(e <= bar)}
    _LOGGED.append(rec)
    print(f"parity {name}: {e:.3e} (bar {bar:.3g}" + ("" if floor is None else f", oracle floor {floor:.3g}") + ")")
    path = os.environ.get("CROCODDYL_AMD_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")
    if os.environ.get("CROCODDYL_AMD_PARITY_MEASURE") != "1":  # measuring runs log every bar, assert none
        assert e <= bar, (name, e, bar, floor)
    return e


def results_dict(r):
    return {f: np.array([getattr(x, f) for x in r]) for f, _ in _abi.Result._fields_}
