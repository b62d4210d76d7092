"""Knot (action) models with the reference's Python API, as parameter carriers.

The models run on the device (crocoddyl_amd/csrc/knots.hpp); these classes
only hold the parameters, validate them like the reference setters, and pack
them into the C-ABI parameter blocks of include/fddp_hip.h (Eigen column-major).

Every matrix/vector parameter may carry a leading batch axis (B, ...): then
each batch element gets its own block (fddp_knot_desc.param_stride > 0).
Without it the block is shared by all elements, as a reference model object
shared by several knots is (benchmark/lqr-optctrl.cpp:28-31).

Reference API mirrored (bindings/python/crocoddyl/core/...):
  ActionModelLQR(nx, nu, driftFree=True)          core/actions/lqr.cpp:23-74
  ActionModelUnicycle()  .costWeights               core/actions/unicycle.cpp:26-57
  DifferentialActionModelLQR(nq, nu, driftFree=True) core/actions/diff-lqr.cpp
  IntegratedActionModelEuler(diffModel, stepTime=1e-3, withCostResidual=True)
                                                   core/integrator/euler.cpp
"""
import numpy as np

from . import _abi

_EPS = np.finfo(float).eps


class StateVector:
    """StateVector (core/states/euclidean.hxx): diff = x1 - x0, integrate = x + dx."""

    def __init__(self, nx):
        self.nx = int(nx)
        self.ndx = int(nx)
        self.nq = self.nx // 2 if self.nx % 2 == 0 else self.nx  # state-base.hxx:12-20
        self.nv = self.ndx - self.nq if self.nx % 2 == 0 else 0

    def zero(self):
        return np.zeros(self.nx)

    def rand(self):
        return np.random.uniform(-1.0, 1.0, self.nx)  # Eigen VectorXs::Random

    def diff(self, x0, x1):
        return np.asarray(x1, float) - np.asarray(x0, float)

    def integrate(self, x, dx):
        return np.asarray(x, float) + np.asarray(dx, float)


def _colmajor(a, r, c, name):
    """(r,c) or (B,r,c) -> (Bm, r*c) column-major rows."""
    a = np.asarray(a, dtype=np.float64)
    if a.ndim == 2:
        if a.shape != (r, c):
            raise ValueError(f"Invalid argument: {name} has wrong dimension (it should be {r},{c})")
        return a.T.reshape(1, -1)
    if a.ndim == 3 and a.shape[1:] == (r, c):
        return np.ascontiguousarray(a.transpose(0, 2, 1)).reshape(a.shape[0], -1)
    raise ValueError(f"Invalid argument: {name} has wrong dimension (it should be {r},{c} or B,{r},{c})")


def _vec(a, n, name):
    a = np.asarray(a, dtype=np.float64)
    if a.ndim == 1:
        if a.shape != (n,):
            raise ValueError(f"Invalid argument: {name} has wrong dimension (it should be {n})")
        return a.reshape(1, -1)
    if a.ndim == 2 and a.shape[1] == n:
        return a
    raise ValueError(f"Invalid argument: {name} has wrong dimension (it should be {n} or B,{n})")


def _stack(parts, header):
    """Concatenate (Bm_i, size_i) parts into (B, size) rows with a header."""
    bs = {p.shape[0] for p in parts if p.shape[0] != 1}
    if len(bs) > 1:
        raise ValueError("Invalid argument: batched parameters have inconsistent batch sizes")
    B = bs.pop() if bs else 1
    hdr = np.broadcast_to(np.asarray(header, float).reshape(1, -1), (B, _abi.PARAM_HEADER))
    cols = [hdr] + [np.broadcast_to(p, (B, p.shape[1])) for p in parts]
    return np.ascontiguousarray(np.concatenate(cols, axis=1))


class _ControlLimits:
    """u_lb / u_ub / has_control_limits of ActionModelAbstract and
    DifferentialActionModelAbstract (core/action-base.hxx:20-22,107-144,
    core/diff-action-base.hxx:21-23,99-136): -inf / +inf by default, setters
    check the size, and has_control_limits = any(isfinite(u_lb)) and
    any(isfinite(u_ub)). A leading batch axis (B, nu) gives every batch
    element its own limits."""

    def _init_limits(self):
        self._u_lb = np.full(self.nu, -np.inf)
        self._u_ub = np.full(self.nu, np.inf)
        self._lim_version = 0

    def _set_limit(self, name, v):
        v = np.array(v, dtype=np.float64)
        if v.shape[-1:] != (self.nu,) or v.ndim not in (1, 2):
            raise ValueError(f"Invalid argument: {'lower' if name == 'u_lb' else 'upper'} bound has wrong "
                             f"dimension (it should be {self.nu})")
        setattr(self, "_" + name, v)
        self._lim_version += 1

    u_lb = property(lambda s: s._u_lb, lambda s, v: s._set_limit("u_lb", v))
    u_ub = property(lambda s: s._u_ub, lambda s, v: s._set_limit("u_ub", v))

    @property
    def has_control_limits(self):
        """update_has_control_limits (action-base.hxx:142-144); per element when batched."""
        lb = np.isfinite(np.atleast_2d(self._u_lb)).any(axis=-1)
        ub = np.isfinite(np.atleast_2d(self._u_ub)).any(axis=-1)
        r = lb & ub
        return r if (np.ndim(self._u_lb) == 2 or np.ndim(self._u_ub) == 2) else bool(r[0])


class ActionModelAbstract(_ControlLimits):
    """Base of the device-backed knot models (core/action-base.hpp:23-99)."""

    kind = None

    def __init__(self, state, nu, nr=0):
        self.state = state
        self.nu = int(nu)
        self.nr = int(nr)
        self.unone = np.zeros(self.nu)  # action-base.hpp: the default control of calc(data, x)
        self._version = 0
        self._init_limits()

    def _touch(self):
        self._version += 1

    def pack(self):
        """(kind, nu, blocks (Bm, size)) for the parameter pool. A Python subclass
        without a device kind overrides calc(data, x, u=None) / calcDiff(data, x,
        u=None) instead (action-base.hpp:18-55); its problems run on the host
        (crocoddyl_amd.host)."""
        raise NotImplementedError

    def calc(self, data, x, u=None):
        raise NotImplementedError("crocoddyl_amd: calc of a Python-defined action model must be overridden")

    def calcDiff(self, data, x, u=None):
        raise NotImplementedError("crocoddyl_amd: calcDiff of a Python-defined action model must be overridden")

    def createData(self):
        return ActionData(self)


class ActionData:
    """Host view of one knot's ActionData (core/action-base.hpp:101-142),
    filled from the device after ShootingProblem.calc/calcDiff."""

    def __init__(self, model):
        n, m = model.state.ndx, model.nu
        self.cost = 0.0
        self.r = np.zeros(getattr(model, "nr", 0))
        self.xnext = np.zeros(model.state.nx)
        self.Fx = np.zeros((n, n))
        self.Fu = np.zeros((n, m))
        self.Lx = np.zeros(n)
        self.Lu = np.zeros(m)
        self.Lxx = np.zeros((n, n))
        self.Lxu = np.zeros((n, m))
        self.Luu = np.zeros((m, m))


ActionDataAbstract = ActionData  # the reference's base name for derived data classes


class ActionModelLQR(ActionModelAbstract):
    """ActionModelLQR (include/crocoddyl/core/actions/lqr.hxx:13-25 defaults)."""

    kind = _abi.KNOT_LQR

    def __init__(self, nx, nu, driftFree=True):
        super().__init__(StateVector(nx), nu, 0)
        nx, nu = int(nx), int(nu)
        self.driftFree = bool(driftFree)
        self._Fx = np.eye(nx)
        self._Fu = np.eye(nx, nu)
        self._f0 = np.ones(nx)
        self._Lxx = np.eye(nx)
        self._Lxu = np.eye(nx, nu)
        self._Luu = np.eye(nu)
        self._lx = np.ones(nx)
        self._lu = np.ones(nu)

    def _set(self, name, v, shape):
        v = np.array(v, dtype=np.float64)
        if v.shape[-len(shape):] != shape or v.ndim not in (len(shape), len(shape) + 1):
            raise ValueError(f"Invalid argument: {name} has wrong dimension (it should be {shape})")
        setattr(self, "_" + name, v)
        self._touch()

    nx_ = property(lambda s: s.state.nx)
    Fx = property(lambda s: s._Fx, lambda s, v: s._set("Fx", v, (s.state.nx, s.state.nx)))
    Fu = property(lambda s: s._Fu, lambda s, v: s._set("Fu", v, (s.state.nx, s.nu)))
    f0 = property(lambda s: s._f0, lambda s, v: s._set("f0", v, (s.state.nx,)))
    Lxx = property(lambda s: s._Lxx, lambda s, v: s._set("Lxx", v, (s.state.nx, s.state.nx)))
    Lxu = property(lambda s: s._Lxu, lambda s, v: s._set("Lxu", v, (s.state.nx, s.nu)))
    Luu = property(lambda s: s._Luu, lambda s, v: s._set("Luu", v, (s.nu, s.nu)))
    lx = property(lambda s: s._lx, lambda s, v: s._set("lx", v, (s.state.nx,)))
    lu = property(lambda s: s._lu, lambda s, v: s._set("lu", v, (s.nu,)))

    def pack(self):
        nx, nu = self.state.nx, self.nu
        parts = [_colmajor(self._Fx, nx, nx, "Fx"), _colmajor(self._Fu, nx, nu, "Fu"), _vec(self._f0, nx, "f0"),
                 _colmajor(self._Lxx, nx, nx, "Lxx"), _colmajor(self._Lxu, nx, nu, "Lxu"),
                 _colmajor(self._Luu, nu, nu, "Luu"), _vec(self._lx, nx, "lx"), _vec(self._lu, nu, "lu")]
        return self.kind, nu, _stack(parts, [1.0 if self.driftFree else 0.0, 0, 0, 0])


class ActionModelUnicycle(ActionModelAbstract):
    """ActionModelUnicycle (core/actions/unicycle.hxx:13-16): nx=3, nu=2, nr=5, dt=0.1."""

    kind = _abi.KNOT_UNICYCLE

    def __init__(self):
        super().__init__(StateVector(3), 2, 5)
        self._w = np.array([10.0, 1.0])
        self._dt = 0.1

    @property
    def costWeights(self):
        return self._w.copy()

    @costWeights.setter
    def costWeights(self, w):
        w = np.asarray(w, float)
        if w.shape != (2,):
            raise ValueError("Invalid argument: costWeights has wrong dimension (it should be 2)")
        self._w = w.copy()
        self._touch()

    @property
    def dt(self):
        return self._dt

    @dt.setter
    def dt(self, v):
        self._dt = float(v)
        self._touch()

    def pack(self):
        return self.kind, 2, np.array([[self._dt, self._w[0], self._w[1], 0.0]])


class DifferentialActionModelLQR(_ControlLimits):
    """DifferentialActionModelLQR (core/actions/diff-lqr.hxx:14-28 defaults).
    Only usable inside IntegratedActionModelEuler on the device."""

    def __init__(self, nq, nu, driftFree=True):
        nq, nu = int(nq), int(nu)
        self.state = StateVector(2 * nq)
        self.nu = nu
        self.nr = 0
        self._init_limits()
        self.driftFree = bool(driftFree)
        nx = 2 * nq
        self._Fq = np.eye(nq)
        self._Fv = np.eye(nq)
        self._Fu = np.eye(nq, nu)
        self._f0 = np.ones(nq)
        self._Lxx = np.eye(nx)
        self._Lxu = np.eye(nx, nu)
        self._Luu = np.eye(nu)
        self._lx = np.ones(nx)
        self._lu = np.ones(nu)
        self._version = 0
        self._owners = []

    def _set(self, name, v, shape):
        v = np.array(v, dtype=np.float64)
        if v.shape[-len(shape):] != shape or v.ndim not in (len(shape), len(shape) + 1):
            raise ValueError(f"Invalid argument: {name} has wrong dimension (it should be {shape})")
        setattr(self, "_" + name, v)
        self._version += 1
        for o in self._owners:
            o._touch()

    @property
    def nq(self):
        return self.state.nx // 2

    Fq = property(lambda s: s._Fq, lambda s, v: s._set("Fq", v, (s.nq, s.nq)))
    Fv = property(lambda s: s._Fv, lambda s, v: s._set("Fv", v, (s.nq, s.nq)))
    Fu = property(lambda s: s._Fu, lambda s, v: s._set("Fu", v, (s.nq, s.nu)))
    f0 = property(lambda s: s._f0, lambda s, v: s._set("f0", v, (s.nq,)))
    Lxx = property(lambda s: s._Lxx, lambda s, v: s._set("Lxx", v, (s.state.nx, s.state.nx)))
    Lxu = property(lambda s: s._Lxu, lambda s, v: s._set("Lxu", v, (s.state.nx, s.nu)))
    Luu = property(lambda s: s._Luu, lambda s, v: s._set("Luu", v, (s.nu, s.nu)))
    lx = property(lambda s: s._lx, lambda s, v: s._set("lx", v, (s.state.nx,)))
    lu = property(lambda s: s._lu, lambda s, v: s._set("lu", v, (s.nu,)))


class IntegratedActionModelEuler(ActionModelAbstract):
    """IntegratedActionModelEuler (core/integrator/euler.hxx:16-35) around a
    device-covered differential model: DifferentialActionModelLQR, or
    DifferentialActionModelFreeFwdDynamics (crocoddyl_amd.multibody)."""

    kind = _abi.KNOT_EULER_DIFFLQR

    def __init__(self, diffModel, stepTime=1e-3, withCostResidual=True):
        from .multibody import DifferentialActionModelFreeFwdDynamics
        self._mb = isinstance(diffModel, DifferentialActionModelFreeFwdDynamics)
        self._host = isinstance(diffModel, DifferentialActionModelAbstract)
        if not (self._mb or self._host or isinstance(diffModel, DifferentialActionModelLQR)):
            raise NotImplementedError("crocoddyl_amd: IntegratedActionModelEuler covers DifferentialActionModelLQR, "
                                      "the multibody DAMs and Python-subclassed DifferentialActionModelAbstract; got "
                                      f"{type(diffModel).__name__}")
        if self._mb:
            self.kind = diffModel.knot_kind
        if self._host:
            # a Python-defined DAM: no device kind, so the knot (and its problem) runs on
            # the host path (crocoddyl_amd.host), the integrator below in numpy
            if diffModel.state.nx != diffModel.state.ndx:
                raise NotImplementedError("crocoddyl_amd: Python-defined differential models are integrated on "
                                          "Euclidean states (nx == ndx)")
            self.kind = None
        super().__init__(diffModel.state, diffModel.nu, diffModel.nr)
        # the integrated model copies the differential model's limits (euler.hxx:25-26)
        self.u_lb = diffModel.u_lb
        self.u_ub = diffModel.u_ub
        self.differential = diffModel
        if not (self._mb or self._host):
            diffModel._owners.append(self)
        self.withCostResidual = bool(withCostResidual)
        dt = float(stepTime)
        if dt < 0.0:  # euler.hxx:27-31
            dt = 1e-3
        self._dt = dt

    # -- host path of a Python-defined DAM: euler.hxx:41-131 on numpy ----------------
    def createData(self):
        if not self.__dict__.get("_host"):
            return ActionData(self)
        return IntegratedActionDataEuler(self)

    def calc(self, data, x, u=None):
        """euler.hxx:41-80 (calc(data, x) evaluates at unone, action-base.hxx:28-37)."""
        if not self.__dict__.get("_host"):
            return super().calc(data, x, u)
        x = np.asarray(x, float)
        u = self.unone if u is None else np.asarray(u, float)
        st, nv = self.differential.state, self.differential.state.nv
        dd = data.differential
        self.differential.calc(dd, x, u)
        v, a = x[st.nx - nv:], np.asarray(dd.xout, float)
        if self._dt != 0.0:  # enable_integration_
            dt = self._dt
            data.dx = np.concatenate([v * dt + a * (dt * dt), a * dt])
            data.xnext = st.integrate(x, data.dx)
            data.cost = dt * dd.cost
        else:
            data.dx = np.zeros(st.ndx)
            data.xnext = x.copy()
            data.cost = dd.cost
        if self.withCostResidual:
            data.r = np.array(dd.r, float, copy=True)

    def calcDiff(self, data, x, u=None):
        """euler.hxx:83-131 on a Euclidean state (Jintegrate = I, JintegrateTransport = id)."""
        if not self.__dict__.get("_host"):
            return super().calcDiff(data, x, u)
        x = np.asarray(x, float)
        u = self.unone if u is None else np.asarray(u, float)
        st, nv, nu = self.differential.state, self.differential.state.nv, self.nu
        dd = data.differential
        self.differential.calcDiff(dd, x, u)
        ndx = st.ndx
        if self._dt != 0.0:
            dt, dt2 = self._dt, self._dt * self._dt
            da_dx, da_du = np.asarray(dd.Fx, float), np.asarray(dd.Fu, float).reshape(nv, nu)
            Fx = np.zeros((ndx, ndx))
            Fx[:nv] = da_dx * dt2
            Fx[nv:] = da_dx * dt
            Fx[np.arange(nv), ndx - nv + np.arange(nv)] += dt
            Fx += np.eye(ndx)  # Jintegrate(first, addto) of a Euclidean state
            data.Fx = Fx
            Fu = np.zeros((ndx, nu))
            Fu[:nv] = da_du * dt2
            Fu[nv:] = da_du * dt
            data.Fu = Fu
            data.Lx, data.Lu = dt * np.asarray(dd.Lx, float), dt * np.asarray(dd.Lu, float)
            data.Lxx, data.Lxu = dt * np.asarray(dd.Lxx, float), dt * np.asarray(dd.Lxu, float)
            data.Luu = dt * np.asarray(dd.Luu, float)
        else:
            data.Fx = np.eye(ndx)
            data.Fu = np.zeros((ndx, nu))
            data.Lx, data.Lu = np.array(dd.Lx, float), np.array(dd.Lu, float)
            data.Lxx, data.Lxu, data.Luu = np.array(dd.Lxx, float), np.array(dd.Lxu, float), np.array(dd.Luu, float)

    # the multibody DAM's parameters (robot, costs, armature) are part of the
    # version the problem compares before re-uploading parameter blocks
    @property
    def _version(self):
        own = self.__dict__.get("_own_version", 0)
        return (own, self.differential.version()) if self.__dict__.get("_mb") else own

    @_version.setter
    def _version(self, v):
        self.__dict__["_own_version"] = v if not isinstance(v, tuple) else v[0]

    def _touch(self):
        self.__dict__["_own_version"] = self.__dict__.get("_own_version", 0) + 1

    @property
    def dt(self):
        return self._dt

    @dt.setter
    def dt(self, v):
        if v < 0.0:
            raise ValueError("Invalid argument: dt has positive value")  # euler.hxx:160-167
        self._dt = float(v)
        self._touch()

    def quasiStatic(self, data, x, maxiter=100, tol=1e-9):
        """IntegratedActionModelEuler::quasiStatic (euler.hxx:185-201): the
        differential model's quasi-static controls (multibody DAMs only)."""
        if not self._mb:
            raise NotImplementedError("crocoddyl_amd: quasiStatic is covered for the multibody models")
        return self.differential.quasiStatic(x, maxiter, tol)

    def pack(self):
        d = self.differential
        if self._mb:
            self.kind = d.knot_kind
            return self.kind, d.nu, d.pack_body(self._dt)
        nq, nu, nx = d.nq, d.nu, d.state.nx
        parts = [_colmajor(d._Fq, nq, nq, "Fq"), _colmajor(d._Fv, nq, nq, "Fv"), _colmajor(d._Fu, nq, nu, "Fu"),
                 _vec(d._f0, nq, "f0"), _colmajor(d._Lxx, nx, nx, "Lxx"), _colmajor(d._Lxu, nx, nu, "Lxu"),
                 _colmajor(d._Luu, nu, nu, "Luu"), _vec(d._lx, nx, "lx"), _vec(d._lu, nu, "lu")]
        return self.kind, nu, _stack(parts, [self._dt, 1.0 if d.driftFree else 0.0, 0, 0])


class IntegratedActionDataEuler(ActionData):
    """IntegratedActionDataEuler (euler.hpp): the differential model's data + dx."""

    def __init__(self, model):
        super().__init__(model)
        self.differential = model.differential.createData()
        self.dx = np.zeros(model.state.ndx)


class DifferentialActionModelAbstract(_ControlLimits):
    """Base of Python-defined differential (continuous-time) action models
    (core/diff-action-base.hpp:41-72; Python overrides as
    bindings/python/crocoddyl/core/diff-action-base.hpp:19-35): override
    calc(data, x, u=None) to fill data.xout (the acceleration, nv), data.cost
    (and data.r), and calcDiff(data, x, u=None) to fill data.Fx (nv x ndx),
    data.Fu (nv x nu), data.Lx, data.Lu, data.Lxx, data.Lxu, data.Luu. Integrated
    with IntegratedActionModelEuler, such a knot runs on the host path."""

    def __init__(self, state, nu, nr=0):
        self.state = state
        self.nu = int(nu)
        self.nr = int(nr)
        self.unone = np.zeros(self.nu)
        self._init_limits()

    def calc(self, data, x, u=None):
        raise NotImplementedError("crocoddyl_amd: calc of a Python-defined differential model must be overridden")

    def calcDiff(self, data, x, u=None):
        raise NotImplementedError("crocoddyl_amd: calcDiff of a Python-defined differential model must be overridden")

    def createData(self):
        return DifferentialActionData(self)


class DifferentialActionData:
    """DifferentialActionDataAbstract (core/diff-action-base.hpp:118-150)."""

    def __init__(self, model):
        nv, ndx, nu = model.state.nv, model.state.ndx, model.nu
        self.cost = 0.0
        self.xout = np.zeros(nv)
        self.r = np.zeros(model.nr)
        self.Fx = np.zeros((nv, ndx))
        self.Fu = np.zeros((nv, nu))
        self.Lx = np.zeros(ndx)
        self.Lu = np.zeros(nu)
        self.Lxx = np.zeros((ndx, ndx))
        self.Lxu = np.zeros((ndx, nu))
        self.Luu = np.zeros((nu, nu))


DifferentialActionDataAbstract = DifferentialActionData


class DifferentialActionModelNumDiff(DifferentialActionModelAbstract):
    """DifferentialActionModelNumDiff(model, gaussApprox=False)
    (core/numdiff/diff-action.hxx:13-93): forward differences of the model's calc
    with disturbance sqrt(2 eps) along state.integrate(x, dx) and u + du; with
    gaussApprox the cost Hessians from the residual Jacobians (Rx^T Rx, Rx^T Ru,
    Ru^T Ru). calcDiff uses the data of the preceding calc at (x, u), as the reference."""

    def __init__(self, model, gaussApprox=False):
        super().__init__(model.state, model.nu, model.nr)
        self.model = model
        self.withGaussApprox = bool(gaussApprox)
        self.disturbance = np.sqrt(2.0 * np.finfo(float).eps)
        if self.withGaussApprox and self.nr == 1:
            raise ValueError("No Gauss approximation possible with nr = 1")

    def createData(self):
        d = DifferentialActionData(self)
        d.data_0 = self.model.createData()
        d.data_x = [self.model.createData() for _ in range(self.state.ndx)]
        d.data_u = [self.model.createData() for _ in range(self.nu)]
        d.Rx = np.zeros((self.nr, self.state.ndx))
        d.Ru = np.zeros((self.nr, self.nu))
        return d

    def calc(self, data, x, u=None):
        u = self.unone if u is None else u
        self.model.calc(data.data_0, x, u)
        data.cost = data.data_0.cost
        data.xout = np.array(data.data_0.xout, float, copy=True)

    def calcDiff(self, data, x, u=None):
        u = self.unone if u is None else np.asarray(u, float)
        x = np.asarray(x, float)
        d0 = data.data_0
        xn0, c0, r0 = np.asarray(d0.xout, float), d0.cost, np.asarray(d0.r, float)
        data.xout, data.cost = xn0.copy(), c0
        h = self.disturbance
        dx = np.zeros(self.state.ndx)
        for ix in range(self.state.ndx):
            dx[ix] = h
            dxi = data.data_x[ix]
            self.model.calc(dxi, self.state.integrate(x, dx), u)
            data.Fx[:, ix] = (np.asarray(dxi.xout, float) - xn0) / h
            data.Lx[ix] = (dxi.cost - c0) / h
            data.Rx[:, ix] = (np.asarray(dxi.r, float) - r0) / h
            dx[ix] = 0.0
        du = np.zeros(self.nu)
        for iu in range(self.nu):
            du[iu] = h
            dui = data.data_u[iu]
            self.model.calc(dui, x, u + du)
            data.Fu[:, iu] = (np.asarray(dui.xout, float) - xn0) / h
            data.Lu[iu] = (dui.cost - c0) / h
            data.Ru[:, iu] = (np.asarray(dui.r, float) - r0) / h
            du[iu] = 0.0
        if self.withGaussApprox:
            data.Lxx = data.Rx.T @ data.Rx
            data.Lxu = data.Rx.T @ data.Ru
            data.Luu = data.Ru.T @ data.Ru
