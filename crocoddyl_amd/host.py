"""Python-subclassed action models: the host path of a horizon that holds any.

The reference lets Python classes derive from ActionModelAbstract and override
calc / calcDiff (bindings/python/crocoddyl/core/action-base.hpp:18-55,
ActionModelAbstract_wrap); ShootingProblem and SolverFDDP then call them knot by
knot. Such a model has no device kind, so a problem containing one runs on the
host, knot by knot, exactly as the reference does:

  * Python knots: the user's calc(data, x, u) / calcDiff(data, x, u) on an
    ActionData (action-base.hpp:101-142);
  * device-kind knots (ActionModelLQR, unicycle, multibody ...): a one-knot
    device problem per model (libfddp_hip, fddp_problem_calc / calc_diff at
    (x, u), the knot cost from FDDP_Q_COST), so the same HIP kernels evaluate them;
  * the solver: SolverFDDP's loop (fddp.cpp:19-225, ddp.cpp:120-310) on numpy.

This is product code (no oracle); it is meant for the reference's Python-model
workflows (prototyping a model before it gets a device kind), not for speed. One
problem per ShootingProblem (B = 1), like the reference.
"""
import numpy as np

from . import _abi
from ._lib import check, lib


def is_host_model(model):
    """A Python-defined action model: no device kind, its own calc / calcDiff."""
    return getattr(model, "kind", None) is None


class DeviceKnot:
    """calc / calcDiff of one device-kind model at a single (x, u), through a
    one-knot device problem whose knot 0 is the model as a running node and knot
    1 the same model as a terminal node."""

    def __init__(self, model, device):
        from .problem import ShootingProblem
        self.model = model
        x0 = model.state.zero()
        self.p = ShootingProblem(x0, [model], model, device=device)
        self.nu = model.nu

    def _costs(self):
        kc = np.zeros((1, 2))
        check(lib().fddp_get_quantity(self.p._calc_handle(), _abi.Q_COST, _abi.dptr(kc)))
        return kc[0]

    def _run(self, x, u, diff):
        u = np.zeros(self.nu) if u is None else u
        xs, us = [np.asarray(x, float), np.asarray(x, float)], [np.asarray(u, float)]
        if diff:
            self.p.calcDiff(xs, us)
        else:
            self.p.calc(xs, us)
        return self._costs()

    @staticmethod
    def _copy(dst, src, diff, running):
        if running:
            dst.xnext = np.array(src.xnext, copy=True)
        if diff:
            for f in ("Fx", "Fu", "Lxx", "Lxu", "Luu", "Lx", "Lu"):
                setattr(dst, f, np.array(getattr(src, f), copy=True))

    def calc(self, data, x, u=None, terminal=False):
        c = self._run(x, u, False)
        src = self.p.terminalData if terminal else self.p.runningDatas[0]
        self._copy(data, src, False, not terminal)
        data.cost = float(c[1] if terminal else c[0])

    def calcDiff(self, data, x, u=None, terminal=False):
        c = self._run(x, u, True)
        src = self.p.terminalData if terminal else self.p.runningDatas[0]
        self._copy(data, src, True, not terminal)
        data.cost = float(c[1] if terminal else c[0])


class HostProblem:
    """The knot-by-knot ShootingProblem (shooting.hxx:133-223) of a host-mode problem."""

    def __init__(self, problem):
        self.pb = problem
        self._dev = {}

    def _knot(self, model):
        if is_host_model(model):
            return None
        k = self._dev.get(id(model))
        if k is None or k.model is not model:
            k = self._dev[id(model)] = DeviceKnot(model, self.pb.device)
        return k

    def calc_node(self, model, data, x, u=None, terminal=False, diff=False):
        k = self._knot(model)
        if k is not None:
            (k.calcDiff if diff else k.calc)(data, x, u, terminal)
        elif diff:  # shooting.hxx:164-195: calcDiff only; the cost is the last calc's
            model.calcDiff(data, x) if u is None else model.calcDiff(data, x, u)
        else:
            model.calc(data, x) if u is None else model.calc(data, x, u)

    def calc(self, xs, us, diff=False):
        pb = self.pb
        total = 0.0
        for t, (m, d) in enumerate(zip(pb._models, pb.runningDatas)):
            self.calc_node(m, d, xs[t], us[t] if m.nu else None, diff=diff)
            total += d.cost
        self.calc_node(pb._terminal, pb.terminalData, xs[-1], None, terminal=True, diff=diff)
        total += pb.terminalData.cost
        return float(total)

    def rollout(self, us):
        pb = self.pb
        xs = [pb._x0b[0].copy()]
        for t, (m, d) in enumerate(zip(pb._models, pb.runningDatas)):
            self.calc_node(m, d, xs[t], us[t] if m.nu else None)
            xs.append(np.array(d.xnext, float))
        return xs


def _raise_if_nan(v):  # solver-base.cpp:175-181
    return bool(np.isnan(v) or np.isinf(v) or v >= 1e30)


class HostSolverFDDP:
    """SolverFDDP (fddp.cpp:19-225 on ddp.cpp:120-310) for a host-mode problem."""

    def __init__(self, problem):
        from .problem import default_params
        self.problem = problem
        self._hp = HostProblem(problem)
        p = default_params()
        self.th_acceptstep, self.th_stop, self.th_grad = p.th_acceptstep, p.th_stop, p.th_grad
        self.th_stepdec, self.th_stepinc, self.th_acceptnegstep = p.th_stepdec, p.th_stepinc, p.th_acceptnegstep
        self.regfactor, self.regmin, self.regmax = p.regfactor, p.regmin, p.regmax
        self.alphas = [float(p.alphas[i]) for i in range(p.n_alphas)]
        T, models = problem.T, problem._models
        n = problem.ndx
        self.xs = [m.state.zero() for m in models] + [problem._terminal.state.zero()]
        self.us = [np.zeros(m.nu) for m in models]
        self.xs_try = [x.copy() for x in self.xs]
        self.us_try = [u.copy() for u in self.us]
        self.fs = [np.zeros(n) for _ in range(T + 1)]
        self.dx = [np.zeros(n) for _ in range(T + 1)]
        self.Vxx = [np.zeros((n, n)) for _ in range(T + 1)]
        self.Vx = [np.zeros(n) for _ in range(T + 1)]
        self.Qxx = [np.zeros((n, n)) for _ in range(T)]
        self.Qx = [np.zeros(n) for _ in range(T)]
        self.Qxu = [np.zeros((n, m.nu)) for m in models]
        self.Quu = [np.zeros((m.nu, m.nu)) for m in models]
        self.Qu = [np.zeros(m.nu) for m in models]
        self.K = [np.zeros((m.nu, n)) for m in models]
        self.k = [np.zeros(m.nu) for m in models]
        self.Quuk = [np.zeros(m.nu) for m in models]
        self.isFeasible = self.was_feasible = False
        self.cost = self.cost_try = self.stop = 0.0
        self.xreg = self.ureg = float("nan")
        self.stepLength = 1.0
        self.iter = 0
        self.dV = self.dVexp = self.dg = self.dq = self.dv = 0.0
        self.d = np.zeros(2)
        self.callbacks = []

    # -- solver-base.cpp:42-67 ----------------------------------------------------
    def setCandidate(self, xs=[], us=[], isFeasible=False):
        pb = self.problem
        if xs is not None and len(xs) > 0:
            if len(xs) != pb.T + 1:
                raise ValueError(f"Invalid argument: xs has wrong dimension (it should be {pb.T + 1})")
            self.xs = [np.array(x, float) for x in xs]
        else:
            self.xs = [m.state.zero() for m in pb._models] + [pb._terminal.state.zero()]
        if us is not None and len(us) > 0:
            if len(us) != pb.T:
                raise ValueError(f"Invalid argument: us has wrong dimension (it should be {pb.T})")
            self.us = [np.array(u, float)[:m.nu] for u, m in zip(us, pb._models)]
        else:
            self.us = [np.zeros(m.nu) for m in pb._models]
        self.isFeasible = bool(isFeasible)

    def setCallbacks(self, callbacks):
        self.callbacks = list(callbacks)

    def getCallbacks(self):
        return list(self.callbacks)

    # the reference's Python names of xreg_ / ureg_ (core/solver-base.cpp:100-126)
    x_reg = property(lambda s: s.xreg, lambda s, v: setattr(s, "xreg", float(v)))
    u_reg = property(lambda s: s.ureg, lambda s, v: setattr(s, "ureg", float(v)))

    # -- ddp.cpp -------------------------------------------------------------------
    def _increase_reg(self):
        self.xreg = min(self.xreg * self.regfactor, self.regmax)
        self.ureg = self.xreg

    def _decrease_reg(self):
        self.xreg = max(self.xreg / self.regfactor, self.regmin)
        self.ureg = self.xreg

    def calcDiff(self):
        pb, hp = self.problem, self._hp
        if self.iter == 0:
            hp.calc(self.xs, self.us)
        self.cost = hp.calc(self.xs, self.us, diff=True)
        if not self.isFeasible:
            st = pb._models[0].state
            self.fs[0] = st.diff(self.xs[0], pb._x0b[0])
            for t, (m, d) in enumerate(zip(pb._models, pb.runningDatas)):
                self.fs[t + 1] = m.state.diff(self.xs[t + 1], d.xnext)
        elif not self.was_feasible:
            for f in self.fs:
                f[:] = 0.0
        return self.cost

    def _gains(self, t):  # ddp.cpp:298-310 (Eigen LLT)
        try:
            L = np.linalg.cholesky(self.Quu[t])
        except np.linalg.LinAlgError:
            raise RuntimeError("backward_error")
        self.K[t] = np.linalg.solve(L.T, np.linalg.solve(L, self.Qxu[t].T))
        self.k[t] = np.linalg.solve(L.T, np.linalg.solve(L, self.Qu[t]))

    def backwardPass(self):
        pb = self.problem
        dT = pb.terminalData
        n = pb.ndx
        self.Vxx[-1] = np.array(dT.Lxx, float).copy()
        self.Vx[-1] = np.array(dT.Lx, float).copy()
        if not np.isnan(self.xreg):
            self.Vxx[-1][np.diag_indices(n)] += self.xreg
        if not self.isFeasible:
            self.Vx[-1] = self.Vx[-1] + self.Vxx[-1] @ self.fs[-1]
        for t in range(pb.T - 1, -1, -1):
            m, d = pb._models[t], pb.runningDatas[t]
            Vxx_p, Vx_p = self.Vxx[t + 1], self.Vx[t + 1]
            FxTVxx = d.Fx.T @ Vxx_p
            self.Qxx[t] = d.Lxx + FxTVxx @ d.Fx
            self.Qx[t] = d.Lx + d.Fx.T @ Vx_p
            if m.nu:
                self.Qxu[t] = d.Lxu + FxTVxx @ d.Fu
                self.Quu[t] = d.Luu + (d.Fu.T @ Vxx_p) @ d.Fu
                self.Qu[t] = d.Lu + d.Fu.T @ Vx_p
                if not np.isnan(self.ureg):
                    self.Quu[t][np.diag_indices(m.nu)] += self.ureg
                self._gains(t)
            Vx = self.Qx[t].copy()
            Vxx = self.Qxx[t].copy()
            if m.nu:
                if np.isnan(self.ureg):
                    Vx = Vx - self.K[t].T @ self.Qu[t]
                else:
                    self.Quuk[t] = self.Quu[t] @ self.k[t]
                    Vx = Vx + self.K[t].T @ self.Quuk[t]
                    Vx = Vx - 2 * (self.K[t].T @ self.Qu[t])
                Vxx = Vxx - self.Qxu[t] @ self.K[t]
            Vxx = 0.5 * (Vxx + Vxx.T)
            if not np.isnan(self.xreg):
                Vxx[np.diag_indices(n)] += self.xreg
            if not self.isFeasible:
                Vx = Vx + Vxx @ self.fs[t]
            self.Vx[t], self.Vxx[t] = Vx, Vxx
            if _raise_if_nan(np.max(np.abs(Vx))) or _raise_if_nan(np.max(np.abs(Vxx))):
                raise RuntimeError("backward_error")

    def computeDirection(self, recalc=True):
        if recalc:
            self.calcDiff()
        self.backwardPass()

    def stoppingCriteria(self):
        self.stop = float(sum(float(self.Qu[t] @ self.Qu[t]) for t, m in enumerate(self.problem._models) if m.nu))
        return self.stop

    # -- fddp.cpp:107-225 ------------------------------------------------------------
    def updateExpectedImprovement(self):
        pb = self.problem
        self.dg = self.dq = 0.0
        if not self.isFeasible:
            self.dg -= float(self.Vx[-1] @ self.fs[-1])
            self.dq += float(self.fs[-1] @ (self.Vxx[-1] @ self.fs[-1]))
        for t, m in enumerate(pb._models):
            if m.nu:
                self.dg += float(self.Qu[t] @ self.k[t])
                self.dq -= float(self.k[t] @ self.Quuk[t])
            if not self.isFeasible:
                self.dg -= float(self.Vx[t] @ self.fs[t])
                self.dq += float(self.fs[t] @ (self.Vxx[t] @ self.fs[t]))

    def expectedImprovement(self):
        pb = self.problem
        self.dv = 0.0
        if not self.isFeasible:
            dx = pb._terminal.state.diff(self.xs_try[-1], self.xs[-1])
            self.dv -= float(self.fs[-1] @ (self.Vxx[-1] @ dx))
            for t, m in enumerate(pb._models):
                dx = m.state.diff(self.xs_try[t], self.xs[t])
                self.dv -= float(self.fs[t] @ (self.Vxx[t] @ dx))
        self.d = np.array([self.dg + self.dv, self.dq - 2 * self.dv])
        return self.d

    def forwardPass(self, steplength):
        if steplength > 1.0 or steplength < 0.0:
            raise ValueError("Invalid argument: invalid step length, value is between 0. to 1.")
        pb, hp = self.problem, self._hp
        self.cost_try = 0.0
        xnext = pb._x0b[0].copy()
        full = self.isFeasible or steplength == 1
        for t, (m, d) in enumerate(zip(pb._models, pb.runningDatas)):
            self.xs_try[t] = xnext if full else m.state.integrate(xnext, self.fs[t] * (steplength - 1))
            self.dx[t] = m.state.diff(self.xs[t], self.xs_try[t])
            if m.nu:
                self.us_try[t] = self.us[t] - self.k[t] * steplength - self.K[t] @ self.dx[t]
                hp.calc_node(m, d, self.xs_try[t], self.us_try[t])
            else:
                hp.calc_node(m, d, self.xs_try[t], None)
            xnext = np.array(d.xnext, float)
            self.cost_try += d.cost
            if _raise_if_nan(self.cost_try) or _raise_if_nan(np.max(np.abs(xnext))):
                raise RuntimeError("forward_error")
        m, d = pb._terminal, pb.terminalData
        self.xs_try[-1] = xnext if full else m.state.integrate(xnext, self.fs[-1] * (steplength - 1))
        hp.calc_node(m, d, self.xs_try[-1], None, terminal=True)
        self.cost_try += d.cost
        if _raise_if_nan(self.cost_try):
            raise RuntimeError("forward_error")

    def tryStep(self, stepLength=1.0):
        self.forwardPass(stepLength)
        return self.cost - self.cost_try

    def solve(self, init_xs=[], init_us=[], maxiter=100, isFeasible=False, regInit=1e-9):
        pb = self.problem
        self.xs_try[0] = pb._x0b[0].copy()
        self.setCandidate(init_xs, init_us, isFeasible)
        self.xreg = self.ureg = self.regmin if regInit is None or np.isnan(regInit) else float(regInit)
        self.was_feasible = False
        recalc = True
        for self.iter in range(maxiter):
            while True:
                try:
                    self.computeDirection(recalc)
                except RuntimeError:
                    recalc = False
                    self._increase_reg()
                    if self.xreg == self.regmax:
                        return False
                    continue
                break
            self.updateExpectedImprovement()
            recalc = False
            for a in self.alphas:
                self.stepLength = a
                try:
                    self.dV = self.tryStep(a)
                except RuntimeError:
                    continue
                self.expectedImprovement()
                self.dVexp = a * (self.d[0] + 0.5 * a * self.d[1])
                if self.dVexp >= 0:
                    accept = self.d[0] < self.th_grad or self.dV > self.th_acceptstep * self.dVexp
                else:
                    accept = self.dV > self.th_acceptnegstep * self.dVexp
                if accept:
                    self.was_feasible = self.isFeasible
                    self.setCandidate([x.copy() for x in self.xs_try], [u.copy() for u in self.us_try],
                                      self.was_feasible or a == 1)
                    self.cost = self.cost_try
                    recalc = True
                    break
            if self.stepLength > self.th_stepdec:
                self._decrease_reg()
            if self.stepLength <= self.th_stepinc:
                self._increase_reg()
                if self.xreg == self.regmax:
                    return False
            self.stoppingCriteria()
            for cb in self.callbacks:
                cb(self)
            if self.was_feasible and self.stop < self.th_stop:
                return True
        self.iter = maxiter
        return False
