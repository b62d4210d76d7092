"""Python-subclassed action models (bindings/python/crocoddyl/core/
action-base.hpp:18-55): a horizon holding any runs knot by knot on the host
(crocoddyl_amd.host), the device-kind knots through one-knot device problems.

The derived models are those of the reference's own binding tests
(bindings/python/crocoddyl/utils/__init__.py UnicycleModelDerived / LQRModelDerived,
used by unittest/bindings/test_actions.py), restated here. CPU tests: all-Python
horizons vs the numpy oracle's solve. GPU tests: a mixed horizon (device unicycle
knots + Python unicycle knots) vs the oracle and vs the all-device solve."""
import numpy as np
import pytest

import crocoddyl_amd as cr
from oracle import fddp_np


class UnicycleModelDerived(cr.ActionModelAbstract):
    def __init__(self):
        cr.ActionModelAbstract.__init__(self, cr.StateVector(3), 2, 5)
        self.dt = .1
        self.costWeights = [10., 1.]

    def calc(self, data, x, u=None):
        if u is None:
            u = self.unone
        v, w = u
        px, py, theta = x
        c, s, dt = np.cos(theta), np.sin(theta), self.dt
        data.xnext[0] = px + c * v * dt
        data.xnext[1] = py + s * v * dt
        data.xnext[2] = theta + w * dt
        data.r[:3] = self.costWeights[0] * x
        data.r[3:] = self.costWeights[1] * u
        data.cost = .5 * sum(data.r**2)

    def calcDiff(self, data, x, u=None):
        if u is None:
            u = self.unone
        v = u[0]
        theta = x[2]
        data.Lx[:] = x * ([self.costWeights[0]**2] * self.state.nx)
        data.Lu[:] = u * ([self.costWeights[1]**2] * self.nu)
        c, s, dt = np.cos(theta), np.sin(theta), self.dt
        data.Fx[0, 2] = -s * v * dt
        data.Fx[1, 2] = c * v * dt
        data.Fu[0, 0] = c * dt
        data.Fu[1, 0] = s * dt
        data.Fu[2, 1] = dt

    def createData(self):
        return UnicycleDataDerived(self)


class UnicycleDataDerived(cr.ActionDataAbstract):
    def __init__(self, model):
        cr.ActionDataAbstract.__init__(self, model)
        nx, nu = model.state.nx, model.nu
        self.Lxx[range(nx), range(nx)] = [model.costWeights[0]**2] * nx
        self.Luu[range(nu), range(nu)] = [model.costWeights[1]**2] * nu
        self.Fx[0, 0] = 1
        self.Fx[1, 1] = 1
        self.Fx[2, 2] = 1


class LQRModelDerived(cr.ActionModelAbstract):
    def __init__(self, nx, nu):
        cr.ActionModelAbstract.__init__(self, cr.StateVector(nx), nu)
        self.Fx = np.eye(self.state.nx)
        self.Fu = np.eye(self.state.nx)[:, :self.nu]
        self.f0 = np.zeros(self.state.nx)
        self.Lxx = np.eye(self.state.nx)
        self.Lxu = np.eye(self.state.nx)[:, :self.nu]
        self.Luu = np.eye(self.nu)
        self.lx = np.ones(self.state.nx)
        self.lu = np.ones(self.nu)

    def calc(self, data, x, u=None):
        if u is None:
            u = self.unone
        data.xnext[:] = np.dot(self.Fx, x) + np.dot(self.Fu, u) + self.f0
        data.cost = 0.5 * np.dot(x.T, np.dot(self.Lxx, x))
        data.cost += 0.5 * np.dot(u.T, np.dot(self.Luu, u))
        data.cost += np.dot(x.T, np.dot(self.Lxu, u))
        data.cost += np.dot(self.lx.T, x) + np.dot(self.lu.T, u)

    def calcDiff(self, data, x, u=None):
        if u is None:
            u = self.unone
        data.Lx[:] = self.lx + np.dot(self.Lxx, x) + np.dot(self.Lxu, u)
        data.Lu[:] = self.lu + np.dot(self.Lxu.T, x) + np.dot(self.Luu, u)

    def createData(self):
        data = cr.ActionDataAbstract(self)
        data.Fx[:] = self.Fx
        data.Fu[:] = self.Fu
        data.Lxx[:] = self.Lxx
        data.Luu[:] = self.Luu
        data.Lxu[:] = self.Lxu
        return data


class PyKnot:
    """The numpy oracle's knot interface over a Python-defined model (checker side)."""

    def __init__(self, m):
        self.m, self.nx, self.ndx, self.nu = m, m.state.nx, m.state.ndx, m.nu
        self.d = m.createData()

    def state_zero(self):
        return np.zeros(self.nx)

    def state_diff(self, x0, x1):
        return x1 - x0

    def state_integrate(self, x, dx):
        return x + dx

    def calc(self, x, u=None):
        self.m.calc(self.d, x) if u is None else self.m.calc(self.d, x, u)
        return np.array(self.d.xnext, float), float(self.d.cost)

    def calc_diff(self, x, u=None):
        self.calc(x, u)
        self.m.calcDiff(self.d, x) if u is None else self.m.calcDiff(self.d, x, u)
        return {k: np.array(getattr(self.d, k), float) for k in ("Fx", "Fu", "Lx", "Lu", "Lxx", "Lxu", "Luu")}


def _oracle_knot(model):
    if getattr(model, "kind", None) is None:
        return PyKnot(model)
    knots, pool = cr.pack_problem([model], model, 1)
    return fddp_np.bind_problem(knots, pool, 0, model.state.nx)[0]


def _solve_both(running, terminal, x0, maxiter=20):
    problem = cr.ShootingProblem(x0, running, terminal)
    assert problem.host_mode
    solver = cr.SolverFDDP(problem)
    conv = solver.solve([], [], maxiter)
    ref = fddp_np.FDDP(x0, [_oracle_knot(m) for m in running] + [_oracle_knot(terminal)])
    rconv = ref.solve(None, None, maxiter=maxiter)
    return solver, conv, ref, rconv


def test_all_python_unicycle_horizon_matches_oracle():
    m = UnicycleModelDerived()
    x0 = np.array([-1.0, -1.0, 1.0])
    solver, conv, ref, rconv = _solve_both([m] * 20, m, x0)
    assert conv and rconv
    assert solver.iter == ref.iter
    assert solver.cost == pytest.approx(ref.cost, rel=1e-10)
    np.testing.assert_allclose(np.array(solver.xs), np.array(ref.xs), atol=1e-10)
    np.testing.assert_allclose(np.array(solver.us), np.array(ref.us), atol=1e-10)


def test_all_python_lqr_horizon_one_newton_step():
    """LQR: FDDP converges in one step (unittest/bindings/test_solvers.py pattern)."""
    m = LQRModelDerived(6, 3)
    x0 = np.linspace(-1, 1, 6)
    solver, conv, ref, rconv = _solve_both([m] * 10, m, x0)
    assert conv and rconv and solver.iter == ref.iter == 1
    np.testing.assert_allclose(np.array(solver.xs), np.array(ref.xs), atol=1e-10)


def test_host_problem_calc_and_rollout():
    m = UnicycleModelDerived()
    x0 = np.array([0.5, -0.3, 0.2])
    problem = cr.ShootingProblem(x0, [m] * 5, m)
    us = [np.array([1.0, 0.5])] * 5
    xs = problem.rollout(us)
    k = PyKnot(m)
    x = x0
    for t in range(5):
        x, _ = k.calc(x, us[t])
        np.testing.assert_allclose(xs[t + 1], x, atol=1e-14)
    c = problem.calcDiff(xs, us)
    assert c == pytest.approx(sum(k.calc(xs[t], us[t])[1] for t in range(5)) + k.calc(xs[5])[1], rel=1e-12)
    np.testing.assert_allclose(problem.runningDatas[2].Fu, k.calc_diff(xs[2], us[2])["Fu"])


def test_host_mode_rejections():
    m = UnicycleModelDerived()
    with pytest.raises(ValueError):
        cr.ShootingProblem(np.zeros((2, 3)), [m] * 3, m)  # batched x0
    problem = cr.ShootingProblem(np.zeros(3), [m] * 3, m)
    with pytest.raises(NotImplementedError):
        cr.SolverBoxFDDP(problem)
    dev = cr.ShootingProblem(np.zeros(3), [cr.ActionModelUnicycle()] * 3, cr.ActionModelUnicycle())
    with pytest.raises(ValueError):
        dev.circularAppend(m)


@pytest.mark.gpu
def test_mixed_horizon_matches_oracle_and_device_solve():
    """Device unicycle knots interleaved with the Python-derived unicycle: the host
    solve equals the numpy oracle's, and the all-device solve of the same horizon."""
    py, dev = UnicycleModelDerived(), cr.ActionModelUnicycle()
    running = [dev if t % 3 else py for t in range(12)]
    x0 = np.array([-1.0, 0.5, 0.7])
    solver, conv, ref, rconv = _solve_both(running, dev, x0, maxiter=100)  # 31 iterations
    assert conv and rconv and solver.iter == ref.iter
    assert solver.cost == pytest.approx(ref.cost, rel=1e-9)
    np.testing.assert_allclose(np.array(solver.xs), np.array(ref.xs), atol=1e-9)
    np.testing.assert_allclose(np.array(solver.us), np.array(ref.us), atol=1e-9)
    full = cr.SolverFDDP(cr.ShootingProblem(x0, [dev] * 12, dev))
    assert full.solve([], [], 100)
    assert full.iter == solver.iter
    np.testing.assert_allclose(np.array(full.xs), np.array(solver.xs), atol=1e-9)


def test_host_solver_callbacks_per_iteration():
    """CallbackLogger / CallbackVerbose on the host path (Python-defined models): one
    record per iteration (fddp.cpp:92-98), the last equal to the solve's final state."""
    import io
    m = UnicycleModelDerived()
    problem = cr.ShootingProblem(np.array([-1.0, -1.0, 1.0]), [m] * 20, m)
    solver = cr.SolverFDDP(problem)
    log = cr.CallbackLogger()
    buf = io.StringIO()
    solver.setCallbacks([log, cr.CallbackVerbose(stream=buf)])
    assert solver.solve([], [], 50)
    assert log.iters == list(range(solver.iter + 1))
    assert log.costs[-1] == solver.cost and log.x_regs[-1] == solver.x_reg
    assert all(np.isfinite(log.grads)) and len(log.fs) == len(log.iters)
    assert buf.getvalue().count("\n") == len(log.iters) + (len(log.iters) + 9) // 10
