"""Python-subclassed differential action models (bindings/python/crocoddyl/core/
diff-action-base.hpp:19-35; the reference's own examples use them, e.g.
examples/notebooks/cartpole_swing_up.py:9-11) under IntegratedActionModelEuler,
on the host path (crocoddyl_amd/host.py, models.py), and DifferentialActionModelNumDiff
(core/numdiff/diff-action.hxx).

The bar: a Python restatement of DifferentialActionModelLQR (diff-lqr.hxx:33-78)
integrated by Euler solves exactly as the device-kind Euler ∘ DifferentialActionModelLQR
knot with the same matrices does in the numpy oracle (same iterations, xs / us / cost
within 1e-9); Euler's derivatives match finite differences of its calc; NumDiff's
match the analytic ones to the forward-difference error.

Note on examples/notebooks/cartpole_swing_up_sol.ipynb (a printed `ddp.us`): it is not
used as a pin. Its run is SolverDDP from state.zero() (pole upright, x0 hanging), whose
rollout-first line search and FDDP's gap-keeping one reach different local minima, and it
predates this reference's Euler cost scaling (cost = dt * cost_c, euler.hxx:69): from a
feasible hanging warm start FDDP here lands 1e-5 away from the printed controls."""
import numpy as np
import pytest

import crocoddyl_amd as cr
from oracle import fddp_np


class DiffLQRDerived(cr.DifferentialActionModelAbstract):
    """diff-lqr.hxx:33-78 in Python: a = Fq q + Fv v + Fu u (+ f0), quadratic cost."""

    def __init__(self, nq, nu, rng, drift_free=True):
        cr.DifferentialActionModelAbstract.__init__(self, cr.StateVector(2 * nq), nu)
        nx = 2 * nq
        self.nq, self.drift_free = nq, drift_free
        self.Fq = np.eye(nq) + 0.1 * rng.standard_normal((nq, nq))
        self.Fv = np.eye(nq) + 0.1 * rng.standard_normal((nq, nq))
        self.Fu = np.eye(nq, nu) + 0.1 * rng.standard_normal((nq, nu))
        self.f0 = rng.standard_normal(nq)
        A = rng.standard_normal((nx, nx))
        self.Lxx = A @ A.T / nx + np.eye(nx)
        self.Lxu = 0.1 * rng.standard_normal((nx, nu))
        C = rng.standard_normal((nu, nu))
        self.Luu = C @ C.T / nu + np.eye(nu)
        self.lx = rng.uniform(-1, 1, nx)
        self.lu = rng.uniform(-1, 1, nu)

    def calc(self, data, x, u=None):
        u = self.unone if u is None else u
        q, v = x[:self.nq], x[self.nq:]
        data.xout = self.Fq @ q + self.Fv @ v + self.Fu @ u + (0 if self.drift_free else self.f0)
        data.cost = (0.5 * x @ (self.Lxx @ x) + 0.5 * u @ (self.Luu @ u) + x @ (self.Lxu @ u) + self.lx @ x
                     + self.lu @ u)

    def calcDiff(self, data, x, u=None):
        u = self.unone if u is None else u
        data.Lx = self.lx + self.Lxx @ x + self.Lxu @ u
        data.Lu = self.lu + self.Lxu.T @ x + self.Luu @ u
        data.Fx = np.hstack([self.Fq, self.Fv])
        data.Fu = self.Fu.copy()
        data.Lxx, data.Lxu, data.Luu = self.Lxx, self.Lxu, self.Luu


def _device_twin(py, dt):
    d = cr.DifferentialActionModelLQR(py.nq, py.nu, py.drift_free)
    d.Fq, d.Fv, d.Fu, d.f0 = py.Fq, py.Fv, py.Fu, py.f0
    d.Lxx, d.Lxu, d.Luu, d.lx, d.lu = py.Lxx, py.Lxu, py.Luu, py.lx, py.lu
    return cr.IntegratedActionModelEuler(d, dt)


@pytest.mark.parametrize("drift_free", [True, False])
def test_python_dam_euler_solves_as_the_device_kind_in_the_oracle(drift_free):
    rng = np.random.default_rng(3)
    dam = DiffLQRDerived(4, 3, rng, drift_free)
    dt, T = 0.05, 15
    iam = cr.IntegratedActionModelEuler(dam, dt)
    assert iam.kind is None  # host path
    x0 = rng.uniform(-1, 1, 8)
    problem = cr.ShootingProblem(x0, [iam] * T, iam)
    assert problem.host_mode
    solver = cr.SolverFDDP(problem)
    conv = solver.solve([], [], 50)
    twin = _device_twin(dam, dt)
    knots, pool = cr.pack_problem([twin] * T, twin, 1)
    ref = fddp_np.FDDP(x0, fddp_np.bind_problem(knots, pool, 0, 8))
    rconv = ref.solve(None, None, maxiter=50)
    assert conv and rconv and solver.iter == ref.iter
    assert solver.cost == pytest.approx(ref.cost, rel=1e-9)
    np.testing.assert_allclose(np.array(solver.xs), np.array(ref.xs), atol=1e-9)
    np.testing.assert_allclose(np.array(solver.us), np.array(ref.us), atol=1e-9)


def test_euler_host_derivatives_match_finite_differences():
    rng = np.random.default_rng(4)
    dam = DiffLQRDerived(3, 2, rng, False)
    iam = cr.IntegratedActionModelEuler(dam, 0.1)
    d = iam.createData()
    x, u = rng.uniform(-1, 1, 6), rng.uniform(-1, 1, 2)
    iam.calc(d, x, u)
    iam.calcDiff(d, x, u)
    h = 1e-6
    for i in range(6):
        e = np.zeros(6)
        e[i] = h
        dp, dm = iam.createData(), iam.createData()
        iam.calc(dp, x + e, u)
        iam.calc(dm, x - e, u)
        np.testing.assert_allclose(d.Fx[:, i], (dp.xnext - dm.xnext) / (2 * h), atol=1e-8)
        assert d.Lx[i] == pytest.approx((dp.cost - dm.cost) / (2 * h), abs=1e-7)
    # dt = 0: xnext = x, cost = cost_c (euler.hxx:71-74, 122-130)
    iam0 = cr.IntegratedActionModelEuler(dam, 0.0)
    d0 = iam0.createData()
    iam0.calc(d0, x, u)
    iam0.calcDiff(d0, x, u)
    np.testing.assert_array_equal(d0.xnext, x)
    np.testing.assert_array_equal(d0.Fx, np.eye(6))
    # the terminal form calc(data, x) evaluates at unone (action-base.hxx:28-37)
    dt_, du_ = iam.createData(), iam.createData()
    iam.calc(dt_, x)
    iam.calc(du_, x, np.zeros(2))
    assert dt_.cost == du_.cost


def test_numdiff_matches_analytic():
    rng = np.random.default_rng(5)
    dam = DiffLQRDerived(3, 2, rng, False)
    nd = cr.DifferentialActionModelNumDiff(dam, False)
    assert nd.disturbance == pytest.approx(np.sqrt(2 * np.finfo(float).eps))
    x, u = rng.uniform(-1, 1, 6), rng.uniform(-1, 1, 2)
    dn, da = nd.createData(), dam.createData()
    nd.calc(dn, x, u)
    nd.calcDiff(dn, x, u)
    dam.calc(da, x, u)
    dam.calcDiff(da, x, u)
    assert dn.cost == da.cost
    np.testing.assert_allclose(dn.Fx, da.Fx, atol=1e-6)
    np.testing.assert_allclose(dn.Fu, da.Fu, atol=1e-6)
    np.testing.assert_allclose(dn.Lx, da.Lx, atol=1e-6 * (1 + np.abs(da.Lx).max()))
    np.testing.assert_allclose(dn.Lu, da.Lu, atol=1e-6 * (1 + np.abs(da.Lu).max()))
    with pytest.raises(ValueError):
        class One(cr.DifferentialActionModelAbstract):
            pass
        cr.DifferentialActionModelNumDiff(One(cr.StateVector(2), 1, 1), True)


class CartpoleDerived(cr.DifferentialActionModelAbstract):
    """examples/notebooks/cartpole_swing_up.py's model (np.asscalar -> float)."""

    def __init__(self):
        cr.DifferentialActionModelAbstract.__init__(self, cr.StateVector(4), 1, 6)
        self.m1, self.m2, self.l, self.g = 1., .1, .5, 9.81
        self.costWeights = [1., 1., 0.1, 0.001, 0.001, 1.]

    def calc(self, data, x, u=None):
        u = self.unone if u is None else u
        y, th, ydot, thdot = (float(v) for v in x)
        f = float(u[0])
        m1, m2, l, g = self.m1, self.m2, self.l, self.g
        s, c = np.sin(th), np.cos(th)
        m, mu = m1 + m2, m1 + m2 * s ** 2
        data.xout = np.array([(f + m2 * c * s * g - m2 * l * s * thdot ** 2) / mu,
                              (c * f / l + m * g * s / l - m2 * c * s * thdot ** 2) / mu])
        data.r = np.array(self.costWeights) * np.array([s, 1 - c, y, ydot, thdot, f])
        data.cost = .5 * float(np.sum(data.r ** 2))

    def calcDiff(self, data, x, u=None):
        pass


def test_cartpole_numdiff_gauss_newton_stationary():
    """The notebook's cartpole (NumDiff with the Gauss approximation, Euler dt = 5e-2,
    T = 50) from a feasible hanging rollout: FDDP converges, and the converged
    trajectory is a stationary point of the problem (zero control gradient of the
    rolled-out cost, checked by central differences)."""
    iam = cr.IntegratedActionModelEuler(cr.DifferentialActionModelNumDiff(CartpoleDerived(), True), 5e-2)
    T, x0 = 50, np.array([0., 3.14, 0., 0.])
    problem = cr.ShootingProblem(x0, [iam] * T, iam)
    us0 = [np.zeros(1)] * T
    xs0 = problem.rollout(us0)
    solver = cr.SolverFDDP(problem)
    assert solver.solve(xs0, us0, 100, True)
    us = [np.array(u, float) for u in solver.us]

    def total(us_):
        xs_ = problem.rollout(us_)
        return problem.calc(xs_, us_)

    h = 1e-5
    for t in (0, 10, 25, 49):
        up = [u.copy() for u in us]
        um = [u.copy() for u in us]
        up[t][0] += h
        um[t][0] -= h
        assert abs((total(up) - total(um)) / (2 * h)) < 1e-4
