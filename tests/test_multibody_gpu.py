"""Multibody knots on the GPU (Euler ∘ DifferentialActionModelFreeFwdDynamics,
crocoddyl_amd/csrc/multibody.hpp) vs the numpy oracle (oracle/multibody_np.py:
ABA + complex-step derivatives, an independent algorithm).

Bars: calc (xnext, knot costs) and calcDiff blocks within 1e-9 relative
(different algorithms for the same functions: GPU CRBA + Gauss-Jordan +
linearised RNEA vs oracle ABA + complex step); full solves with identical
statuses / iteration counts and xs, us, cost within 1e-6 relative (the
north-star tolerance). Parity against Pinocchio itself is unpinned offline
(see oracle/multibody_np.py)."""
import numpy as np
import pytest

import helpers
from crocoddyl_amd import _abi, multibody as mb, synthetic
from crocoddyl_amd.problem import pack_problem
from oracle import fddp_np

pytestmark = pytest.mark.gpu
SOLVE_TOL = 1e-8  # element-wise (helpers.elem_err), converged solves vs the numpy oracle


def _setup(T, B, **kw):
    x0s, running, terminal = synthetic.build_arm(T=T, B=B, **kw)
    knots, pool = pack_problem(running, terminal, B)
    nx = running[0].state.nx
    dims = _abi.Dims(nx, nx, running[0].nu, T, B)
    g = helpers.Gpu(dims, knots, pool, x0s)
    models = [fddp_np.bind_problem(knots, pool, b, nx) for b in range(B)]
    return g, models, x0s, dims


def _candidate(dims, x0s, seed):
    rng = np.random.default_rng(seed)
    xs = np.repeat(x0s[:, None, :], dims.T + 1, axis=1) + 0.1 * rng.standard_normal((dims.B, dims.T + 1, dims.nx))
    us = rng.uniform(-2, 2, (dims.B, dims.T, dims.nu_max))
    return xs, us


CASES = [dict(), dict(weighted=True), dict(robot=mb.sample_tree(6, seed=4), weighted=True),
         dict(robot=mb.sample_tree(9, seed=8, branching=False), armature=np.full(9, 0.05))]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_calc_and_calc_diff(case):
    g, models, x0s, d = _setup(6, 3, **CASES[case])
    xs, us = _candidate(d, x0s, case)
    g.set_candidate(xs, us)
    cost = g.calc()
    xn = g.quantity(_abi.Q_XNEXT, d.T, d.nx)
    g.calc_diff()
    n, m = d.nx, d.nu_max
    Q = {k: g.quantity(q, d.T + 1, s) for k, q, s in [("Fx", _abi.Q_FX, n * n), ("Fu", _abi.Q_FU, n * m),
                                                      ("Lxx", _abi.Q_LXX, n * n), ("Lxu", _abi.Q_LXU, n * m),
                                                      ("Luu", _abi.Q_LUU, m * m), ("Lx", _abi.Q_LX, n),
                                                      ("Lu", _abi.Q_LU, m)]}
    for b in range(d.B):
        ctot = 0.0
        for t in range(d.T + 1):
            k = models[b][t]
            u = us[b, t] if t < d.T else None
            xo, co = k.calc(xs[b, t], u)
            ctot += co
            if t < d.T:
                assert helpers.rel_err(xn[b, t], xo) < 1e-12, (b, t)
            ref = k.calc_diff(xs[b, t], u)
            for name, shape in [("Fx", (n, n)), ("Fu", (n, m)), ("Lxx", (n, n)), ("Lxu", (n, m)),
                                ("Luu", (m, m)), ("Lx", (n,)), ("Lu", (m,))]:
                got = Q[name][b, t].reshape(shape[::-1]).T if len(shape) == 2 else Q[name][b, t]
                err = helpers.rel_err(got, ref[name])
                assert err < 1e-9, (case, b, t, name, err)
        assert abs(cost[b] - ctot) <= 1e-10 * max(1.0, abs(ctot)), (b, cost[b], ctot)


@pytest.mark.parametrize("case", [0, 1, 3])
def test_solve_vs_oracle(case):
    """Full solves to convergence (5-19 iterations). dt = 1e-2 and xReg / uReg
    weights 1e-2: the factory's 1e-4 weights over a short horizon make Quu so
    ill-conditioned (Luu ~ 1e-7) that the iterates are chaotic and
    rounding-level differences (Gauss-Jordan vs LLT, CRBA vs ABA) are amplified
    without bound; that regime is covered step by step in test_steps_vs_oracle."""
    T, B = 20, 2
    g, models, x0s, d = _setup(T, B, dt=1e-2, w_x=1e-2, w_u=1e-2, **CASES[case])
    g.set_candidate(np.repeat(x0s[:, None, :], T + 1, axis=1), None)
    r = helpers.results_dict(g.solve(maxiter=25, is_feasible=False, reg_init=1e-9))
    xs_g, us_g = g.xs(), g.us()
    for b in range(B):
        o = fddp_np.FDDP(x0s[b], models[b])
        conv = o.solve([x0s[b]] * (T + 1), None, maxiter=25, is_feasible=False, reg_init=1e-9)
        assert conv
        assert r["iter"][b] == o.iter, (b, r["iter"][b], o.iter)
        assert bool(r["status"][b] == _abi.STATUS_CONVERGED) == bool(conv)
        helpers.parity(f"arm case {case} b{b} cost", [r["cost"][b]], [o.cost], SOLVE_TOL)
        helpers.parity(f"arm case {case} b{b} xs", xs_g[b], np.array(o.xs), SOLVE_TOL)
        helpers.parity(f"arm case {case} b{b} us", us_g[b], np.array(o.us), SOLVE_TOL)


def test_facade_arm_solve_and_mpc():
    """Python facade on the arm problem: a batched solve, then warm-started
    MPC steps (solve(maxiter=1, regInit=0.1) after the device shift); every
    element's cost must not increase across the first solve's iterations."""
    import crocoddyl_amd as crocoddyl
    x0s, running, terminal = synthetic.build_arm(T=40, B=16)
    problem = crocoddyl.ShootingProblem(x0s, running, terminal)
    solver = crocoddyl.SolverFDDP(problem)
    solver.solve([], [], 30)
    c0 = np.array(solver.cost)
    assert np.all(np.isfinite(c0))
    xs = solver.xs
    assert np.all(np.isfinite(xs))
    # the gripper approaches the target: the final frame cost is below the initial one
    problem2 = crocoddyl.ShootingProblem(x0s, running, terminal)
    s2 = crocoddyl.SolverFDDP(problem2)
    s2.solve([], [], 1)
    assert np.all(c0 <= np.array(s2.cost) + 1e-9)


@pytest.mark.parametrize("case", [0, 3])
def test_steps_vs_oracle(case):
    """Step API (unittest/bindings/test_solvers.py:38-96 design): direction
    (gains), tryStep(1) / tryStep(0.5) trials and the trial trajectories."""
    T, B = 8, 2
    g, models, x0s, d = _setup(T, B, dt=1e-2, **CASES[case])
    xs, us = _candidate(d, x0s, 10 + case)
    g.set_candidate(xs, us)
    g.set_solver_state(0, 1e-6, 1e-6, 0)
    st = g.compute_direction(True)
    assert np.all(st == 0)
    Kg = g.quantity(_abi.Q_K, T, d.nu_max * d.nx)
    kg = g.quantity(_abi.Q_KV, T, d.nu_max)
    for b in range(B):
        o = fddp_np.FDDP(x0s[b], models[b])
        o.set_candidate(list(xs[b]), list(us[b]), False)
        o.xreg = o.ureg = 1e-6
        assert o.compute_direction(True)
        for t in range(T):
            assert helpers.rel_err(Kg[b, t].reshape(d.nx, d.nu_max).T, o.K[t]) < 1e-8, (b, t)
            assert helpers.rel_err(kg[b, t], o.k[t]) < 1e-8, (b, t)
    for alpha in (1.0, 0.5):
        dV, st = g.try_step(alpha)
        xt, ut = g.xs(trial=True), g.us(trial=True)
        for b in range(B):
            o = fddp_np.FDDP(x0s[b], models[b])
            o.set_candidate(list(xs[b]), list(us[b]), False)
            o.xreg = o.ureg = 1e-6
            o.compute_direction(True)
            dVo = o.try_step(alpha)
            assert st[b] == 0
            assert helpers.rel_err(xt[b], np.array(o.xs_try)) < 1e-8, (alpha, b)
            assert helpers.rel_err(ut[b], np.array(o.us_try)) < 1e-8, (alpha, b)
            assert abs(dV[b] - dVo) <= 1e-8 * max(1.0, abs(dVo)), (alpha, b, dV[b], dVo)


def test_full_size_c3_vs_cpp_oracle():
    """C3 at full size (7-DoF arm, T = 250, B = 512, the factory's weights):
    a warm-started MPC step (solve(maxiter=1, regInit=0.1)) of every element;
    all finite, and spot elements identical to the C++ oracle (identical
    branch decisions, xs / us / cost within 1e-6)."""
    import oracle_lib
    x0s, running, terminal = synthetic.build("C3_arm_multibody")
    B, T = x0s.shape[0], len(running)
    knots, pool = pack_problem(running, terminal, B)
    d = _abi.Dims(14, 14, 7, T, B)
    g = helpers.Gpu(d, knots, pool, x0s)
    g.set_candidate(None, None)
    r = helpers.results_dict(g.solve(maxiter=1, is_feasible=False, reg_init=0.1))
    xs, us = g.xs(), g.us()
    assert np.all(np.isfinite(r["cost"])) and np.all(np.isfinite(xs)) and np.all(np.isfinite(us))
    spots = [0, 1, 257, B - 1]
    sub = np.array(spots)
    ds = _abi.Dims(14, 14, 7, T, len(spots))
    ks, ps = pack_problem(running, terminal, len(spots))
    o = oracle_lib.Oracle(ds, ks, ps, x0s[sub], threads=4)
    o.set_candidate(None, None, False)
    ro = o.solve(maxiter=1, is_feasible=False, reg_init=0.1)
    xo, uo = o.xs(), o.us()
    for i, b in enumerate(spots):
        assert r["steplength"][b] == ro[i].steplength and r["status"][b] == ro[i].status
    helpers.parity("C3 full-size cost", r["cost"][sub], np.array([x.cost for x in ro]), 1e-8)
    helpers.parity("C3 full-size xs", xs[sub], xo, 1e-8)
    helpers.parity("C3 full-size us", us[sub], uo, 1e-8)
