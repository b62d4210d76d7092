"""Free-flyer (floating-base) problems on the GPU through the C ABI vs the numpy
oracle: StateMultibody on SE(3) x R^n (x = (p, quat xyzw, q, v), nx = ndx + 1),
ActuationModelFloatingBase, Euler ∘ Free / Contact forward dynamics and impulse
knots (crocoddyl_amd/csrc/multibody.hpp, the manifold gaps / rollout / expected
improvement of fddp_kernels.hpp) vs oracle/multibody_np.py + oracle/fddp_np.py.

Bars (north_star): calc / calcDiff blocks within 1e-9 relative; the step API
(gaps on the manifold, tryStep's integrate(xnext, (alpha - 1) fs) and
diff(xs, xs_try), expectedImprovement's diff(xs_try, xs)) within 1e-9; full solves
with identical iteration counts and statuses, xs / us / cost within 1e-6 relative.
Parity against Pinocchio itself is unpinned offline (oracle/multibody_np.py)."""
import numpy as np
import pytest

import helpers
from crocoddyl_amd import _abi, multibody as mb, synthetic
from crocoddyl_amd.problem import pack_problem
from oracle import fddp_np

pytestmark = pytest.mark.gpu
SOLVE_TOL = 1e-8  # element-wise (helpers.elem_err), solves vs the numpy oracle


def _impulse_mid(T, B, seed=0):
    """free flight -> impulse on the tip (nu = 0) -> tip contact, floating base."""
    x0s, run_c, term_c = synthetic.build_floating(T=T, B=B, seed=seed, contacts=[("6d", "tip")], dt=1e-2)
    model = run_c[0].differential.state.pinocchio
    st = run_c[0].differential.state
    _, run_f, _ = synthetic.build_floating(T=T, B=B, seed=seed, robot=model, dt=1e-2)
    imps = mb.ImpulseModelMultiple(st)
    imps.addImpulse("tip", mb.ImpulseModel6D(st, model.getFrameId("tip")))
    costs = mb.CostModelSum(st, 0)
    costs.addCost("xReg", mb.CostModelState(st, 0), 1e-2)
    imp = mb.ActionModelImpulseFwdDynamics(st, imps, costs)
    h = T // 2
    return x0s, run_f[:h] + [imp] + run_c[h + 1:], term_c


def _setup(T, B, impulse=False, **kw):
    if impulse:
        x0s, running, terminal = _impulse_mid(T, B)
    else:
        x0s, running, terminal = synthetic.build_floating(T=T, B=B, **kw)
    st = running[0].state
    knots, pool = pack_problem(running, terminal, B)
    nu_max = max(r.nu for r in running)
    dims = _abi.Dims(st.nx, st.ndx, nu_max, T, B)
    g = helpers.Gpu(dims, knots, pool, x0s)
    models = [fddp_np.bind_problem(knots, pool, b, st.nx) for b in range(B)]
    return g, models, x0s, dims, [r.nu for r in running], st


CASES = [dict(), dict(weighted=True, com=True), dict(contacts=[("6d", "tip")]),
         dict(contacts=[("3d", "tip"), ("3d", "mid_site")], weighted=True, gains=(0.0, 50.0)),
         dict(contacts=[("6d", "tip"), ("3d", "mid_site")], damping=1e-3, com=True, force_costs=True),
         dict(impulse=True)]


def _candidate(st, d, x0s, rng, nus):
    xs = np.zeros((d.B, d.T + 1, d.nx))
    for b in range(d.B):
        for t in range(d.T + 1):
            dx = np.concatenate([rng.uniform(-0.2, 0.2, st.nv), rng.uniform(-0.3, 0.3, st.nv)])
            xs[b, t] = st.integrate(x0s[b], dx)
    us = rng.uniform(-1, 1, (d.B, d.T, d.nu_max))
    for t, nu in enumerate(nus):
        us[:, t, nu:] = 0.0
    return xs, us


@pytest.mark.parametrize("case", range(len(CASES)))
def test_calc_diff_and_gaps(case):
    g, models, x0s, d, nus, st = _setup(6, 2, **CASES[case])
    rng = np.random.default_rng(case)
    xs, us = _candidate(st, d, x0s, rng, nus)
    g.set_candidate(xs, us)
    cost = g.calc()
    xn = g.quantity(_abi.Q_XNEXT, d.T, d.nx)
    g.set_solver_state(it=0)
    status = g.compute_direction(True)  # calcDiff + gaps on the manifold + backward pass
    assert not status.any()
    n, m = d.ndx, d.nu_max
    Q = {k: g.quantity(q, d.T + 1, s) for k, q, s in [("Fx", _abi.Q_FX, n * n), ("Fu", _abi.Q_FU, n * m),
                                                      ("Lxx", _abi.Q_LXX, n * n), ("Lxu", _abi.Q_LXU, n * m),
                                                      ("Luu", _abi.Q_LUU, m * m), ("Lx", _abi.Q_LX, n),
                                                      ("Lu", _abi.Q_LU, m), ("fs", _abi.Q_FS, n)]}
    for b in range(d.B):
        o = fddp_np.FDDP(x0s[b], models[b])
        o.set_candidate(list(xs[b]), [us[b, t, :] for t in range(d.T)])
        o.iter = 0
        o.calc_diff()
        assert abs(cost[b] - o.cost) <= 1e-10 * max(1.0, abs(o.cost))
        for t in range(d.T + 1):
            assert helpers.rel_err(Q["fs"][b, t], o.fs[t]) < 1e-10, (b, t)
            if t < d.T:
                assert helpers.rel_err(xn[b, t], o.xnext[t]) < 1e-10, (b, t)
            ref = o.data[t]
            for name, shape in [("Fx", (n, n)), ("Fu", (n, m)), ("Lxx", (n, n)), ("Lxu", (n, m)),
                                ("Luu", (m, m)), ("Lx", (n,)), ("Lu", (m,))]:
                got = Q[name][b, t].reshape(shape[::-1]).T if len(shape) == 2 else Q[name][b, t]
                want = ref[name]
                if name in ("Fu", "Lxu"):
                    got = got[:, :want.shape[1]]
                elif name == "Luu":
                    got = got[:want.shape[0], :want.shape[0]]
                elif name == "Lu":
                    got = got[:want.shape[0]]
                if want.size == 0:
                    continue
                err = helpers.rel_err(got, want)
                assert err < (1e-8 if models[b][t].kind == 6 else 1e-9), (case, b, t, name, err)


@pytest.mark.parametrize("case", [0, 2, 4])
def test_step_api_on_the_manifold(case):
    """computeDirection from an infeasible candidate, then tryStep(0.5) (xs_try =
    integrate(xnext, -0.5 fs), us_try = us - 0.5 k - K diff(xs, xs_try)) and
    expectedImprovement (diff(xs_try, xs)) vs the oracle."""
    g, models, x0s, d, nus, st = _setup(6, 2, **CASES[case])
    rng = np.random.default_rng(10 + case)
    xs, us = _candidate(st, d, x0s, rng, nus)
    g.set_candidate(xs, us, is_feasible=False)
    g.set_solver_state(it=0, xreg=1e-6, ureg=1e-6)
    assert not g.compute_direction(True).any()
    g.update_expected_improvement()
    dV, stt = g.try_step(0.5)
    assert not stt.any()
    dd = g.expected_improvement()
    xt, ut = g.xs(trial=True), g.us(trial=True)
    for b in range(d.B):
        o = fddp_np.FDDP(x0s[b], models[b])
        o.set_candidate(list(xs[b]), [us[b, t, :] for t in range(d.T)], is_feasible=False)
        o.iter, o.xreg, o.ureg = 0, 1e-6, 1e-6
        assert o.compute_direction(True)
        o.update_expected_improvement()
        dvo = o.try_step(0.5)
        do = o.expected_improvement()
        assert abs(dV[b] - dvo) <= 1e-9 * max(1.0, abs(dvo)), (b, dV[b], dvo)
        assert helpers.rel_err(dd[b], do) < 1e-9, (b, dd[b], do)
        assert helpers.rel_err(xt[b], np.array(o.xs_try)) < 1e-10
        for t in range(d.T):
            assert helpers.rel_err(ut[b, t, :nus[t]], o.us_try[t][:nus[t]]) < 1e-9


@pytest.mark.parametrize("case", [0, 1, 2, 3, 5])
def test_solve_vs_oracle(case):
    """Full solves: identical iteration counts, xs / us / cost within 1e-6."""
    T, B = 10, 2
    g, models, x0s, d, nus, st = _setup(T, B, **CASES[case])
    g.set_candidate(np.repeat(x0s[:, None, :], T + 1, axis=1), None)
    r = helpers.results_dict(g.solve(maxiter=20, is_feasible=False, reg_init=1e-9))
    xs_g, us_g = g.xs(), g.us()
    for b in range(B):
        o = fddp_np.FDDP(x0s[b], models[b])
        conv = o.solve([x0s[b]] * (T + 1), None, maxiter=20, is_feasible=False, reg_init=1e-9)
        assert r["iter"][b] == o.iter, (b, r["iter"][b], o.iter)
        assert bool(r["status"][b] == _abi.STATUS_CONVERGED) == bool(conv)
        helpers.parity(f"freeflyer case {case} b{b} cost", [r["cost"][b]], [o.cost], SOLVE_TOL)
        helpers.parity(f"freeflyer case {case} b{b} xs", xs_g[b], np.array(o.xs), SOLVE_TOL)
        us_o = np.zeros_like(us_g[b])
        for t in range(T):
            u = np.asarray(o.us[t])
            us_o[t, :u.size] = u
        helpers.parity(f"freeflyer case {case} b{b} us", us_g[b], us_o, SOLVE_TOL)
        np.testing.assert_allclose(np.linalg.norm(xs_g[b][:, 3:7], axis=1), 1.0, atol=1e-9)


def test_neutral_candidate():
    """setCandidate with no xs: state.zero() = (neutral (identity quaternion), 0)
    for every knot (solver-base.cpp:46-52, multibody.hxx:42-44)."""
    g, models, x0s, d, nus, st = _setup(4, 2)
    g.set_candidate(None, None)
    xs = g.xs()
    want = st.zero()
    for b in range(d.B):
        for t in range(d.T + 1):
            np.testing.assert_array_equal(xs[b, t], want)


def test_facade_floating_solve():
    """Python facade (crocoddyl.ShootingProblem / SolverFDDP) on a floating-base
    contact problem: a batched solve converges and keeps unit quaternions."""
    import crocoddyl_amd as crocoddyl
    x0s, running, terminal = synthetic.build_floating(T=20, B=16, contacts=[("6d", "tip")], com=True)
    problem = crocoddyl.ShootingProblem(x0s, running, terminal)
    assert problem.nx == problem.ndx + 1
    solver = crocoddyl.SolverFDDP(problem)
    solver.solve([], [], 30)
    conv = np.array(solver.status) == _abi.STATUS_CONVERGED
    assert conv.mean() >= 0.75, np.array(solver.status)
    xs = np.asarray(solver.xs)
    np.testing.assert_allclose(np.linalg.norm(xs[..., 3:7], axis=-1), 1.0, atol=1e-9)
