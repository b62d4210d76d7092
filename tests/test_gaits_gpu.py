"""Gait problems on the GPU through the C ABI vs the numpy oracle: the Talos walking
gait (utils/biped.py: 6D foot contacts, friction cones, CoM / foot tracking,
pseudo-impulse foot switches with frame-velocity costs) and the Solo12 trotting gait
(utils/quadruped.py: 3D foot contacts with Baumgarte damping, friction cones, state
bounds, impulse foot switches) on the code-built robots (crocoddyl_amd.robots).

Bars (north_star): calc / calcDiff blocks within 1e-8 relative (the contact KKT is
ill-conditioned on these robots: cond(S) ~ 1e7); solves with identical iteration
counts and statuses, xs / us / cost within 1e-6 relative. At full size (T = 100 /
60, B = 1024) spot knots of spot elements against the oracle and the solve's
invariants (finite, unit quaternions, cost not increased by an accepted step).
Parity against Pinocchio itself is unpinned offline (oracle/multibody_np.py)."""
import numpy as np
import pytest

import helpers
from crocoddyl_amd import _abi, synthetic
from crocoddyl_amd.problem import pack_problem
from oracle import fddp_np

pytestmark = pytest.mark.gpu
SOLVE_TOL = 1e-8  # element-wise (helpers.elem_err), solves vs the numpy oracle

GAITS = ["C5_talos_walk", "C4_solo12_trot"]


def _setup(name, T, B):
    x0s, running, terminal = synthetic.build(name, T=T, B=B)
    st = running[0].state
    knots, pool = pack_problem(running, terminal, B)
    nu_max = max(r.nu for r in running)
    dims = _abi.Dims(st.nx, st.ndx, nu_max, T, B)
    g = helpers.Gpu(dims, knots, pool, x0s)
    return g, knots, pool, x0s, dims, running, st


def _warm(name, running, dims, x0):
    xs, us = synthetic.gait_warm_start(name, running, x0)
    ua = np.zeros((dims.T, dims.nu_max))
    for t, u in enumerate(us):
        ua[t, :len(u)] = u
    return np.array(xs), ua


def _blocks(g, d):
    n, m = d.ndx, d.nu_max
    return {k: g.quantity(q, d.T + 1, s) for k, q, s in [
        ("Fx", _abi.Q_FX, n * n), ("Fu", _abi.Q_FU, n * m), ("Lxx", _abi.Q_LXX, n * n), ("Lxu", _abi.Q_LXU, n * m),
        ("Luu", _abi.Q_LUU, m * m), ("Lx", _abi.Q_LX, n), ("Lu", _abi.Q_LU, m), ("fs", _abi.Q_FS, n)]}


def _cmp_knot(Q, b, t, ref, n, m, tol):
    for name, shape in [("Fx", (n, n)), ("Fu", (n, m)), ("Lxx", (n, n)), ("Lxu", (n, m)), ("Luu", (m, m)),
                        ("Lx", (n,)), ("Lu", (m,))]:
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
        assert err < tol, (b, t, name, err)


@pytest.mark.parametrize("name", GAITS)
def test_gait_calc_diff_vs_oracle(name):
    T, B = 10, (1 if name == "C5_talos_walk" else 2)
    g, knots, pool, x0s, d, running, st = _setup(name, T, B)
    rng = np.random.default_rng(5)
    xs = np.zeros((B, T + 1, d.nx))
    for b in range(B):
        for t in range(T + 1):
            xs[b, t] = st.integrate(x0s[b], np.concatenate([rng.uniform(-0.03, 0.03, st.nv),
                                                            rng.uniform(-0.2, 0.2, st.nv)]))
    _, us = _warm(name, running, d, x0s[0])
    us = np.repeat(us[None], B, axis=0) + rng.uniform(-1, 1, (B, T, d.nu_max))
    for t, m in enumerate(running):
        us[:, t, m.nu:] = 0.0
    g.set_candidate(xs, us)
    cost = g.calc()
    g.set_solver_state(it=0)
    assert not g.compute_direction(True).any()
    Q = _blocks(g, d)
    for b in range(B):
        models = fddp_np.bind_problem(knots, pool, b, d.nx)
        o = fddp_np.FDDP(x0s[b], models)
        o.set_candidate(list(xs[b]), [us[b, t, :running[t].nu] for t in range(T)])
        o.iter = 0
        o.calc_diff()
        assert abs(cost[b] - o.cost) <= 1e-9 * max(1.0, abs(o.cost)), (b, cost[b], o.cost)
        for t in range(T + 1):
            assert helpers.rel_err(Q["fs"][b, t], o.fs[t]) < 1e-9, (b, t)
            _cmp_knot(Q, b, t, o.data[t], d.ndx, d.nu_max, 1e-8)


@pytest.mark.parametrize("name", GAITS)
def test_gait_solve_vs_oracle(name):
    """The reference benchmark's warm start (default state, quasi-static controls),
    then solve(maxiter=3): identical iteration counts / statuses, xs / us / cost
    within 1e-6. (Talos: T = 6 — double support, right step + pseudo-impulse switch,
    double support, left step + switch — to keep the oracle's complex-step solve short.)"""
    T, B = (6, 1) if name == "C5_talos_walk" else (10, 2)
    g, knots, pool, x0s, d, running, st = _setup(name, T, B)
    xs0, us0 = _warm(name, running, d, x0s[0])
    g.set_candidate(np.repeat(xs0[None], B, axis=0), np.repeat(us0[None], B, axis=0))
    r = helpers.results_dict(g.solve(maxiter=3, is_feasible=False, reg_init=1e-9))
    xs_g, us_g = g.xs(), g.us()
    for b in range(B):
        models = fddp_np.bind_problem(knots, pool, b, d.nx)
        o = fddp_np.FDDP(x0s[b], models)
        conv = o.solve(list(xs0), [us0[t, :running[t].nu] for t in range(T)], maxiter=3, is_feasible=False,
                       reg_init=1e-9)
        assert r["iter"][b] == o.iter, (b, r["iter"][b], o.iter)
        assert bool(r["status"][b] == _abi.STATUS_CONVERGED) == bool(conv)
        helpers.parity(f"{name} b{b} cost", [r["cost"][b]], [o.cost], SOLVE_TOL)
        helpers.parity(f"{name} b{b} xs", xs_g[b], np.array(o.xs), SOLVE_TOL)
        us_o = np.zeros_like(us_g[b])
        for t in range(T):
            nu = running[t].nu
            us_o[t, :nu] = np.asarray(o.us[t])[:nu]
            us_g[b, t, nu:] = 0.0
        helpers.parity(f"{name} b{b} us", us_g[b], us_o, SOLVE_TOL)


@pytest.mark.parametrize("name", GAITS)
def test_gait_full_size(name):
    """Full size (T, B of the config): warm start, 3 FDDP iterations, 2 MPC shifts;
    every element finite with unit quaternions; spot knots of spot elements vs the oracle."""
    _, _, _, T, B, _ = synthetic.CONFIGS[name]
    g, knots, pool, x0s, d, running, st = _setup(name, T, B)
    xs0, us0 = _warm(name, running, d, x0s[0])
    g.set_candidate(np.repeat(xs0[None], B, axis=0), np.repeat(us0[None], B, axis=0))
    r = helpers.results_dict(g.solve(maxiter=3, is_feasible=False, reg_init=1e-9))
    assert np.all(np.isfinite(r["cost"])) and np.all(r["iter"] >= 1)
    for _ in range(2):
        g.mpc_shift()
        r = helpers.results_dict(g.solve(maxiter=1, is_feasible=False, reg_init=0.1))
        assert np.all(np.isfinite(r["cost"]))
    xs = g.xs()
    assert np.all(np.isfinite(xs))
    np.testing.assert_allclose(np.linalg.norm(xs[..., 3:7], axis=-1), 1.0, atol=1e-9)
    # spot knots: calc + calcDiff at the current candidate vs the oracle
    us = g.us()
    g.set_solver_state(it=0, xreg=0.1, ureg=0.1)
    g.compute_direction(True)  # calcDiff of every knot (the sweep's status is not under test here)
    Q = _blocks(g, d)
    for b in (0, B // 2 + 1, B - 1):
        models = fddp_np.bind_problem(knots, pool, b, d.nx)
        for t in (0, T // 2, T - 1, T):
            m = models[t]
            u = us[b, t, :m.nu] if t < T else None
            ref = m.calc_diff(xs[b, t], u)
            _cmp_knot(Q, b, t, ref, d.ndx, d.nu_max, 1e-8)
