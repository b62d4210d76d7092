"""SolverDDP's phases one at a time through the C ABI — fddp_calc_diff, fddp_backward_pass,
fddp_forward_pass (reference: bindings/python/crocoddyl/core/solvers/ddp.cpp:70-82;
src/core/solvers/ddp.cpp:157-253, fddp.cpp:149-225) — against the C++ oracle's same
phases, element-wise (helpers.elem_err), at the headline knots (C5 Talos walk, T = 8,
from the reference benchmark's warm start) and at C2 (LQR 24/12), plus the Python
facade's calcDiff / backwardPass / forwardPass."""
import numpy as np
import pytest

import helpers
import oracle_lib
from crocoddyl_amd import _abi

pytestmark = pytest.mark.gpu

TOL = 1e-8  # element-wise; 4x the oracle's own one-ulp spread where the knots are worse conditioned

CASES = [("C5_talos_walk", dict(T=8, B=3)), ("C2_lqr", dict(T=100, B=8))]


def _start(name, S):
    d = S["dims"]
    if name.startswith("C5"):
        import bench
        return bench.warm_start_arrays(name, S["running"], S["x0s"], d)
    rng = np.random.default_rng(5)
    return rng.uniform(-1, 1, (d.B, d.T + 1, d.nx)), rng.uniform(-1, 1, (d.B, d.T, d.nu_max))


def _phases(h, xs, us, alphas, xreg):
    """calcDiff, backwardPass, forwardPass(alpha) for each alpha, from a fresh solver state."""
    d = h.dims
    n, m = d.ndx, d.nu_max
    h.set_candidate(xs, us, False)
    h.set_solver_state(it=0, xreg=xreg, ureg=xreg)
    out = {"cost": h.ddp_calc_diff()}
    for name, q, nk, per in (("Fx", _abi.Q_FX, d.T + 1, n * n), ("Fu", _abi.Q_FU, d.T + 1, n * m),
                             ("Lxx", _abi.Q_LXX, d.T + 1, n * n), ("Lx", _abi.Q_LX, d.T + 1, n),
                             ("fs", _abi.Q_FS, d.T + 1, n)):
        out[name] = h.quantity(q, nk, per)
    out["bwd_status"] = h.backward_pass()
    for name, q, nk, per in (("K", _abi.Q_K, d.T, m * n), ("k", _abi.Q_KV, d.T, m), ("Vxx", _abi.Q_VXX, d.T + 1, n * n),
                             ("Vx", _abi.Q_VX, d.T + 1, n), ("Qu", _abi.Q_QU, d.T, m), ("Quu", _abi.Q_QUU, d.T, m * m)):
        out[name] = h.quantity(q, nk, per)
    for a in alphas:
        rc, ct, st = h.forward_pass(a)
        assert rc == 0
        out[f"cost_try@{a}"], out[f"fwd_status@{a}"] = ct, st
        out[f"xs_try@{a}"], out[f"us_try@{a}"] = h.xs(trial=True), h.us(trial=True)
    return out


@pytest.mark.parametrize("xreg", [float("nan"), 1e-9])
@pytest.mark.parametrize("name,kw", CASES)
def test_phases_match_the_oracle(name, kw, xreg):
    S = helpers.setup(name, **kw)
    d = S["dims"]
    xs, us = _start(name, S)
    alphas = (1.0, 0.5, 0.005)  # 0.005: the reference harness's forwardPass (arm-kinova-codegen.cpp:278)
    g = helpers.Gpu(d, S["knots"], S["pool"], S["x0s"])
    g.set_debug(True)  # Vxx / Vx / Q* are stored in debug mode

    def oracle(pool):
        o = oracle_lib.Oracle(d, S["knots"], pool, S["x0s"], threads=4)
        return _phases(o, xs, us, alphas, xreg)

    ro = oracle(S["pool"])
    rg = _phases(g, xs, us, alphas, xreg)
    np.testing.assert_array_equal(rg["bwd_status"], ro["bwd_status"])
    for a in alphas:
        np.testing.assert_array_equal(rg[f"fwd_status@{a}"], ro[f"fwd_status@{a}"])
    keys = [k for k in ro if "status" not in k]
    # the oracle's spread under one-ulp parameter noise (the walk's Quu reaches cond 5e10)
    floors = dict(zip(keys, helpers.ulp_floor(lambda p: tuple(oracle(p)[k] for k in keys), S["pool"], reps=2)[1]))
    for k in keys:
        helpers.parity(f"{name} {k}", rg[k], ro[k], TOL, floors[k] if name.startswith("C5") else None)
    # the phases compose to the step API: tryStep = cost - cost_try (ddp.cpp:127-130)
    g.set_candidate(xs, us, False)
    g.set_solver_state(it=0, xreg=xreg, ureg=xreg)
    cost = g.ddp_calc_diff()
    g.backward_pass()
    dV, _ = g.try_step(0.5)
    _, ct, _ = g.forward_pass(0.5)
    np.testing.assert_array_equal(dV, cost - ct)


def test_phase_argument_checks():
    S = helpers.setup("C2_lqr", T=10, B=2)
    g = helpers.Gpu(S["dims"], S["knots"], S["pool"], S["x0s"])
    g.set_candidate(None, None, False)
    g.ddp_calc_diff()
    g.backward_pass()
    for bad in (1.5, -0.1):  # fddp.cpp:150-153
        rc, _, _ = g.forward_pass(bad)
        assert rc == _abi.FDDP_ERR_INVALID_ARG
        assert "step length" in g.L.fddp_last_error().decode()
    assert g.forward_pass(0.0)[0] == 0 and g.forward_pass(1.0)[0] == 0
    assert g.L.fddp_abi_version() == _abi.ABI_VERSION


def test_facade_phase_methods():
    """crocoddyl_amd.SolverFDDP.calcDiff / backwardPass / forwardPass on one problem, as the
    reference's Python binding exposes them, vs the oracle."""
    from crocoddyl_amd import ActionModelLQR, ShootingProblem, SolverFDDP
    from crocoddyl_amd.problem import pack_problem
    model = ActionModelLQR(24, 12, False)
    T = 50
    x0 = np.linspace(-1, 1, 24)
    problem = ShootingProblem(x0, [model] * T, model)
    solver = SolverFDDP(problem)
    solver.setCandidate([], [], False)
    cost = solver.calcDiff()
    solver.backwardPass()
    solver.forwardPass(0.25)
    knots, pool = pack_problem([model] * T, model, 1)
    o = oracle_lib.Oracle(_abi.Dims(24, 24, 12, T, 1), knots, pool, x0[None])
    o.set_candidate(None, None, False)
    c0 = o.ddp_calc_diff()
    o.backward_pass()
    _, ct, _ = o.forward_pass(0.25)
    helpers.parity("facade cost", np.array([cost]), c0, TOL)
    helpers.parity("facade k", np.array(solver.k), o.quantity(_abi.Q_KV, T, 12)[0], TOL)
    helpers.parity("facade cost_try", np.array([solver.cost_try]), ct, TOL)
    helpers.parity("facade xs_try", np.array(solver.xs_try), o.xs(trial=True)[0], TOL)
    helpers.parity("facade us_try", np.array(solver.us_try), o.us(trial=True)[0], TOL)
    with pytest.raises(Exception, match="step length"):
        solver.forwardPass(2.0)
