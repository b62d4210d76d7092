"""GPU parity of SolverBoxFDDP and BoxQP: libfddp_hip (C ABI) vs the CPU oracle.

Bar as for SolverFDDP (tests/test_gpu.py): identical statuses, iteration
counts and regularisation (branch decisions bit-identical), xs/us/cost
within 1e-6 relative; box-QP solutions within 1e-9. Every solver test runs
on each device code path (8-wave MFMA sweep + fast path, 4-wave MFMA sweep +
generic kernels, generic sweep) through the backward_variant fixture.
"""
import numpy as np
import pytest

import helpers
import oracle_lib
from crocoddyl_amd import _abi
from test_box_oracle import _oracle_box, _qp_params, _random_qps, box_setup
from test_gpu import backward_variant  # noqa: F401  (autouse: every device code path)

pytestmark = pytest.mark.gpu

RTOL = 1e-8  # element-wise (helpers.elem_err); north_star: xs/us/cost within 1e-6 relative


def _gpu_box(S, maxiter=100, th_stop=5e-5, debug=False):
    g = helpers.Gpu(S["dims"], S["knots"], S["pool"], S["x0s"])
    g.set_solver_kind(_abi.SOLVER_BOXFDDP)
    g.set_control_limits(S["lb"], S["ub"])
    p = oracle_lib.default_params()
    p.th_stop = th_stop
    assert g.set_params(p) == 0
    if debug:
        g.set_debug(True)
    g.set_candidate(None, None, False)
    r = helpers.results_dict(g.solve(maxiter=maxiter))
    return g, r


def _assert_same(rg, ro, g, o):
    for f in ("status", "iter", "n_iter_run", "is_feasible", "xreg"):
        np.testing.assert_array_equal(rg[f], ro[f], err_msg=f)
    helpers.parity("xs", g.xs(), o.xs(), RTOL)
    helpers.parity("us", g.us(), o.us(), RTOL)
    assert float(np.max(np.abs(rg["cost"] - ro["cost"]) / np.maximum(1, np.abs(ro["cost"])))) < RTOL
    assert float(np.max(np.abs(rg["stop"] - ro["stop"]) / np.maximum(1, np.abs(ro["stop"])))) < RTOL


@pytest.mark.parametrize("n", [3, 7, 12, 32, 64])
def test_boxqp_batched_vs_oracle(n):
    """fddp_boxqp_solve (one wave per QP) vs the oracle BoxQP."""
    from crocoddyl_amd import BoxQP
    rng = np.random.default_rng(300 + n)
    B = 48
    H, q, lb, ub, x0 = _random_qps(rng, B, n)
    o = oracle_lib.boxqp_solve(H, q, lb, ub, x0, _qp_params(th_grad=1e-9, reg=0.0))
    qp = BoxQP(n, reg=0.0)
    sols = qp.solve(H, q, lb, ub, x0)
    active = 0
    for b, s in enumerate(sols):
        assert s is not None and o["status"][b] == 0
        assert np.max(np.abs(s.x - o["x"][b])) <= 1e-9 * max(1.0, np.max(np.abs(o["x"][b])))
        assert s.free_idx == [i for i in range(n) if (int(o["free_mask"][b]) >> i) & 1]
        inv = [i for i in range(n) if (int(o["inv_mask"][b]) >> i) & 1]
        ref = o["Hinv"][b][np.ix_(inv, inv)]
        assert s.Hff_inv.shape == ref.shape
        assert np.max(np.abs(s.Hff_inv - ref)) <= 1e-9 * max(1.0, np.max(np.abs(ref)))
        active += len(s.clamped_idx)
    assert active > 0


def test_boxqp_known_answers_gpu():
    """unittest/test_boxqp.cpp cases through crocoddyl_amd.BoxQP."""
    from crocoddyl_amd import BoxQP
    rng = np.random.default_rng(5)
    for nx in (2, 3, 5):
        qp = BoxQP(nx)
        qp.reg = 0.0
        g = rng.uniform(-1, 1, nx)
        x0 = rng.uniform(-1, 1, nx)
        inf = np.full(nx, np.inf)
        s = qp.solve(np.eye(nx), g, -inf, inf, x0)
        assert np.max(np.abs(s.x + g)) < 1e-9 and len(s.free_idx) == nx and not s.clamped_idx
        reg = float(rng.uniform(1e-9, 1e2))
        qp.reg = reg
        # from xinit = 0 (a random xinit can make the reference's line search,
        # which prices the regularised direction with the true H, reject every
        # step and return xinit — the oracle does the same)
        s = qp.solve(np.eye(nx), g, -inf, inf, np.zeros(nx))
        assert np.max(np.abs(s.x + g / (1 + reg))) < 1e-9
        qp.reg = 0.0
        s = qp.solve(np.eye(nx), g, np.zeros(nx), np.ones(nx), x0)
        expect = np.clip(-g, 0, 1)
        assert np.max(np.abs(s.x - expect)) < 1e-9
        assert len(s.clamped_idx) == int(np.sum(expect != -g))


CASES = [
    dict(name="C2_lqr", T=10, B=4),
    dict(name="C3_talos_arm", T=12, B=3),
    dict(name="C4_solo12", T=8, B=3),
    dict(name="C5_talos_full", T=5, B=2),
    dict(nx=8, nu=4, T=15, B=4),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c.get("name", "lqr8x4"))
def test_boxfddp_solve_vs_oracle(case):
    S = box_setup(**case)
    o, ro = _oracle_box(S)
    g, rg = _gpu_box(S)
    _assert_same(rg, ro, g, o)
    us = o.us()
    assert np.sum(np.isclose(us, S["ub"]) | np.isclose(us, S["lb"])) > 0  # limits active


@pytest.mark.parametrize("case", [CASES[0], CASES[3]], ids=["C2", "C5"])
def test_boxfddp_quu_inv_and_gains(case):
    """Quu_inv (get_Quu_inv), K, k after a box solve, with the debug stores on."""
    S = box_setup(**case)
    o, ro = _oracle_box(S, maxiter=3)
    g, rg = _gpu_box(S, maxiter=3, debug=True)
    _assert_same(rg, ro, g, o)
    d = S["dims"]
    qi_g, qi_o = g.quu_inv(), o.quu_inv()
    assert np.max(np.abs(qi_o)) > 0
    assert helpers.rel_err(qi_g, qi_o) < 1e-9
    for which, per in ((_abi.Q_K, d.nu_max * d.ndx), (_abi.Q_KV, d.nu_max)):
        assert helpers.rel_err(g.quantity(which, d.T, per), o.quantity(which, d.T, per)) < 1e-9


def test_boxfddp_mpc_warm_started():
    """Repeated warm-started box solves after receding-horizon shifts: the
    box QP warm-starts at the persistent k (box-fddp.cpp:62)."""
    S = box_setup("C3_talos_arm", T=12, B=3)
    o, ro = _oracle_box(S, maxiter=5)
    g, rg = _gpu_box(S, maxiter=5)
    for _ in range(3):
        o.mpc_shift()
        g.mpc_shift()
        ro = helpers.results_dict(o.solve(maxiter=2, is_feasible=False, reg_init=0.1))
        rg = helpers.results_dict(g.solve(maxiter=2, is_feasible=False, reg_init=0.1))
        _assert_same(rg, ro, g, o)


def test_boxfddp_mixed_nu_regmax():
    """A limited knot whose nu differs from runningModels[0]->nu: backward_error until regmax."""
    from crocoddyl_amd import ActionModelLQR, pack_problem
    nx, T, B = 4, 6, 2
    m2, m3 = ActionModelLQR(nx, 2), ActionModelLQR(nx, 3)
    knots, pool = pack_problem([m2] * 3 + [m3] * 3, m3, B)
    S = dict(dims=_abi.Dims(nx, nx, 3, T, B), knots=knots, pool=pool, x0s=np.ones((B, nx)))
    S["ub"] = np.full((B, T, 3), 0.2)
    S["lb"] = -S["ub"]
    o, ro = _oracle_box(S, maxiter=20)
    g, rg = _gpu_box(S, maxiter=20)
    assert (rg["status"] == _abi.STATUS_REGMAX).all()
    _assert_same(rg, ro, g, o)


def test_boxfddp_facade_single_problem():
    """crocoddyl_amd.SolverBoxFDDP with the models' u_lb / u_ub (reference
    Python API), single problem, vs the oracle."""
    import crocoddyl_amd as crocoddyl
    S = box_setup("C2_lqr", T=10, B=1)
    model = S["running"][0]
    model.u_lb = S["lb"][0, 0]
    model.u_ub = S["ub"][0, 0]
    assert model.has_control_limits
    problem = crocoddyl.ShootingProblem(S["x0s"][0], [model] * 10, model)
    solver = crocoddyl.SolverBoxFDDP(problem)
    assert solver.th_stop == 5e-5
    done = solver.solve()
    o, ro = _oracle_box(S)
    assert done and ro["status"][0] == 1
    assert solver.iter == ro["iter"][0]
    helpers.parity("us", np.array(solver.us), o.us()[0], RTOL)
    helpers.parity("xs", np.array(solver.xs), o.xs()[0], RTOL)
