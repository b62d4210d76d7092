"""GPU parity tests: libfddp_hip (through its C ABI) vs the CPU oracle.

Bar (BASELINE.json north_star): knot indexing bit-exact (same knot/element
order, exact iteration counts and statuses), xs/us/cost within 1e-6
relative. Tolerances are written per assertion; the fp64 device arithmetic
typically agrees to ~1e-12.
"""
import numpy as np
import pytest

import helpers
import oracle_lib
from crocoddyl_amd import _abi

pytestmark = pytest.mark.gpu

RTOL = 1e-8  # element-wise (helpers.elem_err); north_star: xs/us/cost within 1e-6 relative


@pytest.fixture(params=["default", "mfma4_slowpath", "generic"], autouse=True)
def backward_variant(request, monkeypatch):
    """Run every parity test on each device code path:
    default         8-wave MFMA Riccati sweep (where the shape allows) and the
                    dense-knot fast path for calc / calcDiff / forward;
    mfma4_slowpath  4-wave MFMA sweep (FDDP_BWD_WAVES=4) and the generic
                    calc / calcDiff / forward kernels (FDDP_FAST=0);
    generic         the generic LDS Riccati sweep (FDDP_BACKWARD=generic)."""
    for var in ("FDDP_BACKWARD", "FDDP_BWD_WAVES", "FDDP_FAST"):
        monkeypatch.delenv(var, raising=False)
    if request.param == "generic":
        monkeypatch.setenv("FDDP_BACKWARD", "generic")
    elif request.param == "mfma4_slowpath":
        monkeypatch.setenv("FDDP_BWD_WAVES", "4")
        monkeypatch.setenv("FDDP_FAST", "0")
    return request.param

CASES = [
    ("C1_unicycle", dict(T=30, B=16)),
    ("C2_lqr", dict(T=20, B=8)),
    ("C2_lqr", dict(T=10, B=4, drift_free=False)),
    ("C3_talos_arm", dict(T=25, B=4)),
    ("C4_solo12", dict(T=12, B=4)),
    ("C5_talos_full", dict(T=6, B=3)),
]


def _pair(S):
    g = helpers.Gpu(S["dims"], S["knots"], S["pool"], S["x0s"])
    o = oracle_lib.Oracle(S["dims"], S["knots"], S["pool"], S["x0s"], threads=8)
    return g, o


def _assert_results(rg, ro, check_counts=True):
    G, O = helpers.results_dict(rg), helpers.results_dict(ro)
    if check_counts:
        np.testing.assert_array_equal(G["status"], O["status"])
        np.testing.assert_array_equal(G["iter"], O["iter"])
        np.testing.assert_array_equal(G["n_iter_run"], O["n_iter_run"])
        np.testing.assert_array_equal(G["is_feasible"], O["is_feasible"])
        np.testing.assert_array_equal(G["xreg"], O["xreg"])
        np.testing.assert_array_equal(G["steplength"], O["steplength"])
    np.testing.assert_allclose(G["cost"], O["cost"], rtol=RTOL, atol=1e-12)


@pytest.mark.parametrize("name,kw", CASES)
def test_solve_parity(name, kw):
    S = helpers.setup(name, **kw)
    g, o = _pair(S)
    for h in (g, o):
        h.set_candidate(None, None, False)
    rg, ro = g.solve(maxiter=30), o.solve(maxiter=30)
    _assert_results(rg, ro)
    helpers.parity("xs", g.xs(), o.xs(), RTOL)
    helpers.parity("us", g.us(), o.us(), RTOL)


@pytest.mark.parametrize("name,kw", CASES)
def test_solve_parity_warm_start_and_feasible(name, kw):
    """Random warm start (infeasible gaps), then a feasible-start solve."""
    S = helpers.setup(name, **kw)
    d = S["dims"]
    rng = np.random.default_rng(1)
    xs = rng.uniform(-1, 1, (d.B, d.T + 1, d.nx))
    us = rng.uniform(-1, 1, (d.B, d.T, d.nu_max))
    g, o = _pair(S)
    for h in (g, o):
        h.set_candidate(xs, us, False)
    _assert_results(g.solve(maxiter=5, reg_init=0.1), o.solve(maxiter=5, reg_init=0.1))
    helpers.parity("xs", g.xs(), o.xs(), RTOL)
    helpers.parity("us", g.us(), o.us(), RTOL)
    for h in (g, o):
        h.set_candidate(None, us, True)
    _assert_results(g.solve(maxiter=3), o.solve(maxiter=3))
    helpers.parity("us", g.us(), o.us(), RTOL)


@pytest.mark.parametrize("name,kw", CASES)
def test_problem_calc_and_calc_diff(name, kw):
    """ShootingProblem::calc/calcDiff blocks (test_shooting.py:32-63 design)."""
    S = helpers.setup(name, **kw)
    d = S["dims"]
    n, m, T = d.ndx, d.nu_max, d.T
    rng = np.random.default_rng(2)
    xs = rng.uniform(-1, 1, (d.B, T + 1, d.nx))
    us = rng.uniform(-1, 1, (d.B, T, m))
    g, o = _pair(S)
    for h in (g, o):
        h.set_candidate(xs, us, False)
    np.testing.assert_allclose(g.calc(), o.calc(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(g.calc_diff(), o.calc_diff(), rtol=1e-12, atol=1e-12)
    for q, nk, per in [(_abi.Q_FX, T + 1, n * n), (_abi.Q_FU, T + 1, n * m), (_abi.Q_LXX, T + 1, n * n),
                       (_abi.Q_LXU, T + 1, n * m), (_abi.Q_LUU, T + 1, m * m), (_abi.Q_LX, T + 1, n),
                       (_abi.Q_LU, T + 1, m), (_abi.Q_XNEXT, T, d.nx)]:
        a, b = g.quantity(q, nk, per), o.quantity(q, nk, per)
        if q == _abi.Q_LU:  # terminal Lu: the reference terminal model keeps nu (unone_ = 0)
            a, b = a[:, :T], b[:, :T]
        np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12, err_msg=f"quantity {q}")


@pytest.mark.parametrize("name,kw", CASES)
def test_step_api_parity(name, kw):
    """computeDirection Q/V blocks, tryStep(1)/(0.5), stop, expected
    improvement (unittest/bindings/test_solvers.py:38-96 design)."""
    S = helpers.setup(name, **kw)
    d = S["dims"]
    n, m, T = d.ndx, d.nu_max, d.T
    rng = np.random.default_rng(3)
    xs = rng.uniform(-1, 1, (d.B, T + 1, d.nx))
    us = rng.uniform(-1, 1, (d.B, T, m))
    g, o = _pair(S)
    g.set_debug(True)
    for h in (g, o):
        h.set_candidate(xs, us, False)
        h.set_solver_state(0, 1e-9, 1e-9, 0)
        assert not h.compute_direction(True).any()
        h.update_expected_improvement()
    tol = dict(rtol=1e-9, atol=1e-9)
    for q, nk, per in [(_abi.Q_FS, T + 1, n), (_abi.Q_K, T, m * n), (_abi.Q_KV, T, m), (_abi.Q_VXX, T + 1, n * n),
                       (_abi.Q_VX, T + 1, n), (_abi.Q_QXX, T, n * n), (_abi.Q_QXU, T, n * m),
                       (_abi.Q_QUU, T, m * m), (_abi.Q_QX, T, n), (_abi.Q_QU, T, m)]:
        a, b = g.quantity(q, nk, per), o.quantity(q, nk, per)
        scale = max(1.0, float(np.max(np.abs(b))))
        np.testing.assert_allclose(a / scale, b / scale, **tol, err_msg=f"quantity {q}")
    np.testing.assert_allclose(g.stopping_criteria(), o.stopping_criteria(), rtol=1e-9)
    for alpha in (1.0, 0.5, 0.125):
        (dg, sg), (do, so) = g.try_step(alpha), o.try_step(alpha)
        np.testing.assert_array_equal(sg, so)
        np.testing.assert_allclose(dg, do, rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(g.xs(trial=True), o.xs(trial=True), rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(g.us(trial=True), o.us(trial=True), rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(g.expected_improvement(), o.expected_improvement(), rtol=1e-8, atol=1e-9)


DATA_Q = [(_abi.Q_FX, "nn"), (_abi.Q_FU, "nm"), (_abi.Q_LXX, "nn"), (_abi.Q_LXU, "nm"), (_abi.Q_LUU, "mm"),
          (_abi.Q_LX, "n"), (_abi.Q_LU, "m")]


def _assert_datas(g, o, d, tol):
    """Knot datas (Fx, Fu, Lxx, Lxu, Luu, Lx, Lu of every knot) vs the oracle."""
    n, m, T = d.ndx, d.nu_max, d.T
    per = dict(nn=n * n, nm=n * m, mm=m * m, n=n, m=m)
    for q, shape in DATA_Q:
        a, b = g.quantity(q, T + 1, per[shape]), o.quantity(q, T + 1, per[shape])
        if q == _abi.Q_LU:
            a, b = a[:, :T], b[:, :T]
        np.testing.assert_allclose(a, b, **tol, err_msg=f"quantity {q}")


@pytest.mark.parametrize("name,kw", [("C2_lqr", dict(T=10, B=4)), ("C4_solo12", dict(T=12, B=4)),
                                     ("C5_talos_full", dict(T=6, B=3))])
def test_datas_after_solve(name, kw):
    """The derivative blocks a solve leaves in the knot datas (on the fast
    path the 8-wave sweep writes calcDiff's blocks itself, two knots ahead of
    its own position) equal the oracle's after the same SolverFDDP::solve."""
    S = helpers.setup(name, **kw)
    d = S["dims"]
    rng = np.random.default_rng(5)
    xs = rng.uniform(-1, 1, (d.B, d.T + 1, d.nx))
    us = rng.uniform(-1, 1, (d.B, d.T, d.nu_max))
    g, o = _pair(S)
    for h in (g, o):
        h.set_candidate(xs, us, False)
    _assert_results(g.solve(maxiter=2, reg_init=0.1), o.solve(maxiter=2, reg_init=0.1))
    _assert_datas(g, o, d, dict(rtol=1e-9, atol=1e-9))


def test_datas_after_regmax_abort():
    """A sweep that fails on every retry still leaves calcDiff's blocks of
    every knot (the reference computes them all before the backward pass)."""
    from crocoddyl_amd.models import ActionModelLQR
    from crocoddyl_amd.problem import pack_problem
    model = ActionModelLQR(4, 2, True)
    model.Luu = -2e10 * np.eye(2)
    T = 7
    knots, pool = pack_problem([model] * T, model, 1)
    dims = _abi.Dims(4, 4, 2, T, 2)
    S = dict(dims=dims, knots=knots, pool=pool, x0s=np.ones((2, 4)))
    g, o = _pair(S)
    for h in (g, o):
        h.set_candidate(None, None, False)
    rg, ro = g.solve(maxiter=10), o.solve(maxiter=10)
    assert ro[0].status == _abi.STATUS_REGMAX
    _assert_results(rg, ro)
    _assert_datas(g, o, dims, dict(rtol=1e-12, atol=1e-12))


def test_unregularised_fresh_solver_direction():
    """A fresh solver has xreg = ureg = NaN: no regularisation and
    Vx = Qx - K^T Qu (ddp.cpp:216-238)."""
    S = helpers.setup("C2_lqr", T=6, B=2)
    d = S["dims"]
    g, o = _pair(S)
    g.set_debug(True)
    rng = np.random.default_rng(4)
    xs = rng.uniform(-1, 1, (d.B, d.T + 1, d.nx))
    us = rng.uniform(-1, 1, (d.B, d.T, d.nu_max))
    for h in (g, o):
        h.set_candidate(xs, us, False)
        h.compute_direction(True)
    for q, nk, per in [(_abi.Q_VX, d.T + 1, d.ndx), (_abi.Q_VXX, d.T + 1, d.ndx ** 2), (_abi.Q_K, d.T, d.nu_max * d.ndx)]:
        np.testing.assert_allclose(g.quantity(q, nk, per), o.quantity(q, nk, per), rtol=1e-9, atol=1e-9)


def test_regularisation_retry_parity():
    """Indefinite Luu: backward_error, reg x10 retries (fddp.cpp:35-48)."""
    from crocoddyl_amd.models import ActionModelLQR
    from crocoddyl_amd.problem import pack_problem
    model = ActionModelLQR(4, 2, True)
    model.Luu = -5.0 * np.eye(2)
    T = 5
    knots, pool = pack_problem([model] * T, model, 2)
    dims = _abi.Dims(4, 4, 2, T, 2)
    x0s = np.ones((2, 4))
    S = dict(dims=dims, knots=knots, pool=pool, x0s=x0s)
    g, o = _pair(S)
    for h in (g, o):
        h.set_candidate(None, None, False)
    rg, ro = g.solve(maxiter=20), o.solve(maxiter=20)
    _assert_results(rg, ro)
    assert rg[0].xreg >= 1.0
    helpers.parity("xs", g.xs(), o.xs(), RTOL)


def test_regmax_abort_parity():
    """A direction that never passes LLT drives xreg to regmax: solve returns
    false with status REGMAX (fddp.cpp:41-43)."""
    from crocoddyl_amd.models import ActionModelLQR
    from crocoddyl_amd.problem import pack_problem
    model = ActionModelLQR(3, 2, True)
    model.Luu = -2e10 * np.eye(2)
    knots, pool = pack_problem([model] * 4, model, 1)
    dims = _abi.Dims(3, 3, 2, 4, 1)
    S = dict(dims=dims, knots=knots, pool=pool, x0s=np.ones((1, 3)))
    g, o = _pair(S)
    for h in (g, o):
        h.set_candidate(None, None, False)
    rg, ro = g.solve(maxiter=10), o.solve(maxiter=10)
    assert ro[0].status == _abi.STATUS_REGMAX
    _assert_results(rg, ro)


def test_mpc_shift_parity():
    S = helpers.setup("C3_talos_arm", T=20, B=4)
    g, o = _pair(S)
    for h in (g, o):
        h.set_candidate(None, None, False)
        h.solve(maxiter=3)
    for _ in range(3):
        for h in (g, o):
            h.mpc_shift()
        rg, ro = g.solve(maxiter=1, reg_init=0.1), o.solve(maxiter=1, reg_init=0.1)
        _assert_results(rg, ro)
        helpers.parity("xs", g.xs(), o.xs(), RTOL)
        helpers.parity("us", g.us(), o.us(), RTOL)


def _subset(S, idx):
    """Oracle inputs for a subset of batch elements."""
    knots, pool = [], []
    pos = 0
    seen = {}
    for kind, nu, off, stride in S["knots"]:
        key = (off, stride)
        if key not in seen:
            from oracle.fddp_np import block_size
            size = block_size(kind, S["dims"].nx, nu)
            blocks = [S["pool"][off + (b if stride else 0) * stride: off + (b if stride else 0) * stride + size]
                      for b in (idx if stride else [0])]
            seen[key] = (pos, size if stride else 0)
            pool.extend(blocks)
            pos += size * len(blocks)
        knots.append((kind, nu) + seen[key])
    d = S["dims"]
    dims = _abi.Dims(d.nx, d.ndx, d.nu_max, d.T, len(idx))
    return dict(dims=dims, knots=knots, pool=np.concatenate(pool), x0s=S["x0s"][idx])


@pytest.mark.parametrize("name", ["C2_lqr", "C3_talos_arm", "C4_solo12", "C5_talos_full"])
def test_full_size_solve(name):
    """BASELINE sizes: every element converges like the LQ problem must (full
    step then a zero step), spot-checked elements match the oracle."""
    S = helpers.setup(name)
    d = S["dims"]
    g = helpers.Gpu(S["dims"], S["knots"], S["pool"], S["x0s"])
    g.set_candidate(None, None, False)
    r = helpers.results_dict(g.solve(maxiter=10))
    assert np.all(r["status"] == _abi.STATUS_CONVERGED)
    assert np.all(r["iter"] == 1)
    idx = [0, d.B // 2, d.B - 1]
    sub = _subset(S, idx)
    o = oracle_lib.Oracle(sub["dims"], sub["knots"], sub["pool"], sub["x0s"], threads=8)
    o.set_candidate(None, None, False)
    ro = helpers.results_dict(o.solve(maxiter=10))
    np.testing.assert_allclose(r["cost"][idx], ro["cost"], rtol=RTOL)
    helpers.parity("xs[idx]", g.xs()[idx], o.xs(), RTOL)
    helpers.parity("us[idx]", g.us()[idx], o.us(), RTOL)


def test_full_size_mpc_properties():
    """C5 at full size, warm-started maxiter=1 solves: finite, monotone
    bookkeeping, spot-checked against the oracle."""
    S = helpers.setup("C5_talos_full")
    d = S["dims"]
    g = helpers.Gpu(S["dims"], S["knots"], S["pool"], S["x0s"])
    g.set_candidate(None, None, False)
    g.solve(maxiter=2)
    idx = [3, 700]
    sub = _subset(S, idx)
    o = oracle_lib.Oracle(sub["dims"], sub["knots"], sub["pool"], sub["x0s"], threads=8)
    o.set_candidate(g.xs()[idx], g.us()[idx], True)
    for it in range(2):
        g.mpc_shift()
        o.mpc_shift()
        rg = helpers.results_dict(g.solve(maxiter=1, reg_init=0.1))
        ro = helpers.results_dict(o.solve(maxiter=1, reg_init=0.1))
        assert np.all(np.isfinite(rg["cost"]))
        assert np.all(rg["n_iter_run"] == 1)
        np.testing.assert_allclose(rg["cost"][idx], ro["cost"], rtol=RTOL)
        helpers.parity("xs[idx]", g.xs()[idx], o.xs(), RTOL)


def test_argument_errors():
    """Setter validation mirrors the reference (ddp.cpp:420-486)."""
    S = helpers.setup("C2_lqr", T=3, B=1)
    g = helpers.Gpu(S["dims"], S["knots"], S["pool"], S["x0s"])
    p = oracle_lib.default_params()
    p.regfactor = 0.5
    assert g.set_params(p) == _abi.FDDP_ERR_INVALID_ARG
    p = oracle_lib.default_params()
    p.alphas[3] = 2.0
    assert g.set_params(p) == _abi.FDDP_ERR_INVALID_ARG
    p = oracle_lib.default_params()
    assert g.set_params(p) == _abi.FDDP_OK
    with pytest.raises(RuntimeError):
        g.try_step(1.5)
