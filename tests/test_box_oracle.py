"""CPU tests of the SolverBoxFDDP / BoxQP restatements (oracle pinning).

The reference cannot be built or imported here, so the box
restatements are pinned the way the reference pins its own box solvers:
  * BoxQP known answers, unittest/test_boxqp.cpp:25-137 (identity Hessian
    with and without bounds and regularisation, random SPD vs the KKT
    solution, free/clamped counts);
  * C++ oracle (oracle/fddp_oracle.cpp) == independent numpy restatement
    (oracle/fddp_np.py) at 1e-9, for BoxQP and for whole SolverBoxFDDP
    solves (the design of unittest/bindings/test_solvers.py);
  * with inactive limits SolverBoxFDDP == SolverFDDP, and with active limits
    the converged BoxFDDP controls solve the box-constrained LQ problem
    (condensed dense QP), the box analogue of the reference's
    DDP == KKT test (unittest/test_solvers.cpp:65-110) and of the legacy
    box-DDP vs box-KKT check (unittest/python/test_boxsolvers.py).
"""
import numpy as np
import pytest

import helpers
import oracle_lib
from crocoddyl_amd import _abi
from oracle import fddp_np

INF = np.inf


def _qp_params(maxiter=100, th_grad=1e-9, reg=1e-9):
    p = _abi.BoxQPParams()
    p.maxiter, p.n_alphas, p.th_acceptstep, p.th_grad, p.reg = maxiter, 10, 0.1, th_grad, reg
    for i in range(10):
        p.alphas[i] = 2.0 ** -i
    return p


def _spd(rng, n):
    A = rng.uniform(-1, 1, (n, n))
    H = A.T @ A
    return 0.5 * (H + H.T) + 1e-3 * np.eye(n)


# ---------------------------------------------------------------- BoxQP ----
@pytest.mark.parametrize("impl", ["oracle", "numpy"])
def test_boxqp_known_answers(impl):
    """unittest/test_boxqp.cpp: identity / random-SPD Hessians, bounded and not."""
    rng = np.random.default_rng(11)

    def solve(H, g, lb, ub, x0, reg):
        if impl == "numpy":
            r = fddp_np.box_qp(H, g, lb, ub, x0, reg=reg)
            return r["x"], len(r["free_idx"]), len(r["clamped_idx"])
        o = oracle_lib.boxqp_solve(H[None], g[None], lb[None], ub[None], x0[None], _qp_params(reg=reg))
        nf = bin(int(o["free_mask"][0])).count("1")
        return o["x"][0], nf, g.size - nf

    for nx in (2, 3, 5):
        I = np.eye(nx)
        g = rng.uniform(-1, 1, nx)
        x0 = rng.uniform(-1, 1, nx)
        lo, hi = np.full(nx, -INF), np.full(nx, INF)
        reg = float(rng.uniform(1e-9, 1e2))
        # unconstrained, identity Hessian (test_unconstrained_qp_with_identity_hessian)
        x, nf, nc = solve(I, g, lo, hi, x0, 0.0)
        assert np.max(np.abs(x + g)) < 1e-9 and (nf, nc) == (nx, 0)
        # regularised: from xinit = 0 (from a random xinit the line search, which
        # prices the regularised direction with the true H, may reject every
        # step and return xinit — reference behaviour, kept)
        x, nf, nc = solve(I, g, lo, hi, np.zeros(nx), reg)
        assert np.max(np.abs(x + g / (1 + reg))) < 1e-9 and (nf, nc) == (nx, 0)
        # unconstrained, random SPD vs the KKT solution (test_unconstrained_qp)
        H = _spd(rng, nx)
        x, nf, nc = solve(H, g, lo, hi, x0, 0.0)
        assert np.max(np.abs(x + np.linalg.solve(H, g))) < 1e-9 and (nf, nc) == (nx, 0)
        x, nf, nc = solve(H, g, lo, hi, np.zeros(nx), reg)
        assert np.max(np.abs(x + np.linalg.solve(H + reg * I, g))) < 1e-9
        # box [0, 1], identity Hessian: the bounded negative gradient (test_box_qp_with_identity_hessian)
        lb, ub = np.zeros(nx), np.ones(nx)
        x, nf, nc = solve(I, g, lb, ub, x0, 0.0)
        expect = np.clip(-g, lb, ub)
        assert np.max(np.abs(x - expect)) < 1e-9
        assert nc == int(np.sum(expect != -g)) and nf == nx - nc


def _random_qps(rng, B, n):
    H = np.stack([_spd(rng, n) for _ in range(B)])
    q = rng.uniform(-2, 2, (B, n))
    lb = rng.uniform(-1.0, -0.1, (B, n))
    ub = rng.uniform(0.1, 1.0, (B, n))
    lb[:, ::4] = -INF  # partially unbounded
    x0 = rng.uniform(-1, 1, (B, n))
    return H, q, lb, ub, x0


@pytest.mark.parametrize("n", [3, 7, 12])
def test_boxqp_oracle_matches_numpy(n):
    rng = np.random.default_rng(100 + n)
    B = 40
    H, q, lb, ub, x0 = _random_qps(rng, B, n)
    prm = _qp_params(th_grad=1e-9, reg=0.0)
    o = oracle_lib.boxqp_solve(H, q, lb, ub, x0, prm)
    active = 0
    for b in range(B):
        r = fddp_np.box_qp(H[b], q[b], lb[b], ub[b], x0[b], reg=0.0)
        assert o["status"][b] == 0
        np.testing.assert_allclose(o["x"][b], r["x"], rtol=0, atol=1e-9)
        assert [i for i in range(n) if (int(o["free_mask"][b]) >> i) & 1] == r["free_idx"]
        inv = [i for i in range(n) if (int(o["inv_mask"][b]) >> i) & 1]
        assert inv == r["inv_idx"]
        np.testing.assert_allclose(o["Hinv"][b][np.ix_(inv, inv)], r["Hff_inv"], rtol=0, atol=1e-9)
        active += len(r["clamped_idx"])
    assert active > 0  # the bounds bite


def test_boxqp_llt_failure_is_backward_error():
    """A free Hessian that is not PD fails the LLT (box-qp.cpp:150-154)."""
    H = -np.eye(3)[None]
    o = oracle_lib.boxqp_solve(H, np.ones((1, 3)), -np.ones((1, 3)), np.ones((1, 3)), np.zeros((1, 3)),
                               _qp_params(reg=0.0))
    assert o["status"][0] == 1
    assert fddp_np.box_qp(H[0], np.ones(3), -np.ones(3), np.ones(3), np.zeros(3), reg=0.0) is None


# ---------------------------------------------------------- SolverBoxFDDP ----
def box_setup(name="C2_lqr", T=10, B=4, bound=0.3, seed=None, nx=None, nu=None):
    """A seeded problem with control limits [-bound, bound] on every running
    knot (per element: scaled by 1 + 0.5 b / B), lb[:, :, 0] = -inf."""
    if nx is not None:
        from crocoddyl_amd import synthetic
        rng = np.random.default_rng(7 if seed is None else seed)
        model = synthetic.lqr_models(nx, nu, B, rng)
        x0s = rng.uniform(-1, 1, (B, nx))
        running, terminal = [model] * T, model
        knots, pool = helpers.pack_problem(running, terminal, B)
        dims = _abi.Dims(nx, nx, nu, T, B)
        S = dict(dims=dims, knots=knots, pool=pool, x0s=x0s, running=running, terminal=terminal)
    else:
        S = helpers.setup(name, T=T, B=B, seed=seed)
    d = S["dims"]
    scale = bound * (1 + 0.5 * np.arange(d.B) / d.B)
    ub = np.broadcast_to(scale[:, None, None], (d.B, d.T, d.nu_max)).copy()
    lb = -ub
    lb[:, :, 0] = -INF
    S["lb"], S["ub"] = lb, ub
    return S


def _oracle_box(S, maxiter=100, th_stop=5e-5):
    o = oracle_lib.Oracle(S["dims"], S["knots"], S["pool"], S["x0s"], threads=8)
    o.set_solver_kind(_abi.SOLVER_BOXFDDP)
    o.set_control_limits(S["lb"], S["ub"])
    p = oracle_lib.default_params()
    p.th_stop = th_stop
    o.set_params(p)
    o.set_candidate(None, None, False)
    r = helpers.results_dict(o.solve(maxiter=maxiter))
    return o, r


def _numpy_box(S, b, maxiter=100, th_stop=5e-5):
    models = fddp_np.bind_problem(S["knots"], S["pool"], b, S["dims"].nx)
    T = S["dims"].T
    lb = [S["lb"][b, t, :models[t].nu] for t in range(T)]
    ub = [S["ub"][b, t, :models[t].nu] for t in range(T)]
    p = fddp_np.default_params()
    p["th_stop"] = th_stop
    s = fddp_np.FDDP(S["x0s"][b], models, p, box=True, u_lb=lb, u_ub=ub)
    s.solve(maxiter=maxiter)
    return s


@pytest.mark.parametrize("case", [dict(name="C2_lqr", T=10, B=4), dict(name="C3_talos_arm", T=12, B=3),
                                  dict(nx=8, nu=4, T=15, B=4)])
def test_boxfddp_oracle_matches_numpy(case):
    S = box_setup(**case)
    o, r = _oracle_box(S)
    xs, us = o.xs(), o.us()
    clamped = 0
    for b in range(S["dims"].B):
        s = _numpy_box(S, b)
        assert r["status"][b] == s.status == 1
        assert r["iter"][b] == s.iter
        np.testing.assert_allclose(xs[b], np.array(s.xs), rtol=0, atol=1e-9)
        np.testing.assert_allclose(us[b], np.array(s.us), rtol=0, atol=1e-9)
        assert abs(r["cost"][b] - s.cost) <= 1e-9 * max(1.0, abs(s.cost))
        clamped += int(np.sum(np.isclose(us[b], S["ub"][b]) | np.isclose(us[b], S["lb"][b])))
    assert clamped > 0  # the limits are active at the solution


def test_boxfddp_inactive_limits_equal_fddp():
    """Limits that never bind: SolverBoxFDDP takes the vanilla steps."""
    S = box_setup("C2_lqr", T=10, B=3, bound=1e3)
    o, r = _oracle_box(S, th_stop=1e-9)
    f = oracle_lib.Oracle(S["dims"], S["knots"], S["pool"], S["x0s"], threads=8)
    f.set_candidate(None, None, False)
    rf = helpers.results_dict(f.solve(maxiter=100))
    np.testing.assert_array_equal(r["iter"], rf["iter"])
    np.testing.assert_allclose(o.xs(), f.xs(), rtol=0, atol=1e-10)
    np.testing.assert_allclose(o.us(), f.us(), rtol=0, atol=1e-10)


def _condensed(models, x0, T):
    """The LQ problem as a dense QP in the stacked controls: cost(u) =
    0.5 u'Hu + g'u + c (rollout of the linear dynamics)."""
    nx, nu = models[0].nx, models[0].nu
    P = models[0]
    Fx, Fu, f0 = P.Fx, P.Fu, (0.0 if P.drift_free else P.f0)
    N = T * nu
    # x_t = A_t x0 + S_t u + c_t
    A, S, c = [np.eye(nx)], [np.zeros((nx, N))], [np.zeros(nx)]
    for t in range(T):
        A.append(Fx @ A[-1])
        St = Fx @ S[-1]
        St[:, t * nu:(t + 1) * nu] += Fu
        S.append(St)
        c.append(Fx @ c[-1] + f0)
    H, g = np.zeros((N, N)), np.zeros(N)
    for t in range(T + 1):
        m = models[t]
        xa = A[t] @ x0 + c[t]
        H += S[t].T @ m.Lxx @ S[t]
        g += S[t].T @ (m.Lxx @ xa + m.lx)
        if t < T:
            E = np.zeros((nu, N))
            E[:, t * nu:(t + 1) * nu] = np.eye(nu)
            H += E.T @ m.Luu @ E + S[t].T @ m.Lxu @ E + E.T @ m.Lxu.T @ S[t]
            g += E.T @ (m.Luu @ np.zeros(nu) + m.lu + m.Lxu.T @ xa)
    return 0.5 * (H + H.T), g


def test_boxfddp_solves_the_box_constrained_problem():
    """Converged SolverBoxFDDP controls == the minimiser of the condensed
    box-constrained QP (projected Newton run to full precision)."""
    S = box_setup(nx=6, nu=3, T=8, B=3)
    o, r = _oracle_box(S, maxiter=200)
    us = o.us()
    active = 0
    for b in range(S["dims"].B):
        models = fddp_np.bind_problem(S["knots"], S["pool"], b, S["dims"].nx)
        H, g = _condensed(models, S["x0s"][b], S["dims"].T)
        lb, ub = S["lb"][b].reshape(-1), S["ub"][b].reshape(-1)
        ref = fddp_np.box_qp(H, g, lb, ub, np.zeros(g.size), maxiter=500, th_grad=1e-13, reg=0.0)
        assert r["status"][b] == 1
        active += int(np.sum((ref["x"] == lb) | (ref["x"] == ub)))
        np.testing.assert_allclose(us[b].reshape(-1), ref["x"], rtol=0, atol=1e-9)
    assert active > 0


def test_boxfddp_mixed_nu_is_backward_error():
    """qp_ is sized by runningModels[0]->nu (box-fddp.cpp:16): a limited knot
    with another nu makes BoxQP::solve throw, which solve() treats as a
    backward_error until regmax (fddp.cpp:37-43)."""
    from crocoddyl_amd import ActionModelLQR, pack_problem
    nx, T, B = 4, 6, 2
    m2, m3 = ActionModelLQR(nx, 2), ActionModelLQR(nx, 3)
    running = [m2] * 3 + [m3] * 3
    knots, pool = pack_problem(running, m3, B)
    S = dict(dims=_abi.Dims(nx, nx, 3, T, B), knots=knots, pool=pool, x0s=np.ones((B, nx)))
    S["ub"] = np.full((B, T, 3), 0.2)
    S["lb"] = -S["ub"]
    o, r = _oracle_box(S, maxiter=20)
    assert (r["status"] == _abi.STATUS_REGMAX).all()
