"""The C++ oracle's free-flyer knots (oracle/floating_oracle.hpp) and its manifold
solver state operations vs the numpy oracle (oracle/multibody_np.py,
oracle/fddp_np.py) on the legged gaits — CPU only.

floating_oracle.hpp restates the same reference functions analytically (RNEA
derivatives by the linearised recursion, KKT-inverse force derivatives, Jexp6 /
Jlog6 on the free-flyer), the numpy oracle by complex step; agreement to 1e-9
pins the C++ port that bench.py times as the CPU baseline of C4 / C5."""
import numpy as np
import pytest

import oracle_lib
from crocoddyl_amd import _abi, synthetic
from crocoddyl_amd.problem import pack_problem
from oracle import fddp_np


def _problem(name, idx, B=2, seed=3):
    """A problem of the gait's knots ``idx[:-1]`` (running) + knot ``idx[-1]`` as the terminal."""
    g, running, _ = synthetic.gait_models(name, None)
    run = [running[i] for i in idx[:-1]]
    terminal = running[idx[-1]]
    st = g.state
    knots, pool = pack_problem(run, terminal, B)
    nu = max(m.nu for m in run)
    dims = _abi.Dims(st.nx, st.ndx, nu, len(run), B)
    rng = np.random.default_rng(seed)
    x0 = g.rmodel.defaultState
    x0s = np.stack([st.integrate(x0, np.concatenate([rng.uniform(-0.03, 0.03, st.nv), rng.uniform(-0.2, 0.2, st.nv)]))
                    for _ in range(B)])
    return g, run, dims, knots, pool, x0s, rng


CASES = [("C5_talos_walk", [0, 1, 20, 49, 50, 99, 99]),  # double / single support, pseudo-impulse (dt = 0) switches
         ("C4_solo12_trot", [0, 2, 15, 28, 29, 30, 59])]  # ... and the impulse foot switches


@pytest.mark.parametrize("case", range(len(CASES)))
def test_cpp_free_flyer_knots_vs_numpy(case):
    name, idx = CASES[case]
    g, run, d, knots, pool, x0s, rng = _problem(name, idx)
    st = g.state
    xs = np.stack([[st.integrate(x0s[b], np.concatenate([rng.uniform(-0.05, 0.05, st.nv),
                                                         rng.uniform(-0.3, 0.3, st.nv)]))
                    for _ in range(d.T + 1)] for b in range(d.B)])
    us = np.zeros((d.B, d.T, d.nu_max))
    for t, m in enumerate(run):
        if m.nu:
            us[:, t, :m.nu] = m.quasiStatic(None, g.rmodel.defaultState) + rng.uniform(-3, 3, (d.B, m.nu))
    o = oracle_lib.Oracle(d, knots, pool, x0s, threads=2)
    o.set_candidate(xs, us)
    cost = o.calc()
    xn = o.quantity(_abi.Q_XNEXT, d.T, d.nx)
    o.calc_diff()
    n, m = d.ndx, d.nu_max
    Q = {k: o.quantity(q, d.T + 1, s) for k, q, s in [("Fx", _abi.Q_FX, n * n), ("Fu", _abi.Q_FU, n * m),
                                                      ("Lxx", _abi.Q_LXX, n * n), ("Lxu", _abi.Q_LXU, n * m),
                                                      ("Lx", _abi.Q_LX, n), ("Luu", _abi.Q_LUU, m * m),
                                                      ("Lu", _abi.Q_LU, m)]}
    for b in range(d.B):
        models = fddp_np.bind_problem(knots, pool, b, d.nx)
        tot = 0.0
        for t in range(d.T + 1):
            k = models[t]
            u = us[b, t, :run[t].nu] if t < d.T and run[t].nu else None
            xo, co = k.calc(xs[b, t], u)
            tot += co
            if t < d.T:
                np.testing.assert_allclose(xn[b, t], xo, rtol=1e-10, atol=1e-11)
            ref = k.calc_diff(xs[b, t], u)
            nut = ref["Fu"].shape[1]
            for q in Q:
                want = ref[q]
                if q in ("Fx", "Lxx"):
                    got = Q[q][b, t].reshape(n, n).T
                elif q in ("Fu", "Lxu"):
                    got = Q[q][b, t].reshape(m, n).T[:, :nut]
                elif q == "Luu":
                    got = Q[q][b, t].reshape(m, m).T[:nut, :nut]
                else:
                    got = Q[q][b, t][:want.size]
                if want.size == 0:
                    continue
                scale = max(1.0, float(np.max(np.abs(want))))
                assert float(np.max(np.abs(got - want))) / scale < 1e-9, (name, b, t, q)
        assert cost[b] == pytest.approx(tot, rel=1e-11)


def test_cpp_free_flyer_solve_vs_numpy():
    """Two FDDP iterations on the manifold state (gaps diff(xs, f(xs, us)), rollout
    integrate(xnext, fs (alpha - 1)), the expected improvement's diff(xs_try, xs)):
    the C++ solver vs fddp_np on the same Talos knots."""
    g, run, d, knots, pool, x0s, _ = _problem("C5_talos_walk", [0, 1, 20, 99], B=1)
    x0 = g.rmodel.defaultState
    xs0 = np.repeat(x0[None, None, :], d.T + 1, axis=1)
    us0 = np.stack([m.quasiStatic(None, x0) for m in run])[None]
    o = oracle_lib.Oracle(d, knots, pool, x0s, threads=1)
    o.set_candidate(xs0, us0)
    r = o.solve(maxiter=2, is_feasible=False, reg_init=1e-9)
    models = fddp_np.bind_problem(knots, pool, 0, d.nx)
    s = fddp_np.FDDP(x0s[0], models)
    s.solve(list(xs0[0]), list(us0[0]), maxiter=2, is_feasible=False, reg_init=1e-9)
    assert r[0].iter == s.iter
    assert r[0].cost == pytest.approx(s.cost, rel=1e-8)
    np.testing.assert_allclose(o.xs()[0], np.array(s.xs), rtol=1e-7, atol=1e-8)
    np.testing.assert_allclose(o.us()[0], np.array(s.us), rtol=1e-7, atol=1e-7)
