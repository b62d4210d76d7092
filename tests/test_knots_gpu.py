"""GPU half of tests/test_knots.py: heterogeneous knot sequences and knot
updates (fddp_set_knots, ShootingProblem.circularAppend) vs the oracle, on
every device code path."""
import numpy as np
import pytest

import helpers
import oracle_lib
from crocoddyl_amd import _abi, synthetic
from crocoddyl_amd.problem import pack_problem
from test_gpu import backward_variant  # noqa: F401  (autouse: every device code path)
from test_knots import _live, _same, _solve, hetero_setup

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,T,B", [("C2_lqr", 30, 4), ("C4_solo12", 20, 3), ("C5_talos_full", 12, 2)])
def test_hetero_gpu_vs_oracle(name, T, B):
    S = hetero_setup(name, T, B)
    g = helpers.Gpu(S["dims"], S["knots"], S["pool"], S["x0s"])
    o = oracle_lib.Oracle(S["dims"], S["knots"], S["pool"], S["x0s"], threads=8)
    _same(_solve(g), _solve(o), g, o)


def test_set_knots_gpu_vs_oracle():
    """MPC loop with a rotating knot sequence: shift the warm start, append
    the next phase's model (fddp_set_knots), re-solve."""
    S = hetero_setup("C4_solo12", 16, 3)
    g = helpers.Gpu(S["dims"], S["knots"], S["pool"], S["x0s"])
    o = oracle_lib.Oracle(S["dims"], S["knots"], S["pool"], S["x0s"], threads=8)
    _same(_solve(g, 5), _solve(o, 5), g, o)
    seq = list(S["running"])
    for step in range(4):
        seq = seq[1:] + [S["running"][step % len(S["running"])]]
        knots, pool = pack_problem(seq, S["terminal"], S["dims"].B)
        kd = (_abi.KnotDesc * len(knots))(*[_abi.KnotDesc(*k) for k in knots])
        assert g.L.fddp_set_knots(g.h, kd, _abi.dptr(pool), pool.size) == 0
        assert o.L.oracle_set_knots(o.h, kd, _abi.dptr(pool), pool.size) == 0
        g.mpc_shift()
        o.mpc_shift()
        rg = helpers.results_dict(g.solve(maxiter=2, is_feasible=False, reg_init=0.1))
        ro = helpers.results_dict(o.solve(maxiter=2, is_feasible=False, reg_init=0.1))
        _same(rg, ro, g, o, knots)


def test_facade_circular_append_gpu():
    """Python facade: problem.circularAppend(model) between solves equals a
    fresh problem built on the rotated sequence."""
    import crocoddyl_amd as crocoddyl
    x0s, running, terminal = synthetic.build_hetero("C2_lqr", T=20, B=3)
    problem = crocoddyl.ShootingProblem(x0s, running, terminal)
    solver = crocoddyl.SolverFDDP(problem)
    solver.solve(maxiter=5)
    xs, us = solver.xs, solver.us
    problem.circularAppend(running[6])  # nu = 0 knot
    fresh = crocoddyl.ShootingProblem(x0s, running[1:] + [running[6]], terminal)
    fsolver = crocoddyl.SolverFDDP(fresh)
    r1 = solver.solve(xs, us, maxiter=3)
    r2 = fsolver.solve(xs, us, maxiter=3)
    np.testing.assert_array_equal(r1, r2)
    np.testing.assert_array_equal(solver.iter, fsolver.iter)
    assert helpers.rel_err(solver.xs, fsolver.xs) < 1e-12
    knots, _ = pack_problem(problem.runningModels, terminal, 3)
    assert helpers.rel_err(_live(solver.us, knots), _live(fsolver.us, knots)) < 1e-12
