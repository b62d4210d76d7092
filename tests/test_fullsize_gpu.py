"""The headline workloads at full size, solve-checked against the C++ oracle.

C5 (Talos walk, T = 100, B = 1024) and C4 (Solo12 trot, T = 60, B = 1024) are built
with bench.py's own code (make_shard_solver, FixedWarmStart, mpc_step) and run the
bench's steps on the GPU:
  * protocol fixed: solve(xs_w, us_w, maxiter=1, isFeasible=False, regInit=0.1) from
    the reference benchmark's warm start (bipedal_walk_optctrl.py:36-43);
  * protocol shift: solve(maxiter=5) from the warm start, then two receding-horizon
    steps (gait knots rotated, x0 / xs / us shifted, solve(maxiter=1, regInit=0.1)).
Spot elements {0, B/2, B-1} are replayed on the C++ oracle (oracle/floating_oracle.hpp)
from the same x0 and warm start with the same knot rotation: identical status,
iteration count and step length (every branch decision of the line search), xs / us /
cost element-wise (helpers.elem_err: each coordinate at its own scale) within 1e-8, or
within 4x the oracle's own spread under one-ulp noise in the model parameters where the
protocol's conditioning is worse than that (helpers.ulp_floor: the five-iteration
presolve of the shift protocol); north_star's bar is 1e-6 relative. The achieved
errors and floors are printed and logged.

The parallel line search (groups of 4 trials, the default on Talos) is also compared
with the serial one on the same problems: identical to the last bit, including
elements that accept in a later group, accept in a slot above 0, or reject every trial.
"""
import os
import sys

import numpy as np
import pytest

import helpers
import oracle_lib
from crocoddyl_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

pytestmark = pytest.mark.gpu

FULL = {"C5_talos_walk": (100, 1024), "C4_solo12_trot": (60, 1024)}
TOL = 1e-8  # element-wise (helpers.elem_err); north_star's bar is 1e-6 relative


def _oracle_spots(solver, spots, pool=None, threads=3):
    p = solver.problem
    knots, pool0 = p._packed()
    d = _abi.Dims(p.nx, p.ndx, p.nu_max, p.T, len(spots))
    o = oracle_lib.Oracle(d, knots, pool0 if pool is None else pool, p.x0[spots], threads=threads)
    xs, us = solver.warm
    o.set_candidate(None if xs is None else xs[spots], None if us is None else us[spots], False)
    return o, knots


def _live_us(solver, us):
    """controls of the knots' own nu (the rows of nu = 0 impulse knots carry no control)"""
    live = np.zeros(us.shape[-2:], bool)
    for t, m in enumerate(solver.problem.runningModels):
        live[t, :m.nu] = True
    return np.where(live, us, 0.0)


def _snap(o):
    return helpers.results_dict(o.results()), o.xs(), o.us()


def _compare(solver, spots, what, ref, floors):
    """ref = the oracle's (results, xs, us) of the spot elements; floors = its
    conditioning floors (helpers.ulp_floor) of (cost, xs, us) for this protocol point."""
    ro, xo, uo = ref
    r = helpers.results_dict(solver._res())
    xs, us = np.asarray(solver.xs), np.asarray(solver.us)
    for i, b in enumerate(spots):
        for f in ("status", "iter", "n_iter_run", "steplength", "is_feasible"):
            assert r[f][b] == ro[f][i], (what, b, f, r[f][b], ro[f][i])
    # element-wise, each state / control coordinate at its own scale (helpers.elem_err)
    helpers.parity(f"{what} cost", r["cost"][spots], ro["cost"], TOL, floors[0])
    helpers.parity(f"{what} xs", xs[spots], xo, TOL, floors[1])
    helpers.parity(f"{what} us", _live_us(solver, us[spots]), _live_us(solver, uo), TOL, floors[2])
    assert np.all(np.isfinite(xs)) and np.all(np.isfinite(r["cost"])), what


def _with_floors(run, pool):
    """run(pool) -> list of oracle snapshots (results, xs, us); the snapshots at the
    unperturbed pool and, per snapshot, the floors of (cost, xs, us) (helpers.ulp_floor)"""
    flat = lambda p: tuple(a for r, x, u in run(p) for a in (r["cost"], x, u))  # noqa: E731
    base = run(pool)
    _, fl = helpers.ulp_floor(flat, pool)
    return base, [fl[3 * k:3 * k + 3] for k in range(len(base))]


@pytest.mark.parametrize("cfg", list(FULL))
def test_fullsize_fixed_protocol_vs_oracle(cfg):
    T, B = FULL[cfg]
    solver = bench.make_shard_solver(cfg, B, 0, 0, presolve=False)
    step = bench.FixedWarmStart(solver, 0)
    spots = np.array([0, B // 2, B - 1])

    def run(pool):
        o, _ = _oracle_spots(solver, spots, pool)
        o.solve(maxiter=1, is_feasible=False, reg_init=0.1)
        return [_snap(o)]

    (ref,), (floors,) = _with_floors(run, solver.problem._packed()[1])
    first = None
    for k in range(2):  # every step starts from the same warm start: same result twice
        step(1)
        _compare(solver, spots, f"{cfg} fixed step {k}", ref, floors)
        # (step 1's rollout dispatches the elements longest line search first, from step 0's
        # trial counts: the same solves to the last bit)
        cur = (np.asarray(solver.xs).copy(), np.asarray(solver.cost).copy(), np.asarray(solver.stepLength).copy())
        if first is None:
            first = cur
        else:
            for a, b2 in zip(first, cur):
                np.testing.assert_array_equal(a, b2)
    trials = bench.line_search_trials(solver)
    assert trials.min() >= 1 and trials.max() <= 10


@pytest.mark.parametrize("cfg", list(FULL))
def test_fullsize_shift_protocol_vs_oracle(cfg):
    T, B = FULL[cfg]
    solver = bench.make_shard_solver(cfg, B, 0, 0, presolve=True)
    spots = np.array([0, B // 2, B - 1])

    def run(pool):  # presolve, then two receding-horizon steps with the knot rotation
        o, knots = _oracle_spots(solver, spots, pool)
        o.solve(maxiter=5)
        out = [_snap(o)]
        for k in range(2):
            knots = knots[1:T] + knots[:1] + knots[T:]
            kd = (_abi.KnotDesc * len(knots))(*[_abi.KnotDesc(*x) for x in knots])
            assert o.L.oracle_set_knots(o.h, kd, _abi.dptr(o.pool), o.pool.size) == 0
            o.mpc_shift()
            o.solve(maxiter=1, is_feasible=False, reg_init=0.1)
            out.append(_snap(o))
        return out

    refs, floors = _with_floors(run, solver.problem._packed()[1])
    _compare(solver, spots, f"{cfg} presolve", refs[0], floors[0])
    for k in range(2):
        bench.mpc_step(solver, 1, rotate=True)
        _compare(solver, spots, f"{cfg} shift step {k}", refs[k + 1], floors[k + 1])
    q = np.linalg.norm(np.asarray(solver.xs)[..., 3:7], axis=-1)
    np.testing.assert_allclose(q, 1.0, atol=1e-9)


def _solver_with_npar(cfg, B, npar, monkeypatch):
    monkeypatch.setenv("CROCODDYL_AMD_LS_PAR", str(npar))  # read per handle at fddp_create
    return bench.make_shard_solver(cfg, B, 0, 0, presolve=True)


def test_parallel_line_search_equals_serial(monkeypatch):
    """the 4-trial groups of the parallel line search give the serial
    search's result bit for bit, on receding-horizon steps whose line searches accept
    at every alpha index 0..9 (slots above 0, later groups) or reject every trial."""
    cfg, B = "C5_talos_walk", 512
    out = {}
    for npar in (4, 1):
        s = _solver_with_npar(cfg, B, npar, monkeypatch)
        hist = np.zeros(11, int)
        snaps = []
        for _ in range(3):
            bench.mpc_step(s, 1, rotate=True)
            r = helpers.results_dict(s._res())
            L = s._h.refresh()
            xt = np.zeros((B, s.problem.T + 1, s.problem.nx))
            ut = np.zeros((B, s.problem.T, s.problem.nu_max))
            from crocoddyl_amd._lib import lib
            assert lib().fddp_get_xs_try(L, _abi.dptr(xt)) == 0 and lib().fddp_get_us_try(L, _abi.dptr(ut)) == 0
            snaps.append((r, np.asarray(s.xs).copy(), np.asarray(s.us).copy(), xt, ut))
            hist += np.bincount(bench.line_search_trials(s).astype(int), minlength=11)
        out[npar] = (snaps, hist)
    (par, hist), (ser, _) = out[4], out[1]
    for k, (a, b) in enumerate(zip(par, ser)):
        ra, rb = a[0], b[0]
        for f in ("status", "iter", "n_iter_run", "is_feasible"):
            np.testing.assert_array_equal(ra[f], rb[f], err_msg=f"step {k} {f}")
        for f in ("steplength", "cost", "dV", "dVexp", "xreg", "stop"):
            np.testing.assert_array_equal(ra[f], rb[f], err_msg=f"step {k} {f}")
        np.testing.assert_array_equal(a[1], b[1], err_msg=f"step {k} xs")
        np.testing.assert_array_equal(a[2], b[2], err_msg=f"step {k} us")
        # the trial buffer: the accepted trial, or the last rejected one (alpha_9)
        np.testing.assert_array_equal(a[3], b[3], err_msg=f"step {k} xs_try")
        np.testing.assert_array_equal(a[4], b[4], err_msg=f"step {k} us_try")
    # coverage of the parallel search's cases: accepted in group 0 slot > 0, in a
    # later group, and the 10-trial searches (accepted at alpha_9 or all rejected)
    assert hist[2:5].sum() > 0 and hist[5:10].sum() > 0 and hist[10] > 0, hist.tolist()


def test_adaptive_trial_groups_give_the_same_solves():
    """The trial-group size chosen per solve from the last line search's trial counts
    (fddp_hip.hip choose_npar) changes the work, not the result: the default handle's
    receding-horizon steps equal the serial handle's bit for bit."""
    cfg, B = "C5_talos_walk", 256
    res = []
    for env in (None, "1"):
        if env:
            os.environ["CROCODDYL_AMD_LS_PAR"] = env
        try:
            s = bench.make_shard_solver(cfg, B, 0, 0, presolve=True)
        finally:
            os.environ.pop("CROCODDYL_AMD_LS_PAR", None)
        snaps = []
        for _ in range(3):
            bench.mpc_step(s, 1, rotate=True)
            snaps.append((np.asarray(s.xs).copy(), np.asarray(s.cost).copy(), np.asarray(s.stepLength).copy()))
        res.append(snaps)
    for (xa, ca, sa), (xb, cb, sb) in zip(*res):
        np.testing.assert_array_equal(sa, sb)
        np.testing.assert_array_equal(ca, cb)
        np.testing.assert_array_equal(xa, xb)
