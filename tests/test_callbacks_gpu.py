"""Per-iteration callbacks (fddp.cpp:92-98) on the HIP path: the reference's
CallbackLogger (bindings/python/crocoddyl/__init__.py:356-381) records one entry per
iteration, and its cost / stop / steplength / xreg / ureg / grad traces equal the
C++ oracle's per-iteration trace (recorded at the same point of the loop body).
Batched: every element's trace through ``solver.callbackMask``. The bar is the
solver bar (1e-9 relative for the LQ / unicycle problems, 1e-8 element-wise on the C5 knots)."""
import io

import numpy as np
import pytest

import helpers
import oracle_lib
from crocoddyl_amd import _abi

pytestmark = pytest.mark.gpu


def _oracle_traces(d, knots, pool, x0s, xs=None, us=None, maxiter=100):
    o = oracle_lib.Oracle(d, knots, pool, x0s, threads=4)
    o.set_candidate(xs, us, False)
    o.solve(maxiter=maxiter)
    return [o.trace(b) for b in range(d.B)]


def _close(a, b, tol):
    return abs(a - b) <= tol * max(1.0, abs(b))


def test_callback_logger_unicycle():
    import crocoddyl_amd as crocoddyl
    model = crocoddyl.ActionModelUnicycle()
    x0 = np.array([-1.0, -1.0, 1.0])
    problem = crocoddyl.ShootingProblem(x0, [model] * 30, model)
    solver = crocoddyl.SolverFDDP(problem)
    log = crocoddyl.CallbackLogger()
    buf = io.StringIO()
    solver.setCallbacks([log, crocoddyl.CallbackVerbose(crocoddyl.VerboseLevel._2, stream=buf)])
    assert solver.solve()
    knots, pool = crocoddyl.pack_problem([model] * 30, model, 1)
    tr = _oracle_traces(_abi.Dims(3, 3, 2, 30, 1), knots, pool, x0[None])[0]
    assert len(log.costs) == len(tr) == solver.iter + 1
    assert log.iters == list(range(len(tr)))
    for i, rec in enumerate(tr):
        assert _close(log.costs[i], rec[0], 1e-9), (i, log.costs[i], rec[0])
        assert _close(log.stops[i], rec[1], 1e-9)
        assert log.steps[i] == rec[6]
        assert _close(log.x_regs[i], rec[4], 1e-12) and _close(log.u_regs[i], rec[5], 1e-12)
        # grad: -expectedImprovement()[1] called inside the loop (xs_try == xs after an
        # accepted step, so the trial term drops out: -dq)
        assert np.isfinite(log.grads[i])
    np.testing.assert_array_equal(np.asarray(log.xs), np.asarray(solver.xs))
    text = buf.getvalue()
    assert text.count("\n") == len(tr) + (len(tr) + 9) // 10 and "dV-exp" in text


def test_callbacks_batched_mask():
    """Elements converge at different iterations: each element's trace, read through
    callbackMask, equals its own oracle trace."""
    S = helpers.setup("C1_unicycle", T=30, B=6, seed=3)
    d = S["dims"]
    import crocoddyl_amd as crocoddyl
    problem = crocoddyl.ShootingProblem(S["x0s"], S["running"], S["terminal"])
    solver = crocoddyl.SolverFDDP(problem)
    rows = [[] for _ in range(d.B)]

    def cb(s):
        m = s.callbackMask
        assert m is not None and m.shape == (d.B,)
        cost, stop, sl, xr, it = s.cost, s.stop, s.stepLength, s.x_reg, s.iter
        for b in np.flatnonzero(m):
            rows[b].append((it[b], cost[b], stop[b], sl[b], xr[b]))

    solver.setCallbacks([cb])
    solver.solve()
    traces = _oracle_traces(d, S["knots"], S["pool"], S["x0s"])
    lens = [len(t) for t in traces]
    assert len(set(lens)) > 1, lens  # the mask is exercised
    for b in range(d.B):
        assert len(rows[b]) == lens[b], (b, len(rows[b]), lens[b])
        for i, (it, cost, stop, sl, xr) in enumerate(rows[b]):
            rec = traces[b][i]
            assert it == i and sl == rec[6] and _close(cost, rec[0], 1e-9) and _close(stop, rec[1], 1e-9)
            assert _close(xr, rec[4], 1e-12)
    assert solver.callbackMask is None  # cleared after solve


def test_callbacks_c5_walk_trace():
    """The headline knots: C5 Talos walk, T = 8, B = 2, solve(maxiter = 3) from the
    reference benchmark's warm start through the C ABI hook; per-iteration traces vs
    the oracle's."""
    import ctypes as C
    import bench
    S = helpers.setup("C5_talos_walk", T=8, B=2)
    d = S["dims"]
    xs, us = bench.warm_start_arrays("C5_talos_walk", S["running"], S["x0s"], d)
    g = helpers.Gpu(d, S["knots"], S["pool"], S["x0s"])
    g.set_candidate(xs, us, False)
    got = []

    def on_iter(_u, it, res, rep, B):
        got.append((it, [(res[b].cost, res[b].stop, res[b].steplength, res[b].xreg, res[b].d1) for b in range(B)],
                    [rep[b] for b in range(B)]))
        return 0

    cfn = _abi.IterationCallback(on_iter)
    g._ok(g.L.fddp_set_callback(g.h, cfn, None))
    g.solve(maxiter=3)
    g._ok(g.L.fddp_set_callback(g.h, _abi.IterationCallback(), None))
    traces = _oracle_traces(d, S["knots"], S["pool"], S["x0s"], xs, us, maxiter=3)
    for b in range(d.B):
        mine = [(it, vals[b]) for it, vals, rep in got if rep[b]]
        assert len(mine) == len(traces[b])
        for (it, (cost, stop, sl, xr, d1)), rec in zip(mine, traces[b]):
            assert sl == rec[6] and xr == rec[4]
            helpers.parity(f"C5 callback trace b{b} it{it}", [cost, stop, d1], [rec[0], rec[1], rec[3]], 1e-8)


def test_callback_exception_propagates():
    import crocoddyl_amd as crocoddyl
    model = crocoddyl.ActionModelUnicycle()
    solver = crocoddyl.SolverFDDP(crocoddyl.ShootingProblem(np.array([-1.0, -1.0, 1.0]), [model] * 10, model))

    calls = []

    def boom(s):
        calls.append(int(s.iter))
        if s.iter == 2:
            raise KeyError("from callback")

    solver.setCallbacks([boom])
    with pytest.raises(KeyError):
        solver.solve()
    # the exception left solve() in the iteration that raised (fddp.cpp:92-98): no
    # further iterations ran or called back, and the solver's state is that iteration's
    assert calls == [0, 1, 2]
    assert solver.iter == 2
    cost_at_2 = solver.cost
    ref = crocoddyl.SolverFDDP(crocoddyl.ShootingProblem(np.array([-1.0, -1.0, 1.0]), [model] * 10, model))
    ref.solve([], [], 3)
    assert cost_at_2 == ref.cost  # (ref.iter is 3: its loop ran to maxiter)
    np.testing.assert_array_equal(np.asarray(solver.xs), np.asarray(ref.xs))
    solver.setCallbacks([])
    assert solver.solve()


def test_c_abi_callback_abort():
    """fddp_iteration_callback returning nonzero stops fddp_solve after that iteration:
    FDDP_ERR_CALLBACK_ABORT, `out` holding that iteration's results (iter, cost), and
    the trajectories equal a solve that stopped there by maxiter."""
    S = helpers.setup("C1_unicycle", T=30, B=3, seed=5)
    d = S["dims"]
    g = helpers.Gpu(d, S["knots"], S["pool"], S["x0s"])
    g.set_candidate(None, None, False)
    seen = []

    def on_iter(_u, it, res, rep, B):
        seen.append(it)
        return 1 if it == 1 else 0

    cfn = _abi.IterationCallback(on_iter)
    g._ok(g.L.fddp_set_callback(g.h, cfn, None))
    r = (_abi.Result * d.B)()
    rc = g.L.fddp_solve(g.h, 100, 0, 1e-9, r)
    g._ok(g.L.fddp_set_callback(g.h, _abi.IterationCallback(), None))
    assert rc == _abi.FDDP_ERR_CALLBACK_ABORT
    assert seen == [0, 1]
    assert [x.iter for x in r] == [1] * d.B
    xs_abort = g.xs()
    g2 = helpers.Gpu(d, S["knots"], S["pool"], S["x0s"])
    g2.set_candidate(None, None, False)
    r2 = g2.solve(maxiter=2)
    np.testing.assert_array_equal(xs_abort, g2.xs())
    assert [x.cost for x in r] == [x.cost for x in r2]
