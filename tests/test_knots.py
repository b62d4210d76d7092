"""Heterogeneous knot sequences and the MPC plumbing of
ShootingProblem (§8f #3: circularAppend / updateNode / updateModel,
shooting.hxx:235-346, through fddp_set_knots).

CPU: the C++ oracle == the numpy restatement on heterogeneous sequences
(two parameter sets alternating along t, nu = 0 knots); the oracle's
set_knots == a fresh oracle built on the new sequence.
GPU: the device == the oracle on the same sequences, on every device path,
and after knot-sequence updates (C ABI and the Python facade).
"""
import numpy as np
import pytest

import helpers
import oracle_lib
from crocoddyl_amd import _abi, synthetic
from crocoddyl_amd.problem import pack_problem
from oracle import fddp_np

RTOL = 1e-8  # element-wise (helpers.elem_err); north_star: xs/us/cost within 1e-6 relative


def hetero_setup(name, T, B, **kw):
    x0s, running, terminal = synthetic.build_hetero(name, T=T, B=B, **kw)
    knots, pool = pack_problem(running, terminal, B)
    nx = running[0].state.nx
    dims = _abi.Dims(nx, nx, max(m.nu for m in running), T, B)
    return dict(dims=dims, knots=knots, pool=pool, x0s=x0s, running=running, terminal=terminal)


def _solve(h, maxiter=100):
    h.set_candidate(None, None, False)
    return helpers.results_dict(h.solve(maxiter=maxiter))


def _live(us, knots):
    """Controls with the entries beyond each knot's nu zeroed: a trial never
    writes them (fddp.cpp:163-170), so after a knot-sequence change they hold
    whatever the buffer held (the reference keeps stale values, the device
    zeros)."""
    us = np.array(us)
    for t, k in enumerate(knots[:-1]):
        us[:, t, k[1]:] = 0.
    return us


def _same(rg, ro, g, o, knots=None):
    for f in ("status", "iter", "n_iter_run", "is_feasible", "xreg"):
        np.testing.assert_array_equal(rg[f], ro[f], err_msg=f)
    helpers.parity("xs", g.xs(), o.xs(), RTOL)
    if knots is None:
        helpers.parity("us", g.us(), o.us(), RTOL)
    else:
        helpers.parity("us (live)", _live(g.us(), knots), _live(o.us(), knots), RTOL)
    assert float(np.max(np.abs(rg["cost"] - ro["cost"]) / np.maximum(1, np.abs(ro["cost"])))) < RTOL


@pytest.mark.parametrize("name,T,B", [("C2_lqr", 30, 3), ("C3_talos_arm", 24, 2)])
def test_hetero_oracle_matches_numpy(name, T, B):
    S = hetero_setup(name, T, B)
    assert 0 in [k[1] for k in S["knots"]] and len({k[2] for k in S["knots"]}) >= 3
    o = oracle_lib.Oracle(S["dims"], S["knots"], S["pool"], S["x0s"], threads=4)
    r = _solve(o)
    xs, us = o.xs(), o.us()
    for b in range(B):
        models = fddp_np.bind_problem(S["knots"], S["pool"], b, S["dims"].nx)
        s = fddp_np.FDDP(S["x0s"][b], models)
        s.solve(maxiter=100)
        assert r["status"][b] == s.status == 1 and r["iter"][b] == s.iter
        np.testing.assert_allclose(xs[b], np.array(s.xs), rtol=0, atol=1e-9)
        np.testing.assert_allclose(us[b], np.array(s.us), rtol=0, atol=1e-9)


def _rotated(S, new_model):
    """knots / pool after circularAppend(new_model) on S's sequence."""
    running = S["running"][1:] + [new_model]
    knots, pool = pack_problem(running, S["terminal"], S["dims"].B)
    return running, knots, pool


def test_oracle_set_knots_equals_fresh():
    S = hetero_setup("C2_lqr", 20, 2)
    o = oracle_lib.Oracle(S["dims"], S["knots"], S["pool"], S["x0s"], threads=4)
    _solve(o, 5)
    xs, us = o.xs(), o.us()
    running, knots, pool = _rotated(S, S["running"][6])  # a nu = 0 knot appended
    kd = (_abi.KnotDesc * len(knots))(*[_abi.KnotDesc(*k) for k in knots])
    assert o.L.oracle_set_knots(o.h, kd, _abi.dptr(pool), pool.size) == 0
    f = oracle_lib.Oracle(S["dims"], knots, pool, S["x0s"], threads=4)
    for h in (o, f):
        h.set_candidate(xs, us, False)
    ro, rf = helpers.results_dict(o.solve(3)), helpers.results_dict(f.solve(3))
    np.testing.assert_array_equal(ro["iter"], rf["iter"])
    np.testing.assert_array_equal(o.xs(), f.xs())
    # controls of nu = 0 knots are never written by a trial (fddp.cpp:163-170):
    # they keep whatever the buffer held; compare the live entries
    for t, m in enumerate(running):
        np.testing.assert_array_equal(o.us()[:, t, :m.nu], f.us()[:, t, :m.nu])


def test_facade_node_updates_validate():
    """Argument checks of circularAppend / updateNode / updateModel (shooting.hxx:241-252, 286-303, 321-333)."""
    import crocoddyl_amd as crocoddyl
    m = crocoddyl.ActionModelLQR(4, 2)
    p = crocoddyl.ShootingProblem(np.zeros(4), [m] * 5, m)
    with pytest.raises(ValueError):
        p.circularAppend(crocoddyl.ActionModelLQR(5, 2))
    with pytest.raises(ValueError):
        p.circularAppend(crocoddyl.ActionModelLQR(4, 3))  # nu > nu_max
    with pytest.raises(ValueError):
        p.updateNode(7, m, m.createData())
    with pytest.raises(ValueError):
        p.updateModel(5, m)  # i == T: the reference indexes past its running models
    m1 = crocoddyl.ActionModelLQR(4, 1)
    p.circularAppend(m1)
    assert p.runningModels[-1] is m1 and p.runningModels[0] is m and p.T == 5
    p.updateModel(6, m1)
    assert p.terminalModel is m1
    p.updateNode(0, m1, m1.createData())
    assert p.runningModels[0] is m1


