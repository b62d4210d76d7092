"""CPU side of SolverDDP's phase entry points (calcDiff / backwardPass / forwardPass,
reference ddp.cpp:157-253, fddp.cpp:149-225): the C++ oracle's phases compose to its
step API bit for bit (computeDirection = calcDiff + backwardPass, ddp.cpp:120-125;
tryStep = cost - cost_try, ddp.cpp:127-130), and forwardPass checks its step length
(fddp.cpp:150-153). The device entry points are compared with these in
tests/test_phases_gpu.py."""
import numpy as np
import pytest

import helpers
import oracle_lib
from crocoddyl_amd import _abi


@pytest.mark.parametrize("name,kw", [("C2_lqr", dict(T=20, B=3)), ("C5_talos_walk", dict(T=4, B=2))])
def test_oracle_phases_compose_to_the_step_api(name, kw):
    S = helpers.setup(name, **kw)
    d = S["dims"]
    rng = np.random.default_rng(3)
    xs = S["x0s"][:, None, :].repeat(d.T + 1, axis=1) + (0.0 if name.startswith("C5") else
                                                          rng.uniform(-0.1, 0.1, (d.B, d.T + 1, d.nx)))
    us = np.zeros((d.B, d.T, d.nu_max))
    a = oracle_lib.Oracle(d, S["knots"], S["pool"], S["x0s"])
    b = oracle_lib.Oracle(d, S["knots"], S["pool"], S["x0s"])
    for h in (a, b):
        h.set_candidate(xs, us, False)
        h.set_solver_state(it=0, xreg=1e-9, ureg=1e-9)
    cost = a.ddp_calc_diff()
    sa = a.backward_pass()
    sb = b.compute_direction(True)
    np.testing.assert_array_equal(sa, sb)
    for q, nk, per in ((_abi.Q_K, d.T, d.nu_max * d.ndx), (_abi.Q_KV, d.T, d.nu_max), (_abi.Q_FS, d.T + 1, d.ndx)):
        np.testing.assert_array_equal(a.quantity(q, nk, per), b.quantity(q, nk, per))
    for alpha in (1.0, 0.25):
        rc, ct, st = a.forward_pass(alpha)
        dV, st2 = b.try_step(alpha)
        assert rc == 0
        np.testing.assert_array_equal(st, st2)
        np.testing.assert_array_equal(cost - ct, dV)
        np.testing.assert_array_equal(a.xs(trial=True), b.xs(trial=True))
        np.testing.assert_array_equal(a.us(trial=True), b.us(trial=True))
    rc, _, _ = a.forward_pass(1.5)
    assert rc == _abi.FDDP_ERR_INVALID_ARG


def test_header_declares_the_phase_entry_points():
    import os
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                            "fddp_hip.h")).read()
    for sym in ("fddp_calc_diff(", "fddp_backward_pass(", "fddp_forward_pass(", "fddp_abi_version("):
        assert sym in hdr
    assert f"#define FDDP_ABI_VERSION {_abi.ABI_VERSION}" in hdr
