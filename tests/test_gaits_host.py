"""Gait problems (crocoddyl_amd.gaits: utils/biped.py, utils/quadruped.py) on the
code-built Talos (nv = 38) and Solo12 (nv = 18) — CPU only.

The device knot code compiled for the host (tests/cpp/mb_host.cpp) vs the numpy
oracle (oracle/multibody_np.py) on every knot kind the gaits produce: swing knots
(contacts, CoM, friction cones with QuadraticBarrier, swing-foot placement /
translation), double support, the biped's pseudo-impulse foot switch (Euler dt = 0,
CostModelFrameVelocity) and the quadruped's impulse foot switch; plus the
quasi-static controls (contact-fwddyn.hxx:169-207: zero acceleration) and the gait
geometry (feet / CoM references as biped.py:36-62 / quadruped.py:173-205)."""
import numpy as np
import pytest

from crocoddyl_amd import gaits, robots, synthetic
from oracle import multibody_np as onp
from test_multibody_host import lib, _p  # noqa: F401


@pytest.fixture(scope="module")
def talos_walk():
    talos = robots.sample_talos()
    g = gaits.SimpleBipedGaitProblem(talos, "right_sole_link", "left_sole_link")
    return g, g.createWalkingModels(talos.defaultState, 0.6, 0.1, 0.0375, 48, 1)


@pytest.fixture(scope="module")
def solo_trot():
    solo = robots.sample_solo12()
    g = gaits.SimpleQuadrupedalGaitProblem(solo, "FL_FOOT", "FR_FOOT", "HL_FOOT", "HR_FOOT")
    return g, g.createTrottingModels(solo.defaultState, 0.15, 0.1, 1e-2, 27, 2)


def test_gait_shapes(talos_walk, solo_trot):
    g, models = talos_walk
    assert len(models) == 100
    kinds = [type(m.differential).__name__ for m in models]
    assert set(kinds) == {"DifferentialActionModelContactFwdDynamics"}
    assert [m.dt for m in models].count(0.0) == 2  # the two pseudo-impulse foot switches
    ncs = [m.differential.contacts.nc for m in models]
    assert ncs[0] == 12 and ncs[1] == 6 and ncs[49] == 6 and ncs[50] == 12  # double / single support
    gq, qm = solo_trot
    assert len(qm) == 60
    imp = [i for i, m in enumerate(qm) if type(m).__name__ == "ActionModelImpulseFwdDynamics"]
    assert imp == [29, 59]
    # the last swing knot's CoM target has advanced by half the (half) step
    com = qm[28].differential.costs.costs["comTrack"].cost.cref
    q0 = gq.rmodel.defaultState[:gq.state.nq]
    feet = [gq.rmodel.framePlacement(q0, f).translation for f in gq._all]
    np.testing.assert_allclose(com[:2], (sum(feet) / 4)[:2] + [0.5 * 0.075, 0.0], atol=1e-12)


def _check_knot(lib, model, x, u, terminal=False, tol=1e-9):  # noqa: F811
    kind, nu, blk = model.pack()
    blk = np.ascontiguousarray(blk[0])
    st = model.state
    nx, n = st.nx, st.ndx
    k = {5: onp.ContactFwdKnot, 6: onp.ImpulseFwdKnot}.get(kind, onp.FreeFwdKnot)(blk, nx, nu)
    use_u = 0 if (terminal or nu == 0) else 1
    uo = None if not use_u else u
    xn = np.zeros(nx)
    uu = u if nu else np.zeros(1)
    c = lib.mb_host_calc(_p(blk), nx, _p(x), _p(uu), use_u, _p(xn))
    xo, co = k.calc(x, uo)
    np.testing.assert_allclose(xn, xo, rtol=1e-10, atol=1e-10)
    assert c == pytest.approx(co, rel=1e-10, abs=1e-12)
    m = max(nu, 1)
    out = {q: np.zeros(s) for q, s in [("Fx", n * n), ("Fu", n * m), ("Lxx", n * n), ("Lxu", n * m),
                                       ("Luu", m * m), ("Lx", n), ("Lu", m)]}
    xn2, c2 = np.zeros(nx), np.zeros(1)
    lib.mb_host_calc_diff(_p(blk), nx, m, _p(x), _p(uu), use_u,
                          *[_p(out[q]) for q in ["Fx", "Fu", "Lxx", "Lxu", "Luu", "Lx", "Lu"]], _p(xn2), _p(c2))
    np.testing.assert_allclose(xn2, xo, rtol=1e-10, atol=1e-10)
    assert c2[0] == pytest.approx(co, rel=1e-10, abs=1e-12)
    ref = k.calc_diff(x, uo)
    for q, a in out.items():
        if kind == 6 and q not in ("Fx", "Lxx", "Lx"):
            continue
        rows = m if q == "Luu" else n
        got = a.reshape(-1, rows).T if q in ("Fx", "Fu", "Lxx", "Lxu", "Luu") else a
        want = ref[q]
        if q in ("Fu", "Lxu"):
            got = got[:, :nu]
        if q == "Luu":
            got = got[:nu, :nu]
        if q == "Lu":
            got = got[:nu]
        if want.size == 0:
            continue
        scale = max(1.0, float(np.max(np.abs(want))))
        err = float(np.max(np.abs(got - want)))
        assert err / scale < tol, (q, err, scale)


TALOS_KNOTS = [0, 1, 20, 49, 50, 75, 99]


@pytest.mark.parametrize("t", TALOS_KNOTS)
def test_talos_walk_knots_vs_oracle(lib, talos_walk, t):  # noqa: F811
    g, models = talos_walk
    rng = np.random.default_rng(t)
    x0 = g.rmodel.defaultState
    x = g.state.integrate(x0, np.concatenate([rng.uniform(-0.05, 0.05, g.state.nv), rng.uniform(-0.3, 0.3, g.state.nv)]))
    u = models[t].quasiStatic(None, x0) + rng.uniform(-2, 2, models[t].nu)
    _check_knot(lib, models[t], x, u, tol=1e-8)


@pytest.mark.parametrize("t", [0, 2, 15, 29, 30, 59])
def test_solo_trot_knots_vs_oracle(lib, solo_trot, t):  # noqa: F811
    g, models = solo_trot
    rng = np.random.default_rng(100 + t)
    x0 = g.rmodel.defaultState
    x = g.state.integrate(x0, np.concatenate([rng.uniform(-0.1, 0.1, g.state.nv), rng.uniform(-0.5, 0.5, g.state.nv)]))
    u = rng.uniform(-1, 1, models[t].nu) if models[t].nu else np.zeros(0)
    if models[t].nu:
        u = u + models[t].quasiStatic(None, x0)
    _check_knot(lib, models[t], x, u, tol=1e-8)


def test_quasi_static_holds_still(talos_walk, solo_trot):
    for g, models, ts in ((talos_walk[0], talos_walk[1], (0, 20)), (solo_trot[0], solo_trot[1], (0, 10))):
        x0 = g.rmodel.defaultState
        for t in ts:
            m = models[t]
            u = m.quasiStatic(None, x0)
            k = onp.ContactFwdKnot(m.pack()[2][0], g.state.nx, m.nu)
            a, _ = k.accel_force(x0, u)
            assert np.max(np.abs(a)) < 1e-8


@pytest.mark.parametrize("t", [0, 1, 49])
def test_talos_active_friction_cones(lib, talos_walk, t):  # noqa: F811
    """Large tangential forces put the friction-cone barriers on (Arr = 1 rows) at the
    reference posture (v = 0): knots whose first cost-derivative group is a control
    diagonal (double support: ctrlReg before the cones in name order) included."""
    g, models = talos_walk
    x = g.rmodel.defaultState.copy()
    rng = np.random.default_rng(20 + t)
    m = models[t]
    hit = 0
    for _ in range(6):
        u = m.quasiStatic(None, x) + rng.uniform(-300, 300, m.nu)
        k = onp.ContactFwdKnot(m.pack()[2][0], x.size, m.nu)
        _, res = k._calc_res(x, u)
        hit += sum(int(np.any(c.a_hess(np.real(r)) > 0)) for c, r in zip(k.costs, res) if c.type == onp.FRICTION_CONE)
        _check_knot(lib, m, x, u, tol=1e-8)
    assert hit > 0


@pytest.mark.parametrize("t", [0, 1, 49, 99])
def test_talos_spilled_plan_equals_lds_plan(lib, talos_walk, t, monkeypatch):  # noqa: F811
    """The spilled calcDiff plan (multibody.hpp diff_spill: dtau/dx, the body maps and
    their subtree sums, the jac-cost Jacobians, d lambda / dx in the knot's own output
    blocks; the Talos
    knots fit two workgroups per CU under it) computes the all-LDS plan's blocks bit for
    bit: only where the arrays live changes."""
    import ctypes as C
    g, models = talos_walk
    model = models[t]
    kind, nu, blk = model.pack()
    blk = np.ascontiguousarray(blk[0])
    nx, n, m = model.state.nx, model.state.ndx, max(nu, 1)
    lib.mb_host_plan.argtypes = [C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_int64)]
    lds = C.c_int64(0)
    flags = lib.mb_host_plan(_p(blk), m, C.byref(lds))
    assert flags & 3 == 3, flags  # blocks and Jacobians spilled (and d lambda / dx with contacts)
    assert lds.value <= 80 * 1024, lds.value
    rng = np.random.default_rng(t)
    x0 = g.rmodel.defaultState
    x = g.state.integrate(x0, np.concatenate([rng.uniform(-0.05, 0.05, g.state.nv), rng.uniform(-0.3, 0.3, g.state.nv)]))
    u = model.quasiStatic(None, x0) + rng.uniform(-2, 2, nu)
    outs = []
    for spill in (None, "0"):
        if spill is None:
            monkeypatch.delenv("MB_HOST_SPILL", raising=False)
        else:
            monkeypatch.setenv("MB_HOST_SPILL", spill)
        o = [np.zeros(s) for s in (n * n, n * m, n * n, n * m, m * m, n, m, nx, 1)]
        lib.mb_host_calc_diff(_p(blk), nx, m, _p(x), _p(u), 1 if nu else 0, *[_p(a) for a in o])
        outs.append(o)
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)



def test_talos_rollout_fits_three_workgroups_per_cu(lib, talos_walk):  # noqa: F811
    """The multibody rollout's LDS on the C5 walk's knots (the dense knot calc of
    multibody.hpp knot_calc_dense_x, its factorisation over the dead recursion records,
    and dx in that scratch's tail): at most 53,248 B per workgroup with 256 B to spare for
    the kernel's static LDS, i.e. three workgroups per CU with the LDS allocated in 2 KB
    granules (tools/occ_probe.hip: 53,248 B fit three, 53,776 B two); the dense calc's
    scratch is smaller than the tree calc's."""
    import ctypes as C
    g, models = talos_walk
    lib.mb_host_rollout_lds.restype = C.c_int64
    lib.mb_host_rollout_lds.argtypes = [C.POINTER(C.c_double), C.c_int, C.c_int, C.POINTER(C.c_int64),
                                        C.POINTER(C.c_int64)]
    nu_max = max(m.nu for m in models)
    worst = 0
    for model in models:
        kind, nu, blk = model.pack()
        blk = np.ascontiguousarray(blk[0])
        dense, work = C.c_int64(0), C.c_int64(0)
        lds = lib.mb_host_rollout_lds(_p(blk), model.state.nx, nu_max, C.byref(dense), C.byref(work))
        assert dense.value < work.value, (dense.value, work.value)
        worst = max(worst, lds)
    granule = 2048
    assert 3 * (-(-(worst + 256) // granule) * granule) <= 160 * 1024, worst
