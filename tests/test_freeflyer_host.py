"""Free-flyer roots (StateMultibody on SE(3) x R^n) — CPU only.

1. Pins the numpy oracle's free-flyer arithmetic (oracle/multibody_np.py):
   * the state's Lie-group identities: integrate(x, diff(x, y)) == y,
     diff(x, integrate(x, dx)) == dx, exp6 / log6 round trips, unit quaternions
     kept by integrate (pinocchio SpecialEuclideanOperationTpl<3>);
   * rigid-body identities with a 6-dof root: ABA == CRBA^-1 (tau - RNEA(q, v, 0)),
     RNEA(q, v, ABA) == tau, and a single free body's Newton-Euler equations in
     closed form (m (a_lin + w x v) = R^T m g, I dw + w x I w = 0 about the CoM);
   * tangent-space derivatives vs central finite differences on the manifold at the
     reference's numdiff tolerance (unittest/test_actions.cpp:70-110 design).
2. The device multibody knot code compiled for the host (tests/cpp/mb_host.cpp)
   vs that oracle on floating-base knots: free dynamics with
   ActuationModelFloatingBase, 3D / 6D contacts, impulses, state costs on the
   manifold (Jlog6 block), frame / CoM / contact-force costs, the Euler step's
   Jexp6 / Ad(exp6^-1) assembly (euler.hxx:83-131 + multibody.hxx:147-240).
"""
import numpy as np
import pytest

from crocoddyl_amd import multibody as mb, synthetic
from oracle import multibody_np as onp
from test_multibody_host import lib, _p  # noqa: F401  (the host build of the device code)


def _robot(model):
    body = model.pack_robot(np.zeros(model.nv))
    r, _ = onp.parse_robot(body, model.nv)
    return r


def _rand_q(model, rng):
    st = mb.StateMultibody(model)
    return synthetic.random_floating_state(model, rng, 1, spread=0.8)[0][:st.nq]


def test_state_group_identities():
    model = mb.sample_tree(4, seed=1, freeflyer=True)
    r = _robot(model)
    st = mb.StateMultibody(model)
    rng = np.random.default_rng(0)
    for _ in range(20):
        x = synthetic.random_floating_state(model, rng, 1, spread=1.5, v_spread=1.0)[0]
        y = synthetic.random_floating_state(model, rng, 1, spread=1.5, v_spread=1.0)[0]
        np.testing.assert_allclose(np.linalg.norm(x[3:7]), 1.0, atol=1e-12)
        d = r.state_diff(x, y)
        z = r.state_integrate(x, d)
        # same pose (the quaternion up to sign)
        np.testing.assert_allclose(onp.quat_to_R(z[3:7]), onp.quat_to_R(y[3:7]), atol=1e-10)
        np.testing.assert_allclose(z[:3], y[:3], atol=1e-10)
        np.testing.assert_allclose(z[7:], y[7:], atol=1e-10)
        dx = rng.uniform(-1, 1, st.ndx)
        np.testing.assert_allclose(r.state_diff(x, r.state_integrate(x, dx)), dx, atol=1e-10)
        # the product-side StateMultibody agrees with the oracle's restatement
        np.testing.assert_allclose(st.diff(x, y), d, atol=1e-12)
        np.testing.assert_allclose(st.integrate(x, dx), r.state_integrate(x, dx), atol=1e-12)
        # exp6 / log6
        nu = rng.uniform(-2, 2, 6)
        R, p = onp.exp6(nu)
        np.testing.assert_allclose(onp.log6(R, p), nu, atol=1e-10)


def test_aba_crba_rnea_with_freeflyer():
    model = mb.sample_tree(6, seed=7, freeflyer=True)
    r = _robot(model)
    rng = np.random.default_rng(2)
    for _ in range(5):
        q = _rand_q(model, rng)
        v, tau = rng.uniform(-1, 1, r.nv), rng.uniform(-2, 2, r.nv)
        M = r.crba(q)
        np.testing.assert_allclose(M, M.T, atol=1e-12)
        assert np.all(np.linalg.eigvalsh(M) > 0)
        a = r.aba(q, v, tau)
        nle = r.rnea(q, v, np.zeros(r.nv))
        np.testing.assert_allclose(a, np.linalg.solve(M, tau - nle), rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(r.rnea(q, v, a), tau, rtol=1e-9, atol=1e-9)


def test_free_body_newton_euler_closed_form():
    """A single free body: the base twist (v, w) in body axes obeys
    m (dv + w x v) = R^T m g and I_c dw + w x I_c w = 0 about its CoM (here the CoM
    is at the joint origin)."""
    model = mb.RobotModel(mb.JointModelFreeFlyer())
    m, Ic = 2.3, np.diag([0.11, 0.23, 0.31])
    model.appendBodyToJoint(1, mb.Inertia(m, np.zeros(3), Ic))
    r = _robot(model)
    rng = np.random.default_rng(4)
    for _ in range(5):
        q = _rand_q(model, rng)
        v = rng.uniform(-1, 1, 6)
        a = r.aba(q, v, np.zeros(6))
        R = onp.quat_to_R(q[3:7])
        g = np.array([0.0, 0.0, -9.81])
        np.testing.assert_allclose(m * (a[:3] + np.cross(v[3:], v[:3])), R.T @ (m * g), atol=1e-10)
        np.testing.assert_allclose(Ic @ a[3:] + np.cross(v[3:], Ic @ v[3:]), np.zeros(3), atol=1e-10)


FF_CASES = [dict(), dict(weighted=True, com=True),
            dict(contacts=[("6d", "tip")]), dict(contacts=[("3d", "tip"), ("3d", "mid_site")], weighted=True),
            dict(contacts=[("6d", "tip"), ("3d", "mid_site")], damping=1e-3, com=True, gains=(0.0, 50.0)),
            dict(contacts=[("6d", "tip")], force_costs=True), dict(contacts=[("3d", "mid_site")], force_costs=True,
                                                                     weighted=True),
            dict(robot=mb.sample_tree(8, seed=9, freeflyer=True), contacts=[("6d", "tip")], com=True,
                 armature=np.concatenate([np.zeros(6), np.full(8, 0.02)])),
            # friction cones (QuadraticBarrier on the cone), frame velocity, barrier activations
            dict(contacts=[("6d", "tip"), ("3d", "mid_site")], friction=True),
            dict(contacts=[("3d", "mid_site")], friction=True, fvel=True, barrier=True, com=True),
            dict(fvel=True, barrier=True),
            dict(contacts=[("6d", "tip")], friction=True, enable_force=False, fvel=True)]


def _fd_check(k, x, u, ref, nu):
    """Central finite differences on the manifold of the oracle's calc."""
    h = 1e-6
    n = k.ndx
    xn0 = k.calc(x, u)[0]
    Fx = np.zeros((n, n))
    for j in range(n):
        e = np.zeros(n)
        e[j] = h
        xp, xm = k.calc(k.state_integrate(x, e), u)[0], k.calc(k.state_integrate(x, -e), u)[0]
        Fx[:, j] = (k.state_diff(xn0, xp) - k.state_diff(xn0, xm)) / (2 * h)
    tol = 3e4 * np.sqrt(2 * np.finfo(float).eps) * 1e-2
    assert np.max(np.abs(Fx - ref["Fx"])) / max(1.0, np.max(np.abs(ref["Fx"]))) < tol


@pytest.mark.parametrize("case", range(len(FF_CASES)))
@pytest.mark.parametrize("terminal", [False, True])
def test_freeflyer_device_code_vs_oracle(lib, case, terminal):  # noqa: F811
    x0s, running, term = synthetic.build_floating(T=2, B=1, seed=case, **FF_CASES[case])
    em = term if terminal else running[0]
    kind, nu, blk = em.pack()
    blk = np.ascontiguousarray(blk[0])
    st = em.state
    nx, n = st.nx, st.ndx
    k = onp.ContactFwdKnot(blk, nx, nu) if kind == 5 else onp.FreeFwdKnot(blk, nx, nu)
    rng = np.random.default_rng(300 + case)
    model = st.pinocchio
    for it in range(3):
        x = synthetic.random_floating_state(model, rng, 1, spread=0.6, v_spread=0.8)[0]
        u = rng.uniform(-2, 2, nu)
        use_u = 0 if terminal else 1
        uo = None if terminal else u
        xn = np.zeros(nx)
        c = lib.mb_host_calc(_p(blk), nx, _p(x), _p(u), use_u, _p(xn))
        xo, co = k.calc(x, uo)
        np.testing.assert_allclose(xn, xo, rtol=1e-10, atol=1e-10)
        assert c == pytest.approx(co, rel=1e-10, abs=1e-14)
        m = max(nu, 1)
        out = {q: np.zeros(s) for q, s in [("Fx", n * n), ("Fu", n * m), ("Lxx", n * n), ("Lxu", n * m),
                                           ("Luu", m * m), ("Lx", n), ("Lu", m)]}
        xn2, c2 = np.zeros(nx), np.zeros(1)
        lib.mb_host_calc_diff(_p(blk), nx, m, _p(x), _p(u), use_u,
                              *[_p(out[q]) for q in ["Fx", "Fu", "Lxx", "Lxu", "Luu", "Lx", "Lu"]], _p(xn2), _p(c2))
        np.testing.assert_allclose(xn2, xo, rtol=1e-10, atol=1e-10)
        assert c2[0] == pytest.approx(co, rel=1e-10, abs=1e-14)
        ref = k.calc_diff(x, uo)
        if it == 0 and not terminal:
            _fd_check(k, x, uo, ref, nu)
        for q, a in out.items():
            rows = m if q == "Luu" else n
            got = a.reshape(-1, rows).T if q in ("Fx", "Fu", "Lxx", "Lxu", "Luu") else a
            want = ref[q]
            if q in ("Fu", "Lxu"):
                got = got[:, :nu]
            if q == "Luu":
                got = got[:nu, :nu]
            if q == "Lu":
                got = got[:nu]
            scale = max(1.0, float(np.max(np.abs(want)))) if want.size else 1.0
            err = float(np.max(np.abs(got - want))) if want.size else 0.0
            assert err / scale < 1e-9, (q, case, terminal, err)


IMP_CASES = [dict(kind="6d"), dict(kind="3d+3d", r_coeff=0.0, damping=1e-3), dict(kind="6d", r_coeff=0.4)]


@pytest.mark.parametrize("case", range(len(IMP_CASES)))
def test_freeflyer_impulse_vs_oracle(lib, case):  # noqa: F811
    kw = IMP_CASES[case]
    model = mb.sample_tree(5, seed=3, freeflyer=True)
    model.addFrame("mid_site", 3, mb.SE3(np.eye(3), (0.0, 0.05, -0.1)))
    st = mb.StateMultibody(model)
    imps = mb.ImpulseModelMultiple(st)
    kinds = kw["kind"].split("+")
    tip, mid = model.getFrameId("tip"), model.getFrameId("mid_site")
    imps.addImpulse("a", mb.ImpulseModel6D(st, tip) if kinds[0] == "6d" else mb.ImpulseModel3D(st, tip))
    if len(kinds) > 1:
        imps.addImpulse("b", mb.ImpulseModel3D(st, mid))
    costs = mb.CostModelSum(st, 0)
    xref = synthetic.random_floating_state(model, np.random.default_rng(1), 1)[0]
    costs.addCost("xReg", mb.CostModelState(st, xref, 0), 1e-2)
    costs.addCost("midTrans", mb.CostModelFrameTranslation(st, mb.FrameTranslation(mid, (0.1, 0.0, 0.2)), 0), 0.3)
    am = mb.ActionModelImpulseFwdDynamics(st, imps, costs, kw.get("r_coeff", 0.0), kw.get("damping", 0.0))
    kind, nu, blk = am.pack()
    blk = np.ascontiguousarray(blk[0])
    nx, n = st.nx, st.ndx
    k = onp.ImpulseFwdKnot(blk, nx, 0)
    rng = np.random.default_rng(400 + case)
    u = np.zeros(1)
    for _ in range(3):
        x = synthetic.random_floating_state(model, rng, 1, spread=0.6, v_spread=0.8)[0]
        xn = np.zeros(nx)
        c = lib.mb_host_calc(_p(blk), nx, _p(x), _p(u), 0, _p(xn))
        xo, co = k.calc(x)
        np.testing.assert_allclose(xn, xo, rtol=1e-10, atol=1e-10)
        assert c == pytest.approx(co, rel=1e-12, abs=1e-14)
        m = 1
        out = {q: np.zeros(s) for q, s in [("Fx", n * n), ("Fu", n * m), ("Lxx", n * n), ("Lxu", n * m),
                                           ("Luu", m * m), ("Lx", n), ("Lu", m)]}
        xn2, c2 = np.zeros(nx), np.zeros(1)
        lib.mb_host_calc_diff(_p(blk), nx, m, _p(x), _p(u), 0,
                              *[_p(out[q]) for q in ["Fx", "Fu", "Lxx", "Lxu", "Luu", "Lx", "Lu"]], _p(xn2), _p(c2))
        np.testing.assert_allclose(xn2, xo, rtol=1e-10, atol=1e-10)
        ref = k.calc_diff(x)
        Fx = out["Fx"].reshape(n, n).T
        scale = max(1.0, float(np.max(np.abs(ref["Fx"]))))
        assert float(np.max(np.abs(Fx - ref["Fx"]))) / scale < 1e-8, (case, float(np.max(np.abs(Fx - ref["Fx"]))))
        for q in ("Lxx", "Lx"):
            got = out[q].reshape(n, n).T if q == "Lxx" else out[q]
            assert float(np.max(np.abs(got - ref[q]))) / max(1.0, float(np.max(np.abs(ref[q])))) < 1e-10, q
