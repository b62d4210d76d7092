"""The device multibody knot code (crocoddyl_amd/csrc/multibody.hpp), compiled
for the host with the sequential-lane executor (tests/cpp/mb_host.cpp), vs the
numpy oracle (oracle/multibody_np.py: ABA + complex-step derivatives). CPU
only: the same arithmetic the GPU runs, checked without a GPU (the GPU run of
it is tests/test_multibody_gpu.py)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from crocoddyl_amd import multibody as mb, synthetic
from oracle import multibody_np as onp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "mb_host.cpp")
OUT = os.path.join(ROOT, "tests", "_build", "libmb_host.so")
D = C.POINTER(C.c_double)


@pytest.fixture(scope="module")
def lib():
    hdr = os.path.join(ROOT, "crocoddyl_amd", "csrc", "multibody.hpp")
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(SRC), os.path.getmtime(hdr)):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O2", "-std=c++17",
                               "-shared", "-fPIC", "-o", OUT, SRC])
    L = C.CDLL(OUT)
    L.mb_host_calc.restype = C.c_double
    L.mb_host_calc.argtypes = [D, C.c_int, D, D, C.c_int, D]
    L.mb_host_calc_diff.argtypes = [D, C.c_int, C.c_int, D, D, C.c_int] + [D] * 9
    return L


def _p(a):
    return a.ctypes.data_as(D)


CASES = [dict(), dict(weighted=True), dict(robot=mb.sample_tree(6, seed=4), weighted=True),
         dict(robot=mb.sample_tree(9, seed=8, branching=False), armature=np.full(9, 0.05)),
         dict(robot=mb.sample_tree(12, seed=2), weighted=True, armature=np.linspace(0.0, 0.2, 12))]


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("terminal", [False, True])
def test_device_code_vs_oracle(lib, case, terminal):
    x0s, running, term = synthetic.build_arm(T=2, B=1, **CASES[case])
    em = term if terminal else running[0]
    _, nu, blk = em.pack()
    blk = np.ascontiguousarray(blk[0])
    nx = em.state.nx
    k = onp.FreeFwdKnot(blk, nx, nu)
    rng = np.random.default_rng(case)
    for _ in range(3):
        x, u = rng.uniform(-2, 2, nx), rng.uniform(-3, 3, nu)
        use_u = 0 if terminal else 1
        uo = None if terminal else u
        xn = np.zeros(nx)
        c = lib.mb_host_calc(_p(blk), nx, _p(x), _p(u), use_u, _p(xn))
        xo, co = k.calc(x, uo)
        np.testing.assert_allclose(xn, xo, rtol=1e-12, atol=1e-12)
        assert c == pytest.approx(co, rel=1e-12, abs=1e-14)
        n, m = nx, nu
        out = {q: np.zeros(s) for q, s in [("Fx", n * n), ("Fu", n * m), ("Lxx", n * n), ("Lxu", n * m),
                                           ("Luu", m * m), ("Lx", n), ("Lu", m)]}
        xn2, c2 = np.zeros(nx), np.zeros(1)
        lib.mb_host_calc_diff(_p(blk), nx, m, _p(x), _p(u), use_u,
                              *[_p(out[q]) for q in ["Fx", "Fu", "Lxx", "Lxu", "Luu", "Lx", "Lu"]], _p(xn2), _p(c2))
        # the calc fused into calcDiff (iteration 0 of a solve)
        np.testing.assert_allclose(xn2, xo, rtol=1e-12, atol=1e-12)
        assert c2[0] == pytest.approx(co, rel=1e-12, abs=1e-14)
        ref = k.calc_diff(x, uo)
        for q, a in out.items():
            rows = m if q == "Luu" else n
            got = a.reshape(-1, rows).T if q in ("Fx", "Fu", "Lxx", "Lxu", "Luu") else a
            scale = max(1.0, float(np.max(np.abs(ref[q]))))
            assert float(np.max(np.abs(got - ref[q]))) / scale < 1e-10, (q, case, terminal)


CONTACT_CASES = [dict(contact="6d"), dict(contact="3d", weighted=True), dict(contact="3d+3d", armature=np.full(7, 0.02)),
                 dict(contact="6d+3d", damping=1e-3, inactive=True),
                 dict(contact="6d", gains=(0.0, 0.0)), dict(contact="3d", gains=(5.0, 0.0)),
                 dict(contact="6d+3d", robot=mb.sample_tree(10, seed=5), damping=1e-2, weighted=True),
                 # CostModelContactForce with the force Jacobians (enable_force), and without them
                 dict(contact="6d+3d", damping=1e-3, force_costs=True), dict(contact="3d", force_costs=True),
                 dict(contact="6d", force_costs=True, enable_force=False)]


@pytest.mark.parametrize("case", range(len(CONTACT_CASES)))
@pytest.mark.parametrize("terminal", [False, True])
def test_contact_device_code_vs_oracle(lib, case, terminal):
    """Euler∘ContactFwdDynamics: device KKT solve + analytic derivatives vs the
    oracle's single KKT solve + complex-step derivatives."""
    x0s, running, term = synthetic.build_arm_contact(T=2, B=1, **CONTACT_CASES[case])
    em = term if terminal else running[0]
    kind, nu, blk = em.pack()
    assert kind == 5
    blk = np.ascontiguousarray(blk[0])
    nx = em.state.nx
    k = onp.ContactFwdKnot(blk, nx, nu)
    rng = np.random.default_rng(100 + case)
    for _ in range(3):
        x, u = rng.uniform(-1.5, 1.5, nx), rng.uniform(-3, 3, nu)
        use_u = 0 if terminal else 1
        uo = None if terminal else u
        xn = np.zeros(nx)
        c = lib.mb_host_calc(_p(blk), nx, _p(x), _p(u), use_u, _p(xn))
        xo, co = k.calc(x, uo)
        np.testing.assert_allclose(xn, xo, rtol=1e-10, atol=1e-10)
        assert c == pytest.approx(co, rel=1e-10, abs=1e-14)  # (force costs: lambda from two solves)
        n, m = nx, nu
        out = {q: np.zeros(s) for q, s in [("Fx", n * n), ("Fu", n * m), ("Lxx", n * n), ("Lxu", n * m),
                                           ("Luu", m * m), ("Lx", n), ("Lu", m)]}
        xn2, c2 = np.zeros(nx), np.zeros(1)
        lib.mb_host_calc_diff(_p(blk), nx, m, _p(x), _p(u), use_u,
                              *[_p(out[q]) for q in ["Fx", "Fu", "Lxx", "Lxu", "Luu", "Lx", "Lu"]], _p(xn2), _p(c2))
        np.testing.assert_allclose(xn2, xo, rtol=1e-10, atol=1e-10)
        assert c2[0] == pytest.approx(co, rel=1e-10, abs=1e-14)
        ref = k.calc_diff(x, uo)
        for q, a in out.items():
            rows = m if q == "Luu" else n
            got = a.reshape(-1, rows).T if q in ("Fx", "Fu", "Lxx", "Lxu", "Luu") else a
            scale = max(1.0, float(np.max(np.abs(ref[q]))))
            assert float(np.max(np.abs(got - ref[q]))) / scale < 1e-9, (q, case, terminal,
                                                                        float(np.max(np.abs(got - ref[q]))))


IMPULSE_CASES = [dict(kind="6d"), dict(kind="3d", weighted=True), dict(kind="6d+3d", damping=1e-3, inactive=True),
                 dict(kind="6d", r_coeff=0.5, armature=np.full(7, 0.02)),
                 dict(kind="6d+3d", robot=mb.sample_tree(10, seed=5), damping=1e-2, weighted=True, r_coeff=0.2)]


@pytest.mark.parametrize("case", range(len(IMPULSE_CASES)))
def test_impulse_device_code_vs_oracle(lib, case):
    """ActionModelImpulseFwdDynamics: device impulse solve + the reference's
    derivative formula vs the oracle's KKT solve + complex-step pieces."""
    am = synthetic.impulse_model(**IMPULSE_CASES[case])
    kind, nu, blk = am.pack()
    assert kind == 6 and nu == 0
    blk = np.ascontiguousarray(blk[0])
    nx = am.state.nx
    k = onp.ImpulseFwdKnot(blk, nx, 0)
    rng = np.random.default_rng(200 + case)
    u = np.zeros(1)
    for _ in range(3):
        x = rng.uniform(-1.5, 1.5, nx)
        xn = np.zeros(nx)
        c = lib.mb_host_calc(_p(blk), nx, _p(x), _p(u), 0, _p(xn))
        xo, co = k.calc(x)
        np.testing.assert_allclose(xn, xo, rtol=1e-10, atol=1e-10)
        assert c == pytest.approx(co, rel=1e-12, abs=1e-14)
        n, m = nx, 1  # one padded control column (nu_max of a mixed horizon)
        out = {q: np.zeros(s) for q, s in [("Fx", n * n), ("Fu", n * m), ("Lxx", n * n), ("Lxu", n * m),
                                           ("Luu", m * m), ("Lx", n), ("Lu", m)]}
        xn2, c2 = np.zeros(nx), np.zeros(1)
        lib.mb_host_calc_diff(_p(blk), nx, m, _p(x), _p(u), 0,
                              *[_p(out[q]) for q in ["Fx", "Fu", "Lxx", "Lxu", "Luu", "Lx", "Lu"]], _p(xn2), _p(c2))
        np.testing.assert_allclose(xn2, xo, rtol=1e-10, atol=1e-10)
        assert c2[0] == pytest.approx(co, rel=1e-12, abs=1e-14)
        ref = k.calc_diff(x)
        Fx = out["Fx"].reshape(n, n).T
        scale = max(1.0, float(np.max(np.abs(ref["Fx"]))))
        # 1e-8: G and H come from S = Jc M^-1 Jc^T, whose condition number reaches
        # 2e7 on these random states (Gauss-Jordan here, LAPACK inverses there)
        assert float(np.max(np.abs(Fx - ref["Fx"]))) / scale < 1e-8, (case, float(np.max(np.abs(Fx - ref["Fx"]))))
        for q in ("Lxx", "Lx"):
            got = out[q].reshape(n, n).T if q == "Lxx" else out[q]
            assert float(np.max(np.abs(got - ref[q]))) / max(1.0, float(np.max(np.abs(ref[q])))) < 1e-10, q
        assert not out["Fu"].any() and not out["Lxu"].any() and not out["Luu"].any() and not out["Lu"].any()


def test_calc_diff_lds_plans_have_no_live_overlap(lib):
    """The calcDiff's LDS plans (multibody.hpp diff_layout: the all-LDS plan and the
    spilled one, whose arrays share areas by live range) checked statically: any two
    arrays whose LDS areas overlap have disjoint live ranges over the calcDiff's phases
    (diff_layout_regions / diff_layout_check), and every array lies inside the plan."""
    msg = C.create_string_buffer(512)
    lib.mb_host_layout_check.argtypes = [C.c_int] * 7 + [C.c_char_p, C.c_int]
    n = 0
    for nj in (3, 6, 7, 12, 18, 21, 24, 30, 38, 48, 64):
        for nc in (0, 3, 6, 12, 24):
            for njac in (0, 1, 3, 8):
                for vcols in (0, 1):
                    for nu in {nj, max(nj - 6, 1)}:
                        for nrows in (0, 20, 64):
                            for spill in (0, 1, 3, 5, 7):
                                if spill and 84 * nj > 4 * nj * nj:
                                    continue  # (diff_spill: the maps must fit the Fx block)
                                rc = lib.mb_host_layout_check(nj, njac, nc, vcols, nu, nrows, spill, msg, 512)
                                assert rc == 0, (nj, nc, njac, vcols, nu, nrows, spill, msg.value.decode())
                                n += 1
    assert n > 5000

