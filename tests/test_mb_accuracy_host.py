"""Accuracy of the device multibody calcDiff against the numpy oracle on the Talos
walking knots (CPU: the device code compiled for the host, tests/cpp/mb_host.cpp, its
LDS matrices dumped through multibody.hpp's MB_DUMP hook).

Round 4's parity diagnosis (tools/parity_trace.py, tools/mb_dump_check.py): with the
CRBA formed about the world origin, a light distal link 1 m from the origin made its
mass-matrix entries the difference of ~m |c|^2 terms, and cond(M) ~ 1e6 carried the lost
digits into M^-1 and Fu (6.8e-14 normwise; the two oracles agree to 6e-16). The columns
are now formed about their joint (w_crba_column). Bars: M^-1 and the KKT inverse's
top-left block within 1e-14 normwise, Fu within 1e-14 and Fx within 5e-14 of the
oracle's complex-step derivatives (the oracle-to-oracle spread is 6e-16 / 7e-15)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.parametrize("knot", [0, 1, 49])
def test_talos_calc_diff_accuracy_host(knot, tmp_path, monkeypatch):
    import mb_dump_check as mdc
    from crocoddyl_amd import synthetic
    from oracle import multibody_np as onp
    x0s, running, terminal = synthetic.build("C5_talos_walk", B=1)
    mdl = running[knot]
    kind, nu, blk = mdl.pack()
    blk = np.ascontiguousarray(blk[0], np.float64)
    mm = max(r.nu for r in running)
    u = np.zeros(mm)
    u[:nu] = mdl.quasiStatic(None, x0s[0])
    x = x0s[0]
    sh, dm, ob = mdc.host_run(blk, x.size, nu, mm, x, u)
    dev = {}
    for s, name in enumerate(mdc.NAMES):
        r, c = sh[s]
        if r > 0:
            dev[name] = dm[s, :r * c].reshape(c, r).T
    k = onp.ContactFwdKnot(blk, x.size, nu)
    M = k.robot.crba(x[:k.nq]) + np.diag(k.robot.armature)
    Minv = np.linalg.inv(M)
    Jc, _ = k.contact_terms(x)
    Y = Minv @ Jc.T
    G = Minv - (Y @ np.linalg.inv(Jc @ Y + k.damping * np.eye(Jc.shape[0]))) @ Y.T
    def nrm(g, o):  # (the pseudo-impulse knot, dt = 0, has Fu = 0)
        return float(np.max(np.abs(g - o)) / max(float(np.max(np.abs(o))), 1e-300)) if np.any(o) else float(np.max(np.abs(g)))
    assert nrm(dev["Minv"], Minv) < 1e-14
    assert nrm(dev["Kinv_tl"], G) < 1e-14
    n = 2 * k.nv
    d = k.calc_diff(x, u[:nu])
    Fx = ob[:n * n].reshape(n, n).T
    Fu = ob[n * n:n * n + n * mm].reshape(mm, n).T[:, :nu]
    assert nrm(Fu, d["Fu"]) < 1e-14
    assert nrm(Fx, d["Fx"]) < 5e-14
